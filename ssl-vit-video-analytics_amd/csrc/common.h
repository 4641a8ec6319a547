// Shared device helpers for the MI355X (gfx950 / CDNA4) MAE kernels.
// Storage types: float (parity mode) and __bf16 (training mode); every kernel
// accumulates in fp32.  Wave = 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SM_DEV __device__ __forceinline__

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

enum SmDtype { SM_F32 = 0, SM_BF16 = 1 };

// ---------------------------------------------------------------- conversions
template <typename T> SM_DEV float to_f(T x);
template <> SM_DEV float to_f<float>(float x) { return x; }
template <> SM_DEV float to_f<__bf16>(__bf16 x) { return (float)x; }
template <typename T> SM_DEV T from_f(float x);
template <> SM_DEV float from_f<float>(float x) { return x; }
template <> SM_DEV __bf16 from_f<__bf16>(float x) { return (__bf16)x; }

// 8-wide vector load/store of T as fp32 (16 B for bf16, 32 B for f32).
SM_DEV void load8(const float* p, float* v) {
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
SM_DEV void load8(const __bf16* p, float* v) {
  bf16x8 a = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
}
SM_DEV void store8(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
SM_DEV void store8(__bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)v[i];
  *(bf16x8*)p = a;
}
SM_DEV void load4(const float* p, float* v) {
  float4 a = *(const float4*)p;
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
SM_DEV void load4(const __bf16* p, float* v) {
  bf16x4 a = *(const bf16x4*)p;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (float)a[i];
}
SM_DEV void store4(float* p, const float* v) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); }
SM_DEV void store4(__bf16* p, const float* v) {
  bf16x4 a;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = (__bf16)v[i];
  *(bf16x4*)p = a;
}
// The same with the non-temporal hint (`nt` loads / stores): for tensors a kernel streams
// once, larger than the caches, so they do not evict lines other waves still reuse.
SM_DEV void load8_nt(const float* p, float* v) {
  const f32x4 a = __builtin_nontemporal_load((const f32x4*)p), b = __builtin_nontemporal_load((const f32x4*)p + 1);
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[4 + i] = b[i]; }
}
SM_DEV void load8_nt(const __bf16* p, float* v) {
  const bf16x8 a = __builtin_nontemporal_load((const bf16x8*)p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)a[i];
}
SM_DEV void store8_nt(float* p, const float* v) {
  __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, (f32x4*)p);
  __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, (f32x4*)p + 1);
}
SM_DEV void store8_nt(__bf16* p, const float* v) {
  bf16x8 a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)v[i];
  __builtin_nontemporal_store(a, (bf16x8*)p);
}
SM_DEV void load4_nt(const float* p, float* v) {
  const f32x4 a = __builtin_nontemporal_load((const f32x4*)p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = a[i];
}
SM_DEV void load4_nt(const __bf16* p, float* v) {
  const bf16x4 a = __builtin_nontemporal_load((const bf16x4*)p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (float)a[i];
}
SM_DEV void store4_nt(float* p, const float* v) { __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, (f32x4*)p); }
SM_DEV void store4_nt(__bf16* p, const float* v) {
  bf16x4 a;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = (__bf16)v[i];
  __builtin_nontemporal_store(a, (bf16x4*)p);
}

// ---------------------------------------------------------------- math
// Exact (erf) GELU, nn.GELU's default.  Phi(x) = 0.5 (1 + erf(x / sqrt 2)) is formed
// from erfc(z), z = |x| / sqrt 2, as erfc(z) = t P5(t) exp(-z^2), t = 1 / (1 + 0.3275911 z)
// (Abramowitz & Stegun 7.1.26, |error| < 1.5e-7): Phi = erfc / 2 for x < 0 (no
// cancellation in the left tail) and 1 - erfc / 2 for x >= 0.  The exp(-z^2) =
// exp(-x^2 / 2) factor is shared with the normal pdf of the derivative, so GELU is one
// rcp, one exp2 and a 5-term Horner chain (its coefficients pre-halved: erfc / 2 directly),
// and its derivative adds two ops.
// One template for a scalar and a packed pair (f32x2: v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32, two elements per VALU issue -- the f32 vector peak -- for the MFMA-free
// streaming kernels): the same operation sequence with contraction off, so both forms,
// and every kernel that evaluates GELU, produce bit-identical results (recomputed
// activations equal stored ones).
typedef float f32x2 __attribute__((ext_vector_type(2)));
SM_DEV float vfma(float a, float b, float c) { return fmaf(a, b, c); }
SM_DEV f32x2 vfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
SM_DEV float vabs(float a) { return fabsf(a); }
SM_DEV f32x2 vabs(f32x2 a) { return __builtin_elementwise_abs(a); }
SM_DEV float vrcp(float a) { return __builtin_amdgcn_rcpf(a); }
SM_DEV f32x2 vrcp(f32x2 a) { return f32x2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }
SM_DEV float vexp2(float a) { return __builtin_amdgcn_exp2f(a); }
SM_DEV f32x2 vexp2(f32x2 a) { return f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)}; }
SM_DEV float vsel_neg(float x, float a, float b) { return x < 0.f ? a : b; }   // x < 0 ? a : b
SM_DEV f32x2 vsel_neg(f32x2 x, f32x2 a, f32x2 b) { return f32x2{x.x < 0.f ? a.x : b.x, x.y < 0.f ? a.y : b.y}; }

template <typename V>
SM_DEV V gelu_phi_pair_t(V x, V* pdf_out) {
#pragma clang fp contract(off)
  const V t = vrcp(vfma(vabs(x), V(0.3275911f * 0.70710678118654752f), V(1.0f)));
  V p = V(0.5f * 1.061405429f);
  p = vfma(p, t, V(0.5f * -1.453152027f));
  p = vfma(p, t, V(0.5f * 1.421413741f));
  p = vfma(p, t, V(0.5f * -0.284496736f));
  p = vfma(p, t, V(0.5f * 0.254829592f));
  const V e = vexp2((x * x) * V(-0.5f * 1.44269504088896341f));
  const V half_erfc = (p * t) * e;
  if (pdf_out) *pdf_out = e * V(0.39894228040143268f);
  // 1 - half_erfc as an explicit fma with -1 (exact: one rounding, as the subtraction):
  // no contraction setting can fuse (p t) e into it differently in the scalar and the
  // packed form
  return vsel_neg(x, half_erfc, vfma(half_erfc, V(-1.0f), V(1.0f)));
}
template <typename V>
SM_DEV V gelu_t(V x) {
#pragma clang fp contract(off)
  return x * gelu_phi_pair_t<V>(x, nullptr);
}
template <typename V>
SM_DEV V gelu_grad_t(V x) {
#pragma clang fp contract(off)
  V pdf;
  const V cdf = gelu_phi_pair_t<V>(x, &pdf);
  return vfma(x, pdf, cdf);
}
SM_DEV float gelu_phi_pair(float x, float* pdf_out) { return gelu_phi_pair_t<float>(x, pdf_out); }
SM_DEV float gelu_f(float x) { return gelu_t<float>(x); }
SM_DEV float gelu_grad(float x) { return gelu_grad_t<float>(x); }
SM_DEV f32x2 gelu_f2(f32x2 x) { return gelu_t<f32x2>(x); }
SM_DEV f32x2 gelu_grad2(f32x2 x) { return gelu_grad_t<f32x2>(x); }

// BatchNorm shift b - mean * sc as one explicit fma: every kernel that forms the affine
// (bn_apply and each folded consumer) computes the same bits whatever the contraction mode
SM_DEV float bn_shift(float b, float mean, float sc) { return fmaf(-mean, sc, b); }

// Per-channel input transform folded into a consumer's loads: h = act(x * sc + sh)
// with sc = rstd * w, sh = b - mean * sc (train-mode BatchNorm) and act = GELU or
// identity; rounded to the storage type exactly as bn_apply would store h.  A null
// mean means identity.
struct ChanAffine {
  const float *mean, *rstd, *w, *b;
  int gelu;
};
struct Affine8 {
  float sc[8], sh[8];
  bool on, gelu;
  SM_DEV void init(const ChanAffine& a, int c0) {
    on = a.mean != nullptr;
    gelu = a.gelu != 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (on) {
        sc[j] = a.rstd[c0 + j] * a.w[c0 + j];
        sh[j] = bn_shift(a.b[c0 + j], a.mean[c0 + j], sc[j]);
      } else {
        sc[j] = 1.f;
        sh[j] = 0.f;
      }
    }
  }
  // v: 8 values loaded from T storage -> the stored-precision activation
  // (packed pairs: see gelu_phi_pair_t)
  template <typename T>
  SM_DEV void apply(float* v) const {
    if (!on) return;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      f32x2 t = vfma(f32x2{v[j], v[j + 1]}, f32x2{sc[j], sc[j + 1]}, f32x2{sh[j], sh[j + 1]});
      if (gelu) t = gelu_f2(t);
      v[j] = to_f<T>(from_f<T>(t.x));
      v[j + 1] = to_f<T>(from_f<T>(t.y));
    }
  }
};

// ---------------------------------------------------------------- reductions
SM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SM_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
SM_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum; `red` must hold blockDim.x/64 floats.  Result valid in all threads.
SM_DEV float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------- counter RNG
// Dropout / DropPath masks are a pure function of (seed, row, column):
//   h    = fmix32(seed32 + row * 0x9E3779B1 + (col >> 2) * 0x7FEB352D)
//   byte = (h >> 8 * (col & 3)) & 0xFF                 (one hash per 4 columns)
//   keep = byte >= round(256 p)                        (kept values scaled by 256/(256-thr))
// Every kernel that touches an element (forward, checkpoint recompute, backward)
// regenerates the same mask without storing it.  `row` is the tensor row (or the
// attention row (n*H + h)*L + q); fmix32 is MurmurHash3's finalizer.  The 8-bit
// keep threshold is the FlashAttention-2 convention (what the reference's GPU
// SDPA uses): for p = 0.1 the drop rate is 26/256.
SM_DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
SM_DEV uint32_t seed32(uint64_t seed) { return (uint32_t)seed ^ (uint32_t)(seed >> 32); }
SM_DEV uint32_t drop_rowbase(uint32_t s32, uint64_t row) { return s32 + (uint32_t)row * 0x9E3779B1u; }
SM_DEV uint32_t drop_hash(uint32_t rowbase, uint32_t col) { return fmix32(rowbase + (col >> 2) * 0x7FEB352Du); }
SM_DEV uint32_t drop_thr(float p) { return (uint32_t)(p * 256.f + 0.5f); }
// Kept values are scaled by 256 / (256 - thr), the inverse of the quantised keep rate, so
// E[mask * scale] = 1 exactly as nn.Dropout / timm DropPath (1 / (1 - p) with the 8-bit
// threshold would leave E = (256 - thr) / 256 / (1 - p): 0.99826 at p = 0.1).
SM_DEV float drop_scale(float p) {
  const uint32_t t = drop_thr(p);
  return t >= 256u ? 0.f : 256.f / (float)(256u - t);
}
SM_DEV bool drop_keep_bits(uint32_t h, uint32_t col, uint32_t thr) {
  return ((h >> ((col & 3) * 8)) & 0xFFu) >= thr;
}
SM_DEV bool drop_keep(uint32_t s32, uint64_t row, uint32_t col, uint32_t thr) {
  return drop_keep_bits(drop_hash(drop_rowbase(s32, row), col), col, thr);
}

// Reduce partial slabs part[nb][ncols] over nb.  Block = 32 columns x 8 row groups;
// fp64 accumulation, fixed order (deterministic).  Writes fp64 (outd) and/or
// fp32 (outf, optionally accumulating).
static __global__ __launch_bounds__(256) void colred_kernel(const float* part, int nb, int ncols, double* outd,
                                                     float* outf, int accumulate) {
  __shared__ double red[8][32];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < ncols) {
    int b = g;
    for (; b + 24 < nb; b += 32) {
      s0 += part[(int64_t)b * ncols + c];
      s1 += part[(int64_t)(b + 8) * ncols + c];
      s2 += part[(int64_t)(b + 16) * ncols + c];
      s3 += part[(int64_t)(b + 24) * ncols + c];
    }
    for (; b < nb; b += 8) s0 += part[(int64_t)b * ncols + c];
  }
  red[g][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < ncols) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    if (outd) outd[c] = t;
    if (outf) outf[c] = accumulate ? outf[c] + (float)t : (float)t;
  }
}

static inline void colred(const float* part, int nb, int ncols, double* outd, float* outf, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(colred_kernel, dim3((ncols + 31) / 32), dim3(256), 0, st, part, nb, ncols, outd, outf,
                     accumulate);
}

#define SM_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
