// MAE-specific kernels around the encoder/decoder:
//
//  * tube mask from host-drawn noise (get_tube_mask, mae_loader.py:80-90): the
//    int(r*L) largest noise values of each sample are masked (rank by value
//    descending, ties by lower index first), repeated over T; also emits the
//    row-major compaction index list of masked tokens used by the masked gather
//    (train_ssl_mae.py:105).  Integer work, bit-exact.
//  * pos-embed add + mask-token blend (mae_vit_adapter.py:97-104) fwd/bwd.
//  * fused patchify + norm_pix + masked MSE (train_ssl_mae.py:26-31,74-84): the
//    target is read straight from the clip [B,3,T,H,W]; loss reduction is
//    deterministic (per-block partials, fp64 finalize); backward writes dL/dpred.
//  * masked row gather + unbiased std (logging statistic).
//  * AdamW (torch.optim.AdamW semantics) over one flat fp32 parameter buffer with
//    a GradScaler-style non-finite check (step skipped on inf/nan, no host sync),
//    refreshing the bf16 weight shadow in the same pass.
#include "common.h"
#include "sm_api.h"

namespace {

// ------------------------------------------------------------------ tube mask
__global__ __launch_bounds__(256) void tube_mask_kernel(const float* noise, int T, int L, int n_mask,
                                                        uint8_t* mask /*[B][T][L]*/, int32_t* idx /*[B][T][n_mask]*/) {
  extern __shared__ float sn[];           // [L] noise, then [L] flags (as float)
  float* fl = sn + L;
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < L; i += blockDim.x) sn[i] = noise[(int64_t)b * L + i];
  __syncthreads();
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const float v = sn[i];
    int rank = 0;
    for (int j = 0; j < L; ++j) {
      const float u = sn[j];
      rank += (u > v) || (u == v && j < i);
    }
    fl[i] = rank < n_mask ? 1.f : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const uint8_t m = fl[i] != 0.f;
    int pos = 0;
    if (m)
      for (int j = 0; j < i; ++j) pos += fl[j] != 0.f;
    for (int t = 0; t < T; ++t) {
      const int64_t row = (int64_t)b * T + t;
      mask[row * L + i] = m;
      if (m && idx) idx[row * n_mask + pos] = (int32_t)(row * L + i);
    }
  }
}

// ------------------------------------------------------------------ pos + mask blend
template <typename TI, typename TO>
__global__ void pos_blend_fwd_kernel(const TI* y, const float* tpos /*[T][D]*/, const float* spos /*[L][D]*/,
                                     const float* tok /*[D]*/, const uint8_t* mask /*[F*L]*/, TO* x, int T, int L,
                                     int D, int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 8;
    const int64_t row = e / D;
    const int d0 = (int)(e % D);
    const int l = (int)(row % L);
    const int t = (int)((row / L) % T);
    const bool m = mask[row] != 0;
    float v[8];
    load8(y + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float pos = tpos[t * D + d0 + j] + spos[l * D + d0 + j];
      v[j] = m ? tok[d0 + j] : v[j] + pos;
    }
    store8(x + e, v);
  }
}

// dy = dx * (1-m)
template <typename TG, typename TY>
__global__ void pos_blend_dy_kernel(const TG* dx, const uint8_t* mask, TY* dy, int D, int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 8;
    const bool m = mask[e / D] != 0;
    float v[8];
    load8(dx + e, v);
    if (m)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    store8(dy + e, v);
  }
}

// per frame f: pt[f][d] = sum_l dx*(1-m), pm[f][d] = sum_l dx*m   (block per frame)
template <typename TG>
__global__ __launch_bounds__(256) void pos_blend_frame_kernel(const TG* dx, const uint8_t* mask, int L, int D,
                                                              float* pt, float* pm) {
  const int64_t f = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int l = 0; l < L; ++l) {
      const float v = to_f<TG>(dx[(f * L + l) * D + d]);
      if (mask[f * L + l]) b += v; else a += v;
    }
    pt[f * D + d] = a;
    pm[f * D + d] = b;
  }
}

// dspos[l][d] += sum_f dx*(1-m)
template <typename TG>
__global__ void pos_blend_spos_kernel(const TG* dx, const uint8_t* mask, int F, int L, int D, float* dspos) {
  const int64_t total = (int64_t)L * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(i / D), d = (int)(i % D);
    double s = 0.0;
    for (int f = 0; f < F; ++f)
      if (!mask[(int64_t)f * L + l]) s += to_f<TG>(dx[((int64_t)f * L + l) * D + d]);
    dspos[i] += (float)s;
  }
}

// ------------------------------------------------------------------ fused loss
struct LossArgs {
  const void* pred;          // [B][T*L][192]
  const float* clip;         // [B][3][T][H][W] via strides
  int64_t sB, sC, sT, sH, sW;
  const uint8_t* mask;       // [B][T][L]
  int B, T, H, W, L, wp;
  int norm_pix;
};

// target value for feature f of token (b,t,hi,wi): f = (p*8 + q)*3 + c
SM_DEV float tgt_val(const LossArgs& a, int b, int t, int hi, int wi, int f) {
  const int c = f % 3, q = (f / 3) % 8, p = f / 24;
  return a.clip[b * a.sB + c * a.sC + t * a.sT + (int64_t)(hi * 8 + p) * a.sH + (int64_t)(wi * 8 + q) * a.sW];
}

template <typename TP>
SM_DEV void token_terms(const LossArgs& a, int64_t tok, int lane, float (&diff)[3]) {
  const int TL = a.T * a.L;
  const int b = (int)(tok / TL);
  const int rem = (int)(tok % TL);
  const int t = rem / a.L, l = rem % a.L;
  const int hi = l / a.wp, wi = l % a.wp;
  float x[3];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) { x[i] = tgt_val(a, b, t, hi, wi, lane + 64 * i); s += x[i]; }
  if (a.norm_pix) {
    const float mu = wave_sum(s) / 192.f;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) { const float d = x[i] - mu; ss += d * d; }
    const float var = wave_sum(ss) / 191.f;
    const float inv = 1.f / sqrtf(var + 1e-6f);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = (x[i] - mu) * inv;
  }
  const TP* pr = (const TP*)a.pred + tok * 192;
#pragma unroll
  for (int i = 0; i < 3; ++i) diff[i] = to_f<TP>(pr[lane + 64 * i]) - x[i];
}

template <typename TP>
__global__ __launch_bounds__(256) void loss_fwd_kernel(LossArgs a, int64_t ntok, int tok_per_block, double* part) {
  __shared__ double red[2][4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double sl = 0.0, sm = 0.0;
  const int64_t t0 = (int64_t)blockIdx.x * tok_per_block;
  for (int k = w; k < tok_per_block; k += 4) {
    const int64_t tok = t0 + k;
    if (tok >= ntok) break;
    float diff[3];
    token_terms<TP>(a, tok, lane, diff);
    float e = diff[0] * diff[0] + diff[1] * diff[1] + diff[2] * diff[2];
    e = wave_sum(e) / 192.f;
    const float m = a.mask[tok] ? 1.f : 0.f;
    sl += (double)(e * m);
    sm += m;
  }
  if (lane == 0) { red[0][w] = sl; red[1][w] = sm; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void loss_final_kernel(const double* part, int nb, float* loss, float* denom) {
  double sl = 0.0, sm = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) { sl += part[2 * i]; sm += part[2 * i + 1]; }
  sl = wave_sum_d(sl);
  sm = wave_sum_d(sm);
  if (threadIdx.x == 0) {
    const float d = (float)sm + 1e-6f;
    denom[0] = d;
    loss[0] = (float)sl / d;
  }
}

template <typename TP>
__global__ __launch_bounds__(256) void loss_bwd_kernel(LossArgs a, int64_t ntok, const float* gout,
                                                       const float* denom, TP* dpred) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tok >= ntok) return;
  TP* out = dpred + tok * 192;
  if (!a.mask[tok]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) out[lane + 64 * i] = from_f<TP>(0.f);
    return;
  }
  float diff[3];
  token_terms<TP>(a, tok, lane, diff);
  const float g = gout[0] / denom[0] * (2.f / 192.f);
#pragma unroll
  for (int i = 0; i < 3; ++i) out[lane + 64 * i] = from_f<TP>(g * diff[i]);
}

// ------------------------------------------------------------------ gather / std
template <typename T>
__global__ void gather_rows_kernel(const T* src, const int32_t* idx, int64_t nrows, int C, T* dst) {
  const int cc = C / 8;
  const int64_t total = nrows * cc;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cc;
    const int c8 = (int)(i % cc);
    *(uint4*)(dst + r * C + c8 * 8) = *(const uint4*)(src + (int64_t)idx[r] * C + c8 * 8);
    if (sizeof(T) == 4) *(uint4*)(dst + r * C + c8 * 8 + 4) = *(const uint4*)(src + (int64_t)idx[r] * C + c8 * 8 + 4);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* x, int64_t n, double* part) {
  __shared__ double red[2][4];
  double s = 0.0, q = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = to_f<T>(x[i]);
    s += v;
    q += v * v;
  }
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = s; red[1][w] = q; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void std_final_kernel(const double* part, int nb, int64_t n, float* out) {
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) { s += part[2 * i]; q += part[2 * i + 1]; }
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if (threadIdx.x == 0) {
    const double mean = s / (double)n;
    double var = (q - s * mean) / (double)(n - 1);
    if (var < 0) var = 0;
    out[0] = (float)sqrt(var);
  }
}

// ------------------------------------------------------------------ AdamW
__global__ void nonfinite_kernel(const float* g, int64_t n, int* flag) {
  int bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void adamw_kernel(float* p, const float* g, float* m, float* v, __bf16* shadow, int64_t n, float lr,
                             float b1, float b2, float eps, float wd, const int* flag, const int64_t* step) {
  if (flag && *flag) return;
  const double t = (double)(*step + 1);
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, t));
  const float step_size = lr / bc1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pv = p[i] * (1.f - lr * wd);
    const float gv = g[i];
    float mv = m[i];
    mv = mv + (1.f - b1) * (gv - mv);
    const float vv = v[i] * b2 + (1.f - b2) * gv * gv;
    const float denom = sqrtf(vv) / bc2s + eps;
    pv = pv - step_size * (mv / denom);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
    if (shadow) shadow[i] = (__bf16)pv;
  }
}

__global__ void step_incr_kernel(const int* flag, int64_t* step) {
  if (!(flag && *flag)) *step += 1;
}

__global__ void fill_kernel(float* p, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// imgs [B][C][T][H][W] (strided) <-> tokens [B][T*hp*wp][p*p*C], feature (pi,qi,c)
__global__ void patchify_kernel(const float* x, int64_t sB, int64_t sC, int64_t sT, int64_t sH, int64_t sW, int B,
                                int C, int T, int H, int W, int p, float* out, int inverse) {
  const int hp = H / p, wp = W / p;
  const int F = p * p * C;
  const int64_t total = (int64_t)B * T * hp * wp * F;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    int64_t tok = i / F;
    const int w = (int)(tok % wp);
    tok /= wp;
    const int h = (int)(tok % hp);
    tok /= hp;
    const int t = (int)(tok % T);
    const int b = (int)(tok / T);
    const int c = f % C, qi = (f / C) % p, pi = f / (C * p);
    const int64_t src = b * sB + c * sC + t * sT + (int64_t)(h * p + pi) * sH + (int64_t)(w * p + qi) * sW;
    if (inverse) out[src] = x[i];
    else out[i] = x[src];
  }
}

__global__ void scale_kernel(float* p, int64_t n, float a) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] *= a;
}

inline int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

#define DISPATCH1(DT, ...)                                       \
  do {                                                         \
    if ((DT) == SM_F32) { typedef float T; __VA_ARGS__; }      \
    else { typedef __bf16 T; __VA_ARGS__; }                    \
  } while (0)

extern "C" int sm_tube_mask(const float* noise, int B, int T, int L, int n_mask, uint8_t* mask, int32_t* idx,
                            hipStream_t st) {
  if (B <= 0 || T <= 0 || L <= 0) return 0;
  if (L > 8192 || n_mask < 0 || n_mask > L) return -2;
  hipLaunchKernelGGL(tube_mask_kernel, dim3(B), dim3(256), 2 * L * sizeof(float), st, noise, T, L, n_mask, mask, idx);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_pos_blend_fwd(int y_dtype, int x_dtype, const void* y, const float* tpos, const float* spos,
                                const float* tok, const uint8_t* mask, void* x, int B, int T, int L, int D,
                                hipStream_t st) {
  if (D % 8) return -2;
  const int64_t n8 = (int64_t)B * T * L * D / 8;
  if (n8 <= 0) return 0;
#define PB(T1, T2) hipLaunchKernelGGL((pos_blend_fwd_kernel<T1, T2>), dim3(ew_blocks(n8)), dim3(256), 0, st, \
                                      (const T1*)y, tpos, spos, tok, mask, (T2*)x, T, L, D, n8)
  if (y_dtype == SM_BF16 && x_dtype == SM_F32) PB(__bf16, float);
  else if (y_dtype == SM_BF16) PB(__bf16, __bf16);
  else if (x_dtype == SM_F32) PB(float, float);
  else PB(float, __bf16);
#undef PB
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_pos_blend_bwd(int g_dtype, int y_dtype, const void* dx, const uint8_t* mask, void* dy,
                                float* dtpos, float* dspos, float* dtok, float* ws /*[2][F][D]*/, int B, int T,
                                int L, int D, hipStream_t st) {
  if (D % 8) return -2;
  const int F = B * T;
  const int64_t n8 = (int64_t)F * L * D / 8;
  if (n8 <= 0) return 0;
#define PD(T1, T2) hipLaunchKernelGGL((pos_blend_dy_kernel<T1, T2>), dim3(ew_blocks(n8)), dim3(256), 0, st, \
                                      (const T1*)dx, mask, (T2*)dy, D, n8)
  if (g_dtype == SM_F32 && y_dtype == SM_BF16) PD(float, __bf16);
  else if (g_dtype == SM_F32) PD(float, float);
  else if (y_dtype == SM_BF16) PD(__bf16, __bf16);
  else PD(__bf16, float);
#undef PD
  float* pt = ws;
  float* pm = ws + (int64_t)F * D;
  DISPATCH1(g_dtype, hipLaunchKernelGGL(pos_blend_frame_kernel<T>, dim3(F), dim3(128), 0, st, (const T*)dx, mask,
                                        L, D, pt, pm));
  DISPATCH1(g_dtype, hipLaunchKernelGGL(pos_blend_spos_kernel<T>, dim3(ew_blocks((int64_t)L * D)), dim3(256), 0,
                                        st, (const T*)dx, mask, F, L, D, dspos));
  // dtpos[t][d] += sum_b pt[b][t][d] and dtok[d] += sum_f pm[f][d]: fixed-order fp64 column
  // reductions ([B][T*D] and [F][D] views), many threads per column instead of one
  colred(pt, B, T * D, nullptr, dtpos, 1, st);
  colred(pm, F, D, nullptr, dtok, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

static LossArgs make_loss_args(const void* pred, const float* clip, int64_t sB, int64_t sC, int64_t sT, int64_t sH,
                               int64_t sW, const uint8_t* mask, int B, int T, int H, int W, int norm_pix) {
  LossArgs a;
  a.pred = pred; a.clip = clip; a.sB = sB; a.sC = sC; a.sT = sT; a.sH = sH; a.sW = sW; a.mask = mask;
  a.B = B; a.T = T; a.H = H; a.W = W; a.wp = W / 8; a.L = (H / 8) * (W / 8); a.norm_pix = norm_pix;
  return a;
}

extern "C" int64_t sm_loss_workspace_bytes(int B, int T, int L) {
  const int64_t ntok = (int64_t)B * T * L;
  const int64_t nb = (ntok + 255) / 256;
  return nb * 2 * 8;
}

extern "C" int sm_mae_loss_fwd(int pred_dtype, const void* pred, const float* clip, int64_t sB, int64_t sC,
                               int64_t sT, int64_t sH, int64_t sW, const uint8_t* mask, int B, int T, int H, int W,
                               int norm_pix, float* loss, float* denom, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (H % 8 || W % 8) return -2;
  LossArgs a = make_loss_args(pred, clip, sB, sC, sT, sH, sW, mask, B, T, H, W, norm_pix);
  const int64_t ntok = (int64_t)B * T * a.L;
  const int tpb = 256;
  const int nb = (int)((ntok + tpb - 1) / tpb);
  if (ws_bytes < (int64_t)nb * 16) return -4;
  DISPATCH1(pred_dtype, hipLaunchKernelGGL(loss_fwd_kernel<T>, dim3(nb), dim3(256), 0, st, a, ntok, tpb, (double*)ws));
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(64), 0, st, (const double*)ws, nb, loss, denom);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_mae_loss_bwd(int pred_dtype, const void* pred, const float* clip, int64_t sB, int64_t sC,
                               int64_t sT, int64_t sH, int64_t sW, const uint8_t* mask, int B, int T, int H, int W,
                               int norm_pix, const float* grad_out, const float* denom, void* dpred, hipStream_t st) {
  if (H % 8 || W % 8) return -2;
  LossArgs a = make_loss_args(pred, clip, sB, sC, sT, sH, sW, mask, B, T, H, W, norm_pix);
  const int64_t ntok = (int64_t)B * T * a.L;
  const int nb = (int)((ntok + 3) / 4);
  DISPATCH1(pred_dtype, hipLaunchKernelGGL(loss_bwd_kernel<T>, dim3(nb), dim3(256), 0, st, a, ntok, grad_out, denom,
                                           (T*)dpred));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_gather_rows(int dtype, const void* src, const int32_t* idx, int64_t nrows, int C, void* dst,
                              hipStream_t st) {
  if (C % 8) return -2;
  if (nrows <= 0) return 0;
  DISPATCH1(dtype, hipLaunchKernelGGL(gather_rows_kernel<T>, dim3(ew_blocks(nrows * C / 8)), dim3(256), 0, st,
                                      (const T*)src, idx, nrows, C, (T*)dst));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t sm_std_workspace_bytes(void) { return 1024 * 16; }

extern "C" int sm_std(int dtype, const void* x, int64_t n, float* out, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (n <= 1) return -2;
  const int nb = 1024;
  if (ws_bytes < nb * 16) return -4;
  DISPATCH1(dtype, hipLaunchKernelGGL(sumsq_kernel<T>, dim3(nb), dim3(256), 0, st, (const T*)x, n, (double*)ws));
  hipLaunchKernelGGL(std_final_kernel, dim3(1), dim3(64), 0, st, (const double*)ws, nb, n, out);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_nonfinite(const float* g, int64_t n, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, g, n, flag);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_adamw(float* p, const float* g, float* m, float* v, void* bf16_shadow, int64_t n, float lr,
                        float b1, float b2, float eps, float wd, const int* found_inf, int64_t* step,
                        int advance_step, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL(adamw_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, p, g, m, v, (__bf16*)bf16_shadow, n, lr,
                       b1, b2, eps, wd, found_inf, step);
  if (advance_step) hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(1), 0, st, found_inf, step);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_fill(float* p, int64_t n, float v, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, p, n, v);
  SM_CHECK_LAUNCH();
  return 0;
}

// patchify (train_ssl_mae.py:26-31): imgs [B,C,T,H,W] fp32 (strides) -> out [B, T*hp*wp, p*p*C]
extern "C" int sm_patchify(const float* imgs, int B, int C, int T, int H, int W, int64_t sB, int64_t sC, int64_t sT,
                           int64_t sH, int64_t sW, int p, float* out, hipStream_t st) {
  if (p <= 0 || H % p || W % p) return -2;
  const int64_t total = (int64_t)B * C * T * H * W;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(patchify_kernel, dim3(ew_blocks(total)), dim3(256), 0, st, imgs, sB, sC, sT, sH, sW, B, C, T, H,
                     W, p, out, 0);
  SM_CHECK_LAUNCH();
  return 0;
}

// exact inverse of sm_patchify: tokens -> imgs (contiguous [B,C,T,H,W])
extern "C" int sm_unpatchify(const float* tokens, int B, int C, int T, int H, int W, int p, float* imgs,
                             hipStream_t st) {
  if (p <= 0 || H % p || W % p) return -2;
  const int64_t total = (int64_t)B * C * T * H * W;
  if (total <= 0) return 0;
  const int64_t sW = 1, sH = W, sT = (int64_t)H * W, sC = (int64_t)T * H * W, sB = (int64_t)C * T * H * W;
  hipLaunchKernelGGL(patchify_kernel, dim3(ew_blocks(total)), dim3(256), 0, st, tokens, sB, sC, sT, sH, sW, B, C, T,
                     H, W, p, imgs, 1);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_scale(float* p, int64_t n, float a, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, p, n, a);
  SM_CHECK_LAUNCH();
  return 0;
}
