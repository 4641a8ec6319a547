// Normalisation and elementwise kernels, token-major ([rows][C], NHWC) layout.
//
// LayerNorm (tiny_vit.py:112,115; decoder norm1/norm2/decoder_norm):
//   one wave per row, two-pass mean/var in registers, eps 1e-5; saves mean/rstd.
//   Backward: dx per row; dgamma/dbeta as per-block partial slabs + a column
//   reduce (deterministic, no atomics).
// BatchNorm2d in train mode (tiny_vit.py:16, Conv2d_BN): per-channel batch
//   statistics over N*H*W rows: shifted fp32 partial sums per block, fp64 finalize
//   (also the running-stat momentum update with the unbiased variance), apply with
//   an optional fused exact GELU.  Backward recomputes x_hat (and the GELU input)
//   from the saved pre-BN tensor, so only the conv output is kept.
#include "common.h"
#include "sm_api.h"

namespace {

// ============================================================ LayerNorm
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const TI* x, const float* g, const float* b, TO* y,
                                                     float* mean, float* rstd, int64_t M, int C, float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (row >= M) return;
  const TI* xr = x + row * C;
  constexpr int MAXV = 4;  // chunks of 4 per lane: C <= 64*4*4 = 1024
  float v[MAXV][4];
  float s = 0.f;
  const int nch = C / 4;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ci = l + 64 * i;
    if (ci < nch) {
      load4(xr + ci * 4, v[i]);
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    }
  }
  const float mu = wave_sum(s) / C;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ci = l + 64 * i;
    if (ci < nch)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[i][j] - mu; ss += d * d; }
  }
  const float var = wave_sum(ss) / C;
  const float rs = rsqrtf(var + eps);
  TO* yr = y + row * C;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ci = l + 64 * i;
    if (ci < nch) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ci * 4 + j;
        o[j] = (v[i][j] - mu) * rs * g[c] + b[c];
      }
      store4(yr + ci * 4, o);
    }
  }
  if (l == 0) { mean[row] = mu; rstd[row] = rs; }
}

// dx and per-block partial dgamma/dbeta.  Block = 4 waves, ROWS rows per block.
template <typename TI, typename TD, typename TX>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD* dy, const TI* x, const float* mean,
                                                     const float* rstd, const float* g, TX* dx,
                                                     float* part_g, float* part_b, int64_t M, int C,
                                                     int rows_per_block, const TX* dres) {
  constexpr int MAXV = 4;
  __shared__ float red_g[4][1024], red_b[4][1024];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int nch = C / 4;
  float ag[MAXV][4], ab[MAXV][4];
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { ag[i][j] = 0.f; ab[i][j] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  for (int rr = w; rr < rows_per_block; rr += 4) {
    const int64_t row = r0 + rr;
    if (row >= M) break;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXV][4], gg[MAXV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int ci = l + 64 * i;
      if (ci < nch) {
        float xv[4], dv[4];
        load4(x + row * C + ci * 4, xv);
        load4(dy + row * C + ci * 4, dv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = ci * 4 + j;
          xh[i][j] = (xv[j] - mu) * rs;
          gg[i][j] = dv[j] * g[c];
          s1 += gg[i][j];
          s2 += gg[i][j] * xh[i][j];
          ag[i][j] += dv[j] * xh[i][j];
          ab[i][j] += dv[j];
        }
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int ci = l + 64 * i;
      if (ci < nch) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = rs * (gg[i][j] - s1 - xh[i][j] * s2);
        TX* p = dx + row * C + ci * 4;
        if (dres) {
          float prev[4];
          load4(dres + row * C + ci * 4, prev);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] += prev[j];
        }
        store4(p, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int ci = l + 64 * i;
    if (ci < nch)
#pragma unroll
      for (int j = 0; j < 4; ++j) { red_g[w][ci * 4 + j] = ag[i][j]; red_b[w][ci * 4 + j] = ab[i][j]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part_g[(int64_t)blockIdx.x * C + c] = red_g[0][c] + red_g[1][c] + red_g[2][c] + red_g[3][c];
    part_b[(int64_t)blockIdx.x * C + c] = red_b[0][c] + red_b[1][c] + red_b[2][c] + red_b[3][c];
  }
}



// ---------------------------------------------- LayerNorm, 16 lanes per row (C = 192, 384)
// Four rows per wave (one per 16-lane DPP row), 16 rows per block in flight, a block
// walks a contiguous run of rows.  Lane gl of a row owns columns 64u + 4gl + j, so each
// load / store instruction covers 4 rows x one contiguous 128-B (bf16) or 256-B (fp32)
// run; gamma / beta live in registers for the whole run; row sums are 4 DPP adds
// (row_mirror, row_half_mirror, quad swaps) instead of LDS shuffles.
template <int CTRL>
SM_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
SM_DEV float sum16(float v) {
  v += dppf<0x140>(v);   // row_mirror
  v += dppf<0x141>(v);   // row_half_mirror
  v += dppf<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dppf<0xB1>(v);    // quad_perm [1,0,3,2]
  return v;
}

template <typename TI, typename TO, int C>
__global__ __launch_bounds__(256) void ln_fwd16_kernel(const TI* x, const float* g, const float* b, TO* y,
                                                       float* mean, float* rstd, int64_t M, float eps,
                                                       int64_t rows_per_block) {
  constexpr int U = C / 64;
  const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  float gg[U][4], bb[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    load4(g + 64 * u + 4 * gl, gg[u]);
    load4(b + 64 * u + 4 * gl, bb[u]);
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  for (int64_t row = r0 + grp; row < r1; row += 16) {
    const TI* xr = x + row * C + 4 * gl;
    float v[U][4];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load4_nt(xr + 64 * u, v[u]);
      s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
    }
    const float mu = sum16(s) * (1.f / C);
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[u][j] - mu; ss += d * d; }
    const float rs = rsqrtf(sum16(ss) * (1.f / C) + eps);
    TO* yr = y + row * C + 4 * gl;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[u][j] - mu) * rs * gg[u][j] + bb[u][j];
      store4(yr + 64 * u, o);   // (read back by the next GEMM: a normal store measured faster for bf16 x)
    }
    if (gl == 0) { mean[row] = mu; rstd[row] = rs; }
  }
}

// dx (+ dres) and per-block partial dgamma / dbeta (part_g/part_b [block][C]).
// Branch copy (bo != null): the transformer block's backward feeds dx to the residual
// stream AND, through the branch regularisers' backward, to the branch's Linear:
// bo = bf16(bf16(dx) * rs[row / rpg] * keep(row, col) / (1 - p)), i.e. the cast
// (fp32 stream) and sm_dropout_bwd passes over dx folded into this one (same mask,
// same roundings: bit-identical).
struct LnBranch {
  __bf16* bo;
  float p;
  uint64_t seed;
  const float* rs;
  int64_t rpg;
};

// C = 384 runs 32 lanes per row (2 rows per wave, 8 per block in flight): 3 chunks of 4
// columns per lane, as at C = 192, instead of 6 -- the 16-lane form held xhat, gamma dy and
// the dgamma / dbeta partials of 24 columns per lane (188 VGPRs, 2 waves per SIMD; 3.9-4.1
// TB/s where the C = 192 form, 116 VGPRs and 4 waves, streams at 5.2).
template <int C>
constexpr int ln_bwd_lanes() { return C >= 384 ? 32 : 16; }

template <typename TI, typename TD, int C>
__global__ __launch_bounds__(256) void ln_bwd16_kernel(const TD* dy, const TI* x, const float* mean,
                                                       const float* rstd, const float* g, TI* dx, float* part_g,
                                                       float* part_b, int64_t M, int64_t rows_per_block,
                                                       const TI* dres, LnBranch br) {
  constexpr int G = ln_bwd_lanes<C>();   // lanes per row
  constexpr int U = C / (4 * G);         // 4-column chunks per lane, columns 4G u + 4 gl + j
  constexpr int RG = 256 / G;            // rows of a block in flight
  static_assert(U * 4 * G == C, "C must split over the row's lanes");
  __shared__ float red[2][4][C];
  const int gl = threadIdx.x & (G - 1), grp = threadIdx.x / G, w = threadIdx.x >> 6;
  float gw[U][4], ag[U][4], ab[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    load4(g + 4 * G * u + 4 * gl, gw[u]);
#pragma unroll
    for (int j = 0; j < 4; ++j) { ag[u][j] = 0.f; ab[u][j] = 0.f; }
  }
  auto row_sum = [](float v) {
    v = sum16(v);
    if constexpr (G == 32) v += __shfl_xor(v, 16, 64);
    return v;
  };
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  for (int64_t row = r0 + grp; row < r1; row += RG) {
    const float mu = mean[row], rs = rstd[row];
    const int64_t e0 = row * C + 4 * gl;
    float xh[U][4], gy[U][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float xv[4], dv[4];
      load4_nt(x + e0 + 4 * G * u, xv);
      load4_nt(dy + e0 + 4 * G * u, dv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[u][j] = (xv[j] - mu) * rs;
        gy[u][j] = dv[j] * gw[u][j];
        s1 += gy[u][j];
        s2 += gy[u][j] * xh[u][j];
        ag[u][j] += dv[j] * xh[u][j];
        ab[u][j] += dv[j];
      }
    }
    s1 = row_sum(s1) * (1.f / C);
    s2 = row_sum(s2) * (1.f / C);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (gy[u][j] - s1 - xh[u][j] * s2);
      if (dres) {
        float pr[4];
        load4_nt(dres + e0 + 4 * G * u, pr);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += pr[j];
      }
      store4_nt(dx + e0 + 4 * G * u, o);
      if (br.bo) {
        const float rsv = br.rs ? br.rs[row / br.rpg] : 1.f;
        const float ks = br.p > 0.f ? drop_scale(br.p) : 1.f;
        const uint32_t hsh = br.p > 0.f ? drop_hash(drop_rowbase(seed32(br.seed), (uint64_t)row),
                                                     (uint32_t)(4 * G * u + 4 * gl)) : 0u;
        const uint32_t thr = drop_thr(br.p);
        float b4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = (float)(__bf16)to_f<TI>(from_f<TI>(o[j]));   // the stored dx, cast to bf16
          const float mj = br.p > 0.f ? (((hsh >> (8 * j)) & 0xFFu) >= thr ? ks : 0.f) : 1.f;
          b4[j] = d * (rsv * mj);
        }
        store4_nt(br.bo + e0 + 4 * G * u, b4);
      }
    }
  }
  // column partials: the row groups of a wave, then the 4 waves (fixed order)
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = ag[u][j], c = ab[u][j];
      if constexpr (G == 16) {
        a += __shfl_xor(a, 16, 64);
        c += __shfl_xor(c, 16, 64);
      }
      a += __shfl_xor(a, 32, 64);
      c += __shfl_xor(c, 32, 64);
      ag[u][j] = a;
      ab[u][j] = c;
    }
  if ((threadIdx.x & 63) < G) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[0][w][4 * G * u + 4 * gl + j] = ag[u][j];
        red[1][w][4 * G * u + 4 * gl + j] = ab[u][j];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part_g[(int64_t)blockIdx.x * C + c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    part_b[(int64_t)blockIdx.x * C + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
  }
}

// ============================================================ BatchNorm (train)
// Thread layout shared by the column-reduction kernels: thread t owns the 4-wide
// channel chunk t % (C/4) and rows r = t / (C/4) (mod rows-per-pass).
struct ColMap {
  int nch, rpp, chunk, r;
  SM_DEV ColMap(int C) {
    nch = C / 4;
    rpp = 256 / nch;
    if (rpp < 1) rpp = 1;
    chunk = threadIdx.x % nch;
    r = threadIdx.x / nch;
  }
  SM_DEV bool active() const { return r < rpp && chunk < nch; }
};

template <typename T>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* x, int64_t M, int C, int64_t ld, int rows_per_block,
                                                       float* part /*[nb][2][C]*/) {
  __shared__ float red[2][256 * 4];
  ColMap cm(C);
  float s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  float shift[4];
  load4(x + cm.chunk * 4, shift);   // per-channel shift = first row (robust variance)
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  if (cm.active()) {
    for (int64_t row = r0 + cm.r; row < r1; row += cm.rpp) {
      float v[4];
      load4(x + row * ld + cm.chunk * 4, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) { const float d = v[j] - shift[j]; s[j] += d; q[j] += d * d; }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) { red[0][threadIdx.x * 4 + j] = s[j]; red[1][threadIdx.x * 4 + j] = q[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int ch = c / 4, j = c % 4;
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < cm.rpp; ++rr) {
      const int t = rr * cm.nch + ch;
      a += red[0][t * 4 + j];
      b += red[1][t * 4 + j];
    }
    part[((int64_t)blockIdx.x * 2 + 0) * C + c] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

template <typename T>
__global__ void bn_finalize_kernel(const double* sums /*[2][C]*/, const T* x, int64_t M, int C, float eps,
                                   float momentum, float* mean_out, float* rstd_out, float* run_mean,
                                   float* run_var, int updates, int64_t* nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) *nbt += updates;
  if (c >= C) return;
  const double s = sums[c], q = sums[C + c];
  const double shift = x ? (double)to_f<T>(x[c]) : 0.0;   // null: unshifted partials
  const double md = s / (double)M;
  double var = q / (double)M - md * md;
  if (var < 0) var = 0;
  const double mean = shift + md;
  mean_out[c] = (float)mean;
  rstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    float rm = run_mean[c], rv = run_var[c];
    for (int u = 0; u < updates; ++u) {
      rm = (1.f - momentum) * rm + momentum * (float)mean;
      rv = (1.f - momentum) * rv + momentum * (float)unb;
    }
    run_mean[c] = rm;
    run_var[c] = rv;
  }
}

// Channel-owning layout for [M][C] streaming kernels: thread t owns the 8-channel
// chunk t % (C/8) for rows t / (C/8) (+ k * rows-per-pass); per-channel parameters
// live in registers and rows are walked with 16-byte loads.
struct Col8 {
  int nch, rpp, chunk, r;
  SM_DEV Col8(int C) {
    nch = C / 8;
    rpp = 256 / nch;
    if (rpp < 1) rpp = 1;
    chunk = threadIdx.x % nch;
    r = threadIdx.x / nch;
  }
  SM_DEV bool active() const { return r < rpp; }
};

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void bn_apply_kernel(const TI* x, const float* mean, const float* rstd,
                                                       const float* w, const float* b, TO* y, int64_t M, int C,
                                                       int rows_per_block, int gelu, const TO* R,
                                                       const float* row_scale, int64_t rpg, ChanAffine raff) {
  Col8 cm(C);
  if (!cm.active()) return;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cm.chunk * 8 + j;
    sc[j] = rstd[c] * w[c];
    sh[j] = bn_shift(b[c], mean[c], sc[j]);
  }
  // residual stored pre-BatchNorm (raff.mean != null): R's value is the BN output
  // bf16(R * rsc + rsh) exactly as bn_apply would have stored it (no GELU)
  Affine8 ra;
  ra.init(raff, cm.chunk * 8);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  for (int64_t row = r0 + cm.r; row < r1; row += cm.rpp) {
    const int64_t e = row * C + cm.chunk * 8;
    float v[8];
    load8_nt(x + e, v);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {   // packed pairs (gelu_phi_pair_t); = Affine8::apply
      f32x2 t = vfma(f32x2{v[j], v[j + 1]}, f32x2{sc[j], sc[j + 1]}, f32x2{sh[j], sh[j + 1]});
      if (gelu) t = gelu_f2(t);
      v[j] = t.x;
      v[j + 1] = t.y;
    }
    if (row_scale) {
      const float rs = row_scale[row / rpg];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= rs;
    }
    if (R) {
      float rr[8];
      load8_nt(R + e, rr);
      ra.apply<TO>(rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += rr[j];
    }
    store8_nt(y + e, v);
  }
}

// per-channel sums of g and g*x_hat where g = dy (* gelu'(bn(x)) when gelu)
template <typename TI, typename TD>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const TD* dy, const TI* x, const float* mean,
                                                            const float* rstd, const float* w, const float* b,
                                                            int64_t M, int C, int64_t ld, int rows_per_block,
                                                            int gelu, const float* row_scale, int64_t rpg,
                                                            float* part) {
  __shared__ float red[2][256 * 4];
  ColMap cm(C);
  float sg[4] = {0, 0, 0, 0}, sgx[4] = {0, 0, 0, 0};
  float mu[4], rs[4], ww[4], bb[4];
  if (cm.active()) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = cm.chunk * 4 + j;
      mu[j] = mean[c]; rs[j] = rstd[c]; ww[j] = w[c]; bb[j] = b[c];
    }
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(M, r0 + rows_per_block);
    for (int64_t row = r0 + cm.r; row < r1; row += cm.rpp) {
      float xv[4], dv[4];
      load4_nt(x + row * ld + cm.chunk * 4, xv);
      load4_nt(dy + row * ld + cm.chunk * 4, dv);
      const float rsc = row_scale ? row_scale[row / rpg] : 1.f;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {   // packed pairs (gelu_phi_pair_t)
        const f32x2 xh = (f32x2{xv[j], xv[j + 1]} - f32x2{mu[j], mu[j + 1]}) * f32x2{rs[j], rs[j + 1]};
        f32x2 gg = f32x2{dv[j], dv[j + 1]} * rsc;
        if (gelu) gg *= gelu_grad2(vfma(xh, f32x2{ww[j], ww[j + 1]}, f32x2{bb[j], bb[j + 1]}));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          sg[j + i] += gg[i];
          sgx[j + i] += gg[i] * xh[i];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) { red[0][threadIdx.x * 4 + j] = sg[j]; red[1][threadIdx.x * 4 + j] = sgx[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int ch = c / 4, j = c % 4;
    float a = 0.f, bsum = 0.f;
    for (int rr = 0; rr < cm.rpp; ++rr) {
      const int t = rr * cm.nch + ch;
      a += red[0][t * 4 + j];
      bsum += red[1][t * 4 + j];
    }
    part[((int64_t)blockIdx.x * 2 + 0) * C + c] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = bsum;
  }
}

// sums -> dgamma (+=), dbeta (+=), and the two per-channel coefficients for dx
__global__ void bn_bwd_finalize_kernel(const double* sums /*[2][C]*/, int64_t M, int C, float* dw, float* db,
                                       float* coef /*[2][C]: mean(g), mean(g*xhat)*/) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double a = sums[c], b = sums[C + c];
  if (dw) dw[c] += (float)b;
  if (db) db[c] += (float)a;
  coef[c] = (float)(a / (double)M);
  coef[C + c] = (float)(b / (double)M);
}

template <typename TI, typename TD, typename TX>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const TD* dy, const TI* x, const float* mean,
                                                        const float* rstd, const float* w, const float* b,
                                                        const float* coef, TX* dx, int64_t M, int C, int64_t ld,
                                                        int rows_per_block, int gelu, const float* row_scale,
                                                        int64_t rpg) {
  Col8 cm(C);
  if (!cm.active()) return;
  float mu[8], rs[8], ww[8], bb[8], k0[8], k1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cm.chunk * 8 + j;
    mu[j] = mean[c]; rs[j] = rstd[c]; ww[j] = w[c]; bb[j] = b[c];
    k0[j] = coef[c]; k1[j] = coef[C + c];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  // two rows per step with both rows' inputs loaded first (dx may alias dy)
  auto one = [&](int64_t row, const float (&xv)[8], const float (&dv)[8]) {
    const int64_t e = row * ld + cm.chunk * 8;
    float o[8];
    const float rsc = row_scale ? row_scale[row / rpg] : 1.f;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {   // packed pairs (gelu_phi_pair_t)
      const f32x2 xh = (f32x2{xv[j], xv[j + 1]} - f32x2{mu[j], mu[j + 1]}) * f32x2{rs[j], rs[j + 1]};
      f32x2 gg = f32x2{dv[j], dv[j + 1]} * rsc;
      if (gelu) gg *= gelu_grad2(vfma(xh, f32x2{ww[j], ww[j + 1]}, f32x2{bb[j], bb[j + 1]}));
#pragma unroll
      for (int i = 0; i < 2; ++i) o[j + i] = ww[j + i] * rs[j + i] * (gg[i] - k0[j + i] - xh[i] * k1[j + i]);
    }
    store8(dx + e, o);   // (read next by the branch GEMM: normal store, +1 % with nt)
  };
  int64_t row = r0 + cm.r;
  for (; row + cm.rpp < r1; row += 2 * cm.rpp) {
    const int64_t e0 = row * ld + cm.chunk * 8, e1 = e0 + (int64_t)cm.rpp * ld;
    float x0[8], d0[8], x1[8], d1[8];
    load8_nt(x + e0, x0);
    load8_nt(dy + e0, d0);
    load8_nt(x + e1, x1);
    load8_nt(dy + e1, d1);
    one(row, x0, d0);
    one(row + cm.rpp, x1, d1);
  }
  if (row < r1) {
    const int64_t e0 = row * ld + cm.chunk * 8;
    float x0[8], d0[8];
    load8_nt(x + e0, x0);
    load8_nt(dy + e0, d0);
    one(row, x0, d0);
  }
}

// ============================================================ elementwise
// 8 consecutive elements of one row (ncols % 8 == 0): dropout multipliers
SM_DEV void drop_mult8(int64_t e, int ncols, float drop_p, uint64_t seed, float* m) {
  const float ks = drop_scale(drop_p);
  const int64_t row = e / ncols;
  const uint32_t c0 = (uint32_t)(e - row * ncols);
  const uint32_t rb = drop_rowbase(seed32(seed), (uint64_t)row), thr = drop_thr(drop_p);
#pragma unroll
  for (int j4 = 0; j4 < 8; j4 += 4) {
    const uint32_t h = drop_hash(rb, c0 + j4);    // c0 % 8 == 0
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j4 + j] = ((h >> (8 * j)) & 0xFFu) >= thr ? ks : 0.f;
  }
}

template <typename T, typename TG>
__global__ void gelu_bwd_kernel(const T* pre, const TG* dy, TG* dx, int64_t total8, int ncols, float drop_p,
                                uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float p[8], d[8], m[8];
    load8(pre + i * 8, p);
    load8(dy + i * 8, d);
    if (drop_p > 0.f) drop_mult8(i * 8, ncols, drop_p, seed, m);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 gd = gelu_grad2(f32x2{p[j], p[j + 1]});
      d[j] *= (drop_p > 0.f ? m[j] : 1.f) * gd.x;
      d[j + 1] *= (drop_p > 0.f ? m[j + 1] : 1.f) * gd.y;
    }
    store8(dx + i * 8, d);
  }
}

// dx = dy * dropout_mask * row_scale[row / rpg]   (backward of the branch regularisers);
// TO = bf16 < T = fp32: the autocast cast of the fp32 stream's gradient to the bf16
// branch folded in (dy rounded to bf16 first, as the separate cast pass stores it)
template <typename T, typename TO = T>
__global__ void dropout_bwd_kernel(const T* dy, TO* dx, int64_t total8, int ncols, float drop_p, uint64_t seed,
                                   const float* row_scale, int64_t rpg) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float d[8], m[8];
    load8(dy + i * 8, d);
    if (sizeof(TO) < sizeof(T)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = to_f<TO>(from_f<TO>(d[j]));
    }
    const int64_t e = i * 8;
    const float rs = row_scale ? row_scale[(e / ncols) / rpg] : 1.f;
    if (drop_p > 0.f) drop_mult8(e, ncols, drop_p, seed, m);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= rs * (drop_p > 0.f ? m[j] : 1.f);
    store8(dx + i * 8, d);
  }
}

__global__ void droppath_scale_kernel(int n, float p, uint64_t seed, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = drop_keep(seed32(seed), (uint64_t)i, 0u, drop_thr(p)) ? drop_scale(p) : 0.f;
}

template <typename TA, typename TB, typename TO>
__global__ void add_kernel(const TA* a, const TB* b, TO* o, int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float x[8], y[8];
    load8(a + i * 8, x);
    load8(b + i * 8, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += y[j];
    store8(o + i * 8, x);
  }
}

template <typename TA, typename TO>
__global__ void cast_kernel(const TA* a, TO* o, int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float x[8];
    load8(a + i * 8, x);
    store8(o + i * 8, x);
  }
}

template <typename T>
__global__ void gelu_fwd_kernel(const T* x, T* y, int64_t total8, int ncols, float drop_p, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[8], m[8];
    load8(x + i * 8, v);
    if (drop_p > 0.f) drop_mult8(i * 8, ncols, drop_p, seed, m);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 gv = gelu_f2(f32x2{v[j], v[j + 1]});
      v[j] = gv.x * (drop_p > 0.f ? m[j] : 1.f);
      v[j + 1] = gv.y * (drop_p > 0.f ? m[j + 1] : 1.f);
    }
    store8(y + i * 8, v);
  }
}

// per-block column partial sums of x [M][C]
template <typename T>
__global__ __launch_bounds__(256) void colsum_part_kernel(const T* x, int64_t ld, int64_t M, int C,
                                                          int rows_per_block, float* part) {
  __shared__ float red[256 * 4];
  ColMap cm(C);
  float s[4] = {0, 0, 0, 0};
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  if (cm.active())
    for (int64_t row = r0 + cm.r; row < r1; row += cm.rpp) {
      float v[4];
      load4(x + row * ld + cm.chunk * 4, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[j];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int ch = c / 4, j = c % 4;
    float a = 0.f;
    for (int rr = 0; rr < cm.rpp; ++rr) a += red[(rr * cm.nch + ch) * 4 + j];
    part[(int64_t)blockIdx.x * C + c] = a;
  }
}

inline int ew_blocks(int64_t n8) {
  int64_t b = (n8 + 255) / 256;
  if (b > 8192) b = 8192;
  return b < 1 ? 1 : (int)b;
}
// rows per block for the channel-owning streaming kernels (~4096 blocks)
inline int stream_rows_per_block(int64_t M) {
  int64_t r = (M + 4095) / 4096;
  if (r < 16) r = 16;
  return (int)r;
}
inline int red_rows_per_block(int64_t M, int C) {
  // aim for ~2048 blocks, at least 64 rows each
  int64_t r = (M + 2047) / 2048;
  if (r < 64) r = 64;
  return (int)r;
}

}  // namespace

#define DISPATCH2(DT1, DT2, ...)                                                           \
  do {                                                                                   \
    if ((DT1) == SM_F32 && (DT2) == SM_F32) { typedef float T1; typedef float T2; __VA_ARGS__; }     \
    else if ((DT1) == SM_F32 && (DT2) == SM_BF16) { typedef float T1; typedef __bf16 T2; __VA_ARGS__; } \
    else if ((DT1) == SM_BF16 && (DT2) == SM_F32) { typedef __bf16 T1; typedef float T2; __VA_ARGS__; } \
    else { typedef __bf16 T1; typedef __bf16 T2; __VA_ARGS__; }                          \
  } while (0)

extern "C" int sm_layernorm_fwd(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* gamma,
                                const float* beta, void* y, float* mean, float* rstd, float eps,
                                hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 4 || C > 1024) return -2;
  if (C == 384 || C == 192) {
    int64_t rpb = ((M + 4095) / 4096 + 15) / 16 * 16;   // ~4096 blocks, 16-row multiples
    if (rpb < 16) rpb = 16;
    const int nb = (int)((M + rpb - 1) / rpb);
    if (C == 384)
      DISPATCH2(x_dtype, y_dtype,
                hipLaunchKernelGGL((ln_fwd16_kernel<T1, T2, 384>), dim3(nb), dim3(256), 0, st, (const T1*)x, gamma,
                                   beta, (T2*)y, mean, rstd, M, eps, rpb));
    else
      DISPATCH2(x_dtype, y_dtype,
                hipLaunchKernelGGL((ln_fwd16_kernel<T1, T2, 192>), dim3(nb), dim3(256), 0, st, (const T1*)x, gamma,
                                   beta, (T2*)y, mean, rstd, M, eps, rpb));
    SM_CHECK_LAUNCH();
    return 0;
  }
  const int blocks = (int)((M + 3) / 4);
  DISPATCH2(x_dtype, y_dtype,
            hipLaunchKernelGGL((ln_fwd_kernel<T1, T2>), dim3(blocks), dim3(256), 0, st, (const T1*)x, gamma,
                               beta, (T2*)y, mean, rstd, M, C, eps));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t sm_layernorm_bwd_workspace_bytes(int64_t M, int C) {
  const int64_t rpb = red_rows_per_block(M, C);
  const int64_t nb = (M + rpb - 1) / rpb;
  return nb * C * 4 * 2;
}

static int layernorm_bwd(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy, const void* x,
                         const float* mean, const float* rstd, const float* gamma, void* dx, const void* dres,
                         float* dgamma, float* dbeta, void* ws, int64_t ws_bytes, LnBranch br, hipStream_t st);

// dx (+)= LN backward; dgamma/dbeta (+)= (accumulated into the fp32 grad sinks)
extern "C" int sm_layernorm_bwd(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy,
                                const void* x, const float* mean, const float* rstd, const float* gamma,
                                void* dx, const void* dres, float* dgamma, float* dbeta, void* ws,
                                int64_t ws_bytes, hipStream_t st) {
  return layernorm_bwd(x_dtype, dy_dtype, dx_dtype, M, C, dy, x, mean, rstd, gamma, dx, dres, dgamma, dbeta, ws,
                       ws_bytes, LnBranch{nullptr, 0.f, 0, nullptr, 1}, st);
}

// sm_layernorm_bwd plus the branch copy dxb = bf16(bf16(dx) * row_scale[row / rpg] *
// dropout keep / (1 - p)) (C = 192 or 384)
extern "C" int sm_layernorm_bwd_branch(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy,
                                       const void* x, const float* mean, const float* rstd, const float* gamma,
                                       void* dx, const void* dres, float* dgamma, float* dbeta, void* dxb,
                                       float drop_p, uint64_t seed, const float* row_scale, int64_t rows_per_group,
                                       void* ws, int64_t ws_bytes, hipStream_t st) {
  if (C != 192 && C != 384) return -2;
  if (dxb == nullptr || rows_per_group <= 0 || ((uintptr_t)dxb & 7)) return -2;
  return layernorm_bwd(x_dtype, dy_dtype, dx_dtype, M, C, dy, x, mean, rstd, gamma, dx, dres, dgamma, dbeta, ws,
                       ws_bytes, LnBranch{(__bf16*)dxb, drop_p, seed, row_scale, rows_per_group}, st);
}

static int layernorm_bwd(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy, const void* x,
                         const float* mean, const float* rstd, const float* gamma, void* dx, const void* dres,
                         float* dgamma, float* dbeta, void* ws, int64_t ws_bytes, LnBranch br, hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 4 || C > 1024) return -2;
  const int rpb = red_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  if (ws_bytes < (int64_t)nb * C * 8) return -4;
  float* pg = (float*)ws;
  float* pb = pg + (int64_t)nb * C;
  if (x_dtype != dx_dtype) return -3;   // dx has the dtype of the LN input stream
  if (C == 384)
    DISPATCH2(x_dtype, dy_dtype,
              hipLaunchKernelGGL((ln_bwd16_kernel<T1, T2, 384>), dim3(nb), dim3(256), 0, st, (const T2*)dy,
                                 (const T1*)x, mean, rstd, gamma, (T1*)dx, pg, pb, M, (int64_t)rpb, (const T1*)dres, br));
  else if (C == 192)
    DISPATCH2(x_dtype, dy_dtype,
              hipLaunchKernelGGL((ln_bwd16_kernel<T1, T2, 192>), dim3(nb), dim3(256), 0, st, (const T2*)dy,
                                 (const T1*)x, mean, rstd, gamma, (T1*)dx, pg, pb, M, (int64_t)rpb, (const T1*)dres, br));
  else
    DISPATCH2(x_dtype, dy_dtype,
              hipLaunchKernelGGL((ln_bwd_kernel<T1, T2, T1>), dim3(nb), dim3(256), 0, st, (const T2*)dy,
                                 (const T1*)x, mean, rstd, gamma, (T1*)dx, pg, pb, M, C, rpb, (const T1*)dres));
  SM_CHECK_LAUNCH();
  colred(pg, nb, C, nullptr, dgamma, 1, st);
  colred(pb, nb, C, nullptr, dbeta, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t sm_bn_workspace_bytes(int64_t M, int C) {
  const int64_t rpb = red_rows_per_block(M, C);
  const int64_t nb = (M + rpb - 1) / rpb;
  return nb * 2 * C * 4 + 2 * C * 8 + 2 * C * 4 + 64;
}

// batch statistics -> mean/rstd (+ running-stat update `updates` times).  Channels
// above 1024 (stage-4 MBConv, 1536) are processed in column slices of the same
// [M][C] rows (row stride C).
static const int BN_MAX_SLICE = 1024;

static int bn_stats_slice(int x_dtype, int64_t M, int C, int64_t ld, const void* x, float* mean, float* rstd,
                          float* run_mean, float* run_var, int64_t* nbt, float momentum, float eps, int updates,
                          float* part, double* sums, hipStream_t st) {
  const int rpb = red_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  if (x_dtype == SM_BF16) {
    hipLaunchKernelGGL(bn_stats_kernel<__bf16>, dim3(nb), dim3(256), 0, st, (const __bf16*)x, M, C, ld, rpb, part);
    colred(part, nb, 2 * C, sums, nullptr, 0, st);
    hipLaunchKernelGGL(bn_finalize_kernel<__bf16>, dim3((C + 127) / 128), dim3(128), 0, st, sums,
                       (const __bf16*)x, M, C, eps, momentum, mean, rstd, run_mean, run_var, updates, nbt);
  } else {
    hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)x, M, C, ld, rpb, part);
    colred(part, nb, 2 * C, sums, nullptr, 0, st);
    hipLaunchKernelGGL(bn_finalize_kernel<float>, dim3((C + 127) / 128), dim3(128), 0, st, sums,
                       (const float*)x, M, C, eps, momentum, mean, rstd, run_mean, run_var, updates, nbt);
  }
  return 0;
}

extern "C" int sm_bn_stats(int x_dtype, int64_t M, int C, const void* x, float* mean, float* rstd,
                           float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum, float eps,
                           int updates, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (M <= 0) return -2;
  if (C % 4 || C > 4 * BN_MAX_SLICE || (C > BN_MAX_SLICE && C % 8)) return -2;
  const int rpb = red_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  if (ws_bytes < (int64_t)nb * 2 * C * 4 + 2 * C * 8 + 8) return -4;
  float* part = (float*)ws;
  double* sums = (double*)(((uintptr_t)(part + (int64_t)nb * 2 * C) + 7) & ~(uintptr_t)7);
  const int nsl = (C + BN_MAX_SLICE - 1) / BN_MAX_SLICE;
  const int w = nsl == 1 ? C : (C / nsl + 7) / 8 * 8;
  const size_t es = x_dtype == SM_BF16 ? 2 : 4;
  for (int c0 = 0; c0 < C; c0 += w) {
    const int cs = min(w, C - c0);
    bn_stats_slice(x_dtype, M, cs, C, (const char*)x + c0 * es, mean + c0, rstd + c0,
                   run_mean ? run_mean + c0 : nullptr, run_var ? run_var + c0 : nullptr,
                   c0 == 0 ? num_batches_tracked : nullptr, momentum, eps, updates, part, sums, st);
  }
  SM_CHECK_LAUNCH();
  return 0;
}

// eval-mode BatchNorm (running statistics): mean = running_mean, rstd = 1/sqrt(var + eps),
// in the form every BN consumer (bn_apply, the folded ChanAffine loads) takes
__global__ void bn_eval_params_kernel(const float* run_mean, const float* run_var, int C, float eps, float* mean,
                                      float* rstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  rstd[c] = 1.0f / sqrtf(run_var[c] + eps);
}

extern "C" int sm_bn_eval_params(const float* run_mean, const float* run_var, int C, float eps, float* mean,
                                 float* rstd, hipStream_t st) {
  if (C <= 0) return -2;
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps,
                     mean, rstd);
  SM_CHECK_LAUNCH();
  return 0;
}

// BatchNorm statistics from per-block partials [nrows][2][C] (sum, sum of squares,
// unshifted) produced inside another kernel (e.g. the fused depthwise conv): fixed-order
// fp64 column reduction + the same finalize / running-stat update as sm_bn_stats.
extern "C" int64_t sm_bn_partials_workspace_bytes(int C) { return (int64_t)2 * C * 8; }

extern "C" int sm_bn_stats_from_partials(const float* part, int64_t nrows, int C, int64_t M, float* mean,
                                         float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                                         float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                                         hipStream_t st) {
  if (M <= 0 || nrows <= 0 || nrows > 0x7fffffff) return -2;
  if (ws_bytes < (int64_t)2 * C * 8) return -4;
  double* sums = (double*)ws;
  colred(part, (int)nrows, 2 * C, sums, nullptr, 0, st);
  hipLaunchKernelGGL(bn_finalize_kernel<__bf16>, dim3((C + 127) / 128), dim3(128), 0, st, sums,
                     (const __bf16*)nullptr, M, C, eps, momentum, mean, rstd, run_mean, run_var, updates,
                     num_batches_tracked);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_bn_apply(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* mean,
                           const float* rstd, const float* w, const float* b, void* y, int gelu,
                           const void* R, const float* row_scale, int64_t rows_per_group, hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 8 || C / 8 > 256) return -2;
  const int rpb = stream_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  DISPATCH2(x_dtype, y_dtype,
            hipLaunchKernelGGL((bn_apply_kernel<T1, T2>), dim3(nb), dim3(256), 0, st, (const T1*)x,
                               mean, rstd, w, b, (T2*)y, M, C, rpb, gelu, (const T2*)R, row_scale,
                               rows_per_group > 0 ? rows_per_group : 1, ChanAffine{}));
  SM_CHECK_LAUNCH();
  return 0;
}

// sm_bn_apply with the residual R stored before its own BatchNorm (the stem's conv2 output
// a2 when BN2's apply is folded into stage 0's consumers): R's value is bf16(R * r_sc +
// r_sh) with r_sc = r_rstd * r_w, r_sh = r_b - r_mean * r_sc, exactly as sm_bn_apply stores
// the BN output, so y is bit-identical to sm_bn_apply(.., R = sm_bn_apply(R, r_*)).
extern "C" int sm_bn_apply_res_bn(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* mean,
                                  const float* rstd, const float* w, const float* b, void* y, int gelu,
                                  const void* R, const float* r_mean, const float* r_rstd, const float* r_w,
                                  const float* r_b, const float* row_scale, int64_t rows_per_group,
                                  hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 8 || C / 8 > 256 || R == nullptr || r_mean == nullptr || r_rstd == nullptr || r_w == nullptr ||
      r_b == nullptr)
    return -2;
  const int rpb = stream_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  const ChanAffine raff{r_mean, r_rstd, r_w, r_b, 0};
  DISPATCH2(x_dtype, y_dtype,
            hipLaunchKernelGGL((bn_apply_kernel<T1, T2>), dim3(nb), dim3(256), 0, st, (const T1*)x,
                               mean, rstd, w, b, (T2*)y, M, C, rpb, gelu, (const T2*)R, row_scale,
                               rows_per_group > 0 ? rows_per_group : 1, raff));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_bn_bwd(int x_dtype, int g_dtype, int64_t M, int C, const void* dy, const void* x,
                         const float* mean, const float* rstd, const float* w, const float* b, int gelu,
                         const float* row_scale, int64_t rows_per_group, void* dx, float* dw, float* db, void* ws,
                         int64_t ws_bytes, hipStream_t st) {
  const int64_t rpg = rows_per_group > 0 ? rows_per_group : 1;
  if (M <= 0) return 0;
  if (C % 8 || C > 4 * BN_MAX_SLICE) return -2;
  const int rpb = red_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  if (ws_bytes < (int64_t)nb * 2 * C * 4 + 2 * C * 8 + 2 * C * 4 + 8) return -4;
  float* part = (float*)ws;
  double* sums = (double*)(((uintptr_t)(part + (int64_t)nb * 2 * C) + 7) & ~(uintptr_t)7);
  float* coef = (float*)(sums + 2 * C);
  const int srpb = stream_rows_per_block(M);
  const int snb = (int)((M + srpb - 1) / srpb);
  const int nsl = (C + BN_MAX_SLICE - 1) / BN_MAX_SLICE;
  const int wd = (C / nsl + 7) / 8 * 8;
  const size_t xs = x_dtype == SM_BF16 ? 2 : 4, gs = g_dtype == SM_BF16 ? 2 : 4;
  for (int c0 = 0; c0 < C; c0 += wd) {   // channel slices of <= 1024 over the same rows
    const int cs = min(wd, C - c0);
    const void* xo = (const char*)x + c0 * xs;
    const void* dyo = (const char*)dy + c0 * gs;
    void* dxo = (char*)dx + c0 * gs;
    DISPATCH2(x_dtype, g_dtype,
              hipLaunchKernelGGL((bn_bwd_reduce_kernel<T1, T2>), dim3(nb), dim3(256), 0, st, (const T2*)dyo,
                                 (const T1*)xo, mean + c0, rstd + c0, w + c0, b + c0, M, cs, (int64_t)C, rpb, gelu,
                                 row_scale, rpg, part));
    colred(part, nb, 2 * cs, sums, nullptr, 0, st);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((cs + 127) / 128), dim3(128), 0, st, sums, M, cs, dw + c0,
                       db + c0, coef);
    DISPATCH2(x_dtype, g_dtype,
              hipLaunchKernelGGL((bn_bwd_dx_kernel<T1, T2, T2>), dim3(snb), dim3(256), 0, st,
                                 (const T2*)dyo, (const T1*)xo, mean + c0, rstd + c0, w + c0, b + c0, coef, (T2*)dxo,
                                 M, cs, (int64_t)C, srpb, gelu, row_scale, rpg));
  }
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_gelu_bwd(int pre_dtype, int g_dtype, int64_t n, int ncols, const void* pre, const void* dy,
                           void* dx, float drop_p, uint64_t seed, hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8) return -2;
  DISPATCH2(pre_dtype, g_dtype,
            hipLaunchKernelGGL((gelu_bwd_kernel<T1, T2>), dim3(ew_blocks(n / 8)), dim3(256), 0, st,
                               (const T1*)pre, (const T2*)dy, (T2*)dx, n / 8, ncols, drop_p, seed));
  SM_CHECK_LAUNCH();
  return 0;
}

// o = a + b  (a: a_dtype, b/o: o_dtype)
extern "C" int sm_add(int a_dtype, int o_dtype, int64_t n, const void* a, const void* b, void* o, hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8) return -2;
  DISPATCH2(a_dtype, o_dtype,
            hipLaunchKernelGGL((add_kernel<T1, T2, T2>), dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const T1*)a,
                               (const T2*)b, (T2*)o, n / 8));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_cast(int a_dtype, int o_dtype, int64_t n, const void* a, void* o, hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8) return -2;
  DISPATCH2(a_dtype, o_dtype,
            hipLaunchKernelGGL((cast_kernel<T1, T2>), dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const T1*)a,
                               (T2*)o, n / 8));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t sm_colsum_workspace_bytes(int64_t M, int C) {
  const int64_t rpb = red_rows_per_block(M, C);
  return ((M + rpb - 1) / rpb) * C * 4;
}

// out[c] (+)= sum_m x[m][c]   (bias gradients)
extern "C" int sm_colsum(int dtype, int64_t M, int C, const void* x, float* out, int accumulate, void* ws,
                         int64_t ws_bytes, hipStream_t st) {
  if (M <= 0) return 0;
  if (C % 4) return -2;
  const int rpb = red_rows_per_block(M, C);
  const int nb = (int)((M + rpb - 1) / rpb);
  if (ws_bytes < (int64_t)nb * C * 4) return -4;
  const int esz = dtype == SM_BF16 ? 2 : 4;
  for (int c0 = 0; c0 < C; c0 += 1024) {       // 1024-column slices (ColMap covers <= 256 chunks of 4)
    const int cs = C - c0 < 1024 ? C - c0 : 1024;
    const char* xs = (const char*)x + (int64_t)c0 * esz;
    float* part = (float*)ws;
    if (dtype == SM_BF16)
      hipLaunchKernelGGL(colsum_part_kernel<__bf16>, dim3(nb), dim3(256), 0, st, (const __bf16*)xs, (int64_t)C, M,
                         cs, rpb, part);
    else
      hipLaunchKernelGGL(colsum_part_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)xs, (int64_t)C, M, cs,
                         rpb, part);
    colred(part, nb, cs, nullptr, out + c0, accumulate, st);
  }
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_gelu_fwd(int dtype, int64_t n, int ncols, const void* x, void* y, float drop_p, uint64_t seed,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8) return -2;
  if (dtype == SM_BF16)
    hipLaunchKernelGGL(gelu_fwd_kernel<__bf16>, dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const __bf16*)x,
                       (__bf16*)y, n / 8, ncols, drop_p, seed);
  else
    hipLaunchKernelGGL(gelu_fwd_kernel<float>, dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const float*)x, (float*)y,
                       n / 8, ncols, drop_p, seed);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_dropout_bwd(int dtype, int64_t n, int ncols, const void* dy, void* dx, float drop_p, uint64_t seed,
                              const float* row_scale, int64_t rows_per_group, hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8 || ncols % 8) return -2;
  const int64_t rpg = rows_per_group > 0 ? rows_per_group : 1;
  if (dtype == SM_BF16)
    hipLaunchKernelGGL(dropout_bwd_kernel<__bf16>, dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const __bf16*)dy,
                       (__bf16*)dx, n / 8, ncols, drop_p, seed, row_scale, rpg);
  else
    hipLaunchKernelGGL(dropout_bwd_kernel<float>, dim3(ew_blocks(n / 8)), dim3(256), 0, st, (const float*)dy,
                       (float*)dx, n / 8, ncols, drop_p, seed, row_scale, rpg);
  SM_CHECK_LAUNCH();
  return 0;
}

// cast fp32 -> bf16 and dropout backward in one pass (the decoder block's fp32 residual
// gradient entering its bf16 branch): bit-identical to sm_cast + sm_dropout_bwd
extern "C" int sm_cast_dropout_bwd(int64_t n, int ncols, const float* dy, void* dx_bf16, float drop_p, uint64_t seed,
                                   const float* row_scale, int64_t rows_per_group, hipStream_t st) {
  if (n <= 0) return 0;
  if (n % 8 || ncols % 8) return -2;
  const int64_t rpg = rows_per_group > 0 ? rows_per_group : 1;
  hipLaunchKernelGGL((dropout_bwd_kernel<float, __bf16>), dim3(ew_blocks(n / 8)), dim3(256), 0, st, dy,
                     (__bf16*)dx_bf16, n / 8, ncols, drop_p, seed, row_scale, rpg);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_droppath_scale(int n, float p, uint64_t seed, float* out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(droppath_scale_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, p, seed, out);
  SM_CHECK_LAUNCH();
  return 0;
}
