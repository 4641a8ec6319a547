// Convolution-side kernels of the TinyViT encoder, channels-last ([frames][H][W][C]).
//
//  * stem im2col (PatchEmbed conv1 3->48 k3 s2, tiny_vit.py:67) reads the clip
//    [B,3,T,H,W] through strides, so the reference's frame permute copy
//    (mae_vit_adapter.py:84) never exists; K order (ci,ky,kx), padded to 32.
//  * generic 3x3 im2col / col2im for stem conv2 (48->96 k3 s1, tiny_vit.py:69),
//    K order (ky,kx,ci) so each tap is one contiguous channel run.
//  * conv weight pack/unpack between the reference's [Cout][Cin][3][3] layout and
//    the GEMM's [Cout][Kpad] layout.
//  * depthwise 3x3 conv (MBConv, tiny_vit.py:46) fwd, dgrad, wgrad; 8 channels/thread.
//  * SE layer (tiny_vit.py:20-34): per-frame channel mean, the two tiny FCs fused
//    per frame, and the broadcast scale, each with its backward.
#include "common.h"
#include "sm_api.h"

namespace {

inline int ew_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  return b < 1 ? 1 : (int)b;
}

// ------------------------------------------------------------------ stem im2col
struct ClipView {
  const float* p;
  int B, T, H, W;
  int64_t sB, sC, sT, sH, sW;
};

template <typename TO>
__global__ void stem_im2col_kernel(ClipView v, int Ho, int Wo, int stride, TO* col /*[F*Ho*Wo][32]*/) {
  const int64_t P = (int64_t)v.B * v.T * Ho * Wo;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % Wo);
    const int64_t r = i / Wo;
    const int yo = (int)(r % Ho);
    const int64_t f = r / Ho;
    const int t = (int)(f % v.T), b = (int)(f / v.T);
    const float* base = v.p + b * v.sB + t * v.sT;
    float vals[32];
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int yi = yo * stride + ky - 1, xi = xo * stride + kx - 1;
          float x = 0.f;
          if (yi >= 0 && yi < v.H && xi >= 0 && xi < v.W) x = base[ci * v.sC + yi * v.sH + xi * v.sW];
          vals[ci * 9 + ky * 3 + kx] = x;
        }
#pragma unroll
    for (int k = 27; k < 32; ++k) vals[k] = 0.f;
    TO* o = col + i * 32;
#pragma unroll
    for (int k = 0; k < 32; k += 8) store8(o + k, vals + k);
  }
}

// ------------------------------------------------------------------ 3x3 im2col (NHWC)
template <typename T>
__global__ void im2col3_kernel(const T* x, int F, int H, int W, int C, int Ho, int Wo, int stride,
                               T* col /*[F*Ho*Wo][9*C]*/) {
  const int cc = C / 8;
  const int64_t total = (int64_t)F * Ho * Wo * 9 * cc;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cc);
    int64_t r = i / cc;
    const int tap = (int)(r % 9);
    r /= 9;
    const int xo = (int)(r % Wo);
    r /= Wo;
    const int yo = (int)(r % Ho);
    const int64_t f = r / Ho;
    const int yi = yo * stride + tap / 3 - 1, xi = xo * stride + tap % 3 - 1;
    float v[8];
    if (yi >= 0 && yi < H && xi >= 0 && xi < W) load8(x + (((f * H + yi) * W + xi) * C + c8 * 8), v);
    else for (int j = 0; j < 8; ++j) v[j] = 0.f;
    store8(col + ((((f * Ho + yo) * Wo + xo) * 9 + tap) * C + c8 * 8), v);
  }
}

// dx[f][yi][xi][c] = sum over taps of dcol[f][yo][xo][tap][c]  (gather form)
template <typename T>
__global__ void col2im3_kernel(const T* dcol, int F, int H, int W, int C, int Ho, int Wo, int stride, T* dx) {
  const int cc = C / 8;
  const int64_t total = (int64_t)F * H * W * cc;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cc);
    int64_t r = i / cc;
    const int xi = (int)(r % W);
    r /= W;
    const int yi = (int)(r % H);
    const int64_t f = r / H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ty = yi + 1 - ky, tx = xi + 1 - kx;
        if (ty < 0 || tx < 0 || ty % stride || tx % stride) continue;
        const int yo = ty / stride, xo = tx / stride;
        if (yo >= Ho || xo >= Wo) continue;
        float v[8];
        load8(dcol + ((((f * Ho + yo) * Wo + xo) * 9 + ky * 3 + kx) * C + c8 * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    store8(dx + (((f * H + yi) * W + xi) * C + c8 * 8), acc);
  }
}

// ------------------------------------------------------------------ weight pack
// src [Cout][Cin][3][3] fp32 -> dst [Cout][Kpad]; order 0: k=(ci*9+ky*3+kx); 1: k=(ky*3+kx)*Cin+ci
template <typename TO>
__global__ void wpack_kernel(const float* src, TO* dst, int Cout, int Cin, int Kpad, int order) {
  const int total = Cout * Kpad;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int co = i / Kpad, k = i % Kpad;
    float v = 0.f;
    if (k < Cin * 9) {
      int ci, tap;
      if (order == 0) { ci = k / 9; tap = k % 9; }
      else { tap = k / Cin; ci = k % Cin; }
      v = src[(co * Cin + ci) * 9 + tap];
    }
    dst[i] = from_f<TO>(v);
  }
}

__global__ void wunpack_add_kernel(const float* packed, float* grad, int Cout, int Cin, int Kpad, int order) {
  const int total = Cout * Cin * 9;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int co = i / (Cin * 9), rem = i % (Cin * 9), ci = rem / 9, tap = rem % 9;
    const int k = order == 0 ? ci * 9 + tap : tap * Cin + ci;
    grad[i] += packed[co * Kpad + k];
  }
}

// ------------------------------------------------------------------ depthwise 3x3
// One thread = 8 channels (16-B vectors) x PX consecutive output pixels of one row;
// the 72 taps stay in registers and each input vector feeds every output it
// touches (4.5 loads/output at stride 1, 6.75 at stride 2, instead of 9).
constexpr int DW_PX = 4;

template <typename T, int S>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* x, const float* w /*[C][9]*/, T* y, int F, int H,
                                                     int W, int C, int Ho, int Wo) {
  constexpr int PX = DW_PX, NIN = (PX - 1) * S + 3;
  const int cc = C / 8;
  const int nxs = (Wo + PX - 1) / PX;
  const int64_t total = (int64_t)F * Ho * nxs * cc;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % cc);
  int64_t r = idx / cc;
  const int xs = (int)(r % nxs);
  r /= nxs;
  const int yo = (int)(r % Ho);
  const int64_t f = r / Ho;
  float wr[9][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wr[t][j] = w[(c8 * 8 + j) * 9 + t];
  float acc[PX][8];
#pragma unroll
  for (int p = 0; p < PX; ++p)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[p][j] = 0.f;
  const int xo0 = xs * PX;
  const int xi0 = xo0 * S - 1;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yi = yo * S + ky - 1;
    if (yi < 0 || yi >= H) continue;
    const T* row = x + ((f * H + yi) * W) * C + c8 * 8;
#pragma unroll
    for (int ci = 0; ci < NIN; ++ci) {
      const int xi = xi0 + ci;
      if (xi < 0 || xi >= W) continue;
      float v[8];
      load8(row + (int64_t)xi * C, v);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        const int kx = ci - p * S;
        if (kx < 0 || kx > 2) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[p][j] += v[j] * wr[ky * 3 + kx][j];
      }
    }
  }
#pragma unroll
  for (int p = 0; p < PX; ++p)
    if (xo0 + p < Wo) store8(y + (((f * Ho + yo) * Wo + xo0 + p) * C + c8 * 8), acc[p]);
}

// dx[yi][xi] = sum_{ky,kx} dy[(yi+1-ky)/S][(xi+1-kx)/S] w[ky][kx] (terms with exact division)
template <typename T, int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const T* dy, const float* w, T* dx, int F, int H, int W,
                                                       int C, int Ho, int Wo) {
  constexpr int PX = DW_PX;
  constexpr int NCOL = S == 1 ? PX + 2 : PX / 2 + 1;   // dy columns touched by the strip
  const int cc = C / 8;
  const int nxs = (W + PX - 1) / PX;
  const int64_t total = (int64_t)F * H * nxs * cc;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % cc);
  int64_t r = idx / cc;
  const int xs = (int)(r % nxs);
  r /= nxs;
  const int yi = (int)(r % H);
  const int64_t f = r / H;
  float wr[9][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wr[t][j] = w[(c8 * 8 + j) * 9 + t];
  float acc[PX][8];
#pragma unroll
  for (int p = 0; p < PX; ++p)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[p][j] = 0.f;
  const int xi0 = xs * PX;                       // even (PX even)
  const int xob = S == 1 ? xi0 - 1 : xi0 / 2;    // first dy column of the strip
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int ty = yi + 1 - ky;
    if (ty < 0) continue;
    if (S == 2 && (ty & 1)) continue;
    const int yo = ty / S;
    if (yo >= Ho) continue;
    const T* row = dy + ((f * Ho + yo) * Wo) * C + c8 * 8;
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int xo = xob + k;
      if (xo < 0 || xo >= Wo) continue;
      float v[8];
      load8(row + (int64_t)xo * C, v);
#pragma unroll
      for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int d = p + 1 - kx;            // xi + 1 - kx relative to xi0
          bool hit;
          if (S == 1) hit = (d + 1 == k);
          else hit = (d >= 0) && !(d & 1) && (d / 2 == k);
          if (!hit) continue;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[p][j] += v[j] * wr[ky * 3 + kx][j];
        }
    }
  }
#pragma unroll
  for (int p = 0; p < PX; ++p)
    if (xi0 + p < W) store8(dx + (((f * H + yi) * W + xi0 + p) * C + c8 * 8), acc[p]);
}

// partial dw per block: part[blk][C][9]
template <typename T>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* dy, const T* x, int F, int H, int W, int C, int Ho,
                                                       int Wo, int stride, int64_t pix_per_block, float* part) {
  __shared__ float red[256 * 8];
  const int cc = C / 8;
  const int rpp = 256 / cc;
  const int c8 = threadIdx.x % cc, rr = threadIdx.x / cc;
  float acc[72];
#pragma unroll
  for (int k = 0; k < 72; ++k) acc[k] = 0.f;
  const int64_t P = (int64_t)F * Ho * Wo;
  const int64_t p0 = blockIdx.x * pix_per_block;
  const int64_t p1 = min(P, p0 + pix_per_block);
  if (rr < rpp) {
    for (int64_t p = p0 + rr; p < p1; p += rpp) {
      const int xo = (int)(p % Wo);
      const int64_t q = p / Wo;
      const int yo = (int)(q % Ho);
      const int64_t f = q / Ho;
      float g[8];
      load8(dy + p * C + c8 * 8, g);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int yi = yo * stride + ky - 1;
        if (yi < 0 || yi >= H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int xi = xo * stride + kx - 1;
          if (xi < 0 || xi >= W) continue;
          float v[8];
          load8(x + (((f * H + yi) * W + xi) * C + c8 * 8), v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j * 9 + ky * 3 + kx] += g[j] * v[j];
        }
      }
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = acc[j * 9 + tap];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int ch = c / 8, j = c % 8;
      float s = 0.f;
      for (int r2 = 0; r2 < rpp; ++r2) s += red[(r2 * cc + ch) * 8 + j];
      part[(int64_t)blockIdx.x * C * 9 + c * 9 + tap] = s;
    }
    __syncthreads();
  }
}

__global__ void colsum_add_kernel(const float* part, int nb, int n, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[(int64_t)b * n + c];
  out[c] += (float)s;
}

// ------------------------------------------------------------------ SE
// pooled[f][c] = mean_hw x[f][hw][c]   (block per frame)
template <typename T>
__global__ __launch_bounds__(256) void se_pool_kernel(const T* x, int HW, int C, float* pooled) {
  __shared__ float red[256 * 4];
  const int nch = C / 4;
  const int rpp = 256 / nch;
  const int ch = threadIdx.x % nch, r = threadIdx.x / nch;
  const int64_t f = blockIdx.x;
  float s[4] = {0, 0, 0, 0};
  if (r < rpp)
    for (int p = r; p < HW; p += rpp) {
      float v[4];
      load4(x + ((f * HW + p) * C + ch * 4), v);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[j];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int rr = 0; rr < rpp; ++rr) a += red[(rr * nch + c / 4) * 4 + c % 4];
    pooled[f * C + c] = a / HW;
  }
}

// per frame: z1 = W1 p; h1 = relu(z1); z2 = W2 h1; s = sigmoid(z2)
__global__ __launch_bounds__(256) void se_fc_fwd_kernel(const float* pooled, const float* w1 /*[R][C]*/,
                                                        const float* w2 /*[C][R]*/, int C, int R, float* h1_out,
                                                        float* s_out) {
  extern __shared__ float sh[];
  float* p = sh;          // C
  float* h = sh + C;      // R
  const int64_t f = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) p[c] = pooled[f * C + c];
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int j = w; j < R; j += 4) {
    float s = 0.f;
    for (int c = l; c < C; c += 64) s += w1[(int64_t)j * C + c] * p[c];
    s = wave_sum(s);
    if (l == 0) { h[j] = fmaxf(s, 0.f); h1_out[f * R + j] = fmaxf(s, 0.f); }   // relu(z1) saved
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int j = 0; j < R; ++j) s += w2[(int64_t)c * R + j] * h[j];
    s_out[f * C + c] = 1.f / (1.f + __expf(-s));
  }
}

// y = x * s[f][c]
template <typename T>
__global__ void se_scale_kernel(const T* x, const float* s, T* y, int64_t HW, int C, int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 8;
    const int64_t f = e / (HW * C);
    const int c0 = (int)(e % C);
    float v[8];
    load8(x + e, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s[f * C + c0 + j];
    store8(y + e, v);
  }
}

// ds[f][c] = sum_hw dy * x      (block per frame)
template <typename T>
__global__ __launch_bounds__(256) void se_dscale_kernel(const T* dy, const T* x, int HW, int C, float* ds) {
  __shared__ float red[256 * 4];
  const int nch = C / 4;
  const int rpp = 256 / nch;
  const int ch = threadIdx.x % nch, r = threadIdx.x / nch;
  const int64_t f = blockIdx.x;
  float s[4] = {0, 0, 0, 0};
  if (r < rpp)
    for (int p = r; p < HW; p += rpp) {
      float a[4], b[4];
      load4(dy + ((f * HW + p) * C + ch * 4), a);
      load4(x + ((f * HW + p) * C + ch * 4), b);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += a[j] * b[j];
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int rr = 0; rr < rpp; ++rr) a += red[(rr * nch + c / 4) * 4 + c % 4];
    ds[f * C + c] = a;
  }
}

// per frame backward through sigmoid / W2 / relu / W1:
//   dz2 = ds * s (1-s);  dh1 = W2^T dz2;  dz1 = dh1 * (z1 > 0);  dpool = W1^T dz1
__global__ __launch_bounds__(256) void se_fc_bwd_kernel(const float* ds, const float* s, const float* z1,
                                                        const float* w1, const float* w2, int C, int R,
                                                        float* dz2_out, float* dz1_out, float* dpool) {
  extern __shared__ float sh[];
  float* dz2 = sh;      // C
  float* dz1 = sh + C;  // R
  const int64_t f = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float sv = s[f * C + c];
    const float g = ds[f * C + c] * sv * (1.f - sv);
    dz2[c] = g;
    dz2_out[f * C + c] = g;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int j = w; j < R; j += 4) {
    float a = 0.f;
    for (int c = l; c < C; c += 64) a += w2[(int64_t)c * R + j] * dz2[c];
    a = wave_sum(a);
    if (l == 0) {
      const float g = z1[f * R + j] > 0.f ? a : 0.f;   // z1 holds relu(z1): same support
      dz1[j] = g;
      dz1_out[f * R + j] = g;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int j = 0; j < R; ++j) a += w1[(int64_t)j * C + c] * dz1[j];
    dpool[f * C + c] = a;
  }
}

// dx = dy * s + dpool / HW
template <typename T>
__global__ void se_dx_kernel(const T* dy, const float* s, const float* dpool, T* dx, int64_t HW, int C,
                             int64_t total8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 8;
    const int64_t f = e / (HW * C);
    const int c0 = (int)(e % C);
    float v[8];
    load8(dy + e, v);
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * s[f * C + c0 + j] + dpool[f * C + c0 + j] * inv;
    store8(dx + e, v);
  }
}

}  // namespace

#define DISPATCH1(DT, ...)                                       \
  do {                                                         \
    if ((DT) == SM_F32) { typedef float T; __VA_ARGS__; }      \
    else { typedef __bf16 T; __VA_ARGS__; }                    \
  } while (0)

extern "C" int sm_stem_im2col(int out_dtype, const float* clip, int B, int T, int H, int W, int64_t sB, int64_t sC,
                              int64_t sT, int64_t sH, int64_t sW, int stride, void* col, hipStream_t st) {
  ClipView v{clip, B, T, H, W, sB, sC, sT, sH, sW};
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t P = (int64_t)B * T * Ho * Wo;
  if (P <= 0) return 0;
  DISPATCH1(out_dtype, hipLaunchKernelGGL(stem_im2col_kernel<T>, dim3(ew_blocks(P)), dim3(256), 0, st, v, Ho, Wo,
                                          stride, (T*)col));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_im2col3(int dtype, const void* x, int F, int H, int W, int C, int stride, void* col,
                          hipStream_t st) {
  if (C % 8) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t total = (int64_t)F * Ho * Wo * 9 * (C / 8);
  if (total <= 0) return 0;
  DISPATCH1(dtype, hipLaunchKernelGGL(im2col3_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, st, (const T*)x, F,
                                      H, W, C, Ho, Wo, stride, (T*)col));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_col2im3(int dtype, const void* dcol, int F, int H, int W, int C, int stride, void* dx,
                          hipStream_t st) {
  if (C % 8) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t total = (int64_t)F * H * W * (C / 8);
  if (total <= 0) return 0;
  DISPATCH1(dtype, hipLaunchKernelGGL(col2im3_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, st, (const T*)dcol,
                                      F, H, W, C, Ho, Wo, stride, (T*)dx));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_conv_wpack(int out_dtype, const float* src, void* dst, int Cout, int Cin, int Kpad, int order,
                             hipStream_t st) {
  const int total = Cout * Kpad;
  DISPATCH1(out_dtype, hipLaunchKernelGGL(wpack_kernel<T>, dim3((total + 255) / 256), dim3(256), 0, st, src,
                                          (T*)dst, Cout, Cin, Kpad, order));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_conv_wunpack_add(const float* packed, float* grad, int Cout, int Cin, int Kpad, int order,
                                   hipStream_t st) {
  const int total = Cout * Cin * 9;
  hipLaunchKernelGGL(wunpack_add_kernel, dim3((total + 255) / 256), dim3(256), 0, st, packed, grad, Cout, Cin, Kpad,
                     order);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_dwconv_fwd(int dtype, const void* x, const float* w, void* y, int F, int H, int W, int C,
                             int stride, hipStream_t st) {
  if (C % 8) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t total = (int64_t)F * Ho * ((Wo + DW_PX - 1) / DW_PX) * (C / 8);
  if (total <= 0) return 0;
  const int nb = (int)((total + 255) / 256);
  if (stride == 1)
    DISPATCH1(dtype, hipLaunchKernelGGL((dw_fwd_kernel<T, 1>), dim3(nb), dim3(256), 0, st, (const T*)x, w, (T*)y, F,
                                        H, W, C, Ho, Wo));
  else if (stride == 2)
    DISPATCH1(dtype, hipLaunchKernelGGL((dw_fwd_kernel<T, 2>), dim3(nb), dim3(256), 0, st, (const T*)x, w, (T*)y, F,
                                        H, W, C, Ho, Wo));
  else
    return -2;
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t sm_dwconv_wgrad_workspace_bytes(int F, int H, int W, int C, int stride) {
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t P = (int64_t)F * Ho * Wo;
  int64_t ppb = (P + 1023) / 1024;
  if (ppb < 64) ppb = 64;
  const int64_t nb = (P + ppb - 1) / ppb;
  return nb * C * 9 * 4;
}

extern "C" int sm_dwconv_bwd(int dtype, const void* dy, const void* x, const float* w, void* dx, float* dw, int F,
                             int H, int W, int C, int stride, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (C % 8 || C / 8 > 256) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t P = (int64_t)F * Ho * Wo;
  if (P <= 0) return 0;
  if (stride != 1 && stride != 2) return -2;
  if (dx) {
    const int64_t total = (int64_t)F * H * ((W + DW_PX - 1) / DW_PX) * (C / 8);
    const int nb = (int)((total + 255) / 256);
    if (stride == 1)
      DISPATCH1(dtype, hipLaunchKernelGGL((dw_dgrad_kernel<T, 1>), dim3(nb), dim3(256), 0, st, (const T*)dy, w,
                                          (T*)dx, F, H, W, C, Ho, Wo));
    else
      DISPATCH1(dtype, hipLaunchKernelGGL((dw_dgrad_kernel<T, 2>), dim3(nb), dim3(256), 0, st, (const T*)dy, w,
                                          (T*)dx, F, H, W, C, Ho, Wo));
  }
  int64_t ppb = (P + 1023) / 1024;
  if (ppb < 64) ppb = 64;
  const int nb = (int)((P + ppb - 1) / ppb);
  if (ws_bytes < (int64_t)nb * C * 9 * 4) return -4;
  float* part = (float*)ws;
  DISPATCH1(dtype, hipLaunchKernelGGL(dw_wgrad_kernel<T>, dim3(nb), dim3(256), 0, st, (const T*)dy,
                                      (const T*)x, F, H, W, C, Ho, Wo, stride, ppb, part));
  colred(part, nb, C * 9, nullptr, dw, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_se_fwd(int dtype, const void* x, int F, int HW, int C, int R, const float* w1, const float* w2,
                         float* pooled, float* z1, float* s, void* y, hipStream_t st) {
  if (C % 8 || C / 4 > 256) return -2;
  DISPATCH1(dtype, hipLaunchKernelGGL(se_pool_kernel<T>, dim3(F), dim3(256), 0, st, (const T*)x, HW, C, pooled));
  hipLaunchKernelGGL(se_fc_fwd_kernel, dim3(F), dim3(256), (C + R) * 4, st, pooled, w1, w2, C, R, z1, s);
  const int64_t n8 = (int64_t)F * HW * C / 8;
  DISPATCH1(dtype, hipLaunchKernelGGL(se_scale_kernel<T>, dim3(ew_blocks(n8)), dim3(256), 0, st, (const T*)x, s,
                                      (T*)y, (int64_t)HW, C, n8));
  SM_CHECK_LAUNCH();
  return 0;
}

// Backward of y = x * sigmoid(W2 relu(W1 mean_hw(x))).  Writes dx and the per-frame
// FC gradients dz2 [F][C], dz1 [F][R] (the weight grads are two small GEMMs).
extern "C" int sm_se_bwd(int dtype, const void* dy, const void* x, int F, int HW, int C, int R, const float* w1,
                         const float* w2, const float* s, const float* z1, float* ds_ws, float* dz2, float* dz1,
                         float* dpool_ws, void* dx, hipStream_t st) {
  if (C % 8 || C / 4 > 256) return -2;
  DISPATCH1(dtype, hipLaunchKernelGGL(se_dscale_kernel<T>, dim3(F), dim3(256), 0, st, (const T*)dy, (const T*)x,
                                      HW, C, ds_ws));
  hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(F), dim3(256), (C + R) * 4, st, ds_ws, s, z1, w1, w2, C, R, dz2, dz1,
                     dpool_ws);
  const int64_t n8 = (int64_t)F * HW * C / 8;
  DISPATCH1(dtype, hipLaunchKernelGGL(se_dx_kernel<T>, dim3(ew_blocks(n8)), dim3(256), 0, st, (const T*)dy, s,
                                      dpool_ws, (T*)dx, (int64_t)HW, C, n8));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_se_scale(int dtype, const void* x, const float* s, void* y, int F, int HW, int C, hipStream_t st) {
  if (C % 8) return -2;
  const int64_t n8 = (int64_t)F * HW * C / 8;
  if (n8 <= 0) return 0;
  DISPATCH1(dtype, hipLaunchKernelGGL(se_scale_kernel<T>, dim3(ew_blocks(n8)), dim3(256), 0, st, (const T*)x, s,
                                      (T*)y, (int64_t)HW, C, n8));
  SM_CHECK_LAUNCH();
  return 0;
}
