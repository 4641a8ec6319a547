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
#include <algorithm>

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

// ------------------------------------------------------------------ stem conv1, direct
// PatchEmbed conv1 (tiny_vit.py:67: 3 -> 48, 3x3, stride 2, pad 1) straight from the fp32
// clip, no im2col buffer: a wave takes 32 consecutive output pixels, each lane gathers its
// pixel's 16 of the 32 (ci, ky, kx) inputs (K order of stem_im2col, 27 -> 32) as bf16
// A-operand fragments of two v_mfma_f32_32x32x16_bf16 steps per 32-channel block (the
// same products and order as the im2col GEMM's single K-step: bit-identical a1).  Output
// lane = channel, registers = 16 pixels: the BatchNorm-1 sums of the stored bf16 values
// are two registers per lane and block; the bf16 tile goes through a per-wave LDS image
// [32 px][48 ch] to 16-B row stores.  One fixed-order reduction per block ->
// part[block][2][48].  Tap offsets are wave-uniform (scalar) per lane half.
constexpr int SC1_BLOCKS = 2048, SC1_COUT = 48, SC1_PITCH = 56;   // image row: 48 ch + 8 pad (bf16)

__global__ __launch_bounds__(256, 4) void stem_conv1_kernel(ClipView v, int Ho, int Wo, const __bf16* w /*[48][32]*/,
                                                         __bf16* y /*[P][48]*/, float* part /*[grid][2][48]*/) {
  __shared__ __attribute__((aligned(16))) __bf16 img[4][32 * SC1_PITCH];
  __shared__ float red[4][2][64];
  const int l = threadIdx.x & 63, h = l >> 5, wv = threadIdx.x >> 6;
  const int P = v.B * v.T * Ho * Wo;   // host: < 2^31
  const int nseg = (P + 31) / 32;
  bf16x8 wf[2][2];   // B fragments: co = 32 j + (l & 31), k = 16 s + 8 h + 0..7
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int co = 32 * j + (l & 31);
      if (co < SC1_COUT) wf[j][s] = *(const bf16x8*)(w + co * 32 + 16 * s + 8 * h);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) wf[j][s][e] = (__bf16)0.f;
    }
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};   // channel 32 j + (l & 31), this lane's pixels
  const int HWo = Ho * Wo;
  __bf16* im = img[wv];
  for (int seg = blockIdx.x * 4 + wv; seg < nseg; seg += gridDim.x * 4) {
    const int px = seg * 32 + (l & 31);
    const bool ok = px < P;
    const int f = px / HWo, rem = px - f * HWo;
    const int yo = rem / Wo, xo = rem - yo * Wo;
    const float* base = v.p + (int64_t)(f / v.T) * v.sB + (int64_t)(f % v.T) * v.sT + (2 * yo) * v.sH + (2 * xo) * v.sW;
    bf16x8 af[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // k = 16 s + 8 h + e: both halves' taps are compile-time, the offsets scalar
        const int k0 = 16 * s + e, k1 = k0 + 8;
        const int ky = h ? (k1 % 9) / 3 : (k0 % 9) / 3, kx = h ? k1 % 3 : k0 % 3;
        const bool kin = h ? k1 < 27 : k0 < 27;
        const int off = h ? (int)((k1 / 9) * v.sC + ((k1 % 9) / 3 - 1) * v.sH + (k1 % 3 - 1) * v.sW)
                          : (int)((k0 / 9) * v.sC + ((k0 % 9) / 3 - 1) * v.sH + (k0 % 3 - 1) * v.sW);
        const int yi = 2 * yo + ky - 1, xi = 2 * xo + kx - 1;
        // unconditional loads (padding reads the clip's first element, then zero): the
        // sixteen gathers issue back to back instead of one branch each
        const bool in = ok && kin && (unsigned)yi < (unsigned)v.H && (unsigned)xi < (unsigned)v.W;
        const float x = *(in ? base + off : v.p);
        af[s][e] = (__bf16)(in ? x : 0.f);
      }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], wf[j][s], acc, 0, 0, 0);
      const int co = 32 * j + (l & 31);
      if (co < SC1_COUT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {   // pixel (r & 3) + 8 (r >> 2) + 4 h of the segment
          const int pp = (r & 3) + 8 * (r >> 2) + 4 * h;
          const __bf16 o = (__bf16)acc[r];
          if (seg * 32 + pp < P) {
            const float of = (float)o;
            s1[j] += of;
            s2[j] = fmaf(of, of, s2[j]);
          }
          im[pp * SC1_PITCH + co] = o;
        }
      }
    }
    // the wave's [32 px][48 ch] image -> 16-B runs (6 per pixel, 3 per lane)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = l + 64 * i, pp = c / 6, ch = c - pp * 6;
      const uint4 val = *(const uint4*)(im + pp * SC1_PITCH + ch * 8);
      if (seg * 32 + pp < P) *(uint4*)(y + (int64_t)(seg * 32 + pp) * SC1_COUT + ch * 8) = val;
    }
  }
  // fixed-order reduction: the two halves of each wave (the same channels), then the 4 waves
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    s1[j] += __shfl_xor(s1[j], 32, 64);
    s2[j] += __shfl_xor(s2[j], 32, 64);
  }
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      red[wv][0][32 * j + l] = s1[j];
      red[wv][1][32 * j + l] = s2[j];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * SC1_COUT) {
    const int which = threadIdx.x / SC1_COUT, co = threadIdx.x % SC1_COUT;
    part[((int64_t)blockIdx.x * 2 + which) * SC1_COUT + co] =
        ((red[0][which][co] + red[1][which][co]) + red[2][which][co]) + red[3][which][co];
  }
}

// Band form (round 4): a block walks bands of SC1B_R output rows of one frame.  The band's
// 2 R + 1 input rows of the three channels are first staged into LDS as bf16 with
// coalesced loads (16-B loads of 4 consecutive pixels when the clip rows are contiguous and
// aligned), each input element loaded once; the per-pixel 27-tap gathers then read LDS.
// (The gathering kernel above loads every input ~2.25 times, half-coalesced at stride 2:
// its waves waited on those loads 85 % of their cycles, profiles/r03q_stem_pmc.txt.)  The
// A fragments, MFMA products and their order are the gathering kernel's, so a1 is
// bit-identical; the BatchNorm-1 sums are taken in another order (fp32 rounding).
constexpr int SC1B_R = 8, SC1B_NRI = 2 * SC1B_R + 1, SC1B_PADL = 4;

__global__ __launch_bounds__(256, 2) void stem_conv1_band_kernel(ClipView v, int Ho, int Wo, const __bf16* w,
                                                              __bf16* y, float* part, int vec4) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  __shared__ __attribute__((aligned(16))) __bf16 img[4][32 * SC1_PITCH];
  __shared__ float red[4][2][64];
  const int WP = v.W + 2 * SC1B_PADL;                 // staged row pitch (bf16), zero pads both sides
  __bf16* xs = (__bf16*)dyn;                          // [3][SC1B_NRI][WP]
  const int l = threadIdx.x & 63, h = l >> 5, wv = threadIdx.x >> 6;
  const int nbf = (Ho + SC1B_R - 1) / SC1B_R;
  const int nbands = v.B * v.T * nbf;
  bf16x8 wf[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int co = 32 * j + (l & 31);
      if (co < SC1_COUT) wf[j][s] = *(const bf16x8*)(w + co * 32 + 16 * s + 8 * h);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) wf[j][s][e] = (__bf16)0.f;
    }
  // zero pads (columns [0, PADL) and [PADL + W, WP) of every staged row): never overwritten
  for (int i = threadIdx.x; i < 3 * SC1B_NRI * 2 * SC1B_PADL; i += 256) {
    const int row = i / (2 * SC1B_PADL), c = i % (2 * SC1B_PADL);
    xs[row * WP + (c < SC1B_PADL ? c : v.W + c)] = (__bf16)0.f;
  }
  // this lane's 16 taps (k = 16 s + 8 h + e): channel-row base and column offset, compile-time
  // (k >= 27, the K padding: -1, read as zero)
  int toff[2][8];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 16 * s + e + 8 * h;
      // staged row ci * NRI + ky (+ 2 ry), column kx - 1 + PADL (+ 2 xo)
      toff[s][e] = k < 27 ? ((k / 9) * SC1B_NRI + (k % 9) / 3) * WP + k % 3 - 1 + SC1B_PADL : -1;
    }
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  __bf16* im = img[wv];
  const int rowlen = SC1B_NRI * v.W;
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int f = band / nbf, yo0 = (band - f * nbf) * SC1B_R;
    const int reff = min(SC1B_R, Ho - yo0);
    const float* base = v.p + (int64_t)(f / v.T) * v.sB + (int64_t)(f % v.T) * v.sT;
    const int yi0 = 2 * yo0 - 1;
    __syncthreads();   // the previous band's gathers are done with xs
    if (vec4) {        // sW == 1, W % 4 == 0, 16-B aligned rows
      const int q = v.W >> 2;
      for (int i = threadIdx.x; i < 3 * SC1B_NRI * q; i += 256) {
        const int cr = i / q, x4 = (i - cr * q) * 4;
        const int ci = cr / SC1B_NRI, r = cr - ci * SC1B_NRI, yi = yi0 + r;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)yi < (unsigned)v.H) val = *(const float4*)(base + ci * v.sC + (int64_t)yi * v.sH + x4);
        bf16x4 b4 = {(__bf16)val.x, (__bf16)val.y, (__bf16)val.z, (__bf16)val.w};
        *(bf16x4*)(xs + cr * WP + SC1B_PADL + x4) = b4;
      }
    } else {
      for (int i = threadIdx.x; i < 3 * rowlen; i += 256) {
        const int ci = i / rowlen, rem = i - ci * rowlen, r = rem / v.W, x = rem - r * v.W, yi = yi0 + r;
        float val = 0.f;
        if ((unsigned)yi < (unsigned)v.H) val = base[ci * v.sC + (int64_t)yi * v.sH + (int64_t)x * v.sW];
        xs[(ci * SC1B_NRI + r) * WP + SC1B_PADL + x] = (__bf16)val;
      }
    }
    __syncthreads();
    const int npx = reff * Wo, nseg = (npx + 31) / 32;
    const int64_t px0 = ((int64_t)f * Ho + yo0) * Wo;   // the band's first output pixel
    for (int seg = wv; seg < nseg; seg += 4) {
      const int p = min(seg * 32 + (l & 31), npx - 1);    // pixels past the band: recomputed, not stored
      const int ry = p / Wo, xo = p - ry * Wo;
      const int rb = 2 * ry * WP + 2 * xo;
      bf16x8 af[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) af[s][e] = toff[s][e] >= 0 ? xs[toff[s][e] + rb] : (__bf16)0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], wf[j][s], acc, 0, 0, 0);
        const int co = 32 * j + (l & 31);
        if (co < SC1_COUT) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int pp = (r & 3) + 8 * (r >> 2) + 4 * h;
            const __bf16 o = (__bf16)acc[r];
            if (seg * 32 + pp < npx) {
              const float of = (float)o;
              s1[j] += of;
              s2[j] = fmaf(of, of, s2[j]);
            }
            im[pp * SC1_PITCH + co] = o;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int c = l + 64 * i, pp = c / 6, ch = c - pp * 6;
        const uint4 val = *(const uint4*)(im + pp * SC1_PITCH + ch * 8);
        if (seg * 32 + pp < npx) *(uint4*)(y + (px0 + seg * 32 + pp) * SC1_COUT + ch * 8) = val;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    s1[j] += __shfl_xor(s1[j], 32, 64);
    s2[j] += __shfl_xor(s2[j], 32, 64);
  }
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      red[wv][0][32 * j + l] = s1[j];
      red[wv][1][32 * j + l] = s2[j];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * SC1_COUT) {
    const int which = threadIdx.x / SC1_COUT, co = threadIdx.x % SC1_COUT;
    part[((int64_t)blockIdx.x * 2 + which) * SC1_COUT + co] =
        ((red[0][which][co] + red[1][which][co]) + red[2][which][co]) + red[3][which][co];
  }
}

// ------------------------------------------------------------------ stem conv2, direct
// PatchEmbed conv2 (tiny_vit.py:69: 48 -> 96, 3x3, stride 1, pad 1) over h1 =
// GELU(BN1(a1)) (tiny_vit.py:68) with BN2's statistics (tiny_vit.py:70): block = one
// frame, walked in bands of SC2_R output rows.  BN1 + GELU is applied ONCE per input
// element while a row enters an LDS ring of h1 rows (zero halo = the conv's padding of
// h1), so neither h1 nor a 9x im2col exists in HBM.  12 waves = 3 channel blocks x 4
// pixel segments of 32.  The packed weights [96][432] stay in LDS for the block; per
// band and tap row each wave loads its 32 channels' 9 B fragments into registers and
// reads the pixel A fragments from the ring (ds_read_b128; 112-B pixel and 880-B
// weight-row pitches: conflict-free).  K order (tap, ci) and the 16-wide k-steps are the
// implicit-im2col GEMM's, so y is bit-identical to conv3x3_fwd(bn_apply(a1)).  Output
// lane = channel: BN2 sums in 2 registers; each store instruction writes 64-B channel
// runs of two pixels.
constexpr int SC2_CIN = 48, SC2_COUT = 96, SC2_K = 432, SC2_R = 2, SC2_NR = SC2_R + 2;
constexpr int SC2_PXS = 130, SC2_PITCH = 56, SC2_WPITCH = 440;   // bf16 units
constexpr int SC2_NW = 12, SC2_NT = SC2_NW * 64, SC2_CHUNKS = 2;  // staged 16-B chunks per thread per band
constexpr int SC2_RING = SC2_NR * SC2_PXS * SC2_PITCH * 2, SC2_LDS = SC2_RING + SC2_COUT * SC2_WPITCH * 2;

template <bool GELU, bool STAGED>
__global__ __launch_bounds__(SC2_NT, 1) void stem_conv2_kernel(const __bf16* a1, ChanAffine act,
                                                               const __bf16* wpack /*[96][432]*/, __bf16* y,
                                                               float* part /*[F][2][96]*/, int H, int W) {
  __shared__ __attribute__((aligned(16))) char lds[SC2_LDS];   // static: > 64 KB (gfx950: 160 KB per CU)
  __shared__ float aff[2][SC2_CIN];
  __shared__ float red[SC2_NW][2][32];
  __bf16* ring = (__bf16*)lds;
  __bf16* wl = (__bf16*)(lds + SC2_RING);
  const int t = threadIdx.x, l = t & 63, h = l >> 5, wv = t >> 6;
  const int nb = wv % 3, sg = wv / 3;
  const int64_t f = blockIdx.x;
  const __bf16* src = a1 + f * H * W * SC2_CIN;
  if (t < SC2_CIN) {   // = Affine8::init
    const float sc = act.rstd[t] * act.w[t];
    aff[0][t] = sc;
    aff[1][t] = bn_shift(act.b[t], act.mean[t], sc);
  }
  // zero the ring once: halo columns (x = -1, x >= W) and rows outside the image
  for (int i = t; i < SC2_RING / 16; i += SC2_NT) *(uint4*)(lds + 16 * i) = make_uint4(0, 0, 0, 0);
  for (int i = t; i < SC2_COUT * SC2_K / 8; i += SC2_NT) {
    const int co = i / (SC2_K / 8), k8 = i - co * (SC2_K / 8);
    *(uint4*)(wl + co * SC2_WPITCH + 8 * k8) = *(const uint4*)(wpack + co * SC2_K + 8 * k8);
  }
  // this thread's chunks of a band's rows: (row, pixel, 8-channel group) packed
  const int rowc = W * (SC2_CIN / 8);
  int cpos[SC2_CHUNKS];
#pragma unroll
  for (int i = 0; i < SC2_CHUNKS; ++i) {
    const int c = t + SC2_NT * i;
    const int r = c / rowc, rem = c - r * rowc, x = rem / 6;
    cpos[i] = r < SC2_R ? (r << 16) | (x << 3) | (rem - x * 6) : -1;
  }
  __syncthreads();
  auto slot = [&](int iy) { return (iy + 1) % SC2_NR; };
  uint4 raw[SC2_CHUNKS];
  auto load_rows = [&](int iy0) {   // rows iy0 .. iy0 + SC2_R - 1 of a1 (past H: zero)
#pragma unroll
    for (int i = 0; i < SC2_CHUNKS; ++i) {
      const int iy = iy0 + (cpos[i] >> 16);
      raw[i] = make_uint4(0, 0, 0, 0);
      if (cpos[i] >= 0 && iy < H)
        raw[i] = *(const uint4*)(src + ((int64_t)iy * W + ((cpos[i] >> 3) & 0x1FFF)) * SC2_CIN + 8 * (cpos[i] & 7));
    }
  };
  // BN1 + GELU (packed pairs, = bn_apply) of chunk i into its ring row; rows past H are
  // the conv's zero padding of h1
  auto commit_chunk = [&](int i, int iy) {
    const int x = (cpos[i] >> 3) & 0x1FFF, cc = cpos[i] & 7;
    float vv[8];
    load8((const __bf16*)&raw[i], vv);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      f32x2 u = vfma(f32x2{vv[j], vv[j + 1]}, f32x2{aff[0][8 * cc + j], aff[0][8 * cc + j + 1]},
                     f32x2{aff[1][8 * cc + j], aff[1][8 * cc + j + 1]});
      if (GELU) u = gelu_f2(u);
      vv[j] = iy < H ? u.x : 0.f;
      vv[j + 1] = iy < H ? u.y : 0.f;
    }
    store8(ring + (slot(iy) * SC2_PXS + x + 1) * SC2_PITCH + 8 * cc, vv);
  };
  auto commit_rows = [&](int iy0) {
#pragma unroll
    for (int i = 0; i < SC2_CHUNKS; ++i)
      if (cpos[i] >= 0) commit_chunk(i, iy0 + (cpos[i] >> 16));
  };
  // first band: input rows 0 .. SC2_R (row -1 stays zero)
  load_rows(0);
  commit_rows(0);
  load_rows(SC2_R);   // only its first row (SC2_R) belongs to band 0
#pragma unroll
  for (int i = 0; i < SC2_CHUNKS; ++i)
    if (cpos[i] >= 0 && (cpos[i] >> 16) == 0) commit_chunk(i, SC2_R);
  float s1 = 0.f, s2 = 0.f;   // BN2 sums of channel 32 nb + (l & 31) over this lane's pixels
  const int nbands = (H + SC2_R - 1) / SC2_R;
  constexpr bool staged = STAGED;   // host: W >= 110 (stem_conv2_staged)
  const int co = 32 * nb + (l & 31);
  const __bf16* wrow = wl + co * SC2_WPITCH + 8 * h;
  for (int band = 0; band < nbands; ++band) {
    const int y0 = band * SC2_R;
    if (band > 0) {
      __syncthreads();   // the previous band finished reading the slots rewritten here
      commit_rows(y0 + 1);   // rows y0 + 1, y0 + 2 (loaded during the previous band)
    }
    __syncthreads();
    if (band + 1 < nbands) load_rows(y0 + SC2_R + 1);   // the next band's new rows, in flight
    // both rows of the band accumulate tap row by tap row (k order (tap, ci) as the GEMM);
    // per tap row ky the wave holds its 9 B fragments (k = 48 (3 ky + kx) + 16 c16 + 8 h)
    f32x16 acc[SC2_R];
#pragma unroll
    for (int yy = 0; yy < SC2_R; ++yy)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[yy][r] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      bf16x8 wf[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) wf[q] = *(const bf16x8*)(wrow + 16 * (9 * ky + q));
#pragma unroll
      for (int yy = 0; yy < SC2_R; ++yy) {
        const __bf16* rp = ring + (slot(y0 + yy + ky - 1) * SC2_PXS + sg * 32 + (l & 31)) * SC2_PITCH + 8 * h;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int c16 = 0; c16 < 3; ++c16)
            acc[yy] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)(rp + kx * SC2_PITCH + 16 * c16),
                                                              wf[3 * kx + c16], acc[yy], 0, 0, 0);
        if (yy + 1 < SC2_R) __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);   // one tap row's fragments in flight (registers)
    }
    // Output tile: lane = channel co, registers = pixels (r & 3) + 8 (r >> 2) + 4 h of the
    // segment.  Staged (W >= 110, the 112-pixel stem): the tile goes through LDS -- the ring
    // slots of rows y0 - 1 and y0 are dead once every wave has finished this band's MFMAs
    // (one barrier), and the next band's commit rewrites every byte used here (pixel columns
    // 1 .. W; halo columns and the 16-B pad reads never touched) -- and leaves as 16-B stores of
    // 8 channels of one pixel: 2 store instructions per row and wave where the direct form
    // issued 16 2-byte stores (each two 64-B runs).  Direct form: narrow frames.
    char* stg = nullptr;
    if (staged) {
      __syncthreads();
      stg = (char*)(ring + (slot(wv < SC2_NW / 2 ? y0 - 1 : y0) * SC2_PXS + 1) * SC2_PITCH) + (wv % (SC2_NW / 2)) * 2048;
    }
#pragma unroll
    for (int yy = 0; yy < SC2_R; ++yy) {
      const int yo = y0 + yy;
      if (yo >= H) break;
      __bf16* yr = y + ((f * H + yo) * W + sg * 32) * SC2_COUT + co;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pp = (r & 3) + 8 * (r >> 2) + 4 * h;
        const __bf16 o = (__bf16)acc[yy][r];
        if (staged) *(__bf16*)(stg + pp * 64 + (l & 31) * 2) = o;   // [pixel][32 channels]
        if (sg * 32 + pp < W) {
          const float of = (float)o;
          s1 += of;
          s2 = fmaf(of, of, s2);
          if (!staged) yr[pp * SC2_COUT] = o;
        }
      }
      if (staged) {   // lane l: pixels (l >> 2) + 16 k, channels 32 nb + 8 (l & 3) .. + 7
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int px = (l >> 2) + 16 * k;
          const uint4 v = *(const uint4*)(stg + px * 64 + (l & 3) * 16);
          if (sg * 32 + px < W)
            *(uint4*)(y + ((f * H + yo) * W + sg * 32 + px) * SC2_COUT + 32 * nb + 8 * (l & 3)) = v;
        }
      }
    }
  }
  // BN2 partials of this frame: the two halves (same channel), then the 4 segment waves
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 32, 64);
  if (h == 0) {
    red[wv][0][l] = s1;
    red[wv][1][l] = s2;
  }
  __syncthreads();
  if (t < 2 * SC2_COUT) {
    const int which = t / SC2_COUT, c = t % SC2_COUT, b3 = c / 32, cl = c % 32;
    part[(f * 2 + which) * SC2_COUT + c] =
        ((red[b3][which][cl] + red[3 + b3][which][cl]) + red[6 + b3][which][cl]) + red[9 + b3][which][cl];
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
// src [Cout][Cin][3][3] fp32 -> order 0: dst[co][ci * 9 + tap]; order 1: dst[co][tap * Cin
// + ci] (im2col3 / implicit conv3x3 forward); order 2: dst[ci][tap * Cout + co] (conv3x3
// data gradient), tap = ky * 3 + kx; k >= 9 * (reduced channels) is zero padding.
template <typename TO>
__global__ void wpack_kernel(const float* src, TO* dst, int Cout, int Cin, int Kpad, int order) {
  const int rows = order == 2 ? Cin : Cout;
  const int total = rows * Kpad;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / Kpad, k = i % Kpad;
    float v = 0.f;
    if (k < (order == 2 ? Cout : Cin) * 9) {
      int ci, co, tap;
      if (order == 0) { co = row; ci = k / 9; tap = k % 9; }
      else if (order == 1) { co = row; tap = k / Cin; ci = k % Cin; }
      else { ci = row; tap = k / Cout; co = k % Cout; }
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

// ------------------------------------------------------------------ fused depthwise 3x3 (bf16)
// y = dwconv3x3(act(x)) with act = the producer's BatchNorm + GELU folded per channel
// (ChanAffine; identity when absent), plus per-frame BatchNorm statistics partials of
// the bf16 output (part[f][2][C]: sum, sum of squares), so neither act(x) nor a
// statistics pass over y touches HBM.
// Block = (32-channel slice, frame).  It walks the frame in bands of TY output rows
// through an LDS ring of NR = (TY-1)S+3 transformed input rows [NR][W+2][32] bf16
// (zero border columns; rows outside the image are zero: the convolution pads
// act(x)).  Each input row is transformed once; the TY*S new rows of band b+1 are
// loaded into registers while band b is computed (software pipeline).  Every thread
// computes PX = 7 consecutive outputs x 8 channels per item at stride 1 (odd PX keeps
// the 16-lane groups of ds_read_b128 conflict-free: strip pitch 448 B), 2 at stride 2.  Taps accumulate in the
// (ky, kx) order of dw_fwd_kernel: bit-identical y.
constexpr int DWF_CB = 32, DWF_PX = 7, DWF_KV = 7;

template <int S>
constexpr int dwf_ty() { return S == 1 ? 4 : 2; }

template <int S, int TY_ = dwf_ty<S>()>
struct DwRing {
  static constexpr int TY = TY_;
  static constexpr int NR = (TY - 1) * S + 3;
  static constexpr int NEW = TY * S;              // rows entering the ring per band
  const __bf16* x;
  int64_t f;
  int H, W, C, cbase, c8, pitch;
  uint4 raw[DWF_KV];
  SM_DEV int slot(int iy) const { return (iy + 1 + NR) % NR; }
  // raw-load rows [iy_first, iy_first + nrows) (nrows * W * 4 <= 256 * DWF_KV)
  // REMAT: t passes through an empty asm so the per-chunk index math is redone per
  // band rather than hoisted out of the band loop into ~40 long-lived VGPRs (for a
  // consumer that needs the registers)
  template <bool REMAT = false>
  SM_DEV void load(int iy_first, int nrows) {
    int t = threadIdx.x;
    if (REMAT) asm volatile("" : "+v"(t));
    const int nvec = nrows * W * 4;
#pragma unroll
    for (int k = 0; k < DWF_KV; ++k) {
      const int v = t + 256 * k;
      const int q = v >> 2;
      const int r = q / W, xx = q - r * W;
      const int iy = iy_first + r;
      raw[k] = make_uint4(0, 0, 0, 0);
      if (v < nvec && iy >= 0 && iy < H) raw[k] = *(const uint4*)(x + ((f * H + iy) * W + xx) * C + cbase);
    }
  }
  template <bool REMAT = false>
  SM_DEV void commit(char* lds, const Affine8& af, int iy_first, int nrows) const {
    int t = threadIdx.x;
    if (REMAT) asm volatile("" : "+v"(t));
    const int nvec = nrows * W * 4;
#pragma unroll
    for (int k = 0; k < DWF_KV; ++k) {
      const int v = t + 256 * k;
      if (v >= nvec) break;
      const int q = v >> 2;
      const int r = q / W, xx = q - r * W;
      const int iy = iy_first + r;
      float a[8];
      if (iy >= 0 && iy < H) {
        load8((const __bf16*)&raw[k], a);
        af.apply<__bf16>(a);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = 0.f;
      }
      store8((__bf16*)(lds + slot(iy) * pitch + (xx + 1) * 64 + c8 * 16), a);
    }
  }
  SM_DEV void zero_borders(char* lds) const {
    const int t = threadIdx.x;
    if (t < NR * 8) {
      const int r = t >> 3, side = (t >> 2) & 1;
      *(uint4*)(lds + r * pitch + (side ? W + 1 : 0) * 64 + c8 * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  // the first band's NR rows (from iy0 = -1), in two register batches
  template <bool REMAT = false>
  SM_DEV void stage_first(char* lds, const Affine8& af) {
    const int first = (NR + 1) / 2;
    load<REMAT>(-1, first);
    commit<REMAT>(lds, af, -1, first);
    load<REMAT>(-1 + first, NR - first);
    commit<REMAT>(lds, af, -1 + first, NR - first);
    zero_borders(lds);
  }
};

// Block -> (32-channel slice, frame) of the fused depthwise kernels.  1-D grid with
// the bijective XCD remap (as the attention and GEMM kernels): the C/32 slices of a
// frame -- 64-B pieces of the same 128-B lines of every pixel -- run back to back on
// one XCD, so each line is fetched into (and written back from) one L2 once rather
// than half-used by two XCDs.  remap = 0: plain order.
struct DwfBlock {
  int cs;
  int64_t f;
  SM_DEV DwfBlock(int ncs, int remap) {
    const int nwg = gridDim.x, bid = blockIdx.x;
    int v = bid;
    if (remap) {
      const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
      v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    }
    cs = v % ncs;
    f = v / ncs;
  }
};

// STATS: accumulate the BatchNorm partials of y (false for the lite-resident recompute and
// the data-gradient use, which pass part = null: two VALU ops per output fewer)
template <int S, bool STATS = true>
__global__ __launch_bounds__(256, 2) void dwf_fwd_kernel(const __bf16* x, ChanAffine act, const float* w,
                                                         __bf16* y, float* part, int H, int W, int C, int Ho,
                                                         int Wo, int remap) {
  using R = DwRing<S>;
  constexpr int TY = R::TY;
  // stride 2: 2 outputs per item (a band of TY = 2 rows x Wo / 7 strips x 4 chunks left
  // three of the four waves idle while one computed; 2 keeps 88 % of the block busy)
  constexpr int PX = S == 1 ? DWF_PX : 2;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const DwfBlock blk(C / DWF_CB, remap);
  const int cs = blk.cs;
  const int64_t f = blk.f;
  const int t = threadIdx.x;
  const int c8 = t & 3;
  const int cbase = cs * DWF_CB + c8 * 8;
  R ring{x, f, H, W, C, cbase, c8, (W + 2) * 64};
  Affine8 af;
  af.init(act, cbase);
  // taps in LDS after the ring ([9][32] fp32), re-read per row of taps: keeps the
  // 72 weights out of the register file (occupancy); 6 ds_read_b128 per item row
  float* wl = (float*)(lds + R::NR * ring.pitch);
  for (int i = t; i < 9 * DWF_CB; i += 256) {
    const int tap = i / DWF_CB, ch = i % DWF_CB;
    wl[i] = w[(int64_t)(cs * DWF_CB + ch) * 9 + tap];
  }
  float s8[8], q8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s8[j] = 0.f; q8[j] = 0.f; }
  const int nstrip = (Wo + PX - 1) / PX;
  const int items = TY * nstrip * 4;
  const int nbands = (Ho + TY - 1) / TY;
  ring.stage_first(lds, af);
  for (int band = 0; band < nbands; ++band) {
    const int yo0 = band * TY;
    if (band > 0) {
      __syncthreads();                                  // band-1 finished reading the slots we overwrite
      ring.commit(lds, af, (yo0 * S - 1) + (3 - S), R::NEW);
    }
    __syncthreads();
    if (band + 1 < nbands) ring.load(((yo0 + TY) * S - 1) + (3 - S), R::NEW);   // next band, in flight
    for (int it = t; it < items; it += 256) {
      const int q = it >> 2;
      const int ry = q / nstrip, strip = q - ry * nstrip;
      const int yo = yo0 + ry;
      if (yo >= Ho) continue;
      const int xo0 = strip * PX;
      float acc[PX][8];
#pragma unroll
      for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[p][j] = 0.f;
      const float* wlt = wl + c8 * 8;
      asm volatile("" : "+v"(wlt));             // per-item reload: do not hoist the taps
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const char* rowp = lds + ring.slot(yo * S - 1 + ky) * ring.pitch + c8 * 16;
        float wr[3][8];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) load8(wlt + (ky * 3 + kx) * DWF_CB, wr[kx]);
#pragma unroll
        for (int ci = 0; ci < (PX - 1) * S + 3; ++ci) {
          const int col = xo0 * S + ci;          // LDS column = input x + 1
          if (col > W + 1) break;                // ragged last strip
          float v[8];
          load8((const __bf16*)(rowp + col * 64), v);
#pragma unroll
          for (int p = 0; p < PX; ++p) {
            const int kx = ci - p * S;
            if (kx < 0 || kx > 2) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[p][j] += v[j] * wr[kx][j];
          }
        }
      }
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        if (xo0 + p >= Wo) break;
        float r8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          r8[j] = (float)(__bf16)acc[p][j];
          if (STATS) {
            s8[j] += r8[j];
            q8[j] += r8[j] * r8[j];
          }
        }
        store8(y + ((f * Ho + yo) * Wo + xo0 + p) * C + cbase, r8);
      }
    }
  }
  if (!STATS || !part) return;
  __syncthreads();                              // ring dead: reuse for the reduction
  float* red = (float*)lds;                     // [256][16]
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[t * 16 + j] = s8[j]; red[t * 16 + 8 + j] = q8[j]; }
  __syncthreads();
  if (t < 2 * DWF_CB) {
    const int ch = t & (DWF_CB - 1), which = t / DWF_CB;
    const int g = ch >> 3, j = ch & 7;
    float a = 0.f;
    for (int k = 0; k < 64; ++k) a += red[(k * 4 + g) * 16 + which * 8 + j];
    part[(f * 2 + which) * C + cs * DWF_CB + ch] = a;
  }
}

// Fused depthwise weight gradient: dw[c][tap] = sum dy[yo][xo][c] * act(x)[yo*S+ky-1][xo*S+kx-1][c]
// with act(x) recomputed through the same ring as dwf_fwd_kernel (and the same
// register prefetch of the next band).  Block = (32-channel slice, frame); the 72
// (tap, channel) sums of each thread stay in registers over the frame, then reduce
// over the 64 threads that share its 8 channels: part[f][C][9] (colred over frames).
template <int S>
__global__ __launch_bounds__(256, 2) void dwf_wgrad_kernel(const __bf16* dy, const __bf16* x, ChanAffine act,
                                                           float* part, int H, int W, int C, int Ho, int Wo,
                                                           int remap) {
  using R = DwRing<S>;
  constexpr int TY = R::TY;
  constexpr int PX = DWF_PX;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const DwfBlock blk(C / DWF_CB, remap);
  const int cs = blk.cs;
  const int64_t f = blk.f;
  const int t = threadIdx.x;
  const int c8 = t & 3;
  const int cbase = cs * DWF_CB + c8 * 8;
  R ring{x, f, H, W, C, cbase, c8, (W + 2) * 64};
  Affine8 af;
  af.init(act, cbase);
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  const int nstrip = (Wo + PX - 1) / PX;
  const int items = TY * nstrip * 4;
  const int nbands = (Ho + TY - 1) / TY;
  ring.stage_first(lds, af);
  for (int band = 0; band < nbands; ++band) {
    const int yo0 = band * TY;
    if (band > 0) {
      __syncthreads();
      ring.commit(lds, af, (yo0 * S - 1) + (3 - S), R::NEW);
    }
    __syncthreads();
    if (band + 1 < nbands) ring.load(((yo0 + TY) * S - 1) + (3 - S), R::NEW);
    for (int it = t; it < items; it += 256) {
      const int q = it >> 2;
      const int ry = q / nstrip, strip = q - ry * nstrip;
      const int yo = yo0 + ry;
      if (yo >= Ho) continue;
      const int xo0 = strip * PX;
      float g[PX][8];
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        if (xo0 + p < Wo) load8(dy + ((f * Ho + yo) * Wo + xo0 + p) * C + cbase, g[p]);
        else
#pragma unroll
          for (int j = 0; j < 8; ++j) g[p][j] = 0.f;
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const char* rowp = lds + ring.slot(yo * S - 1 + ky) * ring.pitch + c8 * 16;
#pragma unroll
        for (int ci = 0; ci < (PX - 1) * S + 3; ++ci) {
          const int col = xo0 * S + ci;
          if (col > W + 1) break;
          float v[8];
          load8((const __bf16*)(rowp + col * 64), v);
#pragma unroll
          for (int p = 0; p < PX; ++p) {
            const int kx = ci - p * S;
            if (kx < 0 || kx > 2) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[ky * 3 + kx][j] += g[p][j] * v[j];
          }
        }
      }
    }
  }
  __syncthreads();
  float* red = (float*)lds;   // [256][8] per tap
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t * 8 + j] = acc[tap][j];
    __syncthreads();
    if (t < DWF_CB) {
      const int g = t >> 3, j = t & 7;
      float a = 0.f;
      for (int k = 0; k < 64; ++k) a += red[(k * 4 + g) * 8 + j];
      part[(f * C + cs * DWF_CB + t) * 9 + tap] = a;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ depthwise + BN + GELU backward
// MBConv's  y = dwconv3x3(h), h = GELU(u), u = BN(x) with batch statistics of x
// (tiny_vit.py:36-56: conv1 -> act -> conv2), stride 1.  The depthwise data gradient
// g = dL/dh (the 3x3 convolution of dy with the taps rotated 180 degrees) is never
// stored; one pass (dwb_kernel) streams dy through the DwRing (zero halo) and reads x
// at the thread's own pixels only, and from ONE GELU evaluation per element forms
//   h (the forward's stored-precision activation) -> dw[c][tap] partials,
//   dz = g GELU'(u)  -> stored (bf16, into the dx buffer), and the BatchNorm-backward
//                        partial sums of dz and dz xhat;
// a streaming pass (dwb_dx_kernel) then turns dz into dx = w rstd (dz - mean(dz) -
// xhat mean(dz xhat)) in place.  HBM: dy read once, x twice, dz written and read
// once, dx written once; the unfused sequence (depthwise dgrad, depthwise
// wgrad, bn_bwd reduce, bn_bwd dx) reads dy / g four times and x three times, writes
// twice, and evaluates GELU three times per element.
// Thread = 4 channels (c4 = t & 7) x DWB_PX = 7 consecutive pixels of one row; h, GELU
// and xhat of its pixels stay live across the tap loop.  Columns past the row's right
// border read the next ring row (or the zeroed pad after the last one): finite
// values that only reach pixels past W, whose h and GELU' are zero.
constexpr int DWB_PX = 7, DWB_PAD = 8 * 64;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32_t;

// RAG: W % PX != 0 (a ragged last strip per row; the stride-2 form drops the per-pixel
// range selects when every strip is whole, as at all TinyViT widths)
template <bool GELU, bool RAG>
__global__ __launch_bounds__(256, 2) void dwb_kernel(const __bf16* dy, const __bf16* x, ChanAffine bn,
                                                     const float* w, __bf16* dz, float* part_w, float* part_bn,
                                                     int H, int W, int C, int remap) {
  using R = DwRing<1>;
  constexpr int TY = R::TY;
  constexpr int PX = DWB_PX;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const DwfBlock blk(C / DWF_CB, remap);
  const int cs = blk.cs;
  const int64_t f = blk.f;
  const int t = threadIdx.x;
  R ring{dy, f, H, W, C, cs * DWF_CB + (t & 3) * 8, t & 3, (W + 2) * 64};
  Affine8 raw;
  raw.init(ChanAffine{nullptr, nullptr, nullptr, nullptr, 0}, 0);
  const int c4 = t & 7;
  const int c0 = cs * DWF_CB + c4 * 4;
  char* pad = lds + R::NR * ring.pitch;
  for (int i = t; i < DWB_PAD / 16; i += 256) *(uint4*)(pad + 16 * i) = make_uint4(0, 0, 0, 0);
  // rotated taps: wl[tap][ch] = w[ch][8 - tap]
  float* wl = (float*)(pad + DWB_PAD);
  for (int i = t; i < 9 * DWF_CB; i += 256) {
    const int tap = i / DWF_CB, ch = i % DWF_CB;
    wl[i] = w[(int64_t)(cs * DWF_CB + ch) * 9 + 8 - tap];
  }
  // per-channel BN constants [4][32]: scale, shift (u = x sc + sh), mean, rstd
  float* cl = wl + 9 * DWF_CB;
  if (t < DWF_CB) {
    const int c = cs * DWF_CB + t;
    const float r = bn.rstd[c], scv = r * bn.w[c];
    cl[t] = scv;
    cl[DWF_CB + t] = bn_shift(bn.b[c], bn.mean[c], scv);
    cl[2 * DWF_CB + t] = bn.mean[c];
    cl[3 * DWF_CB + t] = r;
  }
  float dwa[9][4], sdz[4], sdzx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sdz[j] = sdzx[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) dwa[k][j] = 0.f;
  }
  const int nstrip = (W + PX - 1) / PX;
  const int items = TY * nstrip;
  const int nbands = (H + TY - 1) / TY;
  // frame-level views of x and dz (wave-uniform descriptors: a per-row descriptor built from
  // each thread's item is divergent, and every buffer access through it became a waterfall
  // loop of up to 8 passes)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + f * H * W * C), (short)0, H * W * C * 2, 0x00020000);
  const auto zr = __builtin_amdgcn_make_buffer_rsrc((void*)(dz + f * H * W * C), (short)0, H * W * C * 2, 0x00020000);
  ring.stage_first<true>(lds, raw);
  for (int band = 0; band < nbands; ++band) {
    const int y0 = band * TY;
    if (band > 0) {
      __syncthreads();
      ring.commit<true>(lds, raw, y0 + 1, R::NEW);
    }
    __syncthreads();
    if (band + 1 < nbands) ring.load<true>(y0 + TY + 1, R::NEW);
#pragma unroll 1
    for (int it = t >> 3; it < items; it += 32) {
      const int ry = it / nstrip, strip = it - ry * nstrip;
      const int yi = y0 + ry;
      if (yi >= H) continue;
      const int xi0 = strip * PX;
      // this pixel row of x and dz as buffer views: pixels past W read 0 / drop stores
      // pixels past W: out-of-range offset (loads read 0, stores are dropped)
      const uint32_t off0 = (uint32_t)((yi * W + xi0) * C + c0) * 2u;
      uint32_t offp[PX];
#pragma unroll
      for (int p = 0; p < PX; ++p) offp[p] = (!RAG || xi0 + p < W) ? off0 + (uint32_t)(p * C * 2) : 0x80000000u;
      float h[PX][4], gg[PX][4], g[PX][4];
      bf16x4 xs[PX];                     // x itself (xhat is formed after the tap loop)
      {
        float sc[4], sh[4];
        load4(cl + c4 * 4, sc);
        load4(cl + DWF_CB + c4 * 4, sh);
#pragma unroll
        for (int p = 0; p < PX; ++p)
          xs[p] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(xr, offp[p], 0, 0));
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          const bool ok = !RAG || xi0 + p < W;
#pragma unroll
          for (int j = 0; j < 4; j += 2) {   // packed pairs (gelu_phi_pair_t)
            const f32x2 u = vfma(f32x2{(float)xs[p][j], (float)xs[p][j + 1]}, f32x2{sc[j], sc[j + 1]},
                                 f32x2{sh[j], sh[j + 1]});
            f32x2 cdf = f32x2{1.f, 1.f}, pdf = f32x2{0.f, 0.f};
            if (GELU) cdf = gelu_phi_pair_t<f32x2>(u, &pdf);
            f32x2 hv = u;
            if (GELU) {
#pragma clang fp contract(off)
              hv = u * cdf;
            }
            const f32x2 gv = vfma(u, pdf, cdf);
            h[p][j] = ok ? (float)(__bf16)hv.x : 0.f;
            h[p][j + 1] = ok ? (float)(__bf16)hv.y : 0.f;
            gg[p][j] = ok ? gv.x : 0.f;
            gg[p][j + 1] = ok ? gv.y : 0.f;
            g[p][j] = g[p][j + 1] = 0.f;
          }
          __builtin_amdgcn_sched_barrier(0);   // bound the interleaved GELU chains (VGPR budget)
        }
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const char* rowp = lds + ring.slot(yi - 1 + ky) * ring.pitch + c4 * 8 + xi0 * 64;
        float wr[3][4];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) load4(wl + (ky * 3 + kx) * DWF_CB + c4 * 4, wr[kx]);
#pragma unroll
        for (int ci = 0; ci < PX + 2; ++ci) {    // LDS column xi0 + ci = dy x + 1
          float v[4];
          load4((const __bf16*)(rowp + ci * 64), v);
#pragma unroll
          for (int p = 0; p < PX; ++p) {
            const int kx = ci - p;
            if (kx < 0 || kx > 2) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              g[p][j] = fmaf(v[j], wr[kx][j], g[p][j]);
              dwa[8 - (ky * 3 + kx)][j] = fmaf(v[j], h[p][j], dwa[8 - (ky * 3 + kx)][j]);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);   // one tap row's reads in flight at a time (VGPR budget)
      }
      float mu[4], rs[4];
      load4(cl + 2 * DWF_CB + c4 * 4, mu);
      load4(cl + 3 * DWF_CB + c4 * 4, rs);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        float d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          d[j] = (float)(__bf16)(g[p][j] * gg[p][j]);   // the stored dz: the sums see what dx will
          sdz[j] += d[j];
          sdzx[j] = fmaf(d[j], ((float)xs[p][j] - mu[j]) * rs[j], sdzx[j]);
        }
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (__bf16)d[j];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, o), zr, offp[p], 0, 0);
      }
    }
  }
  __syncthreads();                     // ring dead: reuse for the reductions
  float* red = (float*)lds;            // [256][4]
  auto reduce = [&](const float* v4, float* dst, int64_t stride) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[t * 4 + j] = v4[j];
    __syncthreads();
    if (t < DWF_CB) {
      const int cc = t >> 2, j = t & 3;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += red[(k * 8 + cc) * 4 + j];
      dst[(int64_t)t * stride] = s;
    }
    __syncthreads();
  };
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) reduce(dwa[tap], part_w + (f * C + cs * DWF_CB) * 9 + tap, 9);
  reduce(sdz, part_bn + (f * 2 + 0) * C + cs * DWF_CB, 1);
  reduce(sdzx, part_bn + (f * 2 + 1) * C + cs * DWF_CB, 1);
}

// Stride-2 form of dwb_kernel (the MBConv that opens stages 1-3: tiny_vit.py:46 with
// stride 2).  The input pixel (yi, xi) receives dy[yo][xo] w[ky][kx] for the taps with
// yi + 1 - ky = 2 yo and xi + 1 - kx = 2 xo: one tap row for even yi (ky = 1), two for
// odd yi (ky = 0, 2), and likewise along x -- 2.25 taps per pixel, each also feeding
// dw[ky][kx] += dy h.  The ring holds dy rows (output resolution, zero halo; rows past
// Ho read zero): a band of 2 DWB2_TYO = 4 input rows needs dy rows yo0 .. yo0 + 2, two
// of them new.  Thread = 4 channels x DWB2_PX = 4 input pixels of one row (an even
// strip start, so the x tap pattern is fixed per pixel: even p one column, odd p two).
// Replaces depthwise dgrad (dh1 written at input resolution), the fused depthwise
// weight gradient and the BatchNorm/GELU backward's two passes over (dh1, x): dy read
// once, x twice, dz written and read once, GELU evaluated once per element.
constexpr int DWB2_PX = 4, DWB2_TYO = 2, DWB2_PAD = 2 * 64;

template <bool GELU, bool RAG>
__global__ __launch_bounds__(256, 2) void dwb2_kernel(const __bf16* dy, const __bf16* x, ChanAffine bn,
                                                      const float* w, __bf16* dz, float* part_w, float* part_bn,
                                                      int H, int W, int C, int Ho, int Wo, int remap) {
  using R = DwRing<1, DWB2_TYO>;
  constexpr int TYI = 2 * DWB2_TYO;      // input rows per band
  constexpr int PX = DWB2_PX;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const DwfBlock blk(C / DWF_CB, remap);
  const int cs = blk.cs;
  const int64_t f = blk.f;
  const int t = threadIdx.x;
  R ring{dy, f, Ho, Wo, C, cs * DWF_CB + (t & 3) * 8, t & 3, (Wo + 2) * 64};
  Affine8 raw;
  raw.init(ChanAffine{nullptr, nullptr, nullptr, nullptr, 0}, 0);
  const int c4 = t & 7;
  const int c0 = cs * DWF_CB + c4 * 4;
  // a ragged last strip's pixels past W read up to two columns past the last ring row:
  // zero pad, so those values (which only meet h = GELU' = 0) are never NaN bit patterns
  char* pad = lds + R::NR * ring.pitch;
  if (t < DWB2_PAD / 16) *(uint4*)(pad + 16 * t) = make_uint4(0, 0, 0, 0);
  float* wl = (float*)(pad + DWB2_PAD);              // taps wl[tap][ch] = w[ch][tap]
  for (int i = t; i < 9 * DWF_CB; i += 256) {
    const int tap = i / DWF_CB, ch = i % DWF_CB;
    wl[i] = w[(int64_t)(cs * DWF_CB + ch) * 9 + tap];
  }
  float* cl = wl + 9 * DWF_CB;                      // BN constants [4][32]: scale, shift, mean, rstd
  if (t < DWF_CB) {
    const int c = cs * DWF_CB + t;
    const float r = bn.rstd[c], scv = r * bn.w[c];
    cl[t] = scv;
    cl[DWF_CB + t] = bn_shift(bn.b[c], bn.mean[c], scv);
    cl[2 * DWF_CB + t] = bn.mean[c];
    cl[3 * DWF_CB + t] = r;
  }
  float dwa[9][4], sdz[4], sdzx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sdz[j] = sdzx[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) dwa[k][j] = 0.f;
  }
  const int nstrip = (W + PX - 1) / PX;
  const int items = TYI * nstrip;
  const int nbands = (H + TYI - 1) / TYI;
  // frame-level views of x and dz (wave-uniform descriptors; see dwb_kernel)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)(x + f * H * W * C), (short)0, H * W * C * 2, 0x00020000);
  const auto zr = __builtin_amdgcn_make_buffer_rsrc((void*)(dz + f * H * W * C), (short)0, H * W * C * 2, 0x00020000);
  // item offsets; the thread's NEXT item's x is loaded while the current one computes
  // (-2 % here, profiles/r04g_dwb_prefetch_ab.txt; the stride-1 kernel, already at 235
  // VGPRs, spilled with it and lost 3 %)
  auto item_offs = [&](int band_, int it_, uint32_t (&o)[PX]) {
    const int ry = it_ / nstrip, strip = it_ - ry * nstrip;
    const int xi_ = strip * PX;
    const uint32_t b = (uint32_t)(((band_ * TYI + ry) * W + xi_) * C + c0) * 2u;
#pragma unroll
    for (int p = 0; p < PX; ++p) o[p] = (!RAG || xi_ + p < W) ? b + (uint32_t)(p * C * 2) : 0x80000000u;
  };
  auto xload = [&](const uint32_t (&o)[PX], bf16x4 (&xv)[PX]) {
#pragma unroll
    for (int p = 0; p < PX; ++p)
      xv[p] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(xr, o[p], 0, 0));
  };
  bf16x4 xn[PX];
  {
    uint32_t o[PX];
    item_offs(0, t >> 3, o);
    xload(o, xn);
  }
  ring.stage_first<true>(lds, raw);
  for (int band = 0; band < nbands; ++band) {
    const int y0 = band * TYI, yo0 = band * DWB2_TYO;
    if (band > 0) {
      __syncthreads();
      ring.commit<true>(lds, raw, yo0 + 1, R::NEW);
    }
    __syncthreads();
    if (band + 1 < nbands) ring.load<true>(yo0 + DWB2_TYO + 1, R::NEW);
#pragma unroll 1
    for (int it = t >> 3; it < items; it += 32) {
      const int ry = it / nstrip, strip = it - ry * nstrip;
      const int yi = y0 + ry;
      const int xi0 = strip * PX;
      bf16x4 xs[PX];
#pragma unroll
      for (int p = 0; p < PX; ++p) xs[p] = xn[p];
      {
        int nb = band, ni = it + 32;
        if (ni >= items) {
          nb = band + 1;
          ni = t >> 3;
        }
        if (nb < nbands) {
          uint32_t o[PX];
          item_offs(nb, ni, o);
          xload(o, xn);
        }
      }
      if (yi >= H) continue;
      uint32_t offp[PX];
      item_offs(band, it, offp);
      float h[PX][4], gg[PX][4], g[PX][4];
      {
        float sc[4], sh[4];
        load4(cl + c4 * 4, sc);
        load4(cl + DWF_CB + c4 * 4, sh);
#pragma unroll
        for (int p = 0; p < PX; ++p) {
          const bool ok = !RAG || xi0 + p < W;
#pragma unroll
          for (int j = 0; j < 4; j += 2) {   // packed pairs (gelu_phi_pair_t)
            const f32x2 u = vfma(f32x2{(float)xs[p][j], (float)xs[p][j + 1]}, f32x2{sc[j], sc[j + 1]},
                                 f32x2{sh[j], sh[j + 1]});
            f32x2 cdf = f32x2{1.f, 1.f}, pdf = f32x2{0.f, 0.f};
            if (GELU) cdf = gelu_phi_pair_t<f32x2>(u, &pdf);
            f32x2 hv = u;
            if (GELU) {
#pragma clang fp contract(off)
              hv = u * cdf;
            }
            const f32x2 gv = vfma(u, pdf, cdf);
            h[p][j] = ok ? (float)(__bf16)hv.x : 0.f;
            h[p][j + 1] = ok ? (float)(__bf16)hv.y : 0.f;
            gg[p][j] = ok ? gv.x : 0.f;
            gg[p][j + 1] = ok ? gv.y : 0.f;
            g[p][j] = g[p][j + 1] = 0.f;
          }
          __builtin_amdgcn_sched_barrier(0);   // bound the interleaved GELU chains (VGPR budget)
        }
      }
      // one tap row ky over dy row yo: LDS columns xi0 / 2 + cj + 1, cj = 0..4 feed pixel
      // 2cj (kx = 1), 2cj - 1 (kx = 0) and 2cj + 1 (kx = 2)
      auto tap_row = [&](int ky, int yo) {
        const char* rowp = lds + ring.slot(yo) * ring.pitch + c4 * 8 + (xi0 / 2 + 1) * 64;
        float wr[3][4];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) load4(wl + (ky * 3 + kx) * DWF_CB + c4 * 4, wr[kx]);
#pragma unroll
        for (int cj = 0; cj <= PX / 2; ++cj) {
          float v[4];
          load4((const __bf16*)(rowp + cj * 64), v);
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int p = 2 * cj + kx - 1;   // xi0 + p + 1 - kx = 2 (xi0 / 2 + cj)
            if (p < 0 || p >= PX) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              g[p][j] = fmaf(v[j], wr[kx][j], g[p][j]);
              dwa[ky * 3 + kx][j] = fmaf(v[j], h[p][j], dwa[ky * 3 + kx][j]);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      if (yi & 1) {
        tap_row(0, (yi + 1) >> 1);
        tap_row(2, (yi - 1) >> 1);
      } else {
        tap_row(1, yi >> 1);
      }
      float mu[4], rs[4];
      load4(cl + 2 * DWF_CB + c4 * 4, mu);
      load4(cl + 3 * DWF_CB + c4 * 4, rs);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        float d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          d[j] = (float)(__bf16)(g[p][j] * gg[p][j]);   // the stored dz: the sums see what dx will
          sdz[j] += d[j];
          sdzx[j] = fmaf(d[j], ((float)xs[p][j] - mu[j]) * rs[j], sdzx[j]);
        }
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (__bf16)d[j];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, o), zr, offp[p], 0, 0);
      }
    }
  }
  __syncthreads();                     // ring dead: reuse for the reductions
  float* red = (float*)lds;            // [256][4]
  auto reduce = [&](const float* v4, float* dst, int64_t stride) {
#pragma unroll
    for (int j = 0; j < 4; ++j) red[t * 4 + j] = v4[j];
    __syncthreads();
    if (t < DWF_CB) {
      const int cc = t >> 2, j = t & 3;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += red[(k * 8 + cc) * 4 + j];
      dst[(int64_t)t * stride] = s;
    }
    __syncthreads();
  };
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) reduce(dwa[tap], part_w + (f * C + cs * DWF_CB) * 9 + tap, 9);
  reduce(sdz, part_bn + (f * 2 + 0) * C + cs * DWF_CB, 1);
  reduce(sdzx, part_bn + (f * 2 + 1) * C + cs * DWF_CB, 1);
}

// dx = w rstd (dz - coef[0] - xhat coef[1]) in place over dz; thread = fixed 8-channel
// chunk (C / 8 <= 256) over a block's rows
__global__ __launch_bounds__(256) void dwb_dx_kernel(const __bf16* x, ChanAffine bn, const float* coef, __bf16* dz,
                                                     int64_t M, int C, int rows_per_block) {
  const int nch = C / 8, rpp = 256 / nch;
  const int chunk = threadIdx.x % nch, r = threadIdx.x / nch;
  if (r >= rpp) return;
  float mu[8], rs[8], wr[8], k0[8], k1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = chunk * 8 + j;
    mu[j] = bn.mean[c];
    rs[j] = bn.rstd[c];
    wr[j] = bn.w[c] * rs[j];
    k0[j] = coef[c];
    k1[j] = coef[C + c];
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  // four rows per step, all loads issued before the first store: dz is rewritten in place,
  // so the compiler cannot hoist the next row's loads above this row's store by itself
  // (one 32-B load pair in flight per lane streamed at ~4.4 TB/s)
  constexpr int U = 4;
  typedef unsigned int nt4 __attribute__((ext_vector_type(4)));
  int64_t row = r0 + r;
  for (; row + (U - 1) * rpp < r1; row += U * rpp) {
    nt4 xr[U], dr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {   // streamed once: non-temporal loads and stores
      const int64_t e = (row + u * rpp) * C + chunk * 8;
      xr[u] = __builtin_nontemporal_load((const nt4*)(x + e));
      dr[u] = __builtin_nontemporal_load((const nt4*)(dz + e));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float xv[8], dv[8], o[8];
      load8((const __bf16*)&xr[u], xv);
      load8((const __bf16*)&dr[u], dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = wr[j] * (dv[j] - k0[j] - (xv[j] - mu[j]) * rs[j] * k1[j]);
      bf16x8 ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) ob[j] = (__bf16)o[j];
      __builtin_nontemporal_store(__builtin_bit_cast(nt4, ob), (nt4*)(dz + (row + u * rpp) * C + chunk * 8));
    }
  }
  for (; row < r1; row += rpp) {
    const int64_t e = row * C + chunk * 8;
    float xv[8], dv[8], o[8];
    load8(x + e, xv);
    load8(dz + e, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = wr[j] * (dv[j] - k0[j] - (xv[j] - mu[j]) * rs[j] * k1[j]);
    store8(dz + e, o);
  }
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
// The SE input h = act(x) (the BN2 + GELU of MBConv, ChanAffine) is recomputed in
// every kernel that reads it instead of being materialised.  Frame reductions are
// split over nsplit pixel ranges per frame (grid (nsplit, F)) into partial slabs
// part[f][k][C], summed in fixed order by the per-frame FC kernels.  Thread layout:
// Col8 (8 channels per thread, 16-B loads, per-channel constants in registers).
constexpr int SE_PX_PER_SPLIT = 784;

__host__ __device__ inline int se_splits(int HW) { return (HW + SE_PX_PER_SPLIT - 1) / SE_PX_PER_SPLIT; }

struct SeCols {
  int nch, rpp, c0, r;
  SM_DEV SeCols(int C) {
    nch = C / 8;
    rpp = 256 / nch;
    c0 = (threadIdx.x % nch) * 8;
    r = threadIdx.x / nch;
  }
};

// part[f][k][c] = sum over split k of h  (h = act(x))      or of dy * h when dy
template <typename T>
__global__ __launch_bounds__(256) void se_reduce_kernel(const T* x, const T* dy, ChanAffine act, int HW, int C,
                                                        float* part) {
  __shared__ float red[256 * 8];
  const SeCols cm(C);
  const int k = blockIdx.x, nsplit = gridDim.x;
  const int64_t f = blockIdx.y;
  const int p0 = k * SE_PX_PER_SPLIT, p1 = min(HW, p0 + SE_PX_PER_SPLIT);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (cm.r < cm.rpp) {
    Affine8 af;
    af.init(act, cm.c0);
    for (int p = p0 + cm.r; p < p1; p += cm.rpp) {
      const int64_t e = (f * HW + p) * C + cm.c0;
      float v[8];
      load8_nt(x + e, v);
      af.apply<T>(v);
      if (dy) {
        float g[8];
        load8_nt(dy + e, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= g[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int rr = 0; rr < cm.rpp; ++rr) a += red[(rr * cm.nch + c / 8) * 8 + c % 8];
    part[(f * nsplit + k) * C + c] = a;
  }
}

// per frame: p = sum_k part / HW; z1 = W1 p; h1 = relu(z1); z2 = W2 h1; s = sigmoid(z2)
__global__ __launch_bounds__(256) void se_fc_fwd_kernel(const float* part, int nsplit, int HW,
                                                        const float* w1 /*[R][C]*/, const float* w2 /*[C][R]*/,
                                                        int C, int R, float* pooled, float* h1_out, float* s_out) {
  extern __shared__ float sh[];
  float* p = sh;          // C
  float* h = sh + C;      // R
  const int64_t f = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f;
    for (int k = 0; k < nsplit; ++k) a += part[(f * nsplit + k) * C + c];
    p[c] = a / HW;
    pooled[f * C + c] = p[c];
  }
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

// y = act(x) * s[f][c]          (dpool == null)
// y = x * s[f][c] + dpool[f][c] / HW   (backward dx, x = dy, act identity)
template <typename T>
__global__ __launch_bounds__(256) void se_apply_kernel(const T* x, ChanAffine act, const float* s,
                                                       const float* dpool, T* y, int HW, int C) {
  const SeCols cm(C);
  if (cm.r >= cm.rpp) return;
  const int k = blockIdx.x;
  const int64_t f = blockIdx.y;
  const int p0 = k * SE_PX_PER_SPLIT, p1 = min(HW, p0 + SE_PX_PER_SPLIT);
  Affine8 af;
  af.init(act, cm.c0);
  float sc[8], add[8];
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = s[f * C + cm.c0 + j];
    add[j] = dpool ? dpool[f * C + cm.c0 + j] * inv : 0.f;
  }
  for (int p = p0 + cm.r; p < p1; p += cm.rpp) {
    const int64_t e = (f * HW + p) * C + cm.c0;
    float v[8];
    load8(x + e, v);
    af.apply<T>(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = dpool ? v[j] * sc[j] + add[j] : v[j] * sc[j];
    store8(y + e, v);
  }
}

// per frame backward through sigmoid / W2 / relu / W1 (ds = sum_k part):
//   dz2 = ds * s (1-s);  dh1 = W2^T dz2;  dz1 = dh1 * (z1 > 0);  dpool = W1^T dz1
__global__ __launch_bounds__(256) void se_fc_bwd_kernel(const float* part, int nsplit, const float* s,
                                                        const float* z1, const float* w1, const float* w2, int C,
                                                        int R, float* dz2_out, float* dz1_out, float* dpool) {
  extern __shared__ float sh[];
  float* dz2 = sh;      // C
  float* dz1 = sh + C;  // R
  const int64_t f = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    float ds = 0.f;
    for (int k = 0; k < nsplit; ++k) ds += part[(f * nsplit + k) * C + c];
    const float sv = s[f * C + c];
    const float g = ds * sv * (1.f - sv);
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

// ------------------------------------------------------------------ fused SE + BN/GELU backward
// MBConv's h2 = GELU(BN2(a2)), h3 = h2 * gate (tiny_vit.py:50-53): the backward of the
// SE layer and of BN2 + GELU in two streaming passes over (dh3, a2) instead of four
// (se_bwd: gate-gradient reduce + dh2 write; bn_bwd: reduce + dx), and dh2 never
// exists in HBM.  dh2 = dh3 * s[f][c] + dpool[f][c] / HW is affine per (frame,
// channel), so BN2's two channel sums over du = dh2 * GELU'(u) split into per-frame
// sums of dh3 and of 1 that the frame's (s, dpool) weight once dpool is known:
//   sum du      = sum_f (s * A_f + dpool/HW * B_f),  A = sum dh3 g',    B = sum g'
//   sum du xhat = sum_f (s * X_f + dpool/HW * D_f),  X = sum dh3 g' xh, D = sum g' xh
// Pass 1 (se_bn_reduce_kernel) produces the SE gate sums (se_reduce layout) and A, B,
// X, D per (frame, split); pass 2 (se_bn_dx_kernel) recomputes dh2 and writes da2.
struct BnCh8 {   // per-channel constants of the BatchNorm + GELU on 8 channels
  float sc[8], sh[8], rs[8], mr[8], wr[8];
  SM_DEV void init(const ChanAffine& a, int c0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      rs[j] = a.rstd[c];
      mr[j] = a.mean[c] * rs[j];
      sc[j] = rs[j] * a.w[c];
      sh[j] = bn_shift(a.b[c], a.mean[c], sc[j]);
      wr[j] = a.w[c] * rs[j];
    }
  }
};

template <typename T>
__global__ __launch_bounds__(256) void se_bn_reduce_kernel(const T* dy, const T* x, ChanAffine act, int HW, int C,
                                                           float* part /*[F][ns][C]*/,
                                                           float* part2 /*[F][ns][4][C]*/) {
  __shared__ float red[256 * 8];
  const SeCols cm(C);
  const int k = blockIdx.x, nsplit = gridDim.x;
  const int64_t f = blockIdx.y;
  const int p0 = k * SE_PX_PER_SPLIT, p1 = min(HW, p0 + SE_PX_PER_SPLIT);
  float acc[5][8];
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[q][j] = 0.f;
  if (cm.r < cm.rpp) {
    BnCh8 bc;
    bc.init(act, cm.c0);
    for (int p = p0 + cm.r; p < p1; p += cm.rpp) {
      const int64_t e = (f * HW + p) * C + cm.c0;
      float v[8], g[8];
      load8_nt(x + e, v);
      load8_nt(dy + e, g);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {   // packed pairs (gelu_phi_pair_t)
        const f32x2 vv = f32x2{v[j], v[j + 1]};
        const f32x2 u = vfma(vv, f32x2{bc.sc[j], bc.sc[j + 1]}, f32x2{bc.sh[j], bc.sh[j + 1]});
        f32x2 pdf;
        const f32x2 cdf = gelu_phi_pair_t<f32x2>(u, &pdf);
        f32x2 hv;
        {
#pragma clang fp contract(off)
          hv = u * cdf;
        }
        const f32x2 gv = vfma(u, pdf, cdf);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float xh = fmaf(v[j + i], bc.rs[j + i], -bc.mr[j + i]);
          const float h = to_f<T>(from_f<T>(hv[i]));   // the stored-precision SE input
          const float gp = act.gelu ? gv[i] : 1.f;
          const float hh = act.gelu ? h : to_f<T>(from_f<T>(u[i]));
          const float t = gp * xh;
          acc[0][j + i] = fmaf(g[j + i], hh, acc[0][j + i]);
          acc[1][j + i] = fmaf(g[j + i], gp, acc[1][j + i]);
          acc[2][j + i] += gp;
          acc[3][j + i] = fmaf(g[j + i], t, acc[3][j + i]);
          acc[4][j + i] += t;
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    if (q) __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = acc[q][j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      float a = 0.f;
      for (int rr = 0; rr < cm.rpp; ++rr) a += red[(rr * cm.nch + c / 8) * 8 + c % 8];
      if (q == 0) part[(f * nsplit + k) * C + c] = a;
      else part2[((f * nsplit + k) * 4 + (q - 1)) * C + c] = a;
    }
  }
}

// per frame: comb[f][0][c] = s A + dpool/HW B, comb[f][1][c] = s X + dpool/HW D
__global__ __launch_bounds__(256) void se_bn_combine_kernel(const float* part2, int nsplit, int HW, int C,
                                                            const float* s, const float* dpool, float* comb) {
  const int64_t f = blockIdx.x;
  const float inv = 1.f / (float)HW;
  for (int c = threadIdx.x; c < C; c += 256) {
    float q[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nsplit; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) q[i] += part2[((f * nsplit + k) * 4 + i) * C + c];
    const float sv = s[f * C + c], dp = dpool[f * C + c] * inv;
    comb[(f * 2 + 0) * C + c] = sv * q[0] + dp * q[1];
    comb[(f * 2 + 1) * C + c] = sv * q[2] + dp * q[3];
  }
}

// sums [2][C] (fp64) -> dgamma (+=), dbeta (+=), coef [2][C] = mean(du), mean(du xhat)
__global__ void se_bn_finalize_kernel(const double* sums, int64_t M, int C, float* dw, float* db, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double a = sums[c], b = sums[C + c];
  if (dw) dw[c] += (float)b;
  if (db) db[c] += (float)a;
  coef[c] = (float)(a / (double)M);
  coef[C + c] = (float)(b / (double)M);
}

// da2 = w rstd (du - mean(du) - xhat mean(du xhat)),  du = (dh3 s + dpool/HW) GELU'(u),
// expanded per (frame, channel) into da2 = GELU'(u) (dh3 A + B) + c0 - c1 x with
// A = w rstd s, B = w rstd dpool/HW, c1 = w rstd^2 mean(du xhat), c0 = w rstd (mean rstd
// mean(du xhat) - mean(du)): 6 constants per channel instead of 9 (the 9 held 72 VGPRs
// and the kernel at 4 waves per SIMD)
template <typename T>
__global__ __launch_bounds__(256) void se_bn_dx_kernel(const T* dy, const T* x, ChanAffine act, const float* s,
                                                       const float* dpool, const float* coef, T* dx, int HW,
                                                       int C) {
  const SeCols cm(C);
  if (cm.r >= cm.rpp) return;
  const int k = blockIdx.x;
  const int64_t f = blockIdx.y;
  const int p0 = k * SE_PX_PER_SPLIT, p1 = min(HW, p0 + SE_PX_PER_SPLIT);
  float sc[8], sh[8], ka[8], kb[8], c0[8], c1[8];
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cm.c0 + j;
    const float rs = act.rstd[c], mu = act.mean[c];
    sc[j] = rs * act.w[c];
    sh[j] = bn_shift(act.b[c], mu, sc[j]);
    const float wr = act.w[c] * rs, k1 = coef[C + c];
    ka[j] = wr * s[f * C + c];
    kb[j] = wr * (dpool[f * C + c] * inv);
    c1[j] = wr * k1 * rs;
    c0[j] = wr * (k1 * (mu * rs) - coef[c]);
  }
  for (int p = p0 + cm.r; p < p1; p += cm.rpp) {
    const int64_t e = (f * HW + p) * C + cm.c0;
    float v[8], g[8], o[8];
    load8_nt(x + e, v);
    load8_nt(dy + e, g);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {   // packed pairs (gelu_phi_pair_t)
      f32x2 gd = f32x2{1.f, 1.f};
      if (act.gelu)
        gd = gelu_grad2(vfma(f32x2{v[j], v[j + 1]}, f32x2{sc[j], sc[j + 1]}, f32x2{sh[j], sh[j + 1]}));
#pragma unroll
      for (int i = 0; i < 2; ++i)
        o[j + i] = fmaf(gd[i], fmaf(g[j + i], ka[j + i], kb[j + i]), fmaf(-c1[j + i], v[j + i], c0[j + i]));
    }
    store8_nt(dx + e, o);
  }
}

}  // namespace

#define DISPATCH1(DT, ...)                                       \
  do {                                                         \
    if ((DT) == SM_F32) { typedef float T; __VA_ARGS__; }      \
    else { typedef __bf16 T; __VA_ARGS__; }                    \
  } while (0)

// every host-side Ho / Wo computation divides by the stride: only 1 and 2 exist
static bool bad_stride(int s) { return s != 1 && s != 2; }

extern "C" int sm_stem_im2col(int out_dtype, const float* clip, int B, int T, int H, int W, int64_t sB, int64_t sC,
                              int64_t sT, int64_t sH, int64_t sW, int stride, void* col, hipStream_t st) {
  ClipView v{clip, B, T, H, W, sB, sC, sT, sH, sW};
  if (bad_stride(stride)) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int64_t P = (int64_t)B * T * Ho * Wo;
  if (P <= 0) return 0;
  DISPATCH1(out_dtype, hipLaunchKernelGGL(stem_im2col_kernel<T>, dim3(ew_blocks(P)), dim3(256), 0, st, v, Ho, Wo,
                                          stride, (T*)col));
  SM_CHECK_LAUNCH();
  return 0;
}

// stem conv1 + BN1 statistics (see stem_conv1_kernel); wpack = sm_conv_wpack order 0 [48][32] bf16
extern "C" int sm_bn_stats_from_partials(const float* part, int64_t nrows, int C, int64_t M, float* mean,
                                         float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                                         float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                                         hipStream_t st);
extern "C" int64_t sm_stem_conv1_workspace_bytes(void) {
  return (int64_t)SC1_BLOCKS * 2 * SC1_COUT * 4 + 2 * SC1_COUT * 8 + 64;
}
extern "C" int sm_stem_conv1_bn_stats(const float* clip, int B, int T, int H, int W, int64_t sB, int64_t sC,
                                      int64_t sT, int64_t sH, int64_t sW, const void* wpack, void* y, float* mean,
                                      float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                                      float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                                      hipStream_t st) {
  ClipView v{clip, B, T, H, W, sB, sC, sT, sH, sW};
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t P = (int64_t)B * T * Ho * Wo;
  if (P <= 0) return 0;
  if (P >= (1LL << 31) - 64 || (int64_t)3 * sC >= (1LL << 31)) return -2;
  if (ws_bytes < sm_stem_conv1_workspace_bytes()) return -4;
  if ((((uintptr_t)wpack) | ((uintptr_t)y)) & 15) return -2;
  float* part = (float*)ws;
  void* fin = (void*)(((uintptr_t)(part + (int64_t)SC1_BLOCKS * 2 * SC1_COUT) + 15) & ~(uintptr_t)15);
  const size_t band_lds = (size_t)3 * SC1B_NRI * (W + 2 * SC1B_PADL) * 2;
  int nb;
  if (band_lds <= 48 * 1024) {   // band form: input rows staged through LDS
    const int64_t nbands = (int64_t)B * T * ((Ho + SC1B_R - 1) / SC1B_R);
    nb = (int)std::min<int64_t>(SC1_BLOCKS, nbands);
    const int vec4 = sW == 1 && W % 4 == 0 && sH % 4 == 0 && sC % 4 == 0 && sT % 4 == 0 && sB % 4 == 0 &&
                     (((uintptr_t)clip) & 15) == 0;
    hipLaunchKernelGGL(stem_conv1_band_kernel, dim3(nb), dim3(256), band_lds, st, v, Ho, Wo, (const __bf16*)wpack,
                       (__bf16*)y, part, vec4);
  } else {
    const int64_t nseg = (P + 31) / 32;
    nb = (int)std::min<int64_t>(SC1_BLOCKS, (nseg + 3) / 4);   // part rows
    hipLaunchKernelGGL(stem_conv1_kernel, dim3(nb), dim3(256), 0, st, v, Ho, Wo, (const __bf16*)wpack, (__bf16*)y,
                       part);
  }
  SM_CHECK_LAUNCH();
  return sm_bn_stats_from_partials(part, nb, SC1_COUT, P, mean, rstd, run_mean, run_var, num_batches_tracked,
                                   momentum, eps, updates, fin, 2 * SC1_COUT * 8, st);
}

// stem conv2 over GELU(BN1(a1)) + BN2 statistics (see stem_conv2_kernel)
extern "C" int64_t sm_stem_conv2_workspace_bytes(int F) { return (int64_t)F * 2 * SC2_COUT * 4 + 2 * SC2_COUT * 8 + 64; }
extern "C" int sm_stem_conv2_bn_stats(const void* a1, int F, int H, int W, const float* bn1_mean,
                                      const float* bn1_rstd, const float* bn1_w, const float* bn1_b, int gelu,
                                      const void* wpack, void* y, float* mean, float* rstd, float* run_mean,
                                      float* run_var, int64_t* num_batches_tracked, float momentum, float eps,
                                      int updates, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (F <= 0) return 0;
  if (H <= 0 || W <= 0 || W > 4 * 32 || (int64_t)F * H * W >= (1LL << 31)) return -2;   // W <= 4 segments
  if ((((uintptr_t)a1) | ((uintptr_t)wpack) | ((uintptr_t)y)) & 15) return -2;
  if (ws_bytes < sm_stem_conv2_workspace_bytes(F)) return -4;
  float* part = (float*)ws;
  void* fin = (void*)(((uintptr_t)(part + (int64_t)F * 2 * SC2_COUT) + 15) & ~(uintptr_t)15);
  // staged epilogue: its LDS image must fit in pixel columns 1 .. W of a ring slot
  const bool staged = (int64_t)(W + 1) * SC2_PITCH * 2 >= SC2_PITCH * 2 + (SC2_NW / 2) * 2048;
  auto kern = gelu ? (staged ? stem_conv2_kernel<true, true> : stem_conv2_kernel<true, false>)
                   : (staged ? stem_conv2_kernel<false, true> : stem_conv2_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(F), dim3(SC2_NT), 0, st, (const __bf16*)a1,
                     ChanAffine{bn1_mean, bn1_rstd, bn1_w, bn1_b, gelu}, (const __bf16*)wpack, (__bf16*)y, part, H, W);
  SM_CHECK_LAUNCH();
  return sm_bn_stats_from_partials(part, F, SC2_COUT, (int64_t)F * H * W, mean, rstd, run_mean, run_var,
                                   num_batches_tracked, momentum, eps, updates, fin, 2 * SC2_COUT * 8, st);
}

extern "C" int sm_im2col3(int dtype, const void* x, int F, int H, int W, int C, int stride, void* col,
                          hipStream_t st) {
  if (C % 8) return -2;
  if (bad_stride(stride)) return -2;
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
  if (bad_stride(stride)) return -2;
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
  if (order == 2 && Kpad < 9 * Cout) return -2;
  const int total = (order == 2 ? Cin : Cout) * Kpad;
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
  if (bad_stride(stride)) return -2;
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

static size_t dwf_lds_bytes(int W, int stride) {
  const int NR = stride == 1 ? DwRing<1>::NR : DwRing<2>::NR;
  size_t lds = (size_t)NR * (W + 2) * 64 + 9 * DWF_CB * 4;   // ring + taps
  return lds < 256 * 16 * 4 ? 256 * 16 * 4 : lds;   // the statistics reduction reuses it
}

static int dwf_remap() { return 1; }

static bool dwf_shape_ok(int F, int W, int C, int stride) {
  return C % DWF_CB == 0 && (stride == 1 || stride == 2) && F > 0 && (int64_t)F * (C / DWF_CB) < (1LL << 31) &&
         DwRing<2>::NEW * W * 4 <= 256 * DWF_KV && DwRing<1>::NEW * W * 4 <= 256 * DWF_KV &&
         dwf_lds_bytes(W, stride) <= 64 * 1024;
}

extern "C" int64_t sm_dwconv_fused_partial_rows(int F, int H, int stride) { return F; }

extern "C" int sm_dwconv_fused_fwd(int F, int H, int W, int C, int stride, const void* x, const float* in_mean,
                                   const float* in_rstd, const float* in_w, const float* in_b, int in_gelu,
                                   const float* w, void* y, float* part, hipStream_t st) {
  if (!dwf_shape_ok(F, W, C, stride)) return -2;
  if (((uintptr_t)w & 15) || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return -2;
  if (bad_stride(stride)) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  ChanAffine act{in_mean, in_rstd, in_w, in_b, in_gelu};
  const dim3 grid((C / DWF_CB) * F);
  const size_t lds = dwf_lds_bytes(W, stride);
  const int remap = dwf_remap();
  if (stride == 1 && part)
    hipLaunchKernelGGL((dwf_fwd_kernel<1>), grid, dim3(256), lds, st, (const __bf16*)x, act, w, (__bf16*)y, part,
                       H, W, C, Ho, Wo, remap);
  else if (stride == 1)
    hipLaunchKernelGGL((dwf_fwd_kernel<1, false>), grid, dim3(256), lds, st, (const __bf16*)x, act, w, (__bf16*)y,
                       part, H, W, C, Ho, Wo, remap);
  else if (part)
    hipLaunchKernelGGL((dwf_fwd_kernel<2>), grid, dim3(256), lds, st, (const __bf16*)x, act, w, (__bf16*)y, part,
                       H, W, C, Ho, Wo, remap);
  else
    hipLaunchKernelGGL((dwf_fwd_kernel<2, false>), grid, dim3(256), lds, st, (const __bf16*)x, act, w, (__bf16*)y,
                       part, H, W, C, Ho, Wo, remap);
  SM_CHECK_LAUNCH();
  return 0;
}

// Fused backward of y = dwconv(act(x)): dx = dL/d act(x) (stride 1: the forward
// kernel with the taps rotated 180 degrees; stride 2: dw_dgrad_kernel), dw += the
// fused weight gradient.
__global__ void dw_rotate_kernel(const float* w, float* wrot, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) wrot[i] = w[(i / 9) * 9 + 8 - i % 9];
}

extern "C" int64_t sm_dwconv_fused_bwd_workspace_bytes(int F, int H, int W, int C, int stride) {
  return (int64_t)F * C * 9 * 4 + (int64_t)C * 9 * 4 + 64;
}

extern "C" int sm_dwconv_fused_bwd(int F, int H, int W, int C, int stride, const void* dy, const void* x,
                                   const float* in_mean, const float* in_rstd, const float* in_w, const float* in_b,
                                   int in_gelu, const float* w, void* dx, float* dw, void* ws, int64_t ws_bytes,
                                   hipStream_t st) {
  if (!dwf_shape_ok(F, W, C, stride)) return -2;
  if (ws_bytes < sm_dwconv_fused_bwd_workspace_bytes(F, H, W, C, stride)) return -4;
  if (bad_stride(stride)) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const size_t lds = dwf_lds_bytes(W, stride);
  float* part = (float*)ws;
  float* wrot = (float*)(((uintptr_t)(part + (int64_t)F * C * 9) + 15) & ~(uintptr_t)15);
  if (dx) {
    if (stride == 1) {
      hipLaunchKernelGGL(dw_rotate_kernel, dim3((C * 9 + 255) / 256), dim3(256), 0, st, w, wrot, C * 9);
      ChanAffine none{nullptr, nullptr, nullptr, nullptr, 0};
      hipLaunchKernelGGL((dwf_fwd_kernel<1, false>), dim3((C / DWF_CB) * F), dim3(256), lds, st, (const __bf16*)dy, none,
                         (const float*)wrot, (__bf16*)dx, (float*)nullptr, Ho, Wo, C, H, W, dwf_remap());
    } else {
      const int64_t total = (int64_t)F * H * ((W + DW_PX - 1) / DW_PX) * (C / 8);
      hipLaunchKernelGGL((dw_dgrad_kernel<__bf16, 2>), dim3((int)((total + 255) / 256)), dim3(256), 0, st,
                         (const __bf16*)dy, w, (__bf16*)dx, F, H, W, C, Ho, Wo);
    }
  }
  ChanAffine act{in_mean, in_rstd, in_w, in_b, in_gelu};
  const dim3 g2((C / DWF_CB) * F);
  if (stride == 1)
    hipLaunchKernelGGL((dwf_wgrad_kernel<1>), g2, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, act, part,
                       H, W, C, Ho, Wo, dwf_remap());
  else
    hipLaunchKernelGGL((dwf_wgrad_kernel<2>), g2, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, act, part,
                       H, W, C, Ho, Wo, dwf_remap());
  colred(part, F, C * 9, nullptr, dw, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

// Stride-1 depthwise + BatchNorm(+GELU) backward (dwb_kernel): dx = dL/dx for
// y = dwconv3x3(GELU(BN(x))), dw += dL/dw, dgamma / dbeta += the BatchNorm's.
extern "C" int64_t sm_dwconv_bn_bwd_workspace_bytes(int F, int H, int W, int C) {
  return ((int64_t)F * C * 9 + (int64_t)F * 2 * C + 2 * C) * 4 + 2 * C * 8 + 64;
}

static int dwconv_bn_bwd(int stride, int F, int H, int W, int C, const void* dy, const void* x, const float* bn_mean,
                         const float* bn_rstd, const float* bn_w, const float* bn_b, int bn_gelu, const float* w,
                         void* dx, float* dw, float* dgamma, float* dbeta, void* ws, int64_t ws_bytes,
                         hipStream_t st) {
  if (bad_stride(stride)) return -2;
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  size_t lds = stride == 1 ? dwf_lds_bytes(W, 1) + DWB_PAD + 4 * DWF_CB * 4
                           : (size_t)DwRing<1, DWB2_TYO>::NR * (Wo + 2) * 64 + DWB2_PAD + 13 * DWF_CB * 4;
  if (lds < 256 * 4 * 4) lds = 256 * 4 * 4;   // the reductions reuse it ([256][4] floats)
  if (!dwf_shape_ok(F, W, C, stride) || !bn_mean || !dx || lds > 64 * 1024) return -2;
  if (stride == 2 && DwRing<1, DWB2_TYO>::NEW * Wo * 4 > 256 * DWF_KV) return -2;
  if (((uintptr_t)x & 15) || ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15) || C / 8 > 256) return -2;
  if (ws_bytes < sm_dwconv_bn_bwd_workspace_bytes(F, H, W, C)) return -4;
  float* part_w = (float*)ws;
  float* part_bn = part_w + (int64_t)F * C * 9;
  float* coef = part_bn + (int64_t)F * 2 * C;
  double* sums = (double*)(((uintptr_t)(coef + 2 * C) + 7) & ~(uintptr_t)7);
  ChanAffine bn{bn_mean, bn_rstd, bn_w, bn_b, bn_gelu};
  const dim3 grid((C / DWF_CB) * F);
  if (stride == 2) {
    const bool rag = W % DWB2_PX != 0;
    if (bn_gelu && !rag)
      hipLaunchKernelGGL((dwb2_kernel<true, false>), grid, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, bn,
                         w, (__bf16*)dx, part_w, part_bn, H, W, C, Ho, Wo, dwf_remap());
    else if (bn_gelu)
      hipLaunchKernelGGL((dwb2_kernel<true, true>), grid, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, bn,
                         w, (__bf16*)dx, part_w, part_bn, H, W, C, Ho, Wo, dwf_remap());
    else
      hipLaunchKernelGGL((dwb2_kernel<false, true>), grid, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, bn,
                         w, (__bf16*)dx, part_w, part_bn, H, W, C, Ho, Wo, dwf_remap());
  } else {
    // (the range-select-free stride-1 form measured 256 VGPRs + 304 B of scratch: the
    // compiler's schedule of the select-free GELU chains; it keeps the ragged form)
    if (bn_gelu)
      hipLaunchKernelGGL((dwb_kernel<true, true>), grid, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, bn,
                         w, (__bf16*)dx, part_w, part_bn, H, W, C, dwf_remap());
    else
      hipLaunchKernelGGL((dwb_kernel<false, true>), grid, dim3(256), lds, st, (const __bf16*)dy, (const __bf16*)x, bn,
                         w, (__bf16*)dx, part_w, part_bn, H, W, C, dwf_remap());
  }
  colred(part_w, F, C * 9, nullptr, dw, 1, st);
  colred(part_bn, F, 2 * C, sums, nullptr, 0, st);
  const int64_t M = (int64_t)F * H * W;
  hipLaunchKernelGGL(se_bn_finalize_kernel, dim3((C + 127) / 128), dim3(128), 0, st, sums, M, C, dgamma, dbeta,
                     coef);
  int64_t rpb = (M + 4095) / 4096;
  if (rpb < 16) rpb = 16;
  hipLaunchKernelGGL(dwb_dx_kernel, dim3((unsigned)((M + rpb - 1) / rpb)), dim3(256), 0, st, (const __bf16*)x, bn,
                     (const float*)coef, (__bf16*)dx, M, C, (int)rpb);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_dwconv_bn_bwd(int F, int H, int W, int C, const void* dy, const void* x, const float* bn_mean,
                                const float* bn_rstd, const float* bn_w, const float* bn_b, int bn_gelu,
                                const float* w, void* dx, float* dw, float* dgamma, float* dbeta, void* ws,
                                int64_t ws_bytes, hipStream_t st) {
  return dwconv_bn_bwd(1, F, H, W, C, dy, x, bn_mean, bn_rstd, bn_w, bn_b, bn_gelu, w, dx, dw, dgamma, dbeta, ws,
                       ws_bytes, st);
}

// Stride-2 form (dwb2_kernel): F, H, W, C are the input's; dy is [F][Ho][Wo][C].
extern "C" int sm_dwconv_s2_bn_bwd(int F, int H, int W, int C, const void* dy, const void* x, const float* bn_mean,
                                   const float* bn_rstd, const float* bn_w, const float* bn_b, int bn_gelu,
                                   const float* w, void* dx, float* dw, float* dgamma, float* dbeta, void* ws,
                                   int64_t ws_bytes, hipStream_t st) {
  return dwconv_bn_bwd(2, F, H, W, C, dy, x, bn_mean, bn_rstd, bn_w, bn_b, bn_gelu, w, dx, dw, dgamma, dbeta, ws,
                       ws_bytes, st);
}

extern "C" int64_t sm_dwconv_wgrad_workspace_bytes(int F, int H, int W, int C, int stride) {
  if (bad_stride(stride)) return 0;
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
  if (bad_stride(stride)) return -2;
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

extern "C" int64_t sm_se_workspace_bytes(int F, int HW, int C) {
  return (int64_t)F * se_splits(HW) * C * 4 + (int64_t)F * C * 4 + 64;
}

// y = act(x) * sigmoid(W2 relu(W1 mean_hw act(x)))  (y nullable: gate only)
extern "C" int sm_se_fwd(int dtype, const void* x, const float* act_mean, const float* act_rstd, const float* act_w,
                         const float* act_b, int act_gelu, int F, int HW, int C, int R, const float* w1,
                         const float* w2, float* pooled, float* z1, float* s, void* y, void* ws, int64_t ws_bytes,
                         hipStream_t st) {
  if (C % 8 || C / 8 > 256 || F <= 0 || F > 65535 || HW <= 0) return -2;
  const int ns = se_splits(HW);
  if (ws_bytes < (int64_t)F * ns * C * 4) return -4;
  float* part = (float*)ws;
  ChanAffine act{act_mean, act_rstd, act_w, act_b, act_gelu};
  DISPATCH1(dtype, hipLaunchKernelGGL(se_reduce_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)x,
                                      (const T*)nullptr, act, HW, C, part));
  hipLaunchKernelGGL(se_fc_fwd_kernel, dim3(F), dim3(256), (C + R) * 4, st, part, ns, HW, w1, w2, C, R, pooled, z1,
                     s);
  if (y)
    DISPATCH1(dtype, hipLaunchKernelGGL(se_apply_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)x, act, s,
                                        (const float*)nullptr, (T*)y, HW, C));
  SM_CHECK_LAUNCH();
  return 0;
}

// Backward of y = h * s(h), h = act(x).  Writes dx = dL/dh and the per-frame FC
// gradients dz2 [F][C], dz1 [F][R] (the weight grads are two small GEMMs).
extern "C" int sm_se_bwd(int dtype, const void* dy, const void* x, const float* act_mean, const float* act_rstd,
                         const float* act_w, const float* act_b, int act_gelu, int F, int HW, int C, int R,
                         const float* w1, const float* w2, const float* s, const float* z1, float* dz2, float* dz1,
                         void* dx, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (C % 8 || C / 8 > 256 || F <= 0 || F > 65535 || HW <= 0) return -2;
  const int ns = se_splits(HW);
  if (ws_bytes < (int64_t)F * ns * C * 4 + (int64_t)F * C * 4) return -4;
  float* part = (float*)ws;
  float* dpool = part + (int64_t)F * ns * C;
  ChanAffine act{act_mean, act_rstd, act_w, act_b, act_gelu};
  ChanAffine none{nullptr, nullptr, nullptr, nullptr, 0};
  DISPATCH1(dtype, hipLaunchKernelGGL(se_reduce_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)x,
                                      (const T*)dy, act, HW, C, part));
  hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(F), dim3(256), (C + R) * 4, st, part, ns, s, z1, w1, w2, C, R, dz2, dz1,
                     dpool);
  DISPATCH1(dtype, hipLaunchKernelGGL(se_apply_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)dy, none, s,
                                      (const float*)dpool, (T*)dx, HW, C));
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_se_scale(int dtype, const void* x, const float* act_mean, const float* act_rstd,
                           const float* act_w, const float* act_b, int act_gelu, const float* s, void* y, int F,
                           int HW, int C, hipStream_t st) {
  if (C % 8 || C / 8 > 256 || F > 65535) return -2;
  if (F <= 0 || HW <= 0) return 0;
  ChanAffine act{act_mean, act_rstd, act_w, act_b, act_gelu};
  DISPATCH1(dtype, hipLaunchKernelGGL(se_apply_kernel<T>, dim3(se_splits(HW), F), dim3(256), 0, st, (const T*)x,
                                      act, s, (const float*)nullptr, (T*)y, HW, C));
  SM_CHECK_LAUNCH();
  return 0;
}

// Fused backward of h3 = SE(h2), h2 = GELU(BN2(x)) (batch statistics mean/rstd of x
// over M = F*HW rows): dx = dL/dx, dz2 / dz1 as sm_se_bwd, dgamma / dbeta += (dw, db).
extern "C" int64_t sm_se_bn_bwd_workspace_bytes(int F, int HW, int C) {
  const int64_t ns = se_splits(HW);
  return (F * ns * C + (int64_t)F * C + F * ns * 4 * C + (int64_t)F * 2 * C + 2 * C) * 4 + 2 * C * 8 + 64;
}

extern "C" int sm_se_bn_bwd(int dtype, const void* dy, const void* x, const float* bn_mean, const float* bn_rstd,
                            const float* bn_w, const float* bn_b, int bn_gelu, int F, int HW, int C, int R,
                            const float* w1, const float* w2, const float* s, const float* z1, float* dz2,
                            float* dz1, void* dx, float* dw, float* db, void* ws, int64_t ws_bytes,
                            hipStream_t st) {
  if (C % 8 || C / 8 > 256 || F <= 0 || F > 65535 || HW <= 0 || !bn_mean) return -2;
  if (ws_bytes < sm_se_bn_bwd_workspace_bytes(F, HW, C)) return -4;
  const int ns = se_splits(HW);
  float* part = (float*)ws;
  float* dpool = part + (int64_t)F * ns * C;
  float* part2 = dpool + (int64_t)F * C;
  float* comb = part2 + (int64_t)F * ns * 4 * C;
  float* coef = comb + (int64_t)F * 2 * C;
  double* sums = (double*)(((uintptr_t)(coef + 2 * C) + 7) & ~(uintptr_t)7);
  ChanAffine act{bn_mean, bn_rstd, bn_w, bn_b, bn_gelu};
  DISPATCH1(dtype, hipLaunchKernelGGL(se_bn_reduce_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)dy,
                                      (const T*)x, act, HW, C, part, part2));
  hipLaunchKernelGGL(se_fc_bwd_kernel, dim3(F), dim3(256), (C + R) * 4, st, part, ns, s, z1, w1, w2, C, R, dz2, dz1,
                     dpool);
  hipLaunchKernelGGL(se_bn_combine_kernel, dim3(F), dim3(256), 0, st, part2, ns, HW, C, s, dpool, comb);
  colred(comb, F, 2 * C, sums, nullptr, 0, st);
  hipLaunchKernelGGL(se_bn_finalize_kernel, dim3((C + 127) / 128), dim3(128), 0, st, sums, (int64_t)F * HW, C, dw,
                     db, coef);
  DISPATCH1(dtype, hipLaunchKernelGGL(se_bn_dx_kernel<T>, dim3(ns, F), dim3(256), 0, st, (const T*)dy, (const T*)x,
                                      act, s, dpool, coef, (T*)dx, HW, C));
  SM_CHECK_LAUNCH();
  return 0;
}
