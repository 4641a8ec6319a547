// Clip normalisation on the GPU: the per-frame transform and channel swap of the
// reference's data path (src/train_ssl_mae.py:137-141 T.PILToTensor ->
// T.ConvertImageDtype(float) -> T.Normalize(ImageNet mean/std), then
// src/datasets/mae_loader.py:70-77 img[[2,1,0]] and the [T,C,H,W] -> [C,T,H,W]
// permute), applied to a whole batch of decoded frames after ONE host-to-device
// copy of uint8 pixels (1/4 of the fp32 bytes the reference's loader ships).
//
// in  : uint8 [B][T][H][W][3] (PIL RGB order, HWC), valid[B] (nullable)
// out : fp32  [B][3][T][H][W]   (the collated clip the reference feeds the model)
// out[b][c][t][h][w] = (u / 255 - mean[s]) / std[s], u = in[b][t][h][w][s], s = c
// or 2 - c (bgr_swap).  Division is IEEE (correctly rounded), as torch's
// ConvertImageDtype / Normalize on the CPU; no FMA is possible (sub, then div), so
// values are bit-identical to the reference transform.  An invalid clip (missing
// directory / no frames, mae_loader.py:35-43) is written as zeros.
//
// HBM-bound: 3 B read + 12 B written per pixel.  A uint8 input has 256 values per
// channel, so each block first tabulates the 3 x 256 outputs in LDS (the two IEEE
// divisions run 768 times per block instead of twice per element) and the stream
// loop is loads, LDS lookups and stores.  One lane handles 4 consecutive pixels:
// three dword loads (12 B of interleaved RGB) and one 16-B store per channel
// plane, so each wave writes three contiguous 1 KiB runs.
#include "common.h"
#include "sm_api.h"

namespace {

struct Norm {
  float mean[3];
  float std[3];
};

SM_DEV float norm1(uint32_t u, float mean, float sd) { return ((float)u / 255.0f - mean) / sd; }

__global__ void __launch_bounds__(256) frames_norm4_kernel(const uint8_t* __restrict__ in,
                                                          const uint8_t* __restrict__ valid, Norm nm, int bgr,
                                                          int T, int64_t hw, int64_t total4,
                                                          float* __restrict__ out) {
  __shared__ float lut[3][256];   // lut[c][u]: output channel c (swap applied), input byte u
  for (int i = threadIdx.x; i < 768; i += blockDim.x) {
    const int c = i >> 8, s = bgr ? 2 - c : c;
    lut[c][i & 255] = norm1(i & 255, nm.mean[s], nm.std[s]);
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total4; g += stride) {
    const int64_t pix = g * 4;                 // first of 4 pixels (never straddles a frame: hw % 4 == 0)
    const int64_t frame = pix / hw;            // b * T + t
    const int64_t off = pix - frame * hw;
    const int64_t b = frame / T, t = frame - b * T;
    const uint32_t* src = (const uint32_t*)(in + pix * 3);
    const uint32_t w0 = src[0], w1 = src[1], w2 = src[2];
    // bytes: r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
    const uint32_t px[3][4] = {{w0 & 255, (w0 >> 24), (w1 >> 16) & 255, (w2 >> 8) & 255},
                               {(w0 >> 8) & 255, w1 & 255, (w1 >> 24), (w2 >> 16) & 255},
                               {(w0 >> 16) & 255, (w1 >> 8) & 255, w2 & 255, (w2 >> 24)}};
    const bool ok = valid == nullptr || valid[b] != 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int s = bgr ? 2 - c : c;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = ok ? lut[c][px[s][e]] : 0.0f;
      float* dst = out + ((b * 3 + c) * (int64_t)T + t) * hw + off;
      __builtin_nontemporal_store(v, (f32x4*)dst);
    }
  }
}

__global__ void frames_norm1_kernel(const uint8_t* __restrict__ in, const uint8_t* __restrict__ valid, Norm nm,
                                    int bgr, int T, int64_t hw, int64_t total, float* __restrict__ out) {
  const int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= total) return;
  const int64_t frame = pix / hw, off = pix - frame * hw;
  const int64_t b = frame / T, t = frame - b * T;
  const bool ok = valid == nullptr || valid[b] != 0;
  for (int c = 0; c < 3; ++c) {
    const int s = bgr ? 2 - c : c;
    out[((b * 3 + c) * (int64_t)T + t) * hw + off] = ok ? norm1(in[pix * 3 + s], nm.mean[s], nm.std[s]) : 0.0f;
  }
}

}  // namespace

extern "C" int sm_frames_normalize(const uint8_t* frames, const uint8_t* valid, int B, int T, int H, int W,
                                   const float* mean3, const float* std3, int bgr_swap, float* out,
                                   hipStream_t st) {
  if (B < 0 || T < 0 || H < 0 || W < 0) return -2;
  const int64_t hw = (int64_t)H * W, total = (int64_t)B * T * hw;
  if (total == 0) return 0;
  if (!frames || !mean3 || !std3 || !out) return -2;   // (mean3 / std3 are host arrays)
  Norm nm;
  for (int c = 0; c < 3; ++c) {
    nm.mean[c] = mean3[c];
    nm.std[c] = std3[c];
  }
  if (hw % 4 == 0 && ((uintptr_t)frames & 3u) == 0 && ((uintptr_t)out & 15u) == 0) {
    const int64_t total4 = total / 4;
    int64_t blocks = (total4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(frames_norm4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, frames, valid, nm, bgr_swap,
                       T, hw, total4, out);
  } else {
    hipLaunchKernelGGL(frames_norm1_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, frames, valid,
                       nm, bgr_swap, T, hw, total, out);
  }
  SM_CHECK_LAUNCH();
  return 0;
}
