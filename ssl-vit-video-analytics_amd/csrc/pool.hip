// Segment means for the frozen-encoder fine-tune head (BASELINE config 4).
//
// The reference's VideoClassifier (src/train_finetune.py:19-40) pools each frame's
// feature map to an embedding (F.adaptive_avg_pool2d(feat, 1), the backbone head
// pattern of src/models/mobilevit.py:164-165) and averages the embeddings over time
// (feats.mean(dim=1), train_finetune.py:38).  Both are "mean over R rows of a
// [G][R][C] block": the channels-last encoder tokens [frames][h*w][C] pooled per
// frame, then the fp32 embeddings [clips][T][C] pooled per clip.
//
// One block per (segment, 64-channel slice): 4 row groups x 64 channels, fixed-order
// fp32 partial sums, fixed-order LDS combine (deterministic), one multiply by 1/R.
// Bytes: read G*R*C*elt once, write G*C*4 -- a single HBM pass.
#include "common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void segment_mean_kernel(const T* __restrict__ x, int R, int C,
                                                           float* __restrict__ out) {
  __shared__ float red[4][64];
  const int nslice = (C + 63) / 64;
  const int g = blockIdx.x / nslice;
  const int c = (blockIdx.x % nslice) * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C) {
    const T* p = x + (int64_t)g * R * C + c;
    for (int r = rg; r < R; r += 4) s += to_f<T>(p[(int64_t)r * C]);
  }
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < C) out[(int64_t)g * C + c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                                   (red[2][threadIdx.x] + red[3][threadIdx.x])) * (1.0f / (float)R);
}

template <typename T>
__global__ __launch_bounds__(256) void segment_mean_bwd_kernel(const float* __restrict__ dy, int64_t total, int R,
                                                               int C, T* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int64_t g = i / ((int64_t)R * C);
    dx[i] = from_f<T>(dy[g * C + c] * (1.0f / (float)R));
  }
}

}  // namespace

extern "C" int sm_segment_mean(int dtype, const void* x, int G, int R, int C, float* out, hipStream_t st) {
  if (G <= 0 || R <= 0 || C <= 0) return -2;
  const int64_t nb = (int64_t)G * ((C + 63) / 64);
  if (nb > 0x7fffffff) return -2;
  if (dtype == SM_BF16)
    hipLaunchKernelGGL(segment_mean_kernel<__bf16>, dim3((unsigned)nb), dim3(256), 0, st, (const __bf16*)x, R, C,
                       out);
  else
    hipLaunchKernelGGL(segment_mean_kernel<float>, dim3((unsigned)nb), dim3(256), 0, st, (const float*)x, R, C,
                       out);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_segment_mean_bwd(int dtype, const float* dy, int G, int R, int C, void* dx, hipStream_t st) {
  if (G <= 0 || R <= 0 || C <= 0) return -2;
  const int64_t total = (int64_t)G * R * C;
  const int64_t want = (total + 255) / 256;
  const unsigned nb = (unsigned)(want < 65536 ? want : 65536);
  if (dtype == SM_BF16)
    hipLaunchKernelGGL(segment_mean_bwd_kernel<__bf16>, dim3(nb), dim3(256), 0, st, dy, total, R, C, (__bf16*)dx);
  else
    hipLaunchKernelGGL(segment_mean_bwd_kernel<float>, dim3(nb), dim3(256), 0, st, dy, total, R, C, (float*)dx);
  SM_CHECK_LAUNCH();
  return 0;
}
