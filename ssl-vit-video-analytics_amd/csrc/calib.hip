// Box calibration for bench.py: a bare bf16 MFMA loop on random register data.
//
// Why: MI355X devices hold different clocks under the same MFMA load (DVFS;
// MI355X_MICROARCH.md 'DVFS give-back' items 5 and 7: one binary 12 % apart across
// devices), so a bench line alone cannot tell a slow box from slow code.  bench.py
// runs this loop before the timed steps and reports its TFLOP/s and the in-kernel
// clock next to clips/s.
//
// Each workgroup is 4 waves; every wave issues `iters` x (8 v_mfma_f32_32x32x16_bf16 on
// 4 accumulators) or the same FLOPs as 16 v_mfma_f32_16x16x32_bf16 on 8 accumulators,
// operands fixed in registers and filled from a per-lane hash (random bf16 in +-[1, 2):
// zero or trivial operands run at a higher clock and miss the effect, guide item 7).
// Wave 0 stamps s_memtime / s_memrealtime around its loop; stamps[block] =
// {delta shader cycles, delta 100-MHz ticks}, so the clock is delta_mem / delta_real x 100 MHz
// (guide item 6).  The accumulators leave through `sink` so no MFMA is dead.
#include "common.h"
#include "sm_api.h"

namespace {

SM_DEV uint32_t lane_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// random bf16: random sign and mantissa, exponent of 1.0, so |v| in [1, 2)
SM_DEV bf16x8 rand_frag(uint32_t seed) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t h = lane_hash(seed * 8u + (uint32_t)j);
    const uint16_t bits = (uint16_t)(((h & 1u) << 15) | (127u << 7) | ((h >> 1) & 0x7Fu));
    f[j] = __builtin_bit_cast(__bf16, bits);
  }
  return f;
}

template <int SHAPE>
__global__ __launch_bounds__(256) void calib_mfma_kernel(int iters, int64_t* stamps, float* sink) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const bf16x8 a0 = rand_frag(4 * t), a1 = rand_frag(4 * t + 1), b0 = rand_frag(4 * t + 2), b1 = rand_frag(4 * t + 3);
  uint64_t m0 = 0, r0 = 0;
  if (threadIdx.x < 64) {
    m0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  float out = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[i], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) out += acc[i][r];
  } else {
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[i], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) out += acc[i][r];
  }
  if (threadIdx.x < 64) {
    const uint64_t m1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
      stamps[2 * blockIdx.x] = (int64_t)(m1 - m0);
      stamps[2 * blockIdx.x + 1] = (int64_t)(r1 - r0);
    }
  }
  sink[t] = out;
}

}  // namespace

extern "C" int sm_calibrate_mfma(int shape, int iters, int blocks, int64_t* stamps, float* sink, hipStream_t st) {
  if (iters <= 0 || blocks <= 0) return 0;
  if (shape == 32)
    hipLaunchKernelGGL(calib_mfma_kernel<32>, dim3(blocks), dim3(256), 0, st, iters, stamps, sink);
  else if (shape == 16)
    hipLaunchKernelGGL(calib_mfma_kernel<16>, dim3(blocks), dim3(256), 0, st, iters, stamps, sink);
  else
    return -2;
  SM_CHECK_LAUNCH();
  return 0;
}
