// FedAvg aggregation on the GPU (reference: src/federated/fed_loop.py:14-62).
//
// The reference averages client state_dicts on the CPU, key by key:
//   acc = zeros; for (state, w) in clients: acc += state[k].to(f32) * (w / total_w)
// (fed_loop.py:46-49) and takes the max over clients for num_batches_tracked
// (:52-55).  Here every floating-point entry of a state_dict lives in one flat fp32
// buffer per client (same key order), so one launch aggregates the whole model:
// each element is read once from each client and written once — (K + 1) * 4 B per
// parameter, HBM-bound.  The accumulation order and rounding are the reference's:
// acc starts at +0, then for each client in list order acc = acc + (x * w) with
// the product and the sum rounded separately (no FMA contraction), w the fp32
// rounding of w_i / total_w.  The result is therefore bit-identical to
// fedavg_aggregate's.
#include "common.h"
#include "sm_api.h"

// The reference rounds x * w and acc + (x * w) separately: this file is compiled
// with -ffp-contract=off (build.py FILE_FLAGS) so no FMA is formed.

namespace {

constexpr int kMaxClients = SM_FEDAVG_MAX_CLIENTS;

struct ClientPtrs {
  const float* p[kMaxClients];
  float w[kMaxClients];
};

struct ClientCounters {
  const int64_t* p[kMaxClients];
};

// 16 B per lane per client; grid-stride over float4 groups.  KC > 0: client count
// known at compile time, so all KC loads of an element group are issued before the
// first multiply-add (KC x 16 B in flight per lane); KC == 0: runtime count.
template <int KC>
__global__ void __launch_bounds__(256) fedavg_sum4_kernel(ClientPtrs c, int k, int64_t n4, float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (KC > 0) {
      f32x4 x[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) x[j] = __builtin_nontemporal_load((const f32x4*)c.p[j] + i);
#pragma unroll
      for (int j = 0; j < KC; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], __fmul_rn(x[j][e], c.w[j]));
    } else {
      for (int j = 0; j < k; ++j) {
        const f32x4 x = __builtin_nontemporal_load((const f32x4*)c.p[j] + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], __fmul_rn(x[e], c.w[j]));
      }
    }
    __builtin_nontemporal_store(acc, (f32x4*)out + i);
  }
}

__global__ void fedavg_sum1_kernel(ClientPtrs c, int k, int64_t begin, int64_t n, float* __restrict__ out) {
  const int64_t i = begin + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float acc = 0.f;
  for (int j = 0; j < k; ++j) acc = __fadd_rn(acc, __fmul_rn(c.p[j][i], c.w[j]));
  out[i] = acc;
}

__global__ void counters_max_kernel(ClientCounters c, int k, int64_t n, int64_t* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t m = c.p[0][i];
  for (int j = 1; j < k; ++j) m = c.p[j][i] > m ? c.p[j][i] : m;
  out[i] = m;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" int sm_fedavg_weighted_sum(int num_clients, const float* const* client_bufs, const float* weights,
                                      int64_t n, float* out, hipStream_t st) {
  if (num_clients < 1 || num_clients > kMaxClients || n < 0) return -2;
  if (n == 0) return 0;
  if (!client_bufs || !weights || !out) return -2;
  ClientPtrs c{};
  bool vec = aligned16(out);
  for (int j = 0; j < num_clients; ++j) {
    if (!client_bufs[j]) return -2;
    c.p[j] = client_bufs[j];
    c.w[j] = weights[j];
    vec = vec && aligned16(client_bufs[j]);
  }
  int64_t done = 0;
  if (vec && n >= 4) {
    const int64_t n4 = n / 4;
    // 8 resident 256-lane blocks per CU on 256 CUs, grid-stride beyond that.
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    const dim3 g((unsigned)blocks), b(256);
    switch (num_clients) {
      case 1: hipLaunchKernelGGL(fedavg_sum4_kernel<1>, g, b, 0, st, c, num_clients, n4, out); break;
      case 2: hipLaunchKernelGGL(fedavg_sum4_kernel<2>, g, b, 0, st, c, num_clients, n4, out); break;
      case 3: hipLaunchKernelGGL(fedavg_sum4_kernel<3>, g, b, 0, st, c, num_clients, n4, out); break;
      case 4: hipLaunchKernelGGL(fedavg_sum4_kernel<4>, g, b, 0, st, c, num_clients, n4, out); break;
      case 8: hipLaunchKernelGGL(fedavg_sum4_kernel<8>, g, b, 0, st, c, num_clients, n4, out); break;
      default: hipLaunchKernelGGL(fedavg_sum4_kernel<0>, g, b, 0, st, c, num_clients, n4, out); break;
    }
    SM_CHECK_LAUNCH();
    done = n4 * 4;
  }
  if (done < n) {
    const int64_t rest = n - done;
    hipLaunchKernelGGL(fedavg_sum1_kernel, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, st, c, num_clients,
                       done, n, out);
    SM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sm_fedavg_counters_max(int num_clients, const int64_t* const* client_counters, int64_t n,
                                      int64_t* out, hipStream_t st) {
  if (num_clients < 1 || num_clients > kMaxClients || n < 0) return -2;
  if (n == 0) return 0;
  if (!client_counters || !out) return -2;
  ClientCounters c{};
  for (int j = 0; j < num_clients; ++j) {
    if (!client_counters[j]) return -2;
    c.p[j] = client_counters[j];
  }
  hipLaunchKernelGGL(counters_max_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c, num_clients, n, out);
  SM_CHECK_LAUNCH();
  return 0;
}
