// Device-memory arena for the training step, installed through PyTorch's
// pluggable-allocator hook (torch.cuda.memory.CUDAPluggableAllocator, see
// ssl_mae_amd/arena.py).
//
// Why: the step's activations are a few hundred tensors of a dozen sizes from
// 20 MB to 20 GB.  The caching allocator maps one exact-size segment per request
// it cannot serve from its pools and never merges neighbouring segments, so at
// B = 256 it holds ~54 GB of slack between 243 GB allocated and 297 GB reserved
// (profiles/r05ik_allocator_policy.txt, r05st): the stage-0 resident policy
// (263 GiB allocated) cannot fit in the 288 GB of HBM.  This arena takes the
// device's free memory minus a reserve (SM_ARENA_RESERVE_MIB, default 6 GiB, left
// to RCCL, code objects and the HIP runtime) in ONE hipMalloc at the first
// request, places each request best-fit (smallest free block that holds it,
// lowest address on ties) and coalesces a released block with its free
// neighbours, so free space never stays split along segment boundaries.
//
// Stream semantics are the caching allocator's for a single stream: a block is
// reused as soon as it is released, which is stream-ordered on the stream it was
// allocated on (the arena's "home" stream: the stream of the first request).
// Requests from any other stream get their own hipMalloc and are returned with
// hipFree (which synchronises the device), so a block released on the home
// stream never reaches another stream while home-stream work on it is queued.
// Unsupported: using a home-stream block on ANOTHER stream and then releasing it while
// that stream's work on it is still queued.  PyTorch's record_stream is a no-op under a
// pluggable allocator, so such a block would be handed out again at once.  The training
// step only shares persistent buffers across streams (the flat gradient buffer the
// side-stream all-reduce reads, ssl_mae_amd/dist.py), never a temporary.
// No graph-capture pools; statistics through sm_arena_stats.
//
// Running out of memory: PyTorch's pluggable-allocator hook cannot raise, so a request
// that neither the heap nor hipMalloc can serve stops the process with the sizes.
// Explicit memory policies are validated before the step instead
// (tiny_vit.check_memory_policy raises a RuntimeError naming both sizes).
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <utility>

namespace {

constexpr size_t kAlign = 512;             // every block starts on a 512-B boundary
constexpr size_t kGranule = size_t(2) << 20;
constexpr int kMaxDevices = 16;

struct Block {
  size_t size;
  bool free;
};

struct Arena {
  bool tried = false;
  bool attached = false;   // sm_arena_attach (host-memory tests): report exhaustion as nullptr
  char* base = nullptr;
  size_t cap = 0;
  bool home_set = false;
  hipStream_t home = nullptr;
  std::map<size_t, Block> blocks;              // offset -> block, address ordered
  std::set<std::pair<size_t, size_t>> free_set;  // (size, offset) of free blocks
  std::unordered_map<void*, size_t> foreign;  // requests served outside the arena
  size_t in_use = 0, peak = 0, n_alloc = 0, n_foreign = 0, n_oom = 0;
};

// Never destroyed: PyTorch can release blocks from its own static destructors, which may run
// after this library's at process exit.
Arena* const g_arena = new Arena[kMaxDevices];
std::mutex& g_mu = *new std::mutex;

size_t env_reserve() {
  const char* s = std::getenv("SM_ARENA_RESERVE_MIB");
  const long long mib = s ? std::atoll(s) : 6144;
  return size_t(mib > 0 ? mib : 0) << 20;
}

void init(Arena& a, int device) {
  a.tried = true;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return;
  if (cur != device && hipSetDevice(device) != hipSuccess) return;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > env_reserve() + kGranule) {
    size_t want = (fr - env_reserve()) / kGranule * kGranule;
    for (int t = 0; t < 8 && want > kGranule; ++t) {   // shrink by 1 GiB if the runtime refuses
      void* p = nullptr;
      if (hipMalloc(&p, want) == hipSuccess) {
        a.base = static_cast<char*>(p);
        a.cap = want;
        a.blocks[0] = Block{want, true};
        a.free_set.insert({want, 0});
        break;
      }
      (void)hipGetLastError();
      want -= size_t(1) << 30;
    }
  }
  if (!a.base)
    std::fprintf(stderr, "[sm_arena] device %d: no arena (free %zu B); requests go to hipMalloc\n", device, fr);
  if (cur != device) (void)hipSetDevice(cur);
}

void* foreign_alloc(Arena& a, size_t size) {
  void* p = nullptr;
  if (hipMalloc(&p, size) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  a.foreign[p] = size;
  a.n_foreign++;
  return p;
}

void* arena_alloc(Arena& a, size_t size) {
  const size_t sz = (size + kAlign - 1) / kAlign * kAlign;
  auto it = a.free_set.lower_bound({sz, 0});
  if (it == a.free_set.end()) return nullptr;
  const size_t bsz = it->first, off = it->second;
  a.free_set.erase(it);
  Block& b = a.blocks[off];
  b.free = false;
  if (bsz > sz) {
    b.size = sz;
    a.blocks[off + sz] = Block{bsz - sz, true};
    a.free_set.insert({bsz - sz, off + sz});
  }
  a.in_use += sz;
  if (a.in_use > a.peak) a.peak = a.in_use;
  return a.base + off;
}

void arena_free(Arena& a, size_t off) {
  auto it = a.blocks.find(off);
  if (it == a.blocks.end() || it->second.free) {
    std::fprintf(stderr, "[sm_arena] release of an unknown block at offset %zu\n", off);
    std::abort();
  }
  a.in_use -= it->second.size;
  it->second.free = true;
  auto nx = std::next(it);
  if (nx != a.blocks.end() && nx->second.free) {      // merge the following block
    a.free_set.erase({nx->second.size, nx->first});
    it->second.size += nx->second.size;
    a.blocks.erase(nx);
  }
  if (it != a.blocks.begin()) {                        // merge into the preceding block
    auto pv = std::prev(it);
    if (pv->second.free) {
      a.free_set.erase({pv->second.size, pv->first});
      pv->second.size += it->second.size;
      a.blocks.erase(it);
      it = pv;
    }
  }
  a.free_set.insert({it->second.size, it->first});
}

}  // namespace

extern "C" {

// torch.cuda.memory.CUDAPluggableAllocator entry points
void* sm_arena_alloc(ssize_t size, int device, hipStream_t stream) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  Arena& a = g_arena[device];
  if (!a.tried) init(a, device);
  a.n_alloc++;
  const size_t n = size > 0 ? size_t(size) : kAlign;
  if (!a.home_set) {
    a.home = stream;
    a.home_set = true;
  }
  if (a.base && stream == a.home) {
    if (void* p = arena_alloc(a, n)) return p;
    if (a.n_oom++ == 0)
      std::fprintf(stderr, "[sm_arena] device %d: %zu B do not fit (in use %zu of %zu B); using hipMalloc\n",
                   device, n, a.in_use, a.cap);
  }
  if (void* p = foreign_alloc(a, n)) return p;
  if (a.attached) return nullptr;
  // PyTorch's pluggable-allocator hook does not check for null: a null block would reach a
  // kernel as a device address.  Stop here with the numbers instead.
  std::fprintf(stderr, "[sm_arena] device %d: out of device memory for %zu B (arena in use %zu of %zu B, %zu B outside)\n",
               device, n, a.in_use, a.cap, [&] { size_t t = 0; for (const auto& kv : a.foreign) t += kv.second; return t; }());
  std::abort();
}

void sm_arena_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)stream;
  if (!ptr || device < 0 || device >= kMaxDevices) return;
  std::lock_guard<std::mutex> lk(g_mu);
  Arena& a = g_arena[device];
  char* p = static_cast<char*>(ptr);
  if (a.base && p >= a.base && p < a.base + a.cap) {
    arena_free(a, size_t(p - a.base));
    return;
  }
  auto f = a.foreign.find(ptr);
  if (f != a.foreign.end()) {
    a.foreign.erase(f);
    (void)hipFree(ptr);
  }
}

// statistics: out[0..7] = capacity, in use, peak in use, requests, requests served
// by hipMalloc, free blocks, largest free block, bytes held outside the arena
void sm_arena_stats(int device, uint64_t* out) {
  if (device < 0 || device >= kMaxDevices) {
    for (int i = 0; i < 8; ++i) out[i] = 0;
    return;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  const Arena& a = g_arena[device];
  size_t fb = 0, largest = 0, foreign = 0;
  for (const auto& kv : a.blocks)
    if (kv.second.free) {
      fb++;
      if (kv.second.size > largest) largest = kv.second.size;
    }
  for (const auto& kv : a.foreign) foreign += kv.second;
  const uint64_t v[8] = {a.cap, a.in_use, a.peak, a.n_alloc, a.n_foreign, fb, largest, foreign};
  for (int i = 0; i < 8; ++i) out[i] = v[i];
}

void sm_arena_reset_peak(int device) {
  if (device < 0 || device >= kMaxDevices) return;
  std::lock_guard<std::mutex> lk(g_mu);
  g_arena[device].peak = g_arena[device].in_use;
}

// Place the arena of an unused device slot over caller-owned memory instead of a
// hipMalloc (the placement/coalescing tests run it over a host buffer; nothing
// dereferences arena memory).  Returns 0, or -1 if the slot is already in use.
int sm_arena_attach(int device, void* base, uint64_t cap) {
  if (device < 0 || device >= kMaxDevices) return -1;
  std::lock_guard<std::mutex> lk(g_mu);
  Arena& a = g_arena[device];
  if (a.tried) return -1;
  a.tried = true;
  a.attached = true;
  a.base = static_cast<char*>(base);
  a.cap = cap / kAlign * kAlign;
  a.blocks[0] = Block{a.cap, true};
  a.free_set.insert({a.cap, 0});
  return 0;
}

}  // extern "C"
