// Fused multi-head attention (flash-style, no score matrix in HBM), forward and
// backward, for the TinyViT encoder (head_dim 32, L = 3136 / 784, reference
// tiny_vit.py:86-106 -> F.scaled_dot_product_attention) and the MAE decoder
// (head_dim 64, L = T*784, torch MultiheadAttention inside
// nn.TransformerEncoderLayer, mae_vit_adapter.py:40-48).
//
// Operands are read straight out of the packed projection output
//   qkv[n][l][3][h][d]      (row stride 3*H*D)        — Linear(C, 3C) output
// and the output is written as O[n][l][h][d] (= [N*L, C]), i.e. exactly the
// `transpose(1,2).reshape(B,L,C)` layout the following projection consumes, so
// no permute copies exist anywhere.  LSE[n][h][l] (natural log, fp32) is kept
// for the backward.  Backward writes dqkv in the same packed layout.
//
// bf16 kernels: 4 waves x 32 query rows, 64-key tiles in LDS.  The score tile is
// computed transposed (S^T = K Q^T on v_mfma_f32_32x32x16_bf16) so each lane owns
// one query column: the online-softmax max/sum are in-register plus one
// cross-half exchange, the per-row rescale is a per-lane multiply, and P^T feeds
// the P.V MFMA directly from the accumulator registers.  V (and in the backward
// Q / dO / K) are read transposed from LDS with ds_read_b64_tr_b16.
//
// f32 kernels (parity mode): one thread per query (fwd, dQ) or key (dK/dV) with
// LDS-staged tiles; exact fp32.
#include <type_traits>

#include "common.h"
#include "sm_api.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float NEG_BIG = -1e30f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

struct AttnArgs {
  const void* qkv;   // [N][L][3][H][D]
  void* out;         // fwd: O [N][L][H][D]; bwd: dqkv [N][L][3][H][D]
  const void* o;     // bwd: O
  const void* dout;  // bwd: dO [N][L][H][D]
  float* lse;        // [N][H][L]
  float* delta;      // [N][H][L]  rowsum(dO * O)
  __bf16* qc;        // bwd (bf16): bf16(Q * scale * log2 e) [N][L][H][D], written by the dQ kernel
  int N, L, H;
  float scale;
  float drop_p;      // dropout on attention probabilities (0 = off)
  uint64_t seed;
};

// ---------- LDS images for a [rows][D] bf16 tile (row = key or query) -------------
// Row reads (ds_read_b128 of 8 consecutive d) and transposed reads
// (ds_read_b64_tr_b16 of 4 consecutive rows) both address through tile_off.
template <int D>
SM_DEV int tile_off(int row, int d) {
  constexpr int CPR = D / 8;              // 16-B chunks per row
  int chunk = d >> 3;
  if (D == 64) chunk ^= (((row >> 1) & 1) << 2) ^ ((row >> 2) & 3);
  else chunk ^= (row >> 2) & 3;
  return row * (D * 2) + (chunk << 4) + ((d & 7) << 1);
  (void)CPR;
}

// The 16x16x32 kernels' image of the same tile: row reads take rows c = l & 15 at chunk
// 4 ks + (l >> 4), transposed reads rows 4 (l >> 4) + (c >> 2) at columns 16 dt + 4 (c & 3),
// which the 32x32x16 swizzle above serves 2-way on both kinds (SQ_LDS_BANK_CONFLICT ~ 1.3x
// the LDS-active cycles of the first 16x16 build, profiles/r06i_attn_sq.txt).  XORing the
// chunk with 2 ((row >> 1) & 3) (D = 64: two rows per 256-B bank row) or 2 ((row >> 2) & 1)
// (D = 32: four) makes every ds_read_b128 lane group and every ds_read_b64_tr_b16 half-wave
// cover the 64 banks once (checked against the guide's lane groups by enumeration).
template <int D>
SM_DEV int tile_off16(int row, int d) {
  int chunk = d >> 3;
  if (D == 64) chunk ^= 2 * ((row >> 1) & 3);
  else chunk ^= ((row >> 2) & 1) << 1;
  return row * (D * 2) + (chunk << 4) + ((d & 7) << 1);
}

// combine a value with the lane 32 apart (the other half-wave) by v_permlane32_swap
// (no LDS round trip): the two results hold {own, other} in either order
SM_DEV float halves_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
SM_DEV float halves_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// 1-D grid over (query/key block, head, sample) with the bijective XCD remap: all
// blocks of one (sample, head) run on the same XCD, so the K/V (or Q/dO) panel they
// all stream is fetched into that XCD's L2 once instead of once per XCD.
struct AttnTile {
  int qb, hd, n;
  SM_DEV AttnTile(int nqb, int H) {
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    qb = v % nqb;
    hd = (v / nqb) % H;
    n = v / (nqb * H);
  }
};

// accumulator (32x32) -> bf16 B-operand fragment for k-step s (four v_cvt_pk_bf16_f32;
// the per-element form let the compiler mix in v_alignbit / v_perm repacks)
SM_DEV uint32_t cvt_pk_bf16(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
SM_DEV bf16x8 acc_to_frag(const f32x16& a, int s) {
  const int o = 8 * s;
  return __builtin_bit_cast(bf16x8, make_uint4(cvt_pk_bf16(a[o], a[o + 1]), cvt_pk_bf16(a[o + 2], a[o + 3]),
                                               cvt_pk_bf16(a[o + 4], a[o + 5]), cvt_pk_bf16(a[o + 6], a[o + 7])));
}
SM_DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---------- attention-probability dropout mask ------------------------------------
// keep(row, col), row = (n*H + hd)*L + q, col = key:
//   h    = mix24(seed32 + row * AG + (col >> 2) * AC)     one hash per 4 keys
//   keep = (byte (col & 3) of h) & 0x7F >= round(128 p)   (p = 0.1: 13/128 dropped)
// common.h's fmix32 input, but mixed with 24-bit multiplies (v_mul_u32_u24, full
// rate) instead of fmix32's 32-bit ones (v_mul_lo_u32, quarter rate): these kernels
// are bound by VALU issue, and the hash was the largest item in it.  Every term
// that varies along a kernel's tile loop is wave-uniform (scalar ALU), so a hash
// costs one vector add plus the 6-op mix.  (Keep rate, row/column balance and
// neighbour correlations measured equal to fmix32's on 4096 x 4096 masks.)
constexpr uint32_t AG = 0x9E3779B1u;   // row multiplier
constexpr uint32_t AC = 0x7FEB352Du;   // column-group multiplier
SM_DEV uint32_t mix24(uint32_t x) {
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * 0xEBCA6Bu;
  x ^= x >> 13;
  x = (x & 0xFFFFFFu) * 0xB2AE35u;
  x ^= x >> 16;
  return x;
}
SM_DEV uint32_t attn_keep_hash(uint32_t s32, uint64_t row, uint32_t col) {
  return mix24(s32 + (uint32_t)row * AG + (col >> 2) * AC);
}
SM_DEV uint32_t attn_thr(float p) { return (uint32_t)(p * 128.f + 0.5f); }
// keep-value scale 128 / (128 - thr): the inverse of the quantised keep rate (E[mask * scale] = 1)
SM_DEV float attn_drop_scale(float p) {
  const uint32_t t = attn_thr(p);
  return t >= 128u ? 0.f : 128.f / (float)(128u - t);
}
SM_DEV bool attn_keep_byte(uint32_t h, int j, uint32_t thr) { return ((h >> (8 * j)) & 0x7Fu) >= thr; }

// Packed form for bf16 P pairs: bit 7 of byte j of keep_flags() is keep(j) (7-bit
// SWAR compare: (b & 0x7F) + 128 - thr never carries out of its byte), and v_perm's
// sign-replicating selectors (8/9: bit 15/31 of the second source, 10/11: of the
// first) expand two flags into a 16-bit-per-element mask in one instruction.
SM_DEV uint32_t keep_flags(uint32_t h, uint32_t thr) { return (h & 0x7F7F7F7Fu) + (128u - thr) * 0x01010101u; }
SM_DEV uint32_t keep_mask01(uint32_t y) { return __builtin_amdgcn_perm(y << 8, y, 0x08080A0Au); }   // bytes 0, 1
SM_DEV uint32_t keep_mask23(uint32_t y) { return __builtin_amdgcn_perm(y << 8, y, 0x09090B0Bu); }   // bytes 2, 3
// Per-element form for fp32 operands: keep_bytes() turns the four flags into bytes
// 0xFF / 0x00 (one v_perm), and keep_sel() ANDs v with its byte sign-extended to 32
// bits, which the compiler's SDWA peephole folds into one v_and_b32_sdwa (operand
// select BYTE_j with sext) -- one instruction per element, where its lowering of
// `keep ? v : 0` is byte extract + compare + select.  (Written in plain C so the
// compiler still inserts the MFMA / transcendental read-after-write wait states an
// inline-asm operand would not get.)
SM_DEV uint32_t keep_bytes(uint32_t y) { return __builtin_amdgcn_perm(y << 8, y, 0x090B080Au); }
SM_DEV float keep_sel(float v, uint32_t kb, int j) {
  const uint32_t m = (uint32_t)(int32_t)(int8_t)(kb >> (8 * j));
  return __uint_as_float(__float_as_uint(v) & m);
}
SM_DEV uint32_t pack_bf16x2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// Row-per-lane epilogue of a 32x32 accumulator tile (lane l: row l & 31; half-wave h = l >> 5
// holds columns 8g + 4h .. + 3 of 8-column group g): each pair of groups (g, g + 1) leaves as
// ONE 16-B store per lane instead of two 8-B stores (MI355X guide T21: the tail is bound by
// store issue, not bytes).  Two v_permlane32_swap per pair hand the lower half-wave the upper
// half's columns of group g and the upper half the lower half's of group g + 1: the lower
// lanes then hold columns 8g .. 8g + 7, the upper lanes 8g + 8 .. 8g + 15.  Every lane must
// execute it (EXEC full: the swap reads the partner lane); the caller predicates the store.
// va / vb: this lane's 4 values of groups g / g + 1; returns the 16 B for column 8 (g + h).
SM_DEV uint4 wide_pair(const float (&va)[4], const float (&vb)[4]) {
  const uint32_t a0 = pack_bf16x2(va[0], va[1]), a1 = pack_bf16x2(va[2], va[3]);
  const uint32_t b0 = pack_bf16x2(vb[0], vb[1]), b1 = pack_bf16x2(vb[2], vb[3]);
  const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
  return make_uint4(r0[0], r1[0], r0[1], r1[1]);
}

// dropout keep multiplier for P[n,hd,q,k] (f32 kernels)
SM_DEV float drop_keep_scale(const AttnArgs& a, int n, int hd, int q, int k) {
  const uint64_t row = (uint64_t)(n * a.H + hd) * a.L + q;
  const uint32_t h = attn_keep_hash(seed32(a.seed), row, (uint32_t)k);
  return attn_keep_byte(h, k & 3, attn_thr(a.drop_p)) ? attn_drop_scale(a.drop_p) : 0.0f;
}

// 4x4 byte transpose inside a DPP quad: lane i's byte j <- lane j's byte i.  Stage 1
// swaps 16-bit halves with lane i^2, stage 2 bytes with lane i^1 (v_perm selectors
// per lane from quad_sel()).
SM_DEV void quad_sel(int kq, uint32_t& sel1, uint32_t& sel2) {
  sel1 = (kq & 2) ? 0x03020706u : 0x05040100u;
  sel2 = (kq & 1) ? 0x03070105u : 0x06020400u;
}
SM_DEV uint32_t quad_transpose_bytes(uint32_t v, uint32_t sel1, uint32_t sel2) {
  const uint32_t p = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // lane ^ 2
  v = __builtin_amdgcn_perm(p, v, sel1);
  const uint32_t q = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // lane ^ 1
  return __builtin_amdgcn_perm(q, v, sel2);
}

// Per-thread plan for staging a [ROWS][D] bf16 tile (rows of a [L][ld] matrix) into
// the LDS image: byte offsets and LDS offsets are computed once; each tile is then
// CH 16-byte raw buffer loads issued early into registers (prefetch) and CH 16-byte
// LDS stores after the barrier.  The tile's descriptor (scalar) carries the base
// and num_records = valid rows x row bytes, so rows past L read as zero with no
// per-lane address arithmetic, compare or branch in the tile loop.
template <int D, int ROWS, int NT = 256, bool S16 = false>
struct Stager {
  static constexpr int CH = ROWS * D / 8 / NT;
  static_assert(CH >= 1 && CH * NT * 8 == ROWS * D, "tile must split evenly over the block's threads");
  uint32_t voff[CH];
  int loff[CH], ld;
  SM_DEV void init(int ld_) {
    ld = ld_;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + NT * i;
      const int row = c / (D / 8), d = (c % (D / 8)) * 8;
      voff[i] = (uint32_t)(row * ld + d) * 2u;
      loff[i] = S16 ? tile_off16<D>(row, d) : tile_off<D>(row, d);
    }
  }
  SM_DEV void load(const __bf16* base, int rows_left, uint4 (&r)[CH]) const {
    const int rows = rows_left < ROWS ? rows_left : ROWS;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, rows * ld * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < CH; ++i) r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[i], 0, 0));
  }
  SM_DEV void store(char* lds, const uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(uint4*)(lds + loff[i]) = r[i];
  }
};

// LDS byte offsets of this lane's fragments (u = 0, s = 0; +32 rows per u and +16
// rows per s keep the swizzle bits, so those are immediate offsets).
template <int D>
SM_DEV int row_frag_off(int s) {   // A/B fragment of 8 consecutive d for row (l & 31)
  const int l = threadIdx.x & 63;
  return tile_off<D>(l & 31, 16 * s + 8 * (l >> 5));
}
template <int D>
SM_DEV void tr_frag_off(int t, int& lo, int& hi) {
  const int l = threadIdx.x & 63;
  const int h = l >> 5, g1 = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
  const int col = 32 * t + 16 * g1 + 4 * p;
  lo = tile_off<D>(4 * h + q, col);
  hi = tile_off<D>(4 * h + q + 8, col);
}
SM_DEV bf16x8 lds_b128(const char* lds, int off) { return *(const bf16x8*)(lds + off); }
SM_DEV bf16x8 lds_tr(const char* lds, int lo, int hi) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + lo));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + hi));
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// =============================================================== bf16 forward
// Softmax without a running maximum.  Q is pre-scaled by scale*log2(e) once in registers,
// so the MFMA leaves the exp2 argument itself and the fast pass computes P = exp2(S) with
// no maximum, no subtraction and no rescale of O (softmax is shift-invariant and fp32 /
// bf16 keep their relative precision at any scale: only the exponent range matters).  Per
// score that leaves the exp, the row-sum add and half a bf16 pack (the online-softmax form
// also spent a max, an fma and the rescale bookkeeping: ~45 % of the d = 32 loop's VALU).
// A row whose sum leaves [2^-100, 2^100] or whose O is not finite (scores beyond the
// exponent range: |S| > ~100 in log2 units) makes the block rerun the whole key loop with
// the online (max-tracking) softmax, so results never depend on the fast pass's range.
template <int D, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_bf16(AttnArgs a) {
  constexpr int KT = 64;
  constexpr int RB = 32 * D * 2;   // bytes of 32 tile rows
  __shared__ __attribute__((aligned(16))) char lk[KT * D * 2];
  __shared__ __attribute__((aligned(16))) char lv[KT * D * 2];
  __shared__ int lbad;
  const AttnTile tl((a.L + 127) / 128, a.H);
  const int n = tl.n, hd = tl.hd;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
  const int C = a.H * D;
  const int ldq = 3 * C;
  const __bf16* qkv = (const __bf16*)a.qkv + (int64_t)n * a.L * ldq;
  const __bf16* qb = qkv + hd * D;
  const __bf16* kb = qkv + C + hd * D;
  const __bf16* vb = qkv + 2 * C + hd * D;
  const int q = tl.qb * 128 + w * 32 + (l & 31);
  // a wave whose 32 query rows all lie past L (the last block of a (sample, head) when L
  // is not a multiple of 128: 3.5 of 4 waves at L = 784) only helps stage the tiles
  const bool wact = tl.qb * 128 + w * 32 < a.L;
  if (threadIdx.x == 0) lbad = 0;   // ordered before any write by the first tile's barriers

  const float c = a.scale * LOG2E;
  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (q < a.L) qf[s] = *(const bf16x8*)(qb + (int64_t)q * ldq + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)qf[s][j] * c);
  }
  Stager<D, KT> stg;
  stg.init(ldq);
  int koff[D / 16], vlo[D / 32], vhi[D / 32];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) koff[s] = row_frag_off<D>(s);
#pragma unroll
  for (int t = 0; t < D / 32; ++t) tr_frag_off<D>(t, vlo[t], vhi[t]);

  f32x16 o[D / 32];
  float m = 0.f, lsum = 0.f;
  // hash input minus its wave-uniform column part: row term + this half's group
  const uint32_t dlb = seed32(a.seed) + (uint32_t)((uint64_t)(n * a.H + hd) * a.L + q) * AG + (uint32_t)h * AC;
  const uint32_t dthr = attn_thr(a.drop_p);

  uint4 rk[Stager<D, KT>::CH], rv[Stager<D, KT>::CH];
  // one pass over the keys; SAFE: online softmax with the running maximum m
  auto pass = [&](auto safe) {
    constexpr bool SAFE = decltype(safe)::value;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
    m = SAFE ? NEG_BIG : 0.f;
    lsum = 0.f;
    stg.load(kb, a.L, rk);
    stg.load(vb, a.L, rv);
    // one key tile; the ragged last tile is its own instantiation: the compiler turned the
    // uniform `if (ragged)` key-range masking into per-element selects executed on EVERY
    // tile (~80 VALU per tile of the d=32 kernels)
    auto tile = [&](int k0, auto rag) {
      constexpr bool RAGGED = decltype(rag)::value;
      __syncthreads();
      stg.store(lk, rk);
      stg.store(lv, rv);
      __syncthreads();
      if (k0 + KT < a.L) {                       // prefetch the next tile under this tile's math
        stg.load(kb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rk);
        stg.load(vb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rv);
      }
      if (!wact) return;
      // ragged tile: the second 32-key half has no key below L when <= 32 keys remain (its
      // scores are masked to -inf below either way): no MFMAs for it
      const bool half1 = !RAGGED || k0 + 32 < a.L;
      f32x16 st[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) st[u][r] = 0.f;
        if (u == 1 && !half1) continue;
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
          st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_b128(lk, koff[s] + u * RB), qf[s], st[u], 0, 0, 0);
      }
      if constexpr (RAGGED) {   // keys past L: P = exp2(-huge) = 0
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (k0 + 32 * u + acc_row(r, h) >= a.L) st[u][r] = NEG_BIG;
      }
      float alpha = 1.f, mn = 0.f;
      bool grow = false;
      if constexpr (SAFE) {
        float mt = NEG_BIG;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) mt = fmaxf(mt, st[u][r]);
        mt = halves_max(mt);
        // rescale only when some row's max grew (exact: alpha == 1 otherwise)
        grow = mt > m;
        mn = grow ? mt : m;
        alpha = grow ? __builtin_amdgcn_exp2f(m - mn) : 1.f;
        m = mn;
      }
      float ps = 0.f;
      uint32_t pw[2][4][2];   // bf16 pairs of P (dropout applied): [u][g][keys 4g+0,1 | 4g+2,3]
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float p4[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            p4[j] = __builtin_amdgcn_exp2f(SAFE ? st[u][4 * g + j] - mn : st[u][4 * g + j]);
            ps += p4[j];
          }
          uint32_t w0 = pack_bf16x2(p4[0], p4[1]), w1 = pack_bf16x2(p4[2], p4[3]);
          if (DROP) {   // keys k0+32u+8g+4h+j, j = 0..3, share one hash; masks on the packed pairs
            const uint32_t y = keep_flags(mix24(dlb + (uint32_t)((k0 >> 2) + 8 * u + 2 * g) * AC), dthr);
            w0 &= keep_mask01(y);
            w1 &= keep_mask23(y);
          }
          pw[u][g][0] = w0;
          pw[u][g][1] = w1;
        }
      }
      if constexpr (SAFE) {
        lsum = lsum * alpha + ps;
        if (__any(grow)) {
#pragma unroll
          for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
        }
      } else {
        lsum += ps;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (u == 1 && !half1) continue;   // P = 0 there
          const bf16x8 pf = __builtin_bit_cast(
              bf16x8, make_uint4(pw[u][2 * s][0], pw[u][2 * s][1], pw[u][2 * s + 1][0], pw[u][2 * s + 1][1]));
#pragma unroll
          for (int t = 0; t < D / 32; ++t)
            o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                lds_tr(lv, vlo[t] + u * RB + s * (RB / 2), vhi[t] + u * RB + s * (RB / 2)), pf, o[t], 0, 0, 0);
        }
    };
    int k0 = 0;
    for (; k0 + KT <= a.L; k0 += KT) tile(k0, std::false_type{});
    if (k0 < a.L) tile(k0, std::true_type{});
    lsum = halves_sum(lsum);
  };
  pass(std::false_type{});
  bool bad = !(lsum >= 0x1p-100f && lsum <= 0x1p100f);
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) bad |= !__builtin_isfinite(o[t][r]);
  if (wact && __any(bad && q < a.L) && l == 0) lbad = 1;
  __syncthreads();
  if (lbad) pass(std::true_type{});   // block-uniform: the rerun's barriers are safe
  {
    const float inv = (DROP ? attn_drop_scale(a.drop_p) : 1.f) / lsum;
    __bf16* ob = (__bf16*)a.out + ((int64_t)n * a.L + q) * C + hd * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        float va[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          va[i] = o[t][4 * g + i] * inv;
          vb[i] = o[t][4 * g + 4 + i] * inv;
        }
        const uint4 w16 = wide_pair(va, vb);
        if (q < a.L) *(uint4*)(ob + 32 * t + 8 * g + 8 * h) = w16;
      }
    if (q < a.L && h == 0) a.lse[((int64_t)n * a.H + hd) * a.L + q] = (m + log2f(lsum)) * LN2;
  }
}

// =============================================================== delta = rowsum(dO*O)
template <typename T>
__global__ void attn_delta_kernel(AttnArgs a, int D) {
  // one wave per (n, l) row: H*D values; lanes split over heads
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (row >= (int64_t)a.N * a.L) return;
  const int C = a.H * D;
  const T* o = (const T*)a.o + row * C;
  const T* dout = (const T*)a.dout + row * C;
  const int n = (int)(row / a.L), q = (int)(row % a.L);
  for (int hd = 0; hd < a.H; ++hd) {
    float s = 0.f;
    for (int d = l; d < D; d += 64) s += to_f<T>(o[hd * D + d]) * to_f<T>(dout[hd * D + d]);
    s = wave_sum(s);
    if (l == 0) a.delta[((int64_t)n * a.H + hd) * a.L + q] = s;
  }
}

// =============================================================== bf16 backward dK, dV
// Keys on lanes (32 per wave, 128 per block); Q / dO tiles (64 rows) staged to LDS
// with register prefetch and read both row-wise (S, dP) and transposed (dV, dK).
// Software-pipelined form: per 64-row tile the wave's two 32-row halves u = 0, 1 run
// as  S,dP(0)  S,dP(1) | softmax(0) | dV,dK(0) | softmax(1) | dV,dK(1)  so each
// half's exp / dropout / dS VALU stream has the other half's MFMAs to hide under.
// Row constants folded in: without dropout the dP accumulator starts at -Delta
// (dS = P * acc); with it, log2 of the keep scale is folded into the LSE so the exp yields
// P' = P/(1-p) directly (dV needs no final scale) and Delta is stored as Delta(1-p).
template <int D, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dkdv_bf16(AttnArgs a) {
  constexpr int QT = 64;
  constexpr int RB = 32 * D * 2;
  constexpr int KB = 32 * NW;   // keys per block
  __shared__ __attribute__((aligned(16))) char lq[QT * D * 2];
  __shared__ __attribute__((aligned(16))) char ldo[QT * D * 2];
  __shared__ __attribute__((aligned(16))) float llse[QT];
  __shared__ __attribute__((aligned(16))) float ldel[QT];
  const AttnTile tl((a.L + KB - 1) / KB, a.H);
  const int n = tl.n, hd = tl.hd;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
  const int C = a.H * D;
  const int ldq = 3 * C;
  const __bf16* qkv = (const __bf16*)a.qkv + (int64_t)n * a.L * ldq;
  const __bf16* qb = a.qc + (int64_t)n * a.L * C + hd * D;   // bf16(Q * scale * log2 e), row stride C
  const __bf16* kb = qkv + C + hd * D;
  const __bf16* vb = qkv + 2 * C + hd * D;
  const __bf16* dob = (const __bf16*)a.dout + (int64_t)n * a.L * C + hd * D;
  const float* lse = a.lse + ((int64_t)n * a.H + hd) * a.L;
  const float* del = a.delta + ((int64_t)n * a.H + hd) * a.L;
  const int key = tl.qb * KB + w * 32 + (l & 31);
  const bool wact = tl.qb * KB + w * 32 < a.L;   // else: only stages tiles (see the forward)

  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (key < a.L) {
      kf[s] = *(const bf16x8*)(kb + (int64_t)key * ldq + 16 * s + 8 * h);
      vf[s] = *(const bf16x8*)(vb + (int64_t)key * ldq + 16 * s + 8 * h);
    } else {
      for (int j = 0; j < 8; ++j) { kf[s][j] = (__bf16)0.f; vf[s][j] = (__bf16)0.f; }
    }
  }
  // The Q tiles are the dQ kernel's bf16(Q * scale * log2 e) (a.qc) and the S accumulator
  // starts at -LSE2 of its query row: the MFMA leaves the exp2 argument itself (one VALU op
  // per score fewer than exp2(fma(S, c, -LSE2))), and S is formed from exactly the rounded
  // operand the forward and the dQ kernel use (bf16(Q c) . K), so the rebuilt P rows match
  // the forward's normalisation.  dK = dS^T Q scale = dS^T Qc ln 2.
  Stager<D, QT, 64 * NW> sq, sd;
  sq.init(C);
  sd.init(C);
  int roff[D / 16], tlo[D / 32], thi[D / 32];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) roff[s] = row_frag_off<D>(s);
#pragma unroll
  for (int t = 0; t < D / 32; ++t) tr_frag_off<D>(t, tlo[t], thi[t]);

  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[t][r] = 0.f; dv[t][r] = 0.f; }
  const float lkeep = DROP ? -log2f(attn_drop_scale(a.drop_p)) : 0.f;   // log2 of 1/ks
  const float dkeep = DROP ? (attn_drop_scale(a.drop_p) > 0.f ? 1.f / attn_drop_scale(a.drop_p) : 0.f) : -1.f;   // Delta factor
  const uint32_t dthr = attn_thr(a.drop_p);
  const int kq = l & 3;
  const uint32_t dlb = seed32(a.seed) + ((uint32_t)((uint64_t)(n * a.H + hd) * a.L) + 4 * h + kq) * AG +
                       (uint32_t)(key >> 2) * AC;
  uint32_t sel1, sel2;
  quad_sel(kq, sel1, sel2);

  // S = Q K^T and dP = dO V^T for query rows q0 + 32u .. +31 (keys on lanes)
  auto sdp = [&](int u, f32x16& sa, f32x16& da) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {   // -LSE2 of rows 32u + 8g + 4h + j (stored negated: no VALU)
      const float4 a4 = *(const float4*)&llse[32 * u + 8 * g + 4 * h];
      sa[4 * g] = a4.x; sa[4 * g + 1] = a4.y; sa[4 * g + 2] = a4.z; sa[4 * g + 3] = a4.w;
    }
    if (DROP) {
#pragma unroll
      for (int r = 0; r < 16; ++r) da[r] = 0.f;
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // -Delta of rows 32u + 8g + 4h + j
        const float4 b4 = *(const float4*)&ldel[32 * u + 8 * g + 4 * h];
        da[4 * g] = b4.x; da[4 * g + 1] = b4.y; da[4 * g + 2] = b4.z; da[4 * g + 3] = b4.w;
      }
    }
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_b128(lq, roff[s] + u * RB), kf[s], sa, 0, 0, 0);
      da = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_b128(ldo, roff[s] + u * RB), vf[s], da, 0, 0, 0);
    }
  };
  // P (dropped, x the keep scale) and dS as bf16 B-operand fragments
  auto softmax = [&](int q0, int u, const f32x16& sa, const f32x16& da, bf16x8 (&pf)[2], bf16x8 (&sf)[2]) {
    f32x16 pv, dsv;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint32_t kb4 = 0;
      if (DROP)
        kb4 = keep_bytes(keep_flags(quad_transpose_bytes(mix24(dlb + (uint32_t)(q0 + 32 * u + 8 * g) * AG), sel1, sel2), dthr));
      float del4[4] = {0.f, 0.f, 0.f, 0.f};
      if (DROP) {
        const float4 b4 = *(const float4*)&ldel[32 * u + 8 * g + 4 * h];
        del4[0] = b4.x; del4[1] = b4.y; del4[2] = b4.z; del4[3] = b4.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * g + j;
        const float p = __builtin_amdgcn_exp2f(sa[r]);
        if (DROP) {
          const float pk = keep_sel(p, kb4, j);
          pv[r] = pk;
          dsv[r] = fmaf(pk, da[r], -(p * del4[j]));
        } else {
          pv[r] = p;
          dsv[r] = p * da[r];
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) { pf[s] = acc_to_frag(pv, s); sf[s] = acc_to_frag(dsv, s); }
  };
  auto dvdk = [&](int u, const bf16x8 (&pf)[2], const bf16x8 (&sf)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < D / 32; ++t) {
        const int ob = u * RB + s * (RB / 2);
        dv[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr(ldo, tlo[t] + ob, thi[t] + ob), pf[s], dv[t], 0, 0, 0);
        dk[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr(lq, tlo[t] + ob, thi[t] + ob), sf[s], dk[t], 0, 0, 0);
      }
  };

  uint4 rq[Stager<D, QT, 64 * NW>::CH], rd[Stager<D, QT, 64 * NW>::CH];
  // the tile's row constants (LSE, Delta) are prefetched with its Q / dO rows (wave 0,
  // one row per lane, index clamped: no branch); loading them between the two barriers
  // held every wave of the block for a global-load round trip per tile
  float rlse = 0.f, rdel = 0.f;
  auto rowc_load = [&](int q0) {
    if (threadIdx.x < QT) {
      const int qq = min(q0 + (int)threadIdx.x, a.L - 1);
      rlse = lse[qq];
      rdel = del[qq];
    }
  };
  sq.load(qb, a.L, rq);
  sd.load(dob, a.L, rd);
  rowc_load(0);
  for (int q0 = 0; q0 < a.L; q0 += QT) {
    __syncthreads();
    sq.store(lq, rq);
    sd.store(ldo, rd);
    if (threadIdx.x < QT) {
      const bool ok = q0 + (int)threadIdx.x < a.L;
      llse[threadIdx.x] = ok ? -fmaf(rlse, LOG2E, lkeep) : -1e30f;   // negated; invalid rows -> P = 0
      ldel[threadIdx.x] = ok ? rdel * dkeep : 0.f;
    }
    __syncthreads();
    if (q0 + QT < a.L) {
      sq.load(qb + (int64_t)(q0 + QT) * C, a.L - q0 - QT, rq);
      sd.load(dob + (int64_t)(q0 + QT) * C, a.L - q0 - QT, rd);
      rowc_load(q0 + QT);
    }
    if (!wact) continue;
    f32x16 s0, p0, s1, p1;
    bf16x8 pf0[2], sf0[2], pf1[2], sf1[2];
    sdp(0, s0, p0);
    sdp(1, s1, p1);
    softmax(q0, 0, s0, p0, pf0, sf0);
    dvdk(0, pf0, sf0);
    softmax(q0, 1, s1, p1, pf1, sf1);
    dvdk(1, pf1, sf1);
  }
  {
    __bf16* out = (__bf16*)a.out + ((int64_t)n * a.L + key) * ldq + hd * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        float ka[4], kb2[4], va[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ka[i] = dk[t][4 * g + i] * LN2;
          kb2[i] = dk[t][4 * g + 4 + i] * LN2;
          va[i] = dv[t][4 * g + i];
          vb[i] = dv[t][4 * g + 4 + i];
        }
        const uint4 wk = wide_pair(ka, kb2), wv = wide_pair(va, vb);
        if (key < a.L) {
          *(uint4*)(out + C + 32 * t + 8 * g + 8 * h) = wk;
          *(uint4*)(out + 2 * C + 32 * t + 8 * g + 8 * h) = wv;
        }
      }
  }
}

// =============================================================== bf16 backward dQ
// Queries on lanes; K / V tiles staged with prefetch; dQ^T = K^T dS^T.
template <int D, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dq_bf16(AttnArgs a) {
  constexpr int KT = 64;
  constexpr int RB = 32 * D * 2;
  constexpr int QB = 32 * NW;   // queries per block
  __shared__ __attribute__((aligned(16))) char lk[KT * D * 2];
  __shared__ __attribute__((aligned(16))) char lv[KT * D * 2];
  const AttnTile tl((a.L + QB - 1) / QB, a.H);
  const int n = tl.n, hd = tl.hd;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
  const int C = a.H * D;
  const int ldq = 3 * C;
  const __bf16* qkv = (const __bf16*)a.qkv + (int64_t)n * a.L * ldq;
  const __bf16* qb = qkv + hd * D;
  const __bf16* kb = qkv + C + hd * D;
  const __bf16* vb = qkv + 2 * C + hd * D;
  const __bf16* dob = (const __bf16*)a.dout + (int64_t)n * a.L * C + hd * D;
  const int q = tl.qb * QB + w * 32 + (l & 31);
  const bool qok = q < a.L;
  const bool wact = tl.qb * QB + w * 32 < a.L;   // else: only stages tiles (see the forward)
  const float lse2 = qok ? a.lse[((int64_t)n * a.H + hd) * a.L + q] * LOG2E : 1e30f;

  // This lane's half of dO's and O's row for query q (D/2 values): Delta = rowsum(dO*O)
  // is formed here (the two halves combined by a lane-32 swap) and written for the
  // dK/dV kernel, which runs after this one -- no separate Delta pass over O and dO.
  const __bf16* ob = (const __bf16*)a.o + (int64_t)n * a.L * C + hd * D;
  bf16x8 qf[D / 16], df[D / 16];
  float dpart = 0.f;
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (qok) {
      qf[s] = *(const bf16x8*)(qb + (int64_t)q * ldq + 16 * s + 8 * h);
      df[s] = *(const bf16x8*)(dob + (int64_t)q * C + 16 * s + 8 * h);
      const bf16x8 of = *(const bf16x8*)(ob + (int64_t)q * C + 16 * s + 8 * h);
#pragma unroll
      for (int j = 0; j < 8; ++j) dpart = fmaf((float)df[s][j], (float)of[j], dpart);
    } else {
      for (int j = 0; j < 8; ++j) { qf[s][j] = (__bf16)0.f; df[s][j] = (__bf16)0.f; }
    }
  }
  const float dl = halves_sum(dpart);
  if (qok && h == 0) a.delta[((int64_t)n * a.H + hd) * a.L + q] = dl;
  // Q pre-scaled by scale * log2(e) in registers and S started at -LSE2: the MFMA leaves
  // the exp2 argument (as in the dK/dV kernel); dQ = dS K needs no Q
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)qf[s][j] * (a.scale * LOG2E));
    // the same rounded operand for the dK/dV kernel's S (it runs after this one)
    if (qok) *(bf16x8*)(a.qc + ((int64_t)n * a.L + q) * C + hd * D + 16 * s + 8 * h) = qf[s];
  }
  Stager<D, KT, 64 * NW> stg;
  stg.init(ldq);
  int roff[D / 16], tlo[D / 32], thi[D / 32];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) roff[s] = row_frag_off<D>(s);
#pragma unroll
  for (int t = 0; t < D / 32; ++t) tr_frag_off<D>(t, tlo[t], thi[t]);
  f32x16 dq[D / 32];
#pragma unroll
  for (int t = 0; t < D / 32; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[t][r] = 0.f;
  const float ks = DROP ? attn_drop_scale(a.drop_p) : 1.f;
  const uint32_t dlb = seed32(a.seed) + (uint32_t)((uint64_t)(n * a.H + hd) * a.L + q) * AG + (uint32_t)h * AC;
  const uint32_t dthr = attn_thr(a.drop_p);

  uint4 rk[Stager<D, KT, 64 * NW>::CH], rv[Stager<D, KT, 64 * NW>::CH];
  stg.load(kb, a.L, rk);
  stg.load(vb, a.L, rv);
  // one key tile; the ragged last tile is its own instantiation (see the forward)
  auto tile = [&](int k0, auto rag) {
    constexpr bool RAGGED = decltype(rag)::value;
    __syncthreads();
    stg.store(lk, rk);
    stg.store(lv, rv);
    __syncthreads();
    if (k0 + KT < a.L) {
      stg.load(kb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rk);
      stg.load(vb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rv);
    }
    if (!wact) return;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (RAGGED && u == 1 && k0 + 32 >= a.L) continue;   // no key below L in this half
      f32x16 sacc, dpacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = -lse2; dpacc[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_b128(lk, roff[s] + u * RB), qf[s], sacc, 0, 0, 0);
        dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_b128(lv, roff[s] + u * RB), df[s], dpacc, 0, 0, 0);
      }
      if constexpr (RAGGED) {   // keys past L: P = exp2(-huge) = 0 (last tile only)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (k0 + 32 * u + acc_row(r, h) >= a.L) sacc[r] = NEG_BIG;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint32_t hv = 0;
        if (DROP) hv = keep_bytes(keep_flags(mix24(dlb + (uint32_t)((k0 >> 2) + 8 * u + 2 * g) * AC), dthr));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          const float p = __builtin_amdgcn_exp2f(sacc[r]);
          const float dp = dpacc[r];
          if (DROP) dpacc[r] = p * fmaf(keep_sel(dp, hv, j), ks, -dl);
          else dpacc[r] = p * (dp - dl);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sf = acc_to_frag(dpacc, s);
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          const int ob = u * RB + s * (RB / 2);
          dq[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr(lk, tlo[t] + ob, thi[t] + ob), sf, dq[t], 0, 0, 0);
        }
      }
    }
  };
  int k0 = 0;
  for (; k0 + KT <= a.L; k0 += KT) tile(k0, std::false_type{});
  if (k0 < a.L) tile(k0, std::true_type{});
  {
    __bf16* out = (__bf16*)a.out + ((int64_t)n * a.L + q) * ldq + hd * D;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        float va[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          va[i] = dq[t][4 * g + i] * a.scale;
          vb[i] = dq[t][4 * g + 4 + i] * a.scale;
        }
        const uint4 w16 = wide_pair(va, vb);
        if (qok) *(uint4*)(out + 32 * t + 8 * g + 8 * h) = w16;
      }
  }
}

// =============================================================== bf16 backward on 16x16x32
// The same two kernels (dK/dV with keys on lanes, dQ with queries on lanes) on
// v_mfma_f32_16x16x32_bf16 instead of 32x32x16: equal MFMA cycles per FLOP, equal LDS
// bytes and registers per wave, but the chip holds a higher clock on this shape
// (MI355X_MICROARCH.md 'DVFS give-back' item 7: 1.12-1.15x the FLOP/s of the 32x32x16
// loop on random data), and each product is a quarter of the size, so the softmax / dS
// VALU of one 16x16 score block can start while the others are still in the matrix core.
//
// Fragment maps (lane l, c = l & 15, g = l >> 4): A[row c][k = 8g + j], B[k = 8g + j][col c],
// D[row 4g + i][col c].  A wave owns 32 keys (dK/dV) or 32 queries (dQ) as two 16-column
// groups.  A 16x16 accumulator feeds the next product as its B operand over its ROW index,
// two blocks per 32-deep k-step: element j < 4 is row 4g + j of the first block, j >= 4 row
// 4g + j - 4 of the second (16 rows further); the A operand of that product reads the same
// k order with two ds_read_b64_tr_b16 (rows 4g.. and 16 + 4g..).
template <int D>
SM_DEV int row16_off(int ks) {   // A fragment: 8 consecutive d at k-step ks of row c
  const int l = threadIdx.x & 63;
  return tile_off16<D>(l & 15, 32 * ks + 8 * (l >> 4));
}
template <int D>
SM_DEV int tr16_off(int dt) {    // transposed A fragment (first block): rows 4g + (c>>2), cols 16 dt + 4 (c&3)
  const int l = threadIdx.x & 63, c = l & 15;
  return tile_off16<D>(4 * (l >> 4) + (c >> 2), 16 * dt + 4 * (c & 3));
}
SM_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
SM_DEV bf16x8 pack_frag16(const f32x4& lo, const f32x4& hi) {
  return __builtin_bit_cast(bf16x8, make_uint4(pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]),
                                               pack_bf16x2(hi[0], hi[1]), pack_bf16x2(hi[2], hi[3])));
}
SM_DEV uint2 pack4(float a, float b, float c, float d) { return make_uint2(pack_bf16x2(a, b), pack_bf16x2(c, d)); }

// dK, dV: keys on lanes (key = kbase + 16 kg + c), Q / dO tiles of 64 rows in LDS, per
// 32-row half u: S, dP for the 2 x 2 (query group, key group) blocks, then P / dS packed
// as B fragments per key group and dV^T / dK^T += dO^T P, Qc^T dS over 16-wide d tiles.
// Row constants, dropout (quad byte transpose: the four keys of a hash are the four lanes
// of a DPP quad) and the pipelined order are the 32x32x16 kernel's.
template <int D, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dkdv16_bf16(AttnArgs a) {
  constexpr int QT = 64;
  constexpr int RB = 16 * D * 2;   // bytes of 16 tile rows
  constexpr int KB = 32 * NW;      // keys per block
  constexpr int KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) char lq[QT * D * 2];
  __shared__ __attribute__((aligned(16))) char ldo[QT * D * 2];
  __shared__ __attribute__((aligned(16))) float llse[QT];
  __shared__ __attribute__((aligned(16))) float ldel[QT];
  const AttnTile tl((a.L + KB - 1) / KB, a.H);
  const int n = tl.n, hd = tl.hd;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  const int C = a.H * D;
  const int ldq = 3 * C;
  const __bf16* qkv = (const __bf16*)a.qkv + (int64_t)n * a.L * ldq;
  const __bf16* qb = a.qc + (int64_t)n * a.L * C + hd * D;
  const __bf16* kb = qkv + C + hd * D;
  const __bf16* vb = qkv + 2 * C + hd * D;
  const __bf16* dob = (const __bf16*)a.dout + (int64_t)n * a.L * C + hd * D;
  const float* lse = a.lse + ((int64_t)n * a.H + hd) * a.L;
  const float* del = a.delta + ((int64_t)n * a.H + hd) * a.L;
  const int kbase = tl.qb * KB + w * 32;
  const bool wact = kbase < a.L;

  bf16x8 kf[2][KS], vf[2][KS];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    const int key = kbase + 16 * kg + c;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (key < a.L) {
        kf[kg][ks] = *(const bf16x8*)(kb + (int64_t)key * ldq + 32 * ks + 8 * g);
        vf[kg][ks] = *(const bf16x8*)(vb + (int64_t)key * ldq + 32 * ks + 8 * g);
      } else {
        for (int j = 0; j < 8; ++j) { kf[kg][ks][j] = (__bf16)0.f; vf[kg][ks][j] = (__bf16)0.f; }
      }
    }
  }
  Stager<D, QT, 64 * NW, true> sq, sd;
  sq.init(C);
  sd.init(C);
  int roff[KS], toff[DT];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = row16_off<D>(ks);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) toff[dt] = tr16_off<D>(dt);

  f32x4 dk[2][DT], dv[2][DT];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) { dk[kg][dt][i] = 0.f; dv[kg][dt][i] = 0.f; }
  const float ksc = DROP ? attn_drop_scale(a.drop_p) : 1.f;
  const float lkeep = DROP ? -log2f(ksc) : 0.f;
  const float dkeep = DROP ? (ksc > 0.f ? 1.f / ksc : 0.f) : -1.f;
  const uint32_t dthr = attn_thr(a.drop_p);
  const int kq = l & 3;
  // hash input of row q0 + 32u + 16qg + 4g + kq, key group (kbase + 16kg + c) >> 2 (+ 4 kg, scalar)
  const uint32_t dlb = seed32(a.seed) + ((uint32_t)((uint64_t)(n * a.H + hd) * a.L) + 4 * g + kq) * AG +
                       (uint32_t)((kbase + c) >> 2) * AC;
  uint32_t sel1, sel2;
  quad_sel(kq, sel1, sel2);

  auto sdp = [&](int u, f32x4 (&sa)[2][2], f32x4 (&da)[2][2]) {
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      const float4 a4 = *(const float4*)&llse[32 * u + 16 * qg + 4 * g];   // -LSE2 of rows 4g + i
      float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!DROP) b4 = *(const float4*)&ldel[32 * u + 16 * qg + 4 * g];     // -Delta
#pragma unroll
      for (int kg = 0; kg < 2; ++kg) {
        sa[qg][kg][0] = a4.x; sa[qg][kg][1] = a4.y; sa[qg][kg][2] = a4.z; sa[qg][kg][3] = a4.w;
        da[qg][kg][0] = b4.x; da[qg][kg][1] = b4.y; da[qg][kg][2] = b4.z; da[qg][kg][3] = b4.w;
      }
    }
#pragma unroll
    for (int qg = 0; qg < 2; ++qg)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 aq = lds_b128(lq, roff[ks] + (2 * u + qg) * RB);
        const bf16x8 ad = lds_b128(ldo, roff[ks] + (2 * u + qg) * RB);
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
          sa[qg][kg] = mfma16(aq, kf[kg][ks], sa[qg][kg]);
          da[qg][kg] = mfma16(ad, vf[kg][ks], da[qg][kg]);
        }
      }
  };
  auto softmax = [&](int q0, int u, const f32x4 (&sa)[2][2], const f32x4 (&da)[2][2], bf16x8 (&pf)[2],
                     bf16x8 (&sf)[2]) {
    f32x4 pv[2][2], dsv[2][2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
      float del4[4] = {0.f, 0.f, 0.f, 0.f};
      if (DROP) {
        const float4 b4 = *(const float4*)&ldel[32 * u + 16 * qg + 4 * g];
        del4[0] = b4.x; del4[1] = b4.y; del4[2] = b4.z; del4[3] = b4.w;
      }
#pragma unroll
      for (int kg = 0; kg < 2; ++kg) {
        uint32_t kb4 = 0;
        if (DROP)
          kb4 = keep_bytes(keep_flags(
              quad_transpose_bytes(mix24(dlb + (uint32_t)(q0 + 32 * u + 16 * qg) * AG + (uint32_t)(4 * kg) * AC),
                                   sel1, sel2), dthr));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(sa[qg][kg][i]);
          if (DROP) {
            const float pk = keep_sel(p, kb4, i);
            pv[qg][kg][i] = pk;
            dsv[qg][kg][i] = fmaf(pk, da[qg][kg][i], -(p * del4[i]));
          } else {
            pv[qg][kg][i] = p;
            dsv[qg][kg][i] = p * da[qg][kg][i];
          }
        }
      }
    }
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
      pf[kg] = pack_frag16(pv[0][kg], pv[1][kg]);
      sf[kg] = pack_frag16(dsv[0][kg], dsv[1][kg]);
    }
  };
  auto dvdk = [&](int u, const bf16x8 (&pf)[2], const bf16x8 (&sf)[2]) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int o = toff[dt] + 2 * u * RB;
      const bf16x8 ado = lds_tr(ldo, o, o + RB);
      const bf16x8 aq = lds_tr(lq, o, o + RB);
#pragma unroll
      for (int kg = 0; kg < 2; ++kg) {
        dv[kg][dt] = mfma16(ado, pf[kg], dv[kg][dt]);
        dk[kg][dt] = mfma16(aq, sf[kg], dk[kg][dt]);
      }
    }
  };

  uint4 rq[Stager<D, QT, 64 * NW, true>::CH], rd[Stager<D, QT, 64 * NW, true>::CH];
  float rlse = 0.f, rdel = 0.f;
  auto rowc_load = [&](int q0) {
    if (threadIdx.x < QT) {
      const int qq = min(q0 + (int)threadIdx.x, a.L - 1);
      rlse = lse[qq];
      rdel = del[qq];
    }
  };
  sq.load(qb, a.L, rq);
  sd.load(dob, a.L, rd);
  rowc_load(0);
  for (int q0 = 0; q0 < a.L; q0 += QT) {
    __syncthreads();
    sq.store(lq, rq);
    sd.store(ldo, rd);
    if (threadIdx.x < QT) {
      const bool ok = q0 + (int)threadIdx.x < a.L;
      llse[threadIdx.x] = ok ? -fmaf(rlse, LOG2E, lkeep) : -1e30f;
      ldel[threadIdx.x] = ok ? rdel * dkeep : 0.f;
    }
    __syncthreads();
    if (q0 + QT < a.L) {
      sq.load(qb + (int64_t)(q0 + QT) * C, a.L - q0 - QT, rq);
      sd.load(dob + (int64_t)(q0 + QT) * C, a.L - q0 - QT, rd);
      rowc_load(q0 + QT);
    }
    if (!wact) continue;
    f32x4 s0[2][2], p0[2][2], s1[2][2], p1[2][2];
    bf16x8 pf0[2], sf0[2], pf1[2], sf1[2];
    sdp(0, s0, p0);
    sdp(1, s1, p1);
    softmax(q0, 0, s0, p0, pf0, sf0);
    dvdk(0, pf0, sf0);
    softmax(q0, 1, s1, p1, pf1, sf1);
    dvdk(1, pf1, sf1);
  }
  // lane: dK / dV [key kbase + 16 kg + c][16 dt + 4g + i]: 8-B runs
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    const int key = kbase + 16 * kg + c;
    if (key >= a.L) continue;
    __bf16* out = (__bf16*)a.out + ((int64_t)n * a.L + key) * ldq + hd * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      *(uint2*)(out + C + 16 * dt) = pack4(dk[kg][dt][0] * LN2, dk[kg][dt][1] * LN2, dk[kg][dt][2] * LN2,
                                           dk[kg][dt][3] * LN2);
      *(uint2*)(out + 2 * C + 16 * dt) = pack4(dv[kg][dt][0], dv[kg][dt][1], dv[kg][dt][2], dv[kg][dt][3]);
    }
  }
}

// dQ: queries on lanes (q = qbase + 16 qg + c), K / V tiles of 64 keys in LDS; per 32-key
// half s the 2 x 2 (key group, query group) blocks of S^T, dP^T, then dS^T packed per
// query group and dQ^T += K^T dS^T over 16-wide d tiles.  The prologue forms Delta and
// writes bf16(Q scale log2 e) for the dK/dV kernel, as the 32x32x16 kernel.
template <int D, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dq16_bf16(AttnArgs a) {
  constexpr int KT = 64;
  constexpr int RB = 16 * D * 2;
  constexpr int QB = 32 * NW;
  constexpr int KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) char lk[KT * D * 2];
  __shared__ __attribute__((aligned(16))) char lv[KT * D * 2];
  const AttnTile tl((a.L + QB - 1) / QB, a.H);
  const int n = tl.n, hd = tl.hd;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, c = l & 15, g = l >> 4;
  const int C = a.H * D;
  const int ldq = 3 * C;
  const __bf16* qkv = (const __bf16*)a.qkv + (int64_t)n * a.L * ldq;
  const __bf16* qb = qkv + hd * D;
  const __bf16* kb = qkv + C + hd * D;
  const __bf16* vb = qkv + 2 * C + hd * D;
  const __bf16* dob = (const __bf16*)a.dout + (int64_t)n * a.L * C + hd * D;
  const __bf16* ob = (const __bf16*)a.o + (int64_t)n * a.L * C + hd * D;
  const int qbase = tl.qb * QB + w * 32;
  const bool wact = qbase < a.L;

  bf16x8 qf[2][KS], df[2][KS];
  float lse2[2], dl[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = qbase + 16 * qg + c;
    const bool qok = q < a.L;
    lse2[qg] = qok ? a.lse[((int64_t)n * a.H + hd) * a.L + q] * LOG2E : 1e30f;
    float dpart = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (qok) {
        qf[qg][ks] = *(const bf16x8*)(qb + (int64_t)q * ldq + 32 * ks + 8 * g);
        df[qg][ks] = *(const bf16x8*)(dob + (int64_t)q * C + 32 * ks + 8 * g);
        const bf16x8 of = *(const bf16x8*)(ob + (int64_t)q * C + 32 * ks + 8 * g);
#pragma unroll
        for (int j = 0; j < 8; ++j) dpart = fmaf((float)df[qg][ks][j], (float)of[j], dpart);
      } else {
        for (int j = 0; j < 8; ++j) { qf[qg][ks][j] = (__bf16)0.f; df[qg][ks][j] = (__bf16)0.f; }
      }
    }
    // the row's four d groups live in lanes c, c + 16, c + 32, c + 48
    dpart += __shfl_xor(dpart, 16);
    dpart += __shfl_xor(dpart, 32);
    dl[qg] = dpart;
    if (qok && g == 0) a.delta[((int64_t)n * a.H + hd) * a.L + q] = dpart;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qg][ks][j] = (__bf16)((float)qf[qg][ks][j] * (a.scale * LOG2E));
      if (qok) *(bf16x8*)(a.qc + ((int64_t)n * a.L + q) * C + hd * D + 32 * ks + 8 * g) = qf[qg][ks];
    }
  }
  Stager<D, KT, 64 * NW, true> stg;
  stg.init(ldq);
  int roff[KS], toff[DT];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = row16_off<D>(ks);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) toff[dt] = tr16_off<D>(dt);
  f32x4 dq[2][DT];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) dq[qg][dt][i] = 0.f;
  const float ksc = DROP ? attn_drop_scale(a.drop_p) : 1.f;
  const uint32_t dthr = attn_thr(a.drop_p);
  uint32_t dlb[2];   // hash input of this lane's row, key group (k0 + 32 s + 16 kk + 4 g) >> 2 minus its scalar part
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
    dlb[qg] = seed32(a.seed) + (uint32_t)((uint64_t)(n * a.H + hd) * a.L + qbase + 16 * qg + c) * AG +
              (uint32_t)g * AC;

  uint4 rk[Stager<D, KT, 64 * NW, true>::CH], rv[Stager<D, KT, 64 * NW, true>::CH];
  stg.load(kb, a.L, rk);
  stg.load(vb, a.L, rv);
  auto tile = [&](int k0, auto rag) {
    constexpr bool RAGGED = decltype(rag)::value;
    __syncthreads();
    stg.store(lk, rk);
    stg.store(lv, rv);
    __syncthreads();
    if (k0 + KT < a.L) {
      stg.load(kb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rk);
      stg.load(vb + (int64_t)(k0 + KT) * ldq, a.L - k0 - KT, rv);
    }
    if (!wact) return;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (RAGGED && s == 1 && k0 + 32 >= a.L) continue;   // no key below L in this half
      f32x4 sacc[2][2], dpacc[2][2];   // [key group kk][query group]
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int qg = 0; qg < 2; ++qg)
#pragma unroll
          for (int i = 0; i < 4; ++i) { sacc[kk][qg][i] = -lse2[qg]; dpacc[kk][qg][i] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 ak = lds_b128(lk, roff[ks] + (2 * s + kk) * RB);
          const bf16x8 av = lds_b128(lv, roff[ks] + (2 * s + kk) * RB);
#pragma unroll
          for (int qg = 0; qg < 2; ++qg) {
            sacc[kk][qg] = mfma16(ak, qf[qg][ks], sacc[kk][qg]);
            dpacc[kk][qg] = mfma16(av, df[qg][ks], dpacc[kk][qg]);
          }
        }
      if constexpr (RAGGED) {   // keys past L: P = exp2(-huge) = 0 (last tile only)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int qg = 0; qg < 2; ++qg)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (k0 + 32 * s + 16 * kk + 4 * g + i >= a.L) sacc[kk][qg][i] = NEG_BIG;
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) {
          uint32_t hv = 0;
          if (DROP) hv = keep_bytes(keep_flags(mix24(dlb[qg] + (uint32_t)((k0 >> 2) + 8 * s + 4 * kk) * AC), dthr));
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(sacc[kk][qg][i]);
            const float dp = dpacc[kk][qg][i];
            if (DROP) dpacc[kk][qg][i] = p * fmaf(keep_sel(dp, hv, i), ksc, -dl[qg]);
            else dpacc[kk][qg][i] = p * (dp - dl[qg]);
          }
        }
      bf16x8 sf[2];
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) sf[qg] = pack_frag16(dpacc[0][qg], dpacc[1][qg]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int o = toff[dt] + 2 * s * RB;
        const bf16x8 ak = lds_tr(lk, o, o + RB);
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) dq[qg][dt] = mfma16(ak, sf[qg], dq[qg][dt]);
      }
    }
  };
  int k0 = 0;
  for (; k0 + KT <= a.L; k0 += KT) tile(k0, std::false_type{});
  if (k0 < a.L) tile(k0, std::true_type{});
  // lane: dQ [q][16 dt + 4g + i]: 8-B runs
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = qbase + 16 * qg + c;
    if (q >= a.L) continue;
    __bf16* out = (__bf16*)a.out + ((int64_t)n * a.L + q) * ldq + hd * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *(uint2*)(out + 16 * dt) = pack4(dq[qg][dt][0] * a.scale, dq[qg][dt][1] * a.scale, dq[qg][dt][2] * a.scale,
                                       dq[qg][dt][3] * a.scale);
  }
}

// =============================================================== f32 kernels
template <int D>
__global__ __launch_bounds__(128) void attn_fwd_f32(AttnArgs a) {
  constexpr int KT = 32;
  __shared__ float lk[KT][D], lv[KT][D];
  const int n = blockIdx.z, hd = blockIdx.y;
  const int C = a.H * D;
  const int64_t ldq = 3 * (int64_t)C;
  const float* qkv = (const float*)a.qkv + (int64_t)n * a.L * ldq;
  const int q = blockIdx.x * 128 + threadIdx.x;
  const bool qok = q < a.L;
  float qv[D], o[D];
  for (int d = 0; d < D; ++d) { qv[d] = qok ? qkv[(int64_t)q * ldq + hd * D + d] : 0.f; o[d] = 0.f; }
  float m = NEG_BIG, lsum = 0.f;
  for (int k0 = 0; k0 < a.L; k0 += KT) {
    __syncthreads();
    for (int i = threadIdx.x; i < KT * D; i += 128) {
      const int r = i / D, d = i % D, key = k0 + r;
      lk[r][d] = key < a.L ? qkv[(int64_t)key * ldq + C + hd * D + d] : 0.f;
      lv[r][d] = key < a.L ? qkv[(int64_t)key * ldq + 2 * C + hd * D + d] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < KT && k0 + r < a.L; ++r) {
      float s = 0.f;
      for (int d = 0; d < D; ++d) s += qv[d] * lk[r][d];
      s *= a.scale;
      const float mn = fmaxf(m, s);
      const float al = __expf(m - mn);
      float p = __expf(s - mn);
      lsum = lsum * al + p;
      if (a.drop_p > 0.f) p *= drop_keep_scale(a, n, hd, q, k0 + r);
      for (int d = 0; d < D; ++d) o[d] = o[d] * al + p * lv[r][d];
      m = mn;
    }
  }
  if (qok) {
    float* ob = (float*)a.out + ((int64_t)n * a.L + q) * C + hd * D;
    for (int d = 0; d < D; ++d) ob[d] = o[d] / lsum;
    a.lse[((int64_t)n * a.H + hd) * a.L + q] = m + logf(lsum);
  }
}

template <int D>
__global__ __launch_bounds__(128) void attn_bwd_dq_f32(AttnArgs a) {
  constexpr int KT = 32;
  __shared__ float lk[KT][D], lv[KT][D];
  const int n = blockIdx.z, hd = blockIdx.y;
  const int C = a.H * D;
  const int64_t ldq = 3 * (int64_t)C;
  const float* qkv = (const float*)a.qkv + (int64_t)n * a.L * ldq;
  const float* dob = (const float*)a.dout + (int64_t)n * a.L * C;
  const int q = blockIdx.x * 128 + threadIdx.x;
  const bool qok = q < a.L;
  float qv[D], dov[D], dq[D];
  for (int d = 0; d < D; ++d) {
    qv[d] = qok ? qkv[(int64_t)q * ldq + hd * D + d] : 0.f;
    dov[d] = qok ? dob[(int64_t)q * C + hd * D + d] : 0.f;
    dq[d] = 0.f;
  }
  const float lse = qok ? a.lse[((int64_t)n * a.H + hd) * a.L + q] : 0.f;
  const float dl = qok ? a.delta[((int64_t)n * a.H + hd) * a.L + q] : 0.f;
  for (int k0 = 0; k0 < a.L; k0 += KT) {
    __syncthreads();
    for (int i = threadIdx.x; i < KT * D; i += 128) {
      const int r = i / D, d = i % D, key = k0 + r;
      lk[r][d] = key < a.L ? qkv[(int64_t)key * ldq + C + hd * D + d] : 0.f;
      lv[r][d] = key < a.L ? qkv[(int64_t)key * ldq + 2 * C + hd * D + d] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < KT && k0 + r < a.L; ++r) {
      float s = 0.f, dp = 0.f;
      for (int d = 0; d < D; ++d) { s += qv[d] * lk[r][d]; dp += dov[d] * lv[r][d]; }
      const float p = __expf(s * a.scale - lse);
      if (a.drop_p > 0.f) dp *= drop_keep_scale(a, n, hd, q, k0 + r);
      const float ds = p * (dp - dl);
      for (int d = 0; d < D; ++d) dq[d] += ds * lk[r][d];
    }
  }
  if (qok) {
    float* out = (float*)a.out + ((int64_t)n * a.L + q) * ldq + hd * D;
    for (int d = 0; d < D; ++d) out[d] = dq[d] * a.scale;
  }
}

template <int D>
__global__ __launch_bounds__(128) void attn_bwd_dkdv_f32(AttnArgs a) {
  constexpr int QT = 32;
  __shared__ float lq[QT][D], ldo[QT][D], llse[QT], ldel[QT];
  const int n = blockIdx.z, hd = blockIdx.y;
  const int C = a.H * D;
  const int64_t ldq = 3 * (int64_t)C;
  const float* qkv = (const float*)a.qkv + (int64_t)n * a.L * ldq;
  const float* dob = (const float*)a.dout + (int64_t)n * a.L * C;
  const int key = blockIdx.x * 128 + threadIdx.x;
  const bool kok = key < a.L;
  float kv[D], vv[D], dk[D], dv[D];
  for (int d = 0; d < D; ++d) {
    kv[d] = kok ? qkv[(int64_t)key * ldq + C + hd * D + d] : 0.f;
    vv[d] = kok ? qkv[(int64_t)key * ldq + 2 * C + hd * D + d] : 0.f;
    dk[d] = 0.f; dv[d] = 0.f;
  }
  for (int q0 = 0; q0 < a.L; q0 += QT) {
    __syncthreads();
    for (int i = threadIdx.x; i < QT * D; i += 128) {
      const int r = i / D, d = i % D, qq = q0 + r;
      lq[r][d] = qq < a.L ? qkv[(int64_t)qq * ldq + hd * D + d] : 0.f;
      ldo[r][d] = qq < a.L ? dob[(int64_t)qq * C + hd * D + d] : 0.f;
    }
    if (threadIdx.x < QT) {
      const int qq = q0 + threadIdx.x;
      llse[threadIdx.x] = qq < a.L ? a.lse[((int64_t)n * a.H + hd) * a.L + qq] : 0.f;
      ldel[threadIdx.x] = qq < a.L ? a.delta[((int64_t)n * a.H + hd) * a.L + qq] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < QT && q0 + r < a.L; ++r) {
      float s = 0.f, dp = 0.f;
      for (int d = 0; d < D; ++d) { s += lq[r][d] * kv[d]; dp += ldo[r][d] * vv[d]; }
      const float p = __expf(s * a.scale - llse[r]);
      float pd = p;
      if (a.drop_p > 0.f) {
        const float ks = drop_keep_scale(a, n, hd, q0 + r, key);
        pd = p * ks;
        dp *= ks;
      }
      const float ds = p * (dp - ldel[r]);
      for (int d = 0; d < D; ++d) { dv[d] += pd * ldo[r][d]; dk[d] += ds * lq[r][d]; }
    }
  }
  if (kok) {
    float* out = (float*)a.out + ((int64_t)n * a.L + key) * ldq + hd * D;
    for (int d = 0; d < D; ++d) { out[C + d] = dk[d] * a.scale; out[2 * C + d] = dv[d]; }
  }
}

// dQ first: it forms Delta = rowsum(dO*O) in its prologue for the dK/dV kernel
// dQ first: it forms Delta = rowsum(dO*O) in its prologue and writes bf16(Q scale log2 e)
// for the dK/dV kernel.  (8-wave blocks and a static s_setprio for one wave of each SIMD
// pair measured 1-10 % slower, profiles/r04c_attn_bwd_variants.txt.)
// MFMA shape of the bf16 backward per head dim (sm_attn_tuning: 32 = v_mfma_f32_32x32x16_bf16,
// 16 = v_mfma_f32_16x16x32_bf16); key 0: D = 64 (decoder), key 1: D = 32 (encoder).
int g_attn_bwd_shape[2] = {16, 32};   // measured: profiles/r06cd_attn_bwd16_variants.txt
template <int D, bool DROP>
void launch_attn_bwd(const AttnArgs& a, hipStream_t st) {
  const dim3 g4((unsigned)((a.L + 127) / 128) * (unsigned)(a.H * a.N));
  const int shape = g_attn_bwd_shape[D == 64 ? 0 : 1];
  if (shape == 16) {
    hipLaunchKernelGGL((attn_bwd_dq16_bf16<D, DROP>), g4, dim3(256), 0, st, a);
    hipLaunchKernelGGL((attn_bwd_dkdv16_bf16<D, DROP>), g4, dim3(256), 0, st, a);
    return;
  }
  hipLaunchKernelGGL((attn_bwd_dq_bf16<D, DROP>), g4, dim3(256), 0, st, a);
  hipLaunchKernelGGL((attn_bwd_dkdv_bf16<D, DROP>), g4, dim3(256), 0, st, a);
}

}  // namespace

extern "C" int sm_attn_fwd(int dtype, int N, int L, int H, int D, const void* qkv, void* out,
                           float* lse, float scale, float drop_p, uint64_t seed, hipStream_t st) {
  if (N <= 0 || L <= 0) return 0;
  if (D != 32 && D != 64) return -2;
  AttnArgs a{};
  a.qkv = qkv; a.out = out; a.lse = lse; a.N = N; a.L = L; a.H = H; a.scale = scale;
  a.drop_p = drop_p; a.seed = seed;
  dim3 grid((L + 127) / 128, H, N);
  const dim3 grid1((unsigned)(((L + 127) / 128) * H * N));   // bf16 kernels: 1-D, XCD-remapped
  const bool drop = drop_p > 0.f;
  if (dtype == SM_BF16) {
    if (D == 32) {
      if (drop) hipLaunchKernelGGL((attn_fwd_bf16<32, true>), grid1, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_fwd_bf16<32, false>), grid1, dim3(256), 0, st, a);
    } else {
      if (drop) hipLaunchKernelGGL((attn_fwd_bf16<64, true>), grid1, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((attn_fwd_bf16<64, false>), grid1, dim3(256), 0, st, a);
    }
  } else {
    if (D == 32) hipLaunchKernelGGL(attn_fwd_f32<32>, grid, dim3(128), 0, st, a);
    else hipLaunchKernelGGL(attn_fwd_f32<64>, grid, dim3(128), 0, st, a);
  }
  SM_CHECK_LAUNCH();
  return 0;
}

// workspace of sm_attn_bwd: Delta [N][H][L] fp32, then (bf16) bf16(Q scale log2 e) [N][L][H][D]
static int64_t attn_delta_bytes(int N, int L, int H) { return ((int64_t)N * H * L * 4 + 255) / 256 * 256; }
extern "C" int64_t sm_attn_bwd_workspace_bytes(int dtype, int N, int L, int H, int D) {
  if (N <= 0 || L <= 0) return 0;
  return attn_delta_bytes(N, L, H) + (dtype == SM_BF16 ? (int64_t)N * L * H * D * 2 : 0);
}

extern "C" int sm_attn_bwd(int dtype, int N, int L, int H, int D, const void* qkv, const void* o,
                           const void* dout, const float* lse, float* delta_ws, void* dqkv,
                           float scale, float drop_p, uint64_t seed, hipStream_t st) {
  if (N <= 0 || L <= 0) return 0;
  if (D != 32 && D != 64) return -2;
  if (((uintptr_t)delta_ws) & 255) return -2;
  AttnArgs a{};
  a.qkv = qkv; a.o = o; a.dout = dout; a.lse = (float*)lse; a.delta = delta_ws; a.out = dqkv;
  a.qc = (__bf16*)((char*)delta_ws + attn_delta_bytes(N, L, H));
  a.N = N; a.L = L; a.H = H; a.scale = scale; a.drop_p = drop_p; a.seed = seed;
  dim3 grid((L + 127) / 128, H, N);
  const bool drop = drop_p > 0.f;
  if (dtype == SM_BF16) {
    // dQ first: it forms Delta = rowsum(dO*O) in its prologue for the dK/dV kernel
    if (D == 32) { if (drop) launch_attn_bwd<32, true>(a, st); else launch_attn_bwd<32, false>(a, st); }
    else { if (drop) launch_attn_bwd<64, true>(a, st); else launch_attn_bwd<64, false>(a, st); }
  } else {
    const int dblocks = (int)(((int64_t)N * L + 3) / 4);
    hipLaunchKernelGGL(attn_delta_kernel<float>, dim3(dblocks), dim3(256), 0, st, a, D);
    if (D == 32) {
      hipLaunchKernelGGL(attn_bwd_dkdv_f32<32>, grid, dim3(128), 0, st, a);
      hipLaunchKernelGGL(attn_bwd_dq_f32<32>, grid, dim3(128), 0, st, a);
    } else {
      hipLaunchKernelGGL(attn_bwd_dkdv_f32<64>, grid, dim3(128), 0, st, a);
      hipLaunchKernelGGL(attn_bwd_dq_f32<64>, grid, dim3(128), 0, st, a);
    }
  }
  SM_CHECK_LAUNCH();
  return 0;
}

// A/B switch of the bf16 backward's MFMA shape (see launch_attn_bwd): key 0 = D 64, 1 = D 32;
// *prev <- current shape; set > 0 stores value (16 or 32), set < 0 restores the default.  Host-side only.
extern "C" int sm_attn_tuning(int key, int set, int value, int* prev) {
  if (key < 0 || key > 1) return -2;
  int& v = g_attn_bwd_shape[key];
  if (prev) *prev = v;
  if (set > 0) {
    if (value != 16 && value != 32) return -2;
    v = value;
  } else if (set < 0) {
    v = key == 0 ? 16 : 32;
  }
  return 0;
}
