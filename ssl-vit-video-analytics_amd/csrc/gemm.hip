// General GEMM for the MAE step: every nn.Linear / 1x1-conv forward and both of
// its backward products.
//
//   C[M,N] = beta*C + alpha * sum_k A(m,k) B(k,n) (+ bias[n]) (then optional GELU)
//
//   a_layout 0: A stored [M][K] (K contiguous)     1: A stored [K][M] (M contiguous)
//   b_layout 0: B stored [N][K] (nn.Linear weight) 1: B stored [K][N] (N contiguous)
//
// Linear fwd  Y = X W^T      : (a 0, b 0)
// Linear dX   dX = dY W      : (a 0, b 1)
// Linear dW   dW = dY^T X    : (a 1, b 1)   -> split-K over the token axis
//
// bf16 path (gemm_bf16_kernel; gemm_bf16_v2 below is the default, see there):
// 128x128x64 block tile, 4 waves (2x2), each wave 64x64 = 2x2
// v_mfma_f32_32x32x16_bf16 tiles.  K-contiguous operands are staged to an
// XOR-swizzled [row][64] LDS image read with ds_read_b128; M/N-contiguous operands
// are staged as a [k][128] image and read with ds_read_b64_tr_b16 (hardware
// transpose), so no operand ever needs a transposed copy in HBM.  Register-staged
// prefetch of tile k+1 is issued before the MFMAs of tile k (async-STAGE split).
// f32 path (parity mode): 64x64x16 tile on v_mfma_f32_32x32x2_f32 (exact fp32).
#include "common.h"
#include "sm_api.h"
#include <stdlib.h>

namespace {

struct GemmArgs {
  int M, N, K;
  int k_begin, k_chunk;  // split-K: this launch's z covers [k_begin + z*k_chunk, +k_chunk)
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  const float* bias;
  float alpha, beta;
  int epi;          // bit0: exact GELU; bit1: round the branch to bf16 before the residual add;
                    // bit2: GELU backward, C = acc * GELU'(aux) (aux = the saved pre-activation)
  void* aux;        // pre-activation output (same dtype/ld as C) when GELU; input with bit2
  const void* R;    // residual input (dtype/ld of C); null with beta != 0 -> C itself
  float drop_p;     // dropout on the branch (before the residual add / after GELU)
  uint64_t seed;
  const float* row_scale;   // DropPath: branch *= row_scale[row / rows_per_group]
  int64_t rows_per_group;
  float* partial;   // split-K fp32 slabs [z][M][N] (when non-null: raw store, no epilogue)
  float* colsum;    // bf16 v2, M/N-contiguous A only: per-split row sums of A, [z][M]
  // implicit 3x3 / stride-1 / pad-1 convolution operand (conv3x3_* entry points): the
  // operand is the im2col view of a channels-last [F][cH][cW][cC] tensor, k or n =
  // tap * cC + c with tap = ky * 3 + kx, source pixel = pixel + (ky-1, kx-1), or
  // + (1-ky, 1-kx) when cflip (data gradient).  Pixels outside the frame read zero.
  int cH, cW, cC, cflip;
  // weight-gradient B operand formed on load (XformColsB): IMP 5 dropout after the GELU
  float xb_p;
  uint64_t xb_seed;
  // IMP 7 (B) / IMP 6 (A): the SE output act(x) * gate[frame][channel] with act = the
  // BatchNorm + GELU of the stored pre-activation (ChanAffine), xb_hw token rows per frame
  ChanAffine xb_act;
  const float* xb_gate;
  int xb_hw;
  // BatchNorm statistics of the bf16 output (IMP 8, sm_linear_bn_stats): per-wave column sums
  // and sums of squares of the stored values, [m-tile x waves along M][2][N]
  float* stat_part;
  // split-K reduce only: store C transposed, C[col * ldc + row] (a weight gradient computed
  // as dW^T = x^T dy, sm_linear_dw_bias)
  int ctrans;
  // IMP 9 only (sm_linear_dx_gelu): side output of the GELU input aux, aux_out = bf16(GELU(aux)
  // * dropout keep / (1 - p)) = sm_gelu_fwd(aux) -- the fc2 weight gradient's operand
  void* aux_out;
};

template <typename TC>
SM_DEV void epilogue_store(const GemmArgs& g, int64_t row, int col, float acc, int zs) {
  if (g.partial) {
    g.partial[(int64_t)zs * g.M * g.N + row * g.N + col] = acc;
    return;
  }
  float v = g.alpha * acc;
  if (g.bias) v += g.bias[col];
  TC* C = (TC*)g.C;
  const int64_t idx = g.ctrans ? (int64_t)col * g.ldc + row : row * g.ldc + col;
  if (g.epi & 2) v = (float)(__bf16)v;   // autocast: the Linear output is bf16 before the fp32 add
  if (g.epi & 4) v *= gelu_grad(to_f<TC>(((const TC*)g.aux)[idx]));
  if (g.epi & 1) {
    if (g.aux) ((TC*)g.aux)[idx] = from_f<TC>(v);
    v = gelu_f(v);
  }
  if (g.drop_p > 0.f)
    v *= drop_keep(seed32(g.seed), (uint64_t)row, (uint32_t)col, drop_thr(g.drop_p)) ? drop_scale(g.drop_p) : 0.f;
  if (g.row_scale) v *= g.row_scale[row / g.rows_per_group];
  if (g.beta != 0.f) v += g.beta * to_f<TC>(g.R ? ((const TC*)g.R)[idx] : C[idx]);
  C[idx] = from_f<TC>(v);
}

// ============================================================ bf16 MFMA kernel
constexpr int BM = 128, BN = 128, BKT = 64;

// byte offset inside a K-major [rows][64] bf16 tile (128-B rows, 16-B chunks swizzled)
SM_DEV int kmaj_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// byte offset inside an MN-major [64][128] bf16 tile (256-B rows)
SM_DEV int mnmaj_off(int krow, int col) {
  return krow * 256 + ((((col >> 3) ^ ((krow & 3) << 2))) << 4) + ((col & 7) << 1);
}

template <bool KMAJ>
SM_DEV void gload_tile(const __bf16* base, int64_t ld, int rows_total, int row0, int k0, int kend,
                       uint4 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + 256 * i;
    int row, kk;
    if (KMAJ) { row = c >> 3; kk = (c & 7) * 8; }       // [row][k] chunks
    else      { kk = c >> 4; row = (c & 15) * 8; }      // [k][row] chunks
    const int gr = row0 + row, gk = k0 + kk;
    bool ok = KMAJ ? (gr < rows_total && gk < kend) : (gk < kend && gr < rows_total);
    if (ok) {
      const __bf16* p = KMAJ ? base + (int64_t)gr * ld + gk : base + (int64_t)gk * ld + gr;
      r[i] = *(const uint4*)p;
    } else {
      r[i] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KMAJ>
SM_DEV void lstore_tile(char* lds, const uint4 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + 256 * i;
    int off;
    if (KMAJ) off = kmaj_off(c >> 3, c & 7);
    else      off = mnmaj_off(c >> 4, (c & 15) * 8);
    *(uint4*)(lds + off) = r[i];
  }
}

// Fragment for 32 rows (row base rb inside the tile) at k-substep s (16 k values).
template <bool KMAJ>
SM_DEV bf16x8 lread_frag(const char* lds, int rb, int s) {
  const int l = threadIdx.x & 63;
  if (KMAJ) {
    const int row = rb + (l & 31);
    const int chunk = 2 * s + (l >> 5);
    return *(const bf16x8*)(lds + kmaj_off(row, chunk));
  } else {
    const int h = l >> 5, g1 = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
    const int col = rb + 16 * g1 + 4 * p;
    const int k0 = 16 * s + 8 * h + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off(k0, col)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off(k0 + 4, col)));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Row-staged stores (gemm_bf16_v2).  A row run is 8 consecutive columns of one output
// row held by one lane; stored straight from the lanes, a store instruction covers 32
// rows x 32 B (32 partial cache lines).  Staged, each wave writes its runs into a
// 32-row x 128-B LDS image and stores it back as 8 rows x 128 B per instruction (whole
// lines).  Chunk index XOR-swizzled with rs_swz(row) = (row ^ row >> 3) & 7: the run
// writes (8 consecutive rows per 8-lane ds_write_b128 group) hit 8 distinct chunk slots,
// and the per-run reads (16 rows per ds_read_b128 group) and the 8 x 128-B flush reads
// stay conflict-free.  (The earlier (row >> 1) & 7 put rows 2i and 2i + 1 on the same
// banks: a 2-way conflict on every run write, 44 % extra LDS cycles in the stage-0
// expand GEMM, profiles/r04g_gemm_sq_counters.txt.)
SM_DEV int rs_swz(int row) { return (row ^ (row >> 3)) & 7; }
// v + v(lane ^ 8) + v(lane ^ 16) + v(lane ^ 32), summed in that order (= three __shfl_xor
// steps, bit for bit: each step adds one partner, and the two operands of an add commute):
// a DPP row rotate by 8 and two lane swaps instead of three ds_bpermute round trips
SM_DEV float xor8_16_32_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));   // row_ror:8
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// per-lane column sums / sums of squares of one 16-B run of 8 bf16 outputs (masked by `in`),
// as packed pairs (v_pk_add_f32 / v_pk_fma_f32: the per-element add and fma, two per issue)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
SM_DEV void stats_acc8(uint4 v, bool in, float* st1, float* st2) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t u = in ? w[q] : 0u;
    const f32x2_t f = {__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
    f32x2_t a = {st1[2 * q], st1[2 * q + 1]}, b = {st2[2 * q], st2[2 * q + 1]};
    a = a + f;
    b = __builtin_elementwise_fma(f, f, b);
    st1[2 * q] = a.x; st1[2 * q + 1] = a.y;
    st2[2 * q] = b.x; st2[2 * q + 1] = b.y;
  }
}
// the wave's per-lane partials -> totals of its 8 lane groups (lanes l & 7 = one 8-column chunk)
SM_DEV void stats_reduce8(float* st1, float* st2) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    st1[e] = xor8_16_32_sum(st1[e]);
    st2[e] = xor8_16_32_sum(st2[e]);
  }
}
struct RowStage {
  char* base;   // this wave's 2 x 4 KB: [0] C, [1] aux
  SM_DEV void put(int region, int row, int chunk, uint4 v) const {
    *(uint4*)(base + region * 4096 + row * 128 + ((chunk ^ rs_swz(row)) << 4)) = v;
  }
  // rows: tile rows [row0, row0 + 32) of out (ld elements) at column col0; 16-B chunk
  // c holds `cpc` columns; rows >= M or chunk columns >= N are not stored
  // st1 / st2 (bf16 images): this lane's partial column sums / sums of squares of the
  // stored rows of this 32-row image (its chunk l & 7 = 8 columns), for BatchNorm
  // statistics of the output; stats_reduce8 totals them over the lane groups once per tile
  template <typename TC, bool STATS = false>
  SM_DEV void flush(int region, TC* out, int64_t ld, int64_t row0, int col0, int M, int N, int l,
                    float* st1 = nullptr, float* st2 = nullptr, int wcols = 128 / (int)sizeof(TC)) const {
    constexpr int cpc = 16 / sizeof(TC);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int c = l & 7;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (l >> 3) + 8 * q;
      const uint4 v = *(const uint4*)(base + region * 4096 + r * 128 + ((c ^ rs_swz(r)) << 4));
      const int64_t row = row0 + r;
      const int col = col0 + c * cpc;
      const bool ok = row < M && col < N && c * cpc < wcols;   // wcols: the wave's own columns of the image
      // non-temporal: the output streams past L2, where the operand panels the tile's
      // neighbours still read live
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4s;
      if (ok) __builtin_nontemporal_store(u32x4s{v.x, v.y, v.z, v.w}, (u32x4s*)(out + row * ld + col));
      if constexpr (STATS) stats_acc8(v, ok, st1, st2);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};
SM_DEV uint4 pack8(const float* v, __bf16*) {
  bf16x8 a;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)v[i];
  return __builtin_bit_cast(uint4, a);
}

// one 8-column run (row l & 31 of the wave's 32-row slice) into the stage image:
// bf16 -> chunk 4j + 2p + h of a 64-column image; fp32 -> chunks 4p + 2h, +1 of a
// 32-column image (one per j)
template <typename TC>
SM_DEV void stage_put(const RowStage& rs, int region, int j, int p, int h, int l, const float* v) {
  const int row = l & 31;
  if (sizeof(TC) == 2) {
    rs.put(region, row, 4 * j + 2 * p + h, pack8(v, (__bf16*)nullptr));
  } else {
    rs.put(region, row, 4 * p + 2 * h, make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                  __float_as_uint(v[2]), __float_as_uint(v[3])));
    rs.put(region, row, 4 * p + 2 * h + 1, make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]),
                                                      __float_as_uint(v[6]), __float_as_uint(v[7])));
  }
}

// Epilogue of one wave's (32 MI) x (32 NJ) tile from the (swapped-operand) accumulators.  stage:
// non-null -> RowStage stores (VEC, non-split-K path); zs: the split-K slab of this block.
template <typename TC, bool VEC, int MI = 2, int NJ = 2, bool STATS = false, bool AUXS = false>
SM_DEV __attribute__((always_inline)) void gemm_epilogue(const GemmArgs& g, f32x16 (&acc)[MI][NJ], int m0, int n0,
                                                         int wm, int wn, int l, int zs, char* stage = nullptr) {
  // The MFMAs run with swapped operands (D = B_frag x A_frag), so each lane owns
  // one output ROW (token) and registers r hold its columns
  // wn + 32j + (r&3) + 8(r>>2) + 4h: row-per-lane, no LDS round trip.
  const int h = l >> 5;
  const int64_t rbase = m0 + wm + (l & 31);
  if (!VEC) {   // N % 8 or ldc % 8 != 0 (launch-uniform; chosen at launch)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t row = rbase + 32 * i;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int col = n0 + wn + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (col < g.N) epilogue_store<TC>(g, row, col, acc[i][j][r], zs);
        }
    }
    return;
  }
  // Row-run epilogue: one v_permlane32_swap per register pair gives every lane two
  // runs of 8 consecutive columns per (i, j): cols wn + 32j + 16p + 8h + 0..7,
  // values acc[i][j][8p + 0..3] and acc[i][j][8p + 4..7].  All epilogue math is
  // per element on those runs; each run is one 16-B (bf16) / 32-B (fp32) store.
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                     __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
          acc[i][j][8 * p + e] = __uint_as_float(sw[0]);
          acc[i][j][8 * p + 4 + e] = __uint_as_float(sw[1]);
        }
  if (g.partial) {   // split-K: raw fp32 runs into this z's slab
    float* slab = g.partial + (int64_t)zs * g.M * g.N;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t row = rbase + 32 * i;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
          if (col < g.N) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = acc[i][j][8 * p + e];
            store8(slab + row * g.N + col, v);
          }
        }
    }
    return;
  }
  const RowStage rs_{stage};
  float st1[8], st2[8];   // output statistics (g.stat_part, bf16 staged path)
#pragma unroll
  for (int e = 0; e < 8; ++e) st1[e] = st2[e] = 0.f;
  const bool bias_vec = g.bias && ((uintptr_t)g.bias & 15) == 0;
  const bool has_r = g.beta != 0.f;
  const TC* Rsrc = g.R ? (const TC*)g.R : (const TC*)g.C;
  const uint32_t s32 = seed32(g.seed), thr = drop_thr(g.drop_p);
  const float ks = g.drop_p > 0.f ? drop_scale(g.drop_p) : 1.f;
  constexpr int RW = sizeof(TC) * 8 / 16;   // 16-B words per 8-column run
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t row = rbase + 32 * i;
    const bool rok = row < g.M;   // (staged: out-of-range lanes still take part in the flushes)
    if (!rok && !stage) continue;
    const float rs = (g.row_scale && rok) ? g.row_scale[row / g.rows_per_group] : 1.f;
    const uint32_t rb = drop_rowbase(s32, (uint64_t)row);
    if constexpr (AUXS && sizeof(TC) == 2) {
      // GELU backward's pre-activation (aux) for this 32-row x 64-column image, loaded as
      // 8 rows x 128 B per instruction into stage region 1 (whole lines, where a run per
      // lane touches 32 rows x 32 B), then read back per run in the stage_put layout
      if (stage) {
        const int c = l & 7;
        uint4 av[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = (l >> 3) + 8 * q;
          const int64_t rowq = m0 + wm + 32 * i + r;
          const int colq = n0 + wn + 8 * c;
          av[q] = (rowq < g.M && colq < g.N) ? *(const uint4*)((const TC*)g.aux + rowq * g.ldc + colq)
                                              : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = (l >> 3) + 8 * q;
          *(uint4*)(stage + 4096 + r * 128 + ((c ^ rs_swz(r)) << 4)) = av[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      uint4 rr[2][RW];   // the residual runs of this (row, j), in flight before the stores (R may alias C)
      if (has_r) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
          if (col < g.N && rok) {
            const uint4* src = (const uint4*)(Rsrc + row * g.ldc + col);
#pragma unroll
            for (int q = 0; q < RW; ++q) rr[p][q] = src[q];
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
        if (col >= g.N || !rok) continue;
        float b8[8];
        if (bias_vec) {
          const float4 b0 = *(const float4*)(g.bias + col);
          const float4 b1 = *(const float4*)(g.bias + col + 4);
          b8[0] = b0.x; b8[1] = b0.y; b8[2] = b0.z; b8[3] = b0.w; b8[4] = b1.x; b8[5] = b1.y; b8[6] = b1.z; b8[7] = b1.w;
        } else if (g.bias) {   // a flat-buffer parameter view need not be 16-B aligned
#pragma unroll
          for (int e = 0; e < 8; ++e) b8[e] = g.bias[col + e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) b8[e] = 0.f;
        }
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = fmaf(acc[i][j][8 * p + e], g.alpha, b8[e]);
          if (g.epi & 2) v[e] = (float)(__bf16)v[e];
        }
        const int64_t idx = row * g.ldc + col;
        float hg[8];       // AUXS side output: GELU(pre) (x keep / (1 - p) below)
        if (g.epi & 4) {   // GELU backward: the saved pre-activation run of this (row, cols)
          float pre[8];
          if (AUXS && sizeof(TC) == 2 && stage) {
            const int rr_ = l & 31, ch_ = 4 * j + 2 * p + h;
            load8((const __bf16*)(stage + 4096 + rr_ * 128 + ((ch_ ^ rs_swz(rr_)) << 4)), pre);
          } else {
            load8((const TC*)g.aux + idx, pre);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= gelu_grad(pre[e]);
          if (AUXS && g.aux_out) {
#pragma unroll
            for (int e = 0; e < 8; ++e) hg[e] = gelu_f(pre[e]);
          }
        }
        if (g.epi & 1) {
          if (g.aux) {
            if (stage) stage_put<TC>(rs_, 1, j, p, h, l, v);
            else store8((TC*)g.aux + idx, v);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
        }
        if (g.drop_p > 0.f) {
#pragma unroll
          for (int e4 = 0; e4 < 8; e4 += 4) {
            const uint32_t hv = drop_hash(rb, (uint32_t)(col + e4));   // col % 8 == 0
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float m = ((hv >> (8 * e)) & 0xFFu) >= thr ? ks : 0.f;
              v[e4 + e] *= m;
              if (AUXS && g.aux_out) hg[e4 + e] *= m;
            }
          }
        }
        if (AUXS && g.aux_out) {   // over this lane's own pre run in stage region 1 (read above)
          if (stage && sizeof(TC) == 2) stage_put<TC>(rs_, 1, j, p, h, l, hg);
          else store8((TC*)g.aux_out + idx, hg);
        }
        if (g.row_scale) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= rs;
        }
        if (has_r) {
          float r8[8];
          load8((const TC*)&rr[p][0], r8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaf(g.beta, r8[e], v[e]);
        }
        if (stage) stage_put<TC>(rs_, 0, j, p, h, l, v);
        else store8((TC*)g.C + idx, v);
      }
      if (stage && sizeof(TC) == 4) {   // fp32: one 32-column (128-B) image per (i, j)
        const int64_t r0 = m0 + wm + 32 * i;
        const int c0 = n0 + wn + 32 * j;
        if (g.aux && (g.epi & 1)) rs_.flush<TC>(1, (TC*)g.aux, g.ldc, r0, c0, g.M, g.N, l);
        rs_.flush<TC>(0, (TC*)g.C, g.ldc, r0, c0, g.M, g.N, l);
      }
    }
    if (stage && sizeof(TC) == 2) {     // bf16: one 64-column (128-B) image per i
      const int64_t r0 = m0 + wm + 32 * i;
      const int c0 = n0 + wn;
      if (g.aux && (g.epi & 1)) rs_.flush<TC>(1, (TC*)g.aux, g.ldc, r0, c0, g.M, g.N, l, nullptr, nullptr, 32 * NJ);
      if (AUXS && g.aux_out) rs_.flush<TC>(1, (TC*)g.aux_out, g.ldc, r0, c0, g.M, g.N, l);
      if constexpr (STATS) rs_.flush<TC, true>(0, (TC*)g.C, g.ldc, r0, c0, g.M, g.N, l, st1, st2);
      else rs_.flush<TC>(0, (TC*)g.C, g.ldc, r0, c0, g.M, g.N, l, nullptr, nullptr, 32 * NJ);
    }
  }
  if constexpr (STATS) {
    if (stage && sizeof(TC) == 2) stats_reduce8(st1, st2);   // every lane (lane swaps)
  }
  if (STATS && stage && sizeof(TC) == 2 && l < 8 && m0 + wm < g.M) {   // this wave's 64 rows x 64 cols
    const int wrow = (m0 + wm) >> 6;                         // part row = 64-row slab of the output
    const int col = n0 + wn + 8 * l;
    if (col < g.N) {
      float* ps = g.stat_part + (int64_t)wrow * 2 * g.N + col;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ps[e] = st1[e];
        ps[g.N + e] = st2[e];
      }
    }
  }
}

// (Round 4: an LDS-DMA ring form of the v2 kernel -- buffer_load ... lds into a 3- or 6-slot
// ring of 32-K stages, no staging registers or ds_write, one barrier per stage -- gave
// bit-identical outputs 4-40 % slower on every K-major forward and data-gradient shape of
// the step, profiles/r04d_gemm_dma_ab_and_ksweep.txt; removed.)
// One 128x128 output tile per block; 1-D grid over (m-tile, n-tile) with an
// XCD-aware bijective remap: the n-tiles of one m-tile (which share the A panel)
// are dispatched to the same XCD's L2.  (A persistent variant that prefetched the
// next tile's first K-step under the epilogue measured 5-20 % slower: with three
// resident blocks per CU the hardware already overlaps one block's epilogue with
// another's prologue.)
template <bool AK, bool BK, typename TC, bool VEC>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char lds[2 * BM * BKT * 2];
  char* la = lds;
  char* lb = lds + BM * BKT * 2;
  const int ntn = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const __bf16* A = (const __bf16*)g.A;
  const __bf16* B = (const __bf16*)g.B;
  const int kb = g.k_begin + blockIdx.z * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  uint4 ra[4], rb[4];
  if (kb < ke) {
    gload_tile<AK>(A, g.lda, g.M, m0, kb, ke, ra);
    gload_tile<BK>(B, g.ldb, g.N, n0, kb, ke, rb);
  }
  for (int k0 = kb; k0 < ke; k0 += BKT) {
    lstore_tile<AK>(la, ra);
    lstore_tile<BK>(lb, rb);
    __syncthreads();
    if (k0 + BKT < ke) {
      gload_tile<AK>(A, g.lda, g.M, m0, k0 + BKT, ke, ra);
      gload_tile<BK>(B, g.ldb, g.N, n0, k0 + BKT, ke, rb);
    }
#pragma unroll
    for (int s = 0; s < BKT / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lread_frag<AK>(la, wm + 32 * i, s);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = lread_frag<BK>(lb, wn + 32 * j, s);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  gemm_epilogue<TC, VEC>(g, acc, m0, n0, wm, wn, l, blockIdx.z);
}

// ============================================================ bf16 MFMA kernel, v2
// BM x 128 block tile, BK = 64, each wave 64 x 64 (2 x 2 v_mfma_f32_32x32x16_bf16):
// BM = 256 -> 8 waves (4 along M x 2 along N, 512 threads), BM = 128 -> 4 waves.
// Operands are staged with raw buffer loads: each thread's chunk offsets are 32-bit
// voffsets computed once, the K advance moves the wave-uniform base of the buffer
// descriptor, and rows / columns past the matrix or the K tail read as zero through
// an out-of-range voffset.  The main loop therefore carries no per-step address
// arithmetic in VGPRs (the first kernel spent ~10 VALU instructions per MFMA on 64-bit
// pointer updates and zero-fill moves), which frees the registers for 4 waves per
// SIMD at BM = 256.
constexpr uint32_t BUF_OOB = 0x40000000u;   // >= num_records: the load returns 0
constexpr int XA_MAXK = 1536;                // IMP 6: channels of the transformed A operand
constexpr int XB_MAXK = 256;                 // IMP 11 / 12: channels of the BatchNorm-input A operand

// [64][ROWS] MN-major tile (ROWS*2-B rows), 16-B chunks XOR-swizzled by k-row bits 0-1 and 3:
// the transposed fragment reads of both MFMA shapes are bank-conflict free (32x32x16: k-rows
// 8h + 0..3 x 32 columns per half-wave; 16x16x32: k-rows {0..3, 8..11} x 16 columns) and so
// are the 8-lane 16-B stores (simulated: every read / write pattern at ROWS 64 / 128 / 256).
// The key is invariant under the loaders' k-row step (a multiple of 16).
template <int ROWS>
SM_DEV int mnmaj_off_r(int krow, int col) {
  return krow * (ROWS * 2) + (((col >> 3) ^ ((krow & 3) << 2) ^ (((krow >> 3) & 1) << 1)) << 4) + ((col & 7) << 1);
}

template <int ROWS, int NT, bool KMAJ>
struct TileLoader {
  static constexpr int CH = ROWS * 64 * 2 / 16 / NT;   // 16-B chunks per thread per tile
  static constexpr int KSTEP = NT / (ROWS / 8);        // MN-major: k rows between chunks
  static constexpr int LSTEP = KMAJ ? (NT / 8) * 128 : KSTEP * ROWS * 2;
  uint32_t voff[CH];
  int loff0, kk0;
  // lines: rows (K-major) or columns (MN-major) of this panel that exist
  SM_DEV void init(int64_t ld, int lines) {
    const int t = threadIdx.x;
    if (KMAJ) {
      const int row = t >> 3, ch = t & 7;
      kk0 = ch * 8;
      loff0 = kmaj_off(row, ch);   // rows row + (NT/8) i keep the swizzle: + i * LSTEP
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int r = row + (NT / 8) * i;
        voff[i] = r < lines ? (uint32_t)(((int64_t)r * ld + kk0) * 2) : BUF_OOB;
      }
    } else {
      const int kk = t / (ROWS / 8), col = (t % (ROWS / 8)) * 8;
      kk0 = kk;
      loff0 = mnmaj_off_r<ROWS>(kk, col);
#pragma unroll
      for (int i = 0; i < CH; ++i)
        voff[i] = col < lines ? (uint32_t)(((int64_t)(kk + KSTEP * i) * ld + col) * 2) : BUF_OOB;
    }
  }
  SM_DEV void load(__amdgpu_buffer_rsrc_t rs, int kvalid, uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int k = KMAJ ? kk0 : kk0 + KSTEP * i;
      const uint32_t o = k < kvalid ? voff[i] : BUF_OOB;
      r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
  }
  SM_DEV void store(char* lds, const uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(uint4*)(lds + loff0 + i * LSTEP) = r[i];
  }
};

// descriptor over a panel whose K-step k0 starts at element `off` of P
SM_DEV __amdgpu_buffer_rsrc_t panel_rsrc(const __bf16* P, int64_t off) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(P + off), (short)0, (int)BUF_OOB, 0x00020000);
}

template <bool KMAJ, int ROWS>
SM_DEV bf16x8 lread_frag_r(const char* lds, int rb, int s, int l = threadIdx.x & 63) {
  if (KMAJ) {
    return *(const bf16x8*)(lds + kmaj_off(rb + (l & 31), 2 * s + (l >> 5)));
  } else {
    const int h = l >> 5, g1 = (l >> 4) & 1, i = l & 15, q = i >> 2, p = i & 3;
    const int col = rb + 16 * g1 + 4 * p;
    const int k0 = 16 * s + 8 * h + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off_r<ROWS>(k0, col)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off_r<ROWS>(k0 + 4, col)));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// v_mfma_f32_16x16x32_bf16 fragment of the 16-row (or column) block rb, 32-deep K substep s:
// lane l holds row rb + (l & 15), k = 32 s + 8 (l >> 4) + 0..7 (the same map for both operands)
template <bool KMAJ, int ROWS>
SM_DEV bf16x8 lread_frag16(const char* lds, int rb, int s, int l = threadIdx.x & 63) {
  if (KMAJ) {
    return *(const bf16x8*)(lds + kmaj_off(rb + (l & 15), 4 * s + (l >> 4)));
  } else {
    // each 16-lane group reads k-rows 32 s + 8 g + 0..3 (then + 4..7) x 16 columns; the
    // transposing read hands lane i of the group column rb + i of those 4 rows
    const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int col = rb + 4 * p, k0 = 32 * s + 8 * g + q;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off_r<ROWS>(k0, col)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + mnmaj_off_r<ROWS>(k0 + 4, col)));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// A wave's 64 x 64 (or 64 x 32) tile on v_mfma_f32_16x16x32_bf16.  The accumulators keep the
// 32x32x16 storage (f32x16 per 32 x 32 block) so the epilogues are shared: during the K loop
// block (i, j) holds its four 16 x 16 sub-blocks q = 2a + b (a: row half, b: column half) in
// elements 4q .. 4q + 3, each in the 16x16 output map (operands swapped as in the 32x32 loop:
// lane l has tile row 16a + (l & 15), columns 16b + 4 (l >> 4) + 0..3).  acc16_to_32 then
// moves them into the 32x32 map (row l & 31, columns (r & 3) + 8 (r >> 2) + 4 (l >> 5)):
// per column half b and element e, v_permlane16_swap(X, Y) of the a = 0 / a = 1 values gives
// {X0 Y0 X2 Y2} / {X1 Y1 X3 Y3} (16-lane rows), and v_permlane32_swap of those
// {X0 Y0 X1 Y1} = element 8b + e and {X2 Y2 X3 Y3} = element 8b + 4 + e.
// one 16-column B fragment (column block j of the wave tile) against the four A fragments
// (the B fragments are read one at a time: 20 live fragment registers instead of 32)
template <int NJ>
SM_DEV __attribute__((always_inline)) void mma16_col(f32x16 (&acc)[2][NJ], const bf16x8 (&af)[4], bf16x8 bj,
                                                      int j) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = 2 * (i & 1) + (j & 1);
    f32x16& v = acc[i >> 1][j >> 1];
    f32x4 c = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj, af[i], c, 0, 0, 0);
    v[4 * q] = c[0];
    v[4 * q + 1] = c[1];
    v[4 * q + 2] = c[2];
    v[4 * q + 3] = c[3];
  }
}
// issue order of a substep: the A fragments and B fragments 0 and 1, then per column block j
// its four MFMAs with B fragment j + 2 read in front of them (one B fragment in flight behind
// the MFMAs instead of a full wait per block; 24 live fragment registers)
template <bool AK, bool BK, int NB>
SM_DEV __attribute__((always_inline)) void mma16_schedule() {
  constexpr int RA = AK ? 1 : 2, RB = BK ? 1 : 2;   // LDS read instructions per fragment
  __builtin_amdgcn_sched_group_barrier(0x100, 4 * RA + 2 * RB, 0);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (j + 2 < NB) __builtin_amdgcn_sched_group_barrier(0x100, RB, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
}
template <int NJ>
SM_DEV __attribute__((always_inline)) void acc16_to_32(f32x16 (&acc)[2][NJ]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {   // elements {e, 4 + e, 8 + e, 12 + e} in, the same four out
        f32x16& v = acc[i][j];
        const auto x0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[e]), __float_as_uint(v[8 + e]), false, false);
        const auto x1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[4 + e]), __float_as_uint(v[12 + e]), false,
                                                         false);
        const auto y0 = __builtin_amdgcn_permlane32_swap(x0[0], x0[1], false, false);
        const auto y1 = __builtin_amdgcn_permlane32_swap(x1[0], x1[1], false, false);
        v[e] = __uint_as_float(y0[0]);
        v[4 + e] = __uint_as_float(y0[1]);
        v[8 + e] = __uint_as_float(y1[0]);
        v[12 + e] = __uint_as_float(y1[1]);
      }
    }
}

// ------------------------------------------------------------ implicit im2col loaders
// The stem's 3x3 convolution (tiny_vit.py:69, 48 -> 96 channels at 112x112) as a GEMM
// over the never-materialised im2col matrix (the 9x-inflated [pixels][9C] buffer the
// explicit path writes and reads back): each 16-B chunk of a tile is 8 consecutive
// channels of ONE source pixel (C % 8 == 0), so a chunk is still one buffer load, at
// an offset computed per K-step from the chunk's tap and the row pixel's (y, x).
// ConvRowsA: A(m, k) with m = output pixel (forward / data gradient), K-major tile.
template <int ROWS, int NT>
struct ConvRowsA {
  static constexpr int CH = ROWS * 64 * 2 / 16 / NT;
  int yx[CH];            // (y << 16) | x of row m, -1 past M
  uint32_t roff[CH];     // bytes of row m's pixel relative to the block base (m0 - W - 1)
  int loff0, kcur, tap, c;
  SM_DEV void init(const GemmArgs& g, int m0, int kbeg) {
    const int t = threadIdx.x, row = t >> 3, ch = t & 7;
    loff0 = kmaj_off(row, ch);
    const int HW = g.cH * g.cW;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int r = row + (NT / 8) * i;
      const int m = m0 + r;
      if (m < g.M) {
        const int rem = m % HW;
        yx[i] = ((rem / g.cW) << 16) | (rem % g.cW);
      } else {
        yx[i] = -1;
      }
      roff[i] = (uint32_t)((r + g.cW + 1) * g.cC) * 2u;
    }
    kcur = kbeg + ch * 8;
    tap = kcur / g.cC;
    c = kcur - tap * g.cC;
  }
  SM_DEV void load(__amdgpu_buffer_rsrc_t rs, const GemmArgs& g, int kend, uint4 (&r)[CH]) {
    const int ky = (tap * 11) >> 5, kx = tap - 3 * ky;      // tap / 3, tap % 3 for tap < 9
    const int oy = g.cflip ? 1 - ky : ky - 1, ox = g.cflip ? 1 - kx : kx - 1;
    const bool kok = kcur < kend && tap < 9;
    const int delta = ((oy * g.cW + ox) * g.cC + c) * 2;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int y = yx[i] >> 16, x = yx[i] & 0xFFFF;
      const bool ok = kok && yx[i] >= 0 && (unsigned)(y + oy) < (unsigned)g.cH && (unsigned)(x + ox) < (unsigned)g.cW;
      const uint32_t o = ok ? (uint32_t)((int)roff[i] + delta) : BUF_OOB;
      r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
    kcur += BKT;
    c += BKT;
    while (c >= g.cC) {
      c -= g.cC;
      ++tap;
    }
  }
  SM_DEV void store(char* lds, const uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(uint4*)(lds + loff0 + i * (NT / 8) * 128) = r[i];
  }
};

// ConvColsB: B(k, n) with k = pixel (the reduction axis of the weight gradient) and
// n = (tap, c), M/N-major tile: a thread's column chunk (tap, c) is fixed, its rows'
// pixels advance by BKT per K-step (y, x kept incrementally).
template <int ROWS, int NT>
struct ConvColsB {
  static constexpr int CH = ROWS * 64 * 2 / 16 / NT;
  static constexpr int KSTEP = NT / (ROWS / 8);
  int yx[CH];            // (y << 16) | x of pixel k0 + kk0 + KSTEP * i
  int loff0, kk0, oy, ox;
  uint32_t coff;         // bytes of (tap offset + c) relative to the row pixel at the step base
  bool nok;
  SM_DEV void init(const GemmArgs& g, int n0, int kbeg) {
    const int t = threadIdx.x;
    kk0 = t / (ROWS / 8);
    const int col = (t % (ROWS / 8)) * 8;
    loff0 = mnmaj_off_r<ROWS>(kk0, col);
    const int n = n0 + col;
    nok = n < g.N;
    const int tap = n / g.cC, c = n - tap * g.cC;
    const int ky = (tap * 11) >> 5, kx = tap - 3 * ky;
    oy = ky - 1;
    ox = kx - 1;
    coff = (uint32_t)(((oy + 1) * g.cW + (ox + 1)) * g.cC + c) * 2u;
    const int HW = g.cH * g.cW;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int rem = (kbeg + kk0 + KSTEP * i) % HW;
      yx[i] = ((rem / g.cW) << 16) | (rem % g.cW);
    }
  }
  SM_DEV void load(__amdgpu_buffer_rsrc_t rs, const GemmArgs& g, int kvalid, uint4 (&r)[CH]) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int k = kk0 + KSTEP * i;
      int y = yx[i] >> 16, x = yx[i] & 0xFFFF;
      const bool ok = nok && k < kvalid && (unsigned)(y + oy) < (unsigned)g.cH && (unsigned)(x + ox) < (unsigned)g.cW;
      const uint32_t o = ok ? (uint32_t)(k * g.cC * 2) + coff : BUF_OOB;
      r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
      x += BKT;                       // next K-step: BKT pixels further
      while (x >= g.cW) {
        x -= g.cW;
        if (++y == g.cH) y = 0;
      }
      yx[i] = (y << 16) | x;
    }
  }
  SM_DEV void store(char* lds, const uint4 (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) *(uint4*)(lds + loff0 + i * KSTEP * ROWS * 2) = r[i];
  }
};

// Weight-gradient B operand formed on load (IMP 5).  B(k, n) = dropout(GELU(x[k][n]))
// with x the fc1 pre-activation stored [K = token rows][N] (M/N-major) and the fc1
// output's keep mask, formed per 16-B chunk in the staging registers on its way to LDS
// and rounded to bf16 exactly as the gelu kernel stores it, so the fc2 weight gradient
// is bit-identical to recompute-then-GEMM without the recompute pass (read pre, write
// h, read h back).  Rows past K and columns past N read zero.  Pays when the weight
// gradient has one m-tile (nout <= 256: every B chunk activated once); with two the
// activation runs twice per element and the recompute pass is cheaper (kernels.py).
// (A LayerNorm form of this operand -- the qkv / fc1 weight gradients without the LN
// recompute -- measured neutral: its extra registers force 2 waves / SIMD, which costs
// what the recompute pass did.)
// (IMP 7, sm_linear_dw_se: the MBConv projection's weight gradient over the SE output
// h3 = bf16(bf16(GELU(BN2(a2))) * gate[frame][c]), formed per chunk exactly as
// se_apply_kernel stores it -- bit-identical to se_scale + GEMM without the h3 round trip.
// The per-column BN affine stays in registers (a thread's columns are fixed); each
// 64-row K-step lies in one frame (host: xb_hw % 64 == 0, split chunks multiples of 64),
// so the gate is one 8-float run per K-step, prefetched with the operand.  Rows past K
// are zeroed after the transform: GELU(BN(0)) is not 0.)
template <int ROWS, int NT, int IMP>
struct XformColsB {
  static constexpr int CH = ROWS * 64 * 2 / 16 / NT;
  static constexpr int KSTEP = NT / (ROWS / 8);
  uint32_t voff[CH];
  int loff0, kk0, col;
  uint4 raw[CH];
  uint32_t kvalid_mask;
  float gt[IMP == 7 ? 8 : 1];
  Affine8 af;
  SM_DEV void init(const GemmArgs& g, int n0) {
    const int t = threadIdx.x;
    kk0 = t / (ROWS / 8);
    col = (t % (ROWS / 8)) * 8;
    loff0 = mnmaj_off_r<ROWS>(kk0, col);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      voff[i] = n0 + col < g.N ? (uint32_t)(((int64_t)(kk0 + KSTEP * i) * g.ldb + col) * 2) : BUF_OOB;
    if constexpr (IMP == 7) af.init(g.xb_act, n0 + col < g.N ? n0 + col : 0);
  }
  // K-step at k0 (absolute token row); kvalid rows left
  SM_DEV void load(const GemmArgs& g, int n0, int k0, int kvalid) {
    const __bf16* xb = (const __bf16*)g.B + (int64_t)k0 * g.ldb + n0;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, (int)BUF_OOB, 0x00020000);
    kvalid_mask = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const bool ok = kk0 + KSTEP * i < kvalid;
      kvalid_mask |= ok ? 1u << i : 0u;
      raw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? voff[i] : BUF_OOB, 0, 0));
    }
    if constexpr (IMP == 7) {
      const int c = n0 + col < g.N ? n0 + col : 0;
      if (g.xb_gate) load8(g.xb_gate + (int64_t)(k0 / g.xb_hw) * g.N + c, gt);
      else for (int j = 0; j < 8; ++j) gt[j] = 1.f;   // no gate: x = bf16(BN(a)), as bn_apply stores it
    }
  }
  SM_DEV void store(char* lds, const GemmArgs& g, int n0, int k0) const {
    if constexpr (IMP == 7) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        float v[8];
        load8((const __bf16*)&raw[i], v);
        af.apply<__bf16>(v);   // = se_apply_kernel: act rounded to bf16, then * gate
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (kvalid_mask >> i) & 1u ? v[j] * gt[j] : 0.f;
        *(uint4*)(lds + loff0 + i * KSTEP * ROWS * 2) = pack8(v, (__bf16*)nullptr);
      }
    } else {
      const uint32_t thr = drop_thr(g.xb_p);
      const float ks = g.xb_p > 0.f ? drop_scale(g.xb_p) : 1.f;
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        float x[8], v[8];
        load8((const __bf16*)&raw[i], x);
        const uint32_t rb = drop_rowbase(seed32(g.xb_seed), (uint64_t)(k0 + kk0 + KSTEP * i));
#pragma unroll
        for (int e4 = 0; e4 < 8; e4 += 4) {   // = gelu_fwd_kernel / drop_mult8
          const uint32_t h = g.xb_p > 0.f ? drop_hash(rb, (uint32_t)(n0 + col + e4)) : 0xFFFFFFFFu;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e4 + e] = gelu_f(x[e4 + e]) * (g.xb_p > 0.f ? (((h >> (8 * e)) & 0xFFu) >= thr ? ks : 0.f) : 1.f);
        }
        *(uint4*)(lds + loff0 + i * KSTEP * ROWS * 2) = pack8(v, (__bf16*)nullptr);
      }
    }
  }
};

// IMP: 0 plain operands (8: plus the output's BatchNorm statistics in the epilogue,
// sm_linear_bn_stats; 9: the GELU-backward pre-activation staged through LDS by whole
// lines); 1 A is the implicit im2col of a conv (ConvRowsA; 10: plus the output's
// BatchNorm statistics as IMP 8, sm_conv3x3_fwd_bn_stats);
// 2 B is (ConvColsB); 5 / 7 B is formed on load (XformColsB); 6 A (K-major) is the
// SE output formed on load (below).
// (IMP 5: the activation's registers do not fit beside the staging set at 4 waves /
// SIMD -- scratch spills inside the K loop -- so it runs at 2 waves / SIMD.)
// BNV: block columns, 128 (waves 64 wide) or 64 (waves 32 wide: narrow outputs such as the
// stem conv's 48-channel data gradient, where a 128-column tile computed 62.5 % padding).
// MF: MFMA shape of the K loop, 32 (v_mfma_f32_32x32x16_bf16) or 16 (v_mfma_f32_16x16x32_bf16,
// mma16_col; same operand images and epilogue)
template <bool AK, bool BK, typename TC, bool VEC, int BMV, int IMP = 0, int BNV = 128, int MF = 32>
__global__ __launch_bounds__(BMV * 2, (BMV == 256 && IMP != 5 && IMP != 6 && IMP != 7) ? 4 : 2) void gemm_bf16_v2(GemmArgs g) {
  constexpr int NT = BMV * 2, NJ = BNV / 64;
  static_assert(MF == 32 || (MF == 16 && IMP == 0), "16x16x32 K loop: plain operands only");
  static_assert(BNV == 128 || (BNV == 64 && IMP != 8 && IMP != 9 && IMP != 10 && IMP != 11),
                "64-column tiles: no statistics / side-output epilogue");
  constexpr bool XB = IMP == 5 || IMP == 7;
  // A (K-major) formed on load: IMP 6 act(x) * gate (SE output); IMP 11 / 12 a BatchNorm
  // output x = bf16(a sc + sh) from its stored input a (11: plus the IMP 8 statistics)
  constexpr bool XA = IMP == 6 || IMP == 11 || IMP == 12;
  constexpr int LDS_MAIN = (BMV + BNV) * BKT * 2, LDS_EPI = (NT / 64) * 8192;   // operand tiles | row stage
  __shared__ __attribute__((aligned(16))) char lds[LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI];
  char* la = lds;
  char* lb = lds + BMV * BKT * 2;
  // IMP 6: per-channel table of the A transform (BN scale, shift, SE gate of the tile's frame)
  // (IMP 11 / 12: scale and shift of at most XB_MAXK channels -- a small table keeps two
  // 256-row blocks per CU)
  constexpr int XT = IMP == 6 ? XA_MAXK : XB_MAXK;
  __shared__ __attribute__((aligned(16))) float xtab[IMP == 6 ? 3 * XA_MAXK : XA ? 2 * XB_MAXK : 4];
  // 1-D grid over (split zs, tile), split-major, with the bijective XCD remap: the
  // n-tiles of one m-tile (sharing the A panel) and, under split-K, all tiles of one
  // split (sharing its token rows of both operands) are dealt to one XCD's L2.
  const int ntn = (g.N + BNV - 1) / BNV;
  const int ntiles = ntn * ((g.M + BMV - 1) / BMV);
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int zs = idx / ntiles, tile = idx - zs * ntiles;
  const int m0 = (tile / ntn) * BMV, n0 = (tile % ntn) * BNV;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (w >> 1) * 64, wn = (w & 1) * (BNV / 2);
  const __bf16* A = (const __bf16*)g.A;
  const __bf16* B = (const __bf16*)g.B;
  const int kb = g.k_begin + zs * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);
  if constexpr (XA) {   // IMP 6: the tile's rows lie in one frame (host: xb_hw % BMV == 0)
    const int64_t frame = IMP == 6 ? (int64_t)m0 / g.xb_hw : 0;
    for (int c = threadIdx.x; c < g.K; c += NT) {
      const float sc = g.xb_act.rstd[c] * g.xb_act.w[c];   // = Affine8::init
      xtab[c] = sc;
      xtab[XT + c] = bn_shift(g.xb_act.b[c], g.xb_act.mean[c], sc);
      if constexpr (IMP == 6) xtab[2 * XA_MAXK + c] = g.xb_gate[frame * g.K + c];
    }
    __syncthreads();
  }

  TileLoader<BMV, NT, AK> tla;
  TileLoader<BNV, NT, BK> tlb;
  ConvRowsA<BMV, NT> cla;
  ConvColsB<BNV, NT> clb;
  XformColsB<BNV, NT, IMP> xlb;
  if constexpr (IMP == 1 || IMP == 10) cla.init(g, m0, kb);
  else tla.init(g.lda, g.M - m0);
  if constexpr (IMP == 2) clb.init(g, n0, kb);
  else if constexpr (XB) xlb.init(g, n0);
  else tlb.init(g.ldb, g.N - n0);

  // element offset of K-step k0 of each panel
  const int64_t abase = AK ? (int64_t)m0 * g.lda : (int64_t)m0;
  const int64_t bbase = BK ? (int64_t)n0 * g.ldb : (int64_t)n0;
  const int64_t astep = AK ? 1 : g.lda, bstep = BK ? 1 : g.ldb;
  // implicit operands: A's descriptor sits at the block's first row pixel minus the
  // (W + 1)-pixel halo; B's advances with K (its rows are pixels)
  const int64_t cbase = -(int64_t)(g.cW + 1) * g.cC;
  auto load_a = [&](int k0, uint4 (&r)[TileLoader<BMV, NT, AK>::CH]) {
    if constexpr (IMP == 1 || IMP == 10) cla.load(panel_rsrc(A, (int64_t)m0 * g.cC + cbase), g, ke, r);
    else tla.load(panel_rsrc(A, abase + k0 * astep), ke - k0, r);
  };
  auto load_b = [&](int k0, uint4 (&r)[TileLoader<BNV, NT, BK>::CH]) {
    if constexpr (IMP == 2) clb.load(panel_rsrc(B, (int64_t)k0 * g.cC + cbase), g, ke - k0, r);
    else if constexpr (XB) xlb.load(g, n0, k0, ke - k0);
    else tlb.load(panel_rsrc(B, bbase + k0 * bstep), ke - k0, r);
  };

  f32x16 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  uint4 ra[TileLoader<BMV, NT, AK>::CH], rb[TileLoader<BNV, NT, BK>::CH];
  if (kb < ke) {
    load_a(kb, ra);
    load_b(kb, rb);
  }
  // Bias gradient of a weight-gradient GEMM (A = dy^T, M/N-contiguous): the n0 == 0
  // block of each m-tile also sums its A chunks over K (8 rows of M per thread, from
  // the staging registers), so db needs no separate pass over dy.
  const bool csum = !AK && g.colsum != nullptr && n0 == 0;
  float cs8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs8[j] = 0.f;
  for (int k0 = kb; k0 < ke; k0 += BKT) {
    if (csum) {
#pragma unroll
      for (int i = 0; i < TileLoader<BMV, NT, AK>::CH; ++i) {
        const bf16x8 v = __builtin_bit_cast(bf16x8, ra[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) cs8[j] += (float)v[j];
      }
    }
    if constexpr (IMP == 1 || IMP == 10) {
      cla.store(la, ra);
    } else if constexpr (XA) {
      // h3 = bf16(bf16(GELU(a2 sc + sh)) * gate), exactly as se_apply_kernel stores it
      // (no gate: x = bf16(a2 sc + sh), exactly as bn_apply stores it); the thread's 8
      // channels are fixed per K-step (k0 + kk0 ..)
      const int c0 = k0 + tla.kk0;
      if constexpr (IMP == 6) {
        float sc[8], sh[8], gt[8];
        load8(xtab + c0, sc);
        load8(xtab + XA_MAXK + c0, sh);
        load8(xtab + 2 * XA_MAXK + c0, gt);
#pragma unroll
        for (int i = 0; i < TileLoader<BMV, NT, AK>::CH; ++i) {
          float v[8];
          load8((const __bf16*)&ra[i], v);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float t = fmaf(v[j], sc[j], sh[j]);
            v[j] = to_f<__bf16>(from_f<__bf16>(g.xb_act.gelu ? gelu_f(t) : t)) * gt[j];
          }
          ra[i] = pack8(v, (__bf16*)nullptr);
        }
      } else if (c0 < ke) {   // chunks past K stay the zeros the loads returned
        // x = bf16(a sc + sh), as bn_apply stores it; one channel pair at a time (few live
        // registers beside the accumulators: the plain kernel's 4 waves / SIMD)
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const float2 sc2 = *(const float2*)(xtab + c0 + 2 * jp);
          const float2 sh2 = *(const float2*)(xtab + XT + c0 + 2 * jp);
#pragma unroll
          for (int i = 0; i < TileLoader<BMV, NT, AK>::CH; ++i) {
            uint32_t* wv = (uint32_t*)&ra[i];
            const float lo = __uint_as_float(wv[jp] << 16), hi = __uint_as_float(wv[jp] & 0xFFFF0000u);
            typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
            const bf16x2 o = {(__bf16)fmaf(lo, sc2.x, sh2.x), (__bf16)fmaf(hi, sc2.y, sh2.y)};
            wv[jp] = __builtin_bit_cast(uint32_t, o);
          }
        }
      }
      tla.store(la, ra);
    } else {
      tla.store(la, ra);
    }
    if constexpr (IMP == 2) clb.store(lb, rb);
    else if constexpr (XB) xlb.store(lb, g, n0, k0);
    else tlb.store(lb, rb);
    __syncthreads();
    if (k0 + BKT < ke) {
      load_a(k0 + BKT, ra);
      load_b(k0 + BKT, rb);
    }
    if constexpr (MF == 16) {
#pragma unroll
      for (int s = 0; s < BKT / 32; ++s) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = lread_frag16<AK, BMV>(la, wm + 16 * i, s);
#pragma unroll
        for (int j = 0; j < 2 * NJ; ++j) mma16_col<NJ>(acc, af, lread_frag16<BK, BNV>(lb, wn + 16 * j, s), j);
        mma16_schedule<AK, BK, 2 * NJ>();
      }
    } else {
#pragma unroll
      for (int s = 0; s < BKT / 16; ++s) {
        bf16x8 af[2], bfr[NJ];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = lread_frag_r<AK, BMV>(la, wm + 32 * i, s);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = lread_frag_r<BK, BNV>(lb, wn + 32 * j, s);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if constexpr (MF == 16) acc16_to_32<NJ>(acc);
  if (csum) {   // block-uniform: reduce the NT / (BMV / 8) threads that share 8 rows
    constexpr int G = BMV / 8;
    float* red = (float*)lds;
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = cs8[j];
    __syncthreads();
    if ((int)threadIdx.x < BMV) {
      const int c = threadIdx.x, cg = c >> 3, j = c & 7;
      float sum = 0.f;
      for (int q = 0; q < NT / G; ++q) sum += red[(q * G + cg) * 8 + j];
      if (m0 + c < g.M) g.colsum[(int64_t)zs * g.M + m0 + c] = sum;
    }
    __syncthreads();
  }
  gemm_epilogue<TC, VEC, 2, NJ, IMP == 8 || IMP == 10 || IMP == 11, IMP == 9>(g, acc, m0, n0, wm, wn, l, zs,
                                                                           lds + w * 8192);
}

// ============================================================ weight gradient, 384 x 128, one block per CU
// gemm_dw384: the split-K weight gradient (A = dy^T and B = x both M/N-major, fp32 slabs or C)
// on a 384 x 128 tile -- the step's weight-gradient shapes (384 / 1152 / 1536 x 384 / 1536) divide
// it exactly -- with one 8-wave block per CU (96 x 64 per wave: 3 x 2 v_mfma_f32_32x32x16_bf16
// blocks, 5 fragment reads per 6 MFMAs against v2's 4 per 4) and a software pipeline inside the
// block instead of v2's two resident blocks: two LDS stages (2 x 64 KB) and two register
// staging sets, so the operands of K-step k + 2 load while k computes and k + 1 is written to the
// other stage, one barrier per K-step.  The A image is three [64][128] sub-images (the v2 loader
// and swizzle at ROWS = 128).  The per-element K order is v2's: at the same split count the
// slabs are bit-identical to v2's (profiles/r06zjk_dw384_ab.txt); it takes its own split count
// (dw384_splits: whole rounds of one block per CU), which made it 1.6-7.7 % faster than v2 on the
// step's decoder / stage-2 weight gradients.  CSUM: the n0 == 0 blocks also sum their A chunks per
// row (v2's fused bias gradient).
constexpr int DW3_BM = 384, DW3_BN = 128, DW3_SUB = 128;
constexpr int DW3_STAGE = (DW3_BM + DW3_BN) * BKT * 2;   // 64 KB
template <bool CSUM>
__global__ __launch_bounds__(512, 1) void gemm_dw384(GemmArgs g) {
  constexpr int NT = 512;
  __shared__ __attribute__((aligned(16))) char lds[2 * DW3_STAGE];
  const int ntn = (g.N + DW3_BN - 1) / DW3_BN;
  const int ntiles = ntn * ((g.M + DW3_BM - 1) / DW3_BM);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int zs = idx / ntiles, tile = idx - zs * ntiles;
  const int m0 = (tile / ntn) * DW3_BM, n0 = (tile % ntn) * DW3_BN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (w >> 1) * 96, wn = (w & 1) * 64;
  const __bf16* A = (const __bf16*)g.A;
  const __bf16* B = (const __bf16*)g.B;
  const int kb = g.k_begin + zs * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);
  const int nk = ke > kb ? (ke - kb + BKT - 1) / BKT : 0;

  // one loader for the three sub-images (same offsets): the launch requires M % 384 == 0 and
  // N % 128 == 0, so every column of the tile exists; rows past the split's K read zero
  TileLoader<DW3_SUB, NT, false> tla;
  TileLoader<DW3_BN, NT, false> tlb;
  tla.init(g.lda, DW3_SUB);
  tlb.init(g.ldb, DW3_BN);
  typedef uint4 SetA[3][TileLoader<DW3_SUB, NT, false>::CH];
  typedef uint4 SetB[TileLoader<DW3_BN, NT, false>::CH];
  auto load = [&](int k0, SetA& ra, SetB& rb) {
#pragma unroll
    for (int q = 0; q < 3; ++q) tla.load(panel_rsrc(A, (int64_t)k0 * g.lda + m0 + DW3_SUB * q), ke - k0, ra[q]);
    tlb.load(panel_rsrc(B, (int64_t)k0 * g.ldb + n0), ke - k0, rb);
  };
  const bool csum = CSUM && g.colsum != nullptr && n0 == 0;
  float cs[3][8];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[q][j] = 0.f;
  auto store = [&](char* st, const SetA& ra, const SetB& rb) {
    if (csum) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int i = 0; i < TileLoader<DW3_SUB, NT, false>::CH; ++i) {
          const bf16x8 v = __builtin_bit_cast(bf16x8, ra[q][i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) cs[q][j] += (float)v[j];
        }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) tla.store(st + q * (DW3_SUB * BKT * 2), ra[q]);
    tlb.store(st + DW3_BM * BKT * 2, rb);
  };
  f32x16 acc[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto compute = [&](const char* st) {
    const char* lb = st + DW3_BM * BKT * 2;
#pragma unroll
    for (int s = 0; s < BKT / 16; ++s) {
      bf16x8 af[3], bfr[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = wm + 32 * i;   // 32-row blocks never straddle a 128-row sub-image
        af[i] = lread_frag_r<false, DW3_SUB>(st + (r >> 7) * (DW3_SUB * BKT * 2), r & (DW3_SUB - 1), s);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = lread_frag_r<false, DW3_BN>(lb, wn + 32 * j, s);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  char* L0 = lds;
  char* L1 = lds + DW3_STAGE;
  SetA ra0, ra1;
  SetB rb0, rb1;
  if (nk > 0) load(kb, ra0, rb0);
  if (nk > 1) load(kb + BKT, ra1, rb1);
  if (nk > 0) store(L0, ra0, rb0);
  __syncthreads();
  for (int k = 0; k < nk; k += 2) {
    // even half: K-step k from L0; k + 2 loads into set 0; k + 1 (set 1) goes to L1
    if (k + 2 < nk) load(kb + (k + 2) * BKT, ra0, rb0);
    compute(L0);
    if (k + 1 < nk) store(L1, ra1, rb1);
    __syncthreads();
    if (k + 1 >= nk) break;
    // odd half: K-step k + 1 from L1; k + 3 loads into set 1; k + 2 (set 0) goes to L0
    if (k + 3 < nk) load(kb + (k + 3) * BKT, ra1, rb1);
    compute(L1);
    if (k + 2 < nk) store(L0, ra0, rb0);
    __syncthreads();
  }
  if (csum) {   // block-uniform: the 32 threads of each sub-image's 8-row chunk group
    float* red = (float*)lds;   // [512][24]
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[threadIdx.x * 24 + q * 8 + j] = cs[q][j];
    __syncthreads();
    if ((int)threadIdx.x < DW3_BM) {
      const int c = threadIdx.x, q = c >> 7, cc = c & 127, cg = cc >> 3, j = cc & 7;
      float sum = 0.f;
      for (int u = 0; u < NT / 16; ++u) sum += red[(u * 16 + cg) * 24 + q * 8 + j];
      if (m0 + c < g.M) g.colsum[(int64_t)zs * g.M + m0 + c] = sum;
    }
    __syncthreads();
  }
  // split-K slab of this z: raw fp32 runs (gemm_epilogue's partial path; splits > 1 only)
  const int h = l >> 5;
  float* slab = g.partial + (int64_t)zs * g.M * g.N;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int64_t row = m0 + wm + 32 * i + (l & 31);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                           __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
        const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
        if (row < g.M && col < g.N) store8(slab + row * g.N + col, v);
      }
  }
}

// ============================================================ bf16 GEMM, persistent + pipelined
// gemm_bf16_pp: v2's tile (256 x 128 x 64 on 8 waves of 64 x 64, the same operand images,
// fragment reads, MFMA order and elementwise epilogue: outputs bit-identical to v2) in
// persistent blocks that walk their XCD group's tiles.  Between two tiles:
//   1. the epilogue math writes the finished tile into LDS (the dead operand area: each wave
//      its own 2 x 4 KB row images) -- the accumulators are free after this;
//   2. the next tile's first K-step operands are issued;
//   3. the images leave as unconditional 16-B buffer stores (8 rows x 128 B per instruction);
//   4. the next tile's first K-step waits only for its own loads (they are older than the
//      stores: a counted vmcnt), so the stores drain under its MFMAs.
// v2 (one tile per block) serialises per tile: the first operand loads' latency, the K loop,
// the epilogue and the store drain before the block's slots free (t(K) = 0.83 ms + K 3.52 us
// at N = 1152: the fixed part is the output at 4.5 TB/s, profiles/r04d_gemm_dma_ab_and_ksweep.txt).
// The stores are raw buffer stores with out-of-range offsets instead of branches, and the
// tile loop is rotated (epilogue first) with K-step 0 peeled out of the K loop: where paths
// with different counts of younger memory operations merge, the compiler's waits count the
// shortest and would wait for the stores.  bf16 output only (an fp32 tile needs 128 KB).
constexpr int PP_LDS = 8 * 8192;   // operand tiles (48 KB) | 8 waves x two 4 KB row images

// the thread index as a value the compiler cannot hoist out of (or keep across) the tile
// loop: per-thread offsets are recomputed where they are used instead of holding VGPRs
SM_DEV int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
SM_DEV void bstore128(uint4 v, __amdgpu_buffer_rsrc_t rs, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rs, off, 0, 2);   // aux 2: nt
}

// descriptor over rows [0, rows_valid) of a row-major matrix (row_bytes apart) at base
SM_DEV __amdgpu_buffer_rsrc_t rows_rsrc(const void* base, int64_t rows_valid, int64_t row_bytes) {
  int64_t n = rows_valid > 0 ? rows_valid * row_bytes : 0;
  if (n > (int64_t)BUF_OOB) n = BUF_OOB;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)n, 0x00020000);
}

// Epilogue math of one wave's 64 x 64 tile into its two 32-row images (img, img + 4096):
// gemm_epilogue's VEC staged path for a bf16 output without aux / side outputs, with the
// residual and bias reads as raw buffer loads (columns past N read zero).
SM_DEV __attribute__((always_inline)) void pp_stage(const GemmArgs& g, const f32x16 (&acc)[2][2], int m0, int n0,
                                                    int wm, int wn, int l, char* img) {
  const int h = l >> 5;
  const bool has_r = g.beta != 0.f;
  const __bf16* Rsrc = g.R ? (const __bf16*)g.R : (const __bf16*)g.C;
  const uint32_t s32 = seed32(g.seed), thr = drop_thr(g.drop_p);
  const float ks = g.drop_p > 0.f ? drop_scale(g.drop_p) : 1.f;
  const auto brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.bias, (short)0, g.bias ? g.N * 4 : 0, 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const RowStage rs_{img + i * 4096};
    const int r0 = m0 + wm + 32 * i;
    const int row = r0 + (l & 31);
    const float rsc = g.row_scale ? g.row_scale[(row < g.M ? row : g.M - 1) / (int)g.rows_per_group] : 1.f;
    const uint32_t rb = drop_rowbase(s32, (uint64_t)row);
    const auto rrs = rows_rsrc(Rsrc + (int64_t)r0 * g.ldc, (int64_t)g.M - r0, g.ldc * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint4 rr[2];
      if (has_r) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
          rr[p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rrs, col < g.N ? (uint32_t)(((l & 31) * g.ldc + col) * 2) : BUF_OOB, 0, 0));
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
        float b8[8];
        if (g.bias) {
          const uint32_t o = col < g.N ? (uint32_t)col * 4u : BUF_OOB;
          const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(brs, o, 0, 0));
          const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(brs, o + 16, 0, 0));
          b8[0] = b0.x; b8[1] = b0.y; b8[2] = b0.z; b8[3] = b0.w; b8[4] = b1.x; b8[5] = b1.y; b8[6] = b1.z; b8[7] = b1.w;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) b8[e] = 0.f;
        }
        // the run's 8 columns (v_permlane32_swap on copies: the accumulators stay intact)
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                           __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = fmaf(v[e], g.alpha, b8[e]);
          if (g.epi & 2) v[e] = (float)(__bf16)v[e];
        }
        if (g.epi & 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
        }
        if (g.drop_p > 0.f) {
#pragma unroll
          for (int e4 = 0; e4 < 8; e4 += 4) {
            const uint32_t hv = drop_hash(rb, (uint32_t)(col + e4));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e4 + e] *= ((hv >> (8 * e)) & 0xFFu) >= thr ? ks : 0.f;
          }
        }
        if (g.row_scale) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= rsc;
        }
        if (has_r) {
          float r8[8];
          load8((const __bf16*)&rr[p], r8);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaf(g.beta, r8[e], v[e]);
        }
        stage_put<__bf16>(rs_, 0, j, p, h, l, v);
      }
    }
  }
}

// GELU with the pre-activation side output (fc1: y = drop(GELU(pre)), pre = bf16(acc + bias)
// saved for the backward), no residual / row scale: pass 1 stages pre into the images and
// leaves y in the accumulators in run order (acc[i][j][8p + e] = run (i, j, p) element e);
// the images go to g.aux, then pp_stage_runs stages y for C -- the v2 epilogue's values and
// roundings (gemm_epilogue: fma, epi & 2 rounding, GELU, keep mask), so bit-identical.
SM_DEV __attribute__((always_inline)) void pp_stage_gelu_aux(const GemmArgs& g, f32x16 (&acc)[2][2], int m0, int n0,
                                                             int wm, int wn, int l, char* img) {
  const int h = l >> 5;
  const uint32_t s32 = seed32(g.seed), thr = drop_thr(g.drop_p);
  const float ks = g.drop_p > 0.f ? drop_scale(g.drop_p) : 1.f;
  const auto brs = __builtin_amdgcn_make_buffer_rsrc((void*)g.bias, (short)0, g.bias ? g.N * 4 : 0, 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const RowStage rs_{img + i * 4096};
    const int row = m0 + wm + 32 * i + (l & 31);
    const uint32_t rb = drop_rowbase(s32, (uint64_t)row);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
        float b8[8];
        if (g.bias) {
          const uint32_t o = col < g.N ? (uint32_t)col * 4u : BUF_OOB;
          const float4 b0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(brs, o, 0, 0));
          const float4 b1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(brs, o + 16, 0, 0));
          b8[0] = b0.x; b8[1] = b0.y; b8[2] = b0.z; b8[3] = b0.w; b8[4] = b1.x; b8[5] = b1.y; b8[6] = b1.z; b8[7] = b1.w;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) b8[e] = 0.f;
        }
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                           __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = fmaf(v[e], g.alpha, b8[e]);
          if (g.epi & 2) v[e] = (float)(__bf16)v[e];
        }
        stage_put<__bf16>(rs_, 0, j, p, h, l, v);   // pre
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
        if (g.drop_p > 0.f) {
#pragma unroll
          for (int e4 = 0; e4 < 8; e4 += 4) {
            const uint32_t hv = drop_hash(rb, (uint32_t)(col + e4));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e4 + e] *= ((hv >> (8 * e)) & 0xFFu) >= thr ? ks : 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[i][j][8 * p + e] = v[e];
      }
  }
}
// y (run order in acc, pp_stage_gelu_aux) into the images
SM_DEV __attribute__((always_inline)) void pp_stage_runs(const f32x16 (&acc)[2][2], int l, char* img) {
  const int h = l >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const RowStage rs_{img + i * 4096};
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = acc[i][j][8 * p + e];
        stage_put<__bf16>(rs_, 0, j, p, h, l, v);
      }
  }
}

// GELU backward with the activation side output (fc2 data gradient, sm_linear_dx_gelu: v2's IMP 9
// epilogue): each 32-row image first receives the saved pre-activation as whole 128-B lines (8 rows
// per 16-B buffer load, rows / columns past M / N read zero), every lane reads its own four runs
// back, leaves dx = drop(v GELU'(pre)) in the accumulators in run order and writes
// h = bf16(drop(GELU(pre))) over the run it read.  The images then go to g.aux_out, pp_stage_runs
// stages dx for C -- gemm_epilogue's values and roundings (AUXS path), so bit-identical.  No bias /
// residual / row scale (the launch checks).
SM_DEV __attribute__((always_inline)) void pp_stage_gelu_bwd(const GemmArgs& g, f32x16 (&acc)[2][2], int m0, int n0,
                                                             int wm, int wn, int l, char* img) {
  const int h = l >> 5, c = l & 7;
  const uint32_t s32 = seed32(g.seed), thr = drop_thr(g.drop_p);
  const float ks = g.drop_p > 0.f ? drop_scale(g.drop_p) : 1.f;
  const int colq = n0 + wn + 8 * c;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = m0 + wm + 32 * i;
    const auto prs = rows_rsrc((const __bf16*)g.aux + (int64_t)r0 * g.ldc, (int64_t)g.M - r0, g.ldc * 2);
    uint4 av[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (l >> 3) + 8 * q;
      av[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            prs, colq < g.N ? (uint32_t)((r * g.ldc + colq) * 2) : BUF_OOB, 0, 0));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (l >> 3) + 8 * q;
      *(uint4*)(img + i * 4096 + r * 128 + ((c ^ rs_swz(r)) << 4)) = av[q];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the lines other lanes staged
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const RowStage rs_{img + i * 4096};
    const int row = m0 + wm + 32 * i + (l & 31);
    const uint32_t rb = drop_rowbase(s32, (uint64_t)row);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int col = n0 + wn + 32 * j + 16 * p + 8 * h;
        const int rr_ = l & 31, ch_ = 4 * j + 2 * p + h;
        float pre[8];
        load8((const __bf16*)(img + i * 4096 + rr_ * 128 + ((ch_ ^ rs_swz(rr_)) << 4)), pre);
        float v[8], hg[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                           __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = fmaf(v[e], g.alpha, 0.f);
          if (g.epi & 2) v[e] = (float)(__bf16)v[e];
          v[e] *= gelu_grad(pre[e]);
          hg[e] = gelu_f(pre[e]);
        }
        if (g.drop_p > 0.f) {
#pragma unroll
          for (int e4 = 0; e4 < 8; e4 += 4) {
            const uint32_t hv = drop_hash(rb, (uint32_t)(col + e4));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float m = ((hv >> (8 * e)) & 0xFFu) >= thr ? ks : 0.f;
              v[e4 + e] *= m;
              hg[e4 + e] *= m;
            }
          }
        }
        if (g.aux_out) stage_put<__bf16>(rs_, 0, j, p, h, l, hg);   // over this lane's own pre run
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[i][j][8 * p + e] = v[e];
      }
  }
}

// The wave's two images -> C by unconditional buffer stores (RowStage::flush's order and
// statistics); rows past M are dropped by the descriptor, columns past N by the offset.
template <bool STATS>
SM_DEV __attribute__((always_inline)) void pp_flush(const GemmArgs& g, const void* out, int m0, int n0, int wm, int wn,
                                                    int l, const char* img) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's image writes
  const int c = l & 7;
  const int col = n0 + wn + 8 * c;
  const bool cok = col < g.N;
  float st1[8], st2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) st1[e] = st2[e] = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = m0 + wm + 32 * i;
    const int rows_valid = g.M - r0;
    const auto rs = rows_rsrc((const __bf16*)out + (int64_t)r0 * g.ldc, rows_valid, g.ldc * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (l >> 3) + 8 * q;
      const uint4 v = *(const uint4*)(img + i * 4096 + r * 128 + ((c ^ rs_swz(r)) << 4));
      bstore128(v, rs, cok ? (uint32_t)((r * g.ldc + col) * 2) : BUF_OOB);
      if constexpr (STATS) stats_acc8(v, cok && r < rows_valid, st1, st2);   // (RowStage::flush's order)
    }
  }
  if constexpr (STATS) {   // this wave's 64 rows x 64 columns -> part row (m0 + wm) / 64, lanes 0..7
    stats_reduce8(st1, st2);
    const int wrow = (m0 + wm) >> 6;
    const int sc = n0 + wn + 8 * l;
    const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)(g.stat_part + (int64_t)wrow * 2 * g.N), (short)0,
                                                       2 * g.N * 4, 0x00020000);
    const bool ok = l < 8 && m0 + wm < g.M && sc < g.N;
    const uint32_t o = ok ? (uint32_t)sc * 4u : BUF_OOB;
    const uint32_t o2 = ok ? (uint32_t)(g.N + sc) * 4u : BUF_OOB;
    bstore128(make_uint4(__float_as_uint(st1[0]), __float_as_uint(st1[1]), __float_as_uint(st1[2]), __float_as_uint(st1[3])), prs, o);
    bstore128(make_uint4(__float_as_uint(st1[4]), __float_as_uint(st1[5]), __float_as_uint(st1[6]), __float_as_uint(st1[7])), prs, o + 16);
    bstore128(make_uint4(__float_as_uint(st2[0]), __float_as_uint(st2[1]), __float_as_uint(st2[2]), __float_as_uint(st2[3])), prs, o2);
    bstore128(make_uint4(__float_as_uint(st2[4]), __float_as_uint(st2[5]), __float_as_uint(st2[6]), __float_as_uint(st2[7])), prs, o2 + 16);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// K-major A; B K-major (forward, y = x W^T) or M/N-major (data gradient, dX = dy W); bf16
// output; IMP 0 plain / 8 output BatchNorm statistics / 11, 12 BatchNorm-input A operand with /
// without the statistics (v2's IMP 11 / 12 transform in put()) / 13 GELU with the
// pre-activation side output (pp_stage_gelu_aux) / 9 GELU backward with the activation side
// output (pp_stage_gelu_bwd).  No split-K (k_begin = 0, k_chunk >=
// K).  Grid: a multiple of 8 blocks, at most T / 8 per XCD group; block b serves group b & 7
// (its tiles are a contiguous m-major range, so concurrently running blocks share A panels in
// the XCD's L2) and walks tiles b >> 3, + gridDim.x / 8, ... of it.
template <bool BK, int IMP>
__global__ __launch_bounds__(512, 4) void gemm_bf16_pp(GemmArgs g) {
  static_assert(IMP == 0 || IMP == 8 || IMP == 9 || IMP == 11 || IMP == 12 || IMP == 13,
                "persistent form: plain, statistics, GELU backward + activation, BatchNorm-input (+ statistics) "
                "or GELU + pre epilogue");
  constexpr bool STATS = IMP == 8 || IMP == 11;
  constexpr bool XA = IMP == 11 || IMP == 12;   // A = bf16(a sc + sh) formed on its way to LDS (as v2)
  __shared__ float xtab[XA ? 2 * XB_MAXK : 4];
  constexpr int BMV = 256, BNV = 128, NT = 512;
  constexpr int CHA = TileLoader<BMV, NT, true>::CH, CHB = TileLoader<BNV, NT, BK>::CH;
  constexpr int KSTEPB = TileLoader<BNV, NT, BK>::KSTEP;
  __shared__ __attribute__((aligned(16))) char lds[PP_LDS];
  char* la = lds;
  char* lb = lds + BMV * BKT * 2;
  // the wave index in a scalar register: the epilogue's descriptors hang off it
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char* img = lds + w * 8192;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int ntn = (g.N + BNV - 1) / BNV;
  const int T = ntn * ((g.M + BMV - 1) / BMV);
  const int x = blockIdx.x & 7, qstep = gridDim.x >> 3;
  const int T8 = T >> 3, R8 = T & 7;
  const int cnt = T8 + (x < R8 ? 1 : 0), tbase = x * T8 + (x < R8 ? x : R8);
  const int it = blockIdx.x >> 3;
  if (it >= cnt) return;
  if constexpr (XA) {   // = Affine8::init per channel (v2's IMP 11 / 12 table)
    for (int c = threadIdx.x; c < g.K; c += NT) {
      const float sc = g.xb_act.rstd[c] * g.xb_act.w[c];
      xtab[c] = sc;
      xtab[XB_MAXK + c] = bn_shift(g.xb_act.b[c], g.xb_act.mean[c], sc);
    }
    __syncthreads();
  }
  const __bf16* A = (const __bf16*)g.A;
  const __bf16* B = (const __bf16*)g.B;
  const int K = g.K;
  const int nk = (K + BKT - 1) / BKT;
  const uint32_t a_rs = (uint32_t)((NT / 8) * g.lda * 2);   // bytes between a thread's chunks
  const uint32_t b_rs = BK ? (uint32_t)((NT / 8) * g.ldb * 2) : (uint32_t)(KSTEPB * g.ldb * 2);

  int lm0 = 0, ln0 = 0;   // the loaders' tile
  auto setup = [&](int i) {
    const int tt = tbase + i;
    lm0 = (tt / ntn) * BMV;
    ln0 = (tt % ntn) * BNV;
  };
  // operand staging (TileLoader's chunk map; rows past the matrix clipped by the descriptor's
  // record count (K-major) or an out-of-range offset (M/N-major columns), chunks past K by
  // the K check).  The K-major chunks' row stride goes in the VGPR offset: the buffer range
  // check covers voffset (+ the instruction offset) but not the scalar offset on CDNA, so a
  // chunk i >= 1 of a ragged last tile addressed through soffset would read rows past the
  // matrix -- past the end of its allocation for an A / B at the end of one.
  uint4 ra[CHA], rb[CHB];
  auto issue = [&](int k0) {
    const int t = opaque_tid();
    const int kv = K - k0;
    const int arows = g.M - lm0 < BMV ? g.M - lm0 : BMV;
    const auto rsa = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)lm0 * g.lda + k0), (short)0,
                                                       (int)(((int64_t)arows * g.lda - k0) * 2), 0x00020000);
    const int kk = (t & 7) * 8;
    const uint32_t a_v = kk < kv ? (uint32_t)(((t >> 3) * g.lda + kk) * 2) : BUF_OOB;
#pragma unroll
    for (int i = 0; i < CHA; ++i)
      ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsa, a_v + i * a_rs, 0, 0));
    const int bcols = g.N - ln0 < BNV ? g.N - ln0 : BNV;
    if constexpr (BK) {
      const auto rsb = __builtin_amdgcn_make_buffer_rsrc((void*)(B + (int64_t)ln0 * g.ldb + k0), (short)0,
                                                         (int)(((int64_t)bcols * g.ldb - k0) * 2), 0x00020000);
      const uint32_t b_v = kk < kv ? (uint32_t)(((t >> 3) * g.ldb + kk) * 2) : BUF_OOB;
#pragma unroll
      for (int i = 0; i < CHB; ++i)
        rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsb, b_v + i * b_rs, 0, 0));
    } else {
      const auto rsb = panel_rsrc(B, (int64_t)k0 * g.ldb + ln0);
      const int bk = t / (BNV / 8), bc = (t % (BNV / 8)) * 8;
      const uint32_t b_v = (uint32_t)((bk * g.ldb + bc) * 2);
#pragma unroll
      for (int i = 0; i < CHB; ++i)
        rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsb, (bc < bcols && bk + KSTEPB * i < kv) ? b_v : BUF_OOB, i * b_rs, 0));
    }
  };
  auto put = [&](int k0) {
    const int t = opaque_tid();
    if constexpr (XA) {   // x = bf16(a sc + sh) of the thread's 8 channels (chunks past K stay zero)
      const int c0 = k0 + (t & 7) * 8;
      if (c0 < K) {
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
          const float2 sc2 = *(const float2*)(xtab + c0 + 2 * jp);
          const float2 sh2 = *(const float2*)(xtab + XB_MAXK + c0 + 2 * jp);
#pragma unroll
          for (int i = 0; i < CHA; ++i) {
            uint32_t* wv = (uint32_t*)&ra[i];
            const float lo = __uint_as_float(wv[jp] << 16), hi = __uint_as_float(wv[jp] & 0xFFFF0000u);
            typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
            const bf16x2 o = {(__bf16)fmaf(lo, sc2.x, sh2.x), (__bf16)fmaf(hi, sc2.y, sh2.y)};
            wv[jp] = __builtin_bit_cast(uint32_t, o);
          }
        }
      }
    }
    const int a_l0 = kmaj_off(t >> 3, t & 7);
    const int b_l0 = BK ? a_l0 : mnmaj_off_r<BNV>(t / (BNV / 8), (t % (BNV / 8)) * 8);
#pragma unroll
    for (int i = 0; i < CHA; ++i) *(uint4*)(la + a_l0 + i * TileLoader<BMV, NT, true>::LSTEP) = ra[i];
#pragma unroll
    for (int i = 0; i < CHB; ++i) *(uint4*)(lb + b_l0 + i * TileLoader<BNV, NT, BK>::LSTEP) = rb[i];
  };
  f32x16 acc[2][2];
  auto kstep = [&]() {
#pragma unroll
    for (int s = 0; s < BKT / 16; ++s) {
      if constexpr (!BK) {
        // M/N-major B (data gradient): the second B fragment (two transposed reads) is read
        // behind the first column's MFMAs -- 4 fragment VGPRs fewer at the 128-register cap
        // (the all-reads-first order spills 4 VGPRs into this loop); same MFMA order per
        // accumulator, so the outputs are unchanged
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = lread_frag_r<true, BMV>(la, wm + 32 * i, s);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 bj = lread_frag_r<BK, BNV>(lb, wn + 32 * j, s);
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bj, af[i], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        continue;
      }
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lread_frag_r<true, BMV>(la, wm + 32 * i, s);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = lread_frag_r<BK, BNV>(lb, wn + 32 * j, s);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      // v2's order: the substep's four fragment reads, then its four MFMAs (left to itself the
      // scheduler here issued the fourth read behind two MFMAs and waited on it)
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
  };
  // the K loop of the loaders' tile, its K-step 0 operands already issued
  auto ksteps = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    put(0);   // K-step 0, outside the loop (see above)
    __syncthreads();
    if (nk > 1) issue(BKT);
    kstep();
    __syncthreads();
    for (int ks = 1; ks < nk; ++ks) {
      put(ks * BKT);
      __syncthreads();
      if (ks + 1 < nk) issue((ks + 1) * BKT);
      kstep();
      __syncthreads();
    }
  };
  setup(it);
  issue(0);
  ksteps();
  int cm0 = lm0, cn0 = ln0;
  for (int in = it + qstep; in < cnt; in += qstep) {
    if constexpr (IMP == 13) pp_stage_gelu_aux(g, acc, cm0, cn0, wm, wn, opaque_tid() & 63, img);
    else if constexpr (IMP == 9) pp_stage_gelu_bwd(g, acc, cm0, cn0, wm, wn, opaque_tid() & 63, img);
    else pp_stage(g, acc, cm0, cn0, wm, wn, opaque_tid() & 63, img);
    setup(in);
    issue(0);
    if constexpr (IMP == 13 || IMP == 9) {   // pre -> aux / h -> aux_out (stores younger than the next operands), then C
      if (IMP == 13 || g.aux_out) pp_flush<false>(g, IMP == 13 ? g.aux : g.aux_out, cm0, cn0, wm, wn, opaque_tid() & 63, img);
      pp_stage_runs(acc, opaque_tid() & 63, img);
    }
    pp_flush<STATS>(g, g.C, cm0, cn0, wm, wn, opaque_tid() & 63, img);
    __syncthreads();   // every wave's images read before the next tile's operands land
    cm0 = lm0;
    cn0 = ln0;
    ksteps();
  }
  if constexpr (IMP == 13) {
    pp_stage_gelu_aux(g, acc, cm0, cn0, wm, wn, threadIdx.x & 63, img);
    pp_flush<false>(g, g.aux, cm0, cn0, wm, wn, threadIdx.x & 63, img);
    pp_stage_runs(acc, threadIdx.x & 63, img);
  } else if constexpr (IMP == 9) {
    pp_stage_gelu_bwd(g, acc, cm0, cn0, wm, wn, threadIdx.x & 63, img);
    if (g.aux_out) pp_flush<false>(g, g.aux_out, cm0, cn0, wm, wn, threadIdx.x & 63, img);
    pp_stage_runs(acc, threadIdx.x & 63, img);
  } else {
    pp_stage(g, acc, cm0, cn0, wm, wn, threadIdx.x & 63, img);
  }
  pp_flush<STATS>(g, g.C, cm0, cn0, wm, wn, threadIdx.x & 63, img);
}

// ============================================================ f32 MFMA kernel
constexpr int FBM = 64, FBN = 64, FBK = 16, FLD = 64 + 4;

template <bool KMAJ>
SM_DEV void f32_stage(const float* base, int64_t ld, int rows_total, int row0, int k0, int kend,
                      float* lds /*[FBK][FLD]*/) {
  const int t = threadIdx.x;
  if (KMAJ) {                     // stored [row][k]: 64 rows x 16 k
    const int row = t >> 2, kc = (t & 3) * 4;
    const int gr = row0 + row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gk = k0 + kc + i;
      lds[(kc + i) * FLD + row] = (gr < rows_total && gk < kend) ? base[(int64_t)gr * ld + gk] : 0.f;
    }
  } else {                        // stored [k][row]: 16 k x 64 rows
    const int kr = t >> 4, rc = (t & 15) * 4;
    const int gk = k0 + kr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gr = row0 + rc + i;
      lds[kr * FLD + rc + i] = (gr < rows_total && gk < kend) ? base[(int64_t)gk * ld + gr] : 0.f;
    }
  }
}

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
  __shared__ float la[FBK * FLD], lb[FBK * FLD];
  const int ntn = (g.N + FBN - 1) / FBN;
  const int m0 = (blockIdx.x / ntn) * FBM, n0 = (blockIdx.x % ntn) * FBN;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const float* A = (const float*)g.A;
  const float* B = (const float*)g.B;
  const int kb = g.k_begin + blockIdx.z * g.k_chunk;
  const int ke = min(g.K, kb + g.k_chunk);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = kb; k0 < ke; k0 += FBK) {
    f32_stage<AK>(A, g.lda, g.M, m0, k0, ke, la);
    f32_stage<BK>(B, g.ldb, g.N, n0, k0, ke, lb);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < FBK / 2; ++s) {
      const float a = la[(2 * s + (l >> 5)) * FLD + wm + (l & 31)];
      const float b = lb[(2 * s + (l >> 5)) * FLD + wn + (l & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int h = l >> 5;
  const int col = n0 + wn + (l & 31);
  if (col < g.N) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < g.M) epilogue_store<float>(g, row, col, acc[r], blockIdx.z);
    }
  }
}

// ============================================================ split-K reduce
template <typename TC>
__global__ void splitk_reduce_kernel(GemmArgs g, int splits) {
  const int64_t total = (int64_t)g.M * g.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += g.partial[(int64_t)z * total + i];
    const int64_t row = i / g.N;
    const int col = (int)(i - row * g.N);
    GemmArgs h = g;
    h.partial = nullptr;
    epilogue_store<TC>(h, row, col, s, 0);
  }
}

int variant_bm(int v);
int variant_bn(int v);
int gemm_variant(int M, int N, int K);

// Resident blocks of a bf16 variant on the whole device (occupancy query of the
// split-K instantiation, cached; 2 / 4 blocks per CU x 256 CUs without a device).
int gemm_slots(int v) {
  static int cache[4] = {0, 0, 0, 0};
  const int vi = v == 2 ? 2 : 3;
  if (cache[vi]) return cache[vi];
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess) {
    const hipError_t e =
        vi == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gemm_bf16_v2<false, false, float, true, 256>, 512, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gemm_bf16_v2<false, false, float, true, 128>, 256, 0);
    if (e != hipSuccess) per = 0;
  }
  if (cus <= 0 || per <= 0) {
    (void)hipGetLastError();
    cus = 256;
    per = vi == 2 ? 2 : 4;
  }
  cache[vi] = cus * per;
  return cache[vi];
}

// Split-K over a long reduction (weight gradients: K = tokens).  bf16: the split count
// makes the grid exactly two rounds of resident blocks (tiles x splits <= 2 x slots):
// every block does the same work, so a grid one block past a round boundary pays a
// whole extra round (the previous rule, ceil(1024 / tiles), gave 1026-1035 blocks for
// 512 slots on every weight gradient of the step).  (A group-major order -- each
// split's tiles sharing a token range dealt consecutively in groups of <= 8 -- measured
// 0-16 % slower than this split-major order on every weight gradient.)
int choose_splits(int M, int N, int K, bool bf16) {
  const int v = gemm_variant(M, N, K);
  const int bm = bf16 ? variant_bm(v) : FBM, bn = bf16 ? variant_bn(v) : FBN, bk = bf16 ? BKT : FBK;
  const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int64_t slots = bf16 ? gemm_slots(v) : 512;
  if (tiles >= slots || K < 4096) return 1;
  // two rounds: 2-16 rounds measured the same time (profiles/r04f_dw_rounds.txt; the A/B knob
  // that pinned the count, and so the reduction order, is gone: results stay reproducible)
  constexpr int rounds = 2;
  int64_t want = bf16 ? (rounds * slots) / tiles : (1024 + tiles - 1) / tiles;
  int64_t max_by_k = K / (4 * bk);
  int64_t s = want < max_by_k ? want : max_by_k;
  if (s > 2048) s = 2048;
  return s < 1 ? 1 : (int)s;
}

// bf16 kernel variant: 1 = gemm_bf16_kernel (128 x 128, 4 waves), 2 = gemm_bf16_v2 at
// BM = 256 (8 waves), 3 = gemm_bf16_v2 at BM = 128.  Default (0): v2, BM = 256 when
// M >= 192 (a 256-row tile half empty loses to BM = 128 there: dW of the 96-channel
// MBConv projection).  sm_gemm_tuning(TUNE_VARIANT) pins one (A/B measurement runs).
// Measured and dropped (round 2): a 256 x 256 tile on 8 waves of 128 x 64 (0.75 KB of
// fragment reads and 256 B of LDS-DMA staging per MFMA instead of v2's 1 KB + 384 B),
// double-buffered buffer -> LDS DMA, one block per CU: 20-30 % slower than v2 on every
// weight gradient of the step (profiles/r02g/dw_wide.txt).  Its operand delivery per CU
// (64 KB in flight, ~21 GB/s) is the bound, not the LDS; v2's two resident blocks keep
// 96 KB in flight.
// Tuning knobs (A/B measurement runs only; scripts/ set them through sm_gemm_tuning, the
// product path never changes them).  Defaults are the measured best per shape family.
enum { TUNE_VARIANT = 0, TUNE_PP = 1, TUNE_PP_MINN = 2, TUNE_PP_MAXK = 3, TUNE_PP_ROUNDS = 4,
       TUNE_PP_ROUNDS_SMALLK = 5, TUNE_PP_ROUNDS_MIDK = 6, TUNE_MF16_MINK = 7, TUNE_DW384 = 8,
       TUNE_DW384_NOTR = 9, TUNE_COUNT = 10 };
constexpr int kMF16Off = 1 << 30;
constexpr int kTuneDefault[TUNE_COUNT] = {0, 1, 128, 6 * BKT, -1, 8, 2, kMF16Off, 1, 1};
int g_tune[TUNE_COUNT] = {0, 1, 128, 6 * BKT, -1, 8, 2, kMF16Off, 1, 1};
int gemm_variant(int M, int N, int K) {
  const int forced = (g_tune[TUNE_VARIANT] >= 1 && g_tune[TUNE_VARIANT] <= 3) ? g_tune[TUNE_VARIANT] : 0;
  if (forced) return forced;
  // 384-row weight gradients with narrow rows (dW [384][384], [384][96]): three full
  // 128-row tiles instead of two 256-row tiles, one a quarter empty -- measured
  // 0.86 -> 0.79 ms and 5.18 -> 4.45 ms; wider (N = 1536) and 192-row ones are faster at
  // BM = 256 (profiles/r02q/dw_bm_ab.txt)
  if (M == 384 && N <= 384) return 3;
  return M >= 192 ? 2 : 3;
  (void)K;
}
int variant_bm(int v) { return v == 2 ? 256 : 128; }
int variant_bn(int v) { return 128; (void)v; }

// Persistent pipelined form (gemm_bf16_pp) for a non-split bf16 GEMM with a K-major A at
// BM = 256 whose epilogue has no side output: used when the grid would take more than one
// round of resident blocks.  sm_gemm_persistent(0) (sm_gemm_tuning(TUNE_PP)) selects
// the one-tile-per-block v2 form; both give bit-identical outputs.
bool pp_enabled() { return g_tune[TUNE_PP] != 0; }
// Where it pays (same-box A/B, profiles/r05b_gemm_persistent_ab.txt, r05aa_gemm_pp_rounds.txt): K <= 128
// (write-bound: stage-0 expand / projection data gradient -4..-13 %), and K <= 384 at N >= 512
// (several n-tiles share each A panel: decoder qkv / fc1 forward -6..-7 %, fc2 data gradient
// -2 %).  At K >= 768 it loses (fc1 / qkv data gradients +2..4 %), and with one n-tile (N = 96)
// there is no A panel to share.  Blocks take at most pp_rounds() tiles each (8 at K <= 128, 2
// above): fully persistent blocks drift apart, so the n-tile blocks that share an A panel no
// longer stream it through L2 together (K = 384: -1..+1 % persistent against -6 % at 2 tiles).
// Round 6: at K <= 384 the persistent form also pays below N = 512 (the old minimum): forward
// N = 192 / 384 -9..-11 %, and, once its K loop reads the data gradient's M/N-major B fragments
// column by column (no spills), the data gradient -1.4..-3.9 % (it lost 6-13 % before); past
// K = 384 the data gradient still loses 2-4 %, the forward gains 1-2.5 % (not taken;
// profiles/r06y_pp_minn_ab.txt).  The minimum N is now 128 (two n-tiles: N = 96 keeps one tile
// per block, see above).
bool pp_ok(const GemmArgs& g) {
  return pp_enabled() && g.partial == nullptr && g.colsum == nullptr && !g.ctrans && !(g.epi & 4) &&
         (!((g.epi & 1) && g.aux) || (g.beta == 0.f && g.row_scale == nullptr)) && g.aux_out == nullptr &&
         g.K > 0 && g.k_begin == 0 && g.k_chunk >= g.K &&
         (g.K <= 2 * BKT || (g.K <= g_tune[TUNE_PP_MAXK] && g.N >= g_tune[TUNE_PP_MINN]));
}
// the GELU-backward data gradient, with or without the activation side output (IMP 9), in the
// persistent form: the same shape rule, no bias / residual / row scale in its epilogue
bool pp_ok_gelu_bwd(const GemmArgs& g) {
  return pp_enabled() && g.partial == nullptr && g.colsum == nullptr && !g.ctrans && g.epi == 4 && g.aux &&
         g.bias == nullptr && g.beta == 0.f && g.row_scale == nullptr && g.K > 0 && g.k_begin == 0 &&
         g.k_chunk >= g.K && (g.K <= 2 * BKT || (g.K <= g_tune[TUNE_PP_MAXK] && g.N >= g_tune[TUNE_PP_MINN]));
}
int pp_rounds(const GemmArgs& g) {
  const int forced = g_tune[TUNE_PP_ROUNDS];   // A/B runs; 0 = fully persistent
  return forced >= 0 ? forced : g.K <= 2 * BKT ? g_tune[TUNE_PP_ROUNDS_SMALLK] : g_tune[TUNE_PP_ROUNDS_MIDK];
}
// K loop on v_mfma_f32_16x16x32_bf16 (v2's MF = 16) for the BM = 256 plain-operand tiles with
// a K-major A whose K per block is at least g_tune[TUNE_MF16_MINK].  (With an M/N-major A -- the
// weight gradients -- and in gemm_bf16_pp the 16x16x32 loop's four A fragments spill 11-36
// VGPRs at the 128-register cap of two 8-wave blocks per CU: not built.)
bool mf16_ok(const GemmArgs& g) { return (g.k_chunk < g.K ? g.k_chunk : g.K) >= g_tune[TUNE_MF16_MINK]; }
template <bool BK, int IMP>
bool launch_pp(const GemmArgs& g, hipStream_t st) {
  static int slots = 0;   // resident blocks on the device, a multiple of 8 (occupancy query, cached)
  if (slots == 0) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gemm_bf16_pp<BK, IMP>, 512, 0) != hipSuccess) {
      (void)hipGetLastError();
      cus = 256;
      per = 2;
    }
    slots = (cus * (per > 0 ? per : 1)) & ~7;
    if (slots < 8) slots = 8;
  }
  const int64_t tiles = (int64_t)((g.N + 127) / 128) * ((g.M + 255) / 256);
  if (tiles <= slots) return false;   // one round: the one-tile-per-block form
  // at most R = pp_rounds() tiles per block (grid 8 ceil(T / 8 / R), at least one resident round)
  const int rounds = pp_rounds(g);
  int64_t grid = slots;
  if (rounds > 0) {
    const int64_t per = ((tiles + 7) / 8 + rounds - 1) / rounds;
    if (8 * per > grid) grid = 8 * per;
  }
  hipLaunchKernelGGL((gemm_bf16_pp<BK, IMP>), dim3((unsigned)grid), dim3(512), 0, st, g);
  return true;
}

// split count for gemm_dw384 (one block per CU): the largest R <= 2 whole rounds of the CUs that
// stays within the v2 split count the caller's workspace was sized for
int dw384_splits(int M, int N, int s_v2) {
  if (!g_tune[TUNE_DW384] || M % DW3_BM || N % DW3_BN || s_v2 <= 1) return s_v2;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      cus = 256;
    }
  }
  const int tiles = (M / DW3_BM) * (N / DW3_BN);
  for (int r = 2; r >= 1; --r) {
    const int sr = r * cus / tiles;
    if (sr >= 2 && sr <= s_v2) return sr;
  }
  return s_v2;
}
template <bool AK, bool BK, typename TC, bool VEC>
void launch_bf16(const GemmArgs& g, int splits, hipStream_t st) {
  if constexpr (!AK && !BK && sizeof(TC) == 4 && VEC) {
    // weight gradients on the 384 x 128 pipelined tile (gemm_dw384) where it divides the output
    if (g_tune[TUNE_DW384] && g.M % DW3_BM == 0 && g.N % DW3_BN == 0 && g.partial != nullptr) {
      const int t384 = (g.N / DW3_BN) * (g.M / DW3_BM);
      if (g.colsum) hipLaunchKernelGGL((gemm_dw384<true>), dim3(t384 * splits), dim3(512), 0, st, g);
      else hipLaunchKernelGGL((gemm_dw384<false>), dim3(t384 * splits), dim3(512), 0, st, g);
      return;
    }
  }
  const int v = gemm_variant(g.M, g.N, g.K);
  const int bm = variant_bm(v), bn = variant_bn(v);
  const int tiles = ((g.N + bn - 1) / bn) * ((g.M + bm - 1) / bm);
  if constexpr (AK && VEC && sizeof(TC) == 2) {
    if (v == 2 && splits == 1 && pp_ok(g)) {
      if ((g.epi & 1) && g.aux) {   // fc1: GELU + pre-activation side output
        if (launch_pp<BK, 13>(g, st)) return;
      } else if (launch_pp<BK, 0>(g, st)) {
        return;
      }
    }
  }
  if (v == 1) hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK, TC, VEC>), dim3(tiles, 1, splits), dim3(256), 0, st, g);
  else if (AK && v == 2 && mf16_ok(g))
    hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, VEC, 256, 0, 128, AK ? 16 : 32>), dim3(tiles * splits), dim3(512), 0, st, g);
  else if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, VEC, 256>), dim3(tiles * splits), dim3(512), 0, st, g);
  else hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, VEC, 128>), dim3(tiles * splits), dim3(256), 0, st, g);
}

template <bool AK, bool BK>
int launch_layout(int abt, int ct, GemmArgs g, int splits, hipStream_t st) {
  if (abt == SM_BF16) {
    const bool vec = !((g.N & 7) || (!g.partial && (g.ldc & 7)));
    if (ct == SM_BF16) {
      if (vec) launch_bf16<AK, BK, __bf16, true>(g, splits, st);
      else launch_bf16<AK, BK, __bf16, false>(g, splits, st);
    } else {
      if (vec) launch_bf16<AK, BK, float, true>(g, splits, st);
      else launch_bf16<AK, BK, float, false>(g, splits, st);
    }
  } else {
    if (ct != SM_F32) return -3;
    dim3 grid(((g.N + FBN - 1) / FBN) * ((g.M + FBM - 1) / FBM), 1, splits);
    hipLaunchKernelGGL((gemm_f32_kernel<AK, BK>), grid, dim3(256), 0, st, g);
  }
  SM_CHECK_LAUNCH();
  return 0;
}

// implicit-conv GEMMs (bf16 operands, N % 8 == 0): IMP 1 = A implicit (forward,
// data gradient: A K-major, B = packed weights [N][K]); IMP 2 = B implicit (weight
// gradient: A = dy stored [K][M], fp32 split-K slabs)
template <int IMP, typename TC>
void launch_conv(const GemmArgs& g, int splits, hipStream_t st) {
  const int v = gemm_variant(g.M, g.N, 0) == 2 ? 2 : 3;
  const int bm = variant_bm(v);
  constexpr bool AK = IMP == 1 || IMP == 10, BK = AK;
  if constexpr (IMP == 1) {
    if (g.N <= 64 && v == 2) {   // narrow output (the stem's 48-channel data gradient): 64-column tiles
      const dim3 grid(((g.N + 63) / 64) * ((g.M + 255) / 256) * splits);
      hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, true, 256, IMP, 64>), grid, dim3(512), 0, st, g);
      return;
    }
  }
  dim3 grid(((g.N + 127) / 128) * ((g.M + bm - 1) / bm) * splits);
  if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, true, 256, IMP>), grid, dim3(512), 0, st, g);
  else hipLaunchKernelGGL((gemm_bf16_v2<AK, BK, TC, true, 128, IMP>), grid, dim3(256), 0, st, g);
}

GemmArgs conv_args(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
                   int H, int W, int Cs, int flip) {
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.alpha = 1.f; g.beta = 0.f; g.rows_per_group = 1; g.k_begin = 0; g.k_chunk = K;
  g.cH = H; g.cW = W; g.cC = Cs; g.cflip = flip;
  return g;
}

bool conv_shape_ok(int64_t P, int H, int W, int Cin, int Cout, const void* a, const void* b, const void* c) {
  return P > 0 && P < (1LL << 31) && H > 0 && W > 0 && W < 0x8000 && H < 0x8000 && Cin % 8 == 0 &&
         Cout % 8 == 0 && ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c)) & 15) == 0;
}

}  // namespace

// ---- stem conv2 (tiny_vit.py:69: 3x3, stride 1, pad 1) as implicit-im2col GEMMs ----
// forward: y[p][co] = sum_{tap, ci} x[p + off(tap)][ci] * wpack[co][tap * Cin + ci]
extern "C" int sm_conv3x3_fwd(const void* x, const void* wpack, void* y, int F, int H, int W, int Cin, int Cout,
                              hipStream_t st) {
  const int64_t P = (int64_t)F * H * W;
  if (!conv_shape_ok(P, H, W, Cin, Cout, x, wpack, y)) return -2;
  GemmArgs g = conv_args((int)P, Cout, 9 * Cin, x, Cin, wpack, 9 * Cin, y, Cout, H, W, Cin, 0);
  launch_conv<1, __bf16>(g, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

// data gradient: dx[p][ci] = sum_{tap, co} dy[p + (1-ky, 1-kx)][co] * wpack_t[ci][tap * Cout + co]
extern "C" int sm_conv3x3_dgrad(const void* dy, const void* wpack_t, void* dx, int F, int H, int W, int Cin, int Cout,
                                hipStream_t st) {
  const int64_t P = (int64_t)F * H * W;
  if (!conv_shape_ok(P, H, W, Cin, Cout, dy, wpack_t, dx)) return -2;
  GemmArgs g = conv_args((int)P, Cin, 9 * Cout, dy, Cout, wpack_t, 9 * Cout, dx, Cin, H, W, Cout, 1);
  launch_conv<1, __bf16>(g, 1, st);
  SM_CHECK_LAUNCH();
  return 0;
}

// weight gradient: dw[co][tap * Cin + ci] (+)= sum_p dy[p][co] * x[p + off(tap)][ci]  (fp32,
// split-K over the pixels with a fixed-order slab reduction)
extern "C" int64_t sm_conv3x3_wgrad_workspace_bytes(int F, int H, int W, int Cin, int Cout) {
  const int64_t P = (int64_t)F * H * W;
  const int s = choose_splits(Cout, 9 * Cin, (int)(P < (1LL << 31) ? P : (1LL << 31) - 1), true);
  return s > 1 ? (int64_t)s * Cout * 9 * Cin * 4 : 0;
}

extern "C" int sm_conv3x3_wgrad(const void* dy, const void* x, float* dw, int accumulate, int F, int H, int W, int Cin,
                                int Cout, void* ws, int64_t ws_bytes, hipStream_t st) {
  const int64_t P = (int64_t)F * H * W;
  if (!conv_shape_ok(P, H, W, Cin, Cout, dy, x, dw)) return -2;
  const int N = 9 * Cin;
  GemmArgs g = conv_args(Cout, N, (int)P, dy, Cout, x, N, dw, N, H, W, Cin, 0);
  g.beta = accumulate ? 1.f : 0.f;
  int splits = choose_splits(Cout, N, (int)P, true);
  if (splits > 1 && (ws == nullptr || ws_bytes < (int64_t)splits * Cout * N * 4)) splits = 1;
  if (splits > 1) {
    int chunk = (int)((P + splits - 1) / splits);
    chunk = (chunk + BKT - 1) / BKT * BKT;
    splits = (int)((P + chunk - 1) / chunk);
    g.k_chunk = chunk;
    g.partial = (float*)ws;
  }
  launch_conv<2, float>(g, splits, st);
  SM_CHECK_LAUNCH();
  if (splits > 1) {
    const int64_t total = (int64_t)Cout * N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, g, splits);
    SM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sm_gemm_persistent(int mode) {
  const int prev = pp_enabled() ? 1 : 0;
  if (mode >= 0) g_tune[TUNE_PP] = mode ? 1 : 0;
  return prev;
}

// A/B tuning knob `key` (TUNE_* above): *prev <- its current value; set != 0 stores `value`
// (set < 0 restores the default).  Host-side only, no launch.  Returns 0, or -2 for an
// unknown key.  Not thread-safe against concurrent GEMM launches: set before the run.
extern "C" int sm_gemm_tuning(int key, int set, int value, int* prev) {
  if (key < 0 || key >= TUNE_COUNT) return -2;
  if (prev) *prev = g_tune[key];
  if (set > 0) g_tune[key] = value;
  else if (set < 0) g_tune[key] = kTuneDefault[key];
  return 0;
}

extern "C" int64_t sm_gemm_workspace_bytes(int ab_dtype, int M, int N, int K) {
  const int s = choose_splits(M, N, K, ab_dtype == SM_BF16);
  return s > 1 ? (int64_t)s * M * N * 4 : 0;
}

static int gemm_run(int ab_dtype, int c_dtype, int a_layout, int b_layout, int M, int N, int K, const void* A,
                    int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, const float* bias, float alpha,
                    float beta, int epi, void* aux, const void* R, float drop_p, uint64_t seed,
                    const float* row_scale, int64_t rows_per_group, void* workspace, int64_t ws_bytes,
                    float* colsum, float* colsum_out, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (ab_dtype == SM_BF16) {
    // a K-major operand is staged in 8-element (16-B) chunks along K: K % 8; M/N-major
    // operands are staged one K row per chunk, so any K (e.g. the token-row reduction
    // of a weight gradient over B * 49 rows) works
    if (((a_layout == 0 || b_layout == 0) && K % 8) || lda % 8 || ldb % 8) return -2;
    if (a_layout == 1 && M % 8) return -2;
    if (b_layout == 1 && N % 8) return -2;
    if (((uintptr_t)A | (uintptr_t)B) & 15) return -2;
  }
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.bias = bias; g.alpha = alpha; g.beta = beta; g.epi = epi; g.aux = aux; g.R = R;
  g.drop_p = drop_p; g.seed = seed; g.row_scale = row_scale; g.rows_per_group = rows_per_group > 0 ? rows_per_group : 1;
  g.colsum = colsum;
  int splits = choose_splits(M, N, K, ab_dtype == SM_BF16);
  if (ab_dtype == SM_BF16 && c_dtype == SM_F32 && a_layout == 1 && b_layout == 1) splits = dw384_splits(M, N, splits);
  if (splits > 1 && (workspace == nullptr || ws_bytes < (int64_t)splits * M * N * 4)) splits = 1;
  const int bk = ab_dtype == SM_BF16 ? BKT : FBK;
  if (K <= 0) {  // empty reduction: C = beta*C + bias (epilogue only)
    g.k_begin = 0; g.k_chunk = 0;
  } else if (splits > 1) {
    int chunk = (K + splits - 1) / splits;
    chunk = (chunk + bk - 1) / bk * bk;
    splits = (K + chunk - 1) / chunk;
    g.k_begin = 0; g.k_chunk = chunk; g.partial = (float*)workspace;
  } else {
    g.k_begin = 0; g.k_chunk = K;
  }
  int rc;
  if ((epi & 4) && ab_dtype == SM_BF16 && c_dtype == SM_BF16 && a_layout == 0 && b_layout == 1 && splits == 1 &&
      !((N & 7) || (ldc & 7)) && K > 0) {   // the GELU-backward dX GEMM: IMP 9 epilogue
    const int v = gemm_variant(M, N, K);
    const int tiles = ((N + 127) / 128) * ((M + variant_bm(v) - 1) / variant_bm(v));
    if (v == 2 && pp_ok_gelu_bwd(g) && launch_pp<false, 9>(g, stream)) {
      SM_CHECK_LAUNCH();
      return 0;
    }
    if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<true, false, __bf16, true, 256, 9>), dim3(tiles), dim3(512), 0, stream, g);
    else hipLaunchKernelGGL((gemm_bf16_v2<true, false, __bf16, true, 128, 9>), dim3(tiles), dim3(256), 0, stream, g);
    SM_CHECK_LAUNCH();
    rc = 0;
  } else if (a_layout == 0 && b_layout == 0) rc = launch_layout<true, true>(ab_dtype, c_dtype, g, splits, stream);
  else if (a_layout == 0 && b_layout == 1) rc = launch_layout<true, false>(ab_dtype, c_dtype, g, splits, stream);
  else if (a_layout == 1 && b_layout == 0) rc = launch_layout<false, true>(ab_dtype, c_dtype, g, splits, stream);
  else rc = launch_layout<false, false>(ab_dtype, c_dtype, g, splits, stream);
  if (rc) return rc;
  if (splits > 1) {
    const int64_t total = (int64_t)M * N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (c_dtype == SM_BF16) hipLaunchKernelGGL(splitk_reduce_kernel<__bf16>, dim3(blocks), dim3(256), 0, stream, g, splits);
    else hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, stream, g, splits);
    SM_CHECK_LAUNCH();
  }
  if (colsum) {
    colred(colsum, K > 0 ? splits : 0, M, nullptr, colsum_out, 1, stream);
    SM_CHECK_LAUNCH();
  }
  return 0;
}

// fc2 data gradient through dropout(GELU(pre)) plus the fc2 weight gradient's operand
// (tiny_vit.py:74-84 Mlp / mae_vit_adapter.py:40-48 decoder FF backward): dx = (dy w) *
// keep / (1 - p) * GELU'(pre) and h = bf16(GELU(pre) * keep / (1 - p)) (bit-identical to
// sm_gelu_fwd(pre)) from one epilogue that reads pre once -- no recompute pass of h.
// dy [M][N], w [N][K], pre / dx / h [M][K] bf16; K % 8 == 0, N % 8 == 0.
extern "C" int sm_linear_dx_gelu(int M, int N, int K, const void* dy, const void* w, const void* pre, void* dx,
                                 void* h, float drop_p, uint64_t seed, hipStream_t stream) {
  if (M <= 0 || K <= 0) return 0;
  if (N <= 0 || N % 8 || K % 8 || (((uintptr_t)dy | (uintptr_t)w | (uintptr_t)pre | (uintptr_t)dx | (uintptr_t)h) & 15))
    return -2;
  GemmArgs g{};
  g.M = M; g.N = K; g.K = N; g.A = dy; g.lda = N; g.B = w; g.ldb = K; g.C = dx; g.ldc = K;
  g.alpha = 1.f; g.beta = 0.f; g.epi = 4; g.aux = const_cast<void*>(pre); g.aux_out = h;
  g.drop_p = drop_p; g.seed = seed; g.rows_per_group = 1; g.k_begin = 0; g.k_chunk = N;
  const int v = gemm_variant(g.M, g.N, g.K);
  const int tiles = ((g.N + 127) / 128) * ((g.M + variant_bm(v) - 1) / variant_bm(v));
  if (v == 2 && pp_ok_gelu_bwd(g) && launch_pp<false, 9>(g, stream)) {
    SM_CHECK_LAUNCH();
    return 0;
  }
  if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<true, false, __bf16, true, 256, 9>), dim3(tiles), dim3(512), 0, stream, g);
  else hipLaunchKernelGGL((gemm_bf16_v2<true, false, __bf16, true, 128, 9>), dim3(tiles), dim3(256), 0, stream, g);
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_gemm(int ab_dtype, int c_dtype, int a_layout, int b_layout, int M, int N, int K,
                       const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
                       const float* bias, float alpha, float beta, int epi, void* aux, const void* R,
                       float drop_p, uint64_t seed, const float* row_scale, int64_t rows_per_group,
                       void* workspace, int64_t ws_bytes, hipStream_t stream) {
  return gemm_run(ab_dtype, c_dtype, a_layout, b_layout, M, N, K, A, lda, B, ldb, C, ldc, bias, alpha, beta, epi,
                  aux, R, drop_p, seed, row_scale, rows_per_group, workspace, ws_bytes, nullptr, nullptr, stream);
}

// Weight and bias gradients of y = x W^T + b in one pass over dy: dW[nout][nin] (+)=
// dy^T x and db[nout] += column sums of dy (reference: the Linear / 1x1-conv
// backward autograd runs as two ops, a GEMM and a sum over rows).  bf16 operands.
extern "C" int64_t sm_colsum_workspace_bytes(int64_t M, int C);
extern "C" int sm_colsum(int dtype, int64_t M, int C, const void* x, float* out, int accumulate, void* ws,
                         int64_t ws_bytes, hipStream_t st);

namespace {
// Output rows x columns the bf16 v2 kernel computes for an M x N product (tile quantisation).
int64_t tiled_area(int M, int N) {
  const int bm = variant_bm(gemm_variant(M, N, 0));
  return (int64_t)((M + bm - 1) / bm) * bm * ((N + 127) / 128) * 128;
}
// dW = dy^T x computed transposed (dW^T = x^T dy: M = nin, N = nout) when that tiles the
// output with less waste and still splits K (the transposed store lives in the split-K
// reduce).  fc2's [384][1536] weight gradient: two 256-row m-tiles, one half empty, vs six
// exact ones -- the shape of fc1's [1536][384] gradient, which ran 2x faster.
// Only when the transposed tiling is exact: [576][192] tiles smaller transposed (192 rows on
// a 256-row tile) yet ran 3.45 -> 4.40 ms (profiles/r03g_dw_ab.txt).
bool dw_transposed(int rows, int nout, int nin) {
  // the 384 x 128 weight-gradient tile divides [384 k][128 n] outputs as they are (fc2's [384][1536]):
  // no transposed store, and the bias gradient stays fused (no separate column-sum pass): -3.9 %
  // (profiles/r06zjk_dw384_ab.txt, r06zm)
  if (g_tune[TUNE_DW384] && g_tune[TUNE_DW384_NOTR] && nout % DW3_BM == 0 && nin % DW3_BN == 0) return false;
  return tiled_area(nin, nout) == (int64_t)nin * nout && tiled_area(nout, nin) * 10 > (int64_t)nout * nin * 11 &&
         choose_splits(nin, nout, rows, true) > 1;
}
}  // namespace

extern "C" int64_t sm_linear_dw_bias_workspace_bytes(int rows, int nout, int nin) {
  const int s = choose_splits(nout, nin, rows, true);
  const int64_t plain = (s > 1 ? (int64_t)s * nout * nin * 4 : 0) + (int64_t)s * nout * 4 + 256;
  if (!dw_transposed(rows, nout, nin)) return plain;
  const int st = choose_splits(nin, nout, rows, true);
  const int64_t tr = (int64_t)st * nout * nin * 4 + 256 + sm_colsum_workspace_bytes(rows, nout);
  return plain > tr ? plain : tr;
}

// fc2's weight gradient dW[nout][nin] (+)= dy^T dropout(GELU(pre)), db += colsum(dy),
// with the activation formed in the GEMM's operand loads (XformColsB): pre is the fc1
// pre-activation [rows][nin] bf16, (drop_p, seed) the fc1 output's dropout.
extern "C" int sm_linear_dw_bias_gelu(int rows, int nout, int nin, const void* dy, const void* pre, float drop_p,
                                      uint64_t seed, float* dW, float* db, int accumulate, void* ws, int64_t ws_bytes,
                                      hipStream_t stream) {
  if (nout <= 0 || nin <= 0 || rows <= 0) return 0;
  if (ws_bytes < sm_linear_dw_bias_workspace_bytes(rows, nout, nin)) return -4;
  if (nout % 8 || nin % 8 || (((uintptr_t)dy | (uintptr_t)pre) & 15)) return -2;
  const int v = gemm_variant(nout, nin, rows);
  if (v == 1) return -2;
  const int s = choose_splits(nout, nin, rows, true);
  const int64_t gbytes = s > 1 ? (int64_t)s * nout * nin * 4 : 0;
  float* colsum = (float*)(((uintptr_t)ws + gbytes + 15) & ~(uintptr_t)15);
  GemmArgs g{};
  g.M = nout; g.N = nin; g.K = rows; g.A = dy; g.lda = nout; g.B = pre; g.ldb = nin; g.C = dW; g.ldc = nin;
  g.alpha = 1.f; g.beta = accumulate ? 1.f : 0.f; g.rows_per_group = 1; g.colsum = colsum;
  g.xb_p = drop_p; g.xb_seed = seed;
  int splits = s;
  if (splits > 1) {
    int chunk = (rows + splits - 1) / splits;
    chunk = (chunk + BKT - 1) / BKT * BKT;
    splits = (rows + chunk - 1) / chunk;
    g.k_begin = 0; g.k_chunk = chunk; g.partial = (float*)ws;
  } else {
    g.k_begin = 0; g.k_chunk = rows;
  }
  const int bm = variant_bm(v);
  const dim3 grid(((nin + 127) / 128) * ((nout + bm - 1) / bm) * splits);
  if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<false, false, float, true, 256, 5>), grid, dim3(512), 0, stream, g);
  else hipLaunchKernelGGL((gemm_bf16_v2<false, false, float, true, 128, 5>), grid, dim3(256), 0, stream, g);
  SM_CHECK_LAUNCH();
  if (splits > 1) {
    const int64_t total = (int64_t)nout * nin;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, stream, g, splits);
    SM_CHECK_LAUNCH();
  }
  colred(colsum, splits, nout, nullptr, db, 1, stream);
  SM_CHECK_LAUNCH();
  return 0;
}

// The MBConv projection's weight gradient over the SE output (tiny_vit.py:29-34, 53):
// dW[nout][nin] (+)= dy^T h3 with h3[r][c] = bf16(bf16(GELU(a2[r][c] sc[c] + sh[c])) *
// gate[r / hw][c]) formed in the B-operand loads (IMP 7): se_scale's h3 pass (read a2,
// write h3, read it back) disappears.  a2 [rows][nin] bf16, dy [rows][nout] bf16;
// rows = frames * hw with hw % 64 == 0 (each 64-row K-step inside one frame).
// The MBConv projection's forward over the SE output (tiny_vit.py:29-34, 53): y[rows][nout]
// (bf16) = h3 W^T with h3[r][c] = bf16(bf16(act(a2[r][c])) * gate[r / hw][c]) formed in the
// A-operand loads (IMP 6): se_apply's h3 pass (read a2, write h3, read it back) is gone;
// bit-identical to sm_se_fwd's h3 + sm_gemm.  hw % 128 == 0 (a tile inside one frame),
// nin % 64 == 0, nin <= 1536.
extern "C" int sm_linear_se(int rows, int nout, int nin, const void* a2, const void* w, const float* act_mean,
                            const float* act_rstd, const float* act_w, const float* act_b, int act_gelu,
                            const float* gate, int hw, void* y, hipStream_t stream) {
  if (rows <= 0 || nout <= 0) return 0;
  if (nin <= 0 || nin % BKT || nin > XA_MAXK || nout % 8 || hw <= 0 || hw % 128 || rows % hw ||
      act_mean == nullptr || (((uintptr_t)a2 | (uintptr_t)w | (uintptr_t)y) & 15))
    return -2;
  GemmArgs g{};
  g.M = rows; g.N = nout; g.K = nin; g.A = a2; g.lda = nin; g.B = w; g.ldb = nin; g.C = y; g.ldc = nout;
  g.alpha = 1.f; g.beta = 0.f; g.rows_per_group = 1; g.k_begin = 0; g.k_chunk = nin;
  g.xb_act = ChanAffine{act_mean, act_rstd, act_w, act_b, act_gelu};
  g.xb_gate = gate; g.xb_hw = hw;
  const dim3 grid(((nout + 127) / 128) * ((rows + 127) / 128));
  hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 128, 6>), grid, dim3(256), 0, stream, g);
  SM_CHECK_LAUNCH();
  return 0;
}

// y = x W^T (bf16 out, nn.Linear / 1x1 conv without bias) plus the train-mode BatchNorm
// statistics of y (tiny_vit.py:16, the BN of the MBConv expand conv, :43): the GEMM epilogue
// sums the stored bf16 values per 64-row slab and column (part [M / 64][2][N]), then the
// fixed-order fp64 reduction + finalize / running-stat update of sm_bn_stats_from_partials
// -- no separate statistics pass over y.  x [M][K], w [N][K] bf16, N % 8 == 0.
constexpr int LBS_CHUNKS = 512;   // first-level row chunks of the slab partials

// part[nb][ncols] -> out[chunk][ncols]: fixed-order fp64 sums of row chunks (chunk =
// blockIdx.y), rounded to fp32 -- a many-block first level ahead of the 24-block colred
// (hundreds of thousands of 64-row slabs at the stage-0 shape)
__global__ __launch_bounds__(256) void rowchunk_sum_kernel(const float* part, int64_t nb, int ncols, int64_t chunk,
                                                           float* out) {
  __shared__ double red[8][32];
  const int cl = threadIdx.x & 31, gq = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = min(nb, r0 + chunk);
  double s = 0.0;
  if (c < ncols)
    for (int64_t r = r0 + gq; r < r1; r += 8) s += part[r * ncols + c];
  red[gq][cl] = s;
  __syncthreads();
  if (gq == 0 && c < ncols) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    out[(int64_t)blockIdx.y * ncols + c] = (float)t;
  }
}

extern "C" int64_t sm_linear_bn_stats_workspace_bytes(int M, int N) {
  return ((int64_t)(M + 63) / 64) * 2 * N * 4 + (int64_t)LBS_CHUNKS * 2 * N * 4 + 2 * (int64_t)N * 8 + 64;
}

extern "C" int sm_bn_stats_from_partials(const float* part, int64_t nrows, int C, int64_t M, float* mean,
                                         float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                                         float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                                         hipStream_t st);

extern "C" int sm_linear_bn_stats(int M, int N, int K, const void* x, const void* w, void* y, float* mean, float* rstd,
                                  float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum,
                                  float eps, int updates, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (M <= 0 || N <= 0) return -2;
  if (K <= 0 || K % 8 || N % 8 || (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & 15)) return -2;
  if (ws_bytes < sm_linear_bn_stats_workspace_bytes(M, N)) return -4;
  const int64_t nparts = (M + 63) / 64;
  float* part = (float*)ws;
  float* part2 = part + nparts * 2 * N;
  void* fin = (void*)(((uintptr_t)(part2 + (int64_t)LBS_CHUNKS * 2 * N) + 15) & ~(uintptr_t)15);
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = x; g.lda = K; g.B = w; g.ldb = K; g.C = y; g.ldc = N;
  g.alpha = 1.f; g.beta = 0.f; g.rows_per_group = 1; g.k_begin = 0; g.k_chunk = K;
  g.stat_part = part;
  const int tiles_n = (N + 127) / 128;
  if (gemm_variant(M, N, K) == 2 && pp_ok(g) && launch_pp<true, 8>(g, stream)) {
  } else if (gemm_variant(M, N, K) == 2)
    hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 256, 8>), dim3(tiles_n * ((M + 255) / 256)), dim3(512),
                       0, stream, g);
  else
    hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 128, 8>), dim3(tiles_n * ((M + 127) / 128)), dim3(256),
                       0, stream, g);
  SM_CHECK_LAUNCH();
  const int64_t chunk = (nparts + LBS_CHUNKS - 1) / LBS_CHUNKS;
  const int nch = (int)((nparts + chunk - 1) / chunk);
  hipLaunchKernelGGL(rowchunk_sum_kernel, dim3((2 * N + 31) / 32, nch), dim3(256), 0, stream, part, nparts, 2 * N,
                     chunk, part2);
  SM_CHECK_LAUNCH();
  return sm_bn_stats_from_partials(part2, nch, N, M, mean, rstd, run_mean, run_var, num_batches_tracked, momentum,
                                   eps, updates, fin, 2 * (int64_t)N * 8, stream);
}

// stem conv2 forward + the output's train-mode BatchNorm statistics from the GEMM epilogue (as
// sm_linear_bn_stats: no read pass of y for the statistics); the stem's conv2 -> BN2
extern "C" int sm_conv3x3_fwd_bn_stats(const void* x, const void* wpack, void* y, int F, int H, int W, int Cin,
                                       int Cout, float* mean, float* rstd, float* run_mean, float* run_var,
                                       int64_t* num_batches_tracked, float momentum, float eps, int updates, void* ws,
                                       int64_t ws_bytes, hipStream_t st) {
  const int64_t P = (int64_t)F * H * W;
  if (!conv_shape_ok(P, H, W, Cin, Cout, x, wpack, y)) return -2;
  if (ws_bytes < sm_linear_bn_stats_workspace_bytes((int)P, Cout)) return -4;
  const int64_t nparts = (P + 63) / 64;
  float* part = (float*)ws;
  float* part2 = part + nparts * 2 * Cout;
  void* fin = (void*)(((uintptr_t)(part2 + (int64_t)LBS_CHUNKS * 2 * Cout) + 15) & ~(uintptr_t)15);
  GemmArgs g = conv_args((int)P, Cout, 9 * Cin, x, Cin, wpack, 9 * Cin, y, Cout, H, W, Cin, 0);
  g.stat_part = part;
  launch_conv<10, __bf16>(g, 1, st);
  SM_CHECK_LAUNCH();
  const int64_t chunk = (nparts + LBS_CHUNKS - 1) / LBS_CHUNKS;
  const int nch = (int)((nparts + chunk - 1) / chunk);
  hipLaunchKernelGGL(rowchunk_sum_kernel, dim3((2 * Cout + 31) / 32, nch), dim3(256), 0, st, part, nparts, 2 * Cout,
                     chunk, part2);
  SM_CHECK_LAUNCH();
  return sm_bn_stats_from_partials(part2, nch, Cout, P, mean, rstd, run_mean, run_var, num_batches_tracked, momentum,
                                   eps, updates, fin, 2 * (int64_t)Cout * 8, st);
}

// The stem's BN2 folded into stage 0's first MBConv (tiny_vit.py:62-72 -> :43): the expand
// conv's A operand is the BatchNorm output x = bf16(a sc + sh) formed from the stored conv
// output a in the operand loads (IMP 11 / 12; sc = rstd w, sh = b - mean sc, exactly as
// sm_bn_apply stores x), so x is never written.  _bn_stats: plus the output's BatchNorm
// statistics (IMP 11, as sm_linear_bn_stats).  a [M][K] bf16, K % 8 == 0, K <= 1536.
static int linear_bnin_launch(int M, int N, int K, const void* a, const float* mean, const float* rstd,
                              const float* bw, const float* bb, const void* w, void* y, float* stat_part,
                              hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || K % 8 || K > XB_MAXK || N % 8 || mean == nullptr || rstd == nullptr || bw == nullptr ||
      bb == nullptr || (((uintptr_t)a | (uintptr_t)w | (uintptr_t)y) & 15))
    return -2;
  GemmArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = a; g.lda = K; g.B = w; g.ldb = K; g.C = y; g.ldc = N;
  g.alpha = 1.f; g.beta = 0.f; g.rows_per_group = 1; g.k_begin = 0; g.k_chunk = K;
  g.xb_act = ChanAffine{mean, rstd, bw, bb, 0};
  g.stat_part = stat_part;
  const int tiles_n = (N + 127) / 128;
  if (gemm_variant(M, N, K) == 2 && pp_ok(g)) {   // persistent form (K <= 128: the stage-0 expand)
    if (stat_part ? launch_pp<true, 11>(g, stream) : launch_pp<true, 12>(g, stream)) {
      SM_CHECK_LAUNCH();
      return 0;
    }
  }
  if (gemm_variant(M, N, K) == 2) {
    const dim3 grid(tiles_n * ((M + 255) / 256));
    if (stat_part) hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 256, 11>), grid, dim3(512), 0, stream, g);
    else hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 256, 12>), grid, dim3(512), 0, stream, g);
  } else {
    const dim3 grid(tiles_n * ((M + 127) / 128));
    if (stat_part) hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 128, 11>), grid, dim3(256), 0, stream, g);
    else hipLaunchKernelGGL((gemm_bf16_v2<true, true, __bf16, true, 128, 12>), grid, dim3(256), 0, stream, g);
  }
  SM_CHECK_LAUNCH();
  return 0;
}

extern "C" int sm_linear_bnin(int M, int N, int K, const void* a, const float* a_mean, const float* a_rstd,
                              const float* a_w, const float* a_b, const void* w, void* y, hipStream_t stream) {
  return linear_bnin_launch(M, N, K, a, a_mean, a_rstd, a_w, a_b, w, y, nullptr, stream);
}

extern "C" int sm_linear_bnin_bn_stats(int M, int N, int K, const void* a, const float* a_mean, const float* a_rstd,
                                       const float* a_w, const float* a_b, const void* w, void* y, float* mean,
                                       float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                                       float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                                       hipStream_t stream) {
  if (M <= 0 || N <= 0) return -2;
  if (ws_bytes < sm_linear_bn_stats_workspace_bytes(M, N)) return -4;
  const int64_t nparts = (M + 63) / 64;
  float* part = (float*)ws;
  float* part2 = part + nparts * 2 * N;
  void* fin = (void*)(((uintptr_t)(part2 + (int64_t)LBS_CHUNKS * 2 * N) + 15) & ~(uintptr_t)15);
  const int rc = linear_bnin_launch(M, N, K, a, a_mean, a_rstd, a_w, a_b, w, y, part, stream);
  if (rc) return rc;
  const int64_t chunk = (nparts + LBS_CHUNKS - 1) / LBS_CHUNKS;
  const int nch = (int)((nparts + chunk - 1) / chunk);
  hipLaunchKernelGGL(rowchunk_sum_kernel, dim3((2 * N + 31) / 32, nch), dim3(256), 0, stream, part, nparts, 2 * N,
                     chunk, part2);
  SM_CHECK_LAUNCH();
  return sm_bn_stats_from_partials(part2, nch, N, M, mean, rstd, run_mean, run_var, num_batches_tracked, momentum,
                                   eps, updates, fin, 2 * (int64_t)N * 8, stream);
}

extern "C" int64_t sm_linear_dw_se_workspace_bytes(int rows, int nout, int nin) {
  const int s = choose_splits(nout, nin, rows, true);
  return s > 1 ? (int64_t)s * nout * nin * 4 : 16;
}

extern "C" int sm_linear_dw_se(int rows, int nout, int nin, const void* dy, const void* a2, const float* act_mean,
                               const float* act_rstd, const float* act_w, const float* act_b, int act_gelu,
                               const float* gate, int hw, float* dW, int accumulate, void* ws, int64_t ws_bytes,
                               hipStream_t stream) {
  if (nout <= 0 || nin <= 0 || rows <= 0) return 0;
  if (ws_bytes < sm_linear_dw_se_workspace_bytes(rows, nout, nin)) return -4;
  if (nout % 8 || nin % 8 || (((uintptr_t)dy | (uintptr_t)a2) & 15)) return -2;
  if (gate != nullptr && (hw <= 0 || hw % BKT || rows % hw)) return -2;   // no gate: any rows (x = BN(a2))
  if (act_mean == nullptr) return -2;
  const int v = gemm_variant(nout, nin, rows);
  if (v == 1) return -2;
  GemmArgs g{};
  g.M = nout; g.N = nin; g.K = rows; g.A = dy; g.lda = nout; g.B = a2; g.ldb = nin; g.C = dW; g.ldc = nin;
  g.alpha = 1.f; g.beta = accumulate ? 1.f : 0.f; g.rows_per_group = 1;
  g.xb_act = ChanAffine{act_mean, act_rstd, act_w, act_b, act_gelu};
  g.xb_gate = gate; g.xb_hw = gate ? hw : 1;
  int splits = choose_splits(nout, nin, rows, true);
  if (splits > 1) {
    int chunk = (rows + splits - 1) / splits;
    chunk = (chunk + BKT - 1) / BKT * BKT;     // K-steps never straddle a frame (hw % BKT == 0)
    splits = (rows + chunk - 1) / chunk;
    g.k_begin = 0; g.k_chunk = chunk; g.partial = (float*)ws;
  } else {
    g.k_begin = 0; g.k_chunk = rows;
  }
  const int bm = variant_bm(v);
  const dim3 grid(((nin + 127) / 128) * ((nout + bm - 1) / bm) * splits);
  if (v == 2) hipLaunchKernelGGL((gemm_bf16_v2<false, false, float, true, 256, 7>), grid, dim3(512), 0, stream, g);
  else hipLaunchKernelGGL((gemm_bf16_v2<false, false, float, true, 128, 7>), grid, dim3(256), 0, stream, g);
  SM_CHECK_LAUNCH();
  if (splits > 1) {
    const int64_t total = (int64_t)nout * nin;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, stream, g, splits);
    SM_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int sm_linear_dw_bias(int rows, int nout, int nin, const void* dy, const void* x, float* dW, float* db,
                                 int accumulate, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (nout <= 0 || nin <= 0) return 0;
  if (ws_bytes < sm_linear_dw_bias_workspace_bytes(rows, nout, nin)) return -4;
  if (gemm_variant(nout, nin, rows) == 1 || nout % 8 || nin % 8) return -2;   // the row sums live in the v2 kernel
  if (dw_transposed(rows, nout, nin)) {
    // dW^T[nin][nout] = x^T dy (split-K slabs), reduced into dW[nout][nin] through the
    // transposed store; db = column sums of dy by the colsum kernel (the fused row sums
    // follow the A operand, which is x here)
    const int s = dw384_splits(nin, nout, choose_splits(nin, nout, rows, true));
    const int64_t gbytes = (int64_t)s * nout * nin * 4;
    GemmArgs g{};
    g.M = nin; g.N = nout; g.K = rows; g.A = x; g.lda = nin; g.B = dy; g.ldb = nout; g.C = dW; g.ldc = nin;
    g.alpha = 1.f; g.beta = accumulate ? 1.f : 0.f; g.rows_per_group = 1; g.ctrans = 1;
    int chunk = (rows + s - 1) / s;
    chunk = (chunk + BKT - 1) / BKT * BKT;
    const int splits = (rows + chunk - 1) / chunk;
    g.k_begin = 0; g.k_chunk = chunk; g.partial = (float*)ws;
    launch_bf16<false, false, float, true>(g, splits, stream);
    SM_CHECK_LAUNCH();
    const int64_t total = (int64_t)nout * nin;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, stream, g, splits);
    SM_CHECK_LAUNCH();
    void* cws = (void*)(((uintptr_t)ws + gbytes + 255) & ~(uintptr_t)255);
    return sm_colsum(SM_BF16, rows, nout, dy, db, 1, cws, sm_colsum_workspace_bytes(rows, nout), stream);
  }
  const int s = choose_splits(nout, nin, rows, true);
  const int64_t gbytes = s > 1 ? (int64_t)s * nout * nin * 4 : 0;
  float* colsum = (float*)(((uintptr_t)ws + gbytes + 15) & ~(uintptr_t)15);
  return gemm_run(SM_BF16, SM_F32, 1, 1, nout, nin, rows, dy, nout, x, nin, dW, nin, nullptr, 1.f,
                  accumulate ? 1.f : 0.f, 0, nullptr, nullptr, 0.f, 0, nullptr, 1, ws, gbytes, colsum, db, stream);
}
