/* C ABI of libsslmae.so — the MI355X (gfx950) kernels of the video-MAE
 * pretraining step of lzc452/SSL-VIT-VIDEO-ANALYTICS.
 *
 * The reference has no FFI: its path is the Python module API used by
 * src/train_ssl_mae.py:13-16 (tiny_vit_21m_variant, TinyVideoMAE, get_tube_mask,
 * patchify) on stock aten ops.  Each entry point below replaces one aten op (or
 * a fused group of them) on that path; the citation is the reference line whose
 * computation it performs.  The host mirror of the reference API
 * (ssl-vit-video-analytics_amd/ssl_mae_amd) binds these with ctypes.
 *
 * Conventions: raw device pointers, element counts, row strides in ELEMENTS,
 * dtype enum (0 = f32, 1 = bf16), the caller's hipStream_t; kernels never
 * allocate — scratch comes from the caller (`*_workspace_bytes`).  Every
 * function returns 0 on success, a hipError_t (>0) on launch failure, or a
 * negative code: -2 unsupported shape/alignment, -3 unsupported dtype combo,
 * -4 workspace too small.  No exceptions cross the ABI; no host syncs.
 */
#ifndef SM_API_H
#define SM_API_H
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GEMM: every nn.Linear / 1x1 Conv2d and their dX/dW products.
 * Replaces aten::addmm/mm of tiny_vit.py:79,81,93,94 (Mlp, Attention qkv/proj),
 * tiny_vit.py:43,49 (MBConv 1x1 convs), mae_vit_adapter.py:24,53 (enc_to_dec,
 * decoder_pred) and torch TransformerEncoderLayer in_proj/out_proj/linear1/2.
 * C = alpha*op(A)op(B) + bias (+ beta*R, R = C when null); epi bit0 = exact GELU
 * (aux <- pre-activation), bit1 = round the branch to bf16 before adding R (autocast).
 * Branch regularisers of the training step: elementwise dropout (drop_p, counter-hash
 * RNG keyed by seed and the element index, nn.Dropout semantics: keep w.p. 1-p, scale
 * 1/(1-p)) and DropPath (branch *= row_scale[row / rows_per_group]).
 * a_layout 0: A[M][K], 1: A[K][M];  b_layout 0: B[N][K], 1: B[K][N]. */
int64_t sm_gemm_workspace_bytes(int ab_dtype, int M, int N, int K);
int sm_gemm(int ab_dtype, int c_dtype, int a_layout, int b_layout, int M, int N, int K,
            const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
            const float* bias, float alpha, float beta, int epi, void* aux, const void* R,
            float drop_p, uint64_t seed, const float* row_scale, int64_t rows_per_group,
            void* workspace, int64_t ws_bytes, hipStream_t stream);
/* Form of the non-split bf16 GEMMs with a K-major A and a plain bf16 epilogue (every
 * forward / data-gradient Linear of the step): 1 = persistent blocks with each tile's
 * output stores drained under the next tile's K loop (default), 0 = one tile per block.
 * Outputs are bit-identical either way.  mode < 0 only queries.  Returns the previous mode.
 * (= sm_gemm_tuning key 1.) */
int sm_gemm_persistent(int mode);
/* GEMM dispatch tuning for A/B measurement scripts (never changed by the product path):
 * key 0 tile variant (0 = per-shape rule, 1-3 pinned), 1 persistent form on/off,
 * 2 / 3 persistent form's minimum N / maximum K at K > 128, 4 tiles per persistent block
 * (-1 = per-K rule, 0 = fully persistent), 5 / 6 tiles per block at K <= 128 / above,
 * 7 minimum K per block for the v_mfma_f32_16x16x32_bf16 K loop of K-major-A tiles
 * (default 1 << 30 = off: measured neutral), 8 the 384 x 128 pipelined weight-gradient tile
 * (gemm_dw384) for outputs it divides (default 1 = on), 9 keep such outputs untransposed in
 * sm_linear_dw_bias (fused bias gradient; default 1).
 * *prev <- the current value; set > 0 stores value, set < 0 restores the default.
 * Returns 0, or -2 for an unknown key.  Host-side only (no launch). */
int sm_gemm_tuning(int key, int set, int value, int* prev);
/* Weight + bias gradient of y = x W^T + b (Linear / 1x1 conv backward, e.g.
 * tiny_vit.py:74-84 Mlp, mae_vit_adapter.py:40-48 decoder layers): dW[nout][nin]
 * (+)= dy^T x and db[nout] += sum_rows dy in one GEMM pass over dy (bf16 dy, x;
 * fp32 dW, db).  Replaces sm_gemm (dW) followed by sm_colsum (db). */
int64_t sm_linear_dw_bias_workspace_bytes(int rows, int nout, int nin);
int sm_linear_dw_bias(int rows, int nout, int nin, const void* dy, const void* x, float* dW, float* db,
                      int accumulate, void* ws, int64_t ws_bytes, hipStream_t stream);
/* The fc2 data gradient through dropout(GELU(pre)) with the fc2 weight gradient's operand
 * as a side output (Mlp tiny_vit.py:74-84, decoder FF mae_vit_adapter.py:40-48): dx = (dy w)
 * * keep / (1 - p) * GELU'(pre) and h = bf16(GELU(pre) * keep / (1 - p)) (= sm_gelu_fwd(pre))
 * from one epilogue.  dy [M][N], w [N][K], pre / dx / h [M][K] bf16; N, K % 8 == 0. */
int sm_linear_dx_gelu(int M, int N, int K, const void* dy, const void* w, const void* pre, void* dx, void* h,
                      float drop_p, uint64_t seed, hipStream_t stream);
/* fc2's weight gradient with the activation formed in the GEMM's operand loads:
 * dW[nout][nin] (+)= dy^T dropout(GELU(pre)), db += colsum(dy); pre = the fc1
 * pre-activation [rows][nin] bf16, (drop_p, seed) the fc1 output's dropout (the Mlp of
 * tiny_vit.py:74-84, the decoder feed-forward).  Bit-identical to sm_gelu_fwd followed by
 * sm_linear_dw_bias without the recompute pass; workspace as
 * sm_linear_dw_bias_workspace_bytes. */
int sm_linear_dw_bias_gelu(int rows, int nout, int nin, const void* dy, const void* pre, float drop_p,
                           uint64_t seed, float* dW, float* db, int accumulate, void* ws, int64_t ws_bytes,
                           hipStream_t stream);
/* y = x W^T (bf16, no bias) plus the train-mode BatchNorm statistics of y (Conv2d_BN,
 * tiny_vit.py:12-18, of the MBConv expand conv tiny_vit.py:43): the GEMM epilogue sums the
 * stored values per 64-row slab; fixed-order fp64 reduction, mean / rstd and the running
 * statistics update (`updates` times) as sm_bn_stats -- replaces sm_gemm + sm_bn_stats
 * (one read pass of y fewer).  x [M][K], w [N][K] bf16. */
int64_t sm_linear_bn_stats_workspace_bytes(int M, int N);
int sm_linear_bn_stats(int M, int N, int K, const void* x, const void* w, void* y, float* mean, float* rstd,
                       float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum, float eps,
                       int updates, void* ws, int64_t ws_bytes, hipStream_t stream);
/* The MBConv projection's forward over the SE output (tiny_vit.py:29-34, 53): y[rows][nout]
 * bf16 = h3 W^T, h3 = bf16(bf16(act(a2)) * gate[r / hw][c]) formed in the GEMM's operand
 * loads exactly as sm_se_fwd stores it (bit-identical to sm_se_fwd's y + sm_gemm), w
 * [nout][nin] bf16; hw % 128 == 0, nin % 64 == 0, nin <= 1536. */
int sm_linear_se(int rows, int nout, int nin, const void* a2, const void* w, const float* act_mean,
                 const float* act_rstd, const float* act_w, const float* act_b, int act_gelu, const float* gate,
                 int hw, void* y, hipStream_t stream);
/* The MBConv projection's weight gradient over the SE output (tiny_vit.py:29-34, 53,
 * replacing the Conv2d weight-gradient autograd node fed by SELayer.forward's product):
 * dW[nout][nin] (+)= dy^T h3, h3[r][c] = bf16(bf16(act(a2[r][c])) * gate[r / hw][c]),
 * act = BatchNorm(mean, rstd, w, b) + GELU (act_gelu) of the depthwise output a2
 * [rows][nin] bf16, gate [rows / hw][nin] fp32 (the SE sigmoid), dy [rows][nout] bf16,
 * fp32 dW.  h3 is formed in the GEMM's operand loads exactly as sm_se_scale stores it:
 * bit-identical to sm_se_scale + sm_gemm.  hw % 64 == 0. */
/* ---- the stem's BN2 folded into stage 0's first MBConv (tiny_vit.py:62-72 feeding :43;
 * replaces the aten batch_norm output the reference materialises between PatchEmbed and
 * stages[0][0]): y = x W^T with x = bf16(a sc + sh), sc = a_rstd a_w, sh = a_b - a_mean sc,
 * formed in the A-operand loads exactly as sm_bn_apply stores x (bit-identical to
 * sm_bn_apply + sm_gemm / sm_linear_bn_stats).  a [M][K] bf16, K % 8 == 0, K <= 256, w [N][K]
 * bf16, y [M][N] bf16.  _bn_stats: plus the output's train-mode BatchNorm statistics
 * (workspace sm_linear_bn_stats_workspace_bytes). */
int sm_linear_bnin(int M, int N, int K, const void* a, const float* a_mean, const float* a_rstd,
                   const float* a_w, const float* a_b, const void* w, void* y, hipStream_t stream);
int sm_linear_bnin_bn_stats(int M, int N, int K, const void* a, const float* a_mean, const float* a_rstd,
                            const float* a_w, const float* a_b, const void* w, void* y, float* mean,
                            float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                            float momentum, float eps, int updates, void* ws, int64_t ws_bytes,
                            hipStream_t stream);
/* sm_bn_apply whose residual R is stored before its own BatchNorm (r_*): R's value is the
 * BN output bf16(R r_sc + r_sh) exactly as sm_bn_apply stores it (the MBConv residual of
 * stages[0][0] over the stem's BN2, tiny_vit.py:54-56). */
int sm_bn_apply_res_bn(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* mean,
                       const float* rstd, const float* w, const float* b, void* y, int gelu, const void* R,
                       const float* r_mean, const float* r_rstd, const float* r_w, const float* r_b,
                       const float* row_scale, int64_t rows_per_group, hipStream_t st);
/* sm_linear_dw_se with gate == NULL: the B operand is the BatchNorm output act(a2) (act_gelu
 * 0: x = bf16(a2 sc + sh)); rows need not be a multiple of hw. */
int64_t sm_linear_dw_se_workspace_bytes(int rows, int nout, int nin);
int sm_linear_dw_se(int rows, int nout, int nin, const void* dy, const void* a2, const float* act_mean,
                    const float* act_rstd, const float* act_w, const float* act_b, int act_gelu, const float* gate,
                    int hw, float* dW, int accumulate, void* ws, int64_t ws_bytes, hipStream_t stream);

/* ---- fused attention (tiny_vit.py:103 F.scaled_dot_product_attention;
 * torch MultiheadAttention core of the decoder, mae_vit_adapter.py:40-48).
 * qkv packed [N][L][3][H][D] bf16|f32, out O [N][L][H][D], lse [N][H][L]. */
int sm_attn_fwd(int dtype, int N, int L, int H, int D, const void* qkv, void* out, float* lse,
                float scale, float drop_p, uint64_t seed, hipStream_t st);
/* delta_ws: workspace of sm_attn_bwd_workspace_bytes (256-B aligned): rowsum(dO * O)
 * [N][H][L] fp32, then for bf16 the dQ kernel's bf16(Q * scale * log2 e) [N][L][H][D], the
 * operand the dK/dV kernel's scores are formed from (the forward's and dQ's S exactly). */
int64_t sm_attn_bwd_workspace_bytes(int dtype, int N, int L, int H, int D);
int sm_attn_bwd(int dtype, int N, int L, int H, int D, const void* qkv, const void* o,
                const void* dout, const float* lse, float* delta_ws, void* dqkv,
                float scale, float drop_p, uint64_t seed, hipStream_t st);
/* MFMA shape of the bf16 attention backward (A/B and tests; the default is the measured best):
 * key 0 = head dim 64, key 1 = head dim 32; value 32 (v_mfma_f32_32x32x16_bf16) or 16
 * (v_mfma_f32_16x16x32_bf16).  *prev <- the current shape; set > 0 stores value, set < 0
 * restores the default.  Returns 0, or -2 for an unknown key / shape.  Host-side only. */
int sm_attn_tuning(int key, int set, int value, int* prev);

/* ---- LayerNorm (tiny_vit.py:112,115; decoder norm1/norm2; mae_vit_adapter.py:50) */
int sm_layernorm_fwd(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* gamma,
                     const float* beta, void* y, float* mean, float* rstd, float eps, hipStream_t st);
int64_t sm_layernorm_bwd_workspace_bytes(int64_t M, int C);
int sm_layernorm_bwd(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy,
                     const void* x, const float* mean, const float* rstd, const float* gamma,
                     void* dx, const void* dres, float* dgamma, float* dbeta, void* ws,
                     int64_t ws_bytes, hipStream_t st);
/* sm_layernorm_bwd plus the block branch's copy of dx (C = 192 or 384): dxb [M][C] bf16 =
 * bf16(bf16(dx) * row_scale[row / rows_per_group] * keep(row, col) / (1 - drop_p)) with
 * sm_dropout_bwd's mask (row_scale may be null, drop_p 0): the cast / dropout-backward
 * passes over dx that feed the branch's Linear backward (tiny_vit.py:126-128 DropPath,
 * mae_vit_adapter.py:40-48 dropout1) folded into the LayerNorm backward; bit-identical. */
int sm_layernorm_bwd_branch(int x_dtype, int dy_dtype, int dx_dtype, int64_t M, int C, const void* dy,
                            const void* x, const float* mean, const float* rstd, const float* gamma, void* dx,
                            const void* dres, float* dgamma, float* dbeta, void* dxb, float drop_p, uint64_t seed,
                            const float* row_scale, int64_t rows_per_group, void* ws, int64_t ws_bytes,
                            hipStream_t st);

/* ---- BatchNorm2d, train mode (tiny_vit.py:16 Conv2d_BN), channels-last [M][C] */
int64_t sm_bn_workspace_bytes(int64_t M, int C);
int sm_bn_stats(int x_dtype, int64_t M, int C, const void* x, float* mean, float* rstd,
                float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum, float eps,
                int updates, void* ws, int64_t ws_bytes, hipStream_t st);
/* eval mode (running statistics; tiny_vit.py:16 BatchNorm2d under model.eval(),
 * train_finetune.py:127-138 evaluate): mean = run_mean, rstd = 1/sqrt(run_var + eps),
 * the form every BN consumer takes.  sm_bn_stats / sm_bn_bwd process C > 1024
 * (stage-4 MBConv, 1536 channels) in column slices. */
int sm_bn_eval_params(const float* run_mean, const float* run_var, int C, float eps, float* mean, float* rstd,
                      hipStream_t st);
/* statistics from per-block partials [nrows][2][C] written by a fused producer */
int64_t sm_bn_partials_workspace_bytes(int C);
int sm_bn_stats_from_partials(const float* part, int64_t nrows, int C, int64_t M, float* mean, float* rstd,
                              float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum,
                              float eps, int updates, void* ws, int64_t ws_bytes, hipStream_t st);
/* y = R + row_scale[row/rows_per_group] * act(BN(x)) (R / row_scale nullable: MBConv
 * residual with DropPath, tiny_vit.py:53-56) */
int sm_bn_apply(int x_dtype, int y_dtype, int64_t M, int C, const void* x, const float* mean,
                const float* rstd, const float* w, const float* b, void* y, int gelu, const void* R,
                const float* row_scale, int64_t rows_per_group, hipStream_t st);
int sm_bn_bwd(int x_dtype, int g_dtype, int64_t M, int C, const void* dy, const void* x,
              const float* mean, const float* rstd, const float* w, const float* b, int gelu,
              const float* row_scale, int64_t rows_per_group, void* dx, float* dw, float* db, void* ws,
              int64_t ws_bytes, hipStream_t st);

/* ---- elementwise (GELU tiny_vit.py:44,47,68,80; residual adds; casts) */
int sm_gelu_bwd(int pre_dtype, int g_dtype, int64_t n, int ncols, const void* pre, const void* dy, void* dx,
                float drop_p, uint64_t seed, hipStream_t st);
int sm_add(int a_dtype, int o_dtype, int64_t n, const void* a, const void* b, void* o, hipStream_t st);
int sm_cast(int a_dtype, int o_dtype, int64_t n, const void* a, void* o, hipStream_t st);
int sm_fill(float* p, int64_t n, float v, hipStream_t st);
int sm_gelu_fwd(int dtype, int64_t n, int ncols, const void* x, void* y, float drop_p, uint64_t seed,
                hipStream_t st);
/* backward of the branch regularisers: dx = dy * dropout-mask * row_scale[row/rows_per_group]
 * (nn.Dropout of the decoder layers; timm DropPath of tiny_vit.py:52,114) */
int sm_dropout_bwd(int dtype, int64_t n, int ncols, const void* dy, void* dx, float drop_p, uint64_t seed,
                   const float* row_scale, int64_t rows_per_group, hipStream_t st);
/* sm_cast (fp32 -> bf16) and sm_dropout_bwd in one pass: dx_bf16 = bf16(bf16(dy) *
 * row_scale * keep / (1 - p)); the decoder block's fp32 residual-stream gradient entering
 * its bf16 branch (torch.autocast's cast + nn.Dropout backward, mae_vit_adapter.py:40-48). */
int sm_cast_dropout_bwd(int64_t n, int ncols, const float* dy, void* dx_bf16, float drop_p, uint64_t seed,
                        const float* row_scale, int64_t rows_per_group, hipStream_t st);
/* DropPath per-sample keep scales: out[i] = keep ? 1/(1-p) : 0 */
int sm_droppath_scale(int n, float p, uint64_t seed, float* out, hipStream_t st);
/* column sums (Linear bias gradients): out[c] (+)= sum_m x[m][c] */
int64_t sm_colsum_workspace_bytes(int64_t M, int C);
int sm_colsum(int dtype, int64_t M, int C, const void* x, float* out, int accumulate, void* ws,
              int64_t ws_bytes, hipStream_t st);

/* ---- convolutions (PatchEmbed tiny_vit.py:62-72; depthwise 3x3 tiny_vit.py:46)
 * stem im2col folds the frame permute of mae_vit_adapter.py:84 into its loads. */
int sm_stem_im2col(int out_dtype, const float* clip, int B, int T, int H, int W, int64_t sB,
                   int64_t sC, int64_t sT, int64_t sH, int64_t sW, int stride, void* col, hipStream_t st);
int sm_im2col3(int dtype, const void* x, int F, int H, int W, int C, int stride, void* col, hipStream_t st);
int sm_col2im3(int dtype, const void* dcol, int F, int H, int W, int C, int stride, void* dx, hipStream_t st);
int sm_conv_wpack(int out_dtype, const float* src, void* dst, int Cout, int Cin, int Kpad, int order,
                  hipStream_t st);
int sm_conv_wunpack_add(const float* packed, float* grad, int Cout, int Cin, int Kpad, int order,
                        hipStream_t st);
/* Stem conv1 (tiny_vit.py:67: 3 -> 48, 3x3, stride 2, pad 1) straight from the fp32 clip
 * (strides as sm_stem_im2col) on the matrix cores, plus the train-mode BatchNorm statistics
 * of its bf16 output y [B*T*Ho*Wo][48] (tiny_vit.py:68, as sm_linear_bn_stats): replaces
 * sm_stem_im2col + sm_linear_bn_stats (y bit-identical), no [pixels][32] buffer.
 * wpack = sm_conv_wpack order 0 [48][32] bf16. */
int64_t sm_stem_conv1_workspace_bytes(void);
int sm_stem_conv1_bn_stats(const float* clip, int B, int T, int H, int W, int64_t sB, int64_t sC, int64_t sT,
                           int64_t sH, int64_t sW, const void* wpack, void* y, float* mean, float* rstd,
                           float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum, float eps,
                           int updates, void* ws, int64_t ws_bytes, hipStream_t st);
/* Stem conv2 over h1 = act(BN1(a1)) (tiny_vit.py:68-70: BN1 + GELU, 3x3 48 -> 96 stride 1
 * pad 1) plus the train-mode BatchNorm statistics of its bf16 output, one frame per
 * workgroup: BN1 + GELU applied once per element into an LDS ring of h1 rows, so h1 is
 * never written (y bit-identical to sm_bn_apply + sm_conv3x3_fwd).  a1 [F*H*W][48] bf16,
 * wpack = sm_conv_wpack order 1 [96][432] bf16, y [F*H*W][96] bf16, W <= 128; BN1 =
 * (mean, rstd, weight, bias), gelu = act is GELU.  Workspace sm_stem_conv2_workspace_bytes(F). */
int64_t sm_stem_conv2_workspace_bytes(int F);
int sm_stem_conv2_bn_stats(const void* a1, int F, int H, int W, const float* bn1_mean, const float* bn1_rstd,
                           const float* bn1_w, const float* bn1_b, int gelu, const void* wpack, void* y, float* mean,
                           float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked, float momentum,
                           float eps, int updates, void* ws, int64_t ws_bytes, hipStream_t st);
/* Stem conv2 (tiny_vit.py:69, 3x3 / stride 1 / pad 1, bf16, channels-last) as GEMMs over
 * the implicit im2col matrix -- no [pixels][9C] buffer in HBM.  wpack = sm_conv_wpack
 * order 1 ([Cout][9*Cin]); wpack_t = order 2 ([Cin][9*Cout]); Cin, Cout % 8 == 0.
 * fwd: y = conv(x); dgrad: dx = conv^T(dy); wgrad: dw[Cout][9*Cin] (+)= fp32 weight
 * gradient (unpack with sm_conv_wunpack_add order 1). */
int sm_conv3x3_fwd(const void* x, const void* wpack, void* y, int F, int H, int W, int Cin, int Cout, hipStream_t st);
/* conv fwd + the train-mode BatchNorm statistics of y (tiny_vit.py:69-70, the stem's conv2
 * -> BN) from the GEMM epilogue, as sm_linear_bn_stats (workspace =
 * sm_linear_bn_stats_workspace_bytes(F*H*W, Cout)); replaces sm_conv3x3_fwd + sm_bn_stats. */
int sm_conv3x3_fwd_bn_stats(const void* x, const void* wpack, void* y, int F, int H, int W, int Cin, int Cout,
                            float* mean, float* rstd, float* run_mean, float* run_var, int64_t* num_batches_tracked,
                            float momentum, float eps, int updates, void* ws, int64_t ws_bytes, hipStream_t st);
int sm_conv3x3_dgrad(const void* dy, const void* wpack_t, void* dx, int F, int H, int W, int Cin, int Cout,
                     hipStream_t st);
int64_t sm_conv3x3_wgrad_workspace_bytes(int F, int H, int W, int Cin, int Cout);
int sm_conv3x3_wgrad(const void* dy, const void* x, float* dw, int accumulate, int F, int H, int W, int Cin, int Cout,
                     void* ws, int64_t ws_bytes, hipStream_t st);
int sm_dwconv_fwd(int dtype, const void* x, const float* w, void* y, int F, int H, int W, int C,
                  int stride, hipStream_t st);
int64_t sm_dwconv_wgrad_workspace_bytes(int F, int H, int W, int C, int stride);
/* Fused MBConv depthwise path (tiny_vit.py:48-51, bf16): y = dwconv3x3(act(x)) with the
 * producer's BN + GELU folded into the loads (in_mean == NULL: identity) and per-block
 * BN statistics partials of y written to part[sm_dwconv_fused_partial_rows][2][C]
 * (part nullable); backward: dx = dL/d act(x), dw += weight gradient with act(x)
 * recomputed. C % 32 == 0, stride 1 or 2. */
int64_t sm_dwconv_fused_partial_rows(int F, int H, int stride);
int sm_dwconv_fused_fwd(int F, int H, int W, int C, int stride, const void* x, const float* in_mean,
                        const float* in_rstd, const float* in_w, const float* in_b, int in_gelu,
                        const float* w, void* y, float* part, hipStream_t st);
int64_t sm_dwconv_fused_bwd_workspace_bytes(int F, int H, int W, int C, int stride);
int sm_dwconv_fused_bwd(int F, int H, int W, int C, int stride, const void* dy, const void* x,
                        const float* in_mean, const float* in_rstd, const float* in_w, const float* in_b,
                        int in_gelu, const float* w, void* dx, float* dw, void* ws, int64_t ws_bytes,
                        hipStream_t st);
// Stride-1 depthwise conv + BatchNorm(+GELU) backward that never stores the depthwise
// data gradient (one pass over dy forming dw, dz = g GELU' and the BN sums, one
// streaming pass dz -> dx, dx doubling as the dz buffer): dx = dL/dx for y = dwconv3x3(GELU(BN(x))), dw += dL/dw,
// dgamma / dbeta += the BatchNorm's (MBConv conv1 -> act -> conv2, tiny_vit.py:36-56;
// replaces sm_dwconv_fused_bwd + sm_bn_bwd on that path).
int64_t sm_dwconv_bn_bwd_workspace_bytes(int F, int H, int W, int C);
int sm_dwconv_bn_bwd(int F, int H, int W, int C, const void* dy, const void* x, const float* bn_mean,
                     const float* bn_rstd, const float* bn_w, const float* bn_b, int bn_gelu, const float* w,
                     void* dx, float* dw, float* dgamma, float* dbeta, void* ws, int64_t ws_bytes,
                     hipStream_t st);
/* Stride-2 form (the MBConv opening stages 1-3): F, H, W, C are the input's, dy is
 * [F][(H-1)/2+1][(W-1)/2+1][C]; same outputs and workspace (sm_dwconv_bn_bwd_workspace_bytes). */
int sm_dwconv_s2_bn_bwd(int F, int H, int W, int C, const void* dy, const void* x, const float* bn_mean,
                        const float* bn_rstd, const float* bn_w, const float* bn_b, int bn_gelu, const float* w,
                        void* dx, float* dw, float* dgamma, float* dbeta, void* ws, int64_t ws_bytes,
                        hipStream_t st);
int sm_dwconv_bwd(int dtype, const void* dy, const void* x, const float* w, void* dx, float* dw, int F,
                  int H, int W, int C, int stride, void* ws, int64_t ws_bytes, hipStream_t st);

/* ---- SELayer (tiny_vit.py:20-34).  The SE input h = act(x) is recomputed from the
 * pre-BatchNorm tensor x by every kernel that reads it (act = BN2 + GELU of MBConv,
 * tiny_vit.py:50-51; act_mean == NULL: h = x). */
int64_t sm_se_workspace_bytes(int F, int HW, int C);
int sm_se_fwd(int dtype, const void* x, const float* act_mean, const float* act_rstd, const float* act_w,
              const float* act_b, int act_gelu, int F, int HW, int C, int R, const float* w1, const float* w2,
              float* pooled, float* z1, float* s, void* y, void* ws, int64_t ws_bytes, hipStream_t st);
int sm_se_bwd(int dtype, const void* dy, const void* x, const float* act_mean, const float* act_rstd,
              const float* act_w, const float* act_b, int act_gelu, int F, int HW, int C, int R,
              const float* w1, const float* w2, const float* s, const float* z1, float* dz2, float* dz1,
              void* dx, void* ws, int64_t ws_bytes, hipStream_t st);
int sm_se_scale(int dtype, const void* x, const float* act_mean, const float* act_rstd, const float* act_w,
                const float* act_b, int act_gelu, const float* s, void* y, int F, int HW, int C, hipStream_t st);
/* Fused backward of SE(GELU(BN2(x))) -- sm_se_bwd followed by sm_bn_bwd(gelu) on its
 * dx (tiny_vit.py:50-53), in two passes over (dy, x); dh2 is never materialised.
 * dw / db accumulate BN2's weight / bias gradients. */
int64_t sm_se_bn_bwd_workspace_bytes(int F, int HW, int C);
int sm_se_bn_bwd(int dtype, const void* dy, const void* x, const float* bn_mean, const float* bn_rstd,
                 const float* bn_w, const float* bn_b, int bn_gelu, int F, int HW, int C, int R, const float* w1,
                 const float* w2, const float* s, const float* z1, float* dz2, float* dz1, void* dx, float* dw,
                 float* db, void* ws, int64_t ws_bytes, hipStream_t st);

/* ---- MAE glue: tube mask (mae_loader.py:80-90) + masked-token compaction
 * (train_ssl_mae.py:105), pos-embed/mask-token blend (mae_vit_adapter.py:97-104),
 * fused patchify + norm_pix + masked MSE (train_ssl_mae.py:26-31,74-84). */
int sm_tube_mask(const float* noise, int B, int T, int L, int n_mask, uint8_t* mask, int32_t* idx,
                 hipStream_t st);
int sm_pos_blend_fwd(int y_dtype, int x_dtype, const void* y, const float* tpos, const float* spos,
                     const float* tok, const uint8_t* mask, void* x, int B, int T, int L, int D,
                     hipStream_t st);
int sm_pos_blend_bwd(int g_dtype, int y_dtype, const void* dx, const uint8_t* mask, void* dy,
                     float* dtpos, float* dspos, float* dtok, float* ws, int B, int T, int L, int D,
                     hipStream_t st);
int64_t sm_loss_workspace_bytes(int B, int T, int L);
int sm_mae_loss_fwd(int pred_dtype, const void* pred, const float* clip, int64_t sB, int64_t sC,
                    int64_t sT, int64_t sH, int64_t sW, const uint8_t* mask, int B, int T, int H, int W,
                    int norm_pix, float* loss, float* denom, void* ws, int64_t ws_bytes, hipStream_t st);
int sm_mae_loss_bwd(int pred_dtype, const void* pred, const float* clip, int64_t sB, int64_t sC,
                    int64_t sT, int64_t sH, int64_t sW, const uint8_t* mask, int B, int T, int H, int W,
                    int norm_pix, const float* grad_out, const float* denom, void* dpred, hipStream_t st);
int sm_patchify(const float* imgs, int B, int C, int T, int H, int W, int64_t sB, int64_t sC, int64_t sT,
                int64_t sH, int64_t sW, int p, float* out, hipStream_t st);
int sm_unpatchify(const float* tokens, int B, int C, int T, int H, int W, int p, float* imgs, hipStream_t st);
int sm_gather_rows(int dtype, const void* src, const int32_t* idx, int64_t nrows, int C, void* dst,
                   hipStream_t st);
int64_t sm_std_workspace_bytes(void);
int sm_std(int dtype, const void* x, int64_t n, float* out, void* ws, int64_t ws_bytes, hipStream_t st);

/* ---- fine-tune head (BASELINE config 4; src/train_finetune.py:19-40 VideoClassifier):
 * out[g][c] = mean_r x[g][r][c] for x [G][R][C] -- per-frame embedding pooling of the
 * channels-last encoder tokens (F.adaptive_avg_pool2d(feat, 1), mobilevit.py:164-165)
 * and the temporal mean of the fp32 embeddings (feats.mean(dim=1), :38); backward
 * dx[g][r][c] = dy[g][c] / R. */
int sm_segment_mean(int dtype, const void* x, int G, int R, int C, float* out, hipStream_t st);
int sm_segment_mean_bwd(int dtype, const float* dy, int G, int R, int C, void* dx, hipStream_t st);

/* ---- optimizer (train_ssl_mae.py:163 AdamW, :87-89 GradScaler inf-skip) */
int sm_nonfinite(const float* g, int64_t n, int* flag, hipStream_t st);
/* p *= a (data-parallel gradient averaging after a SUM all-reduce) */
int sm_scale(float* p, int64_t n, float a, hipStream_t st);
int sm_adamw(float* p, const float* g, float* m, float* v, void* bf16_shadow, int64_t n, float lr,
             float b1, float b2, float eps, float wd, const int* found_inf, int64_t* step,
             int advance_step, hipStream_t st);

/* ---- federated averaging (src/federated/fed_loop.py:14-62 fedavg_aggregate).
 * out[i] = sum_j client_bufs[j][i] * weights[j], accumulated from +0 in client order
 * with the product and the sum rounded separately (fed_loop.py:46-49, weights[j] =
 * fp32(w_j / total_w)): bit-identical to the reference's CPU loop.  client_bufs is a
 * HOST array of num_clients device pointers (1 <= num_clients <= SM_FEDAVG_MAX_CLIENTS),
 * each holding one client's floating-point state_dict entries flattened in key order.
 * sm_fedavg_counters_max: out[i] = max_j client_counters[j][i] (num_batches_tracked,
 * fed_loop.py:52-55). */
#define SM_FEDAVG_MAX_CLIENTS 32
int sm_fedavg_weighted_sum(int num_clients, const float* const* client_bufs, const float* weights, int64_t n,
                           float* out, hipStream_t st);
int sm_fedavg_counters_max(int num_clients, const int64_t* const* client_counters, int64_t n, int64_t* out,
                           hipStream_t st);

/* ---- clip input pipeline (src/train_ssl_mae.py:137-141 PILToTensor + ConvertImageDtype +
 * Normalize; src/datasets/mae_loader.py:70-77 BGR swap img[[2,1,0]] and [C,T,H,W] stack).
 * frames uint8 [B][T][H][W][3] (decoded RGB) -> out fp32 [B][3][T][H][W],
 * out = (u / 255 - mean[s]) / std[s] with s = 2 - c when bgr_swap (IEEE division,
 * bit-identical to the CPU transform); valid[b] == 0 (nullable) writes a zero clip
 * (mae_loader.py:35-43).  mean3 / std3 are HOST arrays of 3 floats. */
int sm_frames_normalize(const uint8_t* frames, const uint8_t* valid, int B, int T, int H, int W, const float* mean3,
                        const float* std3, int bgr_swap, float* out, hipStream_t st);

/* ---- box calibration (bench.py; csrc/calib.hip): `blocks` workgroups of 4 waves, each wave
 * `iters` x 8 v_mfma_f32_32x32x16_bf16 (shape 32) or the same FLOPs as 16
 * v_mfma_f32_16x16x32_bf16 (shape 16) on random register operands.  stamps [blocks][2] int64:
 * wave 0's s_memtime / s_memrealtime deltas (clock = d_mem / d_real x 100 MHz); sink
 * [blocks * 256] fp32 receives the accumulators.  Returns 0 or -2 (unknown shape). */
int sm_calibrate_mfma(int shape, int iters, int blocks, int64_t* stamps, float* sink, hipStream_t st);

#ifdef __cplusplus
}
#endif
#endif /* SM_API_H */
