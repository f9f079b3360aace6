/* libivit_hip — C ABI of the MI355X-native IntentNetViT hot path (gfx950 / CDNA4).
 *
 * Every entry point is stream-ordered and stateless: buffers are caller-owned device
 * pointers (PyTorch caching allocator on the Python side), sizes are plain integers,
 * the stream is a hipStream_t passed as void*. Return value: 0 on success, <0 for bad
 * arguments (message in ivit_last_error()), >0 for a hipError_t from the launch.
 * dtype selects the compute path: IVIT_F32 (exact f32 MFMA; the parity path) or
 * IVIT_BF16 (bf16 MFMA, f32 accumulation; the throughput path).
 *
 * Each function names the reference interface (file:line under the reference repo) whose
 * arithmetic it implements; the Python host layer mirrors those interfaces.
 */
#ifndef IVIT_H
#define IVIT_H
#ifdef __cplusplus
extern "C" {
#endif

#define IVIT_OK 0
#define IVIT_ERR_ARG (-1)
#define IVIT_ERR_UNSUPPORTED (-2)

#define IVIT_F32 0
#define IVIT_BF16 1

#define IVIT_ACT_NONE 0
#define IVIT_ACT_GELU 1
#define IVIT_ACT_RELU 2
#define IVIT_ACT_GELU_D 3 /* ivit_linear_fwd_panel only: GELU, second output = GELU'(pre-activation) */

/* Tuning knobs (no effect on results; process-wide; defaults from the environment variable named,
 * read once when the library loads):
 *   IVIT_KNOB_WIDE_EPI   (IVIT_WIDE_EPI, default 0): epilogue form of the wide row-panel kernels —
 *                        0 the LDS-tile form for every epilogue, 1 transposed accumulators for the
 *                        Q-prescale and GELU + GELU' outputs, 2 transposed for all;
 *   IVIT_KNOB_CONV_PANEL (IVIT_CONV_PANEL, default 1): 0 runs the stride-1 bf16 convolutions on the
 *                        128 x 128 engine instead of the panel kernels (the tests compare the two). */
#define IVIT_KNOB_WIDE_EPI 0
#define IVIT_KNOB_CONV_PANEL 1
#define IVIT_KNOB_COUNT 2

const char* ivit_version(void);
const char* ivit_last_error(void);
int ivit_set_knob(int knob, int value);
long ivit_get_knob(int knob);

/* ---- Linear layers: timm Attention.qkv/proj, Mlp.fc1/fc2 (reached from model_vit.py:64,71,119)
 *      and the adapters nn.Linear(384,192) (model_vit.py:82-83).                              */
/* Y[M,N] = act(X[M,K] W[N,K]^T + b)  (Ypre: optional pre-activation copy), or, when resid != 0,
 * Y(f32) = resid + row_scale[m / rows_per_scale] * (X W^T + b)   (residual + DropPath, timm Block). */
int ivit_linear_fwd(int dtype, const void* X, long ldx, const void* W, const float* bias, long M, long N, long K,
                    int act, void* Y, long ldy, int y_dtype, void* Ypre, const float* resid, long ldr,
                    const float* row_scale, long rows_per_scale, void* stream);
/* Y = X W^T + bias with columns n < scale_cols multiplied by col_scale (after the bias): the
 * fused qkv projection of timm Attention (attn.qkv, timm Attention.forward) writing its Q block
 * pre-multiplied by log2(e)/sqrt(Dh) for ivit_attn_fwd_q2 / ivit_attn_bwd_q2. */
int ivit_linear_fwd_qs(int dtype, const void* X, long ldx, const void* W, const float* bias, long M, long N, long K,
                       void* Y, long ldy, int y_dtype, long scale_cols, float col_scale, void* stream);
/* dX[M,K] = dY[M,N] W[N,K]  (optionally * gelu'(pre[M,K])). */
int ivit_linear_dgrad(int dtype, const void* dY, long lddy, const void* W, long M, long N, long K, void* dX,
                      long lddx, int dx_dtype, const void* gelu_pre, long ldpre, void* stream);
/* dW[N,K] (+)= dY^T X ; dbias[N] (+)= colsum(dY). f32 outputs; split-K through `work`. */
long ivit_linear_wgrad_workspace(long M, long N, long K);
int ivit_linear_wgrad(int dtype, const void* dY, long lddy, const void* X, long ldx, long M, long N, long K,
                      float* dW, float* dbias, int accumulate, void* work, long work_bytes, void* stream);
/* Residual GEMM + the following LayerNorm in one kernel (timm Block: x1 = x + dp1(proj(.)), then
 * norm2(x1); model_vit.py:64,71 -> timm Block.forward), bf16 operands, N = 384:
 *   X = R + scale[m / rps] * (A W^T + bias)  (f32)   Y = bf16(LN(X; gamma, beta, eps)), mean, rstd [M]
 * W packed by ivit_patch_weight_pack(W f32 [N][K], N, K / 64, ...); K % 64 == 0; scale may be null. */
int ivit_linear_resid_ln_fwd(const void* A, long lda, long M, long N, long K, const void* wpack, const float* bias,
                             const float* R, long ldr, const float* scale, long rps, const float* gamma,
                             const float* beta, float eps, float* X, long ldx, void* Y, long ldy, float* mean,
                             float* rstd, void* stream);

/* Backward twin: the LayerNorm input's dgrad with the LayerNorm backward in the epilogue (timm
 * norm1 / norm2 backward after Attention.qkv / Mlp.fc1 dgrad), N = 384, bf16 dY [M][K]:
 *   G = dY W (W [K][N], packed transposed by ivit_weight_pack_t);  dX = dres + LN_bwd(G; X, gamma,
 *   mean, rstd);  dXs = bf16(dX * scale[m / rps]) if non-null;  dgamma / dbeta (+)= column sums.
 * dX may alias dres; work >= ivit_linear_dgrad_ln_bwd_workspace(M, N). */
long ivit_linear_dgrad_ln_bwd_workspace(long M, long N);
int ivit_linear_dgrad_ln_bwd(const void* dY, long lddy, long M, long N, long K, const void* wpack_t, const float* X,
                             long ldx, const float* gamma, const float* mean, const float* rstd, const float* dres,
                             long ldr, float* dX, long lddx, void* dXs, const float* scale, long rps, float* dgamma,
                             float* dbeta, int accumulate, void* work, long work_bytes, void* stream);
/* Row-panel forms of the wide token GEMMs (bf16, N a multiple of 384, K of 64): each workgroup
 * writes one 144-row x 192-column block (two workgroups per CU) (timm Attention.qkv, Mlp.fc1).
 *   act NONE: Y = (A W^T + bias), columns n < qcols times qscale (qkv with the Q block prescaled)
 *   act GELU: Ypre = A W^T + bias (if non-null), Y = gelu(Ypre)   (W packed by ivit_patch_weight_pack) */
int ivit_linear_fwd_panel(const void* A, long lda, long M, long N, long K, const void* wpack, const float* bias,
                          int act, long qcols, float qscale, void* Y, long ldy, void* Ypre, long ldpre, void* stream);
/*   act GELU_D: Ypre = gelu'(A W^T + bias) (if non-null), Y = gelu(A W^T + bias): the derivative
 *   the backward needs, from the f32 pre-activation, instead of the pre-activation itself.
 * dX[M,N] = (dY[M,K] W[K,N]) * gelu'(pre[M,N])  (Mlp.fc2 dgrad into fc1's pre-activation; W packed
 * transposed by ivit_weight_pack_t), bf16. */
int ivit_linear_dgrad_gelu_panel(const void* dY, long lddy, long M, long N, long K, const void* wpack_t,
                                 const void* pre, long ldpre, void* dX, long lddx, void* stream);
/* dX[M,N] = (dY[M,K] W[K,N]) * G[M,N]  (bf16; G = the GELU' that ivit_linear_fwd_panel wrote with
 * act GELU_D: the same fc2 dgrad with no GELU' evaluation in its epilogue). */
int ivit_linear_dgrad_mul_panel(const void* dY, long lddy, long M, long N, long K, const void* wpack_t, const void* G,
                                long ldg, void* dX, long lddx, void* stream);
/* The weight and bias gradients of one timm Block's four linears (Mlp.fc2, Mlp.fc1, Attention.proj,
 * Attention.qkv; model_vit.py:64,71 -> timm Block backward) in one grouped launch + one reduce:
 *   dW_g = dY_g^T X_g (f32 [N][K]), db_g = colsum(dY_g) (f32 [N], may be null), bf16 token-major
 *   operands [M][*], for (dY, X) = (dy2 [M][D], a [M][Hd]), (dh [M][Hd], x2 [M][D]),
 *   (dyp [M][D], o [M][D]), (dyq [M][3D], x1 [M][D]). D = 384, Hd % 384 == 0, operands 16-B aligned. */
long ivit_vit_block_wgrad_workspace(long M, long D, long Hd);
int ivit_vit_block_wgrad(long M, long D, long Hd, const void* dy2, const void* a, const void* dh, const void* x2,
                         const void* dyp, const void* o, const void* dyq, const void* x1, float* dw2, float* db2,
                         float* dw1, float* db1, float* dwp, float* dbp, float* dwq, float* dbq, void* work,
                         long work_bytes, void* stream);
/* W [K][N] f32 -> the row-panel packed bf16 layout of W^T (ivit_patch_weight_pack_bytes(N, K / 64) bytes). */
int ivit_weight_pack_t(const float* w, long K, long N, void* wpack, void* stream);
/* Many packs in one launch: jobs = device array of n records {const float* w; void* wpack; long rows;
 * long cols; int transposed (+4 pad)} (40 B each); transposed 0 = ivit_patch_weight_pack(w, rows,
 * cols / 64), 1 = ivit_weight_pack_t(w, rows, cols); max_rows_cols >= every rows * cols. */
int ivit_weight_pack_multi(long n, const void* jobs, long max_rows_cols, void* stream);
/* ---- timm PatchEmbed (Conv2d k=s=8) + CLS concat + pos_embed (model_vit.py:64,71 → timm). */
int ivit_patch_embed_fwd(int dtype, const float* img, long B, long C, long H, long W, const void* Wt,
                         const float* bias, const float* pos, const float* cls, long D, float* out, void* stream);
long ivit_patch_embed_wgrad_workspace(long B, long C, long H, long W, long D);
int ivit_patch_embed_wgrad(int dtype, const void* dtok, const float* img, long B, long C, long H, long W, long D,
                           float* dW, float* dbias, float* dpos, float* dcls, int accumulate, void* work,
                           long work_bytes, void* stream);
/* bf16 throughput path of the same PatchEmbed: one coalesced pass over the f32 raster writes the
 * bf16 patch matrix cols[b*Np + gy*Wp + gx][(c*8 + ky)*8 + kx] = img[b][c][8gy+ky][8gx+kx]
 * (full 128-B rows per (patch, channel)); the forward and the weight gradient then stream it
 * as dense GEMM operands by LDS-DMA instead of re-gathering the raster. Same outputs and
 * workspace as ivit_patch_embed_fwd / _wgrad with dtype IVIT_BF16.                          */
int ivit_patch_im2col(const float* img, long B, long C, long H, long W, void* cols, void* stream);
int ivit_patch_embed_fwd_cols(const void* cols, long B, long C, long H, long W, const void* Wt, const float* bias,
                              const float* pos, const float* cls, long D, float* out, void* stream);
int ivit_patch_embed_wgrad_cols(const void* dtok, const void* cols, long B, long C, long H, long W, long D,
                                float* dW, float* dbias, float* dpos, float* dcls, int accumulate, void* work,
                                long work_bytes, void* stream);
/* Fused bf16 forward of the same PatchEmbed: the f32 raster streams through LDS once (converted to
 * bf16 in the operand read), every workgroup computing all D columns of 144 patches; no patch
 * matrix. The weight is first packed (once per weight version) into MFMA fragment order:
 * wpack = ivit_patch_weight_pack_bytes(D, C) bytes, from W [D][C][8][8] f32. D = 384 or 192;
 * img and wpack 16-byte aligned. Same output as ivit_patch_embed_fwd with dtype IVIT_BF16. */
long ivit_patch_weight_pack_bytes(long D, long C);
int ivit_patch_weight_pack(const float* w, long D, long C, void* wpack, void* stream);
int ivit_patch_embed_fwd_packed(const float* img, long B, long C, long H, long W, const void* wpack,
                                const float* bias, const float* pos, const float* cls, long D, float* out,
                                void* stream);

/* ---- Differing patch grids (model_vit.py:64,71 with e.g. vit_small_patch16_224 for one stream,
 *      and the bilinear re-grid of model_vit.py:139).
 * PatchEmbed with patch P != 8 = patch matrix + ivit_linear_fwd + token assembly:
 *   cols[b*Np + gy*Wp + gx][(c*P + ky)*P + kx] = img[b][c][gy*P + ky][gx*P + kx]  (cols_dtype)
 *   out[b][0] = cls + pos[0];  out[b][1 + p] = Y[b*Np + p] + pos[1 + p]           (f32)
 * tokens_bwd: dY[b*Np + p] = dtok[b][1 + p] (dy_dtype, the weight gradient's operand);
 *   dpos (+)= sum_b dtok[b];  dcls (+)= sum_b dtok[b][0].                                    */
int ivit_patch_im2col_p(const float* img, long B, long C, long H, long W, long P, void* cols, int cols_dtype,
                        void* stream);
int ivit_patch_tokens(const float* Y, long B, long Np, long D, const float* pos, const float* cls, float* out,
                      void* stream);
int ivit_patch_tokens_bwd(const void* dtok, int dtok_dtype, long B, long Np, long D, void* dY, int dy_dtype,
                          float* dpos, float* dcls, int accumulate, void* stream);
/* F.interpolate(x, size=(Ho, Wo), mode='bilinear', align_corners=False) on Z = B*C planes of
 * Hi x Wi f32 (ATen's linear taps: src = max((o + 0.5) * in/out - 0.5, 0)), and its adjoint
 * dX = R_h^T dY R_w as a gather (deterministic, no atomics; dX is overwritten).             */
int ivit_bilinear_fwd(const float* X, long Z, long Hi, long Wi, float* Y, long Ho, long Wo, void* stream);
int ivit_bilinear_bwd(const float* dY, long Z, long Hi, long Wi, long Ho, long Wo, float* dX, void* stream);

/* ---- k x k stride-1 "same" convolution on NHWC maps (BasicBlock conv3x3/conv1x1,
 *      model_vit.py:12-17; DetectionHead/IntentionHead conv, heads.py:16,37; k = 5: model_cnn.py:7-9).
 *      Weights packed [Cout][k][k][Cin] (see ivit_pack_conv_weight).                           */
int ivit_conv_fwd(int dtype, const void* X, long B, long H, long W, long Cin, const void* Wp, const float* bias,
                  long Cout, long ks, void* Y, long ldy, int y_dtype, void* stream);
int ivit_conv_dgrad(int dtype, const void* dY, long lddy, long B, long H, long W, long Cout, const void* Wp,
                    long Cin, long ks, void* dX, int dx_dtype, void* stream);
long ivit_conv_wgrad_workspace(long B, long H, long W, long Cin, long Cout, long ks);
int ivit_conv_wgrad(int dtype, const void* dY, long lddy, const void* X, long B, long H, long W, long Cin,
                    long Cout, long ks, float* dWp, float* dbias, int accumulate, void* work, long work_bytes,
                    void* stream);
/* Data gradient on the transposed, tap-flipped pack of ivit_pack_conv_weight_t (bf16; the 288 x 256
 * panel kernel: Cout % 64 == 0, Cin % 8 == 0, B*H*W >= 288); same sums as ivit_conv_dgrad. */
int ivit_conv_dgrad_t(int dtype, const void* dY, long lddy, long B, long H, long W, long Cout, const void* WpT,
                      long Cin, long ks, void* dX, int dx_dtype, void* stream);
/* Convolution + the following BatchNorm2d's training-mode batch statistics in one pass (BasicBlock
 * conv -> bn, model_vit.py:24-27,35-43): Y = conv(X, Wp) (no bias, dense: ldy == Cout) and mean /
 * invstd (biased variance, eps) of Y's channels, running mean / var updated with momentum (unbiased
 * variance) as ivit_bn_stats. bf16 panel shapes fold the statistics into the convolution's epilogue
 * (per-tile sums and centred squares, merged across tiles in a fixed order); other shapes run
 * ivit_conv_fwd + ivit_bn_stats. */
long ivit_conv_bn_fwd_workspace(long B, long H, long W, long Cout);
int ivit_conv_bn_fwd(int dtype, const void* X, long B, long H, long W, long Cin, const void* Wp, long Cout, long ks,
                     void* Y, long ldy, int y_dtype, float* mean, float* invstd, float* run_mean, float* run_var,
                     float momentum, float eps, void* work, long work_bytes, void* stream);
/* torch [Cout][Cin][k][k] f32  ->  [Cin][k][k][Cout_pad] (dtype) with the taps flipped: the K-contiguous
 * weight of the data gradient, WpT[ci][ky][kx][co] = w[co][ci][k-1-ky][k-1-kx], zero for co >= Cout
 * (the pack for a gradient zero-padded to Cout_pad channels). */
int ivit_pack_conv_weight_t(int dtype, const float* w, long Cout, long Cin, long ks, long Cout_pad, void* out,
                            void* stream);
/* torch [Cout][Cin][k][k] f32  ->  packed [Cout_pad][k][k][Cin] (dtype), rows >= Cout zeroed. */
int ivit_pack_conv_weight(int dtype, const float* w, long Cout, long Cin, long ks, long Cout_pad, void* out,
                          void* stream);
/* packed f32 gradient [Cout_pad][k][k][Cin] -> torch layout [Cout][Cin][k][k] (+= if accumulate). */
int ivit_unpack_conv_grad(const float* gp, long Cout, long Cin, long ks, float* out, int accumulate, void* stream);

/* ---- Multi-head self-attention core: timm Attention -> F.scaled_dot_product_attention
 *      (softmax(Q K^T / sqrt(Dh)) V, no mask, no dropout). qkv: [B, N, 3, H, Dh] rows of 3*H*Dh;
 *      out: [B, N, H*Dh]; lse: [B, H, N] f32 (natural-log-sum-exp of the scaled scores).
 *      IVIT_BF16 is flash-style (no N x N buffer: the workspace holds the backward's row
 *      constants and a prescaled Q copy). IVIT_F32, the exact parity path, materialises the scores:
 *      its workspace is 4 B*H*N*ldS bytes (ldS >= N; twice that for the backward) — 0.49 GB per
 *      sample at N = 4501, H = 6, and 7.8 GB at N = 18 001: sized for the parity tests and
 *      config 1 (B = 1), not for training at scale.                                           */
long ivit_attn_workspace(int dtype, long B, long N, long H, long Dh, int backward);
int ivit_attn_fwd(int dtype, const void* qkv, long B, long N, long H, long Dh, void* out, float* lse, void* work,
                  long work_bytes, void* stream);
int ivit_attn_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, long B, long N,
                  long H, long Dh, void* dqkv, void* work, long work_bytes, void* stream);
/* bf16 path with the Q block of qkv pre-multiplied by log2(e)/sqrt(Dh) (ivit_linear_fwd_qs):
 * the kernels take exp2 of the raw MFMA output (the running max / -lse as the initial
 * accumulator), no per-score scaling. Same outputs as ivit_attn_fwd / ivit_attn_bwd with dtype
 * IVIT_BF16 on the unscaled q; dqkv is the gradient w.r.t. the UNSCALED q, k, v.            */
int ivit_attn_fwd_q2(const void* qkv, long B, long N, long H, long Dh, void* out, float* lse, void* work,
                     long work_bytes, void* stream);
int ivit_attn_bwd_q2(const void* qkv, const void* out, const void* dout, const float* lse, long B, long N, long H,
                     long Dh, void* dqkv, void* work, long work_bytes, void* stream);

/* ---- Kernel execution timing (bench.py's roofline figure; no reference counterpart).
 * While armed, ivit_attn_fwd_q2 / ivit_attn_bwd_q2 launch through hipExtLaunchKernel with a
 * start / stop event pair bound to the kernel itself: HIP stamps them at the kernel's own begin
 * and end, not at submission, so kernels of a concurrent stream queued ahead of it do not count
 * (the same interval rocprofv3 --kernel-trace reports). arm(1) clears the records and starts
 * recording, arm(0) stops; read() waits for the recorded events of one tag and returns their
 * launch count and, for the first min(count, cap), each kernel's start / stop in ms relative to
 * the first recorded launch's start (a common origin for all tags, so intervals of kernels on
 * concurrent streams can be merged).                                                          */
enum { IVIT_KT_ATTN_FWD = 0, IVIT_KT_ATTN_BWD_DQ = 1, IVIT_KT_ATTN_BWD_DKV = 2, IVIT_KT_NTAGS = 3 };
int ivit_ktime_arm(int on);
int ivit_ktime_read(int tag, double* start_ms, double* stop_ms, long cap, long* count);

/* ---- Diagnostic per-workgroup stamps (no reference counterpart; tools/panel_stamps.py).
 * buf (device, 8 x u64 per workgroup, cap u64 in all) non-null: the row-panel kernels
 * (ivit_linear_fwd_panel, ivit_linear_dgrad_gelu_panel, ivit_linear_resid_ln_fwd,
 * ivit_linear_dgrad_ln_bwd) launch their stamping builds and write, per workgroup b at
 * buf[8 b ..]: shader clock at entry, at the first K stage's data ready, after the main loop,
 * at exit; 100-MHz real time at entry and exit; HW_ID | XCC_ID << 32; 0. Null: off (default).  */
int ivit_debug_stamps(void* buf, long cap);

/* ---- LayerNorm over the last dim D (timm norm1/norm2/norm eps 1e-6; adapters eps 1e-5).
 *      Input rows r -> (r / rpb) * rstride + roff + r % rpb (rpb = 0: identity) of X (f32).    */
int ivit_layernorm_fwd(const float* X, long ldx, long rpb, long rstride, long roff, long M, long D,
                       const float* gamma, const float* beta, float eps, void* Y, long ldy, int y_dtype,
                       float* mean, float* rstd, void* stream);
/* dX(f32) = dres + LN_bwd(dY);  dXs = dtype(dX * row_scale[m / rows_per_scale]) if non-null;
 * dgamma/dbeta (+)= column sums. work >= ivit_layernorm_bwd_workspace(M, D). dX may alias dres.
 * X, dres and dX use the row map; dY (lddy) and dXs ([M, D] contiguous) use plain rows.      */
long ivit_layernorm_bwd_workspace(long M, long D);
int ivit_layernorm_bwd(const float* X, long ldx, long rpb, long rstride, long roff, long M, long D,
                       const float* gamma, const float* mean, const float* rstd, const void* dY, long lddy,
                       int dy_dtype, const float* dres, float* dX, long lddx, void* dXs, int dxs_dtype,
                       const float* row_scale, long rows_per_scale, float* dgamma, float* dbeta, int accumulate,
                       void* work, long work_bytes, void* stream);

/* ---- BatchNorm2d (train: batch statistics, biased var for normalisation, unbiased for the
 *      running update, momentum 0.1, eps 1e-5) on NHWC [M, C] maps (model_vit.py:24-31). */
long ivit_bn_workspace(long M, long C);
int ivit_bn_stats(const void* X, int x_dtype, long M, long C, float* mean, float* invstd, float* run_mean,
                  float* run_var, float momentum, float eps, void* work, long work_bytes, void* stream);
/* Y = [relu]( (X - mean) * invstd * g + b  [+ R] ), Y/R in y_dtype. */
/* eval-mode statistics of nn.BatchNorm2d (model_vit.py:19-34 in eval): mean = running_mean,
 * invstd = rsqrt(running_var + eps), as torch computes them on the device. */
int ivit_bn_eval_stats(const float* run_mean, const float* run_var, long C, float eps, float* mean, float* invstd,
                       void* stream);
int ivit_bn_apply(const void* X, int x_dtype, long M, long C, const float* mean, const float* invstd,
                  const float* g, const float* b, const void* R, int relu, void* Y, int y_dtype, void* stream);
/* Backward of Y = relu?(BN(X) + R): dYin masked by (Y > 0) if relu; dR = masked dY;
 * dX = invstd*g*(dy - mean(dy) - xhat*mean(dy*xhat)); dg, db (+)= sums. */
int ivit_bn_bwd(const void* X, int x_dtype, const void* Y, int y_dtype, const void* dY, int dy_dtype, long M, long C,
                const float* mean, const float* invstd, const float* g, int relu, void* dX, int dx_dtype, void* dR,
                float* dg, float* db, int accumulate, void* work, long work_bytes, void* stream);

/* ---- Small kernels: casts, column sums, token scatter, AdamW ---------------------------- */
int ivit_cast(const void* x, int x_dtype, void* y, int y_dtype, long n, void* stream);
/* out = (a [+ b]) [* gelu'(pre)] [* row_scale[i / (cols * rows_per_scale)]] elementwise over n values. */
int ivit_add_act_grad(const void* a, int a_dtype, const void* b, int b_dtype, const void* pre, int pre_dtype,
                      const float* row_scale, long row_elems, void* out, int out_dtype, long n, void* stream);
/* Standalone activation modules (nn.GELU exact-erf / nn.ReLU used outside the fused GEMM
 * epilogues, e.g. a caller running adapter_lidar[2] on its own): y = act(x); dx = dy * act'(x). */
int ivit_act_fwd(int act, const void* x, int x_dtype, void* y, int y_dtype, long n, void* stream);
int ivit_act_bwd(int act, const void* dy, int dy_dtype, const void* x, int x_dtype, void* dx, int dx_dtype, long n,
                 void* stream);
int ivit_colsum(const void* X, int x_dtype, long ld, long rpb, long rstride, long roff, long M, long N, float* out,
                int accumulate, void* work, long work_bytes, void* stream);
long ivit_colsum_workspace(long M, long N);
/* Adapter output tokens [B*Np, C] -> slice [.., coff:coff+C] of an NHWC map with ld channels. */
int ivit_copy_cols(const void* src, long lds, void* dst, long ldd, long rows, long cols, int dtype, void* stream);
/* Head output [M, ldh] (det A*7 cols, then intent A*K cols) -> cls [M*A], box [M*A, 6], intent [M*A, K]. */
int ivit_split_heads(const float* h, long ldh, long M, long A, long K, float* cls, float* box, float* intent,
                     void* stream);
int ivit_merge_heads_grad(const float* dcls, const float* dbox, const float* dint, long M, long A, long K,
                          void* dh, long ldh, int dh_dtype, void* stream);
/* torch.optim.AdamW (foreach semantics) over n_tensors tensors given by device pointer tables. */
int ivit_adamw(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
               void* const* exp_avg_sq, const long* sizes, long max_size, float lr, float beta1, float beta2,
               float eps, float weight_decay, float bc1, float bc2_sqrt, void* stream);
/* Same update, and shadows[t] (bf16, may be null per tensor) receives bf16(p_new): the
 * compute-dtype copies the next forward reads (replaces one cast launch per weight per step). */
int ivit_adamw_shadow(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                      void* const* exp_avg_sq, void* const* shadows, const long* sizes, long max_size, float lr,
                      float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2_sqrt,
                      void* stream);
/* Same update (shadows may be null, or null per tensor) with the non-finite-loss guard of
 * train_vit.py:163-165 / loss.py:190-198 without a host sync: finite (device f32, may be null) = 0
 * skips the whole update. steps_in / steps_out (device f32 [n_tensors], both null or both set,
 * distinct): per-tensor step counts before / after; when set, bc1 / bc2_sqrt are ignored and come
 * from steps_in[t] + 1 in f64 with beta1 / beta2, and a skipped update does not advance the count
 * (torch.optim.AdamW's state['step'] when the reference's disconnected zero loss leaves no grad). */
int ivit_adamw_guarded(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                       void* const* exp_avg_sq, void* const* shadows, const long* sizes, long max_size, float lr,
                       double beta1, double beta2, float eps, float weight_decay, float bc1, float bc2_sqrt,
                       const float* finite, const float* steps_in, float* steps_out, void* stream);
/* ivit_adamw_guarded's update over a flat chunk list: chunks (device int32 [n_chunks][2]) =
 * (tensor t, chunk c) for every c < ceil(sizes[t] / ivit_adamw_chunk_elems()) of every tensor; one
 * workgroup per chunk (no idle workgroups for the small tensors), 16-B accesses where the arrays
 * allow. shadows may be null or hold null entries. Bit-identical to ivit_adamw_guarded. */
long ivit_adamw_chunk_elems(void);
int ivit_adamw_chunked(long n_tensors, void* const* params, void* const* grads, void* const* exp_avg,
                       void* const* exp_avg_sq, void* const* shadows, const long* sizes, const int* chunks,
                       long n_chunks, float lr, double beta1, double beta2, float eps, float weight_decay, float bc1,
                       float bc2_sqrt, const float* finite, const float* steps_in, float* steps_out, void* stream);

/* ---- Detection / intention loss (loss.py:58-206): assignment + focal + Smooth-L1 + CE. ----- */
/* gt: [B, Gmax, 5] f32 padded, ngt[B] int32, gint[B, Gmax] int32. keep: [B, NA] f32 0/1 (dominant
 * intent keep mask) or null. stats (f32[8]): focal_sum, box_sum, ce_sum, num_pos, keep_sum, loss,
 * cls_loss, box_loss, intent_loss (written). The workspace starts with the per-anchor targets,
 * int32 [B, NA]: (cls target + 1) | (intent target + 1) << 2 (cls -1 = ignored, intent -1 = none). */
long ivit_det_loss_workspace(long B, long NA, long Gmax);
int ivit_det_loss_fwd(const float* cls, const float* box, const float* intent, const float* anchors, long B,
                      long NA, long K, const float* gt, const int* ngt, const int* gint, long Gmax,
                      const float* keep, unsigned dominant_mask, int downsampling, const float* class_w,
                      float pos_thr, float neg_thr, float alpha, float gamma, float beta, float w_cls,
                      float w_box, float w_int, int use_rotated, float* stats, void* work, long work_bytes,
                      void* stream);
int ivit_det_loss_bwd(const float* cls, const float* box, const float* intent, long B, long NA, long K,
                      const float* keep, unsigned dominant_mask, int downsampling, const float* class_w,
                      float alpha, float gamma, float beta, float w_cls, float w_box, float w_int,
                      const float* stats, const float* grad_loss, float* dcls, float* dbox, float* dintent,
                      void* work, long work_bytes, void* stream);

/* ---- Geometry (utils.py) ----------------------------------------------------------------- */
int ivit_generate_anchors(long bev_h, long bev_w, long stride, const float* cfgs, long A, float voxel, float off_x,
                          float off_y, float* out, void* stream);
int ivit_axis_iou(const float* b1, long n1, const float* b2, long n2, float* out, void* stream);
int ivit_rotated_iou(const float* b1, long n1, const float* b2, long n2, float* out, void* stream);
int ivit_decode_boxes(const float* rel, const float* anchors, const long* idx, long n, float* out, void* stream);
/* torchvision CPU nms semantics, bit-exact: keep (int64, score order), count (int64[1]). */
long ivit_nms_workspace(long n);
int ivit_nms(const float* boxes_xywha, const float* scores, long n, double iou_thr, long* keep, long* count,
             void* work, long work_bytes, void* stream);

/* ---- Detection mAP / intention matching (eval_vit.py:191-292, calculate_ap utils.py:564-575;
 * SURVEY.md §8f rank 2). Sample s: iou rows = its predictions in score order (descending,
 * stable), columns = its GTs: [npred[s], ngt[s]] f32 at iou + iou_off[s]; its predictions occupy
 * pred_off[s] .. pred_off[s] + npred[s] - 1 of the [total_pred] outputs. Per (sample, threshold):
 * ap[s * n_thr + t] (f64) with the reference's empty-set rules; tp[t * total_pred + p] (u8) the
 * greedy TP flags; best_gt[p] (int32) the first-max GT of each prediction (intention pairs are
 * the TPs at 0.5). work >= 8 * n_thr * total_pred bytes; max_gt <= 4096.                     */
int ivit_det_match(const float* iou, const long* iou_off, const int* npred, const int* ngt, const long* pred_off,
                   long n_samples, long total_pred, const float* thresholds, long n_thr, double* ap, int* best_gt,
                   unsigned char* tp, void* work, long work_bytes, int max_gt, void* stream);

/* ---- LiDAR BEV voxelisation ----------------------------------------
 * Replaces utils.create_intentnet_lidar_bev (utils.py:62-106) and, when sweep_tf is given, the
 * per-sweep transform_points(pts, rel_tf) of dataset.py:319-340 (utils.py:27-33) in one pass.
 * points: [P, ld] f32 (points_f64 = 0) or f64 rows, x y z in columns 0..2; intensity: [P] f32.
 * Sweep s owns rows sweep_start[s] .. sweep_start[s+1]-1 (int64 prefix offsets, n_sweeps + 1);
 * max_points >= the largest sweep. sweep_tf: [n_sweeps, 4, 4] f64 row-major or null (points
 * already in the current ego frame). Sweep s scatters into planes sweep_plane[s] ..
 * sweep_plane[s] + height_channels - 1 of bev ([planes, H, W] f32), which the caller zero-fills
 * (np.zeros in the reference): bev[c, floor(off_y - x/voxel), floor(off_x + y/voxel)] =
 * max(bev, intensity) for z in [z_min, z_max), c = clip(floor((z - z_min)/z_range * C)).
 * z_range = z_max - z_min as the caller computes it (constants.py). f64 binning, bit-exact. */
int ivit_lidar_bev(const void* points, int points_f64, long ld, const float* intensity, const long* sweep_start,
                   long n_sweeps, long max_points, const double* sweep_tf, const int* sweep_plane, float* bev,
                   long H, long W, long height_channels, double voxel, double off_x, double off_y, double z_min,
                   double z_max, double z_range, void* stream);

/* Batched NMS (eval_vit.py:170 for every sample of a batch, one launch per stage): sample s
 * owns rows seg[s] .. seg[s+1]-1 (int64 device offsets) of boxes / scores / keep and the mask
 * words mask_off[s] .. + n_s * ceil(n_s / 64); keep receives LOCAL kept indices in score order,
 * count[s] their number; the score order is a stable descending radix sort (one workgroup per
 * sample). n_s <= 131072. work >= ivit_nms_batched_workspace(n_samples, total, mask_words) bytes. */
long ivit_nms_batched_workspace(long n_samples, long total, long mask_words);
int ivit_nms_batched(const float* boxes_xywha, const float* scores, const long* seg, const long* mask_off,
                     long n_samples, long total, long max_n, long mask_words, double iou_thr, long* keep,
                     long* count, void* work, long work_bytes, void* stream);

/* Eval post-processing of a batch (replaces the per-sample loop of eval_vit.py:156-176: sigmoid,
 * torch.where(score >= CONFIDENCE_THRESHOLD), decode_box_predictions utils.py:227-257, apply_nms
 * utils.py:259-274, argmax of the intention logits) with no host round trip. cls [B, NA] f32
 * logits, box_rel [B, NA, 6], intent [B, NA, K], anchors [NA, 5]; NA <= 131072. Sample s's kept
 * detections, in NMS (descending score) order, go to rows s*NA .. s*NA + out_count[s] - 1 of
 * out_scores [B, NA], out_boxes [B, NA, 5] (decoded xywha) and out_intent [B, NA] (int64);
 * out_count [B] int64 is the one value the caller reads back. Scores are torch's f32 GPU sigmoid,
 * boxes ivit_decode_boxes', keep order torchvision CPU nms's (bit-exact).
 * work >= ivit_eval_post_workspace(B, NA) bytes.                                               */
long ivit_eval_post_workspace(long B, long NA);
int ivit_eval_post(const float* cls, const float* box_rel, const float* intent, const float* anchors, long B, long NA,
                   long K, float conf_thr, double iou_thr, float* out_scores, float* out_boxes, long* out_intent,
                   long* out_count, void* work, long work_bytes, void* stream);

/* ---- BEV augmentation passes ----------------------------------------
 * Replaces the raster side of utils.augment_bev (utils.py:500-517): random_flip_bev's np.flip
 * (:399-401), random_rotate_bev's per-channel cv2.warpAffine (:425-438), random_scale_bev's
 * per-channel cv2.resize + centre crop / pad (:455-474) and random_bev_dropout's rectangles
 * (:483-493). passes: device array of n_passes ivit_bev_pass entries (192 B each); entry i reads
 * the [C, H, W] f32 stack at src and writes the one at dst (distinct buffers). All stacks share
 * H x W; max_planes >= every entry's C (C = 0 skips the entry). The caller draws the random
 * parameters (python `random`, the reference's order) and chains passes: flip is fused into
 * the first pass's reads, the dropout rectangles into the last pass's writes.               */
typedef struct ivit_bev_pass {
  unsigned long long src, dst; /* device addresses of plane 0; plane stride H * W floats */
  int C;                       /* planes (0 = skip) */
  int op;                      /* 0 copy, 1 warpAffine INTER_LINEAR / BORDER_CONSTANT 0, 2 resize + crop / pad */
  int flip;                    /* read source columns mirrored (np.flip(axis=2) fused) */
  int n_rect;                  /* dropout rectangles zeroed in the output, 0..5 */
  double m[6];                 /* op 1: the INVERTED 2x3 map dst -> src, as warpAffine inverts M */
  double scale_x, scale_y;     /* op 2: 1 / (new_w / W), 1 / (new_h / H) */
  int new_w, new_h;            /* op 2: resized size (int(W s), int(H s)) */
  int off_x, off_y;            /* op 2: out(y, x) = resized(y + off_y, x + off_x), zero outside */
  int rect[5][4];              /* y0, x0, h, w */
} ivit_bev_pass;
int ivit_bev_augment(const void* passes, long n_passes, long H, long W, long max_planes, void* stream);

/* HD-map rasterisation (utils.py:108-182 rasterize_map_ego_centric):
 * cv2.polylines / cv2.fillPoly (LINE_8, 1 px, shift 0, colour 1) into zero-filled f32 planes.
 * seg [n_seg, 5] int32 (x0, y0, x1, y1, plane bitmask): open-polyline segments AND polygon
 * edges (fillPoly draws every edge with cv::Line); seg_base [n_seg] int64 element offset of the
 * segment's [planes, H, W] image. edges [*, 4] int64 (y0, y1, x_top << 16, dx << 16 truncated)
 * of the non-horizontal polygon edges; polys [n_polys, 3] int32 (first edge, edge count <=
 * max_edges <= 256, plane bitmask), poly_base [n_polys] int64; rows [n_rows, 2] int32
 * (polygon, scanline y) fill work items (polygons with >= 2 edges, y0_min <= y < min(y1_max, H)).
 * Replaces utils.py:148-182's per-lane cv2 calls. */
int ivit_map_raster(const int* seg, long n_seg, const long* seg_base, const long* edges, const int* polys,
                    long n_polys, const long* poly_base, const int* rows, long n_rows, long max_edges, long H, long W,
                    float* out, void* stream);

/* ---- Strided convolutions of the CNN variant (model_cnn.py:7-12, 14-33, 86-100; SURVEY.md
 * §8f rank 4) as im2col + the dense GEMMs above. X: NHWC [B, H, W, C] (f32 or bf16); cols:
 * [B*Ho*Wo, ldc] row (b, oy, ox), column (ky*k + kx)*C + c = X[b, oy*s - pad + ky,
 * ox*s - pad + kx, c] (0 outside the map and in columns k*k*C .. ldc-1), i.e. the
 * [Cout][k][k][Cin] packed weight viewed [Cout, k*k*C] is the GEMM operand; Ho, Wo follow
 * nn.Conv2d (floor((H + 2 pad - k) / s) + 1). col2im (C <= 512) is the adjoint as a gather: dX (f32, NHWC)
 * = sum over (ky, kx) ascending of the dcols entries whose window covers the pixel.       */
int ivit_im2col(int x_dtype, const void* X, long B, long H, long W, long C, long k, long stride, long pad, long Ho,
                long Wo, void* cols, long ldc, int cols_dtype, void* stream);
int ivit_col2im(const float* dcols, long ldc, long B, long H, long W, long C, long k, long stride, long pad, long Ho,
                long Wo, float* dX, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* IVIT_H */
