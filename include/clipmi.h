/*
 * libclipmi — MI355X-native (gfx950 / CDNA4) kernels for the CLIP dual-encoder +
 * adapter contrastive fine-tuning step of Quillboltcode/VLM-CLIP.
 *
 * C ABI only: plain pointers, sizes and dtype codes; no torch types.  Every entry point
 * enqueues work on the caller's hipStream_t (passed as void*) and returns 0 on success
 * or a negative status; clipmi_last_error() returns a thread-local message.  The
 * library never allocates or frees caller memory; scratch comes from caller workspace.
 *
 * The reference has no native boundary: its hot path is PyTorch/HF
 * module calls.  Each entry point below names the reference op it replaces.
 *
 * Collectives: clipmi_allgather_embed / clipmi_reducescatter_grad /
 * clipmi_allreduce_grads below run the data-parallel exchanges over RCCL for FFI hosts with one process
 * per GPU (communicator from clipmi_comm_unique_id + clipmi_comm_init).  The PyTorch host issues the same
 * exchanges through torch.distributed (backend "nccl" = RCCL over xGMI) in clipmi/towers.py (ContrastiveFn)
 * and clipmi/trainer.py (GradBucketReducer), on the same HIP streams these entry points run on.
 * Workspaces are sized per call by the *_ws() queries (no context object).
 */
#ifndef CLIPMI_H
#define CLIPMI_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define CLIPMI_OK 0
#define CLIPMI_ERR_INVALID -1   /* bad shape/arg -> Python ValueError */
#define CLIPMI_ERR_HIP -2       /* HIP runtime error -> RuntimeError */
#define CLIPMI_ERR_UNSUPPORTED -3

enum clipmi_dtype { CLIPMI_F32 = 0, CLIPMI_BF16 = 1, CLIPMI_FP8 = 2 /* MXFP8: OCP e4m3 + E8M0 per 32 k */ };

int clipmi_version(void);
const char* clipmi_last_error(void);
/* sha256 (hex) of the sources this library was compiled from (vlm-clip_amd/Makefile DIGEST_SRC) */
const char* clipmi_build_digest(void);

/* ---- GEMM:  C[m,n] = epi( alpha * sum_k A(m,k) B(n,k) )  --------------------------
 * Replaces nn.Linear forward/backward inside HF CLIPAttention/CLIPMLP
 * ([HF] modeling_clip.py:313-315,332,348-350), the adapters' down/up projections
 * (adapter/clip_adapter.py:19-21,146-148) and the CLIP projections (model_m.py:103,123).
 * A(m,k) = A[m*lda+k] if a_kmajor else A[k*lda+m]; same for B with n.
 * flags: bit0 bias[n] | bit1 quick_gelu | bit2 gelu_erf | bit3 += residual[m,n]
 *        bit4 *= quick_gelu'(aux[m,n]) | bit5 *= gelu_erf'(aux[m,n])
 *        bit6 C += result (beta = 1) | bit7 store pre-activation to aux[m,n]
 *        bit8 store act'(pre-activation) to aux[m,n] | bit9 *= aux[m,n]
 * dtypes: A/B bf16 (MFMA path) or f32 (exact-f32 parity path); C/residual/aux in c_dtype.
 * split_k > 1 (fp32 C, beta flag only) uses workspace of split_k*M*N floats (+ split_k*M with
 * bias_grad: per-split bias partials summed in split order, so results are run-to-run identical).
 */
typedef struct clipmi_gemm_desc {
  int M, N, K;
  const void* A; int64_t lda; int a_kmajor;
  const void* B; int64_t ldb; int b_kmajor;
  void* C; int64_t ldc;
  const void* bias;
  const void* residual; int64_t ldr;
  void* aux; int64_t ldaux;
  float alpha;
  int flags;
  int ab_dtype;   /* clipmi_dtype */
  int c_dtype;    /* clipmi_dtype */
  int bias_dtype; /* clipmi_dtype */
  int split_k;
  void* workspace; int64_t workspace_bytes;
  float* bias_grad;     /* wgrad only: bias_grad[m] += sum_k A(m,k) (fused Linear bias gradient, fp32) */
  int force_small_tile; /* 1: 128x128 register-staged kernel; >=2: 256-kernel schedule variant (bench) */
  /* ab_dtype == CLIPMI_FP8 (BASELINE config 5, forward GEMMs of the frozen towers): A, B are OCP e4m3
   * bytes, both k-major, K % 128 == 0; a_scale / b_scale are E8M0 bytes [rows][K/32] (OCP MX:
   * element value = fp8 * 2^(scale - 127)); v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation,
   * the bf16 epilogues.  c_dtype == CLIPMI_FP8 (flags bias and/or quick_gelu / gelu only, ldc == N,
   * N % 32 == 0, C 16-byte and c_scale 2-byte aligned): C is written as MXFP8 too, e4m3 bytes [M, N]
   * and E8M0 scales c_scale [M, N/32] (fc1 -> fc2 without a bf16 round trip). */
  const uint8_t* a_scale;
  const uint8_t* b_scale;
  uint8_t* c_scale;
} clipmi_gemm_desc;

#define CLIPMI_EPI_BIAS 1
#define CLIPMI_EPI_QGELU 2
#define CLIPMI_EPI_GELU 4
#define CLIPMI_EPI_RESID 8
#define CLIPMI_EPI_DQGELU 16
#define CLIPMI_EPI_DGELU 32
#define CLIPMI_EPI_BETA 64
#define CLIPMI_EPI_STORE_PRE 128
/* store the activation's derivative at the pre-activation to aux[m,n] (quick_gelu' with bit1,
 * gelu_erf' with bit2), computed from the fp32 pre-activation beside the activation itself, so
 * the backward is a plain product (bit9) instead of a load + derivative per element */
#define CLIPMI_EPI_STORE_DACT 256
/* C *= aux[m,n] (the stored derivative: d_pre = d_act * act'(pre)) */
#define CLIPMI_EPI_MUL_AUX 512

/* Not an epilogue: ab_dtype and c_dtype CLIPMI_F32, computed on the bf16 MFMA kernels as a split-operand
 * product (precision "bf16x3"): x = bf16(x) + bf16(x - bf16(x)) for both operands and
 * A.B^T ~ Ah.Bh^T + Ah.Bl^T + Al.Bh^T in one bf16 GEMM over 3K (fp32 accumulation), ~2^-16 relative
 * error per product instead of bf16's 2^-8.  Any epilogue flag except bias_grad; K % 8 == 0 when an operand
 * is k-major (the bf16 kernels' layout rules apply to the split images: row-major A needs M % 8 == 0); workspace
 * >= clipmi_gemm_split3_ws(...) bytes, 256-byte aligned (it also holds the split-K slabs). */
#define CLIPMI_GEMM_SPLIT3 1024
int64_t clipmi_gemm_split3_ws(int M, int N, int K, int a_kmajor, int b_kmajor, int split_k);

int clipmi_gemm(void* stream, const clipmi_gemm_desc* d);
/* Strided batch of nb1 x nb2 fp32 products (exact f32; flags: beta only): product z = i1 * nb2 + i2 reads
 * A + i1 * sa1 + i2 * sa2, B + i1 * sb1 + i2 * sb2 and writes C + i1 * sc1 + i2 * sc2 (elements), the
 * rest as clipmi_gemm.  One launch for the per-(sample, head) score / context products of attention at
 * head widths the flash kernels do not take (peclip ContextAdapter / SharedAdapter, adapter/peclip.py:21-48). */
int clipmi_gemm_batched(void* stream, const clipmi_gemm_desc* d, int nb1, int nb2, int64_t sa1, int64_t sa2,
                        int64_t sb1, int64_t sb2, int64_t sc1, int64_t sc2);
/* Diagnostic (no reference counterpart): arm / disarm (nullptr) the in-kernel s_memtime stamps of
 * the 4-wave GEMM's timing variant (force_small_tile = 22); buf holds 512 * 4 * 128 u64 of device
 * memory (layout: csrc/gemm4.hip, reader: tools/w4_stamps.py). */
int clipmi_gemm_stamps(void* buf);
/* MXFP8 quantisation of a [R, K] bf16/f32 matrix (row stride ldx elements) into OCP e4m3 bytes
 * q [R, K] and E8M0 block scales [R, K/32]: per 32-element block the smallest power of two that
 * brings the block's max |x| to <= 448, round-to-nearest-even. */
int clipmi_quant_mxfp8(void* stream, int dtype, const void* x, int64_t ldx, int64_t R, int K, uint8_t* q,
                       uint8_t* scales);

/* ---- LayerNorm ([HF] modeling_clip.py:357,359,605,642,559; adapter/clip_adapter.py:15,142) -------
 * y = LN(x [+ pos[row % period] (+ cls at row % period == 0)]) * w + b; mean/rstd saved (fp32).
 * With pos != NULL the sum is written back to x: the vision embedding ([HF] :209-219) fused
 * into pre_layrnorm. Weights in the activation dtype. 1 <= D <= 4096: register-resident kernels for D / 64
 * in {1, 2, 3, 4, 6, 8, 12, 16} (every CLIP width), a one-wave-per-row kernel for any other width. */
int clipmi_layernorm_fwd(void* stream, int dtype, void* x, int64_t ldx, void* y, int64_t ldy, const void* w,
                         const void* b, float* mean, float* rstd, int R, int D, float eps, const void* pos,
                         const void* cls, int period);
/* The same with the input x (and pos / cls) in x_dtype and y, w, b in dtype: x_dtype == dtype, or an fp32 x
 * normalised into a bf16 y (the bf16 mode's fp32 residual stream -> the next GEMM's bf16 operand). */
int clipmi_layernorm_fwd2(void* stream, int x_dtype, int dtype, void* x, int64_t ldx, void* y, int64_t ldy,
                          const void* w, const void* b, float* mean, float* rstd, int R, int D, float eps,
                          const void* pos, const void* cls, int period);
/* The same LayerNorm (bf16 x, no embedding add) with its output written as MXFP8, quantised
 * from the fp32 result as clipmi_quant_mxfp8 does: q8 [R, D] e4m3, s8 [R, D/32] E8M0.  Feeds the
 * fp8 tower GEMMs (BASELINE config 5) without a bf16 round trip. D % 256 == 0, D <= 1024. */
int clipmi_layernorm_fwd_mxfp8(void* stream, int dtype, const void* x, int64_t ldx, uint8_t* q8, uint8_t* s8,
                               const void* w, const void* b, float* mean, float* rstd, int R, int D, float eps);
int64_t clipmi_layernorm_bwd_ws(int R, int D);
/* dx = [dres +] LN'(dy); dw/db (fp32, may be NULL) accumulate when beta_wb.  Widths as clipmi_layernorm_fwd. */
int clipmi_layernorm_bwd(void* stream, int dtype, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                         const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx, const void* dres,
                         int64_t ldres, float* dw, float* db, int beta_wb, void* ws, int64_t ws_bytes, int R, int D);
/* The same with x in x_dtype (fp32 residual stream) and dy, dx, dres, w in dtype (bf16 gradients). */
int clipmi_layernorm_bwd2(void* stream, int x_dtype, int dtype, const void* dy, int64_t lddy, const void* x,
                          int64_t ldx, const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx,
                          const void* dres, int64_t ldres, float* dw, float* db, int beta_wb, void* ws,
                          int64_t ws_bytes, int R, int D);
/* the same with the affine weight's dtype given: w_dtype = dtype, or CLIPMI_F32 with fp32 x (the vision
   pre_layrnorm on the fp32 residual stream normalises with the fp32 master weights in its forward) */
int clipmi_layernorm_bwd3(void* stream, int x_dtype, int dtype, int w_dtype, const void* dy, int64_t lddy,
                          const void* x, int64_t ldx, const float* mean, const float* rstd, const void* w, void* dx,
                          int64_t lddx, const void* dres, int64_t ldres, float* dw, float* db, int beta_wb, void* ws,
                          int64_t ws_bytes, int R, int D);
/* out[n] (+)= sum_r x[r][n]  (bias gradients of every Linear on the path) */
int64_t clipmi_colsum_ws(int R, int N);
int clipmi_colsum(void* stream, int dtype, const void* x, int64_t ldx, int R, int N, float* out, int beta, void* ws,
                  int64_t ws_bytes);
/* out[t][c] (+)= sum_b x[(b*period+t)][c] for t < nt  (position / class embedding gradients) */
int clipmi_period_sum(void* stream, int dtype, const void* x, int64_t ldx, int nb, int period, int nt, int D,
                      float* out, int beta);

/* ---- Bottleneck adapter (adapter/clip_adapter.py:17-23 TextAdapter.forward, :144-150
 * VisionAdapter.forward; adapter/peclip.py:13-18 TextualAdapter with ln = 0) --------------------
 * y = LN(up(gelu_erf(down(x))) + x) * ln_w + ln_b (ln = 0: without the LayerNorm) for R rows
 * (row strides ldx / ldy): w_down [A, D], b_down [A], w_up [D, A], b_up [D] (nn.Linear layout,
 * activation dtype).  One call sequences the library's own kernels on the stream (csrc/adapter.cpp):
 * down GEMM (+ bias + gelu_erf; pre-activation stored when pre != NULL), up GEMM (+ bias + residual),
 * LayerNorm -- the path the Python mirror runs.  act [R, A] is required (it carries the bottleneck
 * between the GEMMs); with ln also z [R, D] (the pre-LN sum) and mean / rstd [R] (fp32).  pre [R, A]
 * is saved for the backward (NULL in inference).  D % 8 == 0, A % 8 == 0; with ln D <= 4096. */
int clipmi_adapter_fwd(void* stream, int dtype, int R, int D, int A, const void* x, int64_t ldx, const void* w_down,
                       const void* b_down, const void* w_up, const void* b_up, const void* ln_w, const void* ln_b,
                       float eps, int ln, void* y, int64_t ldy, void* pre, void* act, void* z, float* mean,
                       float* rstd);
int64_t clipmi_adapter_bwd_ws(int R, int D, int A);
/* dx = dL/dx given dy = dL/dy (the forward's saved tensors); the fp32 parameter gradients g_*
 * (each may be NULL; g_ln_* ignored when ln = 0) ACCUMULATE (+=, AccumulateGrad): LN backward, the
 * up / down weight-gradient GEMMs (bias gradients fused in bf16, a column sum in fp32), the
 * gelu_erf'-fused input-gradient GEMM and the residual-fused dx GEMM; no atomics across tiles, so a
 * replay is bitwise equal. */
int clipmi_adapter_bwd(void* stream, int dtype, int R, int D, int A, const void* dy, int64_t lddy, const void* x,
                       int64_t ldx, const void* pre, const void* act, const void* z, const float* mean,
                       const float* rstd, const void* w_down, const void* w_up, const void* ln_w, int ln, void* dx,
                       int64_t lddx, float* g_w_down, float* g_b_down, float* g_w_up, float* g_b_up, float* g_ln_w,
                       float* g_ln_b, void* ws, int64_t ws_bytes);

/* ---- Embeddings ------------------------------------------------------------------------------
 * text: x0[r] = tok[ids[r]] + pos[r % S]   ([HF] CLIPTextEmbeddings.forward :232-256);
 * *bad_flag |= 1 on an out-of-vocabulary id (Python raises IndexError like nn.Embedding). */
int clipmi_text_embed(void* stream, int dtype, const int64_t* ids, const void* tok, const void* pos, void* x0, int R,
                      int S, int D, int V, int* bad_flag);
int64_t clipmi_text_embed_bwd_ws(int R, int V);
/* gtok[v] (+)= sum_{r: ids[r]==v} dx0[r]  (counting sort, one wave per id, no float atomics) */
int clipmi_text_embed_bwd(void* stream, int dtype, const int64_t* ids, const void* dx0, int R, int D, int V,
                          float* gtok, int beta, void* ws, int64_t ws_bytes);
/* vision: Conv2d(k=s=P, no bias) as im2col + GEMM ([HF] :148-154, :211-212).  X is
 * [B*(G*G+1), Kp] with a zero row in each image's CLS slot, K index c*P*P+ky*P+kx. */
int clipmi_im2col(void* stream, int dtype, const float* pixels, void* X, int B, int C, int H, int P, int Kp);
/* The input step (CLIPImageProcessor's center_crop + rescale + normalize, [HF]
 * image_processing_clip.py) fused into the same im2col: uint8 images [B, Hin, Win, 3]
 * (channels last), centre-cropped to image_size, (u/255 - mean[c]) / std[c].  The shortest-edge
 * resize before it is clipmi_resize_u8 below.  P even (16/32: 8 pixels per thread; ViT-L/14: 2), Kp == 3*P*P or padded
 * to a multiple of 8 (the pad columns are zeroed: L/14's 588 -> 640); mean/std are 3 host floats. */
int clipmi_im2col_u8(void* stream, int dtype, const uint8_t* images, void* X, int B, int Hin, int Win, int image_size,
                     int P, int Kp, const float* mean, const float* std);
/* Input-step resize (dataset.py:152-164 -> CLIPImageProcessor, shortest edge = image size):
 * PIL Image.resize(BICUBIC) of channels-last RGB uint8 [B, Hin, Win, 3] -> [B, Hout, Wout, 3],
 * bit-exact (fp64 tap weights -> 22-bit fixed point, horizontal then vertical 8-bit pass; a pass
 * whose size is unchanged is skipped).  Workspace: clipmi_resize_u8_ws bytes. */
int64_t clipmi_resize_u8_ws(int B, int Hin, int Win, int Hout, int Wout);
int clipmi_resize_u8(void* stream, const uint8_t* in, int B, int Hin, int Win, uint8_t* out, int Hout, int Wout,
                     void* ws, int64_t ws_bytes);
/* pooled token per row: mode 0 first token (model_m.py:102), 1 first EOS, 2 argmax id ([HF] :561-581) */
int clipmi_pool_index(void* stream, const int64_t* ids, int B, int S, int64_t eos, int mode, int* idx);
int clipmi_gather_rows(void* stream, int dtype, const void* src, const int* idx, int B, int S, int D, void* out);
int clipmi_scatter_rows(void* stream, int dtype, const void* src, const int* idx, int B, int S, int D, void* dst,
                        int beta);

/* ---- Attention (head_dim 64, N <= 4096: K/V resident in LDS up to N = 288, K/V streamed above;
 * [HF] CLIPAttention :298-335, eager core :259-277) -----
 * qkv: [B*N, 3D] (q | k | v, head h at h*64), o: [B*N, D], lse: [B*H*N] fp32.
 * attention_mask: int64 [B, N] key padding (1 keep) or NULL; causal for the text tower. */
int clipmi_attention_fwd(void* stream, int dtype, const void* qkv, void* o, float* lse, const int64_t* attention_mask,
                         int causal, int B, int H, int N, int D);
/* The K/V-streaming forward with O written as MXFP8 (OCP e4m3 o8 [B*N, D], 4-byte aligned + E8M0 s8 [B*N, D/32],
 * clipmi_quant_mxfp8's rule applied to the fp32 O): the fp8 towers' out-projection operand without a
 * bf16 round trip (BASELINE config 5).  bf16 q/k/v. */
int clipmi_attention_fwd_mxfp8(void* stream, const void* qkv, uint8_t* o8, uint8_t* s8, float* lse,
                               const int64_t* attention_mask, int causal, int B, int H, int N, int D);
int clipmi_attention_bwd(void* stream, int dtype, const void* qkv, const void* o, const float* lse, const void* dout,
                         void* dqkv, const int64_t* attention_mask, int causal, int B, int H, int N, int D);
/* bf16x3 split images (the layout of CLIPMI_GEMM_SPLIT3's operands): clipmi_split3 writes the image of an fp32
   operand -- k-major X [rows][K] -> bf16 [rows][3K], else X [K][rows] -> [3K][round8(rows)] -- with segments
   (h, h, l) for pattern 0 or (h, l, h) for pattern 1, h = bf16(x), l = bf16(x - h); clipmi_split3_elems gives its
   size in elements.  clipmi_split3_colsum writes the k-major image of x [R, N] and, with colsum, adds x's column
   sums to colsum[N] (+= when beta; ws >= clipmi_split3_colsum_ws(R, N) bytes, 16-byte aligned). */
int64_t clipmi_split3_elems(int rows, int K, int kmajor);
int clipmi_split3(void* stream, const float* X, int64_t ldx, int rows, int K, int kmajor, void* out, int pattern);
int64_t clipmi_split3_colsum_ws(int R, int N);
int clipmi_split3_colsum(void* stream, const float* x, int64_t ldx, int R, int N, void* out, int pattern,
                         float* colsum, int beta, void* ws, int64_t ws_bytes);
/* A bf16 GEMM (d->ab_dtype CLIPMI_BF16, d->c_dtype CLIPMI_F32: the epilogue computes in fp32) whose result is
   written as its split image instead -- d->C bf16 [M][d->ldc], ldc >= 3N, segments at columns n, N + n, 2N + n in
   the pattern above -- by the producing kernel's epilogue (the bf16x3 mode's fc1 output and fc2 input gradient,
   which clipmi_split3_colsum would otherwise split from an fp32 copy).  Flags: bias + quick_gelu (+ store_dact:
   the derivative to fp32 aux), or mul_aux (fp32 aux).  colsum (+= when beta): the column sums of the fp32 result,
   ws >= clipmi_gemm_x3out_ws(M, N) bytes, 256-byte aligned.  clipmi_gemm_x3out_ok: whether a shape / layout /
   flag set has this form (k-major A, M >= 256, N >= 128, N % 8 == 0, K % 64 == 0). */
int64_t clipmi_gemm_x3out_ws(int M, int N);
int clipmi_gemm_x3out_ok(int M, int N, int K, int a_kmajor, int b_kmajor, int flags);
int clipmi_gemm_x3out(void* stream, const clipmi_gemm_desc* d, int pattern, float* colsum, int beta, void* ws,
                      int64_t ws_bytes);
/* bf16x3 engine: the fp32 LayerNorm backward (as clipmi_layernorm_bwd with dtype CLIPMI_F32, dw / db required) that
   also writes dx as its pattern-1 split image dimg bf16 [R][3D] and adds dx's column sums onto colsum[D] (+= when
   beta_cs) -- the next GEMMs' operand and a Linear's bias gradient without a split pass.  D / 64 in
   {1, 2, 3, 4, 6, 8, 12, 16}; ws >= clipmi_layernorm_bwd_x3_ws(R, D) bytes, 16-byte aligned. */
int64_t clipmi_layernorm_bwd_x3_ws(int R, int D);
int clipmi_layernorm_bwd_x3(void* stream, const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* mean,
                            const float* rstd, const float* w, float* dx, int64_t lddx, const float* dres,
                            int64_t ldres, float* dw, float* db, int beta_wb, void* dimg, float* colsum, int beta_cs,
                            void* ws, int64_t ws_bytes, int R, int D);
/* LayerNorm of fp32 x with fp32 affine weights written as the bf16x3 split image y3 [R][3D] of its output
   (pattern as above); mean / rstd saved as in clipmi_layernorm_fwd.  D / 64 in {1, 2, 3, 4, 6, 8, 12, 16}. */
int clipmi_layernorm_fwd_x3(void* stream, const float* x, int64_t ldx, void* y3, int pattern, const float* w,
                            const float* b, float* mean, float* rstd, int R, int D, float eps);
/* The bf16x3 precision mode's attention (csrc/attention_x3.hip): fp32 operands and outputs exactly as
   clipmi_attention_fwd / _bwd with dtype CLIPMI_F32, every product (q k^T, P v, dO v^T, dS k, dS^T q, P^T dO)
   run as three bf16 MFMA products of the hi / lo operand splits (~2^-16 relative per product).  N > 288 falls
   back to the exact-f32 kernels. */
int clipmi_attention_fwd_x3(void* stream, const void* qkv, void* o, float* lse, const int64_t* attention_mask,
                            int causal, int B, int H, int N, int D);
int clipmi_attention_bwd_x3(void* stream, const void* qkv, const void* o, const float* lse, const void* dout,
                            void* dqkv, const int64_t* attention_mask, int causal, int B, int H, int N, int D);
/* clipmi_attention_fwd_x3 that also writes O's pattern-0 split image oimg bf16 [B*N][3D] (8-byte aligned) beside the
   fp32 O: the out-projection's operand in the bf16x3 engine without a split pass.  N <= 288. */
int clipmi_attention_fwd_x3img(void* stream, const void* qkv, void* o, void* oimg, float* lse,
                               const int64_t* attention_mask, int causal, int B, int H, int N, int D);
/* clipmi_attention_bwd_x3 with d_qkv written as its pattern-1 split image dimg bf16 [B*N][9D] (the layout of
   clipmi_split3_colsum) and d_qkv's column sums (the q / k / v bias gradient) added onto colsum[3D] (+= when beta),
   instead of the fp32 dqkv; N <= 288, ws >= clipmi_attention_bwd_x3img_ws(B, D) bytes, 256-byte aligned. */
int64_t clipmi_attention_bwd_x3img_ws(int B, int D);
int clipmi_attention_bwd_x3img(void* stream, const void* qkv, const void* o, const float* lse, const void* dout,
                               void* dimg, float* colsum, int beta, void* ws, int64_t ws_bytes,
                               const int64_t* attention_mask, int causal, int B, int H, int N, int D);

/* ---- Encoder engine: whole CLIPEncoder fwd/bwd in one call ([HF] :477-482, :362-383) ---------- */
typedef struct clipmi_layer_w { /* activation dtype; qkv_w = [q;k;v] rows, [3D, D] */
  const void *ln1_w, *ln1_b, *qkv_w, *qkv_b, *out_w, *out_b, *ln2_w, *ln2_b, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} clipmi_layer_w;
typedef struct clipmi_layer_grad { /* fp32, accumulated */
  float *ln1_w, *ln1_b, *qkv_w, *qkv_b, *out_w, *out_b, *ln2_w, *ln2_b, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} clipmi_layer_grad;
typedef struct clipmi_layer_act { /* saved activations; pre == NULL in inference.  The fp8 encoder
  * (dtype CLIPMI_FP8) with N > 288 sends the attention output straight to the out-projection's
  * MXFP8 operand and does NOT write o: read act[l].o only after a bf16 / f32 forward or N <= 288. */
  void *x_in, *ln1, *qkv, *o, *h, *ln2, *pre, *act;
  float *mean1, *rstd1, *lse, *mean2, *rstd2;
} clipmi_layer_act;
typedef struct clipmi_layer_w8 { /* MXFP8 GEMM weights: e4m3 [out, in] + E8M0 scales [out, in/32] */
  const void *qkv_w, *qkv_s, *out_w, *out_s, *fc1_w, *fc1_s, *fc2_w, *fc2_s;
} clipmi_layer_w8;
typedef struct clipmi_encoder_desc {
  int dtype, B, N, D, F, H, L;  /* dtype CLIPMI_FP8: bf16 activations / LN / attention, MXFP8 GEMMs (forward only) */
  float eps;
  int causal;
  const int64_t* attention_mask;
  const clipmi_layer_w* layers;  /* [L] (bf16 LN weights and biases also for CLIPMI_FP8) */
  clipmi_layer_grad* grads;      /* [L], backward only */
  clipmi_layer_act* act;         /* [L]; layer l writes its output to act[l+1].x_in (x_out for the last) */
  void* x_out;
  void* workspace;
  int64_t workspace_bytes;
  const clipmi_layer_w8* layers8; /* [L], CLIPMI_FP8 only */
  void* q8;                       /* CLIPMI_FP8: MXFP8 activation scratch, align256(R*D) + R*F bytes (R = B*N) */
  void* s8;                       /* CLIPMI_FP8: its block scales, align256(R*D/32) + R*F/32 bytes */
  /* dtype CLIPMI_BF16 only: the residual stream in fp32 -- act[l].x_in, act[l].h and x_out are fp32
   * (LayerNorms read them as fp32, the out-projection / fc2 epilogues add and write fp32), every GEMM
   * operand stays bf16.  The reference is fp32 end to end (trainer.py:81-99); rounding the residual sum
   * to bf16 at each of the 2L residual adds was the largest bf16-mode error (profiles/r05_bf16_error_sources.log). */
  int resid_f32;
  /* dtype CLIPMI_F32 only (precision "bf16x3"): every GEMM of the forward and backward runs as three bf16
   * products of hi / lo operand splits, over split images (clipmi_split3) that each activation's and activation
   * gradient's producer writes once; attention as clipmi_attention_fwd_x3 / _bwd_x3; LayerNorm, softmax,
   * residual stream and all accumulation fp32.  Scratch in x3_ws (x3_ws_bytes >= clipmi_encoder_x3_ws, 256-byte
   * aligned; one scratch per concurrently running encoder).  The saved activations change form in this mode:
   * act[l].ln1 / .ln2 hold the bf16 [R][3D] images of the LayerNorm outputs, act[l].o the fp32 [R][D] attention
   * output followed (at the next 256-byte boundary) by its [R][3D] image, act[l].act the bf16 [R][3F] image of
   * fc1's output; x_in, qkv, h and pre stay fp32 (csrc/engine.cpp encoder_fwd_x3). */
  int gemm_x3;
  void* x3_ws;
  int64_t x3_ws_bytes;
} clipmi_encoder_desc;
int clipmi_encoder_fwd(void* stream, const clipmi_encoder_desc* d);
int64_t clipmi_encoder_bwd_ws(const clipmi_encoder_desc* d);
/* the split-image scratch of a gemm_x3 encoder (forward and backward; 0 when gemm_x3 is off) */
int64_t clipmi_encoder_x3_ws(const clipmi_encoder_desc* d);
/* dx: dL/d(encoder output) in, dL/d(encoder input) out */
int clipmi_encoder_bwd(void* stream, const clipmi_encoder_desc* d, void* dx);
/* the same for layers layer_hi-1 .. layer_lo only (chunked backward: each chunk's gradient slice
 * can be all-reduced while the next chunk runs) */
int clipmi_encoder_bwd_layers(void* stream, const clipmi_encoder_desc* d, void* dx, int layer_hi, int layer_lo);

/* ---- Contrastive head (model_m.py:146-171), fp32 -------------------------------------------- */
int clipmi_l2norm_fwd(void* stream, const float* x, float* y, float* nrm, int B, int E);
int clipmi_l2norm_bwd(void* stream, const float* dy, const float* y, const float* nrm, float* dx, int B, int E);
/* logits = exp(*logit_scale) * S over a [B, Bg] cosine block; lse, ce per row (label0 + i) */
int clipmi_contrastive_ce_fwd(void* stream, const float* S, float* logits, const float* logit_scale, int B, int Bg,
                              int label0, float* lse, float* ce);
/* dS = g*exp(ls)*(softmax - onehot)*norm ; dls_row = sum_j dlogit*logit */
int clipmi_contrastive_ce_bwd(void* stream, const float* logits, const float* lse, const float* logit_scale,
                              const float* grad_out, int B, int Bg, int label0, float norm, float* dS, float* dls_row);
/* Column-streamed form (the [B, Bg] blocks never materialised): the caller walks chunks
 * [col0, col0 + C) of the cosine block S (row stride C).  fwd_chunk merges the chunk into the
 * running per-row (max, sum-of-exp) pairs run [B][2] (col0 == 0 initialises them) and stores
 * the label logit lab[i] when column label0 + i lies in the chunk; finish turns them into lse, ce.
 * bwd_chunk writes the chunk's dS [B][C] and sets (beta = 0) or accumulates dls_row. */
int clipmi_contrastive_ce_fwd_chunk(void* stream, const float* S, const float* logit_scale, int B, int C, int col0,
                                    int Bg, int label0, float* run, float* lab);
int clipmi_contrastive_ce_finish(void* stream, const float* run, const float* lab, int B, float* lse, float* ce);
int clipmi_contrastive_ce_bwd_chunk(void* stream, const float* S, const float* lse, const float* logit_scale,
                                    const float* grad_out, int B, int C, int col0, int Bg, int label0, float norm,
                                    float* dS, float* dls_row, int beta);
int clipmi_sum2(void* stream, const float* a, const float* b, int n, float scale, float* out, int beta);

/* ---- Optimizer (trainer.py:95,98; [HF] optimization.py:101-129) ------------------------------ */
int64_t clipmi_grad_norm_ws(void);
/* norm_out[0] = ||g||_2, norm_out[1] = min(1, max_norm/(norm+1e-6)) (device memory) */
int clipmi_grad_norm(void* stream, const float* g, int64_t n, float max_norm, float* norm_out, void* ws,
                     int64_t ws_bytes);
int64_t clipmi_grad_norm_multi_ws(int count);
int clipmi_grad_norm_multi(void* stream, const float* const* gs, const int64_t* ns, int count, float max_norm,
                           float* norm_out, void* ws, int64_t ws_bytes);
int clipmi_grad_scale(void* stream, float* g, int64_t n, const float* norm_out);
/* torch.optim.AdamW step on a flat fp32 arena; grads scaled by clip[1] when clip != NULL;
 * shadow (bf16, may be NULL) refreshed from the new parameters. */
int clipmi_adamw(void* stream, float* p, const float* g, float* m, float* v, void* shadow_bf16, int64_t n, double lr,
                 double beta1, double beta2, double eps, double weight_decay, int step, const float* clip);
int clipmi_cast_f32_bf16(void* stream, const float* src, void* dst, int64_t n);

/* ---- Feature-level adapter heads (model_t.py CLIPAdapter / ZeroShot) -----
 * All fp32, rows of E <= 1024 features, bottleneck A <= 256, C <= 1024 classes.
 * clipmi_feature_adapter_fwd replaces VisualAdapter/TextAdapter.forward (model_t.py:13-33) fused
 * with the residual blend and renormalisation of model_t.py:186-197 (visual, norm_in = 1: the
 * input is normalised first, model_t.py:182-183) and :113-119 / :200-207 (text prototypes,
 * norm_in = 0): xn = norm_in ? x/|x| : x; h = relu(W1 xn + b1); z = alpha (W2 h + b2) +
 * (1 - alpha) xn; out = z/|z|; rz = 1/|z|.  W1 [A, E], W2 [E, A] (nn.Linear layout). */
int clipmi_feature_adapter_fwd(void* stream, const float* x, int B, int E, int A, const float* W1, const float* b1,
                               const float* W2, const float* b2, float alpha, int norm_in, float* xn, float* h,
                               float* out, float* rz, const uint8_t* keep, float keep_scale);
/* keep (uint8 [B, A], may be NULL): training-mode nn.Dropout on the ReLU output (model_v.py:18-27:
 * fc2(dropout(relu(fc1(x))))), h *= keep * keep_scale with keep_scale = 1/(1-p). */
int clipmi_feature_adapter_bwd_ws(int B, int E, int A);
/* grads = [dW1 | db1 | dW2 | db2] (flat, fp32) += the batch's gradients given dout = dL/dout;
 * keep_scale: the forward's (1 when it ran without dropout). */
int clipmi_feature_adapter_bwd(void* stream, const float* dout, const float* out, const float* rz, const float* xn,
                               const float* h, int B, int E, int A, const float* W2, float alpha, float* grads,
                               void* workspace, int64_t workspace_bytes, float keep_scale);
/* Dropout masks (nn.Dropout(p) in model_v.BaseAdapter and SharedMHSAttentionAdapter,
 * adapter/clip_adapter.py:84,96): keep[i] = u(seed, offset + i) >= p with a counter-based hash,
 * so a (seed, offset) pair reproduces its mask; apply: y = x * keep * scale (+ res, may be NULL). */
int clipmi_dropout_mask(void* stream, uint8_t* keep, int64_t n, float p, uint64_t seed, uint64_t offset);
int clipmi_dropout_apply(void* stream, const float* x, const uint8_t* keep, int64_t n, float scale, const float* res,
                         float* y);
/* Average fusion of model_v.EnhancedCLIPAdapter (model_v.py:310-315): out = normalise((a + b) / 2),
 * ru = 1/|(a+b)/2|; backward d a = d b = dab. */
int clipmi_fuse_avg(void* stream, const float* a, const float* b, int B, int E, float* out, float* ru);
int clipmi_fuse_avg_bwd(void* stream, const float* dout, const float* out, const float* ru, int B, int E, float* dab);
/* Class scores (model_t.py:200-203 logits, :240-247 predict, :252-298 predict_with_all_descriptions):
 * s[b, c] = max over descriptions j in [off[c], off[c+1]) of scale * img[b] . desc[j]; probs =
 * softmax_c.  Any output may be NULL.  With labels (int64 [B]): loss_rows[b] = CE of row b,
 * dscore = softmax - onehot, *bad = 1 on an out-of-range label. */
int clipmi_class_scores(void* stream, const float* img, int B, int E, const float* desc, const int* off, int C,
                        float scale, float* scores, float* probs, const int64_t* labels, float* loss_rows,
                        float* dscore, int* bad);
int clipmi_row_mean(void* stream, const float* v, int B, float* out);
/* Mean-CE backward through prototype scores (one description per class): d = dscore * gscale[0] / B;
 * dimg = scale d P, dprotos = scale d^T img.  gscale may be NULL (1). */
int clipmi_class_ce_bwd(void* stream, const float* dscore, const float* img, const float* protos, int B, int C, int E,
                        float scale, const float* gscale, float* dimg, float* dprotos);

/* Row softmax of scale*x (fp32, y may alias x) and its backward dx = scale*y*(dy - <dy, y>):
 * the shared cross-attention adapter's probabilities (adapter/clip_adapter.py:117). */
int clipmi_softmax_rows(void* stream, const float* x, float* y, int R, int N, float scale);
int clipmi_softmax_rows_bwd(void* stream, const float* y, const float* dy, float* dx, int R, int N, float scale);

/* ---- Live kernel timing (bench.py roofline) --------------------------------------------------
 * While armed, every launch whose variant label is in the comma-separated list `variants`
 * (e.g. "gemm256_fwd_bias_qgelu_pre,gemm256_dgrad", "gemm256_wgrad", "attn_fwd") is bracketed by
 * hipEvents on its own stream, up to max_launches.  clipmi_prof_read (after a synchronize)
 * returns the launch count and fills per-launch milliseconds and algorithmic FLOPs;
 * clipmi_prof_read_labels gives each launch's index in the list. */
int clipmi_prof_arm(const char* variants, int max_launches);
int clipmi_prof_read_labels(int max, int* which);
int clipmi_prof_disarm(void);
/* Restrict the armed profiler to launches on one HIP stream (which may be the null stream):
 * with the towers on
 * two streams, launches on the side stream share the GPU with the other tower's kernels and
 * their event-bracketed durations are not the kernel's own. */
int clipmi_prof_stream(void* stream);
int clipmi_prof_read(int max, float* ms, double* flops);

/* ---- Data-parallel collectives over RCCL --------------------------------------------
 * One communicator per process / GPU.  Rank 0 creates the 128-byte id, the host distributes it (any channel)
 * and every rank calls clipmi_comm_init with it; librccl is opened on first use (CLIPMI_ERR_UNSUPPORTED when
 * it is absent).  All enqueue on `stream`; counts are elements.
 *   allgather_embed     global[r * count + i] = local_r[i]  (the L2-normalised [B, E] features of every rank
 *                       before the [B, Bg] similarities; model_m.py:146-171 on one device)   dtype f32 / bf16
 *   reducescatter_grad  local_r[i] = sum_s global_s[r * count + i]  (the column-direction feature gradients back
 *                       to their owners)
 *   allreduce_grads     grads[i] = sum_s grads_s[i], in place, fp32  (a bucket of the gradient arena: the
 *                       data-parallel sum of trainer.py:92's loss.backward) */
int clipmi_comm_unique_id(void* id /* 128 bytes */);
int clipmi_comm_init(void** comm, const void* id, int nranks, int rank);
int clipmi_comm_destroy(void* comm);
int clipmi_allgather_embed(void* stream, void* comm, int dtype, const void* local, void* global, int64_t count);
int clipmi_reducescatter_grad(void* stream, void* comm, int dtype, const void* global, void* local, int64_t count);
int clipmi_allreduce_grads(void* stream, void* comm, float* grads, int64_t count);
/* in-place sum over the ranks, fp32 or bf16 (the product path's optional bf16 gradient buckets: half the
   bytes per ring, ~2^-9 relative rounding of each rank's contribution) */
int clipmi_allreduce(void* stream, void* comm, int dtype, void* buf, int64_t count);

#ifdef __cplusplus
}
#endif
#endif
