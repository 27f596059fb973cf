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

enum clipmi_dtype { CLIPMI_F32 = 0, CLIPMI_BF16 = 1 };

int clipmi_version(void);
const char* clipmi_last_error(void);

/* ---- GEMM:  C[m,n] = epi( alpha * sum_k A(m,k) B(n,k) )  --------------------------
 * Replaces nn.Linear forward/backward inside HF CLIPAttention/CLIPMLP
 * ([HF] modeling_clip.py:313-315,332,348-350), the adapters' down/up projections
 * (adapter/clip_adapter.py:19-21,146-148) and the CLIP projections (model_m.py:103,123).
 * A(m,k) = A[m*lda+k] if a_kmajor else A[k*lda+m]; same for B with n.
 * flags: bit0 bias[n] | bit1 quick_gelu | bit2 gelu_erf | bit3 += residual[m,n]
 *        bit4 *= quick_gelu'(aux[m,n]) | bit5 *= gelu_erf'(aux[m,n])
 *        bit6 C += result (beta = 1) | bit7 store pre-activation to aux[m,n]
 * dtypes: A/B bf16 (MFMA path) or f32 (exact-f32 parity path); C/residual/aux in c_dtype.
 * split_k > 1 (fp32 C, beta flag only) uses workspace of split_k*M*N floats.
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
} clipmi_gemm_desc;

#define CLIPMI_EPI_BIAS 1
#define CLIPMI_EPI_QGELU 2
#define CLIPMI_EPI_GELU 4
#define CLIPMI_EPI_RESID 8
#define CLIPMI_EPI_DQGELU 16
#define CLIPMI_EPI_DGELU 32
#define CLIPMI_EPI_BETA 64
#define CLIPMI_EPI_STORE_PRE 128

int clipmi_gemm(void* stream, const clipmi_gemm_desc* d);

#ifdef __cplusplus
}
#endif
#endif
