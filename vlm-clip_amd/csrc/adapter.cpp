// The bottleneck adapter as one C-ABI call per direction: y = LN(up(gelu_erf(down(x))) + x), or
// without the LayerNorm (ln = 0).  Replaces TextAdapter / VisionAdapter.forward
// (adapter/clip_adapter.py:17-23, 144-150) and peclip.TextualAdapter.forward (adapter/peclip.py:13-18):
// nn.Linear(D, A) -> GELU (erf) -> nn.Linear(A, D) -> + x -> nn.LayerNorm(D, eps), and their backward
// (the reference's loss.backward through the adapter, trainer.py:92).
//
// Round 4 built these entry points as their own per-thread FMA kernels (one launch forward, two
// backward); they measured slower than the MFMA GEMM path at every size (R = 256: forward 51 vs 32 us,
// backward 361 vs 150 us; R = 4096 backward 3.8-4.3 ms vs 0.32-0.34 ms: the weight pass walked the rows
// serially, profiles/r04_adapter_fused_vs_gemm.log).  They now sequence the same library kernels the
// Python mirror (clipmi.towers.AdapterFn) runs, so an FFI caller gets the product path itself:
//   forward : down GEMM (+ bias + gelu_erf, pre-activation stored)  -> act [R, A]
//             up GEMM   (+ bias + residual x)                      -> z   [R, D]
//             LayerNorm (mean / rstd saved)                         -> y   [R, D]
//   backward: LayerNorm' (affine gradients accumulated)             -> dz
//             gW_up += dz^T act (bias gradient fused into the bf16 GEMM, column sum in fp32)
//             d_pre = (dz W_up) * gelu_erf'(pre)                   (epilogue-fused derivative)
//             gW_down += d_pre^T x, and its bias gradient
//             dx = d_pre W_down + dz                                (residual fused)
// Every launch is enqueued on the caller's stream, in this order; no host synchronisation.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include "internal.h"

namespace {

int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

int adp_gemm(void* s, int dt, int M, int N, int K, const void* A, int64_t lda, bool akm, const void* B, int64_t ldb,
             bool bkm, void* C, int64_t ldc, int c_dt, int flags, const void* bias = nullptr, const void* res = nullptr,
             int64_t ldr = 0, void* aux = nullptr, int64_t ldaux = 0, float* bias_grad = nullptr) {
  clipmi_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.a_kmajor = akm;
  d.B = B; d.ldb = ldb; d.b_kmajor = bkm;
  d.C = C; d.ldc = ldc;
  d.bias = bias; d.residual = res; d.ldr = ldr; d.aux = aux; d.ldaux = ldaux;
  d.alpha = 1.f; d.flags = flags;
  d.ab_dtype = dt; d.c_dtype = c_dt; d.bias_dtype = dt;
  d.split_k = 1;
  d.bias_grad = bias_grad;
  return clipmi_gemm(s, &d);
}

int adp_check(int dtype, int R, int D, int A, int ln) {
  CLIPMI_REQUIRE(dtype == CLIPMI_BF16 || dtype == CLIPMI_F32, "adapter: bf16 or f32");
  CLIPMI_REQUIRE(R >= 0 && D > 0 && A > 0, "adapter: R >= 0, D > 0, A > 0");
  // the bf16 MFMA GEMMs stage 16-byte rows; the fp32 GEMM (exact-f32 and bf16x3 modes) takes any width,
  // as nn.Linear does
  CLIPMI_REQUIRE(dtype != CLIPMI_BF16 || (D % 8 == 0 && A % 8 == 0), "adapter: bf16 needs D and A multiples of 8");
  CLIPMI_REQUIRE(!ln || D <= 4096, "adapter: with the LayerNorm D <= 4096");
  return CLIPMI_OK;
}

struct BwdWs {
  int64_t dz, dpre, ln, col, total;
};
BwdWs bwd_plan(int R, int D, int A) {  // byte offsets (fp32-sized, so one plan serves both dtypes)
  BwdWs w;
  w.dz = 0;
  w.dpre = w.dz + al256((int64_t)R * D * 4);
  w.ln = w.dpre + al256((int64_t)R * A * 4);
  w.col = w.ln + al256(clipmi_layernorm_bwd_ws(R, D));
  w.total = w.col + al256(clipmi_colsum_ws(R, std::max(D, A)));
  return w;
}

}  // namespace

extern "C" int clipmi_adapter_fwd(void* stream, int dtype, int R, int D, int A, const void* x, int64_t ldx,
                                  const void* w_down, const void* b_down, const void* w_up, const void* b_up,
                                  const void* ln_w, const void* ln_b, float eps, int ln, void* y, int64_t ldy,
                                  void* pre, void* act, void* z, float* mean, float* rstd) {
  CLIPMI_TRY(adp_check(dtype, R, D, A, ln));
  CLIPMI_REQUIRE(x && y && w_down && b_down && w_up && b_up && ldx >= D && ldy >= D, "adapter_fwd: operands");
  CLIPMI_REQUIRE(!ln || (ln_w && ln_b), "adapter_fwd: LayerNorm weights");
  CLIPMI_REQUIRE(act && (!ln || (z && mean && rstd)),
                 "adapter_fwd: act (and z, mean, rstd with the LayerNorm) are required: they carry the bottleneck "
                 "activation, the pre-LN sum and its statistics between the launches");
  if (R == 0) return CLIPMI_OK;
  // bf16 with the LayerNorm: the one-kernel form (adapter_fused.hip) where it measured faster than the sequence
  // (D <= 512: 37.5 vs 38.9 us at R = 1024; D = 768 / 1024: 48 / 59 vs 43 / 46 us, its per-workgroup phases being
  // latency chains at these row counts; profiles/r06_adapter_fused_ab.log).  Bitwise equal either way;
  // CLIPMI_ADAPTER_FUSED=1 / 0 forces the fused kernel / the sequence (A/B).
  const char* fe = getenv("CLIPMI_ADAPTER_FUSED");
  const bool want = fe ? fe[0] == '1' : D <= 512;
  const uintptr_t al16 = (uintptr_t)x | (uintptr_t)w_down | (uintptr_t)w_up | (uintptr_t)b_down | (uintptr_t)b_up |
                         (uintptr_t)ln_w | (uintptr_t)ln_b;
  if (want && adapter_fused_ok(dtype, ln, D, A, ldx, ldy) && (al16 & 15) == 0 && ((uintptr_t)y & 7) == 0)
    return adapter_fwd_fused(stream, R, D, A, x, ldx, w_down, b_down, w_up, b_up, ln_w, ln_b, eps, y, ldy, pre, act, z,
                             mean, rstd);
  const int f_down = CLIPMI_EPI_BIAS | CLIPMI_EPI_GELU | (pre ? CLIPMI_EPI_STORE_PRE : 0);
  CLIPMI_TRY(adp_gemm(stream, dtype, R, A, D, x, ldx, true, w_down, D, true, act, A, dtype, f_down, b_down, nullptr, 0,
                      pre, A));
  void* zout = ln ? z : y;
  const int64_t ldz = ln ? D : ldy;
  CLIPMI_TRY(adp_gemm(stream, dtype, R, D, A, act, A, true, w_up, A, true, zout, ldz, dtype,
                      CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, b_up, x, ldx));
  if (ln) CLIPMI_TRY(clipmi_layernorm_fwd(stream, dtype, z, D, y, ldy, ln_w, ln_b, mean, rstd, R, D, eps, nullptr, nullptr, 0));
  return CLIPMI_OK;
}

extern "C" int64_t clipmi_adapter_bwd_ws(int R, int D, int A) {
  if (R < 0 || D <= 0 || A <= 0) return 0;
  return bwd_plan(R, D, A).total;
}

extern "C" int clipmi_adapter_bwd(void* stream, int dtype, int R, int D, int A, const void* dy, int64_t lddy,
                                  const void* x, int64_t ldx, const void* pre, const void* act, const void* z,
                                  const float* mean, const float* rstd, const void* w_down, const void* w_up,
                                  const void* ln_w, int ln, void* dx, int64_t lddx, float* g_w_down, float* g_b_down,
                                  float* g_w_up, float* g_b_up, float* g_ln_w, float* g_ln_b, void* ws,
                                  int64_t ws_bytes) {
  CLIPMI_TRY(adp_check(dtype, R, D, A, ln));
  CLIPMI_REQUIRE(dy && x && pre && act && dx && w_down && w_up && lddy >= D && ldx >= D && lddx >= D,
                 "adapter_bwd: operands");
  CLIPMI_REQUIRE(!ln || (z && mean && rstd && ln_w), "adapter_bwd: LayerNorm inputs");
  CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_adapter_bwd_ws(R, D, A), "adapter_bwd: workspace too small");
  if (R == 0) return CLIPMI_OK;
  const BwdWs p = bwd_plan(R, D, A);
  char* w = (char*)ws;
  const bool bf = dtype == CLIPMI_BF16;
  // dz = dL/dz (the pre-LN sum's gradient); without the LayerNorm dz is dy itself
  const void* dz = dy;
  int64_t lddz = lddy;
  if (ln) {
    CLIPMI_TRY(clipmi_layernorm_bwd(stream, dtype, dy, lddy, z, D, mean, rstd, ln_w, w + p.dz, D, nullptr, 0, g_ln_w,
                                    g_ln_b, 1, w + p.ln, p.col - p.ln, R, D));
    dz = w + p.dz;
    lddz = D;
  }
  void* col_ws = w + p.col;
  const int64_t col_bytes = p.total - p.col;
  // up projection: gW_up[d][a] += sum_r dz[r][d] act[r][a]; gb_up[d] += sum_r dz[r][d]
  if (g_w_up) {
    CLIPMI_TRY(adp_gemm(stream, dtype, D, A, R, dz, lddz, false, act, A, false, g_w_up, A, CLIPMI_F32, CLIPMI_EPI_BETA,
                        nullptr, nullptr, 0, nullptr, 0, bf ? g_b_up : nullptr));
  }
  if (g_b_up && (!g_w_up || !bf)) CLIPMI_TRY(clipmi_colsum(stream, dtype, dz, lddz, R, D, g_b_up, 1, col_ws, col_bytes));
  // d_pre = (dz W_up) * gelu_erf'(pre)   (W_up is [D, A]: row-major in the reduced index d)
  void* dpre = w + p.dpre;
  CLIPMI_TRY(adp_gemm(stream, dtype, R, A, D, dz, lddz, true, w_up, A, false, dpre, A, dtype, CLIPMI_EPI_DGELU, nullptr,
                      nullptr, 0, const_cast<void*>(pre), A));
  // down projection: gW_down[a][d] += sum_r d_pre[r][a] x[r][d]; gb_down[a] += sum_r d_pre[r][a]
  if (g_w_down) {
    CLIPMI_TRY(adp_gemm(stream, dtype, A, D, R, dpre, A, false, x, ldx, false, g_w_down, D, CLIPMI_F32,
                        CLIPMI_EPI_BETA, nullptr, nullptr, 0, nullptr, 0, bf ? g_b_down : nullptr));
  }
  if (g_b_down && (!g_w_down || !bf)) CLIPMI_TRY(clipmi_colsum(stream, dtype, dpre, A, R, A, g_b_down, 1, col_ws, col_bytes));
  // dx = d_pre W_down + dz   (W_down is [A, D]: row-major in the reduced index a)
  CLIPMI_TRY(adp_gemm(stream, dtype, R, D, A, dpre, A, true, w_down, D, false, dx, lddx, dtype, CLIPMI_EPI_RESID,
                      nullptr, dz, lddz));
  return CLIPMI_OK;
}
