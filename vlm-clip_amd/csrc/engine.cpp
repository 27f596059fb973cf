// Native encoder engine: sequences a whole CLIPEncoder (L pre-LN layers) forward and
// backward on one HIP stream with one C-ABI call per direction.
//
// Replaces CLIPEncoder.forward ([HF] modeling_clip.py:477-482) and, through autograd in
// the reference, its backward.  Per layer ([HF] :362-383):
//   ln1 = LN1(x)                      -> clipmi_layernorm_fwd
//   qkv = ln1 Wqkv^T + bqkv           -> GEMM (q/k/v fused into one [3D, D] weight)
//   o   = attention(qkv)              -> clipmi_attention_fwd
//   h   = x + o Wo^T + bo             -> GEMM, residual fused in the epilogue
//   ln2 = LN2(h)
//   a   = quick_gelu(ln2 W1^T + b1)   -> GEMM, bias+activation fused, pre-activation saved
//   y   = h + a W2^T + b2             -> GEMM, residual fused
// Backward mirrors it with dgrad GEMMs (activation derivative fused in the epilogue),
// split-K wgrad GEMMs accumulating straight into the fp32 gradient arena, deterministic
// column sums for biases, and LN backward with the residual gradient fused.
// Activation buffers are caller-owned (per layer for training; one shared set for
// inference), so the engine holds no state and allocates nothing.
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include "internal.h"
#include <atomic>

extern "C" {
int clipmi_layernorm_fwd(void*, int, void*, int64_t, void*, int64_t, const void*, const void*, float*, float*, int, int,
                         float, const void*, const void*, int);
int clipmi_layernorm_fwd2(void*, int, int, void*, int64_t, void*, int64_t, const void*, const void*, float*, float*, int,
                          int, float, const void*, const void*, int);
int clipmi_layernorm_bwd2(void*, int, int, const void*, int64_t, const void*, int64_t, const float*, const float*,
                          const void*, void*, int64_t, const void*, int64_t, float*, float*, int, void*, int64_t, int,
                          int);
int64_t clipmi_layernorm_bwd_ws(int R, int D);
int clipmi_layernorm_bwd(void*, int, const void*, int64_t, const void*, int64_t, const float*, const float*, const void*,
                         void*, int64_t, const void*, int64_t, float*, float*, int, void*, int64_t, int, int);
int64_t clipmi_colsum_ws(int R, int N);
int clipmi_colsum(void*, int, const void*, int64_t, int, int, float*, int, void*, int64_t);
int clipmi_attention_fwd(void*, int, const void*, void*, float*, const int64_t*, int, int, int, int, int);
int clipmi_attention_bwd(void*, int, const void*, const void*, const float*, const void*, void*, const int64_t*, int,
                         int, int, int, int);
int clipmi_quant_mxfp8(void*, int, const void*, int64_t, int64_t, int, uint8_t*, uint8_t*);
int clipmi_attention_fwd_x3(void*, const void*, void*, float*, const int64_t*, int, int, int, int, int);
int clipmi_attention_bwd_x3(void*, const void*, const void*, const float*, const void*, void*, const int64_t*, int,
                            int, int, int, int);
}

namespace {

size_t esize(int dt) { return dt == CLIPMI_F32 ? 4 : 2; }
int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

int gemm(void* s, int dt, int M, int N, int K, const void* A, int64_t lda, bool akm, const void* B, int64_t ldb,
         bool bkm, void* C, int64_t ldc, int c_dt, int flags, const void* bias = nullptr, const void* res = nullptr,
         int64_t ldr = 0, void* aux = nullptr, int64_t ldaux = 0, int split = 1, void* ws = nullptr,
         int64_t ws_bytes = 0, float* bias_grad = nullptr) {
  clipmi_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.a_kmajor = akm;
  d.B = B; d.ldb = ldb; d.b_kmajor = bkm;
  d.C = C; d.ldc = ldc;
  d.bias = bias; d.residual = res; d.ldr = ldr; d.aux = aux; d.ldaux = ldaux;
  d.alpha = 1.f; d.flags = flags;
  d.ab_dtype = dt; d.c_dtype = c_dt; d.bias_dtype = dt;
  d.split_k = split; d.workspace = ws; d.workspace_bytes = ws_bytes;
  d.bias_grad = bias_grad;
  return clipmi_gemm(s, &d);
}

// CUs of the calling thread's current device (cached per device; racing first calls store the same value)
int cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

// split-K factor for a wgrad GEMM [M x N] reducing over K tokens.  bf16 (256x256 tiles, one
// workgroup per CU): the split maximising round efficiency (workgroups / whole rounds of the
// chip's CUs) minus the fp32 slabs' cost (written by the GEMM, read back by the reduce) relative
// to the GEMM's compute time, with >= 512 tokens per slab.  Measured on ViT-B/16 B=1024
// (tools/gemm_bench.py GEMM_SPLITS): qkv (27 tiles) 9 splits = 243 workgroups in one round,
// 676 us, vs 28 splits (756 in three rounds, 3x the slab bytes) 732 us; fc1/fc2 (36 tiles) 7;
// out-proj (9 tiles) 28; text out-proj (4 tiles) 64.
int wgrad_splits(int M, int N, int K, int dt) {
  const int tile = dt == CLIPMI_BF16 ? 256 : 64;
  const int tiles = ((M + tile - 1) / tile) * ((N + tile - 1) / tile);
  if (dt != CLIPMI_BF16) {
    int s = std::max(1, 1024 / std::max(1, tiles));
    s = std::min(s, 32);
    while (s > 1 && (int64_t)K / s < 512) --s;
    return s;
  }
  const int cus = cu_count();
  const double compute_s = 2.0 * M * N * (double)K / (4.1e12 * cus);  // ~1.05 PF/s on 256 CUs
  int best = 1;
  double best_score = -1e30;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && (int64_t)K / s < 512) break;
    const int64_t wg = (int64_t)tiles * s;
    const int64_t rounds = (wg + cus - 1) / cus;
    const double eff = (double)wg / (double)(rounds * cus);
    const double slab_s = s > 1 ? 2.0 * s * M * N * 4.0 / 4.0e12 : 0.0;  // fp32 slabs out + in, ~4 TB/s
    const double score = eff - slab_s / compute_s;
    if (score > best_score + 0.005) {
      best = s;
      best_score = score;
    }
  }
  return best;
}

// ---- bf16x3 mode (fp32 encoder, every GEMM three bf16 products of hi / lo operand splits).  Round 6: the
// activations and activation gradients are split ONCE, by their producer, into images that serve every GEMM
// that reads them, instead of once per GEMM operand:
//   image of X [R][K] (fp32): bf16 [R][3K], segments (h, h, l) ("pattern 0", forward activations) or (h, l, h)
//   ("pattern 1", activation gradients), h = bf16(X), l = bf16(X - h) -- gemm.hip CLIPMI_GEMM_SPLIT3's layout.
//   As a k-major operand it is the 3K-long reduction A3 = [Xh | Xh | Xl]; read as [3R][K] with ld = K (row
//   3r + j = segment j of row r) it is the 3R-long reduction of a weight gradient, where a pattern-1 gradient
//   image against a pattern-0 activation image pairs (h, h), (l, h), (h, l) row by row: the same three products.
//   Weights are split per GEMM (pattern 1 against forward activations, pattern 0 against gradients).
// Producers: LayerNorm writes ln1 / ln2 as images (clipmi_layernorm_fwd_x3); the attention output, fc1's output
// and the four activation gradients are split by clipmi_split3_colsum, which also sums the gradient's columns
// into its Linear's bias gradient.  Per layer 6 split passes (round 5: 24, one per GEMM operand).
// act[l] in this mode: ln1 / ln2 bf16 [R][3D] images; o fp32 [R][D] followed (256-B aligned) by its image; act
// the bf16 [R][3F] image of fc1's output; x_in, qkv, h, pre (quick_gelu') fp32.
struct X3Plan {
  int64_t img, w, slab, col, total;
};
X3Plan x3_plan(const clipmi_encoder_desc* d) {
  const int64_t R = (int64_t)d->B * d->N, D = d->D, F = d->F;
  X3Plan p;
  p.img = 0;  // the live activation-gradient image, or fc1's fp32 output in the forward
  p.w = p.img + align256(std::max(R * 3 * std::max(F, 3 * D) * 2, R * F * 4));
  int64_t wmax = 0;  // weight images: forward k-major [N][3K], input gradient [3N][round8(K)]
  const int ws_[4][2] = {{3 * (int)D, (int)D}, {(int)D, (int)D}, {(int)F, (int)D}, {(int)D, (int)F}};
  for (auto& w : ws_) {
    wmax = std::max(wmax, clipmi_split3_elems(w[0], w[1], 1));
    wmax = std::max(wmax, clipmi_split3_elems(w[1], w[0], 0));
  }
  p.slab = p.w + align256(wmax * 2);
  int64_t smax = 0;
  const int wg[4][2] = {{(int)D, (int)F}, {(int)F, (int)D}, {(int)D, (int)D}, {3 * (int)D, (int)D}};
  for (auto& w : wg) {
    const int sp = wgrad_splits(w[0], w[1], (int)(3 * R), CLIPMI_BF16);
    if (sp > 1) smax = std::max(smax, (int64_t)sp * w[0] * w[1] * 4);
  }
  p.col = p.slab + align256(smax);
  p.total = p.col + align256(std::max({clipmi_split3_colsum_ws((int)R, (int)std::max(3 * D, F)),
                                       clipmi_gemm_x3out_ws((int)R, (int)F),
                                       clipmi_attention_bwd_x3img_ws(d->B, (int)D)}));
  return p;
}
bool x3_mode(const clipmi_encoder_desc* d) { return d->gemm_x3 && d->dtype == CLIPMI_F32; }
int64_t x3_bytes(const clipmi_encoder_desc* d) { return x3_mode(d) ? x3_plan(d).total : 0; }
// the attention output's image, after its fp32 copy in act[l].o
void* x3_o3(const clipmi_layer_act& a, int64_t R, int D) { return (char*)a.o + align256(R * D * 4); }

// bf16 GEMM over split images, fp32 C / bias / residual / aux
int x3_gemm(void* s, int M, int N, int K3, const void* A, int64_t lda, bool akm, const void* B, int64_t ldb, bool bkm,
            void* C, int64_t ldc, int flags, const void* bias = nullptr, const void* res = nullptr, int64_t ldr = 0,
            void* aux = nullptr, int64_t ldaux = 0, int split = 1, void* ws = nullptr, int64_t ws_bytes = 0) {
  clipmi_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.M = M; g.N = N; g.K = K3;
  g.A = A; g.lda = lda; g.a_kmajor = akm;
  g.B = B; g.ldb = ldb; g.b_kmajor = bkm;
  g.C = C; g.ldc = ldc;
  g.bias = bias; g.residual = res; g.ldr = ldr; g.aux = aux; g.ldaux = ldaux;
  g.alpha = 1.f; g.flags = flags;
  g.ab_dtype = CLIPMI_BF16; g.c_dtype = CLIPMI_F32; g.bias_dtype = CLIPMI_F32;
  g.split_k = split; g.workspace = ws; g.workspace_bytes = ws_bytes;
  return clipmi_gemm(s, &g);
}
// the same product with its result written as a split image by the GEMM's epilogue (clipmi_gemm_x3out): C3 bf16
// [M][3N] in pattern `pattern`, colsum (+=) the result's column sums
int x3_gemm_img(void* s, int M, int N, int K3, const void* A, int64_t lda, const void* B, int64_t ldb, bool bkm,
                void* C3, int pattern, int flags, const void* bias, void* aux, int64_t ldaux, float* colsum, void* ws,
                int64_t ws_bytes) {
  clipmi_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.M = M; g.N = N; g.K = K3;
  g.A = A; g.lda = lda; g.a_kmajor = 1;
  g.B = B; g.ldb = ldb; g.b_kmajor = bkm;
  g.C = C3; g.ldc = 3 * (int64_t)N;
  g.bias = bias; g.aux = aux; g.ldaux = ldaux;
  g.alpha = 1.f; g.flags = flags;
  g.ab_dtype = CLIPMI_BF16; g.c_dtype = CLIPMI_F32; g.bias_dtype = CLIPMI_F32;
  g.split_k = 1;
  return clipmi_gemm_x3out(s, &g, pattern, colsum, 1, ws, ws_bytes);
}
// C[R][N] = epi(X3 W^T): X3 the pattern-0 image [R][3K] of the forward activation, W fp32 [N][K]
int x3_fwd(void* s, char* wimg, int R, int N, int K, const void* X3, const void* W, void* C, int64_t ldc, int flags,
           const void* bias, const void* res = nullptr, int64_t ldr = 0, void* aux = nullptr, int64_t ldaux = 0) {
  CLIPMI_TRY(clipmi_split3(s, (const float*)W, K, N, K, 1, wimg, 1));
  return x3_gemm(s, R, N, 3 * K, X3, 3 * (int64_t)K, true, wimg, 3 * (int64_t)K, true, C, ldc, flags, bias, res, ldr,
                 aux, ldaux);
}
// C[R][Kin] = epi(G3 W): G3 the pattern-1 image [R][3 Nout] of an output gradient, W fp32 [Nout][Kin]
int x3_dgrad(void* s, char* wimg, int R, int Kin, int Nout, const void* G3, const void* W, void* C, int64_t ldc,
             int flags, void* aux = nullptr, int64_t ldaux = 0) {
  CLIPMI_TRY(clipmi_split3(s, (const float*)W, Kin, Kin, Nout, 0, wimg, 0));
  return x3_gemm(s, R, Kin, 3 * Nout, G3, 3 * (int64_t)Nout, true, wimg, (Kin + 7) / 8 * 8, false, C, ldc, flags,
                 nullptr, nullptr, 0, aux, ldaux);
}

struct WsPlan {
  int64_t g2, dln, dbig, split, colsum, ln, total;
};

WsPlan plan(const clipmi_encoder_desc* d) {
  const int64_t R = (int64_t)d->B * d->N;
  const size_t es = esize(d->dtype);
  WsPlan p;
  const int64_t big = std::max<int64_t>(3 * d->D, d->F);
  p.g2 = 0;
  p.dln = p.g2 + align256(R * d->D * es);
  p.dbig = p.dln + align256(R * d->D * es);
  p.split = p.dbig + align256(R * big * es);
  int64_t sp = 0;
  const int shapes[4][2] = {{d->F, d->D}, {d->D, d->F}, {d->D, d->D}, {3 * d->D, d->D}};
  for (auto& sh : shapes) {
    const int s = (d->gemm_x3 && d->dtype == CLIPMI_F32) ? 1 : wgrad_splits(sh[0], sh[1], (int)R, d->dtype);
    if (s > 1) sp = std::max<int64_t>(sp, (int64_t)s * sh[0] * (sh[1] + 1) * 4);  // slabs + bias partials
  }
  // bf16: two slab regions used alternately, so a weight gradient's split-K sum can be deferred into the
  // next persistent GEMM while the following weight gradient writes its own slabs (DeferredReduce)
  if (d->dtype == CLIPMI_BF16) sp = 2 * align256(sp);
  p.colsum = p.split + align256(sp);
  p.ln = p.colsum + align256(clipmi_colsum_ws((int)R, (int)big));
  p.total = p.ln + align256(std::max(clipmi_layernorm_bwd_ws((int)R, d->D), clipmi_layernorm_bwd_x3_ws((int)R, d->D)));
  return p;
}

// MXFP8 forward GEMM: C = epi(q8/s8 W^T), A already quantised (q8 [M, K], s8 [M, K/32])
// (c_scale != NULL: C is written as MXFP8 too, scales [M, N/32] in c_scale)
int gemm8q(void* s, int M, int N, int K, const void* q8, const void* s8, const void* Wq, const void* Ws, void* C,
           int64_t ldc, int flags, const void* bias, const void* res, int64_t ldr, uint8_t* c_scale = nullptr) {
  clipmi_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.M = M; d.N = N; d.K = K;
  d.A = q8; d.lda = K; d.a_kmajor = 1;
  d.B = Wq; d.ldb = K; d.b_kmajor = 1;
  d.a_scale = (const uint8_t*)s8; d.b_scale = (const uint8_t*)Ws;
  d.C = C; d.ldc = ldc;
  d.bias = bias; d.residual = res; d.ldr = ldr;
  d.alpha = 1.f; d.flags = flags;
  d.ab_dtype = CLIPMI_FP8; d.c_dtype = c_scale ? CLIPMI_FP8 : CLIPMI_BF16; d.bias_dtype = CLIPMI_BF16;
  d.c_scale = c_scale;
  d.split_k = 1;
  return clipmi_gemm(s, &d);
}
// the same with A [M, K] bf16 quantised into the q8/s8 scratch first
int gemm8(void* s, int M, int N, int K, const void* A, int64_t lda, const void* Wq, const void* Ws, void* C,
          int64_t ldc, int flags, const void* bias, const void* res, int64_t ldr, void* q8, void* s8) {
  CLIPMI_TRY(clipmi_quant_mxfp8(s, CLIPMI_BF16, A, lda, M, K, (uint8_t*)q8, (uint8_t*)s8));
  return gemm8q(s, M, N, K, q8, s8, Wq, Ws, C, ldc, flags, bias, res, ldr);
}

// Deferred-reduction hazard check: a recorded second stage (DeferredReduce) reads its split-K slabs /
// bias partials or LayerNorm partial rows when the next persistent GEMM hosts it, so no launch queued in between
// may write those bytes.  Today's order never does (the two slab regions alternate, ln_guard runs an outstanding
// affine sum before the next LayerNorm backward); this check makes a future reordering or a new launch that breaks
// it fail with CLIPMI_ERR_INVALID instead of silently corrupting a gradient.  Host pointer arithmetic only.
bool overlaps(const void* a, int64_t na, const void* b, int64_t nb) {
  const char* pa = (const char*)a;
  const char* pb = (const char*)b;
  return a && b && na > 0 && nb > 0 && pa < pb + nb && pb < pa + na;
}
int pending_hazard(const DeferredReduce& r, const void* dst, int64_t bytes, const char* what) {
  bool hit = false;
  if (r.kind == 1) {
    hit = overlaps(dst, bytes, r.ws, (int64_t)r.splits * r.M * r.N * 4) ||
          overlaps(dst, bytes, r.bws, (int64_t)r.splits * r.M * 4);
  } else if (r.kind == 2) {
    hit = overlaps(dst, bytes, r.part, (int64_t)r.P * r.stride * 4);
  }
  if (hit) return clipmi_invalid(std::string("encoder_bwd: ") + what + " would overwrite the inputs of a deferred reduction");
  return CLIPMI_OK;
}

int validate(const clipmi_encoder_desc* d) {
  CLIPMI_REQUIRE(d && d->layers && d->act, "null descriptor");
  CLIPMI_REQUIRE(d->dtype == CLIPMI_BF16 || d->dtype == CLIPMI_F32 || d->dtype == CLIPMI_FP8, "dtype");
  CLIPMI_REQUIRE(d->dtype != CLIPMI_FP8 || (d->layers8 && d->q8 && d->s8), "fp8 encoder needs layers8 / q8 / s8");
  CLIPMI_REQUIRE(d->dtype != CLIPMI_FP8 || (d->D % 256 == 0 && d->F % 128 == 0),
                 "fp8 encoder: hidden size must be a multiple of 256 and the MLP width of 128");
  CLIPMI_REQUIRE(d->D == d->H * 64, "hidden size must be heads * 64");
  CLIPMI_REQUIRE(d->B >= 0 && d->N >= 1 && d->L >= 1, "shape");
  CLIPMI_REQUIRE(!d->gemm_x3 || d->dtype == CLIPMI_F32, "gemm_x3 needs the fp32 encoder");
  CLIPMI_REQUIRE(!d->gemm_x3 || (d->x3_ws && d->x3_ws_bytes >= x3_bytes(d) && ((uintptr_t)d->x3_ws & 255) == 0),
                 "gemm_x3: x3_ws too small or not 256-byte aligned (clipmi_encoder_x3_ws)");
  return CLIPMI_OK;
}

int encoder_fwd_x3(void* s, const clipmi_encoder_desc* d) {
  const int R = d->B * d->N, D = d->D, F = d->F;
  const X3Plan pl = x3_plan(d);
  char* ws = (char*)d->x3_ws;
  char* wimg = ws + pl.w;
  float* fc1o = (float*)(ws + pl.img);  // fc1's fp32 output before its split
  for (int l = 0; l < d->L; ++l) {
    const clipmi_layer_w& w = d->layers[l];
    const clipmi_layer_act& a = d->act[l];
    void* x_out = (l + 1 < d->L) ? d->act[l + 1].x_in : d->x_out;
    void* o3 = x3_o3(a, R, D);
    CLIPMI_TRY(clipmi_layernorm_fwd_x3(s, (const float*)a.x_in, D, a.ln1, 0, (const float*)w.ln1_w,
                                       (const float*)w.ln1_b, a.mean1, a.rstd1, R, D, d->eps));
    CLIPMI_TRY(x3_fwd(s, wimg, R, 3 * D, D, a.ln1, w.qkv_w, a.qkv, 3 * D, CLIPMI_EPI_BIAS, w.qkv_b));
    if (d->N <= 288) {  // O and its image from the attention kernel
      CLIPMI_TRY(clipmi_attention_fwd_x3img(s, a.qkv, a.o, o3, a.lse, d->attention_mask, d->causal, d->B, d->H, d->N,
                                            D));
    } else {
      CLIPMI_TRY(clipmi_attention_fwd_x3(s, a.qkv, a.o, a.lse, d->attention_mask, d->causal, d->B, d->H, d->N, D));
      CLIPMI_TRY(clipmi_split3_colsum(s, (const float*)a.o, D, R, D, o3, 0, nullptr, 0, nullptr, 0));
    }
    CLIPMI_TRY(x3_fwd(s, wimg, R, D, D, o3, w.out_w, a.h, D, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, w.out_b, a.x_in, D));
    CLIPMI_TRY(clipmi_layernorm_fwd_x3(s, (const float*)a.h, D, a.ln2, 0, (const float*)w.ln2_w,
                                       (const float*)w.ln2_b, a.mean2, a.rstd2, R, D, d->eps));
    const int f1 = CLIPMI_EPI_BIAS | CLIPMI_EPI_QGELU | (a.pre ? CLIPMI_EPI_STORE_DACT : 0);
    if (clipmi_gemm_x3out_ok(R, F, 3 * D, 1, 1, f1)) {  // the act image written by fc1's epilogue
      CLIPMI_TRY(clipmi_split3(s, (const float*)w.fc1_w, D, F, D, 1, wimg, 1));
      CLIPMI_TRY(x3_gemm_img(s, R, F, 3 * D, a.ln2, 3 * (int64_t)D, wimg, 3 * (int64_t)D, true, a.act, 0, f1, w.fc1_b,
                             a.pre, F, nullptr, nullptr, 0));
    } else {
      CLIPMI_TRY(x3_fwd(s, wimg, R, F, D, a.ln2, w.fc1_w, fc1o, F, f1, w.fc1_b, nullptr, 0, a.pre, F));
      CLIPMI_TRY(clipmi_split3_colsum(s, fc1o, F, R, F, a.act, 0, nullptr, 0, nullptr, 0));
    }
    CLIPMI_TRY(x3_fwd(s, wimg, R, D, F, a.act, w.fc2_w, x_out, D, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, w.fc2_b, a.h, D));
  }
  return CLIPMI_OK;
}

int encoder_bwd_x3(void* s, const clipmi_encoder_desc* d, void* dx, int layer_hi, int layer_lo) {
  const int R = d->B * d->N, D = d->D, F = d->F;
  const WsPlan p = plan(d);
  CLIPMI_REQUIRE(d->workspace && d->workspace_bytes >= p.total, "encoder_bwd workspace too small");
  char* bws = (char*)d->workspace;
  float* g2 = (float*)(bws + p.g2);
  float* dln = (float*)(bws + p.dln);
  float* dbig = (float*)(bws + p.dbig);
  void* wln = bws + p.ln;
  const int64_t ln_bytes = p.total - p.ln;
  const X3Plan pl = x3_plan(d);
  char* ws = (char*)d->x3_ws;
  void* gimg = ws + pl.img;  // the live activation-gradient image
  char* wimg = ws + pl.w;
  void* slab = ws + pl.slab;
  void* col = ws + pl.col;
  const int64_t slab_bytes = pl.col - pl.slab, col_bytes = pl.total - pl.col;
  // gradient image of G [R][N] (pattern 1) into gimg, its column sums added to the bias gradient
  auto split_g = [&](const float* G, int N, float* bgrad) -> int {
    return clipmi_split3_colsum(s, G, N, R, N, gimg, 1, bgrad, 1, col, col_bytes);
  };
  // C[M][N] += sum over the 3R interleaved rows of G3^T X3 (G3: gradient image, X3: activation image)
  auto wgrad = [&](int M, int N, const void* G3, const void* X3, float* C) -> int {
    const int sp = wgrad_splits(M, N, 3 * R, CLIPMI_BF16);
    return x3_gemm(s, M, N, 3 * R, G3, M, false, X3, N, false, C, N, CLIPMI_EPI_BETA, nullptr, nullptr, 0, nullptr, 0,
                   sp, sp > 1 ? slab : nullptr, sp > 1 ? slab_bytes : 0);
  };
  // fc2's input gradient writes d_pre's image itself where the fused form exists (dbig holds dx's image, 6 D B per
  // row, inside its 4 max(3D, F) B)
  const bool fuse_dpre = clipmi_gemm_x3out_ok(R, F, 3 * D, 1, 0, CLIPMI_EPI_MUL_AUX) && 3 * D <= 2 * std::max(3 * D, F);
  // the LayerNorm backwards write their dx's image and its column sums too (clipmi_layernorm_bwd_x3): LN2's into gimg
  // (dh, the out-projection's gradient) and LN1's into dbig (the next layer's dx) where fuse_dpre keeps it there
  const bool ln_x3 = D % 64 == 0 && (D / 64 == 1 || D / 64 == 2 || D / 64 == 3 || D / 64 == 4 || D / 64 == 6 ||
                                     D / 64 == 8 || D / 64 == 12 || D / 64 == 16);
  bool dx_img = false;  // dbig holds dx's image and this layer's fc2 bias gradient already has its column sums
  for (int l = layer_hi - 1; l >= layer_lo; --l) {
    const clipmi_layer_w& w = d->layers[l];
    const clipmi_layer_act& a = d->act[l];
    const clipmi_layer_grad& g = d->grads[l];
    CLIPMI_REQUIRE(a.pre, "training forward must save pre-activations");
    // MLP branch: dx is dL/dy
    if (fuse_dpre) {  // d_pre's image written by fc2's input-gradient epilogue; dx's image in dbig meanwhile
      if (!dx_img)
        CLIPMI_TRY(clipmi_split3_colsum(s, (const float*)dx, D, R, D, dbig, 1, g.fc2_b, 1, col, col_bytes));  // gb2
      CLIPMI_TRY(clipmi_split3(s, (const float*)w.fc2_w, F, F, D, 0, wimg, 0));
      CLIPMI_TRY(x3_gemm_img(s, R, F, 3 * D, dbig, 3 * (int64_t)D, wimg, (F + 7) / 8 * 8, false, gimg, 1,
                             CLIPMI_EPI_MUL_AUX, nullptr, a.pre, F, g.fc1_b, col, col_bytes));  // d_pre, gb1
      CLIPMI_TRY(wgrad(D, F, dbig, a.act, g.fc2_w));                                        // gW2 += dx^T act
    } else {
      CLIPMI_TRY(split_g((const float*)dx, D, g.fc2_b));                                    // gb2 += sum dx
      CLIPMI_TRY(x3_dgrad(s, wimg, R, F, D, gimg, w.fc2_w, dbig, F, CLIPMI_EPI_MUL_AUX, a.pre, F));  // d_pre
      CLIPMI_TRY(wgrad(D, F, gimg, a.act, g.fc2_w));                                        // gW2 += dx^T act
      CLIPMI_TRY(split_g(dbig, F, g.fc1_b));                                                // gb1 += sum d_pre
    }
    CLIPMI_TRY(wgrad(F, D, gimg, a.ln2, g.fc1_w));                                          // gW1 += d_pre^T ln2
    CLIPMI_TRY(x3_dgrad(s, wimg, R, D, F, gimg, w.fc1_w, dln, D, 0));                       // d_ln2 = d_pre W1
    if (ln_x3) {  // dh = dx + LN2'(d_ln2), its image into gimg, gbo += sum dh
      CLIPMI_TRY(clipmi_layernorm_bwd_x3(s, dln, D, (const float*)a.h, D, a.mean2, a.rstd2, (const float*)w.ln2_w, g2,
                                         D, (const float*)dx, D, g.ln2_w, g.ln2_b, 1, gimg, g.out_b, 1, wln, ln_bytes,
                                         R, D));
    } else {
      CLIPMI_TRY(clipmi_layernorm_bwd2(s, CLIPMI_F32, CLIPMI_F32, dln, D, a.h, D, a.mean2, a.rstd2, w.ln2_w, g2, D, dx,
                                       D, g.ln2_w, g.ln2_b, 1, wln, ln_bytes, R, D));        // dh = dx + LN2'(d_ln2)
      CLIPMI_TRY(split_g(g2, D, g.out_b));                                                  // gbo += sum dh
    }
    // attention branch: g2 is dL/dh
    CLIPMI_TRY(x3_dgrad(s, wimg, R, D, D, gimg, w.out_w, dln, D, 0));                       // d_o = dh Wo
    CLIPMI_TRY(wgrad(D, D, gimg, x3_o3(a, R, D), g.out_w));                                 // gWo += dh^T o
    if (d->N <= 288) {  // d_qkv's image and gbqkv written by the attention backward itself
      CLIPMI_TRY(clipmi_attention_bwd_x3img(s, a.qkv, a.o, a.lse, dln, gimg, g.qkv_b, 1, col, col_bytes,
                                            d->attention_mask, d->causal, d->B, d->H, d->N, D));
    } else {
      CLIPMI_TRY(clipmi_attention_bwd_x3(s, a.qkv, a.o, a.lse, dln, dbig, d->attention_mask, d->causal, d->B, d->H,
                                         d->N, D));                                         // d_qkv
      CLIPMI_TRY(split_g(dbig, 3 * D, g.qkv_b));                                            // gbqkv += sum d_qkv
    }
    CLIPMI_TRY(wgrad(3 * D, D, gimg, a.ln1, g.qkv_w));                                      // gWqkv += d_qkv^T ln1
    CLIPMI_TRY(x3_dgrad(s, wimg, R, D, 3 * D, gimg, w.qkv_w, dln, D, 0));                   // d_ln1
    dx_img = fuse_dpre && ln_x3 && l > layer_lo;
    if (dx_img) {  // dx_in = dh + LN1'(d_ln1), its image into dbig, layer l - 1's gb2 += sum dx_in
      CLIPMI_TRY(clipmi_layernorm_bwd_x3(s, dln, D, (const float*)a.x_in, D, a.mean1, a.rstd1, (const float*)w.ln1_w,
                                         (float*)dx, D, g2, D, g.ln1_w, g.ln1_b, 1, dbig, d->grads[l - 1].fc2_b, 1,
                                         wln, ln_bytes, R, D));
    } else {
      CLIPMI_TRY(clipmi_layernorm_bwd2(s, CLIPMI_F32, CLIPMI_F32, dln, D, a.x_in, D, a.mean1, a.rstd1, w.ln1_w, dx, D,
                                       g2, D, g.ln1_w, g.ln1_b, 1, wln, ln_bytes, R, D));   // dx_in = dh + LN1'(d_ln1)
    }
  }
  return CLIPMI_OK;
}

}  // namespace

extern "C" int64_t clipmi_encoder_bwd_ws(const clipmi_encoder_desc* d) { return plan(d).total; }
extern "C" int64_t clipmi_encoder_x3_ws(const clipmi_encoder_desc* d) { return d ? x3_bytes(d) : 0; }

extern "C" int clipmi_encoder_fwd(void* s, const clipmi_encoder_desc* d) {
  CLIPMI_TRY(validate(d));
  const int dt = d->dtype;
  const int R = d->B * d->N, D = d->D, F = d->F;
  if (R == 0) return CLIPMI_OK;
  if (x3_mode(d)) return encoder_fwd_x3(s, d);
  if (dt == CLIPMI_FP8) {  // BASELINE config 5: frozen towers, MXFP8 GEMMs, bf16 everything else
    const int bf = CLIPMI_BF16;
    // scratch: [R, D] operand (LayerNorm / attention outputs) then [R, F] (fc1 output), each with its scales
    uint8_t* qa = (uint8_t*)d->q8;
    uint8_t* sa = (uint8_t*)d->s8;
    uint8_t* qb = qa + align256((int64_t)R * D);
    uint8_t* sb = sa + align256((int64_t)R * D / 32);
    for (int l = 0; l < d->L; ++l) {
      const clipmi_layer_w& w = d->layers[l];
      const clipmi_layer_w8& w8 = d->layers8[l];
      const clipmi_layer_act& a = d->act[l];
      void* x_out = (l + 1 < d->L) ? d->act[l + 1].x_in : d->x_out;
      // producers write the next GEMM's MXFP8 operand directly (no bf16 round trip); the attention
      // output too where the streaming forward runs (N > 288)
      CLIPMI_TRY(clipmi_layernorm_fwd_mxfp8(s, bf, a.x_in, D, qa, sa, w.ln1_w, w.ln1_b, a.mean1, a.rstd1, R, D, d->eps));
      CLIPMI_TRY(gemm8q(s, R, 3 * D, D, qa, sa, w8.qkv_w, w8.qkv_s, a.qkv, 3 * D, CLIPMI_EPI_BIAS, w.qkv_b, nullptr, 0));
      if (d->N > 288) {  // the streaming forward writes the out-projection's MXFP8 operand itself
        CLIPMI_TRY(clipmi_attention_fwd_mxfp8(s, a.qkv, qa, sa, a.lse, d->attention_mask, d->causal, d->B, d->H, d->N,
                                              D));
        CLIPMI_TRY(gemm8q(s, R, D, D, qa, sa, w8.out_w, w8.out_s, a.h, D, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, w.out_b,
                          a.x_in, D));
      } else {  // the whole-K/V kernels (N <= 288) write bf16 O, quantised by its own pass
        CLIPMI_TRY(clipmi_attention_fwd(s, bf, a.qkv, a.o, a.lse, d->attention_mask, d->causal, d->B, d->H, d->N, D));
        CLIPMI_TRY(gemm8(s, R, D, D, a.o, D, w8.out_w, w8.out_s, a.h, D, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, w.out_b,
                         a.x_in, D, qa, sa));
      }
      CLIPMI_TRY(clipmi_layernorm_fwd_mxfp8(s, bf, a.h, D, qa, sa, w.ln2_w, w.ln2_b, a.mean2, a.rstd2, R, D, d->eps));
      CLIPMI_TRY(gemm8q(s, R, F, D, qa, sa, w8.fc1_w, w8.fc1_s, qb, F, CLIPMI_EPI_BIAS | CLIPMI_EPI_QGELU, w.fc1_b,
                        nullptr, 0, sb));
      CLIPMI_TRY(gemm8q(s, R, D, F, qb, sb, w8.fc2_w, w8.fc2_s, x_out, D, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID, w.fc2_b,
                        a.h, D));
    }
    return CLIPMI_OK;
  }
  // the residual stream's dtype: fp32 in the bf16 mode with resid_f32 (x_in, h, x_out), else dt
  const int xdt = (dt == CLIPMI_BF16 && d->resid_f32) ? CLIPMI_F32 : dt;
  for (int l = 0; l < d->L; ++l) {
    const clipmi_layer_w& w = d->layers[l];
    const clipmi_layer_act& a = d->act[l];
    void* x_out = (l + 1 < d->L) ? d->act[l + 1].x_in : d->x_out;
    CLIPMI_TRY(clipmi_layernorm_fwd2(s, xdt, dt, a.x_in, D, a.ln1, D, w.ln1_w, w.ln1_b, a.mean1, a.rstd1, R, D, d->eps,
                                     nullptr, nullptr, 0));
    CLIPMI_TRY(gemm(s, dt, R, 3 * D, D, a.ln1, D, true, w.qkv_w, D, true, a.qkv, 3 * D, dt, CLIPMI_EPI_BIAS, w.qkv_b));
    CLIPMI_TRY(clipmi_attention_fwd(s, dt, a.qkv, a.o, a.lse, d->attention_mask, d->causal, d->B, d->H, d->N, D));
    CLIPMI_TRY(gemm(s, dt, R, D, D, a.o, D, true, w.out_w, D, true, a.h, D, xdt, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID,
                    w.out_b, a.x_in, D));
    CLIPMI_TRY(clipmi_layernorm_fwd2(s, xdt, dt, a.h, D, a.ln2, D, w.ln2_w, w.ln2_b, a.mean2, a.rstd2, R, D, d->eps,
                                     nullptr, nullptr, 0));
    // training: a.pre receives quick_gelu'(pre) (computed beside the activation from the fp32
    // pre-activation), so fc2's input gradient below is one product per element
    const int f1 = CLIPMI_EPI_BIAS | CLIPMI_EPI_QGELU | (a.pre ? CLIPMI_EPI_STORE_DACT : 0);
    CLIPMI_TRY(gemm(s, dt, R, F, D, a.ln2, D, true, w.fc1_w, D, true, a.act, F, dt, f1, w.fc1_b, nullptr, 0, a.pre, F));
    CLIPMI_TRY(gemm(s, dt, R, D, F, a.act, F, true, w.fc2_w, F, true, x_out, D, xdt, CLIPMI_EPI_BIAS | CLIPMI_EPI_RESID,
                    w.fc2_b, a.h, D));
  }
  return CLIPMI_OK;
}

// dx: gradient w.r.t. the encoder output on entry; overwritten with the gradient w.r.t.
// the encoder input (layer 0's x_in) on exit.  Grads accumulate into d->grads (fp32).
extern "C" int clipmi_encoder_bwd(void* s, const clipmi_encoder_desc* d, void* dx) {
  CLIPMI_TRY(validate(d));
  return clipmi_encoder_bwd_layers(s, d, dx, d->L, 0);
}

// Layers layer_hi-1 down to layer_lo only: the data-parallel path calls the backward in chunks and
// all-reduces each chunk's (contiguous) gradient slice while the next chunk computes.
extern "C" int clipmi_encoder_bwd_layers(void* s, const clipmi_encoder_desc* d, void* dx, int layer_hi, int layer_lo) {
  CLIPMI_TRY(validate(d));
  CLIPMI_REQUIRE(d->dtype != CLIPMI_FP8, "the fp8 encoder is forward-only (frozen towers)");
  CLIPMI_REQUIRE(0 <= layer_lo && layer_lo <= layer_hi && layer_hi <= d->L, "layer range");
  CLIPMI_REQUIRE(d->grads, "encoder_bwd needs gradient destinations");
  const int dt = d->dtype;
  const int xdt = (dt == CLIPMI_BF16 && d->resid_f32) ? CLIPMI_F32 : dt;  // the saved x_in / h
  const int R = d->B * d->N, D = d->D, F = d->F;
  if (R == 0) return CLIPMI_OK;
  if (x3_mode(d)) return encoder_bwd_x3(s, d, dx, layer_hi, layer_lo);
  const WsPlan p = plan(d);
  CLIPMI_REQUIRE(d->workspace && d->workspace_bytes >= p.total, "encoder_bwd workspace too small");
  char* ws = (char*)d->workspace;
  void* g2 = ws + p.g2;
  void* dln = ws + p.dln;
  void* dbig = ws + p.dbig;
  void* wsplit = ws + p.split;
  void* wcol = ws + p.colsum;
  void* wln = ws + p.ln;
  const int64_t split_bytes = p.colsum - p.split;
  const int64_t col_bytes = p.ln - p.colsum;
  const int64_t ln_bytes = p.total - p.ln;
  const int f32 = CLIPMI_F32;
  // bf16: the second stages of the split-K weight gradients and of the LayerNorm affine gradients are
  // deferred into the next persistent GEMM launch (internal.h DeferredReduce; at most one outstanding,
  // the rest launch as usual), the last one launched at the end of this call
  DeferredReduce pend;
  memset(&pend, 0, sizeof(pend));
  const char* denv = getenv("CLIPMI_DEFER");  // 0: launch every reduction on its own (A/B, bitwise test)
  struct Slot {
    explicit Slot(DeferredReduce* r) { deferred_slot() = r; }
    ~Slot() { deferred_slot() = nullptr; }
  } slot(dt == CLIPMI_BF16 && !(denv && denv[0] == '0') ? &pend : nullptr);
  const int64_t region = dt == CLIPMI_BF16 ? split_bytes / 2 : split_bytes;
  int wg_no = 0;
  // wgrad: C[M,N] += sum_tokens A[t][m] B[t][n]; the bf16 path also fuses the Linear bias
  // gradient (sum_tokens A[t][m]) into the same GEMM, fp32 uses a column-sum pass
  auto wgrad = [&](int M, int N, const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                   float* bgrad) -> int {
    const int sp = wgrad_splits(M, N, R, d->dtype);
    const bool fuse = dt == CLIPMI_BF16;
    char* wsl = (char*)wsplit + (dt == CLIPMI_BF16 ? (wg_no++ & 1) * region : 0);
    // an outstanding split-K sum still reading this region runs first (not reached with the alternation)
    if (pend.kind == 1 && (const char*)pend.ws >= wsl && (const char*)pend.ws < wsl + region)
      CLIPMI_TRY(launch_deferred((hipStream_t)s, pend));
    CLIPMI_TRY(pending_hazard(pend, wsl, region, "a weight gradient's split-K slabs"));
    CLIPMI_TRY(gemm(s, dt, M, N, R, A, lda, false, B, ldb, false, C, N, f32, CLIPMI_EPI_BETA, nullptr, nullptr, 0,
                    nullptr, 0, sp, wsl, region, fuse ? bgrad : nullptr));
    if (!fuse) CLIPMI_TRY(clipmi_colsum(s, dt, A, lda, R, M, bgrad, 1, wcol, col_bytes));
    return CLIPMI_OK;
  };
  // LayerNorm backward rewrites the partial rows an outstanding affine sum reads: run that one first
  auto ln_guard = [&]() -> int {
    if (pend.kind == 2) CLIPMI_TRY(launch_deferred((hipStream_t)s, pend));
    return pending_hazard(pend, wln, ln_bytes, "a LayerNorm backward's partial rows");
  };
  // the activation-gradient buffers every other launch of the loop writes (dbig, dln, g2, and the caller's dx) must
  // lie outside the regions a deferred reduction reads (the split-K slabs, the LayerNorm partial rows)
  {
    const int64_t es_ = (int64_t)esize(dt);
    const void* dst[4] = {dbig, dln, g2, dx};
    const int64_t nb[4] = {(int64_t)R * std::max(3 * D, F) * es_, (int64_t)R * D * es_, (int64_t)R * D * es_,
                           (int64_t)R * D * es_};
    for (int i = 0; i < 4; ++i)
      CLIPMI_REQUIRE(!overlaps(dst[i], nb[i], wsplit, split_bytes) && !overlaps(dst[i], nb[i], wln, ln_bytes),
                     "an activation-gradient buffer overlaps the deferred reductions' slabs / partial rows");
  }
  for (int l = layer_hi - 1; l >= layer_lo; --l) {
    const clipmi_layer_w& w = d->layers[l];
    const clipmi_layer_act& a = d->act[l];
    const clipmi_layer_grad& g = d->grads[l];
    CLIPMI_REQUIRE(a.pre, "training forward must save pre-activations");
    // MLP branch: dx is dL/dy
    CLIPMI_TRY(gemm(s, dt, R, F, D, dx, D, true, w.fc2_w, F, false, dbig, F, dt, CLIPMI_EPI_MUL_AUX, nullptr, nullptr,
                    0, a.pre, F));                                          // d_pre = (dx W2) * qgelu'(pre)
    CLIPMI_TRY(wgrad(D, F, dx, D, a.act, F, g.fc2_w, g.fc2_b));            // gW2 += dx^T act, gb2 += sum dx
    CLIPMI_TRY(wgrad(F, D, dbig, F, a.ln2, D, g.fc1_w, g.fc1_b));          // gW1 += d_pre^T ln2
    CLIPMI_TRY(gemm(s, dt, R, D, F, dbig, F, true, w.fc1_w, D, false, dln, D, dt, 0));  // d_ln2 = d_pre W1
    CLIPMI_TRY(ln_guard());
    CLIPMI_TRY(clipmi_layernorm_bwd2(s, xdt, dt, dln, D, a.h, D, a.mean2, a.rstd2, w.ln2_w, g2, D, dx, D, g.ln2_w,
                                     g.ln2_b, 1, wln, ln_bytes, R, D));   // dh = dx + LN2'(d_ln2)
    // attention branch: g2 is dL/dh
    CLIPMI_TRY(gemm(s, dt, R, D, D, g2, D, true, w.out_w, D, false, dln, D, dt, 0));     // d_o = dh Wo
    CLIPMI_TRY(wgrad(D, D, g2, D, a.o, D, g.out_w, g.out_b));                            // gWo += dh^T o
    CLIPMI_TRY(clipmi_attention_bwd(s, dt, a.qkv, a.o, a.lse, dln, dbig, d->attention_mask, d->causal, d->B, d->H,
                                    d->N, D));                              // d_qkv
    CLIPMI_TRY(wgrad(3 * D, D, dbig, 3 * D, a.ln1, D, g.qkv_w, g.qkv_b));  // gWqkv += d_qkv^T ln1
    CLIPMI_TRY(gemm(s, dt, R, D, 3 * D, dbig, 3 * D, true, w.qkv_w, D, false, dln, D, dt, 0));  // d_ln1
    CLIPMI_TRY(ln_guard());
    CLIPMI_TRY(clipmi_layernorm_bwd2(s, xdt, dt, dln, D, a.x_in, D, a.mean1, a.rstd1, w.ln1_w, dx, D, g2, D, g.ln1_w,
                                     g.ln1_b, 1, wln, ln_bytes, R, D));    // dx_in = dh + LN1'(d_ln1)
  }
  if (pend.kind != 0) CLIPMI_TRY(launch_deferred((hipStream_t)s, pend));  // this call's gradients are final
  return CLIPMI_OK;
}
