// Image x text contrastive head: L2 normalisation and symmetric InfoNCE.
//
// Replaces CLIPWithAdapters.forward's contrastive branch (model_m.py:146-171):
//   t^ = t/|t|, i^ = i/|i|                      (:148-149)
//   logits_per_text = exp(logit_scale) t^ i^T   (:152-155), logits_per_image = its transpose
//   loss = (CE(lpt, arange) + CE(lpt^T, arange)) / 2   (:159-163)
// Data-parallel form: a rank holds B local rows and the all-gathered
// [Bg, E] features of the other modality; both directions are computed as row-wise CE
// over [B, Bg] score blocks with label offset rank*B, normalised by 2*Bg so the sum of
// the ranks' losses is the single-device loss.  logit_scale stays on the device (it is
// trainable in full fine-tune), so no host synchronisation happens anywhere.
// The [B, Bg] cosine blocks come from the f32 GEMM (exact f32); these kernels do the
// per-row softmax statistics.  All contrastive arithmetic is fp32, with the accurate expf / logf
// (not the 1-2 ulp __expf / __logf): at small B the loss gradient is a difference of nearly
// equal softmax terms (config 3 at B = 2: text rows identical under quirk Q1, p ~ 0.5), and
// the fast forms amplified to ~1e-3 relative error in every vision gradient; this head is < 1 %
// of a step.
#include "common.h"
#include "internal.h"

namespace {

__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* x, float* y, float* nrm, int B, int E) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  float s = 0.f;
  for (int c = lane; c < E; c += 64) { float v = x[(int64_t)row * E + c]; s += v * v; }
  const float n = sqrtf(wave_sum(s));
  const float inv = 1.f / n;
  for (int c = lane; c < E; c += 64) y[(int64_t)row * E + c] = x[(int64_t)row * E + c] * inv;
  if (lane == 0) nrm[row] = n;
}

// dx = (dy - y (y . dy)) / |x|
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* dy, const float* y, const float* nrm, float* dx,
                                                         int B, int E) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  float s = 0.f;
  for (int c = lane; c < E; c += 64) s += y[(int64_t)row * E + c] * dy[(int64_t)row * E + c];
  s = wave_sum(s);
  const float inv = 1.f / nrm[row];
  for (int c = lane; c < E; c += 64) {
    const int64_t i = (int64_t)row * E + c;
    dx[i] = (dy[i] - y[i] * s) * inv;
  }
}

// logits = exp(ls) * S (written to L); lse[i]; ce[i] = lse[i] - L[i][label0 + i]
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* S, float* L, const float* logit_scale, int B, int Bg,
                                                     int label0, float* lse_out, float* ce_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float sc = expf(*logit_scale);
  const float* s = S + (int64_t)row * Bg;
  float* l = L + (int64_t)row * Bg;
  float mx = -__builtin_huge_valf();
  for (int j = lane; j < Bg; j += 64) { float v = s[j] * sc; l[j] = v; mx = fmaxf(mx, v); }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Bg; j += 64) sum += expf(l[j] - mx);
  sum = wave_sum(sum);
  if (lane == 0) {
    const float lse = mx + logf(sum);
    lse_out[row] = lse;
    ce_out[row] = lse - l[label0 + row];
  }
}

// dS = gout * exp(ls) * (softmax(L) - onehot) / (2 Bg) ; dls_row = sum_j dL_ij (L_ij - lse_i)
// (= sum_j dL_ij L_ij, since sum_j dL_ij = 0 in exact arithmetic: centring the logits on the row's lse keeps
// the terms O(log Bg) instead of O(L), so the softmax-weighted mean and the label logit -- nearly equal when the
// loss sits near ln Bg -- no longer cancel at the logits' magnitude in fp32; B = 2 fixture: logit_scale
// gradient 8.9e-4 -> see tests/test_gpu_model.py::test_b16_full_finetune_gradients_fp32)
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* L, const float* lse, const float* logit_scale,
                                                     const float* gout, int B, int Bg, int label0, float norm,
                                                     float* dS, float* dls_row) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float sc = expf(*logit_scale);
  const float g = (gout ? *gout : 1.f) * norm;
  const float* l = L + (int64_t)row * Bg;
  float* d = dS + (int64_t)row * Bg;
  const float ls = lse[row];
  float acc = 0.f;
  for (int j = lane; j < Bg; j += 64) {
    float dl = g * (expf(l[j] - ls) - (j == label0 + row ? 1.f : 0.f));
    acc += dl * (l[j] - ls);
    d[j] = dl * sc;
  }
  acc = wave_sum(acc);
  if (lane == 0) dls_row[row] = acc;
}

// Column-streamed form (config 5: Bg = 32768 at B = 4096/GPU): the [B, Bg] blocks are never
// materialised; the caller walks column chunks [col0, col0 + C) of the cosine block.  Forward:
// each chunk's row max / sum of exponentials merge into a running (max, sum) pair per row
// (online log-sum-exp), and the label logit is kept when the label column falls in the chunk.
// Backward: the same chunk is recomputed and turned into its dS slice.  Logits are formed as in
// ce_fwd_kernel (v = S * exp(ls)), so a single chunk reproduces the unchunked kernels exactly.
__global__ __launch_bounds__(256) void ce_fwd_chunk_kernel(const float* S, const float* logit_scale, int B, int C,
                                                           int col0, int label0, float* run, float* lab) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float sc = expf(*logit_scale);
  const float* s = S + (int64_t)row * C;
  float mx = -__builtin_huge_valf();
  for (int j = lane; j < C; j += 64) mx = fmaxf(mx, s[j] * sc);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < C; j += 64) sum += expf(s[j] * sc - mx);
  sum = wave_sum(sum);
  if (lane == 0) {
    float* r = run + 2 * (int64_t)row;
    if (col0 == 0) {
      r[0] = mx;
      r[1] = sum;
    } else {
      const float m = fmaxf(r[0], mx);
      r[1] = r[1] * expf(r[0] - m) + sum * expf(mx - m);
      r[0] = m;
    }
    const int lc = label0 + row - col0;
    if (lc >= 0 && lc < C) lab[row] = s[lc] * sc;
  }
}

__global__ __launch_bounds__(256) void ce_finish_kernel(const float* run, const float* lab, int B, float* lse_out,
                                                        float* ce_out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  const float lse = run[2 * row] + logf(run[2 * row + 1]);
  lse_out[row] = lse;
  ce_out[row] = lse - lab[row];
}

// one chunk of ce_bwd_kernel from the cosines: dS[:, 0:C) of columns col0.., dls_row (+)= its share
__global__ __launch_bounds__(256) void ce_bwd_chunk_kernel(const float* S, const float* lse, const float* logit_scale,
                                                           const float* gout, int B, int C, int col0, int label0,
                                                           float norm, float* dS, float* dls_row, int beta) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float sc = expf(*logit_scale);
  const float g = (gout ? *gout : 1.f) * norm;
  const float* s = S + (int64_t)row * C;
  float* d = dS + (int64_t)row * C;
  const float ls = lse[row];
  const int lc = label0 + row - col0;
  float acc = 0.f;
  for (int j = lane; j < C; j += 64) {
    const float l = s[j] * sc;
    const float dl = g * (expf(l - ls) - (j == lc ? 1.f : 0.f));
    acc += dl * (l - ls);
    d[j] = dl * sc;
  }
  acc = wave_sum(acc);
  if (lane == 0) dls_row[row] = beta ? dls_row[row] + acc : acc;
}

// out[0] = scale * sum(a[0:n]) + scale * sum(b[0:n]) ; (beta) accumulate
__global__ __launch_bounds__(1024) void sum2_kernel(const float* a, const float* b, int n, float scale, float* out,
                                                    int beta) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += a[i] + (b ? b[i] : 0.f);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    out[0] = beta ? out[0] + t * scale : t * scale;
  }
}

}  // namespace

extern "C" int clipmi_l2norm_fwd(void* stream, const float* x, float* y, float* nrm, int B, int E) {
  hipLaunchKernelGGL(l2norm_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, y, nrm, B, E);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_l2norm_bwd(void* stream, const float* dy, const float* y, const float* nrm, float* dx, int B,
                                 int E) {
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, dy, y, nrm, dx, B, E);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_contrastive_ce_fwd(void* stream, const float* S, float* logits, const float* logit_scale, int B,
                                         int Bg, int label0, float* lse, float* ce) {
  CLIPMI_REQUIRE(label0 >= 0 && label0 + B <= Bg, "label offset out of range");
  hipLaunchKernelGGL(ce_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, logits, logit_scale, B, Bg,
                     label0, lse, ce);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_contrastive_ce_bwd(void* stream, const float* logits, const float* lse, const float* logit_scale,
                                         const float* grad_out, int B, int Bg, int label0, float norm, float* dS,
                                         float* dls_row) {
  CLIPMI_REQUIRE(label0 >= 0 && label0 + B <= Bg, "label offset out of range");
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, logits, lse, logit_scale,
                     grad_out, B, Bg, label0, norm, dS, dls_row);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_contrastive_ce_fwd_chunk(void* stream, const float* S, const float* logit_scale, int B, int C,
                                               int col0, int Bg, int label0, float* run, float* lab) {
  CLIPMI_REQUIRE(label0 >= 0 && label0 + B <= Bg, "label offset out of range");
  CLIPMI_REQUIRE(C > 0 && col0 >= 0 && col0 + C <= Bg, "chunk out of range");
  hipLaunchKernelGGL(ce_fwd_chunk_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, logit_scale, B, C,
                     col0, label0, run, lab);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_contrastive_ce_finish(void* stream, const float* run, const float* lab, int B, float* lse,
                                            float* ce) {
  hipLaunchKernelGGL(ce_finish_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, run, lab, B, lse, ce);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_contrastive_ce_bwd_chunk(void* stream, const float* S, const float* lse, const float* logit_scale,
                                               const float* grad_out, int B, int C, int col0, int Bg, int label0,
                                               float norm, float* dS, float* dls_row, int beta) {
  CLIPMI_REQUIRE(label0 >= 0 && label0 + B <= Bg, "label offset out of range");
  CLIPMI_REQUIRE(C > 0 && col0 >= 0 && col0 + C <= Bg, "chunk out of range");
  hipLaunchKernelGGL(ce_bwd_chunk_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, lse, logit_scale,
                     grad_out, B, C, col0, label0, norm, dS, dls_row, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_sum2(void* stream, const float* a, const float* b, int n, float scale, float* out, int beta) {
  hipLaunchKernelGGL(sum2_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a, b, n, scale, out, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
