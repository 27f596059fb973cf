// Feature-level adapter heads and class-prototype scoring.
//
// Replaces model_t.py's CLIP-Adapter head (the next caller after the towers):
//   VisualAdapter / TextAdapter  fc2(relu(fc1(x)))                        model_t.py:13-33
//   residual blend + renormalise  a*adapter(x) + (1-a)*x, / |.|           model_t.py:186-197, 113-119
//   class logits + CE             T * img . protos^T, CrossEntropy(labels) model_t.py:200-203
//   predict                       softmax(100 * img . protos^T)          model_t.py:240-247
//   predict_with_all_descriptions max over each class's descriptions     model_t.py:252-298
// Everything is fp32 (the features are fp32 [B, E] rows, E <= 1024, bottleneck A <= 256):
// the head is latency-bound, a few hundred kFLOP per row, so the kernels are one
// workgroup per row with the weights streamed from L2, and the weight gradients are
// deterministic per-element reductions over the batch (no atomics).
#include "common.h"
#include "internal.h"

namespace {

constexpr int HT = 256;  // threads per workgroup
constexpr int MAXE = 1024, MAXA = 256, MAXC = 1024;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// xn = norm_in ? x/|x| : x;  h = relu(W1 xn + b1);  z = alpha (W2 h + b2) + (1 - alpha) xn;
// out = z/|z|, rz = 1/|z|
__global__ __launch_bounds__(HT) void fadapt_fwd_kernel(const float* x, int E, int A, const float* W1, const float* b1,
                                                       const float* W2, const float* b2, float alpha, int norm_in,
                                                       float* xn, float* h, float* out, float* rz,
                                                       const uint8_t* keep, float keep_scale) {
  __shared__ float sx[MAXE];
  __shared__ float sh[MAXA];
  __shared__ float red[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t row = blockIdx.x;
  float ss = 0.f;
  for (int e = t; e < E; e += HT) {
    const float v = x[row * E + e];
    sx[e] = v;
    ss += v * v;
  }
  ss = block_sum(ss, red);  // also orders the sx writes
  const float inv = norm_in ? 1.f / sqrtf(ss) : 1.f;
  for (int e = t; e < E; e += HT) {
    sx[e] *= inv;
    xn[row * E + e] = sx[e];
  }
  __syncthreads();
  for (int a = w; a < A; a += HT / 64) {  // a wave per bottleneck unit, lanes over the input
    float acc = 0.f;
    for (int e = lane; e < E; e += 64) acc = fmaf(W1[(int64_t)a * E + e], sx[e], acc);
    acc = wave_sum(acc) + b1[a];
    if (lane == 0) {
      float r = fmaxf(acc, 0.f);
      if (keep) r *= keep[row * A + a] ? keep_scale : 0.f;  // nn.Dropout after the ReLU (model_v.py:26)
      sh[a] = r;
      h[row * A + a] = r;
    }
  }
  __syncthreads();
  float zl[MAXE / HT];
  float sz = 0.f;
#pragma unroll
  for (int i = 0; i < MAXE / HT; ++i) {
    const int e = t + i * HT;
    zl[i] = 0.f;
    if (e < E) {
      float acc = b2[e];
      const float* wr = W2 + (int64_t)e * A;
      for (int a = 0; a < A; ++a) acc = fmaf(wr[a], sh[a], acc);
      zl[i] = alpha * acc + (1.f - alpha) * sx[e];
      sz += zl[i] * zl[i];
    }
  }
  sz = block_sum(sz, red);
  const float r = 1.f / sqrtf(sz);
#pragma unroll
  for (int i = 0; i < MAXE / HT; ++i) {
    const int e = t + i * HT;
    if (e < E) out[row * E + e] = zl[i] * r;
  }
  if (t == 0) rz[row] = r;
}

// per row: dy = alpha * (dout - out (out . dout)) / |z|;  dh = [h > 0] * W2^T dy
__global__ __launch_bounds__(HT) void fadapt_bwd_rows_kernel(const float* dout, const float* out, const float* rz, int E,
                                                            int A, const float* h, const float* W2, float alpha,
                                                            float* dy, float* dh, float keep_scale) {
  __shared__ float sdy[MAXE];
  __shared__ float red[4];
  const int t = threadIdx.x;
  const int64_t row = blockIdx.x;
  float dot = 0.f;
  for (int e = t; e < E; e += HT) dot += out[row * E + e] * dout[row * E + e];
  dot = block_sum(dot, red);
  const float r = rz[row];
  for (int e = t; e < E; e += HT) {
    const float v = alpha * (dout[row * E + e] - out[row * E + e] * dot) * r;
    sdy[e] = v;
    dy[row * E + e] = v;
  }
  __syncthreads();
  for (int a = t; a < A; a += HT) {  // thread per unit: W2[e, a] reads coalesced across threads
    float acc = 0.f;
    for (int e = 0; e < E; ++e) acc = fmaf(W2[(int64_t)e * A + a], sdy[e], acc);
    // h holds relu(.) * mask / (1 - p): h > 0 <=> kept and active
    dh[row * A + a] = h[row * A + a] > 0.f ? acc * keep_scale : 0.f;
  }
}

// g = [dW1 (A x E) | db1 (A) | dW2 (E x A) | db2 (E)] += batch sums (torch's nn.Linear layout)
__global__ __launch_bounds__(HT) void fadapt_wgrad_kernel(const float* xn, const float* h, const float* dy,
                                                         const float* dh, int B, int E, int A, float* g) {
  const int64_t i = (int64_t)blockIdx.x * HT + threadIdx.x;
  const int64_t n1 = (int64_t)A * E, n2 = n1 + A, n3 = n2 + (int64_t)E * A, n4 = n3 + E;
  if (i >= n4) return;
  float acc = 0.f;
  if (i < n1) {
    const int a = (int)(i / E), e = (int)(i - (int64_t)a * E);
    for (int b = 0; b < B; ++b) acc = fmaf(dh[(int64_t)b * A + a], xn[(int64_t)b * E + e], acc);
  } else if (i < n2) {
    const int a = (int)(i - n1);
    for (int b = 0; b < B; ++b) acc += dh[(int64_t)b * A + a];
  } else if (i < n3) {
    const int e = (int)((i - n2) / A), a = (int)((i - n2) - (int64_t)e * A);
    for (int b = 0; b < B; ++b) acc = fmaf(dy[(int64_t)b * E + e], h[(int64_t)b * A + a], acc);
  } else {
    const int e = (int)(i - n3);
    for (int b = 0; b < B; ++b) acc += dy[(int64_t)b * E + e];
  }
  g[i] += acc;
}

// one workgroup per image row: s[j] = scale * img . desc[j] over all descriptions, then
// per class c the max over its descriptions [off[c], off[c+1]); probs = softmax over classes.
// With one description per class (off = 0..C) this is the prototype score.  Optional
// training outputs: loss_rows[b] = lse - score[label], dscore = softmax - onehot.
__global__ __launch_bounds__(HT) void class_scores_kernel(const float* img, int E, const float* desc, const int* off,
                                                         int C, float scale, float* scores, float* probs,
                                                         const int64_t* labels, float* loss_rows, float* dscore,
                                                         int* bad) {
  __shared__ float simg[MAXE];
  __shared__ float sc[MAXC];
  __shared__ float stat[2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t row = blockIdx.x;
  for (int e = t; e < E; e += HT) simg[e] = img[row * E + e];
  __syncthreads();
  for (int c = w; c < C; c += HT / 64) {
    float best = -__builtin_huge_valf();
    for (int j = off[c]; j < off[c + 1]; ++j) {
      float acc = 0.f;
      for (int e = lane; e < E; e += 64) acc = fmaf(desc[(int64_t)j * E + e], simg[e], acc);
      best = fmaxf(best, scale * wave_sum(acc));
    }
    if (lane == 0) sc[c] = best;
  }
  __syncthreads();
  if (w == 0) {
    float m = -__builtin_huge_valf();
    for (int c = lane; c < C; c += 64) m = fmaxf(m, sc[c]);
    m = wave_max(m);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += expf(sc[c] - m);
    s = wave_sum(s);
    if (lane == 0) { stat[0] = m; stat[1] = s; }
  }
  __syncthreads();
  const float m = stat[0], s = stat[1];
  int64_t lab = -1;
  if (labels) {
    lab = labels[row];
    if (lab < 0 || lab >= C) {
      if (t == 0) *bad = 1;
      lab = -1;
    }
  }
  for (int c = t; c < C; c += HT) {
    const float p = expf(sc[c] - m) / s;
    if (scores) scores[row * C + c] = sc[c];
    if (probs) probs[row * C + c] = p;
    if (dscore) dscore[row * C + c] = p - (c == lab ? 1.f : 0.f);
  }
  if (loss_rows && t == 0) loss_rows[row] = lab >= 0 ? m + logf(s) - sc[lab] : 0.f;
}

// mean over B rows into out[0] (single workgroup, fixed order)
__global__ __launch_bounds__(HT) void row_mean_kernel(const float* v, int B, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += HT) s += v[b];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s / (float)B;
}

// CE backward through the prototype scores: with d = dscore * gscale / B,
//   dimg[b, e] = scale * sum_c d[b, c] P[c, e]   (rows < B)
//   dP[c, e]   = scale * sum_b d[b, c] img[b, e] (rows B .. B + C)
__global__ __launch_bounds__(HT) void class_ce_bwd_kernel(const float* dscore, const float* img, const float* P, int B,
                                                         int C, int E, float scale, const float* gscale, float* dimg,
                                                         float* dP) {
  const int64_t i = (int64_t)blockIdx.x * HT + threadIdx.x;
  if (i >= (int64_t)(B + C) * E) return;
  const float k = scale * (gscale ? gscale[0] : 1.f) / (float)B;
  const int r = (int)(i / E), e = (int)(i - (int64_t)r * E);
  float acc = 0.f;
  if (r < B) {
    for (int c = 0; c < C; ++c) acc = fmaf(dscore[(int64_t)r * C + c], P[(int64_t)c * E + e], acc);
    dimg[(int64_t)r * E + e] = k * acc;
  } else {
    const int c = r - B;
    for (int b = 0; b < B; ++b) acc = fmaf(dscore[(int64_t)b * C + c], img[(int64_t)b * E + e], acc);
    dP[(int64_t)c * E + e] = k * acc;
  }
}

// row softmax of scale * x (fp32, one wave per row; in place allowed): the cross-attention
// probabilities of the shared adapter (nn.MultiheadAttention core, adapter/clip_adapter.py:117)
__global__ __launch_bounds__(HT) void softmax_rows_kernel(const float* x, float* y, int R, int N, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (HT / 64) + (threadIdx.x >> 6);
  if (row >= R) return;
  const float* xr = x + row * N;
  float m = -__builtin_huge_valf();
  for (int j = lane; j < N; j += 64) m = fmaxf(m, scale * xr[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < N; j += 64) s += expf(scale * xr[j] - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < N; j += 64) y[row * N + j] = expf(scale * xr[j] - m) * inv;
}

// dx = scale * y * (dy - sum_j dy_j y_j)
__global__ __launch_bounds__(HT) void softmax_rows_bwd_kernel(const float* y, const float* dy, float* dx, int R, int N,
                                                             float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (HT / 64) + (threadIdx.x >> 6);
  if (row >= R) return;
  float d = 0.f;
  for (int j = lane; j < N; j += 64) d += dy[row * N + j] * y[row * N + j];
  d = wave_sum(d);
  for (int j = lane; j < N; j += 64) dx[row * N + j] = scale * y[row * N + j] * (dy[row * N + j] - d);
}

// keep[i] = u(seed, offset + i) >= p, u uniform in [0, 1) from a counter hash (splitmix64): the
// masks of nn.Dropout(p) (model_v.py:25, adapter/clip_adapter.py:84,96) reproducible by seed
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(HT) void dropout_mask_kernel(uint8_t* keep, int64_t n, float p, uint64_t seed,
                                                         uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * HT + threadIdx.x;
  if (i >= n) return;
  const float u = (float)(splitmix64(seed * 0x632BE59BD9B4E019ull + offset + (uint64_t)i) >> 40) * (1.0f / 16777216.0f);
  keep[i] = u >= p ? 1 : 0;
}
// y = x * keep * scale (+ res)
__global__ __launch_bounds__(HT) void dropout_apply_kernel(const float* x, const uint8_t* keep, int64_t n, float scale,
                                                          const float* res, float* y) {
  const int64_t i = (int64_t)blockIdx.x * HT + threadIdx.x;
  if (i >= n) return;
  float v = keep[i] ? x[i] * scale : 0.f;
  if (res) v += res[i];
  y[i] = v;
}
// average fusion (model_v.py:310-315): u = (a + b) / 2, out = u / |u|, ru = 1 / |u|
__global__ __launch_bounds__(HT) void fuse_avg_kernel(const float* a, const float* b, int E, float* out, float* ru) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  float ss = 0.f;
  for (int e = threadIdx.x; e < E; e += HT) {
    const float u = 0.5f * (a[row * E + e] + b[row * E + e]);
    ss += u * u;
  }
  ss = block_sum(ss, red);
  const float r = 1.f / sqrtf(ss);
  for (int e = threadIdx.x; e < E; e += HT) out[row * E + e] = 0.5f * (a[row * E + e] + b[row * E + e]) * r;
  if (threadIdx.x == 0) ru[row] = r;
}
// d a = d b = (dout - out (out . dout)) * ru / 2
__global__ __launch_bounds__(HT) void fuse_avg_bwd_kernel(const float* dout, const float* out, const float* ru, int E,
                                                         float* dab) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  float dot = 0.f;
  for (int e = threadIdx.x; e < E; e += HT) dot += out[row * E + e] * dout[row * E + e];
  dot = block_sum(dot, red);
  const float r = 0.5f * ru[row];
  for (int e = threadIdx.x; e < E; e += HT) dab[row * E + e] = (dout[row * E + e] - out[row * E + e] * dot) * r;
}

}  // namespace

extern "C" int clipmi_softmax_rows(void* stream, const float* x, float* y, int R, int N, float scale) {
  CLIPMI_REQUIRE(R >= 0 && N >= 1, "softmax: bad shape");
  if (R == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((R + 3) / 4), dim3(HT), 0, (hipStream_t)stream, x, y, R, N, scale);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_softmax_rows_bwd(void* stream, const float* y, const float* dy, float* dx, int R, int N,
                                       float scale) {
  CLIPMI_REQUIRE(R >= 0 && N >= 1, "softmax: bad shape");
  if (R == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(softmax_rows_bwd_kernel, dim3((R + 3) / 4), dim3(HT), 0, (hipStream_t)stream, y, dy, dx, R, N,
                     scale);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_feature_adapter_fwd(void* stream, const float* x, int B, int E, int A, const float* W1,
                                          const float* b1, const float* W2, const float* b2, float alpha, int norm_in,
                                          float* xn, float* h, float* out, float* rz, const uint8_t* keep,
                                          float keep_scale) {
  CLIPMI_REQUIRE(B >= 0 && E >= 1 && E <= MAXE && A >= 1 && A <= MAXA, "feature adapter: E <= 1024, A <= 256");
  CLIPMI_REQUIRE(x && W1 && b1 && W2 && b2 && xn && h && out && rz, "feature adapter: null pointer");
  if (B == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(fadapt_fwd_kernel, dim3(B), dim3(HT), 0, (hipStream_t)stream, x, E, A, W1, b1, W2, b2, alpha,
                     norm_in, xn, h, out, rz, keep, keep_scale);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_feature_adapter_bwd_ws(int B, int E, int A) {
  return (int)(((int64_t)B * (E + A)) * sizeof(float));
}

extern "C" int clipmi_feature_adapter_bwd(void* stream, const float* dout, const float* out, const float* rz,
                                          const float* xn, const float* h, int B, int E, int A, const float* W2,
                                          float alpha, float* grads, void* workspace, int64_t workspace_bytes,
                                          float keep_scale) {
  CLIPMI_REQUIRE(B >= 0 && E >= 1 && E <= MAXE && A >= 1 && A <= MAXA, "feature adapter: E <= 1024, A <= 256");
  CLIPMI_REQUIRE(workspace_bytes >= clipmi_feature_adapter_bwd_ws(B, E, A), "feature adapter: workspace too small");
  if (B == 0) return CLIPMI_OK;
  hipStream_t s = (hipStream_t)stream;
  float* dy = (float*)workspace;
  float* dh = dy + (int64_t)B * E;
  hipLaunchKernelGGL(fadapt_bwd_rows_kernel, dim3(B), dim3(HT), 0, s, dout, out, rz, E, A, h, W2, alpha, dy, dh,
                     keep_scale);
  const int64_t n = 2 * (int64_t)A * E + A + E;
  hipLaunchKernelGGL(fadapt_wgrad_kernel, dim3((unsigned)((n + HT - 1) / HT)), dim3(HT), 0, s, xn, h, dy, dh, B, E, A,
                     grads);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_class_scores(void* stream, const float* img, int B, int E, const float* desc, const int* off,
                                   int C, float scale, float* scores, float* probs, const int64_t* labels,
                                   float* loss_rows, float* dscore, int* bad) {
  CLIPMI_REQUIRE(B >= 0 && E >= 1 && E <= MAXE && C >= 1 && C <= MAXC, "class scores: E <= 1024, C <= 1024");
  CLIPMI_REQUIRE(!labels || (loss_rows && bad), "class scores: labels need loss_rows and bad");
  if (B == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(class_scores_kernel, dim3(B), dim3(HT), 0, (hipStream_t)stream, img, E, desc, off, C, scale,
                     scores, probs, labels, loss_rows, dscore, bad);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_row_mean(void* stream, const float* v, int B, float* out) {
  CLIPMI_REQUIRE(B >= 1, "row mean: B >= 1");
  hipLaunchKernelGGL(row_mean_kernel, dim3(1), dim3(HT), 0, (hipStream_t)stream, v, B, out);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_class_ce_bwd(void* stream, const float* dscore, const float* img, const float* protos, int B,
                                   int C, int E, float scale, const float* gscale, float* dimg, float* dprotos) {
  CLIPMI_REQUIRE(B >= 1 && C >= 1 && E >= 1, "class CE backward: empty shape");
  const int64_t n = (int64_t)(B + C) * E;
  hipLaunchKernelGGL(class_ce_bwd_kernel, dim3((unsigned)((n + HT - 1) / HT)), dim3(HT), 0, (hipStream_t)stream,
                     dscore, img, protos, B, C, E, scale, gscale, dimg, dprotos);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_dropout_mask(void* stream, uint8_t* keep, int64_t n, float p, uint64_t seed, uint64_t offset) {
  CLIPMI_REQUIRE(n >= 0 && p >= 0.f && p < 1.f, "dropout: 0 <= p < 1");
  if (n == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((n + HT - 1) / HT)), dim3(HT), 0, (hipStream_t)stream, keep,
                     n, p, seed, offset);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_dropout_apply(void* stream, const float* x, const uint8_t* keep, int64_t n, float scale,
                                    const float* res, float* y) {
  CLIPMI_REQUIRE(n >= 0 && x && keep && y, "dropout apply: null pointer");
  if (n == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(dropout_apply_kernel, dim3((unsigned)((n + HT - 1) / HT)), dim3(HT), 0, (hipStream_t)stream, x,
                     keep, n, scale, res, y);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_fuse_avg(void* stream, const float* a, const float* b, int B, int E, float* out, float* ru) {
  CLIPMI_REQUIRE(B >= 0 && E >= 1, "fuse_avg: bad shape");
  if (B == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(fuse_avg_kernel, dim3(B), dim3(HT), 0, (hipStream_t)stream, a, b, E, out, ru);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_fuse_avg_bwd(void* stream, const float* dout, const float* out, const float* ru, int B, int E,
                                   float* dab) {
  CLIPMI_REQUIRE(B >= 0 && E >= 1, "fuse_avg: bad shape");
  if (B == 0) return CLIPMI_OK;
  hipLaunchKernelGGL(fuse_avg_bwd_kernel, dim3(B), dim3(HT), 0, (hipStream_t)stream, dout, out, ru, E, dab);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
