// Optimizer step over the flat parameter arena: global-norm clip + AdamW + bf16 shadow.
//
// Replaces trainer.py:95 (nn.utils.clip_grad_norm_(params, max_grad_norm)) and
// trainer.py:98 (torch.optim.AdamW.step, decoupled weight decay) with the lr of
// get_linear_schedule_with_warmup ([HF] optimization.py:101-129) passed per step.
// All trainable parameters live in one fp32 arena (p, grad, exp_avg, exp_avg_sq), so
// the step is 2 launches: a deterministic two-stage sum of squares, then one fused
// elementwise AdamW pass that reads the clip coefficient from device memory and also
// refreshes the bf16 shadow the MFMA kernels read.  28 B/param (p, g, m, v read; p, m, v
// written) + 2 B/param shadow, at 5.4-5.5 TB/s over the B/16 arena (tools/optim_bench.py): near
// the HBM rate, with the IEEE sqrt and two divisions per parameter (torch's arithmetic) making
// it VALU-heavy enough that fp-contraction changes show (profiles/r02_adamw_ab.txt).
#include "common.h"
#include "internal.h"

namespace {

constexpr int NORM_BLOCKS = 1024;

__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* g, int64_t n, float* part) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 v = ((const f32x4*)g)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += 256) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// norm_out[0] = sqrt(sum part), norm_out[1] = min(1, max_norm / (norm + 1e-6))
__global__ __launch_bounds__(1024) void norm_finish_kernel(const float* part, int np, float max_norm, float* norm_out) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 1024) s += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += red[w];
    const float nrm = (float)sqrt(t);
    norm_out[0] = nrm;
    const float c = max_norm / (nrm + 1e-6f);
    norm_out[1] = max_norm > 0.f ? fminf(c, 1.f) : 1.f;
  }
}

// torch.optim.AdamW (foreach=False semantics):
//   p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__device__ __forceinline__ float adamw_elem(float gi, float& pi, float& mi, float& vi, float cf, float step, float decay,
                                            float b1, float b2, float eps, float bc2s) {
  gi *= cf;
  pi *= decay;
  mi = mi + (1.f - b1) * (gi - mi);  // exp_avg.lerp_(grad, 1 - beta1)
  vi = b2 * vi + (1.f - b2) * gi * gi;
  pi -= step * mi / (sqrtf(vi) / bc2s + eps);
  return pi;
}

// 4 parameters per lane (16-B loads/stores, 8-B shadow stores; cdna_hip_programming.md G13),
// scalar tail; the per-element arithmetic is adamw_elem's either way
template <bool VEC>
__global__ __launch_bounds__(256) void adamw_kernel(float* p, const float* g, float* m, float* v, bf16* shadow,
                                                    int64_t n, float lr, float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2s, const float* clip) {
  const float cf = clip ? clip[1] : 1.f;
  const float step = lr / bc1;  // step_size = lr / bias_correction1
  const float decay = 1.f - lr * wd;
  const int64_t n4 = VEC ? n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  // two 4-parameter groups per lane and iteration: all eight 16-B loads in flight before the math
  constexpr int U = 2;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += U * stride) {
    f32x4 gv[U], pv[U], mv[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + u * stride, n4 - 1);  // past the end: a clamped load, never stored
      gv[u] = ((const f32x4*)g)[i];
      pv[u] = ((const f32x4*)p)[i];
      mv[u] = ((const f32x4*)m)[i];
      vv[u] = ((const f32x4*)v)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= n4) break;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = pv[u][e], me = mv[u][e], ve = vv[u][e];
        adamw_elem(gv[u][e], pe, me, ve, cf, step, decay, b1, b2, eps, bc2s);
        pv[u][e] = pe; mv[u][e] = me; vv[u][e] = ve;
      }
      ((f32x4*)p)[i] = pv[u];
      ((f32x4*)m)[i] = mv[u];
      ((f32x4*)v)[i] = vv[u];
      if (shadow) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        ((bf16x4*)shadow)[i] = bf16x4{(bf16)pv[u][0], (bf16)pv[u][1], (bf16)pv[u][2], (bf16)pv[u][3]};
      }
    }
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(g[i], pi, mi, vi, cf, step, decay, b1, b2, eps, bc2s);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (shadow) shadow[i] = (bf16)pi;
  }
}

__global__ __launch_bounds__(256) void cast_kernel(const float* src, bf16* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = (bf16)src[i];
}

__global__ __launch_bounds__(256) void scale_kernel(float* x, int64_t n, const float* coef) {
  const float c = coef[1];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] *= c;
}

}  // namespace

extern "C" int64_t clipmi_grad_norm_ws(void) { return NORM_BLOCKS * 4; }

// norm_out: 2 floats on device {total_norm, clip_coef}
extern "C" int clipmi_grad_norm(void* stream, const float* g, int64_t n, float max_norm, float* norm_out, void* ws,
                                int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ws_bytes >= NORM_BLOCKS * 4, "grad_norm workspace too small");
  CLIPMI_REQUIRE(((uintptr_t)g & 15) == 0, "grad arena must be 16-byte aligned");
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(NORM_BLOCKS), dim3(256), 0, s, g, n, (float*)ws);
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(1024), 0, s, (const float*)ws, NORM_BLOCKS, max_norm, norm_out);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// global norm over several gradient segments (arenas or per-parameter slices)
extern "C" int64_t clipmi_grad_norm_multi_ws(int count) { return (int64_t)count * NORM_BLOCKS * 4; }
extern "C" int clipmi_grad_norm_multi(void* stream, const float* const* gs, const int64_t* ns, int count, float max_norm,
                                      float* norm_out, void* ws, int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(count >= 1, "count");
  CLIPMI_REQUIRE(ws_bytes >= (int64_t)count * NORM_BLOCKS * 4, "grad_norm workspace too small");
  for (int i = 0; i < count; ++i) {
    CLIPMI_REQUIRE(((uintptr_t)gs[i] & 15) == 0, "gradient segments must be 16-byte aligned");
    hipLaunchKernelGGL(sumsq_partial_kernel, dim3(NORM_BLOCKS), dim3(256), 0, s, gs[i], ns[i], (float*)ws + (int64_t)i * NORM_BLOCKS);
  }
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(1024), 0, s, (const float*)ws, count * NORM_BLOCKS, max_norm, norm_out);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// scale grads in place by norm_out[1] (clip_grad_norm_ semantics for callers that keep torch's optimizer)
extern "C" int clipmi_grad_scale(void* stream, float* g, int64_t n, const float* norm_out) {
  hipLaunchKernelGGL(scale_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, g, n, norm_out);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_adamw(void* stream, float* p, const float* g, float* m, float* v, void* shadow_bf16, int64_t n,
                            double lr, double beta1, double beta2, double eps, double weight_decay, int step,
                            const float* clip) {
  CLIPMI_REQUIRE(step >= 1, "step must be >= 1");
  // bias corrections in double, as torch computes them on the host
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2s = sqrt(1.0 - pow(beta2, (double)step));
  const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                   ((uintptr_t)shadow_bf16 & 7) == 0;
  if (vec)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(4096), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (bf16*)shadow_bf16,
                       n, (float)lr, (float)beta1, (float)beta2, (float)eps, (float)weight_decay, (float)bc1,
                       (float)bc2s, clip);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(4096), dim3(256), 0, (hipStream_t)stream, p, g, m, v, (bf16*)shadow_bf16,
                       n, (float)lr, (float)beta1, (float)beta2, (float)eps, (float)weight_decay, (float)bc1,
                       (float)bc2s, clip);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_cast_f32_bf16(void* stream, const float* src, void* dst, int64_t n) {
  hipLaunchKernelGGL(cast_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream, src, (bf16*)dst, n);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
