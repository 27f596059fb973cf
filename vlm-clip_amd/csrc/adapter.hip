// Fused bottleneck adapter on the pooled rows: y = LN(up(gelu_erf(down(x))) + x), or without the
// LayerNorm (ln = 0).  Replaces TextAdapter / VisionAdapter.forward (adapter/clip_adapter.py:17-23,
// 144-150) and peclip.TextualAdapter.forward (adapter/peclip.py:13-18): nn.Linear(D, A) -> GELU (erf)
// -> nn.Linear(A, D) -> + x -> nn.LayerNorm(D, eps 1e-5), and their backward (the reference's
// loss.backward through the adapter, trainer.py:92).
//
// The adapter runs on B rows only (the pooled token: model_m.py:102,122), a few GFLOP, so one launch
// does the whole forward: a workgroup owns RB = adp_rb(R) rows, keeps x, the bottleneck activation and the
// pre-LN sum in LDS (fp32) and computes both products with its 256 threads one output column each
// (weights read as 16-B row pieces, the row values broadcast from LDS), then the LayerNorm per row.
// The backward is two launches: the row pass (LayerNorm backward, d_act = dz Wu, d_pre = d_act *
// gelu'(pre), dx = dz + d_pre Wd, per-workgroup partial sums of the bias / LayerNorm-affine
// gradients) and the weight pass (gWu += dz^T act, gWd += d_pre^T x, the partials summed in
// workgroup order): every sum in a fixed order, so a replayed step is bitwise equal.
// Storage dtype T (bf16 MFMA mode or fp32 parity mode) for x / y / dx and the weights; all math and
// every intermediate in fp32 (the saved pre-activation, activation and pre-LN sum are rounded to T).
#include "common.h"
#include "internal.h"
#include <type_traits>

namespace {

// rows per workgroup: adp_rb(R) in {1, 2, 4, 8} -- the most that still gives every CU a workgroup
// (each workgroup reads both weight matrices once, so more rows per workgroup = fewer re-reads)
__host__ __device__ constexpr int adp_rb(int R) { return R >= 2048 ? 8 : R >= 1024 ? 4 : R >= 512 ? 2 : 1; }
constexpr int ADP_T = 256;    // threads
constexpr int ADP_WO = 8;     // weight-pass outputs per thread along the reduced operand's rows

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float v[8]) {
  if constexpr (std::is_same<T, bf16>::value) {
    const bf16x8 w = *(const bf16x8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)w[e];
  } else {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      v[4 + e] = b[e];
    }
  }
}

struct AdpFwd {
  int R, D, A, ln;
  const void *x, *wd, *bd, *wu, *bu, *lnw, *lnb;
  int64_t ldx, ldy;
  void* y;
  void *pre, *act, *z;  // saved for the backward (or null)
  float *mean, *rstd;
  float eps;
};

// out[r][c] = sum_k in[r][k] W[c][k] for the workgroup's rows: thread c, W rows read in 16-B pieces
template <typename T, int RB>
__device__ __forceinline__ void rows_times_wt(const float* in, int K, const T* W, int c, float acc[RB]) {
  const T* wr = W + (int64_t)c * K;
  for (int k = 0; k < K; k += 8) {
    float w[8];
    ld8(wr + k, w);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float* xr = in + r * K + k;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[r] = fmaf(xr[e], w[e], acc[r]);
    }
  }
}

template <typename T, int RB>
__global__ __launch_bounds__(ADP_T) void adapter_fwd_kernel(AdpFwd a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int D = a.D, A = a.A, t = threadIdx.x;
  const int r0 = blockIdx.x * RB, nr = min(RB, a.R - r0);
  float* xs = sm;                 // [RB][D]
  float* hs = xs + RB * D;    // [RB][A]
  float* zs = hs + RB * A;    // [RB][D]
  for (int i = t; i < RB * D; i += ADP_T) {
    const int r = i / D, k = i - r * D;
    xs[i] = r < nr ? to_f32(((const T*)a.x)[(int64_t)(r0 + r) * a.ldx + k]) : 0.f;
  }
  __syncthreads();
  // down projection + bias + gelu_erf
  for (int c = t; c < A; c += ADP_T) {
    float acc[RB];
    const float b = to_f32(((const T*)a.bd)[c]);
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = b;
    rows_times_wt<T, RB>(xs, D, (const T*)a.wd, c, acc);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const T pre = from_f32<T>(acc[r]);
      const T act = from_f32<T>(gelu_erf(to_f32(pre)));
      hs[r * A + c] = to_f32(act);
      if (r < nr && a.pre) {
        ((T*)a.pre)[(int64_t)(r0 + r) * A + c] = pre;
        ((T*)a.act)[(int64_t)(r0 + r) * A + c] = act;
      }
    }
  }
  __syncthreads();
  // up projection + bias + residual
  for (int c = t; c < D; c += ADP_T) {
    float acc[RB];
    const float b = to_f32(((const T*)a.bu)[c]);
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = b + xs[r * D + c];
    rows_times_wt<T, RB>(hs, A, (const T*)a.wu, c, acc);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const T z = from_f32<T>(acc[r]);
      zs[r * D + c] = to_f32(z);
      if (r < nr) {
        if (!a.ln) ((T*)a.y)[(int64_t)(r0 + r) * a.ldy + c] = z;
        else if (a.z) ((T*)a.z)[(int64_t)(r0 + r) * D + c] = z;
      }
    }
  }
  if (!a.ln) return;
  __syncthreads();
  // LayerNorm: one wave per row (fp32 statistics, two-pass variance)
  const int wave = t >> 6, lane = t & 63;
  for (int r = wave; r < nr; r += ADP_T / 64) {
    const float* zr = zs + r * D;
    float s = 0.f;
    for (int k = lane; k < D; k += 64) s += zr[k];
    const float mean = wave_sum(s) / D;
    float v = 0.f;
    for (int k = lane; k < D; k += 64) {
      const float d = zr[k] - mean;
      v = fmaf(d, d, v);
    }
    const float rstd = rsqrtf(wave_sum(v) / D + a.eps);
    for (int k = lane; k < D; k += 64)
      ((T*)a.y)[(int64_t)(r0 + r) * a.ldy + k] =
          from_f32<T>((zr[k] - mean) * rstd * to_f32(((const T*)a.lnw)[k]) + to_f32(((const T*)a.lnb)[k]));
    if (lane == 0 && a.mean) {
      a.mean[r0 + r] = mean;
      a.rstd[r0 + r] = rstd;
    }
  }
}

struct AdpBwd {
  int R, D, A, ln;
  const void *dy, *x, *pre, *act, *z, *wd, *wu, *lnw;
  const float *mean, *rstd;
  int64_t lddy, ldx, lddx;
  void* dx;
  float *dz, *dpre;        // workspace [R][D], [R][A]
  float *pbu, *pbd, *plw, *plb;  // per-workgroup partials [nwg][D], [nwg][A], [nwg][D], [nwg][D]
};

template <typename T, int RB>
__global__ __launch_bounds__(ADP_T) void adapter_bwd_rows_kernel(AdpBwd a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int D = a.D, A = a.A, t = threadIdx.x, wg = blockIdx.x;
  const int r0 = wg * RB, nr = min(RB, a.R - r0);
  float* dys = sm;                 // [RB][D] dy (LayerNorm branch)
  float* dps = sm + RB * D;    // [RB][A] d_pre
  float* dzs = a.ln ? dps + RB * A : sm;  // [RB][D] dz = dL/d(pre-LN sum)
  const int wave = t >> 6, lane = t & 63;
  if (a.ln) {
    for (int r = wave; r < RB; r += ADP_T / 64) {  // one wave per row
      const bool ok = r < nr;
      const float mean = ok ? a.mean[r0 + r] : 0.f, rstd = ok ? a.rstd[r0 + r] : 0.f;
      float sg = 0.f, sgx = 0.f;
      for (int k = lane; k < D; k += 64) {
        const float dy = ok ? to_f32(((const T*)a.dy)[(int64_t)(r0 + r) * a.lddy + k]) : 0.f;
        const float xh = ok ? (to_f32(((const T*)a.z)[(int64_t)(r0 + r) * D + k]) - mean) * rstd : 0.f;
        const float g = dy * to_f32(((const T*)a.lnw)[k]);
        dys[r * D + k] = dy;
        dzs[r * D + k] = xh;
        sg += g;
        sgx = fmaf(g, xh, sgx);
      }
      sg = wave_sum(sg) / D;
      sgx = wave_sum(sgx) / D;
      for (int k = lane; k < D; k += 64) {
        const float g = dys[r * D + k] * to_f32(((const T*)a.lnw)[k]);
        dzs[r * D + k] = rstd * (g - sg - dzs[r * D + k] * sgx);
      }
    }
    __syncthreads();
    // LayerNorm affine partials over the workgroup's rows (x-hat recomputed from the saved sum)
    for (int k = t; k < D; k += ADP_T) {
      float pw = 0.f, pb = 0.f;
      for (int r = 0; r < nr; ++r) {
        const float dy = dys[r * D + k];
        const float xh = (to_f32(((const T*)a.z)[(int64_t)(r0 + r) * D + k]) - a.mean[r0 + r]) * a.rstd[r0 + r];
        pw = fmaf(dy, xh, pw);
        pb += dy;
      }
      a.plw[(int64_t)wg * D + k] = pw;
      a.plb[(int64_t)wg * D + k] = pb;
    }
  } else {
    for (int i = t; i < RB * D; i += ADP_T) {
      const int r = i / D, k = i - r * D;
      dzs[i] = r < nr ? to_f32(((const T*)a.dy)[(int64_t)(r0 + r) * a.lddy + k]) : 0.f;
    }
    __syncthreads();
  }
  // dz out (weight pass) + the up bias partials
  for (int k = t; k < D; k += ADP_T) {
    float pb = 0.f;
    for (int r = 0; r < nr; ++r) {
      const float v = dzs[r * D + k];
      a.dz[(int64_t)(r0 + r) * D + k] = v;
      pb += v;
    }
    a.pbu[(int64_t)wg * D + k] = pb;
  }
  // d_act = dz Wu (Wu [D][A]: thread c reads column c, rows of Wu coalesced across the wave)
  for (int c = t; c < A; c += ADP_T) {
    float acc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = 0.f;
    const T* wc = (const T*)a.wu + c;
    for (int k = 0; k < D; ++k) {
      const float w = to_f32(wc[(int64_t)k * A]);
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[r] = fmaf(dzs[r * D + k], w, acc[r]);
    }
    float pb = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float dp = 0.f;
      if (r < nr) {
        dp = acc[r] * gelu_erf_grad(to_f32(((const T*)a.pre)[(int64_t)(r0 + r) * A + c]));
        a.dpre[(int64_t)(r0 + r) * A + c] = dp;
        pb += dp;
      }
      dps[r * A + c] = dp;
    }
    a.pbd[(int64_t)wg * A + c] = pb;
  }
  __syncthreads();
  // dx = dz + d_pre Wd (Wd [A][D]: thread k reads column k, coalesced across the wave)
  for (int k = t; k < D; k += ADP_T) {
    float acc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r] = dzs[r * D + k];
    const T* wk = (const T*)a.wd + k;
    for (int c = 0; c < A; ++c) {
      const float w = to_f32(wk[(int64_t)c * D]);
#pragma unroll
      for (int r = 0; r < RB; ++r) acc[r] = fmaf(dps[r * A + c], w, acc[r]);
    }
    for (int r = 0; r < nr; ++r) ((T*)a.dx)[(int64_t)(r0 + r) * a.lddx + k] = from_f32<T>(acc[r]);
  }
}

struct AdpW {
  int R, D, A, nwg, ln;
  const float *dz, *dpre, *pbu, *pbd, *plw, *plb;
  const void *act, *x;
  int64_t ldx;
  float *gwd, *gbd, *gwu, *gbu, *glw, *glb;
};

// weight pass: block ranges [0, nu) gWu tiles (ADP_WO rows d x 256 columns a), [nu, nu + nd) gWd
// tiles (ADP_WO rows a x 256 columns k), then one block per vector of summed partials
template <typename T>
__global__ __launch_bounds__(ADP_T) void adapter_bwd_weights_kernel(AdpW a, int nu, int nd) {
  const int t = threadIdx.x, b = blockIdx.x, D = a.D, A = a.A;
  if (b < nu + nd) {
    const bool up = b < nu;
    const int bb = up ? b : b - nu;
    const int ncol = up ? A : D, nrow = up ? D : A;
    const int cb = (ncol + ADP_T - 1) / ADP_T;
    const int row0 = (bb / cb) * ADP_WO, col = (bb % cb) * ADP_T + t;
    if (!(up ? a.gwu : a.gwd) || col >= ncol) return;
    const float* lhs = up ? a.dz : a.dpre;  // [R][nrow]
    float acc[ADP_WO];
#pragma unroll
    for (int o = 0; o < ADP_WO; ++o) acc[o] = 0.f;
    for (int r = 0; r < a.R; ++r) {
      const float v = up ? to_f32(((const T*)a.act)[(int64_t)r * A + col]) : to_f32(((const T*)a.x)[(int64_t)r * a.ldx + col]);
      const float* lr = lhs + (int64_t)r * nrow + row0;
#pragma unroll
      for (int o = 0; o < ADP_WO; ++o)
        if (row0 + o < nrow) acc[o] = fmaf(lr[o], v, acc[o]);
    }
    float* g = up ? a.gwu : a.gwd;
#pragma unroll
    for (int o = 0; o < ADP_WO; ++o)
      if (row0 + o < nrow) g[(int64_t)(row0 + o) * ncol + col] += acc[o];
    return;
  }
  // summed partials: gbu / glw / glb over D, gbd over A, workgroup order
  const int which = b - nu - nd;  // 0: gbu, 1: gbd, 2: glw, 3: glb
  const float* part = which == 0 ? a.pbu : which == 1 ? a.pbd : which == 2 ? a.plw : a.plb;
  float* g = which == 0 ? a.gbu : which == 1 ? a.gbd : which == 2 ? a.glw : a.glb;
  const int n = which == 1 ? A : D;
  if (!g) return;
  for (int k = t; k < n; k += ADP_T) {
    float s = 0.f;
    for (int w = 0; w < a.nwg; ++w) s += part[(int64_t)w * n + k];
    g[k] += s;
  }
}

}  // namespace

static int adp_check(int dtype, int R, int D, int A) {
  CLIPMI_REQUIRE(dtype == CLIPMI_BF16 || dtype == CLIPMI_F32, "adapter: bf16 or f32");
  CLIPMI_REQUIRE(R >= 0 && D > 0 && A > 0 && D % 8 == 0 && A % 8 == 0, "adapter: D and A multiples of 8");
  CLIPMI_REQUIRE((size_t)8 * (2 * D + A) * 4 <= 160 * 1024, "adapter: D too large for the row tile");
  return CLIPMI_OK;
}

extern "C" int clipmi_adapter_fwd(void* stream, int dtype, int R, int D, int A, const void* x, int64_t ldx,
                                  const void* w_down, const void* b_down, const void* w_up, const void* b_up,
                                  const void* ln_w, const void* ln_b, float eps, int ln, void* y, int64_t ldy,
                                  void* pre, void* act, void* z, float* mean, float* rstd) {
  CLIPMI_TRY(adp_check(dtype, R, D, A));
  CLIPMI_REQUIRE(x && y && w_down && b_down && w_up && b_up && ldx >= D && ldy >= D, "adapter_fwd: operands");
  CLIPMI_REQUIRE(!ln || (ln_w && ln_b), "adapter_fwd: LayerNorm weights");
  CLIPMI_REQUIRE(!pre == !act && (!pre || !ln || (z && mean && rstd)), "adapter_fwd: saved tensors come together");
  CLIPMI_REQUIRE(((uintptr_t)w_down & 15) == 0 && ((uintptr_t)w_up & 15) == 0, "adapter_fwd: weights 16-B aligned");
  if (R == 0) return CLIPMI_OK;
  AdpFwd a{R, D, A, ln, x, w_down, b_down, w_up, b_up, ln_w, ln_b, ldx, ldy, y, pre, act, z, mean, rstd, eps};
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto rbc) {
    constexpr int RB = decltype(rbc)::value;
    const size_t lds = (size_t)RB * (2 * D + A) * 4;
    const unsigned nb = (unsigned)((R + RB - 1) / RB);
    if (dtype == CLIPMI_BF16) {
      (void)lds_optin((const void*)adapter_fwd_kernel<bf16, RB>, (int)lds);
      hipLaunchKernelGGL((adapter_fwd_kernel<bf16, RB>), dim3(nb), dim3(ADP_T), lds, s, a);
    } else {
      (void)lds_optin((const void*)adapter_fwd_kernel<float, RB>, (int)lds);
      hipLaunchKernelGGL((adapter_fwd_kernel<float, RB>), dim3(nb), dim3(ADP_T), lds, s, a);
    }
  };
  switch (adp_rb(R)) {
    case 8: go(std::integral_constant<int, 8>()); break;
    case 4: go(std::integral_constant<int, 4>()); break;
    case 2: go(std::integral_constant<int, 2>()); break;
    default: go(std::integral_constant<int, 1>()); break;
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int64_t clipmi_adapter_bwd_ws(int R, int D, int A) {
  const int rb = adp_rb(R);
  const int64_t nwg = (R + rb - 1) / rb;
  return ((int64_t)R * (D + A) + nwg * (3 * (int64_t)D + A)) * 4;
}

extern "C" int clipmi_adapter_bwd(void* stream, int dtype, int R, int D, int A, const void* dy, int64_t lddy,
                                  const void* x, int64_t ldx, const void* pre, const void* act, const void* z,
                                  const float* mean, const float* rstd, const void* w_down, const void* w_up,
                                  const void* ln_w, int ln, void* dx, int64_t lddx, float* g_w_down, float* g_b_down,
                                  float* g_w_up, float* g_b_up, float* g_ln_w, float* g_ln_b, void* ws,
                                  int64_t ws_bytes) {
  CLIPMI_TRY(adp_check(dtype, R, D, A));
  CLIPMI_REQUIRE(dy && x && pre && act && dx && w_down && w_up && lddy >= D && ldx >= D && lddx >= D,
                 "adapter_bwd: operands");
  CLIPMI_REQUIRE(!ln || (z && mean && rstd && ln_w), "adapter_bwd: LayerNorm inputs");
  CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_adapter_bwd_ws(R, D, A), "adapter_bwd: workspace too small");
  if (R == 0) return CLIPMI_OK;
  const int rb = adp_rb(R);
  const int nwg = (R + rb - 1) / rb;
  float* f = (float*)ws;
  float* dz = f;
  float* dpre = dz + (int64_t)R * D;
  float* pbu = dpre + (int64_t)R * A;
  float* pbd = pbu + (int64_t)nwg * D;
  float* plw = pbd + (int64_t)nwg * A;
  float* plb = plw + (int64_t)nwg * D;
  AdpBwd b{R, D, A, ln, dy, x, pre, act, z, w_down, w_up, ln_w, mean, rstd, lddy, ldx, lddx, dx, dz, dpre,
           pbu, pbd, plw, plb};
  hipStream_t s = (hipStream_t)stream;
  const int nu = ((D + ADP_WO - 1) / ADP_WO) * ((A + ADP_T - 1) / ADP_T);
  const int nd = ((A + ADP_WO - 1) / ADP_WO) * ((D + ADP_T - 1) / ADP_T);
  AdpW w{R, D, A, nwg, ln, dz, dpre, pbu, pbd, plw, plb, act, x, ldx, g_w_down, g_b_down, g_w_up, g_b_up,
         ln ? g_ln_w : nullptr, ln ? g_ln_b : nullptr};
  const bool weights = g_w_down || g_b_down || g_w_up || g_b_up || g_ln_w || g_ln_b;
  auto go = [&](auto rbc) {
    constexpr int RB = decltype(rbc)::value;
    const size_t lds = (size_t)RB * (2 * D + A) * 4;
    if (dtype == CLIPMI_BF16) {
      (void)lds_optin((const void*)adapter_bwd_rows_kernel<bf16, RB>, (int)lds);
      hipLaunchKernelGGL((adapter_bwd_rows_kernel<bf16, RB>), dim3(nwg), dim3(ADP_T), lds, s, b);
    } else {
      (void)lds_optin((const void*)adapter_bwd_rows_kernel<float, RB>, (int)lds);
      hipLaunchKernelGGL((adapter_bwd_rows_kernel<float, RB>), dim3(nwg), dim3(ADP_T), lds, s, b);
    }
  };
  switch (rb) {
    case 8: go(std::integral_constant<int, 8>()); break;
    case 4: go(std::integral_constant<int, 4>()); break;
    case 2: go(std::integral_constant<int, 2>()); break;
    default: go(std::integral_constant<int, 1>()); break;
  }
  if (weights) {
    if (dtype == CLIPMI_BF16)
      hipLaunchKernelGGL(adapter_bwd_weights_kernel<bf16>, dim3(nu + nd + 4), dim3(ADP_T), 0, s, w, nu, nd);
    else
      hipLaunchKernelGGL(adapter_bwd_weights_kernel<float>, dim3(nu + nd + 4), dim3(ADP_T), 0, s, w, nu, nd);
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
