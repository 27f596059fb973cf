// LayerNorm forward/backward, column reductions (bias / LN-affine / position grads) and
// the embedding gathers/scatters of both towers.
//
// Replaces: nn.LayerNorm in [HF] modeling_clip.py:357,359 (layer_norm1/2), :605,642
// (pre_layrnorm), :559 (final_layer_norm), adapter/clip_adapter.py:15,142 (adapter LN);
// CLIPVisionEmbeddings.forward [HF] :202-219 (CLS concat + position add, fused into the
// pre-LN here); CLIPTextEmbeddings.forward [HF] :232-256 (token + position gather).
//
// One wave per row; a lane holds NP pieces of PS contiguous elements at element offset
// (k*64 + lane)*PS, so every load instruction is fully coalesced.  Statistics in fp32,
// two-pass variance from registers (no E[x^2]-E[x]^2 cancellation).
#include "common.h"
#include "internal.h"
#include <cstring>
#include <type_traits>

namespace {

template <typename T, int PS> struct Vec;
template <> struct Vec<float, 4> { typedef f32x4 type; };
template <> struct Vec<float, 2> { typedef __attribute__((ext_vector_type(2))) float type; };
template <> struct Vec<float, 1> { typedef float type; };
template <> struct Vec<bf16, 4> { typedef bf16x4 type; };
template <> struct Vec<bf16, 2> { typedef bf16x2 type; };
template <> struct Vec<bf16, 1> { typedef bf16 type; };

template <typename T, int PS>
__device__ __forceinline__ void vload(const T* p, float* o) {
  typename Vec<T, PS>::type v = *(const typename Vec<T, PS>::type*)p;
  if constexpr (PS == 1) { o[0] = (float)v; }
  else {
#pragma unroll
    for (int j = 0; j < PS; ++j) o[j] = (float)v[j];
  }
}
template <typename T, int PS>
__device__ __forceinline__ void vstore(T* p, const float* o) {
  typename Vec<T, PS>::type v;
  if constexpr (PS == 1) { v = (T)o[0]; }
  else {
#pragma unroll
    for (int j = 0; j < PS; ++j) v[j] = (T)o[j];
  }
  *(typename Vec<T, PS>::type*)p = v;
}

// y = LN(x [+ pos[row % period] + (row % period == 0 ? cls : 0)]) * w + b
// When pos is given the pre-LN sum is written back to x (the vision embedding output).
// A wave normalises LN_RPW rows, issuing every row's loads before the first reduction so
// twice the bytes are in flight per wave (one row per wave ran at 4.2 TB/s, latency bound).
constexpr int LN_RPW = 2;

// Q8: y is written as MXFP8 instead (q8 [R, D] e4m3 bytes, s8 [R, D/32] E8M0): a 32-element
// block is 8 consecutive lanes' 4-element pieces (PS == 4), max-reduced across those lanes; the
// fp8 operand of the next GEMM without a bf16 round trip through HBM.
// X3 (bf16x3 mode, fp32 x / w / b): y is written as the split image of the next GEMM's operand instead --
// bf16 [R][3D] (ldy = 3D), segments (h, h, l) for X3 = 1 or (h, l, h) for X3 = 2 with h = bf16(y), l = bf16(y - h)
// (gemm.hip CLIPMI_GEMM_SPLIT3's layout), so no fp32 copy and no split pass between the LayerNorm and its GEMMs.
template <typename TX, typename T, int PS, int NP, bool Q8 = false, int X3 = 0>
__global__ __launch_bounds__(256) void ln_fwd_kernel(TX* x, int64_t ldx, T* y, int64_t ldy, const T* w, const T* b,
                                                     float* mean_out, float* rstd_out, int R, int D, float eps,
                                                     const TX* pos, const TX* cls, int period, uint8_t* q8 = nullptr,
                                                     uint8_t* s8 = nullptr) {
  static_assert(!Q8 || PS == 4, "MXFP8 output needs 4-element pieces");
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * LN_RPW;
  if (row0 >= R) return;
  float v[LN_RPW][NP][PS];
#pragma unroll
  for (int rr = 0; rr < LN_RPW; ++rr) {
    const int row = min(row0 + rr, R - 1);  // a tail wave recomputes row R-1 and does not store it twice
    TX* xr = x + (int64_t)row * ldx;
#pragma unroll
    for (int k = 0; k < NP; ++k) vload<TX, PS>(xr + (k * 64 + lane) * PS, v[rr][k]);
  }
  float mean[LN_RPW], rstd[LN_RPW];
#pragma unroll
  for (int rr = 0; rr < LN_RPW; ++rr) {
    const int row = min(row0 + rr, R - 1);
    const bool own = row0 + rr < R;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int c = (k * 64 + lane) * PS;
      if (pos) {
        const int t = row % period;
        float pv[PS];
        vload<TX, PS>(pos + (int64_t)t * D + c, pv);
#pragma unroll
        for (int j = 0; j < PS; ++j) v[rr][k][j] += pv[j];
        if (cls && t == 0) {
          vload<TX, PS>(cls + c, pv);
#pragma unroll
          for (int j = 0; j < PS; ++j) v[rr][k][j] += pv[j];
        }
        if (own) vstore<TX, PS>(x + (int64_t)row * ldx + c, v[rr][k]);
      }
#pragma unroll
      for (int j = 0; j < PS; ++j) s += v[rr][k][j];
    }
    mean[rr] = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int j = 0; j < PS; ++j) { const float d = v[rr][k][j] - mean[rr]; q += d * d; }
    rstd[rr] = rsqrtf(wave_sum(q) / D + eps);
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int c = (k * 64 + lane) * PS;
    float wv[PS], bv[PS];
    vload<T, PS>(w + c, wv);
    vload<T, PS>(b + c, bv);
#pragma unroll
    for (int rr = 0; rr < LN_RPW; ++rr) {
      if (row0 + rr >= R) continue;  // wave-uniform
      float o[PS];
#pragma unroll
      for (int j = 0; j < PS; ++j) o[j] = (v[rr][k][j] - mean[rr]) * rstd[rr] * wv[j] + bv[j];
      if constexpr (Q8) {
        // lanes 8u .. 8u + 7 hold one 32-element block; the xor-shuffles stay inside it
        float am = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        am = fmaxf(am, __shfl_xor(am, 2, 64));
        am = fmaxf(am, __shfl_xor(am, 4, 64));
        const int ex = mx_exponent(am);
        const float inv = ldexpf(1.0f, -ex);
        *(uint32_t*)(q8 + (int64_t)(row0 + rr) * D + c) = mx_pack4(o[0], o[1], o[2], o[3], inv);
        if ((lane & 7) == 0) s8[(int64_t)(row0 + rr) * (D >> 5) + (c >> 5)] = (uint8_t)(ex + 127);
      } else if constexpr (X3 != 0) {
        float hv[PS], lv[PS];
#pragma unroll
        for (int j = 0; j < PS; ++j) {
          hv[j] = (float)(bf16)o[j];
          lv[j] = o[j] - hv[j];
        }
        bf16* y3 = (bf16*)y + (int64_t)(row0 + rr) * ldy + c;
        vstore<bf16, PS>(y3, hv);
        vstore<bf16, PS>(y3 + D, X3 == 1 ? hv : lv);
        vstore<bf16, PS>(y3 + 2 * D, X3 == 1 ? lv : hv);
      } else {
        vstore<T, PS>(y + (int64_t)(row0 + rr) * ldy + c, o);
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int rr = 0; rr < LN_RPW; ++rr) {
      if (row0 + rr >= R) continue;
      if (mean_out) mean_out[row0 + rr] = mean[rr];
      if (rstd_out) rstd_out[row0 + rr] = rstd[rr];
    }
  }
}

// dx = [dres +] rstd * (g - mean(g) - xhat * mean(g*xhat)),  g = dy * w
// per-block partial dgamma/dbeta -> ws[blockIdx][2][D]
// TW: the affine weight's dtype (default T; fp32 for the vision pre_layrnorm, whose fp32-residual forward
// normalises with the fp32 master weights)
// PS fp32 values -> their split image segments at dst, dst + seg, dst + 2 seg ((h, h, l) for pattern 0, (h, l, h) for
// 1) with clipmi_split3_colsum's rounding: l from the ROUNDED v (no contraction into a producing multiply)
template <int PS>
__device__ __forceinline__ void split_store_x3(bf16* dst, int64_t seg, const float* v, int pattern) {
#pragma clang fp contract(off)
  float hv[PS], lv[PS];
#pragma unroll
  for (int j = 0; j < PS; ++j) {
    hv[j] = (float)(bf16)v[j];
    lv[j] = v[j] - hv[j];
  }
  vstore<bf16, PS>(dst, hv);
  vstore<bf16, PS>(dst + seg, pattern ? lv : hv);
  vstore<bf16, PS>(dst + 2 * seg, pattern ? hv : lv);
}

// X3 (the bf16x3 engine, fp32 throughout): dx is also written as its pattern-1 split image img [R][3D] (segments
// h, l, h; clipmi_split3_colsum's layout and rounding) and dx's column sums -- the bias gradient of the Linear whose
// output gradient dx is -- join the partial rows: ws[blockIdx][3][D] (dgamma, dbeta, sum dx)
template <typename TX, typename T, int PS, int NP, typename TW = T, bool X3 = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* dy, int64_t lddy, const TX* x, int64_t ldx,
                                                     const float* mean, const float* rstd, const TW* w,
                                                     T* dx, int64_t lddx, const T* dres, int64_t ldres,
                                                     float* ws, int R, int D, bf16* img) {
  constexpr int NPR = X3 ? 3 : 2;
  __shared__ float red[4][NPR][NP * PS * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[NP][PS], pb[NP][PS], pd[NP][PS];
#pragma unroll
  for (int k = 0; k < NP; ++k)
#pragma unroll
    for (int j = 0; j < PS; ++j) { pg[k][j] = 0.f; pb[k][j] = 0.f; pd[k][j] = 0.f; }
  float wv[NP][PS];
#pragma unroll
  for (int k = 0; k < NP; ++k) vload<TW, PS>(w + (k * 64 + lane) * PS, wv[k]);
  // rows per wave and iteration, every load of them (dres, dy, x) issued before the first
  // reduction (as ln_fwd_kernel).  Two rows for D <= 512 (text: 67 -> 65 us at R = 78,848); one for
  // wider rows, where two rows' registers (164 VGPRs at D = 768) cost a wave per SIMD and measured
  // 3-4 % slower (tools/ln_bench.py, profiles/r02_ln_bwd_ab.log)
  // fp32 x with bf16 gradients (the fp32 residual stream): two rows at D = 768 too, 285 vs 293 us at
  // R = 201,728 (profiles/r05_ln_rows_per_wave_ab.log; with bf16 x two rows measured 234 vs 223 us)
  constexpr bool MIXED = std::is_same<TX, float>::value && !std::is_same<T, float>::value;
  constexpr int RPW = (NP * PS <= 8 || MIXED) ? 2 : 1;
  for (int row0 = (blockIdx.x * 4 + wave) * RPW; row0 < R; row0 += gridDim.x * 4 * RPW) {
    float g[RPW][NP][PS], xh[RPW][NP][PS], rr[RPW][NP][PS], d[RPW][NP][PS];
    float mu[RPW], rs[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int row = min(row0 + q, R - 1);  // a clamped duplicate row is computed, not stored
      mu[q] = mean[row];
      rs[q] = rstd[row];
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int c = (k * 64 + lane) * PS;
        if (dres) vload<T, PS>(dres + (int64_t)row * ldres + c, rr[q][k]);
        vload<T, PS>(dy + (int64_t)row * lddy + c, d[q][k]);
        vload<TX, PS>(x + (int64_t)row * ldx + c, xh[q][k]);
      }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const bool live = row0 + q < R;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NP; ++k)
#pragma unroll
        for (int j = 0; j < PS; ++j) {
          xh[q][k][j] = (xh[q][k][j] - mu[q]) * rs[q];
          g[q][k][j] = d[q][k][j] * wv[k][j];
          s1 += g[q][k][j];
          s2 += g[q][k][j] * xh[q][k][j];
          if (live) {
            pg[k][j] += d[q][k][j] * xh[q][k][j];
            pb[k][j] += d[q][k][j];
          }
        }
      s1 = wave_sum(s1) / D;
      s2 = wave_sum(s2) / D;
      if (!live) continue;
      const int row = row0 + q;
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int c = (k * 64 + lane) * PS;
        float o[PS];
#pragma unroll
        for (int j = 0; j < PS; ++j) {
          o[j] = rs[q] * (g[q][k][j] - s1 - xh[q][k][j] * s2);
          if (dres) o[j] += rr[q][k][j];
        }
        vstore<T, PS>(dx + (int64_t)row * lddx + c, o);
        if constexpr (X3) {
          split_store_x3<PS>(img + (int64_t)row * 3 * D + c, D, o, 1);
#pragma unroll
          for (int j = 0; j < PS; ++j) pd[k][j] += o[j];
        }
      }
    }
  }
  if (!ws) return;
#pragma unroll
  for (int k = 0; k < NP; ++k)
#pragma unroll
    for (int j = 0; j < PS; ++j) {
      red[wave][0][(k * 64 + lane) * PS + j] = pg[k][j];
      red[wave][1][(k * 64 + lane) * PS + j] = pb[k][j];
      if constexpr (X3) red[wave][2][(k * 64 + lane) * PS + j] = pd[k][j];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
#pragma unroll
    for (int u = 0; u < NPR; ++u)
      ws[((int64_t)blockIdx.x * NPR + u) * D + c] = red[0][u][c] + red[1][u][c] + red[2][u][c] + red[3][u][c];
  }
}

// ---- any hidden size (the register-resident kernels above take D / 64 in {1, 2, 3, 4, 6, 8, 12, 16}):
// one wave per row, three passes over the row (sum, centred sum of squares, normalise), the row
// re-read from the cache.  For the modules whose width is free (peclip ContextAdapter / SharedAdapter,
// nn.MultiheadAttention accepts any embed_dim divisible by num_heads; the adapters' LayerNorm).
template <typename TX, typename T>
__global__ __launch_bounds__(256) void ln_fwd_any_kernel(TX* x, int64_t ldx, T* y, int64_t ldy, const T* w, const T* b,
                                                         float* mean_out, float* rstd_out, int R, int D, float eps,
                                                         const TX* pos, const TX* cls, int period) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  TX* xr = x + (int64_t)row * ldx;
  const int t = pos ? row % period : 0;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) {
    float v = (float)xr[c];
    if (pos) {
      v += (float)pos[(int64_t)t * D + c];
      if (cls && t == 0) v += (float)cls[c];
      xr[c] = (TX)v;
      v = (float)xr[c];  // the stored (rounded) sum, as the register kernels normalise it
    }
    s += v;
  }
  const float mu = wave_sum(s) / D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = (float)xr[c] - mu;
    q += d * d;
  }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
  T* yr = y + (int64_t)row * ldy;
  for (int c = lane; c < D; c += 64) yr[c] = (T)(((float)xr[c] - mu) * rs * (float)w[c] + (float)b[c]);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mu;
    if (rstd_out) rstd_out[row] = rs;
  }
}

// dx = [dres +] rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w; per-block partial dgamma /
// dbeta -> ws[blockIdx][2][D] (each wave's own LDS row pair, summed in wave order: deterministic)
template <typename TX, typename T, typename TW = T>
__global__ __launch_bounds__(256) void ln_bwd_any_kernel(const T* dy, int64_t lddy, const TX* x, int64_t ldx,
                                                         const float* mean, const float* rstd, const TW* w, T* dx,
                                                         int64_t lddx, const T* dres, int64_t ldres, float* ws, int R,
                                                         int D) {
  extern __shared__ float red_any[];  // [4 waves][2][D] when ws
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* pg = red_any + (int64_t)wave * 2 * D;
  float* pb = pg + D;
  if (ws)
    for (int c = lane; c < D; c += 64) pg[c] = pb[c] = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < R; row += gridDim.x * 4) {
    const float mu = mean[row], rs = rstd[row];
    const T* dyr = dy + (int64_t)row * lddy;
    const TX* xr = x + (int64_t)row * ldx;
    float s1 = 0.f, s2 = 0.f;
    for (int c = lane; c < D; c += 64) {
      const float g = (float)dyr[c] * (float)w[c];
      s1 += g;
      s2 += g * (((float)xr[c] - mu) * rs);
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
    for (int c = lane; c < D; c += 64) {
      const float d = (float)dyr[c], xh = ((float)xr[c] - mu) * rs;
      float o = rs * (d * (float)w[c] - s1 - xh * s2);
      if (dres) o += (float)dres[(int64_t)row * ldres + c];
      dx[(int64_t)row * lddx + c] = (T)o;
      if (ws) {
        pg[c] += d * xh;
        pb[c] += d;
      }
    }
  }
  if (!ws) return;
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    float a = 0.f, bb = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a += red_any[(int64_t)k * 2 * D + c];
      bb += red_any[(int64_t)k * 2 * D + D + c];
    }
    ws[(int64_t)blockIdx.x * 2 * D + c] = a;
    ws[(int64_t)blockIdx.x * 2 * D + D + c] = bb;
  }
}

constexpr int LN_ANY_MAX_D = 4096;  // 4 waves x 2 x D floats of LDS = 128 KiB

// out[c] (+)= sum_p ws[p*stride + c]   (deterministic second stage of every column sum)
// block = 64 columns x 16 partial groups; fixed summation order -> bitwise reproducible
__global__ __launch_bounds__(1024) void reduce_partials_kernel(const float* ws, int64_t stride, int P, int D,
                                                               float* out, int beta) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (c < D) {
    int p = ty;
    for (; p + 16 < P; p += 32) {
      s0 += ws[(int64_t)p * stride + c];
      s1 += ws[(int64_t)(p + 16) * stride + c];
    }
    if (p < P) s0 += ws[(int64_t)p * stride + c];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && c < D) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    out[c] = beta ? out[c] + s : s;
  }
}

// the same sum over up to two column ranges at once: columns [0, D) -> out, [D, 2D) -> out2
// (out2 may be null: grid covers D columns only).  16 lanes x 4 columns per partial group,
// 64 groups, eight loads in flight per lane, fixed-order LDS tree: the one-float-per-lane
// kernel above waits ~P/32 HBM round trips on only D/64 workgroups (43 us at P=1024, D=768).
// D % 4 == 0, stride % 4 == 0, ws 16-B aligned.
__global__ __launch_bounds__(1024) void reduce_partials4_kernel(const float* ws, int64_t stride, int P, int D,
                                                                float* out, float* out2, int beta) {
  __shared__ float4 red[64][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + tx * 4;
  const int Dt = out2 ? 2 * D : D;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < Dt) {
    const float* src = ws + c;
    int p = ty;
    for (; p + 7 * 64 < P; p += 8 * 64) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(src + (int64_t)(p + j * 64) * stride);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w;
      }
    }
    for (; p < P; p += 64) {
      const float4 v = *(const float4*)(src + (int64_t)p * stride);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[ty][tx] = acc;
  __syncthreads();
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ty < 16) {
    a = red[ty * 4][tx];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 b = red[ty * 4 + k][tx];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  __syncthreads();
  if (ty < 16) red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < Dt) {
    float4 t = red[0][tx];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      const float4 b = red[k][tx];
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
    }
    float* o = c < D ? out + c : out2 + (c - D);
    if (beta) {
      t.x += o[0]; t.y += o[1]; t.z += o[2]; t.w += o[3];
    }
    o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
  }
}

// column partial sums of a [R, N] matrix: ws[chunk][N], chunk = blockIdx.y
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* x, int64_t ldx, int R, int N, int rows_per,
                                                             float* ws) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = r0; r < r1; ++r) {
    float v[4];
    load4(x + (int64_t)r * ldx + c, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] += v[j];
  }
  store4(ws + (int64_t)blockIdx.y * N + c, s);
}
// bf16x3 split image of an fp32 [R, N] matrix (k-major [R][3N], segments (h, h, l) for pattern 0 or (h, l, h) for
// pattern 1) and, when ws, its column partial sums ws[chunk][N] in the same pass (the bias gradient of the GEMM the
// matrix is the output gradient of); four rows in flight per thread
__global__ __launch_bounds__(256) void split3_colsum_kernel(const float* x, int64_t ldx, int R, int N, int rows_per,
                                                            bf16* out, int pattern, float* ws) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t ld3 = 3 * (int64_t)N;
  auto one = [&](int r, const f32x4& v) {
    bf16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[j] = (bf16)v[j];
      l[j] = (bf16)(v[j] - (float)h[j]);
      s[j] += v[j];
    }
    bf16* o = out + (int64_t)r * ld3 + c;
    *(bf16x4*)o = h;
    *(bf16x4*)(o + N) = pattern ? l : h;
    *(bf16x4*)(o + 2 * N) = pattern ? h : l;
  };
  int r = r0;
  for (; r + 4 <= r1; r += 4) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const f32x4*)(x + (int64_t)(r + u) * ldx + c);
#pragma unroll
    for (int u = 0; u < 4; ++u) one(r + u, v[u]);
  }
  for (; r < r1; ++r) one(r, *(const f32x4*)(x + (int64_t)r * ldx + c));
  if (ws) store4(ws + (int64_t)blockIdx.y * N + c, s);
}

// the same, one column per thread: any N, ldx and alignment (fp32 adapters of any bottleneck width)
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial1_kernel(const T* x, int64_t ldx, int R, int N, int rows_per,
                                                              float* ws) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += (float)x[(int64_t)r * ldx + c];
  ws[(int64_t)blockIdx.y * N + c] = s;
}

// periodic row sums: out[t][c] (+)= sum_b x[(b*period + t)*ldx + c]   (position-embedding grads)
// out[t][c..c+3] (+)= sum_b x[b*period + t][c..c+3] (position / class embedding gradients).
// One block per (column chunk of 256, position t); its 4 waves split the batch (rows b = w,
// w + 4, ...) with 8 independent loads in flight per lane, then add their partial sums in a
// fixed order through LDS (deterministic).  The one-thread-per-column form it replaces kept one
// load in flight per lane: latency bound at ~1 TB/s.
template <typename T>
__global__ __launch_bounds__(256) void period_sum_kernel(const T* x, int64_t ldx, int nb, int period, int D,
                                                         float* out, int beta) {
  __shared__ f32x4 part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const int t = blockIdx.y;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int b = w;
    for (; b + 28 < nb; b += 32) {
      float v[8][4];
#pragma unroll
      for (int u = 0; u < 8; ++u) load4(x + ((int64_t)(b + 4 * u) * period + t) * ldx + c, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += v[u][j];
    }
    for (; b < nb; b += 4) {
      float v[4];
      load4(x + ((int64_t)b * period + t) * ldx + c, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[j];
    }
  }
  part[w][lane] = f32x4{s[0], s[1], s[2], s[3]};
  __syncthreads();
  if (w == 0 && c < D) {
    f32x4 a = part[0][lane];
    a += part[1][lane];
    a += part[2][lane];
    a += part[3][lane];
    float* o = out + (int64_t)t * D + c;
    if (beta) a += *(const f32x4*)o;
    *(f32x4*)o = a;
  }
}

// x0[r] = tok[ids[r]] + pos[r % S]
template <typename T>
__global__ __launch_bounds__(256) void text_embed_kernel(const int64_t* ids, const T* tok, const T* pos, T* x0,
                                                         int R, int S, int D, int V, int* bad) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  int64_t id = ids[row];
  if (id < 0 || id >= V) { if (lane == 0) atomicOr(bad, 1); id = 0; }
  const T* a = tok + id * D;
  const T* p = pos + (int64_t)(row % S) * D;
  for (int c = lane * 4; c < D; c += 256) {
    float u[4], v[4];
    load4(a + c, u);
    load4(p + c, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) u[j] += v[j];
    store4(x0 + (int64_t)row * D + c, u);
  }
}

// ---- token-embedding backward: counting sort of ids (wave-aggregated atomics: runs of equal
// ids, e.g. EOS padding, take one atomic per run), then fixed 64-row chunks of the sorted
// order are summed by one wave each, flushing a partial row sum whenever the id changes.
// Work per wave is bounded however skewed the id histogram is (a padding id can own half
// the batch).
struct Run {
  int id, leader, len;
};
__device__ __forceinline__ Run lane_run(int id, int lane) {
  int prev = __shfl_up(id, 1, 64);
  const bool start = lane == 0 || id != prev;
  const unsigned long long starts = __ballot(start);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  const int leader = 63 - __builtin_clzll(starts & upto);
  const unsigned long long after = starts & ~upto;
  const int next = after ? __builtin_ctzll(after) : 64;
  return Run{id, leader, next - lane};
}

__global__ void id_count_kernel(const int64_t* ids, int R, int V, int* counts) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int id = -1;
  if (r < R && ids[r] >= 0 && ids[r] < V) id = (int)ids[r];
  const Run run = lane_run(id, lane);
  if (run.leader == lane && id >= 0) atomicAdd(&counts[id], run.len);
}

// exclusive scan of counts[V] -> offs[V+1], cursor[V] = offs[v]; one 1024-thread block.
__global__ __launch_bounds__(1024) void id_scan_kernel(const int* counts, int V, int* offs, int* cursor) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (V + 1023) / 1024;
  const int b = t * per, e = min(V, b + per);
  int s = 0;
  for (int v = b; v < e; ++v) s += counts[v];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int add = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  int run = part[t] - s;
  for (int v = b; v < e; ++v) {
    offs[v] = run;
    cursor[v] = run;
    run += counts[v];
  }
  if (t == 1023) offs[V] = part[1023];
}

__global__ void id_place_kernel(const int64_t* ids, int R, int V, int* cursor, int* perm, int* sorted_id) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int id = -1;
  if (r < R && ids[r] >= 0 && ids[r] < V) id = (int)ids[r];
  const Run run = lane_run(id, lane);
  int base = 0;
  if (run.leader == lane && id >= 0) base = atomicAdd(&cursor[id], run.len);
  base = __shfl(base, run.leader, 64);
  if (id >= 0) {
    perm[base + lane - run.leader] = r;
    sorted_id[base + lane - run.leader] = id;
  }
}

// one wave per 64 sorted rows; gtok[id] += rows of that id (fp32 atomics at id changes)
template <typename T>
__global__ __launch_bounds__(256) void id_chunk_sum_kernel(const int* perm, const int* sorted_id, const int* nvalid,
                                                           const T* dx0, int D, float* gtok) {
  const int n = *nvalid;  // rows with an in-vocabulary id (offs[V])
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = c * 64, e = min(n, b + 64);
  if (b >= n) return;
  for (int c0 = lane * 4; c0 < D; c0 += 256) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    int cur = sorted_id[b];
    for (int i = b; i < e; ++i) {
      const int id = sorted_id[i];
      if (id != cur) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { atomicAdd(gtok + (int64_t)cur * D + c0 + j, s[j]); s[j] = 0.f; }
        cur = id;
      }
      float u[4];
      load4(dx0 + (int64_t)perm[i] * D + c0, u);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += u[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(gtok + (int64_t)cur * D + c0 + j, s[j]);
  }
}

template <typename TX, typename T, int PS, int NP>
void ln_fwd_launch(hipStream_t s, void* x, int64_t ldx, void* y, int64_t ldy, const void* w, const void* b,
                   float* mean, float* rstd, int R, int D, float eps, const void* pos, const void* cls, int period) {
  hipLaunchKernelGGL((ln_fwd_kernel<TX, T, PS, NP>), dim3((R + 4 * LN_RPW - 1) / (4 * LN_RPW)), dim3(256), 0, s, (TX*)x, ldx,
                     (T*)y, ldy, (const T*)w, (const T*)b, mean, rstd, R, D, eps, (const TX*)pos, (const TX*)cls, period);
}
template <typename TX, typename T, int PS, int NP>
void ln_fwd_x3_launch(hipStream_t s, void* x, int64_t ldx, void* y3, int pattern, const void* w, const void* b,
                      float* mean, float* rstd, int R, int D, float eps) {
  const dim3 g((R + 4 * LN_RPW - 1) / (4 * LN_RPW));
  if (pattern == 0)
    hipLaunchKernelGGL((ln_fwd_kernel<TX, T, PS, NP, false, 1>), g, dim3(256), 0, s, (TX*)x, ldx, (T*)y3, (int64_t)3 * D,
                       (const T*)w, (const T*)b, mean, rstd, R, D, eps, (const TX*)nullptr, (const TX*)nullptr, 1,
                       (uint8_t*)nullptr, (uint8_t*)nullptr);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<TX, T, PS, NP, false, 2>), g, dim3(256), 0, s, (TX*)x, ldx, (T*)y3, (int64_t)3 * D,
                       (const T*)w, (const T*)b, mean, rstd, R, D, eps, (const TX*)nullptr, (const TX*)nullptr, 1,
                       (uint8_t*)nullptr, (uint8_t*)nullptr);
}
template <typename TX, typename T, int PS, int NP>
void ln_fwd_q8_launch(hipStream_t s, void* x, int64_t ldx, uint8_t* q8, uint8_t* s8, const void* w, const void* b,
                      float* mean, float* rstd, int R, int D, float eps) {
  if constexpr (PS == 4) {
    hipLaunchKernelGGL((ln_fwd_kernel<TX, T, PS, NP, true>), dim3((R + 4 * LN_RPW - 1) / (4 * LN_RPW)), dim3(256), 0, s,
                       (TX*)x, ldx, (T*)nullptr, (int64_t)0, (const T*)w, (const T*)b, mean, rstd, R, D, eps,
                       (const TX*)nullptr, (const TX*)nullptr, 1, q8, s8);
  }
}
// grid (in: the partial-sum rows the workspace holds; out: the blocks launched = partial rows
// written): at most the blocks the CUs hold at once, so no block starts a second round late
// (the D = 768 form keeps two rows' loads in registers: 164 VGPRs, 3 waves per SIMD)
template <typename TX, typename T, int PS, int NP, typename TW = T, bool X3 = false>
void ln_bwd_launch(hipStream_t s, int& grid, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                   const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx, const void* dres,
                   int64_t ldres, float* ws, int R, int D, void* img = nullptr) {
  static int resident = [] {
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)ln_bwd_kernel<TX, T, PS, NP, TW, X3>, 256,
                                                     0) != hipSuccess || per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    return per_cu * cus;
  }();
  if (grid > resident) grid = resident;
  hipLaunchKernelGGL((ln_bwd_kernel<TX, T, PS, NP, TW, X3>), dim3(grid), dim3(256), 0, s, (const T*)dy, lddy,
                     (const TX*)x, ldx, mean, rstd, (const TW*)w, (T*)dx, lddx, (const T*)dres, ldres, ws, R, D,
                     (bf16*)img);
}
// the bf16x3 form (fp32 everything, dx's image + column sums)
template <typename TX, typename T, int PS, int NP>
void ln_bwd_x3_launch(hipStream_t s, int& grid, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                      const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx, const void* dres,
                      int64_t ldres, float* ws, int R, int D, void* img) {
  ln_bwd_launch<TX, T, PS, NP, T, true>(s, grid, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, ws, R, D, img);
}

template <typename TX, typename T, int PS, int NP>
void ln_bwd_launch_w32(hipStream_t s, int& grid, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                       const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx, const void* dres,
                       int64_t ldres, float* ws, int R, int D) {
  ln_bwd_launch<TX, T, PS, NP, float>(s, grid, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, ws, R, D);
}

// the widths the register-resident kernels take
inline bool ln_fast_width(int D) {
  if (D % 64) return false;
  const int q = D / 64;
  return q == 1 || q == 2 || q == 3 || q == 4 || q == 6 || q == 8 || q == 12 || q == 16;
}

// dispatch on (PS, NP) from D
// (TX: the normalised input x; T: everything else -- output / gradients / affine weights)
#define LN_DISPATCH(D, FN, TX, T, ...)                                          \
  do {                                                                          \
    const int q_ = (D) / 64;                                                    \
    if (q_ == 16) FN<TX, T, 4, 4>(__VA_ARGS__);                                 \
    else if (q_ == 12) FN<TX, T, 4, 3>(__VA_ARGS__);                            \
    else if (q_ == 8) FN<TX, T, 4, 2>(__VA_ARGS__);                             \
    else if (q_ == 4) FN<TX, T, 4, 1>(__VA_ARGS__);                             \
    else if (q_ == 2) FN<TX, T, 2, 1>(__VA_ARGS__);                             \
    else if (q_ == 1) FN<TX, T, 1, 1>(__VA_ARGS__);                             \
    else if (q_ == 6) FN<TX, T, 2, 3>(__VA_ARGS__);                             \
    else if (q_ == 3) FN<TX, T, 1, 3>(__VA_ARGS__);                             \
    else return clipmi_invalid("layernorm: unsupported hidden size");           \
  } while (0)

}  // namespace

// ------------------------------------------------------------------------- C ABI
// x_dtype: the normalised input's dtype; dtype: the output's, the affine weights' and (backward) the
// gradients'.  Combinations: equal dtypes, or fp32 x with bf16 everything else (the bf16 mode's fp32
// residual stream feeding bf16 GEMM operands).
static int ln_types_ok(int x_dtype, int dtype) {
  return (dtype == CLIPMI_BF16 || dtype == CLIPMI_F32) && (x_dtype == dtype || (x_dtype == CLIPMI_F32 && dtype == CLIPMI_BF16));
}

template <typename TX, typename T>
static int ln_fwd_t(hipStream_t s, void* x, int64_t ldx, void* y, int64_t ldy, const void* w, const void* b, float* mean,
                    float* rstd, int R, int D, float eps, const void* pos, const void* cls, int period) {
  if (!ln_fast_width(D)) {  // any other width: the one-wave-per-row kernel
    hipLaunchKernelGGL((ln_fwd_any_kernel<TX, T>), dim3((R + 3) / 4), dim3(256), 0, s, (TX*)x, ldx, (T*)y, ldy,
                       (const T*)w, (const T*)b, mean, rstd, R, D, eps, (const TX*)pos, (const TX*)cls, period);
    return CLIPMI_OK;
  }
  LN_DISPATCH(D, ln_fwd_launch, TX, T, s, x, ldx, y, ldy, w, b, mean, rstd, R, D, eps, pos, cls, period);
  return CLIPMI_OK;
}

extern "C" int clipmi_layernorm_fwd2(void* stream, int x_dtype, int dtype, void* x, int64_t ldx, void* y, int64_t ldy,
                                     const void* w, const void* b, float* mean, float* rstd, int R, int D, float eps,
                                     const void* pos, const void* cls, int period) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ln_types_ok(x_dtype, dtype), "layernorm: dtypes (equal, or fp32 x with bf16 y)");
  CLIPMI_REQUIRE(D >= 1 && D <= LN_ANY_MAX_D, "D must be in [1, 4096]");
  CLIPMI_REQUIRE(!pos || period > 0, "period");
  if (R == 0) return CLIPMI_OK;
  if (dtype == CLIPMI_F32) CLIPMI_TRY((ln_fwd_t<float, float>(s, x, ldx, y, ldy, w, b, mean, rstd, R, D, eps, pos, cls, period)));
  else if (x_dtype == CLIPMI_F32) CLIPMI_TRY((ln_fwd_t<float, bf16>(s, x, ldx, y, ldy, w, b, mean, rstd, R, D, eps, pos, cls, period)));
  else CLIPMI_TRY((ln_fwd_t<bf16, bf16>(s, x, ldx, y, ldy, w, b, mean, rstd, R, D, eps, pos, cls, period)));
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_layernorm_fwd(void* stream, int dtype, void* x, int64_t ldx, void* y, int64_t ldy,
                                    const void* w, const void* b, float* mean, float* rstd, int R, int D,
                                    float eps, const void* pos, const void* cls, int period) {
  return clipmi_layernorm_fwd2(stream, dtype, dtype, x, ldx, y, ldy, w, b, mean, rstd, R, D, eps, pos, cls, period);
}

// fp32 x / weights -> the bf16x3 split image [R][3D] of y (pattern 0: segments h, h, l; 1: h, l, h)
extern "C" int clipmi_layernorm_fwd_x3(void* stream, const float* x, int64_t ldx, void* y3, int pattern, const float* w,
                                       const float* b, float* mean, float* rstd, int R, int D, float eps) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ln_fast_width(D), "layernorm_fwd_x3: D / 64 must be one of 1, 2, 3, 4, 6, 8, 12, 16");
  CLIPMI_REQUIRE(x && y3 && w && b && (pattern == 0 || pattern == 1), "layernorm_fwd_x3: arguments");
  if (R == 0) return CLIPMI_OK;
  LN_DISPATCH(D, ln_fwd_x3_launch, float, float, s, (void*)x, ldx, y3, pattern, w, b, mean, rstd, R, D, eps);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_layernorm_fwd_mxfp8(void* stream, int dtype, const void* x, int64_t ldx, uint8_t* q8,
                                          uint8_t* s8, const void* w, const void* b, float* mean, float* rstd, int R,
                                          int D, float eps) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(dtype == CLIPMI_BF16, "layernorm_fwd_mxfp8: bf16 input");
  CLIPMI_REQUIRE(D % 256 == 0 && D <= 1024, "layernorm_fwd_mxfp8: D must be a multiple of 256, <= 1024");
  CLIPMI_REQUIRE(q8 && s8, "layernorm_fwd_mxfp8: outputs");
  if (R == 0) return CLIPMI_OK;
  LN_DISPATCH(D, ln_fwd_q8_launch, bf16, bf16, s, (void*)x, ldx, q8, s8, w, b, mean, rstd, R, D, eps);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// workspace: >= 2*D*nblk floats where nblk = min(1024, ceil(R/4)); clipmi_layernorm_bwd_ws
extern "C" int64_t clipmi_layernorm_bwd_ws(int R, int D) {
  int nb = (R + 3) / 4;
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  return (int64_t)nb * 2 * D * 4;
}

template <typename TX, typename T, typename TW = T>
static int ln_bwd_t(hipStream_t s, int& nb, const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* mean,
                    const float* rstd, const void* w, void* dx, int64_t lddx, const void* dres, int64_t ldres, float* wsf,
                    int R, int D) {
  if (!ln_fast_width(D)) {
    const size_t lds = wsf ? (size_t)4 * 2 * D * 4 : 0;
    (void)lds_optin((const void*)ln_bwd_any_kernel<TX, T, TW>, (int)lds);
    hipLaunchKernelGGL((ln_bwd_any_kernel<TX, T, TW>), dim3(nb), dim3(256), lds, s, (const T*)dy, lddy, (const TX*)x, ldx,
                       mean, rstd, (const TW*)w, (T*)dx, lddx, (const T*)dres, ldres, wsf, R, D);
    return CLIPMI_OK;
  }
  if constexpr (std::is_same<TW, T>::value)
    LN_DISPATCH(D, ln_bwd_launch, TX, T, s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D);
  else
    LN_DISPATCH(D, ln_bwd_launch_w32, TX, T, s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D);
  return CLIPMI_OK;
}

extern "C" int clipmi_layernorm_bwd(void* stream, int dtype, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                                    const float* mean, const float* rstd, const void* w, void* dx, int64_t lddx,
                                    const void* dres, int64_t ldres, float* dw, float* db, int beta_wb,
                                    void* ws, int64_t ws_bytes, int R, int D) {
  return clipmi_layernorm_bwd2(stream, dtype, dtype, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, dw, db,
                               beta_wb, ws, ws_bytes, R, D);
}

extern "C" int clipmi_layernorm_bwd2(void* stream, int x_dtype, int dtype, const void* dy, int64_t lddy, const void* x,
                                     int64_t ldx, const float* mean, const float* rstd, const void* w, void* dx,
                                     int64_t lddx, const void* dres, int64_t ldres, float* dw, float* db, int beta_wb,
                                     void* ws, int64_t ws_bytes, int R, int D) {
  return clipmi_layernorm_bwd3(stream, x_dtype, dtype, dtype, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, dw,
                               db, beta_wb, ws, ws_bytes, R, D);
}

// w_dtype: the affine weight's dtype -- dtype, or fp32 with fp32 x and bf16 gradients (a LayerNorm whose forward
// normalised with fp32 master weights, e.g. the vision pre_layrnorm on the fp32 residual stream)
extern "C" int clipmi_layernorm_bwd3(void* stream, int x_dtype, int dtype, int w_dtype, const void* dy, int64_t lddy,
                                     const void* x, int64_t ldx, const float* mean, const float* rstd, const void* w,
                                     void* dx, int64_t lddx, const void* dres, int64_t ldres, float* dw, float* db,
                                     int beta_wb, void* ws, int64_t ws_bytes, int R, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ln_types_ok(x_dtype, dtype), "layernorm: dtypes (equal, or fp32 x with bf16 gradients)");
  CLIPMI_REQUIRE(w_dtype == dtype || (w_dtype == CLIPMI_F32 && x_dtype == CLIPMI_F32),
                 "layernorm: weight dtype (the gradients', or fp32 with fp32 x)");
  CLIPMI_REQUIRE(D >= 1 && D <= LN_ANY_MAX_D, "D must be in [1, 4096]");
  if (R == 0) return CLIPMI_OK;
  int nb = (R + 3) / 4;
  if (nb > 1024) nb = 1024;
  float* wsf = (dw || db) ? (float*)ws : nullptr;
  if (wsf) CLIPMI_REQUIRE(ws_bytes >= (int64_t)nb * 2 * D * 4, "layernorm_bwd workspace too small");
  // the fast kernels shrink nb to the resident block count (the partial rows they write)
  if (dtype == CLIPMI_F32) CLIPMI_TRY((ln_bwd_t<float, float>(s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D)));
  else if (x_dtype == CLIPMI_F32 && w_dtype == CLIPMI_F32)
    CLIPMI_TRY((ln_bwd_t<float, bf16, float>(s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D)));
  else if (x_dtype == CLIPMI_F32) CLIPMI_TRY((ln_bwd_t<float, bf16>(s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D)));
  else CLIPMI_TRY((ln_bwd_t<bf16, bf16>(s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R, D)));
  CLIPMI_CHECK_LAUNCH();
  if (((uintptr_t)wsf & 15) != 0 || D % 4 != 0) {
    if (dw) hipLaunchKernelGGL(reduce_partials_kernel, dim3((D + 63) / 64), dim3(1024), 0, s, wsf, (int64_t)2 * D, nb, D, dw, beta_wb);
    if (db) hipLaunchKernelGGL(reduce_partials_kernel, dim3((D + 63) / 64), dim3(1024), 0, s, wsf + D, (int64_t)2 * D, nb, D, db, beta_wb);
  } else if (dw && db) {
    DeferredReduce r;
    memset(&r, 0, sizeof(r));
    r.kind = 2;
    r.part = wsf; r.stride = (int64_t)2 * D; r.P = nb; r.D = D; r.out = dw; r.out2 = db; r.pbeta = beta_wb;
    DeferredReduce* slot = deferred_slot();
    if (slot && slot->kind == 0) *slot = r;  // executed by the next persistent GEMM launch (engine backward)
    else CLIPMI_TRY(launch_partials_reduce(s, r));
  } else if (dw)
    hipLaunchKernelGGL(reduce_partials4_kernel, dim3((D + 63) / 64), dim3(1024), 0, s, wsf, (int64_t)2 * D, nb, D, dw, (float*)nullptr, beta_wb);
  else if (db)
    hipLaunchKernelGGL(reduce_partials4_kernel, dim3((D + 63) / 64), dim3(1024), 0, s, wsf + D, (int64_t)2 * D, nb, D, db, (float*)nullptr, beta_wb);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// bf16x3 engine: clipmi_layernorm_bwd (fp32 throughout, D / 64 in {1, 2, 3, 4, 6, 8, 12, 16}) that also writes dx as
// its pattern-1 split image dimg [R][3D] and adds dx's column sums onto colsum[D] (+= when beta_cs): the next
// GEMMs' operand and the bias gradient of the Linear whose output gradient dx is, without a split pass.  dw / db are
// required; ws >= clipmi_layernorm_bwd_x3_ws(R, D) bytes, 16-byte aligned.
extern "C" int64_t clipmi_layernorm_bwd_x3_ws(int R, int D) { return clipmi_layernorm_bwd_ws(R, D) / 2 * 3; }
extern "C" int clipmi_layernorm_bwd_x3(void* stream, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                                       const float* mean, const float* rstd, const float* w, float* dx, int64_t lddx,
                                       const float* dres, int64_t ldres, float* dw, float* db, int beta_wb, void* dimg,
                                       float* colsum, int beta_cs, void* ws, int64_t ws_bytes, int R, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ln_fast_width(D), "layernorm_bwd_x3: D / 64 must be one of 1, 2, 3, 4, 6, 8, 12, 16");
  CLIPMI_REQUIRE(dy && x && mean && rstd && w && dx && dw && db && dimg && colsum, "layernorm_bwd_x3: arguments");
  CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_layernorm_bwd_x3_ws(R, D) && ((uintptr_t)ws & 15) == 0 &&
                     ((uintptr_t)dimg & 7) == 0,
                 "layernorm_bwd_x3: workspace (clipmi_layernorm_bwd_x3_ws, 16-byte aligned), dimg 8-byte aligned");
  if (R == 0) return CLIPMI_OK;
  int nb = (R + 3) / 4;
  if (nb > 1024) nb = 1024;
  float* wsf = (float*)ws;
  LN_DISPATCH(D, ln_bwd_x3_launch, float, float, s, nb, dy, lddy, x, ldx, mean, rstd, w, dx, lddx, dres, ldres, wsf, R,
              D, dimg);
  CLIPMI_CHECK_LAUNCH();
  DeferredReduce r;
  memset(&r, 0, sizeof(r));
  r.kind = 2;
  r.part = wsf; r.stride = (int64_t)3 * D; r.P = nb; r.D = D; r.out = dw; r.out2 = db; r.pbeta = beta_wb;
  CLIPMI_TRY(launch_partials_reduce(s, r));
  r.part = wsf + 2 * D; r.out = colsum; r.out2 = nullptr; r.pbeta = beta_cs;
  CLIPMI_TRY(launch_partials_reduce(s, r));
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

int launch_partials_reduce(hipStream_t s, const DeferredReduce& r) {
  const int Dt = r.out2 ? 2 * r.D : r.D;
  hipLaunchKernelGGL(reduce_partials4_kernel, dim3((Dt + 63) / 64), dim3(1024), 0, s, r.part, r.stride, r.P, r.D, r.out,
                     r.out2, r.pbeta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int64_t clipmi_colsum_ws(int R, int N) {
  int chunks = (R + 255) / 256;
  if (chunks > 512) chunks = 512;
  if (chunks < 1) chunks = 1;
  return (int64_t)chunks * N * 4;
}

extern "C" int64_t clipmi_split3_colsum_ws(int R, int N) {
  int chunks = (R + 127) / 128;
  if (chunks > 1024) chunks = 1024;
  if (chunks < 1) chunks = 1;
  return (int64_t)chunks * N * 4;
}

// bf16x3 mode: the split image out [R][3N] (pattern 0: h, h, l; 1: h, l, h) of x [R, N] fp32, and with colsum its
// column sums added to colsum[N] (+= when beta) -- the bias gradient read in the same pass
extern "C" int clipmi_split3_colsum(void* stream, const float* x, int64_t ldx, int R, int N, void* out, int pattern,
                                    float* colsum, int beta, void* ws, int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(x && out && (pattern == 0 || pattern == 1) && R >= 0, "split3_colsum: arguments");
  CLIPMI_REQUIRE(N % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 7) == 0,
                 "split3_colsum: N, ldx multiples of 4, x 16-byte and out 8-byte aligned");
  int chunks = (R + 127) / 128;
  if (chunks > 1024) chunks = 1024;
  if (chunks < 1) chunks = 1;
  CLIPMI_REQUIRE(!colsum || (ws && ws_bytes >= (int64_t)chunks * N * 4 && ((uintptr_t)ws & 15) == 0),
                 "split3_colsum: workspace (clipmi_split3_colsum_ws, 16-byte aligned)");
  if (R == 0 || N == 0) return CLIPMI_OK;
  const int rows_per = (R + chunks - 1) / chunks;
  hipLaunchKernelGGL(split3_colsum_kernel, dim3((N / 4 + 255) / 256, chunks), dim3(256), 0, s, x, ldx, R, N, rows_per,
                     (bf16*)out, pattern, colsum ? (float*)ws : nullptr);
  if (colsum)
    hipLaunchKernelGGL(reduce_partials4_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, (const float*)ws, (int64_t)N,
                       chunks, N, colsum, (float*)nullptr, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// out[n] (+)= sum_r x[r][n]   (bias gradients)
extern "C" int clipmi_colsum(void* stream, int dtype, const void* x, int64_t ldx, int R, int N, float* out, int beta,
                             void* ws, int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(N >= 0 && ldx >= N, "colsum: N >= 0, ldx >= N");
  int chunks = (R + 255) / 256;
  if (chunks > 512) chunks = 512;
  if (chunks < 1) chunks = 1;
  CLIPMI_REQUIRE(ws_bytes >= (int64_t)chunks * N * 4, "colsum workspace too small");
  if (N == 0) return CLIPMI_OK;
  int rows_per = (R + chunks - 1) / chunks;
  const size_t al = dtype == CLIPMI_BF16 ? 8 : 16;  // load4's vector width
  if (N % 4 || ldx % 4 || ((uintptr_t)x & (al - 1))) {
    dim3 g1((N + 255) / 256, chunks);
    if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(colsum_partial1_kernel<bf16>, g1, dim3(256), 0, s, (const bf16*)x, ldx, R, N, rows_per, (float*)ws);
    else hipLaunchKernelGGL(colsum_partial1_kernel<float>, g1, dim3(256), 0, s, (const float*)x, ldx, R, N, rows_per, (float*)ws);
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, (const float*)ws, (int64_t)N, chunks, N, out, beta);
    CLIPMI_CHECK_LAUNCH();
    return CLIPMI_OK;
  }
  dim3 g((N / 4 + 255) / 256, chunks);
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(colsum_partial_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)x, ldx, R, N, rows_per, (float*)ws);
  else hipLaunchKernelGGL(colsum_partial_kernel<float>, g, dim3(256), 0, s, (const float*)x, ldx, R, N, rows_per, (float*)ws);
  if (((uintptr_t)ws & 15) == 0 && N % 4 == 0)
    hipLaunchKernelGGL(reduce_partials4_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, (const float*)ws, (int64_t)N, chunks, N, out, (float*)nullptr, beta);
  else
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, (const float*)ws, (int64_t)N, chunks, N, out, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_period_sum(void* stream, int dtype, const void* x, int64_t ldx, int nb, int period, int nt,
                                 int D, float* out, int beta) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D % 4 == 0, "D % 4");
  CLIPMI_REQUIRE(nt >= 1 && nt <= period, "nt must be in [1, period]");
  dim3 g((D / 4 + 63) / 64, nt);
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(period_sum_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)x, ldx, nb, period, D, out, beta);
  else hipLaunchKernelGGL(period_sum_kernel<float>, g, dim3(256), 0, s, (const float*)x, ldx, nb, period, D, out, beta);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_text_embed(void* stream, int dtype, const int64_t* ids, const void* tok, const void* pos,
                                 void* x0, int R, int S, int D, int V, int* bad_flag) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D % 4 == 0, "D % 4");
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(text_embed_kernel<bf16>, dim3((R + 3) / 4), dim3(256), 0, s, ids, (const bf16*)tok, (const bf16*)pos, (bf16*)x0, R, S, D, V, bad_flag);
  else hipLaunchKernelGGL(text_embed_kernel<float>, dim3((R + 3) / 4), dim3(256), 0, s, ids, (const float*)tok, (const float*)pos, (float*)x0, R, S, D, V, bad_flag);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// workspace (ints): counts[V] + offs[V+1] + cursor[V] + perm[R] + sorted_id[R]
extern "C" int64_t clipmi_text_embed_bwd_ws(int R, int V) { return ((int64_t)3 * V + 1 + 2 * (int64_t)R) * 4; }

extern "C" int clipmi_text_embed_bwd(void* stream, int dtype, const int64_t* ids, const void* dx0, int R, int D, int V,
                                     float* gtok, int beta, void* ws, int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(ws_bytes >= clipmi_text_embed_bwd_ws(R, V), "text_embed_bwd workspace too small");
  CLIPMI_REQUIRE(D % 4 == 0, "D % 4");
  int* counts = (int*)ws;
  int* offs = counts + V;
  int* cursor = offs + V + 1;
  int* perm = cursor + V;
  int* sid = perm + R;
  if (!beta) CLIPMI_HIP(hipMemsetAsync(gtok, 0, (size_t)V * D * 4, s));
  CLIPMI_HIP(hipMemsetAsync(counts, 0, (size_t)V * 4, s));
  CLIPMI_HIP(hipMemsetAsync(sid, 0xff, (size_t)R * 4, s));
  hipLaunchKernelGGL(id_count_kernel, dim3((R + 255) / 256), dim3(256), 0, s, ids, R, V, counts);
  hipLaunchKernelGGL(id_scan_kernel, dim3(1), dim3(1024), 0, s, counts, V, offs, cursor);
  hipLaunchKernelGGL(id_place_kernel, dim3((R + 255) / 256), dim3(256), 0, s, ids, R, V, cursor, perm, sid);
  // rows with invalid ids were not placed: the sorted prefix has offs[V] entries
  const int chunks = (R + 63) / 64;
  if (dtype == CLIPMI_BF16) hipLaunchKernelGGL(id_chunk_sum_kernel<bf16>, dim3((chunks + 3) / 4), dim3(256), 0, s, perm, sid, offs + V, (const bf16*)dx0, D, gtok);
  else hipLaunchKernelGGL(id_chunk_sum_kernel<float>, dim3((chunks + 3) / 4), dim3(256), 0, s, perm, sid, offs + V, (const float*)dx0, D, gtok);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
