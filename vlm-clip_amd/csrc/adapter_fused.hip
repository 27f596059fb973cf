// The bottleneck adapter's forward as ONE kernel (bf16): y = LN(up(gelu_erf(down(x))) + x), the reference's
// TextAdapter / VisionAdapter.forward (adapter/clip_adapter.py:17-23, 144-150) and peclip.TextualAdapter
// (adapter/peclip.py:13-18) -- north_star's "fused LayerNorm + adapter", with the LayerNorm's row statistics as
// wavefront reductions inside the same workgroup instead of a third launch (clipmi_adapter_fwd's sequence:
// down GEMM -> up GEMM (+ residual) -> LayerNorm).
//
// One workgroup of 4 waves per 32 rows (R = the pooled rows: B per tower on the product path):
//   x tile   [32][D] bf16 in LDS (row stride D + 8: the 16 row lanes of a fragment read hit distinct banks);
//   down     h = gelu_erf(x Wd^T + bd): wave w owns 16-column tiles [w t, (w+1) t) (t = ceil(A / 64)), both row tiles;
//            operands on v_mfma_f32_16x16x32_bf16, x fragments from LDS, Wd fragments (8 consecutive k of one
//            weight row: 16 B) straight from global / L2 one k-step ahead; pre-activation and h stored (the
//            backward's inputs, as the sequence stores them), h also into an LDS tile [32][A + 8];
//   up       z = h Wu^T + bu + x in 64-column chunks (wave w: chunks w, w + 4, ...), z rounded to bf16 as the
//            sequence's GEMM epilogue does and written over the x tile in place (each lane reads its x element
//            before writing the same element) and to global;
//   LN       wave w normalises rows 8 w .. 8 w + 7 from the z tile: mean, then the centred sum of squares (two
//            wave_sum reductions per row), y = (z - mean) rstd g + b; mean / rstd stored for the backward.
// Accumulator layout (acc = mfma(weight fragment, activation fragment)): lane l holds row (l & 15) of the 16-row
// tile and columns 4 (l >> 4) + r of the 16-column tile -- the GEMM kernels' convention (gemm_common.h).
#include <cstdlib>
#include "common.h"
#include "internal.h"

namespace {

constexpr int AF_ROWS = 32, AF_W = 4, AF_THR = AF_W * 64;
constexpr int AF_MAXD = 1024, AF_MAXA = 512;  // D / A the one-pass prologue covers (adapter_fused_ok)
constexpr int AF_PRO = (AF_ROWS * AF_MAXD / 8 + AF_MAXA / 8 + 3 * AF_MAXD / 8 + AF_THR - 1) / AF_THR;

__device__ __forceinline__ bf16x8 gload8(const bf16* p) { return *(const bf16x8*)p; }

// acc[m][j] += W[n0 + 16 j + row][k] . T[16 m + row][k] over k < K (K % 32 == 0), j < ntl: T a bf16 LDS tile (row
// stride ldt), W a bf16 global [*][ldw] matrix whose fragments (16 B of one row) stream through an 8-step register
// ring.  Every step issues exactly four loads (the refill of its slot, clamped to a valid row and step past the
// end) so the compiler can count them: a use waits only for its own step's loads (vmcnt 28), not for the seven
// steps in flight -- with data-dependent load counts it drained the queue (vmcnt 0) at every step, 0.6 us each.
constexpr int AF_RING = 8;
__device__ __forceinline__ void af_kloop(f32x4 (&acc)[2][4], const bf16* W, int64_t ldw, int n0, int ntl, int K,
                                         const bf16* tile, int ldt, int li, int g) {
  const int ns = K / 32;
  const bf16* wr[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wr[j] = W + (int64_t)(n0 + min(j, ntl - 1) * 16 + li) * ldw + 8 * g;
  bf16x8 ring[AF_RING][4];
#pragma unroll
  for (int u = 0; u < AF_RING; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) ring[u][j] = gload8(wr[j] + min(u, ns - 1) * 32);
  for (int s0 = 0; s0 < ns; s0 += AF_RING) {
#pragma unroll
    for (int u = 0; u < AF_RING; ++u) {
      const int st = s0 + u;
      if (st < ns) {
        bf16x8 tf[2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
          tf[m] = *LDS_PTR(const bf16x8, (const char*)(tile + (m * 16 + li) * ldt + st * 32 + 8 * g));
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < ntl) acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[u][j], tf[m], acc[m][j], 0, 0, 0);
      }
      const int nx = min(st + AF_RING, ns - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) ring[u][j] = gload8(wr[j] + nx * 32);
    }
  }
}

__global__ __launch_bounds__(AF_THR) void adapter_fwd_fused_kernel(int R, int D, int A, const bf16* x, int64_t ldx,
                                                                   const bf16* wd, const bf16* bd, const bf16* wu,
                                                                   const bf16* bu, const bf16* lnw, const bf16* lnb,
                                                                   float eps, bf16* y, int64_t ldy, bf16* pre,
                                                                   bf16* act, bf16* z, float* mean, float* rstd,
                                                                   int diag) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ldt = D + 8, ldh = A + 8;  // LDS row strides (elements)
  bf16* xt = (bf16*)smem;                                        // [32][ldt]: x, then z
  bf16* ht = (bf16*)(smem + (size_t)AF_ROWS * ldt * 2);         // [32][ldh]: gelu(down)
  bf16* vec = ht + AF_ROWS * ldh;                                // bd [A] | bu [D] | lnw [D] | lnb [D]
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int r0 = blockIdx.x * AF_ROWS;
  const int li = lane & 15, g = lane >> 4;
  // ---- x tile (rows past R zero) and the bias / LayerNorm vectors into LDS: every 16-B load of a thread issued
  // before its first LDS write (a load -> write chain per piece waited out one memory round trip each)
  {
    const int xc = AF_ROWS * (D / 8), vc = A / 8 + 3 * (D / 8);
    // unconditional loads from clamped addresses (rows past R read row R - 1 and are zeroed after): straight-line
    // code, so the compiler issues all of them before its first wait
    bf16x8 v[AF_PRO];
#pragma unroll
    for (int u = 0; u < AF_PRO; ++u) {
      const int i = t + u * AF_THR;
      const int r = i / (D / 8), c = (i - r * (D / 8)) * 8;
      const int j = min(max(i - xc, 0), vc - 1) * 8;
      const bf16* xs = x + (int64_t)min(r0 + min(r, AF_ROWS - 1), R - 1) * ldx + (i < xc ? c : 0);
      const bf16* vs = j < A ? bd + j : j < A + D ? bu + (j - A) : j < A + 2 * D ? lnw + (j - A - D) : lnb + (j - A - 2 * D);
      v[u] = gload8(i < xc ? xs : vs);
    }
#pragma unroll
    for (int u = 0; u < AF_PRO; ++u) {
      const int i = t + u * AF_THR;
      if (i < xc) {
        const int r = i / (D / 8), c = (i - r * (D / 8)) * 8;
        *LDS_PTR(bf16x8, (char*)(xt + r * ldt + c)) = r0 + r < R ? v[u] : bf16x8{};
      } else if (i < xc + vc) {
        *LDS_PTR(bf16x8, (char*)(vec + (i - xc) * 8)) = v[u];
      }
    }
  }
  const bf16* bdl = vec;
  const bf16* bul = vec + A;
  const bf16* lnwl = vec + A + D;
  const bf16* lnbl = vec + A + 2 * D;
  __syncthreads();

  // ---- down projection: wave's bottleneck columns in 16-column tiles, both row tiles
  {
    const int nt = A / 16, tpw = (nt + AF_W - 1) / AF_W;  // 16-column tiles, tiles per wave
    const int t0 = wave * tpw, t1 = min(nt, t0 + tpw);
    for (int tt = t0; tt < t1; tt += 4) {  // up to 4 consecutive tiles at a time
      const int n0 = tt * 16, ntl = min(4, t1 - tt);
      f32x4 acc[2][4];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!(diag & 1)) af_kloop(acc, wd, D, n0, ntl, D, xt, ldt, li, g);
      // epilogue: + bias, pre stored, gelu_erf, h stored (global + LDS)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= ntl) continue;
        const int c = n0 + j * 16 + 4 * g;
        const bf16x4 bb = *LDS_PTR(const bf16x4, (const char*)(bdl + c));
        const float bv[4] = {(float)bb[0], (float)bb[1], (float)bb[2], (float)bb[3]};
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int r = m * 16 + li;
          float v[4], a[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // gelu of the fp32 pre-activation, as the sequence's GEMM epilogue
            v[q] = acc[m][j][q] + bv[q];
            a[q] = gelu_erf(v[q]);
          }
          const bf16x4 av = bf16x4{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
          *LDS_PTR(bf16x4, (char*)(ht + r * ldh + c)) = av;
          if (r0 + r < R) {
            *(bf16x4*)(act + (int64_t)(r0 + r) * A + c) = av;
            if (pre) *(bf16x4*)(pre + (int64_t)(r0 + r) * A + c) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          }
        }
      }
    }
  }
  __syncthreads();

  // ---- up projection + bias + residual -> z (bf16), over the x tile in place
  for (int n0 = wave * 64; n0 < D; n0 += AF_W * 64) {  // 64-column chunks, 4 tiles each (D % 64 == 0)
    f32x4 acc[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (!(diag & 2)) af_kloop(acc, wu, A, n0, 4, A, ht, ldh, li, g);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = n0 + j * 16 + 4 * g;
      const bf16x4 bb = *LDS_PTR(const bf16x4, (const char*)(bul + c));
      const float bv[4] = {(float)bb[0], (float)bb[1], (float)bb[2], (float)bb[3]};
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int r = m * 16 + li;
        bf16* zp = xt + r * ldt + c;
        const bf16x4 xv = *LDS_PTR(const bf16x4, (const char*)zp);
        const bf16x4 zv = bf16x4{(bf16)(acc[m][j][0] + bv[0] + (float)xv[0]), (bf16)(acc[m][j][1] + bv[1] + (float)xv[1]),
                                 (bf16)(acc[m][j][2] + bv[2] + (float)xv[2]), (bf16)(acc[m][j][3] + bv[3] + (float)xv[3])};
        *LDS_PTR(bf16x4, (char*)zp) = zv;
        if (r0 + r < R) *(bf16x4*)(z + (int64_t)(r0 + r) * D + c) = zv;
      }
    }
  }
  __syncthreads();

  // ---- LayerNorm of the z rows: wave w normalises rows 8w .. 8w + 7 together (their loads, sums and wavefront
  // reductions interleaved: one row at a time measured 10 us of dependent shuffle chains), lane c .. c + 3 of every
  // 256 columns as ln_fwd_kernel
  if (!(diag & 4)) {
    constexpr int NV = AF_MAXD / 256;
    const int rb = wave * (AF_ROWS / AF_W);
    float v[AF_ROWS / AF_W][NV][4];
#pragma unroll
    for (int q = 0; q < AF_ROWS / AF_W; ++q)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = lane * 4 + 256 * i;
        bf16x4 b4 = bf16x4{};
        if (c < D) b4 = *LDS_PTR(const bf16x4, (const char*)(xt + (rb + q) * ldt + c));
#pragma unroll
        for (int e = 0; e < 4; ++e) v[q][i][e] = (float)b4[e];
      }
    float mu[AF_ROWS / AF_W], rs[AF_ROWS / AF_W];
#pragma unroll
    for (int q = 0; q < AF_ROWS / AF_W; ++q) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) sum += v[q][i][e];  // padding columns hold zeros
      mu[q] = sum;
    }
#pragma unroll
    for (int q = 0; q < AF_ROWS / AF_W; ++q) mu[q] = wave_sum(mu[q]) / D;
#pragma unroll
    for (int q = 0; q < AF_ROWS / AF_W; ++q) {
      float sq = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        if (lane * 4 + 256 * i >= D) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[q][i][e] - mu[q];
          sq += d * d;
        }
      }
      rs[q] = sq;
    }
#pragma unroll
    for (int q = 0; q < AF_ROWS / AF_W; ++q) rs[q] = rsqrtf(wave_sum(rs[q]) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane * 4 + 256 * i;
      if (c >= D) continue;
      const bf16x4 wb = *LDS_PTR(const bf16x4, (const char*)(lnwl + c));
      const bf16x4 bb = *LDS_PTR(const bf16x4, (const char*)(lnbl + c));
#pragma unroll
      for (int q = 0; q < AF_ROWS / AF_W; ++q) {
        if (r0 + rb + q >= R) continue;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)((v[q][i][e] - mu[q]) * rs[q] * (float)wb[e] + (float)bb[e]);
        *(bf16x4*)(y + (int64_t)(r0 + rb + q) * ldy + c) = o;
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < AF_ROWS / AF_W; ++q)
        if (r0 + rb + q < R) {
          mean[r0 + rb + q] = mu[q];
          rstd[r0 + rb + q] = rs[q];
        }
    }
  }
}

}  // namespace

// LDS of the fused form for (D, A): the x / z tile and the bottleneck tile
int64_t adapter_fused_lds(int D, int A) {
  return (int64_t)AF_ROWS * (D + 8) * 2 + (int64_t)AF_ROWS * (A + 8) * 2 + (int64_t)(A + 3 * D) * 2;
}

// whether clipmi_adapter_fwd takes the fused kernel: bf16 with the LayerNorm, D % 64 == 0, A % 64 == 0, the tiles
// within 160 KiB, 16-byte aligned rows
bool adapter_fused_ok(int dtype, int ln, int D, int A, int64_t ldx, int64_t ldy) {
  return dtype == CLIPMI_BF16 && ln && D % 64 == 0 && A % 64 == 0 && D >= 64 && A >= 64 && D <= AF_MAXD &&
         A <= AF_MAXA && ldx % 8 == 0 && ldy % 4 == 0 && adapter_fused_lds(D, A) <= 160 * 1024;
}

int adapter_fwd_fused(void* stream, int R, int D, int A, const void* x, int64_t ldx, const void* w_down,
                      const void* b_down, const void* w_up, const void* b_up, const void* ln_w, const void* ln_b,
                      float eps, void* y, int64_t ldy, void* pre, void* act, void* z, float* mean, float* rstd) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t lds = adapter_fused_lds(D, A);
  (void)lds_optin((const void*)adapter_fwd_fused_kernel, (int)lds);
  hipLaunchKernelGGL(adapter_fwd_fused_kernel, dim3((R + AF_ROWS - 1) / AF_ROWS), dim3(AF_THR), lds, s, R, D, A,
                     (const bf16*)x, ldx, (const bf16*)w_down, (const bf16*)b_down, (const bf16*)w_up,
                     (const bf16*)b_up, (const bf16*)ln_w, (const bf16*)ln_b, eps, (bf16*)y, ldy, (bf16*)pre,
                     (bf16*)act, (bf16*)z, mean, rstd, [] {
                       const char* e = getenv("CLIPMI_ADAPTER_FUSED_DIAG");  // timing builds of the phases only
                       return e ? atoi(e) : 0;
                     }());
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
