// Multi-head attention (head_dim 64) forward/backward for the bf16x3 precision mode: fp32 q/k/v/O/dO in and
// fp32 O / dq / dk / dv out, every product on the bf16 MFMA as three split products.
//
// Replaces CLIPAttention's core + eager_attention_forward ([HF] modeling_clip.py:259-335) -- softmax(q k^T *
// 64^-0.5 + mask) v, fp32 softmax (`:272`), the text tower's causal + key-padding mask ([HF] :543-548) -- and
// its autograd backward, in the mode that keeps north_star's 1e-3 logits (the fp32 reference, trainer.py:81-99,
// has no autocast).  Round 5's bf16x3 mode ran attention on the exact-f32 SIMT kernels (attention.hip
// attn_fwd_f32 / attn_bwd_f32): 3.8 + 17.1 ms per ViT-B/16 layer at B = 1024, a third of that mode's step
// (profiles/r06_bf16x3_kernel_stats.txt).
//
// Every fp32 operand x is split as x = xh + xl, xh = bf16(x), xl = bf16(x - xh) (16 significant bits between
// them), and a product a.b runs as ah.bh + ah.bl + al.bh on v_mfma_f32_16x16x32_bf16 (every bf16 x bf16
// product exact in the fp32 accumulator; the dropped al.bl is ~2^-16 of each term) -- the split the tower
// GEMMs use (gemm.hip CLIPMI_GEMM_SPLIT3).  P and dS are split the same way before their products.  The
// softmax, log-sum-exp, delta = rowsum(dO * O) and all accumulation stay fp32.
//
// Structure: attention.hip's attn_fwd_pf / attn_bwd_mfma with each bf16 LDS image doubled into a hi and a lo
// image (same [Npad][64] swizzled layout, fragment readers from attn_frag.h): one workgroup of 8 waves per
// (batch, head); forward: K/V hi/lo images, each wave owns query blocks wave, wave + 8; backward: phase A (dK,
// dV; each wave owns 16 keys, Q/dO images) then phase B (dQ; 16 queries per wave, K/V images).  N <= 288
// (four images of 288 rows fill 144 KiB of the 160 KiB LDS); larger N run the f32 kernels.
#include "common.h"
#include "internal.h"
#include "attn_frag.h"

namespace {

constexpr int X3_MAX_N = 288;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float NEG_INF = -__builtin_huge_valf();

struct AttnX {
  const float* qkv; float* o; float* lse; const int64_t* kmask;
  const float* dout; float* dqkv;
  int B, H, N, D;
  float scale;
};

// 8 fp32 values -> hi / lo bf16 fragments
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, bf16x8& h, bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = (bf16)a[j];
    h[j + 4] = (bf16)b[j];
    l[j] = (bf16)(a[j] - (float)h[j]);
    l[j + 4] = (bf16)(b[j] - (float)h[j + 4]);
  }
}

// acc += ah.bh + ah.bl + al.bh
__device__ __forceinline__ f32x4 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// rows [0, Npad) of an fp32 [N][64] head slice (row stride ld) -> hi and lo images (rows >= N zero)
__device__ __forceinline__ void stage_x3(char* ih, char* il, const float* src, int64_t ld, int N, int Npad, int t,
                                         int nthr) {
  for (int id = t; id < Npad * 8; id += nthr) {
    const int r = id >> 3, c = id & 7;
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
    if (r < N) {
      a = *(const f32x4*)(src + (int64_t)r * ld + c * 8);
      b = *(const f32x4*)(src + (int64_t)r * ld + c * 8 + 4);
    }
    bf16x8 h, l;
    split8(a, b, h, l);
    *LDS_PTR(bf16x8, ih + img_off(r, c)) = h;
    *LDS_PTR(bf16x8, il + img_off(r, c)) = l;
  }
}

// the MFMA operand fragment of row r (columns kk * 32 + 8 g .. + 7) from global fp32, split; rows >= N zero
__device__ __forceinline__ void gfrag_x3(const float* rowbase, int64_t ld, int r, int N, int kk, int g, bf16x8& h,
                                         bf16x8& l) {
  f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
  if (r < N) {
    const float* p = rowbase + (int64_t)r * ld + kk * 32 + 8 * g;
    a = *(const f32x4*)p;
    b = *(const f32x4*)(p + 4);
  }
  split8(a, b, h, l);
}

// ------------------------------------------------------------------------------------------- forward
template <int NKT, bool MASKED>
__global__ __launch_bounds__(512, 1) void attn_fwd_x3(AttnX p, int causal) {
  constexpr int NPAD = NKT * 16, IMG = NPAD * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kh = smem;
  char* Kl = smem + IMG;
  char* Vh = smem + 2 * IMG;
  char* Vl = smem + 3 * IMG;
  int* keyok = (int*)(smem + 4 * IMG);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int b = blockIdx.x / p.H, h = blockIdx.x - (blockIdx.x / p.H) * p.H;
  const int N = p.N, D = p.D;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = p.qkv + (int64_t)b * N * ld + h * 64;
  stage_x3(Kh, Kl, base + D, ld, N, NPAD, t, 512);
  stage_x3(Vh, Vl, base + 2 * D, ld, N, NPAD, t, 512);
  if (MASKED)
    for (int k = t; k < NPAD; k += 512) keyok[k] = (k < N) && (!p.kmask || p.kmask[(int64_t)b * N + k] != 0);
  __syncthreads();
  const int g = lane >> 4, li = lane & 15;
  const float c2 = p.scale * LOG2E;
  const int nqb = (N + 15) >> 4;
  for (int qb = wave; qb < nqb; qb += 8) {
    const int q = qb * 16 + li;
    bf16x8 qh[2], ql[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) gfrag_x3(base, ld, q, N, kk, g, qh[kk], ql[kk]);
    // key-major scores: lane (g, li) holds keys kt * 16 + 4 g + r of query li
    f32x4 sc[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      sc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        sc[kt] = mfma3(frag_row(Kh, kt * 16 + li, kk * 4 + g), frag_row(Kl, kt * 16 + li, kk * 4 + g), qh[kk], ql[kk],
                       sc[kt]);
      // one tile's fragment reads in flight at a time: hoisting every tile's K fragments (16 VGPRs each) above
      // the MFMAs spilled from NKT = 10 on
      __builtin_amdgcn_sched_barrier(0);
    }
    float mx = NEG_INF;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 16 + 4 * g + r;
        if (MASKED) {
          if (!(keyok[key] && (!causal || key <= q))) sc[kt][r] = NEG_INF;
        } else if (kt >= NKT - 2 && key >= N) {  // NPAD = N rounded up to 32: padding in the last two tiles only
          sc[kt][r] = NEG_INF;
        }
        mx = fmaxf(mx, sc[kt][r]);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mref = mx == NEG_INF ? 0.f : mx * c2;
    float lsum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][r], c2, -mref));
        sc[kt][r] = e;
        lsum += e;
      }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    // O^T = V^T P^T, the P tile split per 32-key step straight from the score registers
    f32x4 acc[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKT / 2; ++ks) {
      bf16x8 ph, pl;
      split8(sc[2 * ks], sc[2 * ks + 1], ph, pl);
#pragma unroll
      for (int v = 0; v < 4; ++v)
        acc[v] = mfma3(frag_tr(Vh, ks * 32, v * 16, lane), frag_tr(Vl, ks * 32, v * 16, lane), ph, pl, acc[v]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (q < N) {
      const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
      float* orow = p.o + ((int64_t)b * N + q) * D + h * 64;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float w[4] = {acc[v][0] * inv, acc[v][1] * inv, acc[v][2] * inv, acc[v][3] * inv};
        store4(orow + v * 16 + 4 * g, w);
      }
      if (g == 0) p.lse[((int64_t)b * p.H + h) * N + q] = lsum > 0.f ? (mref + __log2f(lsum)) * LN2 : NEG_INF;
    }
  }
}

// ------------------------------------------------------------------------------------------ backward
template <bool CAUSAL>
__global__ __launch_bounds__(512, 1) void attn_bwd_x3(AttnX p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int b = blockIdx.x / p.H, h = blockIdx.x - (blockIdx.x / p.H) * p.H;
  const int N = p.N, D = p.D;
  const int NPAD = (N + 31) & ~31;
  const int IMG = NPAD * 128;
  const int64_t ld = 3 * (int64_t)D;
  char* i0h = smem;            // phase A: Q,  phase B: K
  char* i0l = smem + IMG;
  char* i1h = smem + 2 * IMG;  // phase A: dO, phase B: V
  char* i1l = smem + 3 * IMG;
  float* lse2 = (float*)(smem + 4 * IMG);
  float* delta = lse2 + NPAD;
  int* keyok = (int*)(delta + NPAD);
  const float* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const float* dob = p.dout + (int64_t)b * N * D + h * 64;
  stage_x3(i0h, i0l, base, ld, N, NPAD, t, 512);
  stage_x3(i1h, i1l, dob, D, N, NPAD, t, 512);
  {  // delta[q] = sum_d dO * O in fp32, 8 lanes per row
    const float* ob = p.o + (int64_t)b * N * D + h * 64;
    for (int id = t; id < NPAD * 8; id += 512) {
      const int r = id >> 3, c = id & 7;
      float s = 0.f;
      if (r < N) {
        float a[4], bb[4];
        load4(dob + (int64_t)r * D + c * 8, a);
        load4(ob + (int64_t)r * D + c * 8, bb);
        s = a[0] * bb[0] + a[1] * bb[1] + a[2] * bb[2] + a[3] * bb[3];
        load4(dob + (int64_t)r * D + c * 8 + 4, a);
        load4(ob + (int64_t)r * D + c * 8 + 4, bb);
        s += a[0] * bb[0] + a[1] * bb[1] + a[2] * bb[2] + a[3] * bb[3];
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      if (c == 0) delta[r] = s;
    }
  }
  for (int k = t; k < NPAD; k += 512) {
    keyok[k] = (k < N) && (!p.kmask || p.kmask[(int64_t)b * N + k] != 0);
    lse2[k] = k < N ? p.lse[((int64_t)b * p.H + h) * N + k] * LOG2E : __builtin_huge_valf();
  }
  __syncthreads();

  const float c2 = p.scale * LOG2E;
  const int g = lane >> 4, li = lane & 15;
  const int nkb = NPAD >> 4, nstep = NPAD >> 5;

  // ---- phase A: dK, dV for 16 keys per wave (Q images i0, dO images i1)
  for (int kb = wave; kb < nkb; kb += 8) {
    const int key = kb * 16 + li;
    const bool kok = keyok[key];
    bf16x8 kh[2], kl[2], vh[2], vl[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      gfrag_x3(base + D, ld, key, N, kk, g, kh[kk], kl[kk]);
      gfrag_x3(base + 2 * D, ld, key, N, kk, g, vh[kk], vl[kk]);
    }
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { dv[u] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[u] = dv[u]; }
    for (int qs = 0; qs < nstep; ++qs) {
      if (CAUSAL && qs * 32 + 31 < kb * 16) continue;  // every query of this step precedes every key
      f32x4 pt[2], ds[2];
#pragma unroll
      for (int tau = 0; tau < 2; ++tau) {
        f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
        const int qr = qs * 32 + tau * 16 + li;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sc = mfma3(frag_row(i0h, qr, kk * 4 + g), frag_row(i0l, qr, kk * 4 + g), kh[kk], kl[kk], sc);
          dp = mfma3(frag_row(i1h, qr, kk * 4 + g), frag_row(i1l, qr, kk * 4 + g), vh[kk], vl[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qs * 32 + tau * 16 + 4 * g + r;
          const bool ok = kok && (!CAUSAL || key <= q);
          const float pv = ok ? exp2f(sc[r] * c2 - lse2[q]) : 0.f;
          pt[tau][r] = pv;
          ds[tau][r] = pv * (dp[r] - delta[q]);
        }
      }
      bf16x8 ph, pl, sh, sl;
      split8(pt[0], pt[1], ph, pl);
      split8(ds[0], ds[1], sh, sl);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dv[u] = mfma3(frag_tr(i1h, qs * 32, u * 16, lane), frag_tr(i1l, qs * 32, u * 16, lane), ph, pl, dv[u]);
        dk[u] = mfma3(frag_tr(i0h, qs * 32, u * 16, lane), frag_tr(i0l, qs * 32, u * 16, lane), sh, sl, dk[u]);
      }
    }
    if (key < N) {
      float* row = p.dqkv + ((int64_t)b * N + key) * ld + h * 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float a[4] = {dk[u][0] * p.scale, dk[u][1] * p.scale, dk[u][2] * p.scale, dk[u][3] * p.scale};
        float c[4] = {dv[u][0], dv[u][1], dv[u][2], dv[u][3]};
        store4(row + D + u * 16 + 4 * g, a);
        store4(row + 2 * D + u * 16 + 4 * g, c);
      }
    }
  }
  __syncthreads();
  stage_x3(i0h, i0l, base + D, ld, N, NPAD, t, 512);
  stage_x3(i1h, i1l, base + 2 * D, ld, N, NPAD, t, 512);
  __syncthreads();

  // ---- phase B: dQ for 16 queries per wave (K images i0, V images i1)
  const int nqb = (N + 15) >> 4;
  for (int qb = wave; qb < nqb; qb += 8) {
    const int q = qb * 16 + li;
    const float l2 = lse2[q], dl = delta[q];
    bf16x8 qh[2], ql[2], oh[2], ol[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      gfrag_x3(base, ld, q, N, kk, g, qh[kk], ql[kk]);
      gfrag_x3(dob, D, q, N, kk, g, oh[kk], ol[kk]);
    }
    f32x4 dq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) dq[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nstep; ++ks) {
      if (CAUSAL && ks * 32 > qb * 16 + 15) break;
      f32x4 ds[2];
#pragma unroll
      for (int tau = 0; tau < 2; ++tau) {
        f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
        const int kr = ks * 32 + tau * 16 + li;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sc = mfma3(frag_row(i0h, kr, kk * 4 + g), frag_row(i0l, kr, kk * 4 + g), qh[kk], ql[kk], sc);
          dp = mfma3(frag_row(i1h, kr, kk * 4 + g), frag_row(i1l, kr, kk * 4 + g), oh[kk], ol[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = ks * 32 + tau * 16 + 4 * g + r;
          const bool ok = keyok[key] && (!CAUSAL || key <= q);
          const float pv = ok ? exp2f(sc[r] * c2 - l2) : 0.f;
          ds[tau][r] = pv * (dp[r] - dl);
        }
      }
      bf16x8 sh, sl;
      split8(ds[0], ds[1], sh, sl);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        dq[u] = mfma3(frag_tr(i0h, ks * 32, u * 16, lane), frag_tr(i0l, ks * 32, u * 16, lane), sh, sl, dq[u]);
    }
    if (q < N) {
      float* row = p.dqkv + ((int64_t)b * N + q) * ld + h * 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float a[4] = {dq[u][0] * p.scale, dq[u][1] * p.scale, dq[u][2] * p.scale, dq[u][3] * p.scale};
        store4(row + u * 16 + 4 * g, a);
      }
    }
  }
}

template <int NKT, bool M>
void launch_fwd_x3(const AttnX& p, int causal, hipStream_t s) {
  constexpr size_t lds = 4 * (size_t)NKT * 16 * 128 + (size_t)NKT * 16 * sizeof(int);
  static_assert(lds <= 160 * 1024, "attn_fwd_x3: LDS");
  (void)lds_optin((const void*)attn_fwd_x3<NKT, M>, (int)lds);
  hipLaunchKernelGGL((attn_fwd_x3<NKT, M>), dim3(p.B * p.H), dim3(512), lds, s, p, causal);
}

template <bool M>
int fwd_x3_dispatch(const AttnX& p, int causal, hipStream_t s) {
  switch (((p.N + 31) & ~31) / 16) {
    case 2: launch_fwd_x3<2, M>(p, causal, s); return CLIPMI_OK;
    case 4: launch_fwd_x3<4, M>(p, causal, s); return CLIPMI_OK;
    case 6: launch_fwd_x3<6, M>(p, causal, s); return CLIPMI_OK;
    case 8: launch_fwd_x3<8, M>(p, causal, s); return CLIPMI_OK;
    case 10: launch_fwd_x3<10, M>(p, causal, s); return CLIPMI_OK;
    case 12: launch_fwd_x3<12, M>(p, causal, s); return CLIPMI_OK;
    case 14: launch_fwd_x3<14, M>(p, causal, s); return CLIPMI_OK;
    case 16: launch_fwd_x3<16, M>(p, causal, s); return CLIPMI_OK;
    case 18: launch_fwd_x3<18, M>(p, causal, s); return CLIPMI_OK;
    default: return clipmi_invalid("attention_x3: N must be <= 288");
  }
}

size_t bwd_x3_lds(int N) {
  const size_t npad = (size_t)((N + 31) & ~31);
  return 4 * npad * 128 + 3 * npad * 4;
}

}  // namespace

extern "C" int clipmi_attention_fwd(void*, int, const void*, void*, float*, const int64_t*, int, int, int, int, int);
extern "C" int clipmi_attention_bwd(void*, int, const void*, const void*, const float*, const void*, void*,
                                    const int64_t*, int, int, int, int, int);

// fp32 q/k/v [B*N, 3D] -> fp32 O [B*N, D] + lse, products as bf16x3 split MFMAs (N > 288: the exact-f32
// kernels of clipmi_attention_fwd).  Same arguments and outputs as clipmi_attention_fwd with dtype fp32.
extern "C" int clipmi_attention_fwd_x3(void* stream, const void* qkv, void* o, float* lse,
                                       const int64_t* attention_mask, int causal, int B, int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1, "N >= 1");
  CLIPMI_REQUIRE(qkv && o && lse, "operands");
  if (N > X3_MAX_N) return clipmi_attention_fwd(stream, CLIPMI_F32, qkv, o, lse, attention_mask, causal, B, H, N, D);
  if (B == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)o & 15) == 0, "qkv / o must be 16-byte aligned");
  AttnX p{(const float*)qkv, (float*)o, lse, attention_mask, nullptr, nullptr, B, H, N, D, 0.125f};
  const int npad = (N + 31) & ~31;
  const double flops = 3 * 4.0 * B * H * (double)N * npad * 64;  // the MFMA work issued: three products each
  ProfScope ps(s, "attn_fwd_x3", flops);
  CLIPMI_TRY((causal || attention_mask) ? fwd_x3_dispatch<true>(p, causal, s) : fwd_x3_dispatch<false>(p, causal, s));
  ps.finish("attn_fwd_x3", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// the backward of clipmi_attention_fwd_x3 (fp32 dO in, fp32 dq / dk / dv out into dqkv [B*N, 3D])
extern "C" int clipmi_attention_bwd_x3(void* stream, const void* qkv, const void* o, const float* lse,
                                       const void* dout, void* dqkv, const int64_t* attention_mask, int causal, int B,
                                       int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1, "N >= 1");
  CLIPMI_REQUIRE(qkv && o && lse && dout && dqkv, "operands");
  if (N > X3_MAX_N)
    return clipmi_attention_bwd(stream, CLIPMI_F32, qkv, o, lse, dout, dqkv, attention_mask, causal, B, H, N, D);
  if (B == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0 &&
                     ((uintptr_t)dqkv & 15) == 0,
                 "qkv / o / dout / dqkv must be 16-byte aligned");
  AttnX p{(const float*)qkv, (float*)o, (float*)lse, attention_mask, (const float*)dout, (float*)dqkv, B, H, N, D,
          0.125f};
  const size_t lds = bwd_x3_lds(N);
  const int npad = (N + 31) & ~31;
  const double flops = 3 * 10.0 * B * H * (double)N * npad * 64;
  ProfScope ps(s, "attn_bwd_x3", flops);
  if (causal) {
    (void)lds_optin((const void*)attn_bwd_x3<true>, (int)lds);
    hipLaunchKernelGGL(attn_bwd_x3<true>, dim3(B * H), dim3(512), lds, s, p);
  } else {
    (void)lds_optin((const void*)attn_bwd_x3<false>, (int)lds);
    hipLaunchKernelGGL(attn_bwd_x3<false>, dim3(B * H), dim3(512), lds, s, p);
  }
  ps.finish("attn_bwd_x3", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
