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
  // image output of the backward (clipmi_attention_bwd_x3img): d_qkv as its pattern-1 split image [B*N][9D] and the
  // per-batch-row column sums of d_qkv colp[B][3D] (the qkv bias gradient's partials)
  bf16* dimg; float* colp;
  // forward (clipmi_attention_fwd_x3img): O's pattern-0 image [B*N][3D] beside the fp32 O, or null
  bf16* oimg;
};

// four fp32 values of an output row -> the pattern-1 image segments (h, l, h) at row + c, + seg, + 2 seg, with the
// rounding of clipmi_split3_colsum (no contraction of v - h into a producing multiply)
__device__ __forceinline__ void st_x3_4(bf16* row, int64_t seg, int c, const float v[4], bool p1 = true) {
#pragma clang fp contract(off)
  bf16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = (bf16)v[j];
    l[j] = (bf16)(v[j] - (float)h[j]);
  }
  *(bf16x4*)(row + c) = h;
  *(bf16x4*)(row + seg + c) = p1 ? l : h;
  *(bf16x4*)(row + 2 * seg + c) = p1 ? h : l;
}

// sum of v over the 16 row lanes (li) of each lane group g, added by lane li == 0 into red[c .. c + 3]
__device__ __forceinline__ void colsum16_add(float* red, int c, float v[4], int li) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v[r] += __shfl_xor(v[r], o, 64);
  if (li == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) red[c + r] += v[r];
  }
}

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
// NB query blocks per wave at a time (NB = 2: every K / V fragment read from LDS serves both blocks' products,
// halving the fragment reads that bound the one-block form -- 2 x NKT x 2 reads of 1 KiB per 16 queries)
template <int NKT, bool MASKED, int NB>
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
  for (int qb0 = wave * NB; qb0 < nqb; qb0 += 8 * NB) {
    int q[NB];
    bf16x8 qh[NB][2], ql[NB][2];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      q[j] = (qb0 + j) * 16 + li;  // a block past nqb computes on zero rows and stores nothing
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) gfrag_x3(base, ld, q[j], N, kk, g, qh[j][kk], ql[j][kk]);
    }
    // key-major scores: lane (g, li) holds keys kt * 16 + 4 g + r of query li
    f32x4 sc[NB][NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int j = 0; j < NB; ++j) sc[j][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 fh = frag_row(Kh, kt * 16 + li, kk * 4 + g), fl = frag_row(Kl, kt * 16 + li, kk * 4 + g);
#pragma unroll
        for (int j = 0; j < NB; ++j) sc[j][kt] = mfma3(fh, fl, qh[j][kk], ql[j][kk], sc[j][kt]);
      }
      // one tile's fragment reads in flight at a time: hoisting every tile's K fragments (16 VGPRs each) above
      // the MFMAs spilled from NKT = 10 on
      __builtin_amdgcn_sched_barrier(0);
    }
    float mref[NB], lsum[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      float mx = NEG_INF;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + 4 * g + r;
          if (MASKED) {
            if (!(keyok[key] && (!causal || key <= q[j]))) sc[j][kt][r] = NEG_INF;
          } else if (kt >= NKT - 2 && key >= N) {  // NPAD = N rounded up to 32: padding in the last two tiles only
            sc[j][kt][r] = NEG_INF;
          }
          mx = fmaxf(mx, sc[j][kt][r]);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      mref[j] = mx == NEG_INF ? 0.f : mx * c2;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(sc[j][kt][r], c2, -mref[j]));
          sc[j][kt][r] = e;
          ls += e;
        }
      ls += __shfl_xor(ls, 16, 64);
      ls += __shfl_xor(ls, 32, 64);
      lsum[j] = ls;
    }
    // O^T = V^T P^T, the P tiles split per 32-key step straight from the score registers
    f32x4 acc[NB][4];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[j][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKT / 2; ++ks) {
      bf16x8 ph[NB], pl[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) split8(sc[j][2 * ks], sc[j][2 * ks + 1], ph[j], pl[j]);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const bf16x8 fh = frag_tr(Vh, ks * 32, v * 16, lane), fl = frag_tr(Vl, ks * 32, v * 16, lane);
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[j][v] = mfma3(fh, fl, ph[j], pl[j], acc[j][v]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (q[j] < N) {
        const float inv = lsum[j] > 0.f ? 1.f / lsum[j] : 0.f;
        float* orow = p.o + ((int64_t)b * N + q[j]) * D + h * 64;
        bf16* irow = p.oimg ? p.oimg + ((int64_t)b * N + q[j]) * 3 * D + h * 64 : nullptr;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float w[4] = {acc[j][v][0] * inv, acc[j][v][1] * inv, acc[j][v][2] * inv, acc[j][v][3] * inv};
          store4(orow + v * 16 + 4 * g, w);
          if (irow) st_x3_4(irow, D, v * 16 + 4 * g, w, false);
        }
        if (g == 0)
          p.lse[((int64_t)b * p.H + h) * N + q[j]] = lsum[j] > 0.f ? (mref[j] + __log2f(lsum[j])) * LN2 : NEG_INF;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ backward
// NBA / NBB: key blocks per wave in phase A, query blocks per wave in phase B (2: every fragment read from the
// images serves two blocks' products; 1: the one-block form, A/B)
template <bool CAUSAL, int NBA, int NBB, bool XIMG = false>
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
  float* red = (float*)(keyok + NPAD);  // XIMG: per-wave column sums [8 waves][q, k, v][64]
  const float* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const float* dob = p.dout + (int64_t)b * N * D + h * 64;
  if (XIMG)
    for (int i = t; i < 8 * 192; i += 512) red[i] = 0.f;
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

  // ---- phase A: dK, dV for NB blocks of 16 keys per wave at a time (Q images i0, dO images i1): every Q / dO
  // fragment read serves the NB blocks' products
  for (int kb0 = wave * NBA; kb0 < nkb; kb0 += 8 * NBA) {
    int key[NBA];
    bool kok[NBA];
    bf16x8 kh[NBA][2], kl[NBA][2], vh[NBA][2], vl[NBA][2];
#pragma unroll
    for (int j = 0; j < NBA; ++j) {
      key[j] = (kb0 + j) * 16 + li;  // a block past nkb (NPAD >= its rows) computes P = 0 and stores nothing
      kok[j] = key[j] < NPAD && keyok[key[j]];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        gfrag_x3(base + D, ld, key[j], N, kk, g, kh[j][kk], kl[j][kk]);
        gfrag_x3(base + 2 * D, ld, key[j], N, kk, g, vh[j][kk], vl[j][kk]);
      }
    }
    f32x4 dv[NBA][4], dk[NBA][4];
#pragma unroll
    for (int j = 0; j < NBA; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) { dv[j][u] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[j][u] = dv[j][u]; }
    for (int qs = 0; qs < nstep; ++qs) {
      if (CAUSAL && qs * 32 + 31 < kb0 * 16) continue;  // every query of this step precedes every key
      f32x4 pt[NBA][2], ds[NBA][2];
#pragma unroll
      for (int tau = 0; tau < 2; ++tau) {
        f32x4 sc[NBA], dp[NBA];
#pragma unroll
        for (int j = 0; j < NBA; ++j) { sc[j] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[j] = sc[j]; }
        const int qr = qs * 32 + tau * 16 + li;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 qfh = frag_row(i0h, qr, kk * 4 + g), qfl = frag_row(i0l, qr, kk * 4 + g);
          const bf16x8 ofh = frag_row(i1h, qr, kk * 4 + g), ofl = frag_row(i1l, qr, kk * 4 + g);
#pragma unroll
          for (int j = 0; j < NBA; ++j) {
            sc[j] = mfma3(qfh, qfl, kh[j][kk], kl[j][kk], sc[j]);
            dp[j] = mfma3(ofh, ofl, vh[j][kk], vl[j][kk], dp[j]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qs * 32 + tau * 16 + 4 * g + r;
          const float l2 = lse2[q], dl = delta[q];
#pragma unroll
          for (int j = 0; j < NBA; ++j) {
            const bool ok = kok[j] && (!CAUSAL || key[j] <= q);
            const float pv = ok ? exp2f(sc[j][r] * c2 - l2) : 0.f;
            pt[j][tau][r] = pv;
            ds[j][tau][r] = pv * (dp[j][r] - dl);
          }
        }
      }
      bf16x8 ph[NBA], pl[NBA], sh[NBA], sl[NBA];
#pragma unroll
      for (int j = 0; j < NBA; ++j) {
        split8(pt[j][0], pt[j][1], ph[j], pl[j]);
        split8(ds[j][0], ds[j][1], sh[j], sl[j]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bf16x8 ofh = frag_tr(i1h, qs * 32, u * 16, lane), ofl = frag_tr(i1l, qs * 32, u * 16, lane);
        const bf16x8 qfh = frag_tr(i0h, qs * 32, u * 16, lane), qfl = frag_tr(i0l, qs * 32, u * 16, lane);
#pragma unroll
        for (int j = 0; j < NBA; ++j) {
          dv[j][u] = mfma3(ofh, ofl, ph[j], pl[j], dv[j][u]);
          dk[j][u] = mfma3(qfh, qfl, sh[j], sl[j], dk[j][u]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NBA; ++j) {
      if (XIMG) {  // rows past N hold exact zeros (P = dS = 0 there): summed as they are
        bf16* row = p.dimg + ((int64_t)b * N + key[j]) * 3 * ld + h * 64;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float a[4] = {dk[j][u][0] * p.scale, dk[j][u][1] * p.scale, dk[j][u][2] * p.scale, dk[j][u][3] * p.scale};
          float c[4] = {dv[j][u][0], dv[j][u][1], dv[j][u][2], dv[j][u][3]};
          if (key[j] < N) {
            st_x3_4(row, ld, D + u * 16 + 4 * g, a);
            st_x3_4(row, ld, 2 * D + u * 16 + 4 * g, c);
          }
          colsum16_add(red + wave * 192 + 64, u * 16 + 4 * g, a, li);
          colsum16_add(red + wave * 192 + 128, u * 16 + 4 * g, c, li);
        }
      } else if (key[j] < N) {
        float* row = p.dqkv + ((int64_t)b * N + key[j]) * ld + h * 64;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float a[4] = {dk[j][u][0] * p.scale, dk[j][u][1] * p.scale, dk[j][u][2] * p.scale, dk[j][u][3] * p.scale};
          float c[4] = {dv[j][u][0], dv[j][u][1], dv[j][u][2], dv[j][u][3]};
          store4(row + D + u * 16 + 4 * g, a);
          store4(row + 2 * D + u * 16 + 4 * g, c);
        }
      }
    }
  }
  __syncthreads();
  stage_x3(i0h, i0l, base + D, ld, N, NPAD, t, 512);
  stage_x3(i1h, i1l, base + 2 * D, ld, N, NPAD, t, 512);
  __syncthreads();

  // ---- phase B: dQ for NB blocks of 16 queries per wave at a time (K images i0, V images i1)
  const int nqb = (N + 15) >> 4;
  for (int qb0 = wave * NBB; qb0 < nqb; qb0 += 8 * NBB) {
    int q[NBB];
    float l2[NBB], dl[NBB];
    bf16x8 qh[NBB][2], ql[NBB][2], oh[NBB][2], ol[NBB][2];
#pragma unroll
    for (int j = 0; j < NBB; ++j) {
      q[j] = (qb0 + j) * 16 + li;  // a block past nqb computes on zero rows and stores nothing
      l2[j] = q[j] < NPAD ? lse2[q[j]] : __builtin_huge_valf();
      dl[j] = q[j] < NPAD ? delta[q[j]] : 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        gfrag_x3(base, ld, q[j], N, kk, g, qh[j][kk], ql[j][kk]);
        gfrag_x3(dob, D, q[j], N, kk, g, oh[j][kk], ol[j][kk]);
      }
    }
    f32x4 dq[NBB][4];
#pragma unroll
    for (int j = 0; j < NBB; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) dq[j][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nstep; ++ks) {
      if (CAUSAL && ks * 32 > (qb0 + NBB - 1) * 16 + 15) break;
      f32x4 ds[NBB][2];
#pragma unroll
      for (int tau = 0; tau < 2; ++tau) {
        f32x4 sc[NBB], dp[NBB];
#pragma unroll
        for (int j = 0; j < NBB; ++j) { sc[j] = f32x4{0.f, 0.f, 0.f, 0.f}; dp[j] = sc[j]; }
        const int kr = ks * 32 + tau * 16 + li;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 kfh = frag_row(i0h, kr, kk * 4 + g), kfl = frag_row(i0l, kr, kk * 4 + g);
          const bf16x8 vfh = frag_row(i1h, kr, kk * 4 + g), vfl = frag_row(i1l, kr, kk * 4 + g);
#pragma unroll
          for (int j = 0; j < NBB; ++j) {
            sc[j] = mfma3(kfh, kfl, qh[j][kk], ql[j][kk], sc[j]);
            dp[j] = mfma3(vfh, vfl, oh[j][kk], ol[j][kk], dp[j]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = ks * 32 + tau * 16 + 4 * g + r;
          const bool kok = keyok[key];
#pragma unroll
          for (int j = 0; j < NBB; ++j) {
            const bool ok = kok && (!CAUSAL || key <= q[j]);
            const float pv = ok ? exp2f(sc[j][r] * c2 - l2[j]) : 0.f;
            ds[j][tau][r] = pv * (dp[j][r] - dl[j]);
          }
        }
      }
      bf16x8 sh[NBB], sl[NBB];
#pragma unroll
      for (int j = 0; j < NBB; ++j) split8(ds[j][0], ds[j][1], sh[j], sl[j]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bf16x8 kfh = frag_tr(i0h, ks * 32, u * 16, lane), kfl = frag_tr(i0l, ks * 32, u * 16, lane);
#pragma unroll
        for (int j = 0; j < NBB; ++j) dq[j][u] = mfma3(kfh, kfl, sh[j], sl[j], dq[j][u]);
      }
    }
#pragma unroll
    for (int j = 0; j < NBB; ++j) {
      if (XIMG) {  // rows past N: zero query rows give dS = 0 (dO = 0 there), dq = 0
        bf16* row = p.dimg + ((int64_t)b * N + q[j]) * 3 * ld + h * 64;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float a[4] = {dq[j][u][0] * p.scale, dq[j][u][1] * p.scale, dq[j][u][2] * p.scale, dq[j][u][3] * p.scale};
          if (q[j] < N) st_x3_4(row, ld, u * 16 + 4 * g, a);
          if (q[j] >= N) a[0] = a[1] = a[2] = a[3] = 0.f;
          colsum16_add(red + wave * 192, u * 16 + 4 * g, a, li);
        }
      } else if (q[j] < N) {
        float* row = p.dqkv + ((int64_t)b * N + q[j]) * ld + h * 64;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float a[4] = {dq[j][u][0] * p.scale, dq[j][u][1] * p.scale, dq[j][u][2] * p.scale, dq[j][u][3] * p.scale};
          store4(row + u * 16 + 4 * g, a);
        }
      }
    }
  }
  if (XIMG) {  // the workgroup's column sums in wave order -> colp[b][q | k | v columns of head h]
    __syncthreads();
    if (t < 192) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum += red[w * 192 + t];
      p.colp[(int64_t)b * 3 * D + (t >> 6) * D + h * 64 + (t & 63)] = sum;
    }
  }
}

// blocks per wave (tools/attn_x3_bench.py, profiles/r06_attn_x3_blocks_ab.log): the unmasked forward takes two
// (ViT-B/16 890 -> 845 us), the masked forward and the backward one (text forward 140 vs 173 us; backward equal
// within 1 %, two key blocks spill); CLIPMI_ATTN_X3_NB=1 / 2 forces either (A/B, read per call)
int x3_nb(bool fwd_unmasked) {
  const char* e = getenv("CLIPMI_ATTN_X3_NB");
  if (e && (atoi(e) == 1 || atoi(e) == 2)) return atoi(e);
  return fwd_unmasked ? 2 : 1;
}

template <int NKT, bool M>
void launch_fwd_x3(const AttnX& p, int causal, hipStream_t s) {
  constexpr size_t lds = 4 * (size_t)NKT * 16 * 128 + (size_t)NKT * 16 * sizeof(int);
  static_assert(lds <= 160 * 1024, "attn_fwd_x3: LDS");
  // two blocks per wave spill (25-65 VGPRs) only in the masked forms from NKT = 14 on, which keep one
  constexpr bool TWO = !(M && NKT >= 14);
  if constexpr (TWO) {
    if (x3_nb(!M) == 2) {
      (void)lds_optin((const void*)attn_fwd_x3<NKT, M, 2>, (int)lds);
      hipLaunchKernelGGL((attn_fwd_x3<NKT, M, 2>), dim3(p.B * p.H), dim3(512), lds, s, p, causal);
      return;
    }
  }
  (void)lds_optin((const void*)attn_fwd_x3<NKT, M, 1>, (int)lds);
  hipLaunchKernelGGL((attn_fwd_x3<NKT, M, 1>), dim3(p.B * p.H), dim3(512), lds, s, p, causal);
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

// phase A's key blocks per wave with CLIPMI_ATTN_X3_NB=2: CLIPMI_ATTN_X3_NBA (default 1: two blocks spill 6-14
// VGPRs there)
int x3_nba() {
  const char* e = getenv("CLIPMI_ATTN_X3_NBA");
  return (e && atoi(e) == 2) ? 2 : 1;
}
template <bool C, int NBA, int NBB, bool IMG = false>
void launch_bwd_x3(const AttnX& p, size_t lds, hipStream_t s) {
  (void)lds_optin((const void*)attn_bwd_x3<C, NBA, NBB, IMG>, (int)lds);
  hipLaunchKernelGGL((attn_bwd_x3<C, NBA, NBB, IMG>), dim3(p.B * p.H), dim3(512), lds, s, p);
}

size_t bwd_x3_lds(int N) {
  const size_t npad = (size_t)((N + 31) & ~31);
  return 4 * npad * 128 + 3 * npad * 4 + 8 * 192 * 4;  // images, lse2 / delta / keyok, the image form's column sums
}

}  // namespace

extern "C" int clipmi_attention_fwd(void*, int, const void*, void*, float*, const int64_t*, int, int, int, int, int);
extern "C" int clipmi_attention_bwd(void*, int, const void*, const void*, const float*, const void*, void*,
                                    const int64_t*, int, int, int, int, int);

// fp32 q/k/v [B*N, 3D] -> fp32 O [B*N, D] + lse, products as bf16x3 split MFMAs (N > 288: the exact-f32
// kernels of clipmi_attention_fwd).  Same arguments and outputs as clipmi_attention_fwd with dtype fp32.
namespace {
int attention_fwd_x3(void* stream, const void* qkv, void* o, void* oimg, float* lse, const int64_t* attention_mask,
                     int causal, int B, int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1, "N >= 1");
  CLIPMI_REQUIRE(qkv && o && lse, "operands");
  if (N > X3_MAX_N) return clipmi_attention_fwd(stream, CLIPMI_F32, qkv, o, lse, attention_mask, causal, B, H, N, D);
  if (B == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)o & 15) == 0, "qkv / o must be 16-byte aligned");
  AttnX p{(const float*)qkv, (float*)o, lse, attention_mask, nullptr, nullptr, B, H, N, D, 0.125f, nullptr, nullptr,
          (bf16*)oimg};
  const int npad = (N + 31) & ~31;
  const double flops = 3 * 4.0 * B * H * (double)N * npad * 64;  // the MFMA work issued: three products each
  ProfScope ps(s, "attn_fwd_x3", flops);
  CLIPMI_TRY((causal || attention_mask) ? fwd_x3_dispatch<true>(p, causal, s) : fwd_x3_dispatch<false>(p, causal, s));
  ps.finish("attn_fwd_x3", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
}  // namespace

extern "C" int clipmi_attention_fwd_x3(void* stream, const void* qkv, void* o, float* lse,
                                       const int64_t* attention_mask, int causal, int B, int H, int N, int D) {
  return attention_fwd_x3(stream, qkv, o, nullptr, lse, attention_mask, causal, B, H, N, D);
}
// the same with O's pattern-0 split image written beside the fp32 O (oimg bf16 [B*N][3D], 8-byte aligned): the
// out-projection's operand without a split pass.  N <= 288.
extern "C" int clipmi_attention_fwd_x3img(void* stream, const void* qkv, void* o, void* oimg, float* lse,
                                          const int64_t* attention_mask, int causal, int B, int H, int N, int D) {
  CLIPMI_REQUIRE(N >= 1 && N <= X3_MAX_N, "attention_fwd_x3img: 1 <= N <= 288");
  CLIPMI_REQUIRE(oimg && ((uintptr_t)oimg & 7) == 0, "attention_fwd_x3img: oimg 8-byte aligned");
  return attention_fwd_x3(stream, qkv, o, oimg, lse, attention_mask, causal, B, H, N, D);
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
          0.125f, nullptr, nullptr, nullptr};
  const size_t lds = bwd_x3_lds(N);
  const int npad = (N + 31) & ~31;
  const double flops = 3 * 10.0 * B * H * (double)N * npad * 64;
  ProfScope ps(s, "attn_bwd_x3", flops);
  const int nb = x3_nb(false), nba = x3_nba();
  if (nb == 1) {
    if (causal) launch_bwd_x3<true, 1, 1>(p, lds, s);
    else launch_bwd_x3<false, 1, 1>(p, lds, s);
  } else if (nba == 2) {
    if (causal) launch_bwd_x3<true, 2, 2>(p, lds, s);
    else launch_bwd_x3<false, 2, 2>(p, lds, s);
  } else {
    if (causal) launch_bwd_x3<true, 1, 2>(p, lds, s);
    else launch_bwd_x3<false, 1, 2>(p, lds, s);
  }
  ps.finish("attn_bwd_x3", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// The same backward with d_qkv written as its pattern-1 split image dimg bf16 [B*N][9D] (segments h, l, h at columns
// c, 3D + c, 6D + c: clipmi_split3_colsum's layout and rounding) and its column sums -- the q / k / v bias gradient --
// added onto colsum[3D] (+= when beta): the bf16x3 engine's input to the qkv weight and input gradients, without an
// fp32 d_qkv and a split pass over it.  N <= 288; ws >= clipmi_attention_bwd_x3img_ws(B, D) bytes, 256-B aligned.
extern "C" int64_t clipmi_attention_bwd_x3img_ws(int B, int D) {
  return B > 0 && D > 0 ? colsum_partials_ws(B, 3 * D) : 0;
}
extern "C" int clipmi_attention_bwd_x3img(void* stream, const void* qkv, const void* o, const float* lse,
                                          const void* dout, void* dimg, float* colsum, int beta, void* ws,
                                          int64_t ws_bytes, const int64_t* attention_mask, int causal, int B, int H,
                                          int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1 && N <= X3_MAX_N, "attention_bwd_x3img: 1 <= N <= 288");
  CLIPMI_REQUIRE(qkv && o && lse && dout && dimg && colsum, "operands");
  CLIPMI_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0 &&
                     ((uintptr_t)dimg & 7) == 0,
                 "qkv / o / dout 16-byte, dimg 8-byte aligned");
  CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_attention_bwd_x3img_ws(B, D) && ((uintptr_t)ws & 255) == 0,
                 "attention_bwd_x3img: workspace (clipmi_attention_bwd_x3img_ws, 256-byte aligned)");
  if (B == 0) return CLIPMI_OK;
  float* colp = (float*)ws;
  AttnX p{(const float*)qkv, (float*)o, (float*)lse, attention_mask, (const float*)dout, nullptr, B, H, N, D, 0.125f,
          (bf16*)dimg, colp, nullptr};
  const size_t lds = bwd_x3_lds(N);
  const int npad = (N + 31) & ~31;
  const double flops = 3 * 10.0 * B * H * (double)N * npad * 64;
  ProfScope ps(s, "attn_bwd_x3", flops);
  if (causal) launch_bwd_x3<true, 1, 1, true>(p, lds, s);
  else launch_bwd_x3<false, 1, 1, true>(p, lds, s);
  ps.finish("attn_bwd_x3", flops);
  CLIPMI_CHECK_LAUNCH();
  float* fold = (float*)((char*)ws + ((int64_t)B * 3 * D * 4 + 255) / 256 * 256);
  CLIPMI_TRY(colsum_partials_finish(s, colp, B, 3 * D, colsum, beta, fold));
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
