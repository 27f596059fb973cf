// Fused multi-head attention (head_dim 64) forward/backward for both CLIP towers.
//
// Replaces CLIPAttention's core + eager_attention_forward ([HF] modeling_clip.py:259-335):
// softmax(q k^T * 64^-0.5 + mask) v with the text tower's causal + key-padding mask
// ([HF] :543-548) and no mask for the vision tower.  q/k/v are read straight out of the
// fused QKV GEMM output [B*N, 3D] (head h at columns h*64, D+h*64, 2D+h*64); the output O
// is written [B*N, D] so the out-projection GEMM consumes it directly.  The forward saves
// the per-row log-sum-exp so the backward recomputes P without storing N x N scores.
//
// bf16 path (N <= 288, ATTN_MAX_N: two double-buffered K/V images of 288 rows fill the 160 KiB
// LDS; covers ViT-B and ViT-L/14 at 224 px, N = 257): persistent workgroups walk (batch, head) items; the next item's
// operands are LDS-DMA'd while the current one is computed (attn_fwd_pf, attn_bwd_pf).
// K/V (and Q/dO/O in the backward) live in LDS as [Npad][64] bf16 images with 16-B chunk
// c of row r stored at c ^ (r & 6); that single swizzle is conflict-free for the
// ds_read_b128 fragment reads, the ds_read_b64_tr_b16 transposed reads and the lane-linear
// DMA writes (the swizzle is applied to the DMA source address).
// Scores are computed "key-major" so each lane owns whole query rows: the row max/sum
// need two xor-shuffles and the P tile feeds the next MFMA straight from registers
// (cdna_hip_programming.md §3, accumulator as operand, with the k-permutation matched
// on the V side by the transposed read).  Backward: phase A (dK, dV) has each wave own
// 16 keys and sweep all queries; phase B (dQ) has each wave own 16 queries and sweep
// all keys; no atomics, no N x N buffer.
// f32 path: exact-f32 SIMT kernels (4 lanes per row) for the fp32 parity mode.
#include "common.h"
#include "internal.h"
#include "attn_frag.h"
#include <algorithm>
#include <cstdlib>

#ifdef CLIPMI_ATTN_STAMPS
namespace cmg { unsigned long long* gemm_stamp_buffer(); }
#endif

namespace {

constexpr int ATTN_MAX_N = 288;      // whole-K/V-in-LDS kernels (bf16)
constexpr int ATTN_MAX_N_ANY = 4096;  // K/V-streaming kernels (bf16 flash forward, chunked f32 / bwd)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float NEG_INF = -__builtin_huge_valf();

// stage rows [0, Npad) of a [N][64] head slice (row stride ld elements) into an image
__device__ __forceinline__ void stage_img(char* img, const bf16* src, int64_t ld, int N, int Npad, int t, int nthr) {
  for (int id = t; id < Npad * 8; id += nthr) {
    const int r = id >> 3, c = id & 7;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (r < N) v = *(const u32x4*)(src + (int64_t)r * ld + c * 8);
    *LDS_PTR(u32x4, img + img_off(r, c)) = v;
  }
}

struct AttnP {
  const bf16* qkv; bf16* o; float* lse; const int64_t* kmask;
  const bf16* dout; bf16* dqkv;
  int B, H, N, D;
  float scale;
  unsigned long long* dbg = nullptr;  // diagnostic builds only (CLIPMI_ATTN_STAMPS): s_memtime stamps
  uint8_t *o8 = nullptr, *s8 = nullptr;  // MXFP8 output (attn_fwd_fa<.., Q8>): e4m3 [B*N, D], E8M0 [B*N, D/32]
};

// Diagnostic build (-DCLIPMI_ATTN_STAMPS, tools/attn_stamps.py): the prefetching backward stamps
// s_memtime per (workgroup < 256, wave, item < 16) at the phase boundaries of its item loop into the
// buffer armed by clipmi_gemm_stamps: [((blk * 16 + wave) * 16 + item) * 8 + phase].
#ifdef CLIPMI_ATTN_STAMPS
#define ATT_ST(ph)                                                                                   \
  do {                                                                                               \
    if (p.dbg && blockIdx.x < 256 && it < 16 && lane == 0)                                           \
      p.dbg[((blockIdx.x * 16 + wave) * 16 + it) * 8 + (ph)] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define ATT_ST(ph) do { } while (0)
#endif

// ------------------------------------------------------------------- fwd, prefetching
// Persistent forward.  (A first version ran one (batch, head) per workgroup with K/V
// staged through VGPRs and nothing in flight while it computed: HBM-latency bound at 2.2 TB/s.)  A workgroup of 8 waves walks (batch, head) items gridDim.x apart; the K and V
// images of item i + 1 are LDS-DMA'd into the other half of a 2-slot ring, and each wave's
// Q fragments for item i + 1 are loaded, while item i is computed.  DMAs are issued before
// the Q loads so a wave's counted wait for its Q never waits on the ring.  Per wave: q-blocks
// wave and wave + 8 of every item.
template <int NKT, bool MASKED, int NW = 8>
__global__ __launch_bounds__(NW * 64, 1) void attn_fwd_pf(AttnP p, int causal, int nitems) {
  constexpr int NPAD = NKT * 16, IMG = NPAD * 128, QPW = (NKT + NW - 1) / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* keyok_base = (int*)(smem + 4 * IMG);  // [2][NPAD]
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int N = p.N, D = p.D, H = p.H;
  const int64_t ld = 3 * (int64_t)D;
  const int nqb = (N + 15) >> 4;
  const float c2 = p.scale * LOG2E;
  const int g = lane >> 4, li = lane & 15;
  const uint32_t rec = (uint32_t)((int64_t)(N - 1) * ld * 2 + 128);

  auto issue = [&](int item, int slot) {  // K, V images of item into slot (rows >= N read 0)
    const int b = item / H, h = item - b * H;
    const bf16* base = p.qkv + (int64_t)b * N * ld + h * 64;
    const SRsrc rk = make_srsrc(base + D, rec), rv = make_srsrc(base + 2 * D, rec);
    char* kimg = smem + slot * 2 * IMG;
#pragma unroll 1
    for (int j = wave; j < NPAD / 8; j += NW) {
      const int r = 8 * j + (lane >> 3);
      const int voff = r * (int)ld * 2 + (((lane & 7) ^ (r & 6)) << 4);
      dma16(rk, kimg + j * 1024, voff);
      dma16(rv, kimg + IMG + j * 1024, voff);
    }
    if (MASKED) {
      int* ko = keyok_base + slot * NPAD;
      for (int k = t; k < NPAD; k += NW * 64) ko[k] = (k < N) && (!p.kmask || p.kmask[(int64_t)b * N + k] != 0);
    }
  };
  auto load_q = [&](int item, bf16x8 (&qf)[QPW][2]) {
    const int b = item / H, h = item - b * H;
    const bf16* base = p.qkv + (int64_t)b * N * ld + h * 64;
#pragma unroll
    for (int u = 0; u < QPW; ++u) {
      const int qc = min((wave + NW * u) * 16 + li, N - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) qf[u][kk] = *(const bf16x8*)(base + (int64_t)qc * ld + kk * 32 + 8 * g);
    }
  };

  int item = blockIdx.x;
  bf16x8 qn[QPW][2];
  issue(item, 0);
  load_q(item, qn);
  for (int it = 0;; ++it) {
    const int slot = it & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // slot ready for everyone; the other slot's last readers are done
    const int cur = item, nxt = item + gridDim.x;
    bf16x8 qf[QPW][2];
#pragma unroll
    for (int u = 0; u < QPW; ++u) { qf[u][0] = qn[u][0]; qf[u][1] = qn[u][1]; }
    if (nxt < nitems) {
      issue(nxt, slot ^ 1);
      load_q(nxt, qn);
    }
    const char* Kimg = smem + slot * 2 * IMG;
    const char* Vimg = Kimg + IMG;
    const int* keyok = keyok_base + slot * NPAD;
    const int b = cur / H, h = cur - b * H;
    {
      // each of the wave's q-blocks (wave, wave + 8) computes its scores and softmax in turn and
      // keeps P packed as bf16; the P.V products then run together, sharing every V read
      int q[QPW];
      float mref[QPW], l[QPW];
      bf16x8 pf[QPW][NKT / 2];
#pragma unroll
      for (int u = 0; u < QPW; ++u) {
        q[u] = (wave + NW * u) * 16 + li;
        f32x4 sc[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
          sc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            sc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Kimg, kt * 16 + li, kk * 4 + g), qf[u][kk], sc[kt], 0, 0, 0);
        }
        float mx = NEG_INF;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) {
          if (MASKED) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + 4 * g + r;
              if (!(keyok[key] && (!causal || key <= q[u]))) sc[kt][r] = NEG_INF;
            }
          } else if (kt >= NKT - 2) {  // NPAD = N rounded up to 32: only the last two tiles hold padding
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (kt * 16 + 4 * g + r >= N) sc[kt][r] = NEG_INF;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, sc[kt][r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        mref[u] = mx == NEG_INF ? 0.f : mx * c2;
        float lsum = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(sc[kt][r], c2, -mref[u]));
            sc[kt][r] = e;
            lsum += e;
          }
        lsum += __shfl_xor(lsum, 16, 64);
        lsum += __shfl_xor(lsum, 32, 64);
        l[u] = lsum;
#pragma unroll
        for (int ks = 0; ks < NKT / 2; ++ks) pf[u][ks] = pack8(sc[2 * ks], sc[2 * ks + 1]);
        __builtin_amdgcn_sched_barrier(0);  // keep the blocks' score tiles from being live at once
      }
      f32x4 acc[QPW][4];
#pragma unroll
      for (int u = 0; u < QPW; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKT / 2; ++ks) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const bf16x8 tv = frag_tr(Vimg, ks * 32, v * 16, lane);
#pragma unroll
          for (int u = 0; u < QPW; ++u)
            acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tv, pf[u][ks], acc[u][v], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < QPW; ++u) {
        if (wave + NW * u < nqb && q[u] < N) {
          const float inv = l[u] > 0.f ? 1.f / l[u] : 0.f;
          bf16* orow = p.o + ((int64_t)b * N + q[u]) * D + h * 64;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float w[4] = {acc[u][v][0] * inv, acc[u][v][1] * inv, acc[u][v][2] * inv, acc[u][v][3] * inv};
            store4(orow + v * 16 + 4 * g, w);
          }
          if (g == 0)
            p.lse[((int64_t)b * p.H + h) * N + q[u]] = l[u] > 0.f ? (mref[u] + __log2f(l[u])) * LN2 : NEG_INF;
        }
      }
    }
    item = nxt;
    if (item >= nitems) break;
  }
}

// ----------------------------------------------------------------------------- bwd
// Two phases share one LDS region of two [Npad][64] images (~57 KiB at N=197), so two
// 8-wave workgroups fit per CU and one's staging overlaps the other's MFMAs.
//   phase A (dK, dV): LDS holds Q and dO; each wave owns 16 keys whose K/V fragments come
//                     straight from global memory into registers.
//   phase B (dQ):     LDS is restaged with K and V; each wave owns 16 queries whose Q/dO
//                     fragments come from global memory.
__device__ __forceinline__ bf16x8 gfrag(const bf16* rowbase, int64_t ld, int r, int N, int kk, int g) {
  if (r >= N) return bf16x8{};  // padded rows contribute zero
  return *(const bf16x8*)(rowbase + (int64_t)r * ld + kk * 32 + 8 * g);
}

template <bool CAUSAL>
__global__ __launch_bounds__(512, 4) void attn_bwd_mfma(AttnP p) {  // 2 WGs per CU = 4 waves per SIMD
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x % p.H;
  const int N = p.N, D = p.D;
  const int NPAD = (N + 31) & ~31;
  const int64_t ld = 3 * (int64_t)D;
  char* img0 = smem;                    // phase A: Q,  phase B: K
  char* img1 = smem + NPAD * 128;       // phase A: dO, phase B: V
  float* lse2 = (float*)(smem + 2 * NPAD * 128);
  float* delta = lse2 + NPAD;
  int* keyok = (int*)(delta + NPAD);
  const bf16* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const bf16* dob = p.dout + (int64_t)b * N * D + h * 64;
  stage_img(img0, base, ld, N, NPAD, t, 512);
  stage_img(img1, dob, D, N, NPAD, t, 512);
  // delta[q] = sum_d dO*O ; 8 lanes per row
  {
    const bf16* ob = p.o + (int64_t)b * N * D + h * 64;
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

  // ---- phase A: dK, dV for 16 keys per wave (Q image in img0, dO image in img1)
  for (int kb = wave; kb < nkb; kb += 8) {
    const int key = kb * 16 + li;
    const bool kok = keyok[key];
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kk] = gfrag(base + D, ld, key, N, kk, g);
      vf[kk] = gfrag(base + 2 * D, ld, key, N, kk, g);
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
          sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img0, qr, kk * 4 + g), kf[kk], sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img1, qr, kk * 4 + g), vf[kk], dp, 0, 0, 0);
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
      const bf16x8 pf = pack8(pt[0], pt[1]);
      const bf16x8 sf = pack8(ds[0], ds[1]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dv[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img1, qs * 32, u * 16, lane), pf, dv[u], 0, 0, 0);
        dk[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img0, qs * 32, u * 16, lane), sf, dk[u], 0, 0, 0);
      }
    }
    if (key < N) {
      bf16* row = p.dqkv + ((int64_t)b * N + key) * ld + h * 64;
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
  stage_img(img0, base + D, ld, N, NPAD, t, 512);
  stage_img(img1, base + 2 * D, ld, N, NPAD, t, 512);
  __syncthreads();

  // ---- phase B: dQ for 16 queries per wave (K image in img0, V image in img1)
  const int nqb = (N + 15) >> 4;
  for (int qb = wave; qb < nqb; qb += 8) {
    const int q = qb * 16 + li;
    const float l2 = lse2[q], dl = delta[q];
    bf16x8 qf[2], of[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[kk] = gfrag(base, ld, q, N, kk, g);
      of[kk] = gfrag(dob, D, q, N, kk, g);
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
          sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img0, kr, kk * 4 + g), qf[kk], sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img1, kr, kk * 4 + g), of[kk], dp, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = ks * 32 + tau * 16 + 4 * g + r;
          const bool ok = keyok[key] && (!CAUSAL || key <= q);
          const float pv = ok ? exp2f(sc[r] * c2 - l2) : 0.f;
          ds[tau][r] = pv * (dp[r] - dl);
        }
      }
      const bf16x8 sf = pack8(ds[0], ds[1]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        dq[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img0, ks * 32, u * 16, lane), sf, dq[u], 0, 0, 0);
    }
    if (q < N) {
      bf16* row = p.dqkv + ((int64_t)b * N + q) * ld + h * 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float a[4] = {dq[u][0] * p.scale, dq[u][1] * p.scale, dq[u][2] * p.scale, dq[u][3] * p.scale};
        store4(row + u * 16 + 4 * g, a);
      }
    }
  }
}


// ------------------------------------------------------------------- bwd, streamed (N > 288)
// attn_bwd_mfma's two phases with the LDS images replaced by chunks of ST_CH rows: phase A (dK,
// dV; each wave owns 16 keys per round, fragments in registers) streams Q/dO chunks, phase B
// (dQ; 16 queries per wave per round) streams K/V chunks.  lse, delta and the key mask for all N
// stay in LDS.  Used where whole [N][64] images no longer fit (ViT-L/14@336: N = 577).
constexpr int ST_CH = 128;

template <bool CAUSAL>
__global__ __launch_bounds__(512, 1) void attn_bwd_stream(AttnP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = blockIdx.x / p.H, h = blockIdx.x % p.H;
  const int N = p.N, D = p.D;
  const int NPAD = (N + 31) & ~31;
  const int64_t ld = 3 * (int64_t)D;
  char* img0 = smem;                  // phase A: Q chunk,  phase B: K chunk
  char* img1 = smem + ST_CH * 128;    // phase A: dO chunk, phase B: V chunk
  float* lse2 = (float*)(smem + 2 * ST_CH * 128);
  float* delta = lse2 + NPAD;
  int* keyok = (int*)(delta + NPAD);
  const bf16* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const bf16* dob = p.dout + (int64_t)b * N * D + h * 64;
  {
    const bf16* ob = p.o + (int64_t)b * N * D + h * 64;
    for (int id = t; id < NPAD * 8; id += 512) {
      const int r = id >> 3, c = id & 7;
      float sm = 0.f;
      if (r < N) {
        float a[4], bb[4];
        load4(dob + (int64_t)r * D + c * 8, a);
        load4(ob + (int64_t)r * D + c * 8, bb);
        sm = a[0] * bb[0] + a[1] * bb[1] + a[2] * bb[2] + a[3] * bb[3];
        load4(dob + (int64_t)r * D + c * 8 + 4, a);
        load4(ob + (int64_t)r * D + c * 8 + 4, bb);
        sm += a[0] * bb[0] + a[1] * bb[1] + a[2] * bb[2] + a[3] * bb[3];
      }
      sm += __shfl_xor(sm, 1, 64);
      sm += __shfl_xor(sm, 2, 64);
      sm += __shfl_xor(sm, 4, 64);
      if (c == 0) delta[r] = sm;
    }
  }
  for (int k = t; k < NPAD; k += 512) {
    keyok[k] = (k < N) && (!p.kmask || p.kmask[(int64_t)b * N + k] != 0);
    lse2[k] = k < N ? p.lse[((int64_t)b * p.H + h) * N + k] * LOG2E : __builtin_huge_valf();
  }
  __syncthreads();  // keyok / lse2 / delta are read below before the first chunk's barrier
  const float c2 = p.scale * LOG2E;
  const int g = lane >> 4, li = lane & 15;
  const int nkb = (N + 15) >> 4, rounds = (nkb + 7) / 8;

  // ---- phase A: dK, dV
  for (int rd = 0; rd < rounds; ++rd) {
    const int kb = wave + 8 * rd;
    const int key = kb * 16 + li;
    const bool kok = kb < nkb && key < N && keyok[min(key, NPAD - 1)];
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kk] = gfrag(base + D, ld, key, N, kk, g);
      vf[kk] = gfrag(base + 2 * D, ld, key, N, kk, g);
    }
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { dv[u] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[u] = dv[u]; }
    for (int c0 = 0; c0 < N; c0 += ST_CH) {
      const int cn = min(ST_CH, N - c0);
      __syncthreads();  // previous chunk's readers done (first time: lse2/delta/keyok written)
      stage_img(img0, base + (int64_t)c0 * ld, ld, cn, ST_CH, t, 512);
      stage_img(img1, dob + (int64_t)c0 * D, D, cn, ST_CH, t, 512);
      __syncthreads();
      if (kb >= nkb) continue;
      for (int qs = 0; qs < (cn + 31) / 32; ++qs) {
        if (CAUSAL && c0 + qs * 32 + 31 < kb * 16) continue;  // every query of this step precedes every key
        f32x4 pt[2], ds[2];
#pragma unroll
        for (int tau = 0; tau < 2; ++tau) {
          f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
          const int qr = qs * 32 + tau * 16 + li;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img0, qr, kk * 4 + g), kf[kk], sc, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img1, qr, kk * 4 + g), vf[kk], dp, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = c0 + qs * 32 + tau * 16 + 4 * g + r;
            const bool ok = kok && (!CAUSAL || key <= q);
            const float pv = ok ? __builtin_amdgcn_exp2f(sc[r] * c2 - lse2[q]) : 0.f;
            pt[tau][r] = pv;
            ds[tau][r] = pv * (dp[r] - delta[q]);
          }
        }
        const bf16x8 pf = pack8(pt[0], pt[1]);
        const bf16x8 sf = pack8(ds[0], ds[1]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          dv[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img1, qs * 32, u * 16, lane), pf, dv[u], 0, 0, 0);
          dk[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img0, qs * 32, u * 16, lane), sf, dk[u], 0, 0, 0);
        }
      }
    }
    if (kb < nkb && key < N) {
      bf16* row = p.dqkv + ((int64_t)b * N + key) * ld + h * 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float a[4] = {dk[u][0] * p.scale, dk[u][1] * p.scale, dk[u][2] * p.scale, dk[u][3] * p.scale};
        float c[4] = {dv[u][0], dv[u][1], dv[u][2], dv[u][3]};
        store4(row + D + u * 16 + 4 * g, a);
        store4(row + 2 * D + u * 16 + 4 * g, c);
      }
    }
  }

  // ---- phase B: dQ
  const int nqb = (N + 15) >> 4, qrounds = (nqb + 7) / 8;
  for (int rd = 0; rd < qrounds; ++rd) {
    const int qb = wave + 8 * rd;
    const int q = qb * 16 + li;
    const int qc = min(q, NPAD - 1);
    const float l2 = lse2[qc], dl = delta[qc];
    bf16x8 qf[2], of[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[kk] = gfrag(base, ld, q, N, kk, g);
      of[kk] = gfrag(dob, D, q, N, kk, g);
    }
    f32x4 dq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) dq[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < N; c0 += ST_CH) {
      const int cn = min(ST_CH, N - c0);
      __syncthreads();
      stage_img(img0, base + (int64_t)c0 * ld + D, ld, cn, ST_CH, t, 512);
      stage_img(img1, base + (int64_t)c0 * ld + 2 * D, ld, cn, ST_CH, t, 512);
      __syncthreads();
      if (qb >= nqb) continue;
      for (int ks = 0; ks < (cn + 31) / 32; ++ks) {
        if (CAUSAL && c0 + ks * 32 > qb * 16 + 15) break;
        f32x4 ds[2];
#pragma unroll
        for (int tau = 0; tau < 2; ++tau) {
          f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
          const int kr = ks * 32 + tau * 16 + li;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img0, kr, kk * 4 + g), qf[kk], sc, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(img1, kr, kk * 4 + g), of[kk], dp, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = c0 + ks * 32 + tau * 16 + 4 * g + r;
            const bool ok = key < N && keyok[key] && (!CAUSAL || key <= q);
            const float pv = ok ? __builtin_amdgcn_exp2f(sc[r] * c2 - l2) : 0.f;
            ds[tau][r] = pv * (dp[r] - dl);
          }
        }
        const bf16x8 sf = pack8(ds[0], ds[1]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          dq[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(img0, ks * 32, u * 16, lane), sf, dq[u], 0, 0, 0);
      }
    }
    if (qb < nqb && q < N) {
      bf16* row = p.dqkv + ((int64_t)b * N + q) * ld + h * 64;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float a[4] = {dq[u][0] * p.scale, dq[u][1] * p.scale, dq[u][2] * p.scale, dq[u][3] * p.scale};
        store4(row + u * 16 + 4 * g, a);
      }
    }
  }
}

// ------------------------------------------------------------------- bwd, prefetching
// Persistent backward: a workgroup of NW waves walks (batch, head) items gridDim.x apart.
// Per item, LDS holds the Q, dO, O images (phase A + delta) and the K, V images (phase B):
//   top:     wait for Q/dO/O(i) + meta(i); delta(i) = rowsum(dO * O) from the images
//   phase A: DMA K/V(i) into their images while computing dK, dV (each wave owns 16 keys,
//            K/V fragments in registers, loaded from global during phase B(i - 1))
//   phase B: load item i + 1's K/V fragments and lse / key mask (plain loads, issued before
//            any DMA so their waits never wait on the ring), copy this wave's Q/dO(i)
//            fragments out of LDS, then DMA Q/dO/O(i + 1) over those images while computing
//            dQ (each wave owns 16 queries, K/V images).
// So every byte the next phase needs is in flight during the current one.  Barriers that
// must not wait for those plain loads are raw s_barrier (lgkmcnt only).
// CLIPMI_ATTN_PRIO (A/B builds): raise the wave's issue priority over its MFMA clusters so a SIMD's other wave's
// exponentials issue beside them instead of competing for issue slots while the matrix pipe waits
#ifndef CLIPMI_ATTN_PRIO
#define CLIPMI_ATTN_PRIO 0
#endif
__device__ __forceinline__ void prio_hi() {
  if constexpr (CLIPMI_ATTN_PRIO) __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void prio_lo() {
  if constexpr (CLIPMI_ATTN_PRIO) __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void raw_barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


// Per-item context of the prefetching backward's two phases.
struct BwdCtx {
  const char *Qimg, *dOimg, *Kimg, *Vimg;
  const float *lse2, *delta;
  const int* keyok;
  bf16* dq_base;  // dqkv + (b * N) * ld + h * 64
  int64_t ld;
  int N, NPAD, nstep, lane, D;
  float c2, scale;
};

// dK, dV of the wave's NB key blocks (kb = wave, wave + NW): K/V fragments in registers,
// Q/dO images in LDS.
template <bool CAUSAL, int NB, bool LOWREG = false, int NBA>
__device__ __forceinline__ void bwd_phase_a(const BwdCtx& c, const bf16x8 (&kf)[NBA][2], const bf16x8 (&vf)[NBA][2],
                                            int wave, int NW) {
  static_assert(NB <= NBA, "bwd_phase_a: fragments");
  const int lane = c.lane, g = lane >> 4, li = lane & 15;
  bool kok[NB];
  int key[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    key[u] = (wave + NW * u) * 16 + li;
    kok[u] = key[u] < c.N ? c.keyok[key[u]] != 0 : false;  // blocks past N (4-wave form) read nothing
  }
  f32x4 dv[NB][4], dk[NB][4];
#pragma unroll
  for (int u = 0; u < NB; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) { dv[u][v] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[u][v] = dv[u][v]; }
  for (int qs = 0; qs < c.nstep; ++qs) {
    if (CAUSAL && qs * 32 + 31 < wave * 16) continue;  // every query of this step precedes every key
    f32x4 pt[NB][2], ds[NB][2];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      const int qr = qs * 32 + tau * 16 + li;
      bf16x8 qa[2], da[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        qa[kk] = frag_row(c.Qimg, qr, kk * 4 + g);
        da[kk] = frag_row(c.dOimg, qr, kk * 4 + g);
      }
      const int q0 = qs * 32 + tau * 16 + 4 * g;
      const f32x4 l4 = *LDS_PTR(const f32x4, c.lse2 + q0);
      const f32x4 d4 = *LDS_PTR(const f32x4, c.delta + q0);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        // non-causal: the key mask and -delta ride in the accumulators' initial values (a masked key's
        // scores start at -inf, so exp2 gives P = 0; dP starts at -delta): no select and no subtract per
        // element -- the phases are VALU-issue bound beside their MFMAs
        f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
        if constexpr (!CAUSAL) {
          const float s0 = kok[u] ? 0.f : NEG_INF;
          sc = f32x4{s0, s0, s0, s0};
          dp = f32x4{-d4[0], -d4[1], -d4[2], -d4[3]};
        }
        prio_hi();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[kk], kf[u][kk], sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[kk], vf[u][kk], dp, 0, 0, 0);
        }
        prio_lo();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (!CAUSAL) {
            const float pv = __builtin_amdgcn_exp2f(sc[r] * c.c2 - l4[r]);
            pt[u][tau][r] = pv;
            ds[u][tau][r] = pv * dp[r];
          } else {
            const bool ok = kok[u] && key[u] <= q0 + r;
            const float pv = ok ? __builtin_amdgcn_exp2f(sc[r] * c.c2 - l4[r]) : 0.f;
            pt[u][tau][r] = pv;
            ds[u][tau][r] = pv * (dp[r] - d4[r]);
          }
        }
      }
      if constexpr (LOWREG) __builtin_amdgcn_sched_barrier(0);  // one tau's operands live at a time
    }
    bf16x8 pf[NB], sf[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      pf[u] = pack8(pt[u][0], pt[u][1]);
      sf[u] = pack8(ds[u][0], ds[u][1]);
    }
    prio_hi();
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const bf16x8 td = frag_tr(c.dOimg, qs * 32, v * 16, lane), tq = frag_tr(c.Qimg, qs * 32, v * 16, lane);
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        dv[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(td, pf[u], dv[u][v], 0, 0, 0);
        dk[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tq, sf[u], dk[u][v], 0, 0, 0);
      }
    }
    prio_lo();
  }
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    if (key[u] < c.N) {
      bf16* row = c.dq_base + (int64_t)key[u] * c.ld;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float a[4] = {dk[u][v][0] * c.scale, dk[u][v][1] * c.scale, dk[u][v][2] * c.scale, dk[u][v][3] * c.scale};
        float w[4] = {dv[u][v][0], dv[u][v][1], dv[u][v][2], dv[u][v][3]};
        store4(row + c.D + v * 16 + 4 * g, a);
        store4(row + 2 * c.D + v * 16 + 4 * g, w);
      }
    }
  }
}

// dQ of the wave's NB query blocks (qb = wave, wave + NW): Q/dO fragments in registers, K/V
// images in LDS; the blocks advance together over the keys, sharing every K/V read.
template <bool CAUSAL, int NB, bool LOWREG = false, int NBA>
__device__ __forceinline__ void bwd_phase_b(const BwdCtx& c, const bf16x8 (&qf)[NBA][2], const bf16x8 (&of)[NBA][2],
                                            int wave, int NW) {
  static_assert(NB <= NBA, "bwd_phase_b: fragments");
  const int lane = c.lane, g = lane >> 4, li = lane & 15;
  int q[NB];
  float l2[NB], dl[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    q[u] = (wave + NW * u) * 16 + li;
    const int qi = min(q[u], c.NPAD - 1);  // blocks past NPAD (4-wave form): never stored
    l2[u] = c.lse2[qi];
    dl[u] = c.delta[qi];
  }
  f32x4 dq[NB][4];
#pragma unroll
  for (int u = 0; u < NB; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) dq[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kslim = CAUSAL ? min(c.nstep, ((wave + NW * (NB - 1)) * 16 + 15) / 32 + 1) : c.nstep;
  for (int ks = 0; ks < kslim; ++ks) {
    f32x4 ds[NB][2];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      const int kr = ks * 32 + tau * 16 + li;
      bf16x8 ka[2], va[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ka[kk] = frag_row(c.Kimg, kr, kk * 4 + g);
        va[kk] = frag_row(c.Vimg, kr, kk * 4 + g);
      }
      const int k0 = ks * 32 + tau * 16 + 4 * g;
      const i32x4 ko = *LDS_PTR(const i32x4, c.keyok + k0);
      // non-causal: key mask and -delta as the accumulators' initial values (see bwd_phase_a)
      f32x4 seed = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (!CAUSAL) seed = f32x4{ko[0] ? 0.f : NEG_INF, ko[1] ? 0.f : NEG_INF, ko[2] ? 0.f : NEG_INF,
                                          ko[3] ? 0.f : NEG_INF};
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        f32x4 sc = seed, dp = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (!CAUSAL) dp = f32x4{-dl[u], -dl[u], -dl[u], -dl[u]};
        prio_hi();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[kk], qf[u][kk], sc, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[kk], of[u][kk], dp, 0, 0, 0);
        }
        prio_lo();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (!CAUSAL) {
            ds[u][tau][r] = __builtin_amdgcn_exp2f(sc[r] * c.c2 - l2[u]) * dp[r];
          } else {
            const bool ok = ko[r] && k0 + r <= q[u];
            const float pv = ok ? __builtin_amdgcn_exp2f(sc[r] * c.c2 - l2[u]) : 0.f;
            ds[u][tau][r] = pv * (dp[r] - dl[u]);
          }
        }
      }
      if constexpr (LOWREG) __builtin_amdgcn_sched_barrier(0);
    }
    bf16x8 sf[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) sf[u] = pack8(ds[u][0], ds[u][1]);
    prio_hi();
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const bf16x8 tk = frag_tr(c.Kimg, ks * 32, v * 16, lane);
#pragma unroll
      for (int u = 0; u < NB; ++u)
        dq[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tk, sf[u], dq[u][v], 0, 0, 0);
    }
    prio_lo();
  }
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    if (q[u] < c.N) {
      bf16* row = c.dq_base + (int64_t)q[u] * c.ld;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float a[4] = {dq[u][v][0] * c.scale, dq[u][v][1] * c.scale, dq[u][v][2] * c.scale, dq[u][v][3] * c.scale};
        store4(row + v * 16 + 4 * g, a);
      }
    }
  }
}

template <bool CAUSAL, int NW, int NBM>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_pf(AttnP p, int nitems) {
  constexpr int NT = NW * 64;
  // key / query blocks per wave (NBM): two with 8 waves (N <= 256) or 4 waves (N <= 128); one with
  // 16 (N <= 256: 4 waves per SIMD, 128 registers each, so one wave's MFMA -> exp -> MFMA chain
  // hides behind three others); four with 4 waves (N <= 256, non-causal: one wave per SIMD whose
  // four blocks share every Q / dO / K / V fragment read, halving the LDS traffic of the 8-wave form)
  static_assert(NBM == 4 ? (NW == 4 && !CAUSAL) : NBM == (NW >= 16 ? 1 : 2), "attn_bwd_pf: blocks per wave");
  constexpr int NBA = NBM < 2 ? 2 : NBM;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int N = p.N, D = p.D, H = p.H;
  const int NPAD = (N + 31) & ~31, IMG = NPAD * 128;
  const int64_t ld = 3 * (int64_t)D;
  char* Qimg = smem;
  char* dOimg = smem + IMG;
  char* Oimg = smem + 2 * IMG;
  char* Kimg = smem + 3 * IMG;
  char* Vimg = smem + 4 * IMG;
  float* arr = (float*)(smem + 5 * IMG);  // [2 slots][lse2 | delta | keyok][NPAD]
  const uint32_t rec3 = (uint32_t)((int64_t)(N - 1) * ld * 2 + 128);
  const uint32_t rec1 = (uint32_t)((int64_t)(N - 1) * D * 2 + 128);
  const float c2 = p.scale * LOG2E;
  const int g = lane >> 4, li = lane & 15;
  const int nkb = (N + 15) >> 4, nstep = NPAD >> 5;

  auto qkv_of = [&](int item) {
    const int b = item / H, h = item - b * H;
    return p.qkv + (int64_t)b * N * ld + h * 64;
  };
  auto issue_qdo = [&](int item) {
    const int b = item / H, h = item - b * H;
    const SRsrc rq = make_srsrc(qkv_of(item), rec3);
    const SRsrc rd = make_srsrc(p.dout + (int64_t)b * N * D + h * 64, rec1);
    const SRsrc ro = make_srsrc(p.o + (int64_t)b * N * D + h * 64, rec1);
#pragma unroll 1
    for (int j = wave; j < NPAD / 8; j += NW) {
      const int r = 8 * j + (lane >> 3), c = ((lane & 7) ^ (r & 6)) << 4;
      dma16(rq, Qimg + j * 1024, r * (int)ld * 2 + c);
      dma16(rd, dOimg + j * 1024, r * D * 2 + c);
      dma16(ro, Oimg + j * 1024, r * D * 2 + c);
    }
  };
  auto issue_kv = [&](int item) {
    const bf16* base = qkv_of(item);
    const SRsrc rk = make_srsrc(base + D, rec3), rv = make_srsrc(base + 2 * D, rec3);
#pragma unroll 1
    for (int j = wave; j < NPAD / 8; j += NW) {
      const int r = 8 * j + (lane >> 3), c = ((lane & 7) ^ (r & 6)) << 4;
      dma16(rk, Kimg + j * 1024, r * (int)ld * 2 + c);
      dma16(rv, Vimg + j * 1024, r * (int)ld * 2 + c);
    }
  };
  auto load_kvfrag = [&](int item, bf16x8 (&kf)[NBA][2], bf16x8 (&vf)[NBA][2]) {
    const bf16* base = qkv_of(item);
#pragma unroll
    for (int u = 0; u < NBM; ++u) {
      const int key = min((wave + NW * u) * 16 + li, N - 1);  // rows past N are masked by keyok
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        kf[u][kk] = *(const bf16x8*)(base + D + (int64_t)key * ld + kk * 32 + 8 * g);
        vf[u][kk] = *(const bf16x8*)(base + 2 * D + (int64_t)key * ld + kk * 32 + 8 * g);
      }
    }
  };
  // the raw loaded values stay untouched until store_meta: arithmetic on them right after the loads
  // made the compiler wait (vmcnt(0)) there -- for them and for the next item's K/V fragment loads
  // issued just before -- in the middle of the phase-A -> phase-B handover (ViT-B/16 backward
  // 952 -> 933 us, profiles/r05_attn_bwd_meta_ab.log)
  auto load_meta = [&](int item, float& lse_raw, int64_t& km_raw) {
    const int b = item / H, h = item - b * H;
    lse_raw = __builtin_huge_valf();
    km_raw = 0;
    if (t < N) {
      lse_raw = p.lse[((int64_t)b * H + h) * N + t];
      // an opaque 1 for the no-mask arm: with a constant there, instcombine folds store_meta's != 0 into
      // the load's arm (right behind the load, so the compiler waits for it there)
      int64_t one = 1;
      asm volatile("" : "+v"(one));
      km_raw = p.kmask ? p.kmask[(int64_t)b * N + t] : one;
    }
  };
  auto store_meta = [&](int sl, float lse_raw, int64_t km_raw) {
    if (t < NPAD) {
      arr[sl * 3 * NPAD + t] = lse_raw * LOG2E;
      ((int*)arr)[sl * 3 * NPAD + 2 * NPAD + t] = km_raw != 0;
    }
  };

  int item = blockIdx.x;
  bf16x8 kf[NBA][2], vf[NBA][2];
  {
    float l2v;
    int64_t kov;
    load_kvfrag(item, kf, vf);
    load_meta(item, l2v, kov);
    issue_qdo(item);
    store_meta(0, l2v, kov);
  }
  for (int it = 0;; ++it) {
    const int sl = it & 1;
    const float* lse2 = arr + sl * 3 * NPAD;
    float* delta = arr + sl * 3 * NPAD + NPAD;
    const int* keyok = (const int*)(arr + sl * 3 * NPAD + 2 * NPAD);
    ATT_ST(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // Q/dO/O(i), meta(i) ready; K/V images free
    ATT_ST(1);
    const int cur = item, nxt = item + gridDim.x;
    const int b = cur / H, h = cur - b * H;
    const BwdCtx c{Qimg, dOimg, Kimg, Vimg, lse2, delta, keyok, p.dqkv + (int64_t)b * N * ld + h * 64, ld,
                   N, NPAD, nstep, lane, D, c2, p.scale};
    // delta[q] = sum_d dO * O, 8 lanes per row, from the LDS images
    for (int id = t; id < NPAD * 8; id += NT) {
      const int r = id >> 3, c = id & 7;
      const bf16x8 a = frag_row(dOimg, r, c), o8 = frag_row(Oimg, r, c);
      float sum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sum = fmaf((float)a[e], (float)o8[e], sum);
      sum += __shfl_xor(sum, 1, 64);
      sum += __shfl_xor(sum, 2, 64);
      sum += __shfl_xor(sum, 4, 64);
      if (c == 0) delta[r] = sum;
    }
    raw_barrier_lds();
    issue_kv(cur);
    ATT_ST(2);

    // ---- phase A: dK, dV (Q image, dO image); a wave with two key blocks advances them
    // together so each Q/dO fragment read from LDS feeds both
    // (causal: blocks far apart need different query ranges, so they run one at a time)
    if constexpr (NBM == 4) {
      bwd_phase_a<CAUSAL, 4>(c, kf, vf, wave, NW);  // blocks past N compute P = 0 and store nothing
    } else if constexpr (NBM == 1) {
      if (wave < nkb) bwd_phase_a<CAUSAL, 1, true>(c, kf, vf, wave, NW);
    } else if (!CAUSAL && wave + NW < nkb) {
      bwd_phase_a<CAUSAL, 2>(c, kf, vf, wave, NW);
    } else {
      if (wave < nkb) bwd_phase_a<CAUSAL, 1>(c, kf, vf, wave, NW);
      if (wave + NW < nkb) {
        const bf16x8 kf1[2][2] = {{kf[1][0], kf[1][1]}, {kf[1][0], kf[1][1]}};
        const bf16x8 vf1[2][2] = {{vf[1][0], vf[1][1]}, {vf[1][0], vf[1][1]}};
        bwd_phase_a<CAUSAL, 1>(c, kf1, vf1, wave + NW, NW);
      }
    }
    ATT_ST(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // K/V(i) images landed; phase A's reads of Q/dO done
    ATT_ST(4);

    // ---- phase B: dQ (K image, V image)
    const bool more = nxt < nitems;
    float l2n = 0.f;
    int64_t kon = 0;
    if (more) {
      load_kvfrag(nxt, kf, vf);
      load_meta(nxt, l2n, kon);
    }
    const int nqb = (N + 15) >> 4;
    bf16x8 qf[NBA][2], of[NBA][2];
#pragma unroll
    for (int u = 0; u < NBM; ++u) {
      const int q = min((wave + NW * u) * 16, NPAD - 16) + li;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        qf[u][kk] = frag_row(Qimg, q, kk * 4 + g);
        of[u][kk] = frag_row(dOimg, q, kk * 4 + g);
      }
    }
    raw_barrier_lds();  // every wave holds its Q/dO fragments: the images may be overwritten
    if (more) issue_qdo(nxt);
    ATT_ST(5);
    if constexpr (NBM == 4) {
      bwd_phase_b<CAUSAL, 4>(c, qf, of, wave, NW);
    } else if constexpr (NBM == 1) {
      if (wave < nqb) bwd_phase_b<CAUSAL, 1, true>(c, qf, of, wave, NW);
    } else if (!CAUSAL && wave + NW < nqb) {
      bwd_phase_b<CAUSAL, 2>(c, qf, of, wave, NW);
    } else {
      if (wave < nqb) bwd_phase_b<CAUSAL, 1>(c, qf, of, wave, NW);
      if (wave + NW < nqb) {
        const bf16x8 qf1[2][2] = {{qf[1][0], qf[1][1]}, {qf[1][0], qf[1][1]}};
        const bf16x8 of1[2][2] = {{of[1][0], of[1][1]}, {of[1][0], of[1][1]}};
        bwd_phase_b<CAUSAL, 1>(c, qf1, of1, wave + NW, NW);
      }
    }
    ATT_ST(6);
    if (!more) break;
    store_meta(sl ^ 1, l2n, kon);  // slot sl ^ 1's readers (item i - 1) finished long ago
    item = nxt;
  }
}

// ------------------------------------------------------------------- bwd, single pass
// attn_bwd_sp<CAUSAL, NW, NKC>: the backward of one (batch, head) item in ONE sweep over its query
// steps (32 queries each), N <= 32 * NKC.  attn_bwd_pf computes dK/dV in a key-owned phase and dQ
// in a query-owned phase, recomputing S, dP and every exponential for the second; here:
//   per step qs, every wave: S = Q K^T and dP = dO V^T of its key blocks against the step's
//   queries (Q/dO fragments from the LDS images, K/V fragments in registers), P and
//   dS = P (dP - delta), dV += P^T dO and dK += dS^T Q in registers (as attn_bwd_pf's phase A), and
//   dS^T (the bf16 values dK used) into one 32-column half of a [NPAD keys][64] dS image;
//   one barrier; then dQ^T(step) = K^T dS^T over all NPAD keys: wave w owns the (d-tile, query
//   half) tile(s) of the step's [32 x 64] dQ block -- one with 8 waves, two with 4 -- from K^T
//   fragments held in registers for the whole item, and writes it out.  The two dS halves
//   alternate between steps, so one barrier per step covers both hazards.
// So per (16 queries x 32 keys) the MFMA count drops from 28 to 20 and the exponentials halve.
// Next item's operands: its K image DMA'd into the second K slot and its V fragments loaded into
// registers at the start of this item; the Q / dO rows of step qs DMA'd right after the barrier
// that retires them (rolling); O rows (for delta = rowsum(dO o O)) and lse / key mask prefetched
// into registers.  K and K^T fragments are read from the K image where they are used (two
// waves per SIMD leave 256 registers per wave: holding them for the whole item spilled).
// LDS: Q, dO, K x 2, dS images (5 x NPAD x 128 B) + 2 slots of lse2 | delta | keyok.
template <bool CAUSAL, int NW, int NKC>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_sp(AttnP p, int nitems) {  // 2 waves per SIMD
  constexpr int NT = NW * 64, NPAD = NKC * 32, IMG = NPAD * 128;
  constexpr int NB = 2;                                  // key blocks per wave (nkb <= 2 NW)
  constexpr int NQT = 8 / NW;                            // dQ tiles per wave per step
  constexpr int NOC = (NPAD * 8 + NT - 1) / NT;          // O chunks per thread (delta)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int N = p.N, D = p.D, H = p.H;
  const int64_t ld = 3 * (int64_t)D;
  char* Qimg = smem;
  char* dOimg = smem + IMG;
  char* Kimg2 = smem + 2 * IMG;  // [2 slots]
  char* dSimg = smem + 4 * IMG;
  float* arr = (float*)(smem + 5 * IMG);  // [2 slots][lse2 | delta | keyok][NPAD]
  const uint32_t rec3 = (uint32_t)((int64_t)(N - 1) * ld * 2 + 128);
  const uint32_t rec1 = (uint32_t)((int64_t)(N - 1) * D * 2 + 128);
  const float c2 = p.scale * LOG2E;
  const int g = lane >> 4, li = lane & 15;
  const int nkb = (N + 15) >> 4, nstep = (N + 31) >> 5;
  const int dt = wave & 3;  // this wave's dQ d-tile

  auto qkv_of = [&](int item) {
    const int b = item / H, h = item - b * H;
    return p.qkv + (int64_t)b * N * ld + h * 64;
  };
  auto issue_k = [&](int item, int slot) {
    const SRsrc rk = make_srsrc(qkv_of(item) + D, rec3);
    char* kimg = Kimg2 + __builtin_amdgcn_readfirstlane(slot * IMG);  // wave-uniform M0 base
#pragma unroll 1
    for (int j = wave; j < NPAD / 8; j += NW) {
      const int r = 8 * j + (lane >> 3), c = ((lane & 7) ^ (r & 6)) << 4;
      dma16(rk, kimg + j * 1024, r * (int)ld * 2 + c);
    }
  };
  auto load_vf = [&](int item, bf16x8 (&vf)[NB][2]) {  // V fragments of the wave's key blocks
    const bf16* base = qkv_of(item) + 2 * D;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int key = min((wave + NW * u) * 16 + li, N - 1);  // rows past N are masked by keyok
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) vf[u][kk] = *(const bf16x8*)(base + (int64_t)key * ld + kk * 32 + 8 * g);
    }
  };
  // Q / dO rows [8 j0, 8 j1) of item (1 KiB pieces of 8 rows)
  auto issue_qdo = [&](int item, int j0, int j1) {
    const int b = item / H, h = item - b * H;
    const SRsrc rq = make_srsrc(qkv_of(item), rec3);
    const SRsrc rd = make_srsrc(p.dout + (int64_t)b * N * D + h * 64, rec1);
#pragma unroll 1
    for (int j = j0 + wave; j < j1; j += NW) {
      const int r = 8 * j + (lane >> 3), c = ((lane & 7) ^ (r & 6)) << 4;
      dma16(rq, Qimg + j * 1024, r * (int)ld * 2 + c);
      dma16(rd, dOimg + j * 1024, r * D * 2 + c);
    }
  };
  auto load_o = [&](int item, u32x4 (&o)[NOC]) {
    const int b = item / H, h = item - b * H;
    const bf16* base = p.o + (int64_t)b * N * D + h * 64;
#pragma unroll
    for (int j = 0; j < NOC; ++j) {
      const int id = t + NT * j, r = id >> 3, c = id & 7;
      o[j] = u32x4{0u, 0u, 0u, 0u};
      if (id < NPAD * 8 && r < N) o[j] = *(const u32x4*)(base + (int64_t)r * D + c * 8);
    }
  };
  auto load_meta = [&](int item, float& l2v, int& kov) {
    const int b = item / H, h = item - b * H;
    l2v = __builtin_huge_valf();
    kov = 0;
    if (t < N) {
      l2v = p.lse[((int64_t)b * H + h) * N + t] * LOG2E;
      kov = !p.kmask || p.kmask[(int64_t)b * N + t] != 0;
    }
  };
  static_assert(NPAD <= NT, "one thread per key / query row");
  auto store_meta = [&](int sl, float l2v, int kov) {
    if (t < NPAD) {
      arr[sl * 3 * NPAD + t] = l2v;
      ((int*)arr)[sl * 3 * NPAD + 2 * NPAD + t] = kov;
    }
  };

  int item = blockIdx.x;
  u32x4 orow[NOC];
  bf16x8 vfn[NB][2];
  {
    float l2v;
    int kov;
    issue_k(item, 0);
    load_vf(item, vfn);
    issue_qdo(item, 0, NPAD / 8);
    load_o(item, orow);
    load_meta(item, l2v, kov);
    for (int id = t; id < NPAD * 8; id += NT) *LDS_PTR(u32x4, dSimg + id * 16) = u32x4{0u, 0u, 0u, 0u};
    store_meta(0, l2v, kov);
  }
  for (int it = 0;; ++it) {
    const int sl = it & 1;
    const float* lse2 = arr + sl * 3 * NPAD;
    float* delta = arr + sl * 3 * NPAD + NPAD;
    const int* keyok = (const int*)(arr + sl * 3 * NPAD + 2 * NPAD);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // item's images, meta and O rows landed; the dS image idle
    const int cur = item, nxt = item + gridDim.x;
    const bool more = nxt < nitems;
    const int b = cur / H, h = cur - b * H;
    bf16* dq_base = p.dqkv + (int64_t)b * N * ld + h * 64;

    const char* Kimg = Kimg2 + __builtin_amdgcn_readfirstlane(sl * IMG);
    int key[NB], krow[NB];
    bool kok[NB], kbv[NB];
    bf16x8 vf[NB][2];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int kb = wave + NW * u;
      kbv[u] = kb < nkb;
      key[u] = kb * 16 + li;
      krow[u] = min(key[u], NPAD - 1);
      kok[u] = keyok[krow[u]] != 0;
      vf[u][0] = vfn[u][0];
      vf[u][1] = vfn[u][1];
    }
    // delta[q] = sum_d dO * O, 8 lanes per row (dO image, O rows in registers)
#pragma unroll
    for (int j = 0; j < NOC; ++j) {
      const int id = t + NT * j, r = id >> 3, c = id & 7;
      if (NOC * NT == NPAD * 8 || id < NPAD * 8) {  // whole 8-lane groups: NPAD * 8 % 8 == 0
        const bf16x8 a = frag_row(dOimg, r, c);
        float sum = 0.f;
        const u32x4 o4 = orow[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sum = fmaf((float)a[2 * e], __uint_as_float(o4[e] << 16), sum);
          sum = fmaf((float)a[2 * e + 1], __uint_as_float(o4[e] & 0xffff0000u), sum);
        }
        sum += __shfl_xor(sum, 1, 64);
        sum += __shfl_xor(sum, 2, 64);
        sum += __shfl_xor(sum, 4, 64);
        if (c == 0) delta[r] = sum;
      }
    }
    raw_barrier_lds();  // delta visible (the other K slot's readers, item it - 1, are done)
    float l2n = 0.f;
    int kon = 0;
    if (more) {
      issue_k(nxt, sl ^ 1);
      load_vf(nxt, vfn);
      load_o(nxt, orow);
      load_meta(nxt, l2n, kon);
    }

    f32x4 dv[NB][4], dk[NB][4];
#pragma unroll
    for (int u = 0; u < NB; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) { dv[u][v] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[u][v] = dv[u][v]; }

    // dQ^T of step sq (dS^T in half sq & 1): this wave's tile(s) over all keys (causal: keys <= the
    // step's last query).  Run one step late, before the next step's phase A, so its dependent MFMA
    // chain and LDS reads overlap that phase's independent work instead of idling after a barrier.
    auto dq_step = [&](int sq) {
      const int hq = sq & 1;
      const int kcl = CAUSAL ? min(NKC, sq + 1) : NKC;
#pragma unroll
      for (int j = 0; j < NQT; ++j) {
        const int qt = NQT == 1 ? (wave >> 2) : j;
        f32x4 acc2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
          if (kc < kcl) {
            const bf16x8 kt = frag_tr(Kimg, kc * 32, dt * 16, lane);
            const bf16x8 st = frag_tr(dSimg, kc * 32, hq * 32 + qt * 16, lane);
            acc2[kc & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt, st, acc2[kc & 1], 0, 0, 0);
          }
        }
        const f32x4 acc = acc2[0] + acc2[1];
        const int q = sq * 32 + qt * 16 + li;
        if (q < N) {
          float a[4] = {acc[0] * p.scale, acc[1] * p.scale, acc[2] * p.scale, acc[3] * p.scale};
          store4(dq_base + (int64_t)q * ld + dt * 16 + 4 * g, a);
        }
      }
    };
    for (int qs = 0; qs < nstep; ++qs) {
      const int hb = qs & 1;
      // half hb^1 holds dS(qs - 1), made visible by the previous barrier; half hb's last reader
      // (dQ(qs - 2)) ran before that barrier, so this step may overwrite it
      if (qs > 0) dq_step(qs - 1);
      bool act[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) act[u] = kbv[u] && !(CAUSAL && qs * 32 + 31 < (wave + NW * u) * 16);
      // P and dS of each key block, packed to bf16 per 16-query half (tau) as soon as they are
      // formed; dS^T goes to the dS image at once (zeros for a causally skipped block)
      bf16x4 pl[NB][2], sl[NB][2];
#pragma unroll
      for (int tau = 0; tau < 2; ++tau) {
        const int qr = qs * 32 + tau * 16 + li;
        bf16x8 qa[2], da[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          qa[kk] = frag_row(Qimg, qr, kk * 4 + g);
          da[kk] = frag_row(dOimg, qr, kk * 4 + g);
        }
        const int q0 = qs * 32 + tau * 16 + 4 * g;
        const f32x4 l4 = *LDS_PTR(const f32x4, lse2 + q0);
        const f32x4 d4 = *LDS_PTR(const f32x4, delta + q0);
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          float pv4[4] = {0.f, 0.f, 0.f, 0.f}, ds4[4] = {0.f, 0.f, 0.f, 0.f};
          if (act[u]) {
            f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f}, dp = sc;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
              const bf16x8 kf = frag_row(Kimg, krow[u], kk * 4 + g);
              sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[kk], kf, sc, 0, 0, 0);
              dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[kk], vf[u][kk], dp, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const bool ok = kok[u] && (!CAUSAL || key[u] <= q0 + r);
              pv4[r] = ok ? __builtin_amdgcn_exp2f(sc[r] * c2 - l4[r]) : 0.f;
              ds4[r] = pv4[r] * (dp[r] - d4[r]);
            }
          }
          pl[u][tau] = bf16x4{(bf16)pv4[0], (bf16)pv4[1], (bf16)pv4[2], (bf16)pv4[3]};
          sl[u][tau] = bf16x4{(bf16)ds4[0], (bf16)ds4[1], (bf16)ds4[2], (bf16)ds4[3]};
          if (kbv[u])  // dS^T row key[u], columns hb*32 + tau*16 + 4g .. +3
            *LDS_PTR(bf16x4, dSimg + img_off(key[u], hb * 4 + tau * 2 + (g >> 1)) + (g & 1) * 8) = sl[u][tau];
        }
      }
      bf16x8 pf[NB], sf[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        pf[u] = bf16x8{pl[u][0][0], pl[u][0][1], pl[u][0][2], pl[u][0][3], pl[u][1][0], pl[u][1][1], pl[u][1][2], pl[u][1][3]};
        sf[u] = bf16x8{sl[u][0][0], sl[u][0][1], sl[u][0][2], sl[u][0][3], sl[u][1][0], sl[u][1][1], sl[u][1][2], sl[u][1][3]};
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const bf16x8 td = frag_tr(dOimg, qs * 32, v * 16, lane), tq = frag_tr(Qimg, qs * 32, v * 16, lane);
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (!act[u]) continue;
          dv[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(td, pf[u], dv[u][v], 0, 0, 0);
          dk[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tq, sf[u], dk[u][v], 0, 0, 0);
        }
      }
      raw_barrier_lds();  // dS(qs) complete; every wave done with step qs's Q / dO rows
      if (more) issue_qdo(nxt, qs * 4, qs * 4 + 4);
    }
    dq_step(nstep - 1);  // the last step's dS^T, visible after its barrier
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (kbv[u] && key[u] < N) {
        bf16* row = dq_base + (int64_t)key[u] * ld;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          float a[4] = {dk[u][v][0] * p.scale, dk[u][v][1] * p.scale, dk[u][v][2] * p.scale, dk[u][v][3] * p.scale};
          float w[4] = {dv[u][v][0], dv[u][v][1], dv[u][v][2], dv[u][v][3]};
          store4(row + D + v * 16 + 4 * g, a);
          store4(row + 2 * D + v * 16 + 4 * g, w);
        }
      }
    }
    if (!more) break;
    store_meta(sl ^ 1, l2n, kon);  // slot sl ^ 1's readers (item it - 1) finished long ago
    item = nxt;
  }
}

// ------------------------------------------------------------------ fwd, K/V streaming
// Flash-attention forward for any N (ViT-L/14@336: N = 577 does not fit the whole-K/V kernel
// above).  One 4-wave workgroup per (batch, head, chunk of FA_QC(QPW) queries); two or more
// workgroups share a CU, so one's prologue / epilogue overlaps the others' MFMAs.  The chunk's
// Q rows and then K/V tiles of 64 keys arrive by LDS-DMA (Q slot + a 3-slot ring of 16 KiB
// K|V tiles), every wait a counted vmcnt; one barrier per tile.  Per tile and query block:
// scores key-major (each lane owns a query row), online softmax with a deferred maximum (the
// running max moves, and the output/sum are rescaled, only when a tile's max exceeds it by
// more than FA_THR in log2 units: P <= 2^FA_THR, exact after normalisation), P packed to bf16
// feeding the P.V MFMAs from registers, and the row sum accumulated by one more MFMA against
// a ones fragment (the matrix core sums the same bf16 P the P.V product uses; no VALU adds).
constexpr int FA_W = 4, FA_KT = 64, FA_S = 3, FA_TILE = FA_KT * 128 * 2;
constexpr float FA_THR = 8.0f;

__device__ __forceinline__ void fa_vmcnt(int n) {  // n in {0, 4, 8, 12}
  switch (n) {
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void fa_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// rows row0 .. row0 + 8*npieces - 1 of one 64-wide head slice (row stride ld elements) into a
// lane-linear image (img_off layout); rows >= N read zero.  Pieces j = wave, wave + FA_W, ...
__device__ __forceinline__ void fa_stage(char* img, const bf16* col0, int64_t ld, int row0, int N, int npieces,
                                         int wave, int lane) {
  const int rows = N - row0;
  const uint32_t rec = rows > 0 ? (uint32_t)((int64_t)(rows - 1) * ld * 2 + 128) : 0u;
  const SRsrc rs = make_srsrc(col0 + (int64_t)max(0, min(row0, N - 1)) * ld, rec);
  for (int j = wave; j < npieces; j += FA_W) {
    const int r = 8 * j + (lane >> 3);
    dma16(rs, img + j * 1024, r * (int)ld * 2 + (((lane & 7) ^ (r & 6)) << 4));
  }
}

template <int QPW, bool MASKED, bool Q8 = false>
__global__ __launch_bounds__(FA_W * 64, 2) void attn_fwd_fa(AttnP p, int causal, int nqc, int qbase) {
  constexpr int QC = FA_W * QPW * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qimg = smem;
  char* ring = smem + QC * 128;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int N = p.N, D = p.D, H = p.H;
  const int64_t ld = 3 * (int64_t)D;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);  // the chunks of one (b, h) share an XCD's L2
  const int bh = wid / nqc, qc = wid - bh * nqc;
  const int b = bh / H, h = bh - b * H;
  const int q0 = qbase + qc * QC;
  const int nkt = (N + FA_KT - 1) / FA_KT;
  const bf16* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const float c2 = p.scale * LOG2E;
  int* keyok = (int*)(ring + FA_S * FA_TILE);  // MASKED: [nkt * 64]
  if (MASKED) {  // before any DMA is in flight: the compiler's wait for these loads drains nothing else
    for (int k = t; k < nkt * FA_KT; k += FA_W * 64)
      keyok[k] = (k < N) && (!p.kmask || p.kmask[(int64_t)b * N + k] != 0);
  }
  // prologue: the Q chunk (2*QPW pieces per wave), then K/V tiles 0 .. FA_S - 2 (4 pieces per wave each)
  fa_stage(Qimg, base, ld, q0, N, QC / 8, wave, lane);
  auto issue = [&](int kt) {
    char* slot = ring + (kt % FA_S) * FA_TILE;
    fa_stage(slot, base + D, ld, kt * FA_KT, N, FA_KT / 8, wave, lane);
    fa_stage(slot + FA_TILE / 2, base + 2 * D, ld, kt * FA_KT, N, FA_KT / 8, wave, lane);
  };
  for (int kt = 0; kt < FA_S - 1 && kt < nkt; ++kt) issue(kt);
  fa_vmcnt(4 * (min(FA_S - 1, nkt) - 1));  // the Q chunk and K/V tile 0 landed (this wave's part)
  fa_barrier();
  // this wave's query blocks: w + FA_W * u (interleaved: balanced under causal masking)
  bf16x8 qf[QPW][2];
  bool qv[QPW];
  int qrow[QPW];
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    const int blk = wave + FA_W * u;
    qrow[u] = q0 + blk * 16 + li;
    qv[u] = q0 + blk * 16 < N;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[u][kk] = frag_row(Qimg, blk * 16 + li, kk * 4 + g);
  }
  f32x4 acc[QPW][4], accl[QPW];
  float m[QPW];  // running offset (log2 units) per query row of this lane
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    m[u] = NEG_INF;
    accl[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = bf16x8{(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};

  for (int kt = 0; kt < nkt; ++kt) {
    if (kt > 0) {
      fa_vmcnt(kt + 1 < nkt ? 4 : 0);  // tile kt landed (only tile kt + 1 may still be in flight)
      fa_barrier();                    // ... for every wave; and tile kt - 1's slot is free
    }
    if (kt + FA_S - 1 < nkt) issue(kt + FA_S - 1);
    const char* Kimg = ring + (kt % FA_S) * FA_TILE;
    const char* Vimg = Kimg + FA_TILE / 2;
    const int k0 = kt * FA_KT;
    const int nsteps = min(2, (N - k0 + 31) >> 5);  // 32-key steps holding valid keys
    if constexpr (!MASKED) {
      // Unmasked (vision): straight-line code -- every block computed (rows past N read zero-filled Q),
      // every 32-key step computed (keys past N get P = 0).  The tile's K fragments are read from LDS
      // once and serve every query block, and the P.V products run V-fragment-outer over the blocks'
      // packed P, so each V fragment is read once too: the per-block form re-read both for every block
      // (the compiler cannot merge loads across the rescale branch's ballot) -- 4x the LDS fragment
      // traffic of 8 waves per CU, which co-bounded the tile with the MFMAs.  Same MFMAs, operands and
      // accumulation order per output: bitwise the per-block form's results.
      bf16x8 kfr[4][2];
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) kfr[st][kk] = frag_row(Kimg, st * 16 + li, kk * 4 + g);
      const bool tail = k0 + FA_KT > N;  // wave-uniform: only the last tile holds keys past N
      bf16x8 pfu[QPW][2];
#pragma unroll
      for (int u = 0; u < QPW; ++u) {
        f32x4 sc[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          sc[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            sc[st] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfr[st][kk], qf[u][kk], sc[st], 0, 0, 0);
        }
        if (tail) {
#pragma unroll
          for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (k0 + st * 16 + 4 * g + r >= N) sc[st][r] = NEG_INF;
        }
        // the exponent arguments relative to the current offset first, and the tile's max taken over them:
        // fmaf's results are canonical floats, so the max needs no v_max canonicalisation per MFMA output
        // (64 VALU instructions per tile; the softmax is VALU-issue bound beside the MFMAs)
        const bool first = m[u] == NEG_INF;
        const float off = first ? 0.f : m[u];
        float mt = NEG_INF;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
#pragma unroll
          for (int r = 0; r < 4; ++r) sc[st][r] = fmaf(sc[st][r], c2, -off);
          mt = fmaxf(mt, fmaxf(fmaxf(sc[st][0], sc[st][1]), fmaxf(sc[st][2], sc[st][3])));
        }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        // deferred maximum: move the offset (by d) only on the first tile or when this tile's max exceeds it
        // by > FA_THR; the rescale only when some row of the wave moved (wave-uniform branch, untaken on
        // most tiles)
        const float d = (first || mt > FA_THR) ? mt : 0.f;
        if (__builtin_amdgcn_read_exec() && __any(d != 0.f)) {
          const float f = first ? 0.f : __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[u][v][r] *= f;
#pragma unroll
          for (int r = 0; r < 4; ++r) accl[u][r] *= f;
#pragma unroll
          for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[st][r] -= d;
        }
        m[u] = off + d;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int r = 0; r < 4; ++r) sc[st][r] = __builtin_amdgcn_exp2f(sc[st][r]);
        pfu[u][0] = pack8(sc[0], sc[1]);
        pfu[u][1] = pack8(sc[2], sc[3]);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int u = 0; u < QPW; ++u) accl[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pfu[u][ks], accl[u], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const bf16x8 vt = frag_tr(Vimg, ks * 32, v * 16, lane);
#pragma unroll
          for (int u = 0; u < QPW; ++u)
            acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt, pfu[u][ks], acc[u][v], 0, 0, 0);
        }
      }
      continue;
    }
#pragma unroll
    for (int u = 0; u < QPW; ++u) {
      if constexpr (MASKED) {
        if (!qv[u]) continue;
        if (causal && k0 > q0 + (wave + FA_W * u) * 16 + 15) continue;  // every key follows every query
      }
      f32x4 sc[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        sc[st] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!MASKED || st < 2 * nsteps) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            sc[st] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(Kimg, st * 16 + li, kk * 4 + g), qf[u][kk],
                                                             sc[st], 0, 0, 0);
        }
      }
      float mt = NEG_INF;
      const bool tail = k0 + FA_KT > N;  // wave-uniform: only the last tile holds keys past N
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        if (MASKED || tail) {  // unmasked: no per-element test on the other tiles
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + st * 16 + 4 * g + r;
            bool ok = key < N;
            if (MASKED) ok = ok && keyok[key] && (!causal || key <= qrow[u]);
            if (!ok) sc[st][r] = NEG_INF;
          }
        }
        mt = fmaxf(mt, fmaxf(fmaxf(sc[st][0], sc[st][1]), fmaxf(sc[st][2], sc[st][3])));
      }
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mt2 = mt * c2;
      // deferred maximum: move the offset only when this tile's max exceeds it by > FA_THR
      if constexpr (!MASKED) {  // every tile holds a valid key: mt2 finite; the row's 4 lanes agree
        // the rescale only when some row of the wave moved its offset (a wave-uniform branch: the
        // deferred maximum leaves it untaken on most tiles; 867-893 -> 809-832 us at L/14@336,
        // profiles/r04_attn_fwd_ab.log)
        const float mn = mt2 > m[u] + FA_THR ? fmaxf(m[u], mt2) : m[u];
        if (__builtin_amdgcn_read_exec() && __any(mn != m[u])) {
          const float f = __builtin_amdgcn_exp2f(m[u] - mn);  // 1 unmoved, 0 on the first tile
#pragma unroll
          for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[u][v][r] *= f;
#pragma unroll
          for (int r = 0; r < 4; ++r) accl[u][r] *= f;
        }
        m[u] = mn;
      } else if (__builtin_amdgcn_read_exec() && __any(mt2 > m[u] + FA_THR)) {
        const float mn = fmaxf(m[u], mt2);
        const float f = m[u] == NEG_INF ? 0.f : __builtin_amdgcn_exp2f(m[u] - mn);
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[u][v][r] *= f;
#pragma unroll
        for (int r = 0; r < 4; ++r) accl[u][r] *= f;
        m[u] = mn;
      }
      const float off = m[u] == NEG_INF ? 0.f : m[u];
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[st][r] = __builtin_amdgcn_exp2f(fmaf(sc[st][r], c2, -off));
      bf16x8 pf[2];
      pf[0] = pack8(sc[0], sc[1]);
      pf[1] = pack8(sc[2], sc[3]);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (!MASKED || ks < nsteps) {
          accl[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[ks], accl[u], 0, 0, 0);
#pragma unroll
          for (int v = 0; v < 4; ++v)
            acc[u][v] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(Vimg, ks * 32, v * 16, lane), pf[ks],
                                                                acc[u][v], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    if (!qv[u] || qrow[u] >= N) continue;  // whole rows: the four lanes of a row (g) agree
    const float l = accl[u][0];
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int64_t row = (int64_t)b * N + qrow[u];
    if constexpr (Q8) {
      // the out-projection's MXFP8 operand straight from fp32 O (clipmi_quant_mxfp8's rule): the
      // head's two 32-column blocks are v = 0, 1 and v = 2, 3 of the row's four lanes g
      float w[4][4];
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[v][r] = acc[u][v][r] * inv;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        float am = 0.f;
#pragma unroll
        for (int v = 2 * blk; v < 2 * blk + 2; ++v)
#pragma unroll
          for (int r = 0; r < 4; ++r) am = fmaxf(am, fabsf(w[v][r]));
        am = fmaxf(am, __shfl_xor(am, 16, 64));
        am = fmaxf(am, __shfl_xor(am, 32, 64));
        const int ex = mx_exponent(am);
        const float sc = ldexpf(1.0f, -ex);
        uint8_t* q = p.o8 + row * D + h * 64;
#pragma unroll
        for (int v = 2 * blk; v < 2 * blk + 2; ++v)
          *(uint32_t*)(q + v * 16 + 4 * g) = mx_pack4(w[v][0], w[v][1], w[v][2], w[v][3], sc);
        if (g == 0) p.s8[row * (D >> 5) + 2 * h + blk] = (uint8_t)(ex + 127);
      }
    } else {
      bf16* orow = p.o + row * D + h * 64;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float w[4] = {acc[u][v][0] * inv, acc[u][v][1] * inv, acc[u][v][2] * inv, acc[u][v][3] * inv};
        store4(orow + v * 16 + 4 * g, w);
      }
    }
    if (g == 0) p.lse[((int64_t)b * H + h) * N + qrow[u]] = l > 0.f ? (m[u] + __log2f(l)) * LN2 : NEG_INF;
  }
}

template <int QPW, bool M, bool Q8 = false>
void launch_fwd_fa(const AttnP& p, int causal, hipStream_t s, int qbase = 0, int nq = -1) {
  constexpr int QC = FA_W * QPW * 16;
  const int nkt = (p.N + FA_KT - 1) / FA_KT;
  const size_t lds = (size_t)QC * 128 + FA_S * FA_TILE + (M ? (size_t)nkt * FA_KT * 4 : 0);
  (void)lds_optin((const void*)attn_fwd_fa<QPW, M, Q8>, 160 * 1024);
  const int nqc = ((nq < 0 ? p.N - qbase : nq) + QC - 1) / QC;
  hipLaunchKernelGGL((attn_fwd_fa<QPW, M, Q8>), dim3(p.B * p.H * nqc), dim3(FA_W * 64), lds, s, p, causal, nqc, qbase);
}

template <bool Q8>
int fwd_fa_dispatch_t(const AttnP& p, int causal, hipStream_t s) {
  const bool masked = causal || p.kmask;
  const char* e = getenv("CLIPMI_FA_QPW");  // A/B hook (read per call): 2|4 forces the chunk size
  const int env_qpw = e ? atoi(e) : 0;
  const int qpw = env_qpw == 2 || env_qpw == 4 ? env_qpw : (p.N > 256 ? 4 : 2);
  if (qpw == 4 && !masked && p.N % 256 != 0 && p.N > 256) {
    // unmasked: the whole 256-query chunks in one launch and the remainder in 128-query chunks, so
    // the straight-line block loop computes 640 query rows for N = 577 instead of 768 (L/14@336:
    // 820 -> 776 us; profiles/r04_attn_fwd_ab.log)
    const int full = p.N / 256 * 256;
    launch_fwd_fa<4, false, Q8>(p, causal, s, 0, full);
    launch_fwd_fa<2, false, Q8>(p, causal, s, full, p.N - full);
  } else if (qpw == 4) {  // 256-query chunks: K/V streamed once per 256 queries
    if (masked) launch_fwd_fa<4, true, Q8>(p, causal, s); else launch_fwd_fa<4, false, Q8>(p, causal, s);
  } else {
    if (masked) launch_fwd_fa<2, true, Q8>(p, causal, s); else launch_fwd_fa<2, false, Q8>(p, causal, s);
  }
  return CLIPMI_OK;
}
int fwd_fa_dispatch(const AttnP& p, int causal, hipStream_t s) { return fwd_fa_dispatch_t<false>(p, causal, s); }

// ------------------------------------------------------------------ f32 SIMT path
// 4 lanes per row, 16 head dims each.  K/V (or Q/dO) staged in LDS as fp32 [N][64].
struct AttnF {
  const float* qkv; float* o; float* lse; const int64_t* kmask;
  const float* dout; float* dqkv;
  int B, H, N, D, causal;
  float scale;
};

__device__ __forceinline__ float dot16(const float* a, const float* b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s = fmaf(a[i], b[i], s);
  return s;
}
__device__ __forceinline__ float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}

// Keys (forward, dQ) or queries (dK/dV) are staged through LDS in chunks of F32_CH rows, so any
// N <= ATTN_MAX_N_ANY fits (ViT-L/14@336: N = 577); each pass of 256 rows keeps its running
// state in registers across the chunks.
constexpr int F32_CH = 128;

__global__ __launch_bounds__(1024) void attn_fwd_f32(AttnF p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = (float*)smem;
  float* Vs = Ks + F32_CH * 64;
  int* ok = (int*)(Vs + F32_CH * 64);  // [N]
  const int b = blockIdx.x / p.H, h = blockIdx.x % p.H, N = p.N, D = p.D;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = p.qkv + (int64_t)b * N * ld + h * 64;
  for (int k = threadIdx.x; k < N; k += blockDim.x) ok[k] = !p.kmask || p.kmask[(int64_t)b * N + k] != 0;
  const int sub = threadIdx.x & 3;
  for (int qp = 0; qp < N; qp += 256) {  // the 4 lanes of a row share q
    const int q = qp + (threadIdx.x >> 2);
    const bool qok = q < N;
    float qv[16], acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { qv[i] = qok ? base[(int64_t)q * ld + sub * 16 + i] * p.scale : 0.f; acc[i] = 0.f; }
    float m = NEG_INF, l = 0.f;
    const int kend = qok ? (p.causal ? q + 1 : N) : 0;
    for (int c0 = 0; c0 < N; c0 += F32_CH) {
      const int cn = min(F32_CH, N - c0);
      __syncthreads();  // the previous chunk's readers are done (and ok[] is written)
      for (int i = threadIdx.x; i < cn * 64; i += blockDim.x) {
        const int r = i >> 6, c = i & 63;
        Ks[i] = base[(int64_t)(c0 + r) * ld + D + c];
        Vs[i] = base[(int64_t)(c0 + r) * ld + 2 * D + c];
      }
      __syncthreads();
      for (int k = c0; k < min(kend, c0 + cn); ++k) {
        if (!ok[k]) continue;
        const float* kr = Ks + (k - c0) * 64 + sub * 16;
        const float sc = quad_sum(dot16(qv, kr));
        const float mn = fmaxf(m, sc);
        const float corr = expf(m - mn), e = expf(sc - mn);
        l = l * corr + e;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = acc[i] * corr + e * Vs[(k - c0) * 64 + sub * 16 + i];
        m = mn;
      }
    }
    if (qok) {
      const float inv = l > 0.f ? 1.f / l : 0.f;
      float* orow = p.o + ((int64_t)b * N + q) * D + h * 64 + sub * 16;
#pragma unroll
      for (int i = 0; i < 16; ++i) orow[i] = acc[i] * inv;
      if (sub == 0) p.lse[((int64_t)b * p.H + h) * N + q] = l > 0.f ? m + logf(l) : NEG_INF;
    }
  }
}

__global__ __launch_bounds__(1024) void attn_bwd_f32(AttnF p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* A = (float*)smem;            // dQ pass: K chunk, dK/dV pass: Q chunk
  float* Bm = A + F32_CH * 64;        // dQ pass: V chunk, dK/dV pass: dO chunk
  float* lse = Bm + F32_CH * 64;      // [N]
  float* dlt = lse + p.N;             // [N]
  int* ok = (int*)(dlt + p.N);        // [N]
  const int b = blockIdx.x / p.H, h = blockIdx.x % p.H, N = p.N, D = p.D;
  const int64_t ld = 3 * (int64_t)D;
  const float* base = p.qkv + (int64_t)b * N * ld + h * 64;
  const float* dob = p.dout + (int64_t)b * N * D + h * 64;
  const float* ob = p.o + (int64_t)b * N * D + h * 64;
  float* dq_base = p.dqkv + (int64_t)b * N * ld + h * 64;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    ok[k] = !p.kmask || p.kmask[(int64_t)b * N + k] != 0;
    lse[k] = p.lse[((int64_t)b * p.H + h) * N + k];
    float sm = 0.f;
    for (int c = 0; c < 64; ++c) sm += dob[(int64_t)k * D + c] * ob[(int64_t)k * D + c];
    dlt[k] = sm;
  }
  const int sub = threadIdx.x & 3;
  // dQ rows: keys (K, V) streamed through LDS
  for (int qp = 0; qp < N; qp += 256) {
    const int q = qp + (threadIdx.x >> 2);
    const bool qok = q < N;
    float qv[16], dov[16], dq[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      qv[i] = qok ? base[(int64_t)q * ld + sub * 16 + i] : 0.f;
      dov[i] = qok ? dob[(int64_t)q * D + sub * 16 + i] : 0.f;
      dq[i] = 0.f;
    }
    const int kend = qok ? (p.causal ? q + 1 : N) : 0;
    for (int c0 = 0; c0 < N; c0 += F32_CH) {
      const int cn = min(F32_CH, N - c0);
      __syncthreads();
      for (int i = threadIdx.x; i < cn * 64; i += blockDim.x) {
        const int r = i >> 6, c = i & 63;
        A[i] = base[(int64_t)(c0 + r) * ld + D + c];
        Bm[i] = base[(int64_t)(c0 + r) * ld + 2 * D + c];
      }
      __syncthreads();
      for (int k = c0; k < min(kend, c0 + cn); ++k) {
        if (!ok[k]) continue;
        const float* ka = A + (k - c0) * 64 + sub * 16;
        const float sc = quad_sum(dot16(qv, ka)) * p.scale;
        const float pr = expf(sc - lse[q]);
        const float dp = quad_sum(dot16(dov, Bm + (k - c0) * 64 + sub * 16));
        const float ds = pr * (dp - dlt[q]);
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[i] = fmaf(ds, ka[i], dq[i]);
      }
    }
    if (qok) {
#pragma unroll
      for (int i = 0; i < 16; ++i) dq_base[(int64_t)q * ld + sub * 16 + i] = dq[i] * p.scale;
    }
  }
  // dK, dV rows: queries (Q, dO) streamed through LDS
  for (int kp = 0; kp < N; kp += 256) {
    const int k = kp + (threadIdx.x >> 2);
    const bool kok = k < N && ok[k];
    float kv[16], vv[16], dk[16], dv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      kv[i] = k < N ? base[(int64_t)k * ld + D + sub * 16 + i] : 0.f;
      vv[i] = k < N ? base[(int64_t)k * ld + 2 * D + sub * 16 + i] : 0.f;
      dk[i] = 0.f; dv[i] = 0.f;
    }
    for (int c0 = 0; c0 < N; c0 += F32_CH) {
      const int cn = min(F32_CH, N - c0);
      __syncthreads();
      for (int i = threadIdx.x; i < cn * 64; i += blockDim.x) {
        const int r = i >> 6, c = i & 63;
        A[i] = base[(int64_t)(c0 + r) * ld + c];
        Bm[i] = dob[(int64_t)(c0 + r) * D + c];
      }
      __syncthreads();
      if (!kok) continue;
      for (int q = max(c0, p.causal ? k : 0); q < c0 + cn; ++q) {
        const float* qa = A + (q - c0) * 64 + sub * 16;
        const float* da = Bm + (q - c0) * 64 + sub * 16;
        const float sc = quad_sum(dot16(kv, qa)) * p.scale;
        const float pr = expf(sc - lse[q]);
        const float dp = quad_sum(dot16(vv, da));
        const float ds = pr * (dp - dlt[q]);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dv[i] = fmaf(pr, da[i], dv[i]);
          dk[i] = fmaf(ds, qa[i], dk[i]);
        }
      }
    }
    if (k < N) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dq_base[(int64_t)k * ld + D + sub * 16 + i] = kok ? dk[i] * p.scale : 0.f;
        dq_base[(int64_t)k * ld + 2 * D + sub * 16 + i] = kok ? dv[i] : 0.f;
      }
    }
  }
}

template <int NKT, bool M>
void launch_fwd_pf(const AttnP& p, int causal, hipStream_t s) {
  constexpr int NPAD = NKT * 16;
  constexpr size_t lds = 4 * (size_t)NPAD * 128 + 2 * NPAD * sizeof(int);
  const int nitems = p.B * p.H;
  const int per_cu = (int)std::min<size_t>(2, (160 * 1024) / lds);
  const int grid = std::min(nitems, 256 * per_cu);
  // 16 waves (one query block each, 4 per SIMD) where one workgroup fills the CU and the blocks
  // need more than 8 waves; CLIPMI_ATTN_FWD_NW=8 selects the 8-wave form (A/B hook, read per call)
  const char* e = getenv("CLIPMI_ATTN_FWD_NW");
  const bool w16 = (e ? atoi(e) : 16) == 16 && NKT > 8 && NKT <= 16 && per_cu == 1;
  if constexpr (NKT > 8 && NKT <= 16) {  // NKT = 18 (L/14) spills at 128 registers
    if (w16) {
      (void)lds_optin((const void*)attn_fwd_pf<NKT, M, 16>, (int)lds);
      hipLaunchKernelGGL((attn_fwd_pf<NKT, M, 16>), dim3(grid), dim3(1024), lds, s, p, causal, nitems);
      return;
    }
  }
  (void)lds_optin((const void*)attn_fwd_pf<NKT, M>, (int)lds);
  hipLaunchKernelGGL((attn_fwd_pf<NKT, M>), dim3(grid), dim3(512), lds, s, p, causal, nitems);
}

template <bool M>
int fwd_dispatch(const AttnP& p, int causal, hipStream_t s) {
  const int nkt = ((p.N + 31) & ~31) / 16;
  switch (nkt) {
    case 2: launch_fwd_pf<2, M>(p, causal, s); return CLIPMI_OK;
    case 4: launch_fwd_pf<4, M>(p, causal, s); return CLIPMI_OK;
    case 6: launch_fwd_pf<6, M>(p, causal, s); return CLIPMI_OK;
    case 8: launch_fwd_pf<8, M>(p, causal, s); return CLIPMI_OK;
    case 10: launch_fwd_pf<10, M>(p, causal, s); return CLIPMI_OK;
    case 12: launch_fwd_pf<12, M>(p, causal, s); return CLIPMI_OK;
    case 14: launch_fwd_pf<14, M>(p, causal, s); return CLIPMI_OK;
    case 16: launch_fwd_pf<16, M>(p, causal, s); return CLIPMI_OK;
    case 18: launch_fwd_pf<18, M>(p, causal, s); return CLIPMI_OK;  // ViT-L/14 at 224: N = 257
    default: return clipmi_invalid("attention: N must be <= 288");
  }
}


template <bool C, int NW, int NBM = (NW >= 16 ? 1 : 2)>
void launch_bwd_pf(const AttnP& p, hipStream_t s) {
  const int npad = (p.N + 31) & ~31;
  const size_t lds = 5 * (size_t)npad * 128 + 6 * (size_t)npad * 4;
  (void)lds_optin((const void*)attn_bwd_pf<C, NW, NBM>, 160 * 1024);
  const int nitems = p.B * p.H;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
  const int grid = std::min(nitems, 256 * per_cu);
  hipLaunchKernelGGL((attn_bwd_pf<C, NW, NBM>), dim3(grid), dim3(NW * 64), lds, s, p, nitems);
}
template <bool C, int NW, int NKC>
void launch_bwd_sp(const AttnP& p, hipStream_t s) {
  constexpr size_t lds = 5 * (size_t)NKC * 32 * 128 + 6 * (size_t)NKC * 32 * 4;
  static_assert(lds <= 160 * 1024, "attn_bwd_sp: LDS");
  (void)lds_optin((const void*)attn_bwd_sp<C, NW, NKC>, (int)lds);
  const int nitems = p.B * p.H;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / lds));
  const int grid = std::min(nitems, 256 * per_cu);
  hipLaunchKernelGGL((attn_bwd_sp<C, NW, NKC>), dim3(grid), dim3(NW * 64), lds, s, p, nitems);
}
template <bool C>
int bwd_sp_dispatch(const AttnP& p, hipStream_t s) {
  switch ((p.N + 31) >> 5) {  // 8 waves (ViT-B/16: N = 197, 7 steps)
    case 5: launch_bwd_sp<C, 8, 5>(p, s); return CLIPMI_OK;
    case 6: launch_bwd_sp<C, 8, 6>(p, s); return CLIPMI_OK;
    case 7: launch_bwd_sp<C, 8, 7>(p, s); return CLIPMI_OK;
    default: return clipmi_invalid("attn_bwd_sp: N must be in (128, 224]");
  }
}
// the single-pass backward for 128 < N <= 224 with CLIPMI_ATTN_BWD_SP=1 (A/B hook, read per call).
// Not the default: at ViT-B/16 (N = 197, B = 1024) it measured 912-976 us against attn_bwd_pf's
// 889-926, and 938-981 vs 884-896 with dQ one step late (profiles/r03_attn_bwd_single_pass_ab.log):
// the per-step barrier and the dQ reads cost more than the recomputation they remove.  (Its 4-wave form for the
// text tower, N = 77 with the causal mask, spilled at the 256 registers two workgroups per CU leave.)
static bool use_bwd_sp(int N) {
  if (N <= 128 || N > 224) return false;
  const char* e = getenv("CLIPMI_ATTN_BWD_SP");
  return e && atoi(e) != 0;
}

// 4 waves per workgroup for N <= 128 (text: 5 blocks of 16 rows), else 8; each wave owns at
// most 2 key blocks and 2 query blocks.
int bwd_pf_dispatch(const AttnP& p, int causal, hipStream_t s) {
  if (use_bwd_sp(p.N)) return causal ? bwd_sp_dispatch<true>(p, s) : bwd_sp_dispatch<false>(p, s);
  // CLIPMI_ATTN_BWD_NW=16 (A/B hook, read per call): one block per wave, 4 waves per SIMD.  Measured
  // 3-5 % slower than 8 waves at N = 197 (profiles/r02_attn_waves_ab.log): this backward is bound by
  // its LDS fragment traffic (each wave re-reads the Q/dO and K/V fragments of every step), which
  // two blocks per wave share and one block per wave does not
  const char* e = getenv("CLIPMI_ATTN_BWD_NW");
  const int nw = e ? atoi(e) : 8;
#ifdef CLIPMI_GEMM_EXPERIMENTS  // 4 waves x 4 blocks (NPAD <= 256 threads): 1283 vs 880 us, experiments build only
  if (nw == 4 && !causal && p.N > 128 && p.N <= 224) {
    launch_bwd_pf<false, 4, 4>(p, s);
    return CLIPMI_OK;
  }
#endif
  if (p.N <= 128) {
    if (causal) launch_bwd_pf<true, 4>(p, s); else launch_bwd_pf<false, 4>(p, s);
  } else if (nw == 16 && p.N <= 256) {
    if (causal) launch_bwd_pf<true, 16>(p, s); else launch_bwd_pf<false, 16>(p, s);
  } else {
    if (causal) launch_bwd_pf<true, 8>(p, s); else launch_bwd_pf<false, 8>(p, s);
  }
  return CLIPMI_OK;
}
}  // namespace

// attention_mask: int64 [B, N] key-padding mask (1 = keep) or NULL; causal: text tower.
// bf16 forward kernel choice: the K/V-streaming flash kernel for N > ATTN_MAX_N (and for every N
// when CLIPMI_ATTN_FA=1), else the whole-K/V persistent kernel
static bool use_fa(int N) {
  if (N > ATTN_MAX_N) return true;
  const char* e = getenv("CLIPMI_ATTN_FA");  // read per call: tests and benches switch it at run time
  return e && atoi(e) == 1;
}

extern "C" int clipmi_attention_fwd(void* stream, int dtype, const void* qkv, void* o, float* lse,
                                    const int64_t* attention_mask, int causal, int B, int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1 && N <= ATTN_MAX_N_ANY, "N must be in [1, 4096]");
  if (B == 0) return CLIPMI_OK;
  const int npad = (N + 31) & ~31;
  // algorithmic FLOPs: QK^T and PV over the padded key range, B*H heads
  const double flops = 4.0 * B * H * (double)N * npad * 64;
  if (dtype == CLIPMI_BF16) {
    AttnP p{(const bf16*)qkv, (bf16*)o, lse, attention_mask, nullptr, nullptr, B, H, N, D, 0.125f};
    ProfScope ps(s, "attn_fwd", flops);
    if (use_fa(N)) CLIPMI_TRY(fwd_fa_dispatch(p, causal, s));
    else CLIPMI_TRY((causal || attention_mask) ? fwd_dispatch<true>(p, causal, s) : fwd_dispatch<false>(p, causal, s));
    ps.finish("attn_fwd", flops);
  } else {
    AttnF p{(const float*)qkv, (float*)o, lse, attention_mask, nullptr, nullptr, B, H, N, D, causal, 0.125f};
    size_t lds = (size_t)F32_CH * 64 * 4 * 2 + (size_t)N * 4;
    CLIPMI_HIP(lds_optin((const void*)attn_fwd_f32, 160 * 1024));
    hipLaunchKernelGGL(attn_fwd_f32, dim3(B * H), dim3(1024), lds, s, p);
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// The flash forward with its output written as MXFP8 (the fp8 towers' out-projection operand): o8
// e4m3 [B*N, D], s8 E8M0 [B*N, D/32], quantised from the fp32 O by clipmi_quant_mxfp8's rule.
extern "C" int clipmi_attention_fwd_mxfp8(void* stream, const void* qkv, uint8_t* o8, uint8_t* s8, float* lse,
                                          const int64_t* attention_mask, int causal, int B, int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1 && N <= ATTN_MAX_N_ANY, "N must be in [1, 4096]");
  CLIPMI_REQUIRE(qkv && o8 && s8 && lse, "operands");
  CLIPMI_REQUIRE(((uintptr_t)o8 & 3) == 0, "o8 must be 4-byte aligned (the e4m3 rows go out as 32-bit stores)");
  if (B == 0) return CLIPMI_OK;
  AttnP p{(const bf16*)qkv, nullptr, lse, attention_mask, nullptr, nullptr, B, H, N, D, 0.125f};
  p.o8 = o8;
  p.s8 = s8;
  const int npad = (N + 31) & ~31;
  const double flops = 4.0 * B * H * (double)N * npad * 64;
  ProfScope ps(s, "attn_fwd", flops);
  CLIPMI_TRY(fwd_fa_dispatch_t<true>(p, causal, s));
  ps.finish("attn_fwd", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

extern "C" int clipmi_attention_bwd(void* stream, int dtype, const void* qkv, const void* o, const float* lse,
                                    const void* dout, void* dqkv, const int64_t* attention_mask, int causal,
                                    int B, int H, int N, int D) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(D == H * 64, "head_dim must be 64");
  CLIPMI_REQUIRE(N >= 1 && N <= ATTN_MAX_N_ANY, "N must be in [1, 4096]");
  if (B == 0) return CLIPMI_OK;
  if (dtype == CLIPMI_BF16) {
    AttnP p{(const bf16*)qkv, (bf16*)o, (float*)lse, attention_mask, (const bf16*)dout, (bf16*)dqkv, B, H, N, D, 0.125f};
#ifdef CLIPMI_ATTN_STAMPS
    p.dbg = cmg::gemm_stamp_buffer();
#endif
    const int npad = (N + 31) & ~31;
    size_t lds = (size_t)npad * 128 * 2 + (size_t)npad * 12;
    CLIPMI_HIP(lds_optin((const void*)attn_bwd_mfma<true>, 160 * 1024));
    CLIPMI_HIP(lds_optin((const void*)attn_bwd_mfma<false>, 160 * 1024));
    const double flops = 10.0 * B * H * (double)N * npad * 64;
    ProfScope ps(s, nullptr, flops);
    if (5 * (size_t)npad * 128 + 6 * (size_t)npad * 4 <= 160 * 1024) {  // N <= 224: prefetching kernel
      CLIPMI_TRY(bwd_pf_dispatch(p, causal, s));
    } else if (N > ATTN_MAX_N) {  // streamed chunks (ViT-L/14@336)
      const size_t slds = 2 * (size_t)ST_CH * 128 + (size_t)npad * 12;
      CLIPMI_HIP(lds_optin((const void*)attn_bwd_stream<true>, 160 * 1024));
      CLIPMI_HIP(lds_optin((const void*)attn_bwd_stream<false>, 160 * 1024));
      if (causal) hipLaunchKernelGGL(attn_bwd_stream<true>, dim3(B * H), dim3(512), slds, s, p);
      else hipLaunchKernelGGL(attn_bwd_stream<false>, dim3(B * H), dim3(512), slds, s, p);
    } else if (causal) {
      hipLaunchKernelGGL(attn_bwd_mfma<true>, dim3(B * H), dim3(512), lds, s, p);
    } else {
      hipLaunchKernelGGL(attn_bwd_mfma<false>, dim3(B * H), dim3(512), lds, s, p);
    }
    ps.finish("attn_bwd", flops);
  } else {
    AttnF p{(const float*)qkv, (float*)o, (float*)lse, attention_mask, (const float*)dout, (float*)dqkv, B, H, N, D, causal, 0.125f};
    size_t lds = (size_t)F32_CH * 64 * 4 * 2 + (size_t)N * 12;
    CLIPMI_HIP(lds_optin((const void*)attn_bwd_f32, 160 * 1024));
    hipLaunchKernelGGL(attn_bwd_f32, dim3(B * H), dim3(1024), lds, s, p);
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
