// MFMA GEMM for gfx950 with fused epilogues.
//
// Replaces every nn.Linear on the hot path (forward, dgrad and wgrad):
//   [HF] modeling_clip.py:313-315,332 (q/k/v/out_proj), :348-350 (fc1/fc2),
//   adapter/clip_adapter.py:19-21,146-148 (adapter down/up), model_m.py:103,123 (projections).
//
// Design (bf16 path):
//   * 128x128 output tile per 256-thread workgroup, 4 waves in 2x2, each wave 64x64 =
//     4x4 tiles of v_mfma_f32_16x16x32_bf16, fp32 accumulators (64 VGPRs).
//   * K step 64, register-staged global->LDS copy (16 B per lane), two LDS buffers,
//     one barrier per K step; the next tile's global loads are in flight while the
//     current tile's MFMAs run.
//   * Either operand may be k-major ([rows][K], the forward's x and W) or row-major in
//     k ([K][rows], the dgrad's W and both wgrad operands).  k-major tiles are read with
//     ds_read_b128, the other layout with ds_read_b64_tr_b16 (hardware transpose), so
//     backward GEMMs need no transpose pass over HBM.
//   * LDS images are XOR-swizzled (checked conflict-free for the reads and the
//     b128 writes against the gfx950 bank rules, tools/lds_banks.py).
//   * Operands are swapped in the MFMA (acc = W-tile x X-tile) so each lane ends with 4
//     consecutive output columns: 8-byte bf16 / 16-byte fp32 epilogue stores.
//   * Epilogue fuses bias, quick_gelu / gelu_erf (and their derivatives for dgrad),
//     residual add, accumulate-into-C and pre-activation store.
//   * blockIdx is remapped XCD-aware so neighbouring tiles share an XCD's L2.
//   * split-K (wgrad, K = tokens) writes fp32 partial slabs, summed by a reduce kernel.
// f32 path: exact-f32 LDS-tiled SIMT kernel with the same epilogue (parity mode).
#include "common.h"
#include "internal.h"
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <cstdlib>

#include "gemm_common.h"

namespace {
using namespace cmg;

template <bool AK, bool BKM, typename OutT, int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_bf16_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tile = xcd_remap(blockIdx.x, p.ntiles);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  Stager<AK> sa;
  Stager<BKM> sb;
  sa.init((const bf16*)p.A, p.lda, m0, p.M, t);
  sb.init((const bf16*)p.B, p.ldb, n0, p.N, t);

  // LDS: [buf][A 16KB | B 16KB]
#define LDSA(b) (smem + (b) * 32768)
#define LDSB(b) (smem + (b) * 32768 + 16384)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  if (nk > 0) {
    sa.load(ra, kbeg, p.lda, kend - kbeg);
    sb.load(rb, kbeg, p.ldb, kend - kbeg);
    sa.store(LDSA(0), ra);
    sb.store(LDSB(0), rb);
  }
  __syncthreads();

  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    const bool more = it + 1 < nk;
    if (more) {
      const int k1 = kbeg + (it + 1) * BK;
      sa.load(ra, k1, p.lda, kend - k1);
      sb.load(rb, k1, p.ldb, kend - k1);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<AK>(LDSA(cur), wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<BKM>(LDSB(cur), wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(LDSA(cur ^ 1), ra);
      sb.store(LDSB(cur ^ 1), rb);
    }
    __syncthreads();
  }

#undef LDSA
#undef LDSB
  // acc[i][j][r] = C[m0 + wm*64 + i*16 + (lane&15)][n0 + wn*64 + j*16 + (lane>>4)*4 + r]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
      if (n >= p.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (p.ws) {
        st4(p.ws + (int64_t)blockIdx.y * p.M * p.N + (int64_t)m * p.N + n, v, min(4, p.N - n), p.vec && n + 4 <= p.N);
      } else {
        epilogue4<OutT, EPI>(p, m, n, v);
      }
    }
  }
}

template <bool AK, bool BKM, typename OutT, int EPI, bool BIASGRAD, int VAR = 0>
__global__ __launch_bounds__(NT2, 1) void gemm256_kernel(GemmP p, float* bias_grad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  // 1-D grid over (split, tile), XCD-aware over all of it: an XCD walks a contiguous run of
  // tiles of one k-slab, so that slab's A and B panels are fetched into its L2 once
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int kz = wid / p.ntiles, tile = wid - kz * p.ntiles;
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BT, n0 = tn * BT;
  const int kbeg = kz * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;
  const int Kv = kend;  // rows/cols past the split end read as zero

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[8];
  const bool do_bias = BIASGRAD && tn == 0 && wn == 0;
  if (BIASGRAD) {
#pragma unroll
    for (int i = 0; i < 8; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = bf16x8{(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};

#define IMG_A(b) (smem + (b) * 65536)
#define IMG_B(b) (smem + (b) * 65536 + 32768)
  if (nk > 0) {
    if constexpr (VAR == 3) {
      const SRsrc ra = srsrc256<AK>(A, p.lda, m0, p.M, kbeg, Kv), rb = srsrc256<BKM>(B, p.ldb, n0, p.N, kbeg, Kv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        stage256_one<AK>(IMG_A(0), ra, p.lda, wave, lane, i);
        stage256_one<BKM>(IMG_B(0), rb, p.ldb, wave, lane, i);
      }
    } else {
      stage256<AK>(IMG_A(0), A, p.lda, m0, p.M, kbeg, Kv, wave, lane);
      stage256<BKM>(IMG_B(0), B, p.ldb, n0, p.N, kbeg, Kv, wave, lane);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const int cur = it & 1;
    const bool more = it + 1 < nk;
    const int k1 = kbeg + (it + 1) * BK;
    if (VAR == 0 && more) {
      stage256<AK>(IMG_A(cur ^ 1), A, p.lda, m0, p.M, k1, Kv, wave, lane);
      stage256<BKM>(IMG_B(cur ^ 1), B, p.ldb, n0, p.N, k1, Kv, wave, lane);
    }
    typedef typename std::conditional<VAR == 3, SRsrc, __amdgpu_buffer_rsrc_t>::type RS;
    RS ra, rb;
    if constexpr (VAR == 3) {
      ra = srsrc256<AK>(A, p.lda, m0, p.M, more ? k1 : kbeg, Kv);
      rb = srsrc256<BKM>(B, p.ldb, n0, p.N, more ? k1 : kbeg, Kv);
    } else if constexpr (VAR != 0) {
      ra = rsrc256<AK>(A, p.lda, m0, p.M, more ? k1 : kbeg, Kv);
      rb = rsrc256<BKM>(B, p.ldb, n0, p.N, more ? k1 : kbeg, Kv);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = read_frag256<AK>(IMG_A(cur), wm * 128 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag256<BKM>(IMG_B(cur), wn * 64 + j * 16, kk, lane);
      if (VAR >= 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (VAR != 0 && kk == 0 && more) {  // one DMA per 4 MFMAs across the first half of the step
          if (i < 4) stage256_one<AK>(IMG_A(cur ^ 1), ra, p.lda, wave, lane, i);
          else stage256_one<BKM>(IMG_B(cur ^ 1), rb, p.ldb, wave, lane, i - 4);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
      if (BIASGRAD && do_bias) {
#pragma unroll
        for (int i = 0; i < 8; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fa[i], accb[i], 0, 0, 0);
      }
      if (VAR >= 2) __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#undef IMG_A
#undef IMG_B

  if (BIASGRAD && do_bias && lane < 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + lane;
      if (m < p.M) {
        if (p.bws) p.bws[(int64_t)kz * p.M + m] = accb[i][0];  // summed in split order afterwards
        else atomicAdd(bias_grad + m, accb[i][0]);             // one split: one add per element
      }
    }
  }
  finish256<OutT, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane, kz);
}

// ------------------------------------------------------------------ ping-pong 256x256 path
// Same 256x256 tile and 8-wave (2 along M x 4 along N) decomposition as gemm256_kernel, with
// a schedule built so the matrix cores never wait on LDS or on the DMA queue:
//  * k advances in stages of 32 through a ring of PP_S = 5 LDS stages (5 x 32 KiB = all
//    160 KiB); stage s + PP_D is DMA'd while stage s is consumed (PP_D = 3 stages of
//    prefetch, ~1.5 k-steps of the old schedule), waited for with a counted vmcnt, never 0.
//  * each stage is two phases of 16 MFMAs per wave (m-half 0 / 1 of the wave's 128 rows x
//    all 64 columns, k 32).  A phase is [load section: its fragments from LDS + 2 DMA issues
//    (+ the counted wait)] barrier [MFMA section] barrier.
//  * the 4 waves of M-half 1 start one barrier late, so on every SIMD (waves w and w + 4 share
//    one) one wave runs its MFMA section while the other runs its load section: the two
//    groups ping-pong between the matrix core and the LDS/DMA path.
// Ring safety (intervals = spans between barriers; group 0's phase q is intervals 2q (load)
// and 2q + 1 (MFMA), group 1's is 2q + 1 and 2q + 2): stage s + 3 is DMA'd in phases 2s, 2s + 1
// into the slot of stage s - 2, whose last reads (group 1, phase 2s - 3, interval 4s - 5) were
// retired by that group's lgkmcnt wait two intervals before the first overwrite (interval 4s).
// Stage s + 1 is waited for (vmcnt) in both groups' load sections of phase 2s + 1, before the
// barrier that precedes its first read (group 0, phase 2s + 2).
// LDS images per stage: A at +0, B at +16 KiB.  k-major operand: [256 rows][32 k] = 64-B rows,
// 16-B chunk c of row r at c ^ ((r >> 1) & 3); k-row operand: two [32 k][128] halves of 256-B
// rows with gemm128's mimg swizzle.  Both conflict-free (tools/lds_banks.py).
constexpr int PP_S = 5, PP_D = 3, PP_STAGE = 32768;

__device__ __forceinline__ int kimg32_off(int r, int c) { return r * 64 + ((c ^ (r >> 1)) & 3) * 16; }

// Two DMA wave-instructions (i = 0, 1) of this wave for one operand of one stage.
template <bool KMAJ>
__device__ __forceinline__ void stage_pp(char* img, const bf16* X, int64_t ld, int row0, int R, int k0, int K,
                                         int wave, int lane) {
  const bf16* base;
  uint32_t rec;
  if (KMAJ) {
    const int rows = min(BT, R - row0);
    base = X + (int64_t)row0 * ld + k0;
    rec = rows > 0 ? (uint32_t)((int64_t)(rows - 1) * ld * 2 + 64) : 0u;
  } else {
    const int krows = min(32, K - k0);
    const int cols = min(BT, R - row0);
    base = X + (int64_t)k0 * ld + row0;
    rec = krows > 0 ? (uint32_t)((int64_t)(krows - 1) * ld * 2 + (int64_t)cols * 2) : 0u;
  }
  const SRsrc rs = make_srsrc(base, rec);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;  // 0..15, 1 KiB each
    if (KMAJ) {
      const int r = 16 * j + (lane >> 2);
      const int c = (lane & 3) ^ ((r >> 1) & 3);
      dma16(rs, img + j * 1024, (int)((int64_t)r * ld * 2 + c * 16));
    } else {
      const int half = j >> 3;
      const int kr = 4 * (j & 7) + (lane >> 4);
      const int c = (lane & 15) ^ mimg_swz(kr);
      dma16(rs, img + half * 8192 + (j & 7) * 1024, (int)((int64_t)kr * ld * 2 + (half * 128 + c * 8) * 2));
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag_pp(const char* img, int rb, int lane) {
  if (KMAJ) return *LDS_PTR(const bf16x8, img + kimg32_off(rb + (lane & 15), lane >> 4));
  return read_frag<false>(img + (rb >> 7) * 8192, rb & 127, 0, lane);
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// wait until at most n of this wave's DMAs are outstanding (n even, 0..8)
__device__ __forceinline__ void pp_vmcnt(int n) {
  switch (n) {
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// PPV (schedule experiments, 0 = production): bit 0 one phase of 32 MFMAs per stage instead
// of two of 16; bit 1 no ping-pong (both groups in lock-step); bit 2 no s_setprio.
template <bool AK, bool BKM, typename OutT, int EPI, bool BIASGRAD, int PPV = 0>
__global__ __launch_bounds__(NT2, 1) void gemm_pp_kernel(GemmP p, float* bias_grad) {
  constexpr int NPH = (PPV & 1) ? 1 : 2, MPH = 8 / NPH;
  constexpr bool PINGPONG = !(PPV & 2);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  // 1-D grid over (split, tile), XCD-aware over all of it: an XCD walks a contiguous run of
  // tiles of one k-slab, so that slab's A and B panels are fetched into its L2 once
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int kz = wid / p.ntiles, tile = wid - kz * p.ntiles;
  int tm, tn;
  tile_coords(p, tile, tm, tn);
  const int m0 = tm * BT, n0 = tn * BT;
  const int kbeg = kz * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int ns = (kend - kbeg + 31) / 32;
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient (wgrad, n-tile 0): wave wn sums m-fragments wn and 4 + wn
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bool do_bias = BIASGRAD && tn == 0;
  const bf16x8 ones = bf16x8{(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};

  auto slot = [&](int st) { return smem + (st % PP_S) * PP_STAGE; };
  // first-round stagger: half the workgroups of every XCD start later, and since each CU
  // takes its next workgroup when the previous one ends, the offset persists: one half's
  // epilogue stores run beside the other half's main loop instead of all CUs storing at once
  if (p.stagger > 0 && (int)blockIdx.x < p.first_round && ((blockIdx.x >> 3) & 1)) {
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  // prologue: stages 0 .. PP_D - 1
#pragma unroll
  for (int st = 0; st < PP_D; ++st) {
    if (st < ns) {
      stage_pp<AK>(slot(st), A, p.lda, m0, p.M, kbeg + st * 32, kend, wave, lane);
      stage_pp<BKM>(slot(st) + 16384, B, p.ldb, n0, p.N, kbeg + st * 32, kend, wave, lane);
    }
  }
  pp_vmcnt(4 * (min(PP_D, ns) - 1));  // stage 0 landed
  pp_barrier();
  if (PINGPONG && wm == 1) pp_barrier();

  for (int st = 0; st < ns; ++st) {
    const char* img = slot(st);
    const bool issue = st + PP_D < ns;
    const int kn = kbeg + (st + PP_D) * 32;
    bf16x8 fb[4];  // the stage's B fragments, read in the first phase
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      // ---- load section
      bf16x8 fa[MPH];
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = read_frag_pp<BKM>(img + 16384, wn * 64 + j * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < MPH; ++i) fa[i] = read_frag_pp<AK>(img, wm * 128 + (ph * MPH + i) * 16, lane);
      constexpr bool DMA_IN_MFMA = PPV & 16;  // issue the DMAs between this phase's MFMAs
      if (issue && !DMA_IN_MFMA) {
        if (NPH == 1 || ph == 0) stage_pp<AK>(slot(st + PP_D), A, p.lda, m0, p.M, kn, kend, wave, lane);
        if (NPH == 1 || ph == 1) stage_pp<BKM>(slot(st + PP_D) + 16384, B, p.ldb, n0, p.N, kn, kend, wave, lane);
      }
      if (ph == NPH - 1) {  // stage st + 1 landed (with DMA_IN_MFMA this phase's own 2 are not issued yet)
        if (DMA_IN_MFMA && issue) pp_vmcnt(4 * (PP_D - 1) - 2);
        else pp_vmcnt(4 * max(0, min(PP_D - 1, ns - st - 2)));
      }
      pp_barrier();
      // ---- MFMA section
      if (!(PPV & 4)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MPH; ++i) {
        if (DMA_IN_MFMA && issue && i == MPH / 2) {
          if (NPH == 1 || ph == 0) stage_pp<AK>(slot(st + PP_D), A, p.lda, m0, p.M, kn, kend, wave, lane);
          if (NPH == 1 || ph == 1) stage_pp<BKM>(slot(st + PP_D) + 16384, B, p.ldb, n0, p.N, kn, kend, wave, lane);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[ph * MPH + i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[ph * MPH + i][j], 0, 0, 0);
      }
      if (BIASGRAD && do_bias) {
#pragma unroll
        for (int h = 0; h < MPH / 4; ++h) {
          const bf16x8 f = wn == 0 ? fa[h * 4] : wn == 1 ? fa[h * 4 + 1] : wn == 2 ? fa[h * 4 + 2] : fa[h * 4 + 3];
          accb[ph + h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, f, accb[ph + h], 0, 0, 0);
        }
      }
      if (!(PPV & 4)) __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
  }
  if (PINGPONG && wm == 0) pp_barrier();  // pairs with group 1's leading barrier

  if (BIASGRAD && do_bias && lane < 16) {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
      const int m = m0 + wm * 128 + (mh * 4 + wn) * 16 + lane;
      if (m < p.M) {
        if (p.bws) p.bws[(int64_t)kz * p.M + m] = accb[mh][0];  // summed in split order afterwards
        else atomicAdd(bias_grad + m, accb[mh][0]);              // one split: one add per element
      }
    }
  }
  if constexpr (PPV & 8) {  // timing experiment: main loop only, results kept live, nothing stored
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j][0]), "v"(acc[i][j][1]), "v"(acc[i][j][2]), "v"(acc[i][j][3]));
    return;
  }
  // bf16 stores through LDS, whole 128-B rows per instruction (the ring is idle: every wave has
  // passed its last MFMA section and the trailing barrier above pairs the two groups).  fc1's
  // pre-activation still goes out directly, beside its gelu math.  PPV & 64 disables it (A/B).
  constexpr bool STAGE = (PPV & 32) || (!(PPV & 64) && EPI >= 0);
  finish256<OutT, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane, kz, STAGE ? smem + wave * 16384 : nullptr);
}

// ------------------------------------------------------------------ MXFP8 (config 5)
// Block-scaled fp8 GEMM for the frozen ViT-L/14@336 towers (BASELINE config 5): both operands
// OCP e4m3 (k-major, [rows][K] bytes) with one E8M0 scale per 32-element k-block of a row
// ([rows][K/32] bytes: the OCP MX layout), on v_mfma_scale_f32_32x32x64_f8f6f4 (twice the bf16
// MFMA rate; the hardware applies both operands' block scales inside the MFMA).  Epilogues: the
// bf16 kernels' finish256 after a register-layout conversion, or MXFP8 output (epilogue_q8).

// Operand map of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3), measured with exact data
// (tools/probes/mfma_f8f6f4_32x32_layout.hip, profiles/r02_f8f6f4_32x32_layout.txt): lane l holds
// row l & 31; its bytes 0-15 belong to k-block 0 and bytes 16-31 to k-block 1 (32 k each), the two
// lane halves h = l >> 5 splitting each block, and its scale operand is the E8M0 scale of row l & 31,
// block h.  So with k 16h .. 16h+15 in bytes 0-15 and k 32 + 16h .. in bytes 16-31 (the same map for
// both operands), one 64-k ring stage is exactly one MFMA k-step.  (16x16x128 would consume two
// stages per MFMA, halving the ring's prefetch depth: measured at the bf16 kernel's rate only.)
// fp8 stage images use the swizzle chunk ^ ((row >> 2) & 3), conflict-free for this 32-row read.
__device__ __forceinline__ int kimg8_off(int r, int c) { return r * 64 + ((c ^ (r >> 2)) & 3) * 16; }

__device__ __forceinline__ i32x8 read_frag8(const char* img, int rb, int lane) {
  const int r = rb + (lane & 31), h = lane >> 5;
  const i32x4 a = *LDS_PTR(const i32x4, img + kimg8_off(r, h));
  const i32x4 b = *LDS_PTR(const i32x4, img + kimg8_off(r, 2 + h));
  return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// stage_pp<true> for fp8 rows (64 B = 64 k per row and stage) with the fp8 swizzle
__device__ __forceinline__ void stage_pp8(char* img, const uint8_t* X, int64_t ld, int row0, int R, int k0, int wave,
                                          int lane) {
  const int rows = min(BT, R - row0);
  const SRsrc rs = make_srsrc(X + (int64_t)row0 * ld + k0, rows > 0 ? (uint32_t)((int64_t)(rows - 1) * ld + 64) : 0u);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;  // 0..15, 1 KiB = 16 rows each
    const int r = 16 * j + (lane >> 2);
    const int c = (lane & 3) ^ ((r >> 2) & 3);
    dma16(rs, img + j * 1024, (int)((int64_t)r * ld + c * 16));
  }
}

// Async per-lane dword load (vmcnt-counted like the stage DMAs, so the ring's counted waits
// retire it; the compiler does not track it: consumers read it only through asm volatile after
// such a wait, see gemm_fp8_kernel).
__device__ __forceinline__ int ld_dword_async(const SRsrc& r, int voff) {
  int v;
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(r.v) : "memory");
  return v;
}
__device__ __forceinline__ int shr_after_wait(int w, int sh) {
  int o;
  asm volatile("v_lshrrev_b32 %0, %1, %2" : "=v"(o) : "v"(sh), "v"(w));
  return o;
}

// gemm_pp_kernel's schedule with fp8 operands on v_mfma_scale_f32_32x32x64_f8f6f4: the same
// 256x256 tile, 8 waves (2 along M x 4 along N, 128x64 each = 4 x 2 blocks of 32x32), the same
// 5-slot ring of 32 KiB stages (here 64 k each) with 3 stages of prefetch, the same two
// ping-pong phases per stage (m-half: 2 A blocks x 2 B blocks = 4 MFMAs of 64 cycles, the bf16
// section length) and the same counted waits, so the prefetch depth in time equals the bf16
// kernel's while each stage carries twice the k.  E8M0 scales: a lane needs, per stage
// s = 2t + u, byte 2s + h of its row's scales; the dword of blocks 4t .. 4t+3 serves both stages
// of pair t.  It is loaded two pairs ahead (at stage 2t - 4, before that stage's DMA; loaded one
// pair ahead its latency was exposed every pair: 0.6 of the bf16 kernel's stage rate), retired by
// the stage waits, and shifted into both stages' scale registers by asm at the pair's start.
// The MFMA sections are pinned before their closing barrier (asm "+v" on the accumulators),
// else they are sunk towards the loop latch past barriers.
template <typename OutT, int EPI>
__global__ __launch_bounds__(NT2, 1) void gemm_fp8_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  tile_coords(p, tile, tm, tn);
  const int m0 = tm * BT, n0 = tn * BT;
  const int ns = p.K / 64, T = p.K / 128, kb = p.K / 32;
  const uint8_t* A = (const uint8_t*)p.A;
  const uint8_t* B = (const uint8_t*)p.B;
  const SRsrc rsa = make_srsrc(p.a_scale, (uint32_t)((int64_t)p.M * kb));  // rows past M read 0
  const SRsrc rsb = make_srsrc(p.b_scale, (uint32_t)((int64_t)p.N * kb));
  const int offa = (m0 + wm * 128 + (lane & 31)) * kb, offb = (n0 + wn * 64 + (lane & 31)) * kb;
  const int h = lane >> 5;

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  auto slot = [&](int st) { return smem + (st % PP_S) * PP_STAGE; };
  // scale words of pair t (stages 2t, 2t + 1) in nx[t & 1]: [0, 4) A blocks, [4, 6) B blocks;
  // sc[u] = stage 2t + u's bytes.  Pair t + 2's words are loaded at stage 2t, so the stage DMA
  // waits retire them two stages before use, like the stages themselves.
  int nx[2][6], sc[2][6];
#pragma unroll
  for (int a = 0; a < 4; ++a) nx[0][a] = ld_dword_async(rsa, offa + 32 * a * kb);
#pragma unroll
  for (int b = 0; b < 2; ++b) nx[0][4 + b] = ld_dword_async(rsb, offb + 32 * b * kb);
  if (T > 1) {
#pragma unroll
    for (int a = 0; a < 4; ++a) nx[1][a] = ld_dword_async(rsa, offa + 32 * a * kb + 4);
#pragma unroll
    for (int b = 0; b < 2; ++b) nx[1][4 + b] = ld_dword_async(rsb, offb + 32 * b * kb + 4);
  }
#pragma unroll
  for (int st = 0; st < PP_D; ++st) {
    if (st < ns) {
      stage_pp8(slot(st), A, p.lda, m0, p.M, st * 64, wave, lane);
      stage_pp8(slot(st) + 16384, B, p.ldb, n0, p.N, st * 64, wave, lane);
    }
  }
  pp_vmcnt(4 * (min(PP_D, ns) - 1));  // stage 0 and pairs 0, 1's scales landed
  pp_barrier();
  if (wm == 1) pp_barrier();

  // one stage; UU = st % 4 is a template constant so the scale-buffer parity (pair t % 2 = UU / 2)
  // and the stage parity index register arrays statically (a runtime index would demote them to
  // scratch, which an asm-written async register must never be)
  auto stage = [&](auto UU, int st) {
    constexpr int uu = decltype(UU)::value, u = uu & 1, pb = uu >> 1;
    const char* img = slot(st);
    const bool issue = st + PP_D < ns;
    const int kn = (st + PP_D) * 64;
    i32x8 fb[2];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      // ---- load section
      if (ph == 0) {
        if constexpr (u == 0) {  // pair start: both stages' scale bytes, then pair t + 2's words
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            sc[0][i] = shr_after_wait(nx[pb][i], 8 * h);
            sc[1][i] = shr_after_wait(nx[pb][i], 16 + 8 * h);
          }
          if (st + 4 < ns) {
#pragma unroll
            for (int a = 0; a < 4; ++a) nx[pb][a] = ld_dword_async(rsa, offa + 32 * a * kb + 4 * (st / 2 + 2));
#pragma unroll
            for (int b = 0; b < 2; ++b) nx[pb][4 + b] = ld_dword_async(rsb, offb + 32 * b * kb + 4 * (st / 2 + 2));
          }
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) fb[b] = read_frag8(img + 16384, wn * 64 + b * 32, lane);
      }
      i32x8 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = read_frag8(img, wm * 128 + (ph * 2 + i) * 32, lane);
      if (issue) {
        if (ph == 0) stage_pp8(slot(st + PP_D), A, p.lda, m0, p.M, kn, wave, lane);
        else stage_pp8(slot(st + PP_D) + 16384, B, p.ldb, n0, p.N, kn, wave, lane);
      }
      if (ph == 1) {  // stage st + 1 landed; allowed in flight: stages st + 2, st + 3 and the
                      // scale words loaded at this pair's even stage (issued after st + 1's DMA)
        const bool wl = u == 0 ? st + 4 < ns : st + 3 < ns;
        pp_vmcnt(4 * (st + 2 < ns) + 4 * (st + 3 < ns) + (wl ? 6 : 0));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      // ---- MFMA section
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[ph * 2 + i][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              fb[b], fa[i], acc[ph * 2 + i][b], 0, 0, 0, sc[u][4 + b], 0, sc[u][ph * 2 + i]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b) asm volatile("" : "+v"(acc[ph * 2 + i][b]));
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
  };
  for (int st0 = 0; st0 < ns; st0 += 4) {  // ns is even: stages st0, st0 + 1 always exist
    stage(std::integral_constant<int, 0>{}, st0);
    stage(std::integral_constant<int, 1>{}, st0 + 1);
    if (st0 + 2 < ns) {
      stage(std::integral_constant<int, 2>{}, st0 + 2);
      stage(std::integral_constant<int, 3>{}, st0 + 3);
    }
  }
  if (wm == 0) pp_barrier();  // pairs with group 1's leading barrier
  // 32x32 accumulator blocks -> the 16x16 fragment layout of the shared epilogues, through the
  // wave's 16 KiB of the (idle) ring, 64 rows at a time: lane l holds m = 32a + (l & 31),
  // n = 32b + 8q + 4h + (0..3) in registers 4q..4q+3 of block (a, b); [64][64] fp32 rows of 256 B,
  // 16-B chunk c of row r at c ^ (r & 15).
  char* st_w = smem + wave * 16384;
  f32x4 acc16[8][4];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 32 * a2 + (lane & 31), c = 8 * b + 2 * q + h;
          const f32x16& v = acc[2 * hf + a2][b];
          *LDS_PTR(f32x4, st_w + r * 256 + ((c ^ (r & 15)) << 4)) = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 16 * i2 + (lane & 15), c = 4 * j + (lane >> 4);
        acc16[4 * hf + i2][j] = *LDS_PTR(const f32x4, st_w + r * 256 + ((c ^ (r & 15)) << 4));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (std::is_same<OutT, uint8_t>::value) epilogue_q8<EPI>(p, acc16, m0 + wm * 128, n0 + wn * 64, lane);
  else finish256<OutT, EPI>(p, acc16, m0 + wm * 128, n0 + wn * 64, lane, 0, st_w);
}

template <typename OutT, int EPI>
void launch_fp8(const GemmP& p, hipStream_t s) {
  (void)lds_optin((const void*)gemm_fp8_kernel<OutT, EPI>, PP_S * PP_STAGE);
  GemmP q = p;
  q.tiles_n = (p.N + BT - 1) / BT;
  q.ntiles = q.tiles_n * ((p.M + BT - 1) / BT);
  hipLaunchKernelGGL((gemm_fp8_kernel<OutT, EPI>), dim3(q.ntiles), dim3(NT2), PP_S * PP_STAGE, s, q);
}

const char* dispatch_fp8(const GemmP& p, hipStream_t s, bool f32o, bool q8o, int flags) {
  if (const char* l = dispatch_w4_fp8(p, s, f32o, q8o, flags)) return l;  // the persistent 4-wave form
  if (q8o) {
    switch (flags) {
      case E8_B | E8_Q: launch_fp8<uint8_t, E8_B | E8_Q>(p, s); return "gemm_fp8_fwd_bias_qgelu_q8";
      default: return nullptr;
    }
  }
  if (f32o) {
    launch_fp8<float, -1>(p, s);
    return "gemm_fp8";
  }
  switch (flags) {
    case E8_B: launch_fp8<bf16, E8_B>(p, s); return "gemm_fp8_fwd_bias";
    case E8_B | E8_R: launch_fp8<bf16, E8_B | E8_R>(p, s); return "gemm_fp8_fwd_bias_resid";
    case E8_B | E8_Q: launch_fp8<bf16, E8_B | E8_Q>(p, s); return "gemm_fp8_fwd_bias_qgelu";
    case 0: launch_fp8<bf16, 0>(p, s); return "gemm_fp8";
    default: launch_fp8<bf16, -1>(p, s); return "gemm_fp8_generic";
  }
}

// ---- MXFP8 quantisation: one thread per 32-element block of a row.  scale exponent e = the
// smallest with amax / 2^e <= 448 (e4m3's largest normal), E8M0 byte e + 127; values /2^e
// rounded to nearest even (v_cvt_pk_fp8_f32, OCP e4m3 on gfx950).
template <typename T>
__global__ __launch_bounds__(256) void quant_mxfp8_kernel(const T* x, int64_t ldx, int64_t R, int K, uint8_t* q,
                                                         uint8_t* sc) {
  const int nb = K >> 5;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= R * nb) return;
  const int64_t r = id / nb;
  const int blk = (int)(id - r * nb);
  const T* src = x + r * ldx + blk * 32;
  float v[32];
  if constexpr (std::is_same<T, bf16>::value) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 w = *(const bf16x8*)(src + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[8 * c + e] = (float)w[e];
    }
  } else {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const f32x4 w = *(const f32x4*)(src + 4 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * c + e] = w[e];
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
  const int ex = mx_exponent(amax);
  const float inv = ldexpf(1.0f, -ex);
  uint32_t w[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) w[e] = mx_pack4(v[4 * e], v[4 * e + 1], v[4 * e + 2], v[4 * e + 3], inv);
  uint8_t* dst = q + r * (int64_t)K + blk * 32;
  *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
  *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
  sc[r * nb + blk] = (uint8_t)(ex + 127);
}

#ifdef CLIPMI_GEMM_EXPERIMENTS  // persistent ping-pong (var 10) and half-tile pipeline (var 11): measured A/B forms
// ------------------------------------------------------------------ persistent ping-pong
// gemm_pp_kernel's schedule over a flattened stream of (tile, k-stage) pairs.  A workgroup
// walks its tiles gridDim.x apart and the LDS ring runs straight across tile boundaries, so
// the first PP_D stages of the next tile are DMA'd while the current tile's last stages and
// its epilogue run: no pipeline fill per tile, and one wave group's epilogue (VALU + stores)
// runs beside the other group's MFMA section.  Tiles are visited in groups of PP_GM
// row-blocks (every column-block of a group before the next group), so the 32 tiles an
// XCD holds at once share a few row and column panels in its L2.
constexpr int PP_GM = 8;

__device__ __forceinline__ void pps_tile(const GemmP& p, int lin, int& m0, int& n0) {
  const int tiles_m = p.ntiles / p.tiles_n;
  const int grp = lin / (PP_GM * p.tiles_n);
  const int rem = lin - grp * PP_GM * p.tiles_n;
  const int rows = min(PP_GM, tiles_m - grp * PP_GM);
  const int tn = rem / rows;
  const int tm = grp * PP_GM + (rem - tn * rows);
  m0 = tm * BT;
  n0 = tn * BT;
}

template <bool AK, bool BKM, typename OutT, int EPI>
__global__ __launch_bounds__(NT2, 1) void gemm_pps_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int r = xcd_remap(blockIdx.x, G);     // same-XCD workgroups take consecutive slots of a round
  const int nt = (p.ntiles - r + G - 1) / G;  // this workgroup's tiles: rounds j with j*G + r < ntiles
  const int ns = (p.K + 31) / 32;             // k-stages per tile
  const int S = nt * ns;
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;

  // issue stream position: tile ij, stage ik, that tile's origin
  if (p.stagger > 0 && ((blockIdx.x >> 3) & 1)) {  // half of every XCD's workgroups start later
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  int ij = 0, ik = 0, im0, in0;
  pps_tile(p, r, im0, in0);
  auto advance_issue = [&]() {
    if (++ik == ns) {
      ik = 0;
      ++ij;
      if (ij < nt) pps_tile(p, ij * G + r, im0, in0);
    }
  };
  auto slot = [&](int gs) { return smem + (gs % PP_S) * PP_STAGE; };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < PP_D; ++st) {  // prologue: stages 0 .. PP_D - 1 of the stream
    if (st < S) {
      stage_pp<AK>(slot(st), A, p.lda, im0, p.M, ik * 32, p.K, wave, lane);
      stage_pp<BKM>(slot(st) + 16384, B, p.ldb, in0, p.N, ik * 32, p.K, wave, lane);
      advance_issue();
    }
  }
  pp_vmcnt(4 * (min(PP_D, S) - 1));  // stage 0 landed
  pp_barrier();
  if (wm == 1) pp_barrier();

  int cj = 0, ck = 0, cm0, cn0;  // consumed tile, its stage, its origin
  pps_tile(p, r, cm0, cn0);
  for (int gs = 0; gs < S; ++gs) {
    const char* img = slot(gs);
    char* nimg = slot(gs + PP_D);
    const bool issue = gs + PP_D < S;
    bf16x8 fb[4];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      bf16x8 fa[4];
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = read_frag_pp<BKM>(img + 16384, wn * 64 + j * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag_pp<AK>(img, wm * 128 + (ph * 4 + i) * 16, lane);
      if (issue) {
        if (ph == 0) {
          stage_pp<AK>(nimg, A, p.lda, im0, p.M, ik * 32, p.K, wave, lane);
        } else {
          stage_pp<BKM>(nimg + 16384, B, p.ldb, in0, p.N, ik * 32, p.K, wave, lane);
          advance_issue();
        }
      }
      if (ph == 1) pp_vmcnt(4 * max(0, min(PP_D - 1, S - gs - 2)));  // stage gs + 1 landed
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[ph * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[ph * 4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
    if (++ck == ns) {  // tile done: its epilogue runs while the next tile's first stages land
      finish256<OutT, EPI>(p, acc, cm0 + wm * 128, cn0 + wn * 64, lane, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ck = 0;
      if (++cj < nt) pps_tile(p, cj * G + r, cm0, cn0);
    }
  }
  if (wm == 0) pp_barrier();  // pairs with group 1's leading barrier
}

// ------------------------------------------------------------------ half-tile pipeline, BK = 64
// gemm_pp_kernel's ping-pong schedule with every LDS-DMA piece made of full 128-B lines.  With
// BK = 32 stages a k-major piece is 16 rows x 64 B, twice the texture-address requests per
// byte of an 8-row x 128-B piece (cdna_hip_programming.md §5, "Projection GEMM at M = 256":
// 16 x 64 B pieces ran TA_BUSY 2x at equal traffic).  Here K advances in K-tiles of 64 through
// two 64 KiB buffers (A image [256][128 B] | B image, gemm256_kernel's layouts), and a K-tile
// arrives as four 16 KiB half-tiles (2 pieces per wave each) in the order they are first read:
//   i = 0: A m-half 0 (rows 0..63 and 128..191: the first 64 rows of each wave group)
//   i = 1, 2: B rows (k-major) or columns (k-row image) 0..127 / 128..255
//   i = 3: A m-half 1 (rows 64..127 and 192..255)
// A K-tile is consumed in 4 phases of 16 MFMAs per wave, one per quadrant of the wave's 128x64
// block: (m-half 0, n-half 0) reads the A m-half 0 and B n-half 0 fragments, (0, 1) B n-half 1,
// (1, 0) A m-half 1, (1, 1) nothing.  Half-tile s = 4t + i is issued in phase s - HP_D and
// waited for (counted vmcnt(6) / vmcnt(8)) in every wave's load section of the phase before its
// first read, i.e. before the barrier ahead of that read (the staggered group reads one
// interval later).  It overwrites half-tile s - 8, whose last fragment reads (phase s - 8 or
// s - 9 + i) both groups retired (lgkmcnt, in their MFMA section) at least one interval before
// the overwrite is issued.
constexpr int HP_D = 6;

template <bool BKM>
__device__ __forceinline__ void stage_hp(char* buf, const SRsrc& ra, int64_t lda, const SRsrc& rb, int64_t ldb, int i,
                                         int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = wave * 2 + u;  // piece 0..15 of the half-tile, 1 KiB each
    if (i == 0 || i == 3) {      // A rows g*128 + mh*64 + 8*(j & 7) .. +7, g = j >> 3
      const int r = (j >> 3) * 128 + (i == 3 ? 64 : 0) + (j & 7) * 8;
      const int rr = r + (lane >> 3);
      const int c = (lane & 7) ^ ((rr >> 1) & 7);
      dma16(ra, buf + r * 128, (int)((int64_t)rr * lda * 2 + c * 16));
    } else if (BKM) {            // B k-major: rows 128*(i-1) + 8j .. +7
      const int r = (i - 1) * 128 + j * 8;
      const int rr = r + (lane >> 3);
      const int c = (lane & 7) ^ ((rr >> 1) & 7);
      dma16(rb, buf + 32768 + r * 128, (int)((int64_t)rr * ldb * 2 + c * 16));
    } else {                     // B k-row: half image i-1, k rows 4j .. 4j+3
      const int h = i - 1;
      const int kr = 4 * j + (lane >> 4);
      const int c = (lane & 15) ^ mimg_swz(kr);
      dma16(rb, buf + 32768 + h * 16384 + j * 1024, (int)((int64_t)kr * ldb * 2 + (h * 128 + c * 8) * 2));
    }
  }
}

// the 16 MFMAs of quadrant (MH, NH): A m-half MH fragments x B n-half NH fragments, k = 64
template <int MH, int NH>
__device__ __forceinline__ void hp_mfma(f32x4 (&acc)[8][4], const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[4][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[MH * 4 + i][NH * 2 + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[NH * 2 + j][kk], fa[i][kk], acc[MH * 4 + i][NH * 2 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

template <bool BKM, typename OutT, int EPI>
__global__ __launch_bounds__(NT2, 1) void gemm_hp_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BT, n0 = tn * BT;
  const int nk = (p.K + 63) >> 6, S = 4 * nk;
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;
  auto issue = [&](int s) {  // this wave's pieces of half-tile s of the stream
    const int kt = s >> 2;
    const SRsrc ra = srsrc256<true>(A, p.lda, m0, p.M, kt * 64, p.K);
    const SRsrc rb = srsrc256<BKM>(B, p.ldb, n0, p.N, kt * 64, p.K);
    stage_hp<BKM>(smem + (kt & 1) * 65536, ra, p.lda, rb, p.ldb, s & 3, wave, lane);
  };
  // half-tiles 0 .. issued-1 are issued: wait until half-tile `need` has landed
  auto wait_for = [&](int issued, int need) { pp_vmcnt(2 * min(4, max(0, issued - 1 - need))); };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = 0; s < HP_D && s < S; ++s) issue(s);
  wait_for(min(HP_D, S), min(2, S - 1));  // K-tile 0: A m-half 0 and both B halves
  pp_barrier();
  if (wm == 1) pp_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const char* ia = smem + (kt & 1) * 65536;
    const char* ib = ia + 32768;
    const int s0 = 4 * kt + HP_D;  // half-tile issued in this K-tile's phase 0
    bf16x8 fa[4][2], fb[4][2];
    // ---- phase 0: quadrant (0, 0)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = read_frag256<true>(ia, wm * 128 + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = read_frag256<BKM>(ib, wn * 64 + j * 16, kk, lane);
    if (s0 < S) issue(s0);
    pp_barrier();
    hp_mfma<0, 0>(acc, fa, fb);
    pp_barrier();
    // ---- phase 1: quadrant (0, 1)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[2 + j][kk] = read_frag256<BKM>(ib, wn * 64 + 32 + j * 16, kk, lane);
    if (s0 + 1 < S) issue(s0 + 1);
    wait_for(min(s0 + 2, S), 4 * kt + 3);  // this K-tile's A m-half 1, read in phase 2
    pp_barrier();
    hp_mfma<0, 1>(acc, fa, fb);
    pp_barrier();
    // ---- phase 2: quadrant (1, 0)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = read_frag256<true>(ia, wm * 128 + 64 + i * 16, kk, lane);
    if (s0 + 2 < S) issue(s0 + 2);
    pp_barrier();
    hp_mfma<1, 0>(acc, fa, fb);
    pp_barrier();
    // ---- phase 3: quadrant (1, 1)
    if (s0 + 3 < S) issue(s0 + 3);
    if (kt + 1 < nk) wait_for(min(s0 + 4, S), 4 * kt + 6);  // next K-tile's A m-half 0 + B halves
    pp_barrier();
    hp_mfma<1, 1>(acc, fa, fb);
    pp_barrier();
  }
  if (wm == 0) pp_barrier();  // pairs with group 1's leading barrier
  finish256<OutT, EPI>(p, acc, m0 + wm * 128, n0 + wn * 64, lane, 0);
}

#endif  // CLIPMI_GEMM_EXPERIMENTS

// ------------------------------------------------------------------ f32 SIMT path
constexpr int FT = 64, FK = 16;

template <typename OutT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmP p, int akm, int bkm) {
  __shared__ float As[FK][FT + 4];
  __shared__ float Bs[FK][FT + 4];
  if (p.nb2 > 0) {  // strided batch: this block's (i1, i2) slice of A, B, C
    const int i1 = blockIdx.z / p.nb2, i2 = blockIdx.z - i1 * p.nb2;
    p.A = (const float*)p.A + i1 * p.bsa1 + i2 * p.bsa2;
    p.B = (const float*)p.B + i1 * p.bsb1 + i2 * p.bsb2;
    p.C = (OutT*)p.C + i1 * p.bsc1 + i2 * p.bsc2;
  }
  const float* A = (const float*)p.A;
  const float* B = (const float*)p.B;
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const int tile = blockIdx.x;
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * FT, n0 = tn * FT;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  float acc[4][4] = {};
  for (int k0 = kbeg; k0 < kend; k0 += FK) {
    for (int e = t; e < FK * FT; e += 256) {
      int kk, r;
      if (akm) { r = e / FK; kk = e % FK; } else { kk = e / FT; r = e % FT; }
      int gm = m0 + r, gk = k0 + kk;
      float va = 0.f;
      if (gm < p.M && gk < kend) va = akm ? A[(int64_t)gm * p.lda + gk] : A[(int64_t)gk * p.lda + gm];
      As[kk][r] = va;
      if (bkm) { r = e / FK; kk = e % FK; } else { kk = e / FT; r = e % FT; }
      int gn = n0 + r;
      gk = k0 + kk;
      float vb = 0.f;
      if (gn < p.N && gk < kend) vb = bkm ? B[(int64_t)gn * p.ldb + gk] : B[(int64_t)gk * p.ldb + gn];
      Bs[kk][r] = vb;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = m0 + ty * 4 + i, n = n0 + tx * 4;
    if (m >= p.M || n >= p.N) continue;
    float v[4] = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
    if (p.ws) st4(p.ws + (int64_t)blockIdx.y * p.M * p.N + (int64_t)m * p.N + n, v, min(4, p.N - n), p.vec && n + 4 <= p.N);
    else epilogue4<OutT, -1>(p, m, n, v);
  }
}

// split-K reduction: C (fp32) = [C +] alpha * sum_z ws[z]
__global__ void splitk_reduce_kernel(const float* ws, float* C, int64_t ldc, int M, int N, int splits,
                                     float alpha, int beta) {
  const int64_t total = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
    float sum = 0.f;
    for (int z = 0; z < splits; ++z) sum += ws[(int64_t)z * total + i];
    float* c = C + (int64_t)m * ldc + n;
    *c = beta ? *c + alpha * sum : alpha * sum;
  }
}

// same reduction, four columns per lane and eight slabs' loads in flight before the (fixed-order)
// adds: the scalar loop above waits one HBM round trip per slab.  N % 4 == 0, ldc % 4 == 0.
// bias_grad[m] += sum over splits of the per-split partials, in split order (deterministic)
__global__ __launch_bounds__(256) void bias_partials_reduce_kernel(const float* bws, float* bias_grad, int M,
                                                                   int splits) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float acc = 0.f;
  for (int z = 0; z < splits; ++z) acc += bws[(int64_t)z * M + m];
  bias_grad[m] += acc;
}

// Blocks nmain.. (when bws is set) sum the fused bias-gradient partials in split order, as
// bias_partials_reduce_kernel does, so a weight gradient with its bias costs one reduce launch.
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* ws, float* C, int64_t ldc, int M, int N,
                                                             int splits, float alpha, int beta, int nmain,
                                                             const float* bws, float* bias_grad) {
  if ((int)blockIdx.x >= nmain) {
    const int m = ((int)blockIdx.x - nmain) * 256 + threadIdx.x;
    if (m < M) {
      float acc = 0.f;
      for (int z = 0; z < splits; ++z) acc += bws[(int64_t)z * M + m];
      bias_grad[m] += acc;
    }
    return;
  }
  const int64_t total = (int64_t)M * N;
  const int n4 = N >> 2;
  const int64_t total4 = (int64_t)M * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (int64_t)nmain * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i - (int64_t)m * n4) * 4;
    const float* src = ws + (int64_t)m * N + n;
    float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(src + (int64_t)(z + j) * total);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sum.x += v[j].x; sum.y += v[j].y; sum.z += v[j].z; sum.w += v[j].w;
      }
    }
    for (; z < splits; ++z) {
      const float4 v = *(const float4*)(src + (int64_t)z * total);
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    float4* c = (float4*)(C + (int64_t)m * ldc + n);
    float4 r = make_float4(alpha * sum.x, alpha * sum.y, alpha * sum.z, alpha * sum.w);
    if (beta) {
      const float4 o = *c;
      r.x += o.x; r.y += o.y; r.z += o.z; r.w += o.w;
    }
    *c = r;
  }
}

template <bool AK, bool BKM, typename OutT, int EPI>
void launch_bf16(const GemmP& p, int splits, hipStream_t s) {
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKM, OutT, EPI>), dim3(p.ntiles, splits), dim3(NTHR), 65536, s, p);
}

template <bool AK, bool BKM, typename OutT, int EPI, bool BG, int VAR>
void launch256v(const GemmP& p, int splits, hipStream_t s, float* bias_grad) {
  (void)lds_optin((const void*)gemm256_kernel<AK, BKM, OutT, EPI, BG, VAR>, 131072);
  hipLaunchKernelGGL((gemm256_kernel<AK, BKM, OutT, EPI, BG, VAR>), dim3(p.ntiles * splits), dim3(NT2), 131072, s,
                     p, bias_grad);
}
template <bool AK, bool BKM, typename OutT, int EPI, bool BG, int PPV>
void launch_ppv(const GemmP& p, int splits, hipStream_t s, float* bias_grad) {
  (void)lds_optin((const void*)gemm_pp_kernel<AK, BKM, OutT, EPI, BG, PPV>, PP_S * PP_STAGE);
  hipLaunchKernelGGL((gemm_pp_kernel<AK, BKM, OutT, EPI, BG, PPV>), dim3(p.ntiles * splits), dim3(NT2),
                     PP_S * PP_STAGE, s, p, bias_grad);
}
int num_cus() {
  static int n[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  dev &= 63;
  if (!n[dev]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    n[dev] = c;
  }
  return n[dev];
}
#ifdef CLIPMI_GEMM_EXPERIMENTS
template <bool AK, bool BKM, typename OutT, int EPI>
void launch_pps(const GemmP& p, hipStream_t s) {
  (void)lds_optin((const void*)gemm_pps_kernel<AK, BKM, OutT, EPI>, PP_S * PP_STAGE);
  const int grid = std::min(p.ntiles, num_cus());  // one 160 KiB workgroup per CU
  hipLaunchKernelGGL((gemm_pps_kernel<AK, BKM, OutT, EPI>), dim3(grid), dim3(NT2), PP_S * PP_STAGE, s, p);
}
template <bool BKM, typename OutT, int EPI>
void launch_hp(const GemmP& p, hipStream_t s) {
  (void)lds_optin((const void*)gemm_hp_kernel<BKM, OutT, EPI>, 131072);
  hipLaunchKernelGGL((gemm_hp_kernel<BKM, OutT, EPI>), dim3(p.ntiles), dim3(NT2), 131072, s, p);
}
#endif
template <bool AK, bool BKM, typename OutT, int EPI, bool BG>
void launch256(const GemmP& p, int splits, hipStream_t s, float* bias_grad) {
  // production: the 8-wave ping-pong kernel (var 0 / 9); var 4: gemm256_kernel VAR 3 (interleaved asm
  // DMAs, round 2's weight-gradient schedule: the baseline of the 4-wave wgrad bitwise tests).  The
  // measured-and-rejected schedules are compiled only into an EXTRA=-DCLIPMI_GEMM_EXPERIMENTS build.
#ifdef CLIPMI_GEMM_EXPERIMENTS
  if (p.var == 10 && !BG && !p.ws && splits == 1) {
    launch_pps<AK, BKM, OutT, EPI>(p, s);
    return;
  }
  if constexpr (AK && !BG) {  // var 11: half-tile pipeline (k-major A)
    if (p.var == 11 && !p.ws && splits == 1) {
      launch_hp<BKM, OutT, EPI>(p, s);
      return;
    }
  }
  switch (p.var) {
    case 2: launch256v<AK, BKM, OutT, EPI, BG, 0>(p, splits, s, bias_grad); return;   // all DMAs up front
    case 3: launch256v<AK, BKM, OutT, EPI, BG, 2>(p, splits, s, bias_grad); return;   // builtin DMAs
    case 12: launch_ppv<AK, BKM, OutT, EPI, BG, 8>(p, splits, s, bias_grad); return;  // no epilogue (timing)
    case 13: launch_ppv<AK, BKM, OutT, EPI, BG, 16>(p, splits, s, bias_grad); return;  // DMAs between MFMAs
    case 14: launch_ppv<AK, BKM, OutT, EPI, BG, 20>(p, splits, s, bias_grad); return;  // + no setprio
    case 15: launch_ppv<AK, BKM, OutT, EPI, BG, 32>(p, splits, s, bias_grad); return;  // stores through LDS
    case 16: launch_ppv<AK, BKM, OutT, EPI, BG, 64>(p, splits, s, bias_grad); return;  // direct stores only
    case 5: launch_ppv<AK, BKM, OutT, EPI, BG, 1>(p, splits, s, bias_grad); return;
    case 6: launch_ppv<AK, BKM, OutT, EPI, BG, 2>(p, splits, s, bias_grad); return;
    case 7: launch_ppv<AK, BKM, OutT, EPI, BG, 3>(p, splits, s, bias_grad); return;
    case 8: launch_ppv<AK, BKM, OutT, EPI, BG, 4>(p, splits, s, bias_grad); return;
    default: break;
  }
#endif
  if (p.var == 4) launch256v<AK, BKM, OutT, EPI, BG, 3>(p, splits, s, bias_grad);
  else launch_ppv<AK, BKM, OutT, EPI, BG, 0>(p, splits, s, bias_grad);
}

constexpr int E_B = CLIPMI_EPI_BIAS, E_R = CLIPMI_EPI_RESID, E_Q = CLIPMI_EPI_QGELU, E_G = CLIPMI_EPI_GELU;
constexpr int E_P = CLIPMI_EPI_STORE_PRE, E_DQ = CLIPMI_EPI_DQGELU, E_DG = CLIPMI_EPI_DGELU, E_BETA = CLIPMI_EPI_BETA;
constexpr int E_DA = CLIPMI_EPI_STORE_DACT, E_MA = CLIPMI_EPI_MUL_AUX;

// the bf16x3 image-output products (clipmi_gemm_x3out, K' = 3K >= 2304) on the persistent 4-wave kernel; 0: the
// 8-wave kernel (CLIPMI_GEMM_X3_W4=0, A/B; read per call)
bool w4_x3() {
  const char* e = getenv("CLIPMI_GEMM_X3_W4");
  return !(e && e[0] == '0');
}

const char* dispatch256(const GemmP& p, int splits, hipStream_t s, bool f32o, int sel, int flags, float* bg) {
  if (sel == 0 && (p.ws || (f32o && flags == E_BETA))) {
    if (p.var == 28 || p.var == 32) {  // the persistent 4-wave kernel (gemm4.hip; 32: with the L2 prefetch)
      if (const char* l = dispatch_w4_wgrad(p, splits, s, flags, bg)) return l;
    }
    if (p.ws) {
      if (bg) launch256<false, false, float, 0, true>(p, splits, s, bg);
      else launch256<false, false, float, 0, false>(p, splits, s, bg);
      return "gemm256_wgrad_splitk";
    }
    if (bg) launch256<false, false, float, E_BETA, true>(p, splits, s, bg);
    else launch256<false, false, float, E_BETA, false>(p, splits, s, bg);
    return "gemm256_wgrad";
  }
  if (bg) return nullptr;
  // 28: the persistent 4-wave kernel for every shape; 32: the same with the L2 prefetch of the
  // activation operand; 9: the 8-wave ping-pong kernel for every shape.  Experiments build only (CLIPMI_GEMM_EXPERIMENTS):
  // 20: 4-wave kernel, one tile per workgroup; 22-25: its stamped timing builds (22 production
  // schedule, 23 no main-loop DMAs, 24 no fragment reads, 25 neither)
  // production (var 0): the persistent 4-wave kernel for long-K products (K >= 1536), where its main
  // loop is 3-7 % faster than the ping-pong kernel's; at K = 768 / 512 the ping-pong kernel's 8 waves
  // run the VALU-heavy epilogues twice as fast per SIMD (tools/w4_stamps.py, profiles/r03_*)
  // (and for fc2's input gradient with the stored-derivative product, K = 768: 1182 vs 1215 us,
  // profiles/r03_gemm_dact_shapes.log)
  // and, with the L2 prefetch of the activation operand (gemm4.hip w4_prefetch), for the short-K input
  // gradients (fc2's with the stored-derivative product, and out-proj's K = 768): 1.2-1.5 % and
  // 3-4 % over the persistent kernel without it (profiles/r04_gemm_variants.log); the forward shapes
  // and the long-K products measured equal or slower with it
  const bool w4_pf = p.var == 0 && sel == 2 && (flags == E_MA || (flags == 0 && p.K <= 768));
  const bool w4_default = p.var == 0 && (p.K >= 1536 || flags == E_MA);
  if ((w4_default || w4_pf || p.var == 20 || (p.var >= 22 && p.var <= 25 && p.dbg) || p.var == 28 || p.var == 32) &&
      !f32o && !p.ws && splits == 1 && (sel == 3 || sel == 2)) {
    GemmP q = p;
    const int dm = (p.var == 32 || w4_pf) ? 102 : (p.var == 28 || w4_default) ? 100 : p.var >= 22 ? 21 - p.var : 1;
    if (const char* l = dispatch_w4(q, s, sel == 3, flags, dm)) return l;
  }
  // fp32 output of a bf16 product (the bf16 mode's fp32 residual stream: out-projection and fc2 with the
  // residual fused; the patch embedding; the bf16x3 split products): the same kernels, fp32 epilogue
  if (f32o && !p.ws && splits == 1 && sel == 3) {
    if ((w4_default || p.var == 28) && (flags == E_B || flags == (E_B | E_R) || flags == 0 || (p.x3o && w4_x3()))) {
      if (const char* l = dispatch_w4_f32(p, s, flags, true)) return l;
    }
    switch (flags) {
      case E_B: launch256<true, true, float, E_B, false>(p, splits, s, bg); return "gemm256_fwd_bias_f32";
      case E_B | E_R: launch256<true, true, float, E_B | E_R, false>(p, splits, s, bg); return "gemm256_fwd_bias_resid_f32";
      case 0: launch256<true, true, float, 0, false>(p, splits, s, bg); return "gemm256_fwd_f32";
      // the bf16x3 mode's fc1 (training: the derivative stored beside the activation; inference)
      case E_B | E_Q | E_DA: launch256<true, true, float, E_B | E_Q | E_DA, false>(p, splits, s, bg); return "gemm256_fwd_bias_qgelu_dact_f32";
      case E_B | E_Q: launch256<true, true, float, E_B | E_Q, false>(p, splits, s, bg); return "gemm256_fwd_bias_qgelu_f32";
      default: break;
    }
  }
  // the bf16x3 mode's input gradients (fp32 gradients; fc2's with the stored-derivative product); the plain
  // ones (K' = 3K >= 2304) on the persistent 4-wave kernel, whose long-K main loop is the faster one
  if (f32o && !p.ws && splits == 1 && sel == 2) {
    if ((w4_default || p.var == 28) && (flags == 0 || (p.x3o && w4_x3()))) {
      if (const char* l = dispatch_w4_f32(p, s, flags, false)) return l;
    }
    switch (flags) {
      case 0: launch256<true, false, float, 0, false>(p, splits, s, bg); return "gemm256_dgrad_f32";
      case E_MA: launch256<true, false, float, E_MA, false>(p, splits, s, bg); return "gemm256_dgrad_mulaux_f32";
      default: break;
    }
  }
  if (sel == 3 && !f32o) {
    switch (flags) {
      case E_B: launch256<true, true, bf16, E_B, false>(p, splits, s, bg); return "gemm256_fwd_bias";
      case E_B | E_R: launch256<true, true, bf16, E_B | E_R, false>(p, splits, s, bg); return "gemm256_fwd_bias_resid";
      case E_B | E_Q | E_P: launch256<true, true, bf16, E_B | E_Q | E_P, false>(p, splits, s, bg); return "gemm256_fwd_bias_qgelu_pre";
      case E_B | E_Q | E_DA: launch256<true, true, bf16, E_B | E_Q | E_DA, false>(p, splits, s, bg); return "gemm256_fwd_bias_qgelu_dact";
      case E_B | E_Q: launch256<true, true, bf16, E_B | E_Q, false>(p, splits, s, bg); return "gemm256_fwd_bias_qgelu";
      case 0: launch256<true, true, bf16, 0, false>(p, splits, s, bg); return "gemm256_fwd";
      default: break;
    }
  }
  if (sel == 2 && !f32o) {
    switch (flags) {
      case 0: launch256<true, false, bf16, 0, false>(p, splits, s, bg); return "gemm256_dgrad";
      case E_DQ: launch256<true, false, bf16, E_DQ, false>(p, splits, s, bg); return "gemm256_dgrad_dqgelu";
      case E_MA: launch256<true, false, bf16, E_MA, false>(p, splits, s, bg); return "gemm256_dgrad_mulaux";
      default: break;
    }
  }
  return nullptr;  // not specialised: use the 128 kernel
}

// Specialised epilogues for the combinations the CLIP path issues; anything else takes the
// runtime-flag instance.  Returns the variant label (also used by the live profiler).
const char* dispatch_bf16(const GemmP& p, int splits, hipStream_t s, bool f32o, int sel, int flags) {
  if (p.ws) {
    if (sel == 0) { launch_bf16<false, false, float, 0>(p, splits, s); return "gemm_wgrad_splitk"; }
    launch_bf16<true, true, float, -1>(p, splits, s);
    return "gemm_generic";
  }
  if (sel == 3 && !f32o) {
    switch (flags) {
      case E_B: launch_bf16<true, true, bf16, E_B>(p, splits, s); return "gemm_fwd_bias";
      case E_B | E_R: launch_bf16<true, true, bf16, E_B | E_R>(p, splits, s); return "gemm_fwd_bias_resid";
      case E_B | E_Q | E_P: launch_bf16<true, true, bf16, E_B | E_Q | E_P>(p, splits, s); return "gemm_fwd_bias_qgelu_pre";
      case E_B | E_Q: launch_bf16<true, true, bf16, E_B | E_Q>(p, splits, s); return "gemm_fwd_bias_qgelu";
      case E_B | E_G | E_P: launch_bf16<true, true, bf16, E_B | E_G | E_P>(p, splits, s); return "gemm_fwd_bias_gelu_pre";
      case E_B | E_G: launch_bf16<true, true, bf16, E_B | E_G>(p, splits, s); return "gemm_fwd_bias_gelu";
      case 0: launch_bf16<true, true, bf16, 0>(p, splits, s); return "gemm_fwd";
      default: break;
    }
  }
  if (sel == 2 && !f32o) {
    switch (flags) {
      case 0: launch_bf16<true, false, bf16, 0>(p, splits, s); return "gemm_dgrad";
      case E_DQ: launch_bf16<true, false, bf16, E_DQ>(p, splits, s); return "gemm_dgrad_dqgelu";
      case E_DG: launch_bf16<true, false, bf16, E_DG>(p, splits, s); return "gemm_dgrad_dgelu";
      case E_R: launch_bf16<true, false, bf16, E_R>(p, splits, s); return "gemm_dgrad_resid";
      default: break;
    }
  }
  if (sel == 0 && f32o && flags == E_BETA) { launch_bf16<false, false, float, E_BETA>(p, splits, s); return "gemm_wgrad"; }
  if (f32o) {
    switch (sel) {
      case 3: launch_bf16<true, true, float, -1>(p, splits, s); break;
      case 2: launch_bf16<true, false, float, -1>(p, splits, s); break;
      case 1: launch_bf16<false, true, float, -1>(p, splits, s); break;
      default: launch_bf16<false, false, float, -1>(p, splits, s); break;
    }
  } else {
    switch (sel) {
      case 3: launch_bf16<true, true, bf16, -1>(p, splits, s); break;
      case 2: launch_bf16<true, false, bf16, -1>(p, splits, s); break;
      case 1: launch_bf16<false, true, bf16, -1>(p, splits, s); break;
      default: launch_bf16<false, false, bf16, -1>(p, splits, s); break;
    }
  }
  return "gemm_generic";
}

// tile-rows per raster group of the 256x256 kernels; CLIPMI_RASTER overrides (0 = row-major).
// Defaults from profiles/r02_raster_ab.log: bf16 row-major (groups of 4/8/16: within +-3 %, no
// consistent winner), fp8 groups of 8 (fc1 +10 %, the rest neutral).
int raster_rows(bool fp8 = false) {
  const char* e = getenv("CLIPMI_RASTER");  // read per call (tests switch it at run time)
  const int r = e ? atoi(e) : -1;
  return r >= 0 ? r : (fp8 ? 8 : 0);
}

}  // namespace

namespace cmg {
static unsigned long long* g_stamps = nullptr;
unsigned long long* gemm_stamp_buffer() { return g_stamps; }
}  // namespace cmg

// Diagnostic: arm (buf != nullptr) or disarm the 4-wave kernel's in-kernel timing build (variant
// 22): per workgroup < 512 and wave, s_memtime/s_memrealtime stamps of kernel start, main-loop
// start/end, kernel end and every k-step's barrier (before/after), 128 u64 per wave
// (tools/w4_stamps.py).  buf: device memory of 512 * 4 * 128 u64.
extern "C" int clipmi_gemm_stamps(void* buf) {
  cmg::g_stamps = (unsigned long long*)buf;
  return CLIPMI_OK;
}

// Strided-batched fp32 GEMM (exact f32, SIMT kernel): nb1 x nb2 independent products C_z = alpha A_z B_z^T
// (z = i1 * nb2 + i2, each operand offset by i1 * stride1 + i2 * stride2 elements), one launch.  The
// per-(sample, head) products of peclip's general head width (adapter/peclip.py:21-48 through
// nn.MultiheadAttention) without a host loop over B * H.
extern "C" int clipmi_gemm_batched(void* stream, const clipmi_gemm_desc* d, int nb1, int nb2, int64_t sa1,
                                   int64_t sa2, int64_t sb1, int64_t sb2, int64_t sc1, int64_t sc2) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(d && d->M >= 0 && d->N >= 0 && d->K >= 0, "bad shape");
  CLIPMI_REQUIRE(d->ab_dtype == CLIPMI_F32 && d->c_dtype == CLIPMI_F32, "batched GEMM: fp32 operands and output");
  CLIPMI_REQUIRE((d->flags & ~CLIPMI_EPI_BETA) == 0 && d->split_k <= 1 && !d->bias_grad,
                 "batched GEMM: no epilogue besides beta, no split-K");
  CLIPMI_REQUIRE(nb1 >= 0 && nb2 >= 0 && nb2 <= 65535, "batched GEMM: nb1 >= 0, 0 <= nb2 <= 65535");
  CLIPMI_REQUIRE(d->A && d->B && d->C, "batched GEMM: operands");
  if (d->M == 0 || d->N == 0 || nb1 == 0 || nb2 == 0) return CLIPMI_OK;
  // grid z carries (i1, i2) and is capped at 65535: larger batches (e.g. B = 8192 samples x 8 heads) run as
  // several launches over chunks of i1, each with its operands offset to the chunk's first sample
  const int c1 = 65535 / nb2;
  if (nb1 > c1) {
    for (int i0 = 0; i0 < nb1; i0 += c1) {
      clipmi_gemm_desc e = *d;
      e.A = (const float*)d->A + (int64_t)i0 * sa1;
      e.B = (const float*)d->B + (int64_t)i0 * sb1;
      e.C = (float*)d->C + (int64_t)i0 * sc1;
      CLIPMI_TRY(clipmi_gemm_batched(stream, &e, std::min(c1, nb1 - i0), nb2, sa1, sa2, sb1, sb2, sc1, sc2));
    }
    return CLIPMI_OK;
  }
  GemmP p;
  memset(&p, 0, sizeof(p));
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.A = d->A; p.lda = d->lda; p.B = d->B; p.ldb = d->ldb;
  p.C = d->C; p.ldc = d->ldc; p.alpha = d->alpha; p.flags = d->flags;
  p.k_per_split = d->K > 0 ? d->K : 1;
  p.tiles_n = (d->N + FT - 1) / FT;
  p.ntiles = p.tiles_n * ((d->M + FT - 1) / FT);
  p.vec = (d->ldc % 4 == 0) && ((uintptr_t)d->C % 16 == 0) && (sc1 % 4 == 0) && (sc2 % 4 == 0);
  p.nb2 = nb2;
  p.bsa1 = sa1; p.bsa2 = sa2; p.bsb1 = sb1; p.bsb2 = sb2; p.bsc1 = sc1; p.bsc2 = sc2;
  const double flops = 2.0 * d->M * d->N * d->K * nb1 * nb2;
  ProfScope ps(s, nullptr, 0.0);
  hipLaunchKernelGGL(gemm_f32_kernel<float>, dim3(p.ntiles, 1, nb1 * nb2), dim3(256), 0, s, p, d->a_kmajor, d->b_kmajor);
  ps.finish("gemm_f32_batched", flops);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

// ------------------------------------------------------------------ bf16x3 split-operand fp32 GEMM
// An fp32 product on the bf16 MFMA kernels (precision "bf16x3", the fast mode that meets north_star's
// 1e-3 logits): each fp32 operand is split as x = xh + xl with xh = bf16(x), xl = bf16(x - xh) (16
// significant bits between them), and A.B^T ~ Ah.Bh^T + Ah.Bl^T + Al.Bh^T -- the dropped Al.Bl^T is
// ~2^-16 of each product (profiles/r05_bf16x3_precision.log: max |dlogit| 1-2e-4 at config 3).  The
// three products run as ONE bf16 GEMM over a reduction axis of length 3K on concatenated operands
//   A3 = [Ah | Ah | Al],  B3 = [Bh | Bl | Bh]
// (k-major operands: column blocks of width K; operands row-major in k: row blocks of height K), every
// bf16 x bf16 product exact in the fp32 accumulator, so the 256-tile kernels and their epilogues (bias,
// activations, residual, aux, beta, split-K slabs) apply unchanged with fp32 C.  The split images live
// in the caller's workspace (clipmi_gemm_split3_ws); one pass per operand reads 4 B and writes 6 B per
// element.
//   pattern 0 (A): segments h, h, l;  pattern 1 (B): h, l, h.
// One workgroup per source row (nr rows of nc elements), V elements per thread step.
template <int V>
__global__ __launch_bounds__(256) void split3_kernel(const float* X, int64_t ldx, int nc, bf16* out, int64_t ldo,
                                                     int64_t seg, int pattern) {
  const int64_t r = blockIdx.x;
  const float* x = X + r * ldx;
  bf16* o = out + r * ldo;
  for (int c = threadIdx.x * V; c < nc; c += 256 * V) {
    float v[V];
    if constexpr (V == 4) {
      const f32x4 t = *(const f32x4*)(x + c);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
      v[0] = x[c];
    }
    bf16 h[V], l[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      h[j] = (bf16)v[j];
      l[j] = (bf16)(v[j] - (float)h[j]);
    }
    auto put = [&](bf16* q, const bf16 (&w)[V]) {
      if constexpr (V == 4) *(bf16x4*)q = bf16x4{w[0], w[1], w[2], w[3]};
      else q[0] = w[0];
    };
    put(o + c, h);
    put(o + seg + c, pattern ? l : h);
    put(o + 2 * seg + c, pattern ? h : l);
  }
}

namespace {
// the split image of one operand: k-major [rows][3K] (ld 3K), else [3K][round8(rows)]
int64_t split3_elems(int rows, int K, bool kmajor) {
  return kmajor ? (int64_t)rows * 3 * K : (int64_t)3 * K * ((rows + 7) / 8 * 8);
}
int64_t al256b(int64_t x) { return (x + 255) & ~(int64_t)255; }

int split3_operand(hipStream_t s, const float* X, int64_t ldx, int rows, int K, bool kmajor, bf16* out, int pattern) {
  // k-major: X[r][k] (rows x K) -> out[r][j K + k];  row-major in k: X[k][r] (K x rows) -> out[j K + k][r]
  const int nr = kmajor ? rows : K, nc = kmajor ? K : rows;
  const int64_t ldo = kmajor ? (int64_t)3 * K : (rows + 7) / 8 * 8;
  const int64_t seg = kmajor ? (int64_t)K : (int64_t)K * ldo;
  if (nr == 0 || nc == 0) return CLIPMI_OK;
  const bool v4 = nc % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)X & 15) == 0 && ldo % 4 == 0;
  if (v4) hipLaunchKernelGGL(split3_kernel<4>, dim3(nr), dim3(256), 0, s, X, ldx, nc, out, ldo, seg, pattern);
  else hipLaunchKernelGGL(split3_kernel<1>, dim3(nr), dim3(256), 0, s, X, ldx, nc, out, ldo, seg, pattern);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

int gemm_split3(hipStream_t s, const clipmi_gemm_desc* d) {
  CLIPMI_REQUIRE(d->ab_dtype == CLIPMI_F32 && d->c_dtype == CLIPMI_F32, "split3: fp32 operands and output");
  CLIPMI_REQUIRE(!d->bias_grad, "split3: the fused bias gradient would sum the split image (use clipmi_colsum)");
  CLIPMI_REQUIRE((!d->a_kmajor && !d->b_kmajor) || d->K % 8 == 0, "split3: K % 8 == 0 with a k-major operand");
  CLIPMI_REQUIRE(d->A && d->B, "split3: operands");
  const int64_t need = clipmi_gemm_split3_ws(d->M, d->N, d->K, d->a_kmajor, d->b_kmajor, d->split_k);
  CLIPMI_REQUIRE(d->workspace && d->workspace_bytes >= need && ((uintptr_t)d->workspace & 255) == 0,
                 "split3: workspace too small or not 256-byte aligned (clipmi_gemm_split3_ws)");
  if (d->M == 0 || d->N == 0) return CLIPMI_OK;
  char* w = (char*)d->workspace;
  const int64_t a_bytes = al256b(split3_elems(d->M, d->K, d->a_kmajor) * 2);
  const int64_t b_bytes = al256b(split3_elems(d->N, d->K, d->b_kmajor) * 2);
  bf16* A3 = (bf16*)w;
  bf16* B3 = (bf16*)(w + a_bytes);
  CLIPMI_TRY(split3_operand(s, (const float*)d->A, d->lda, d->M, d->K, d->a_kmajor, A3, 0));
  CLIPMI_TRY(split3_operand(s, (const float*)d->B, d->ldb, d->N, d->K, d->b_kmajor, B3, 1));
  clipmi_gemm_desc e = *d;
  e.flags &= ~CLIPMI_GEMM_SPLIT3;
  e.ab_dtype = CLIPMI_BF16;
  e.K = 3 * d->K;
  e.A = A3;
  e.lda = d->a_kmajor ? (int64_t)3 * d->K : (d->M + 7) / 8 * 8;
  e.B = B3;
  e.ldb = d->b_kmajor ? (int64_t)3 * d->K : (d->N + 7) / 8 * 8;
  e.workspace = w + a_bytes + b_bytes;
  e.workspace_bytes = d->workspace_bytes - a_bytes - b_bytes;
  return clipmi_gemm((void*)s, &e);
}
}  // namespace

// The split image of one fp32 operand (CLIPMI_GEMM_SPLIT3's layout): k-major X [rows][K] -> [rows][3K], else X [K][rows]
// -> [3K][round8(rows)]; pattern 0: segments (h, h, l), 1: (h, l, h).  out: clipmi_split3_elems(rows, K, kmajor) bf16.
extern "C" int64_t clipmi_split3_elems(int rows, int K, int kmajor) { return split3_elems(rows, K, kmajor != 0); }
extern "C" int clipmi_split3(void* stream, const float* X, int64_t ldx, int rows, int K, int kmajor, void* out,
                             int pattern) {
  CLIPMI_REQUIRE(X && out && rows >= 0 && K >= 0 && (pattern == 0 || pattern == 1), "split3: arguments");
  return split3_operand((hipStream_t)stream, X, ldx, rows, K, kmajor != 0, (bf16*)out, pattern);
}

extern "C" int64_t clipmi_gemm_split3_ws(int M, int N, int K, int a_kmajor, int b_kmajor, int split_k) {
  if (M < 0 || N < 0 || K < 0) return 0;
  int64_t b = al256b(split3_elems(M, K, a_kmajor) * 2) + al256b(split3_elems(N, K, b_kmajor) * 2);
  if (split_k > 1) b += (int64_t)split_k * M * N * 4;
  return b;
}

namespace {
// clipmi_gemm with the bf16x3 image output of clipmi_gemm_x3out (x3o 1 / 2: pattern 0 / 1, colp: column partials)
int gemm_impl(void* stream, const clipmi_gemm_desc* d, int x3o, float* colp) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(d && d->M >= 0 && d->N >= 0 && d->K >= 0, "bad shape");
  // every operand an epilogue flag reads or writes must be given (a null one would fault the GPU)
  {
    constexpr int AUXF = CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU | CLIPMI_EPI_STORE_PRE | CLIPMI_EPI_STORE_DACT |
                         CLIPMI_EPI_MUL_AUX;
    CLIPMI_REQUIRE(!(d->flags & AUXF) || (d->aux && d->ldaux >= d->N), "epilogue flags need aux (ldaux >= N)");
    CLIPMI_REQUIRE(!(d->flags & CLIPMI_EPI_RESID) || (d->residual && d->ldr >= d->N), "residual flag needs residual (ldr >= N)");
    CLIPMI_REQUIRE(!(d->flags & CLIPMI_EPI_BIAS) || d->bias, "bias flag needs bias");
    CLIPMI_REQUIRE(!(d->flags & CLIPMI_EPI_STORE_DACT) || (d->flags & (CLIPMI_EPI_QGELU | CLIPMI_EPI_GELU)),
                   "store_dact needs an activation flag");
    CLIPMI_REQUIRE((d->flags & ~(1023 | CLIPMI_GEMM_SPLIT3)) == 0, "unknown epilogue flag");
    // aux has one role per launch, and the epilogues read one input stream besides it
    constexpr int AUXR = CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU | CLIPMI_EPI_MUL_AUX;
    constexpr int AUXW = CLIPMI_EPI_STORE_PRE | CLIPMI_EPI_STORE_DACT;
    CLIPMI_REQUIRE((d->flags & AUXW) != AUXW, "store_pre and store_dact both write aux");
    CLIPMI_REQUIRE(!((d->flags & AUXR) && (d->flags & AUXW)), "aux cannot be both read and written");
    CLIPMI_REQUIRE(__builtin_popcount(d->flags & AUXR) <= 1, "at most one aux-reading flag");
    CLIPMI_REQUIRE(!((d->flags & CLIPMI_EPI_MUL_AUX) && (d->flags & (CLIPMI_EPI_RESID | CLIPMI_EPI_BETA))),
                   "mul_aux cannot be combined with residual / beta");
  }
  if (d->flags & CLIPMI_GEMM_SPLIT3) return gemm_split3(s, d);
  if (d->ab_dtype == CLIPMI_FP8) {  // MXFP8 operands (see include/clipmi.h)
    CLIPMI_REQUIRE(d->a_kmajor && d->b_kmajor, "fp8: both operands k-major");
    CLIPMI_REQUIRE(d->K % 128 == 0 && d->lda % 16 == 0 && d->ldb % 16 == 0, "fp8: K % 128 == 0, lda/ldb % 16 == 0");
    CLIPMI_REQUIRE(d->a_scale && d->b_scale, "fp8: block scales required");
    CLIPMI_REQUIRE(((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0, "fp8: A/B 16-byte aligned");
    CLIPMI_REQUIRE(d->c_dtype == CLIPMI_F32 || d->c_dtype == CLIPMI_BF16 || d->c_dtype == CLIPMI_FP8, "c_dtype");
    CLIPMI_REQUIRE(d->split_k <= 1 && !d->bias_grad, "fp8: forward GEMMs only");
    const bool q8o = d->c_dtype == CLIPMI_FP8;
    // epilogue_q8 writes each row's e4m3 bytes as 16-B stores and a row's two scale bytes as one 16-bit store
    CLIPMI_REQUIRE(!q8o || (d->c_scale && d->ldc == d->N && d->N % 32 == 0 && ((uintptr_t)d->C & 15) == 0 &&
                            ((uintptr_t)d->c_scale & 1) == 0),
                   "fp8 output: c_scale (2-byte aligned), ldc == N, N % 32 == 0, C 16-byte aligned");
    if (d->M == 0 || d->N == 0) return CLIPMI_OK;
    GemmP p;
    memset(&p, 0, sizeof(p));
    p.M = d->M; p.N = d->N; p.K = d->K;
    p.A = d->A; p.lda = d->lda; p.B = d->B; p.ldb = d->ldb;
    p.C = d->C; p.ldc = d->ldc; p.bias = d->bias; p.res = d->residual; p.ldr = d->ldr;
    p.aux = d->aux; p.ldaux = d->ldaux; p.alpha = d->alpha; p.flags = d->flags;
    p.bias_f32 = d->bias_dtype == CLIPMI_F32;
    p.k_per_split = d->K;
    p.a_scale = (const uint8_t*)d->a_scale;
    p.b_scale = (const uint8_t*)d->b_scale;
    p.c_scale = d->c_scale;
    p.raster = raster_rows(true);
    p.var = d->force_small_tile;  // 40: the 8-wave fp8 kernel (A/B of the persistent 4-wave one)
    {
      static const int env = [] {  // CLIPMI_FP8_VAR=40 / 41: every fp8 product on the 8-wave / 4-wave kernel (A/B)
        const char* e = getenv("CLIPMI_FP8_VAR");
        return e ? atoi(e) : 0;
      }();
      if (p.var == 0 && (env == 40 || env == 41)) p.var = env;
    }
    p.vec = (d->ldc % 4 == 0) && (d->ldr % 4 == 0) && (d->ldaux % 4 == 0) && ((uintptr_t)d->C % 16 == 0) &&
            ((uintptr_t)d->residual % 16 == 0) && ((uintptr_t)d->aux % 16 == 0);
    p.vec8 = d->c_dtype == CLIPMI_BF16 && d->N % 8 == 0 && d->ldc % 8 == 0 && d->ldr % 8 == 0 && d->ldaux % 8 == 0 &&
             ((uintptr_t)d->C % 16 == 0) && ((uintptr_t)d->residual % 16 == 0) && ((uintptr_t)d->aux % 16 == 0) &&
             ((uintptr_t)d->bias % 16 == 0);
    const double flops = 2.0 * d->M * d->N * d->K;
    ProfScope ps(s, nullptr, 0.0);
    const char* label = dispatch_fp8(p, s, d->c_dtype == CLIPMI_F32, q8o, d->flags);
    if (!label) return clipmi_invalid("fp8 output: supported epilogue flags are bias + quick_gelu");
    ps.finish(label, flops);
    CLIPMI_CHECK_LAUNCH();
    return CLIPMI_OK;
  }
  const bool bf = d->ab_dtype == CLIPMI_BF16;
  CLIPMI_REQUIRE(bf || d->ab_dtype == CLIPMI_F32, "ab_dtype");
  if (d->M == 0 || d->N == 0) return CLIPMI_OK;
  CLIPMI_REQUIRE(bf == false || d->b_kmajor || d->N % 8 == 0, "row-major B needs N % 8 == 0");
  CLIPMI_REQUIRE(d->c_dtype == CLIPMI_F32 || d->c_dtype == CLIPMI_BF16, "c_dtype");

  if (bf) {
    CLIPMI_REQUIRE(!d->a_kmajor || d->K % 8 == 0, "k-major A needs K % 8 == 0");
    CLIPMI_REQUIRE(!d->b_kmajor || d->K % 8 == 0, "k-major B needs K % 8 == 0");
    CLIPMI_REQUIRE(d->a_kmajor || d->M % 8 == 0, "row-major A needs M % 8 == 0");
    CLIPMI_REQUIRE(d->a_kmajor || d->M >= 8, "M >= 8");
    CLIPMI_REQUIRE(((uintptr_t)d->A & 15) == 0 && ((uintptr_t)d->B & 15) == 0, "A/B must be 16-byte aligned");
    CLIPMI_REQUIRE((d->lda % 8) == 0 && (d->ldb % 8) == 0, "lda/ldb must be multiples of 8");
  }
  int splits = d->split_k > 1 ? d->split_k : 1;
  GemmP p;
  memset(&p, 0, sizeof(p));
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.A = d->A; p.lda = d->lda; p.B = d->B; p.ldb = d->ldb;
  p.C = d->C; p.ldc = d->ldc; p.bias = d->bias; p.res = d->residual; p.ldr = d->ldr;
  p.aux = d->aux; p.ldaux = d->ldaux; p.alpha = d->alpha; p.flags = d->flags;
  p.bias_f32 = d->bias_dtype == CLIPMI_F32;
  p.ws = nullptr;
  p.bws = nullptr;
  p.x3o = x3o;
  p.colp = colp;
  // 256-kernel schedule: the ping-pong kernel for the forward / dgrad layouts, the
  // single-group asm-DMA schedule (var 4) for wgrad, where its 64-k steps measured faster
  // (profiles/r01_gemm_variants*.log).  CLIPMI_GEMM_VAR overrides it for A/B runs.
  // (CLIPMI_GEMM_VAR: forward/dgrad layouts, CLIPMI_GEMM_WVAR: wgrad layout)
  static const int env_var = [] {
    const char* e = getenv("CLIPMI_GEMM_VAR");
    return e ? atoi(e) : -1;
  }();
  static const int env_wvar = [] {
    const char* e = getenv("CLIPMI_GEMM_WVAR");
    return e ? atoi(e) : -1;
  }();
  const bool wlayout = !d->a_kmajor && !d->b_kmajor;
  const int evar = wlayout ? env_wvar : env_var;
  p.raster = raster_rows();
  p.dbg = gemm_stamp_buffer();
  p.stagger = 0;
  p.first_round = num_cus();
  if (d->force_small_tile >= 100 && d->force_small_tile < 200) {  // 1xx the 8-wave kernel, first-round stagger xx
    p.var = 9;
    p.stagger = d->force_small_tile % 100;
  } else if (d->force_small_tile >= 2) p.var = d->force_small_tile;
  else if (evar >= 0 && d->force_small_tile == 0) p.var = evar;
  else p.var = wlayout ? 28 : 0;  // wgrad: the persistent 4-wave kernel (5-11 % over var 4, profiles/r03_wgrad_4wave.log)
  p.vec = (d->ldc % 4 == 0) && (d->ldr % 4 == 0) && (d->ldaux % 4 == 0) && ((uintptr_t)d->C % 16 == 0) &&
          ((uintptr_t)d->residual % 16 == 0) && ((uintptr_t)d->aux % 16 == 0);
  p.vec8 = d->c_dtype == CLIPMI_BF16 && d->N % 8 == 0 && d->ldc % 8 == 0 && d->ldr % 8 == 0 && d->ldaux % 8 == 0 &&
           ((uintptr_t)d->C % 16 == 0) && ((uintptr_t)d->residual % 16 == 0) && ((uintptr_t)d->aux % 16 == 0) &&
           ((uintptr_t)d->bias % 16 == 0);
  // 256x256 LDS-DMA kernel for the big shapes (k-major operands need K % 64 == 0: the
  // buffer range check zero-fills rows, not a row's k tail)
  const bool kok = (!d->a_kmajor || d->K % 64 == 0) && (!d->b_kmajor || d->K % 64 == 0);
  const bool use256 = bf && kok && ((d->M >= 256 && d->N >= 128) || d->bias_grad) && d->force_small_tile != 1;
  CLIPMI_REQUIRE(!d->bias_grad || use256, "bias_grad fusion needs the 256 kernel (bf16, wgrad layout)");
  CLIPMI_REQUIRE(!x3o || (use256 && splits == 1), "x3out: needs the 256-tile kernels (M >= 256, N >= 128, K % 64 == 0)");
  const int tile = bf ? (use256 ? BT : BM) : FT;
  const int kstep = bf ? BK : FK;
  if (splits > 1) {
    CLIPMI_REQUIRE(d->c_dtype == CLIPMI_F32, "split_k needs fp32 C");
    CLIPMI_REQUIRE((d->flags & ~CLIPMI_EPI_BETA) == 0, "split_k supports only the beta flag");
    CLIPMI_REQUIRE(d->workspace && d->workspace_bytes >= (int64_t)splits * d->M * (d->N + (d->bias_grad ? 1 : 0)) * 4,
                   "split_k workspace too small (split_k * M * (N + bias_grad ? 1 : 0) floats)");
    int per = (d->K + splits - 1) / splits;
    per = (per + kstep - 1) / kstep * kstep;
    splits = (d->K + per - 1) / per;
    p.k_per_split = per;
    p.ws = (float*)d->workspace;
    if (d->bias_grad) p.bws = p.ws + (int64_t)splits * d->M * d->N;
  } else {
    p.k_per_split = d->K > 0 ? d->K : 1;
  }
  p.tiles_n = (d->N + tile - 1) / tile;
  p.ntiles = p.tiles_n * ((d->M + tile - 1) / tile);
  const double flops = 2.0 * d->M * d->N * d->K;
  if (bf) {
    const bool f32o = d->c_dtype == CLIPMI_F32 || p.ws;
    const int sel = (d->a_kmajor ? 2 : 0) | (d->b_kmajor ? 1 : 0);
    // the label is only known after dispatch; probe the profiler with the would-be label first
    ProfScope ps(s, nullptr, 0.0);
    const char* label = nullptr;
    if (use256) {
      GemmP q = p;
      q.tiles_n = (d->N + BT - 1) / BT;
      q.ntiles = q.tiles_n * ((d->M + BT - 1) / BT);
      // weight gradients with more column than row tiles (fc2: M = 768, N = 3072) walk each k-slab's
      // tiles column-major, so the ~32 items an XCD holds at once share the few row panels instead of
      // spanning every column panel (L2 fetch modelled 1.66x -> 1.25x of the compulsory panels,
      // tools/gemm_l2_model.py); CLIPMI_RASTER overrides
      if (wlayout && !getenv("CLIPMI_RASTER") && q.tiles_n > q.ntiles / q.tiles_n) q.raster = q.ntiles / q.tiles_n;
      label = dispatch256(q, splits, s, f32o, sel, d->flags, d->bias_grad);
      CLIPMI_REQUIRE(label || !x3o, "x3out: no image-output kernel for these flags");
    }
    if (!label) {
      CLIPMI_REQUIRE(!d->bias_grad, "bias_grad needs the wgrad layout (both operands row-major in k)");
      GemmP q = p;  // 128-tile grid (p's tile counts may be sized for the 256 kernel)
      q.tiles_n = (d->N + BM - 1) / BM;
      q.ntiles = q.tiles_n * ((d->M + BM - 1) / BM);
      label = dispatch_bf16(q, splits, s, f32o, sel, d->flags);
    }
    CLIPMI_REQUIRE(label, "no kernel for this GEMM");
    ps.finish(label, flops);
  } else {
    ProfScope ps(s, nullptr, 0.0);
    if (d->c_dtype == CLIPMI_F32 || p.ws)
      hipLaunchKernelGGL(gemm_f32_kernel<float>, dim3(p.ntiles, splits), dim3(256), 0, s, p, d->a_kmajor, d->b_kmajor);
    else
      hipLaunchKernelGGL(gemm_f32_kernel<bf16>, dim3(p.ntiles, splits), dim3(256), 0, s, p, d->a_kmajor, d->b_kmajor);
    ps.finish("gemm_f32", flops);
  }
  CLIPMI_CHECK_LAUNCH();
  if (p.ws) {
    const int64_t total = (int64_t)d->M * d->N;
    const int beta = (d->flags & CLIPMI_EPI_BETA) ? 1 : 0;
    if (d->N % 4 == 0 && d->ldc % 4 == 0 && ((uintptr_t)d->C & 15) == 0 && ((uintptr_t)p.ws & 15) == 0) {
      DeferredReduce r;
      memset(&r, 0, sizeof(r));
      r.kind = 1;
      r.ws = p.ws; r.C = (float*)d->C; r.ldc = d->ldc; r.M = d->M; r.N = d->N; r.splits = splits;
      r.alpha = d->alpha; r.beta = beta; r.bws = p.bws; r.bias_grad = d->bias_grad;
      DeferredReduce* slot = deferred_slot();
      if (slot && slot->kind == 0) *slot = r;  // executed by the next persistent GEMM launch
      else CLIPMI_TRY(launch_deferred(s, r));
    } else {
      const unsigned nblk = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(nblk), dim3(256), 0, s,
                         p.ws, (float*)d->C, d->ldc, d->M, d->N, splits, d->alpha, beta);
      if (p.bws)
        hipLaunchKernelGGL(bias_partials_reduce_kernel, dim3((d->M + 255) / 256), dim3(256), 0, s, p.bws,
                           d->bias_grad, d->M, splits);
    }
    CLIPMI_CHECK_LAUNCH();
  }
  return CLIPMI_OK;
}
}  // namespace

extern "C" int clipmi_gemm(void* stream, const clipmi_gemm_desc* d) { return gemm_impl(stream, d, 0, nullptr); }

namespace {
__global__ __launch_bounds__(256) void fold_rows4_kernel(const float* part, int P, int N, int per, float* out) {
  // out[g][c..c+3] = sum of part rows [g * per, min(P, (g + 1) * per)) in row order; eight rows' loads in flight
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= N) return;
  const int r0 = blockIdx.y * per, r1 = min(P, r0 + per);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
    f32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *(const f32x4*)(part + (int64_t)(r + j) * N + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  for (; r < r1; ++r) acc += *(const f32x4*)(part + (int64_t)r * N + c);
  *(f32x4*)(out + (int64_t)blockIdx.y * N + c) = acc;
}
constexpr int X3_FOLD = 64;  // first-stage groups of the column sums
int x3out_parts(int M) { return (M + 127) / 128; }
}  // namespace

// colsum[N] (+= when beta) = sum of the P partial rows part[P][N]: groups of rows folded in order into fold[<= 64][N],
// then those in order (norm.hip reduce_partials4_kernel); deterministic.  N % 4 == 0, 16-B aligned buffers.
int colsum_partials_finish(hipStream_t s, const float* part, int P, int N, float* colsum, int beta, float* fold) {
  const int per = (P + X3_FOLD - 1) / X3_FOLD, G = (P + per - 1) / per;
  hipLaunchKernelGGL(fold_rows4_kernel, dim3((N / 4 + 255) / 256, G), dim3(256), 0, s, part, P, N, per, fold);
  DeferredReduce r;
  memset(&r, 0, sizeof(r));
  r.kind = 2;
  r.part = fold; r.stride = N; r.P = G; r.D = N; r.out = colsum; r.out2 = nullptr; r.pbeta = beta;
  return launch_partials_reduce(s, r);
}
int64_t colsum_partials_ws(int P, int N) { return ((int64_t)P * N * 4 + 255) / 256 * 256 + (int64_t)X3_FOLD * N * 4; }

extern "C" int64_t clipmi_gemm_x3out_ws(int M, int N) {
  if (M <= 0 || N <= 0) return 0;
  return colsum_partials_ws(x3out_parts(M), N);
}

extern "C" int clipmi_gemm_x3out_ok(int M, int N, int K, int a_kmajor, int b_kmajor, int flags) {
  const int x3e = flags & ~CLIPMI_EPI_STORE_DACT;
  const bool fl = x3e == (CLIPMI_EPI_BIAS | CLIPMI_EPI_QGELU) || flags == CLIPMI_EPI_MUL_AUX;
  return fl && a_kmajor && M >= 256 && N >= 128 && N % 8 == 0 && K % 64 == 0 && (!b_kmajor || K % 64 == 0);
}

extern "C" int clipmi_gemm_x3out(void* stream, const clipmi_gemm_desc* d, int pattern, float* colsum, int beta,
                                 void* ws, int64_t ws_bytes) {
  hipStream_t s = (hipStream_t)stream;
  CLIPMI_REQUIRE(d && (pattern == 0 || pattern == 1), "x3out: arguments");
  CLIPMI_REQUIRE(d->ab_dtype == CLIPMI_BF16 && d->c_dtype == CLIPMI_F32 && d->split_k <= 1 && !d->bias_grad,
                 "x3out: bf16 operands, fp32 epilogue (c_dtype CLIPMI_F32), no split-K / bias gradient");
  CLIPMI_REQUIRE(clipmi_gemm_x3out_ok(d->M, d->N, d->K, d->a_kmajor, d->b_kmajor, d->flags),
                 "x3out: flags bias + quick_gelu (+ store_dact) or mul_aux, k-major A, M >= 256, N >= 128, N % 8 == 0, "
                 "K % 64 == 0");
  CLIPMI_REQUIRE(d->C && d->ldc >= 3 * (int64_t)d->N && d->ldc % 8 == 0 && ((uintptr_t)d->C & 15) == 0,
                 "x3out: C is the bf16 image [M][ldc], ldc >= 3N, ldc % 8 == 0, 16-byte aligned");
  CLIPMI_REQUIRE(!d->aux || (d->ldaux % 4 == 0 && ((uintptr_t)d->aux & 15) == 0),
                 "x3out: fp32 aux 16-byte aligned, ldaux % 4 == 0");
  CLIPMI_REQUIRE(!(d->flags & CLIPMI_EPI_BIAS) || d->bias_dtype == CLIPMI_F32 || ((uintptr_t)d->bias & 15) == 0,
                 "x3out: bf16 bias 16-byte aligned");
  float* colp = nullptr;
  if (colsum) {
    CLIPMI_REQUIRE(ws && ws_bytes >= clipmi_gemm_x3out_ws(d->M, d->N) && ((uintptr_t)ws & 255) == 0,
                   "x3out: column-sum workspace (clipmi_gemm_x3out_ws, 256-byte aligned)");
    colp = (float*)ws;
  }
  CLIPMI_TRY(gemm_impl(stream, d, 1 + pattern, colp));
  if (colsum) {
    const int P = x3out_parts(d->M);
    float* fold = (float*)((char*)ws + ((int64_t)P * d->N * 4 + 255) / 256 * 256);
    CLIPMI_TRY(colsum_partials_finish(s, colp, P, d->N, colsum, beta, fold));
  }
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}

DeferredReduce*& deferred_slot() {
  static thread_local DeferredReduce* slot = nullptr;
  return slot;
}

int launch_deferred(hipStream_t s, DeferredReduce& r) {
  if (r.kind == 1) {
    const int64_t total = (int64_t)r.M * r.N;
    const int nblk = (int)std::min<int64_t>((total / 4 + 255) / 256, 65536);
    const int nbias = r.bws ? (r.M + 255) / 256 : 0;
    hipLaunchKernelGGL(splitk_reduce4_kernel, dim3(nblk + nbias), dim3(256), 0, s, r.ws, r.C, r.ldc, r.M, r.N, r.splits,
                       r.alpha, r.beta, nblk, r.bws, r.bias_grad);
    CLIPMI_CHECK_LAUNCH();
  } else if (r.kind == 2) {
    CLIPMI_TRY(launch_partials_reduce(s, r));
  }
  r.kind = 0;
  return CLIPMI_OK;
}

extern "C" int clipmi_quant_mxfp8(void* stream, int dtype, const void* x, int64_t ldx, int64_t R, int K, uint8_t* q,
                                  uint8_t* scales) {
  CLIPMI_REQUIRE(R >= 0 && K % 32 == 0 && K > 0, "quant_mxfp8: K % 32 == 0");
  CLIPMI_REQUIRE(dtype == CLIPMI_BF16 || dtype == CLIPMI_F32, "quant_mxfp8: bf16 or f32 input");
  CLIPMI_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 15) == 0 && (ldx % 8) == 0, "quant_mxfp8: alignment");
  const int64_t n = R * (K / 32);
  if (n == 0) return CLIPMI_OK;
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (dtype == CLIPMI_BF16)
    hipLaunchKernelGGL(quant_mxfp8_kernel<bf16>, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, ldx, R,
                       K, q, scales);
  else
    hipLaunchKernelGGL(quant_mxfp8_kernel<float>, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const float*)x, ldx,
                       R, K, q, scales);
  CLIPMI_CHECK_LAUNCH();
  return CLIPMI_OK;
}
