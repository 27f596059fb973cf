// 4-wave 256x256 bf16 GEMM (one wave per SIMD): forward, dgrad and weight-gradient layouts.
//
// Replaces the same nn.Linear products as gemm.hip's 8-wave kernels ([HF] modeling_clip.py
// :313-315,332 q/k/v/out_proj, :348-350 fc1/fc2, their input gradients and their weight / bias
// gradients, i.e. the reference's loss.backward through those layers, trainer.py:92) with a
// schedule built around one wave per SIMD instead of two:
//  * 256 threads, 4 waves in 2 (M) x 2 (N); each wave owns a 128x128 block = 8x8 tiles of
//    v_mfma_f32_16x16x32_bf16 (256 fp32 accumulators per lane, pinned in the AGPR half of the
//    unified register file by inline-asm MFMAs).  Per 64-deep k-step a wave issues 128 MFMAs
//    (2048 matrix-pipe cycles) against 32 fragment reads and 16 LDS-DMA pieces: half the LDS
//    fragment bytes per FLOP of the 8-wave 128x64 tiling, and no partner wave competing for the
//    SIMD's issue slots or its matrix pipe.
//  * k advances in 64-deep steps through two 64 KiB LDS stages (A + B images); each step is two
//    half-steps of 64 MFMAs.  The next half-step's fragments are read between this half-step's
//    MFMAs (double-buffered in registers), so the matrix pipe never waits on a ds_read.
//  * one barrier per step, between its two halves: every wave has retired its reads of the step's
//    stage (lgkmcnt) and its DMAs of the next stage (vmcnt); after it the step's stage is refilled
//    (stage s + 2) by LDS-DMA issued between the second half's MFMAs, while the second half reads
//    the first fragments of stage s + 1.  Every DMA piece is 8 whole 128-B rows (k-major operand)
//    or 4 whole 256-B k-rows (row-major-in-k operand, read back with ds_read_b64_tr_b16).
//  * measured limit (tools/w4_stamps.py, profiles/r03_w4_*): the main loop runs at ~2.7-2.9k
//    cycles per step against 2048 of MFMA work, bound by the CU's LDS-DMA issue rate (~24 B/clk:
//    without the DMAs a step takes 2.37k cycles, without the fragment reads 2.87k); cache policy
//    (nt / sc1) and fewer M0 writes do not move it.
//  * persistent form (production): one workgroup per CU walks (split, tile) items; the next
//    item's first two stages are DMA'd before this item's epilogue, which stages its rows in the
//    32 KiB past the two stages, so the prologue latency (~6.7k cycles) hides under the stores.
//  * epilogues: the 8-wave kernel's finish256 (bias, quick_gelu + pre-activation store, residual,
//    gelu' of the stored pre-activation; fp32 beta / split-K slabs for weight gradients) on each
//    128x64 half of the wave's block.  Weight gradients fuse the bias gradient as one extra MFMA
//    per A fragment against a ones fragment (waves wn == 0 of n-tile 0), per-split partials summed
//    in split order afterwards (deterministic).
#include "gemm_common.h"

namespace cmg {
namespace {

constexpr int W4_STAGE = 65536;  // A 32 KiB + B 32 KiB per 64-deep k-step
constexpr int W4_THR = 256;

int num_cus_w4() {
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

// Per-lane byte offsets, all 32-bit (a 256-row tile spans < 2 GiB).  Loop-invariant pieces are
// computed once; a k-step varies only the stage base (LDS) and the descriptor base (DMA).
//   k-major operand ([rows][K]): image [256 rows][128 B], chunk c at c ^ ((r >> 1) & 7);
//     fragment i at rd[kk] + i * 2048; DMA piece i at dma[i & 1] + (64 wave + 8 i) * ld * 2.
//   row-major-in-k operand ([K][rows]): two [64 k][128] images of 16 KiB, chunk c at c ^ swz(k);
//     fragment i at rd[kk] + ((i << 5) ^ sw); DMA piece i at dma[(i >> 1) & 1] + scalar part.
struct W4Lane {
  int a_rd[2], b_rd[2];
  int a_sw, b_sw;
  int a_dma[2], b_dma[2];
};

template <bool KMAJ>
__device__ __forceinline__ void w4_lane_op(int base, int half, int lane, int64_t ld, int (&rd)[2], int& sw,
                                           int (&dma)[2]) {
  const int l15 = lane & 15, l4 = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    if (KMAJ) {
      rd[kk] = base + (half * 128 + l15) * 128 + (((kk * 4 + l4) ^ ((l15 >> 1) & 7)) << 4);
    } else {
      const int q = l15 >> 2, p4 = lane & 3;
      rd[kk] = base + half * 16384 + (kk * 32 + 8 * l4 + q) * 256 + (p4 >> 1) * 16 + (p4 & 1) * 8;
    }
  }
  sw = KMAJ ? 0 : (2 * (((l15 >> 2) & 3) | ((l4 & 1) << 2))) << 4;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (KMAJ) dma[p] = (lane >> 3) * (int)ld * 2 + (((lane & 7) ^ (4 * p + (lane >> 4))) << 4);
    else dma[p] = l4 * (int)ld * 2 + (((lane & 15) ^ (2 * (l4 | (p << 2)))) << 4);
  }
}

template <bool AK, bool BKM>
__device__ __forceinline__ W4Lane w4_lane(int wave, int lane, int64_t lda, int64_t ldb) {
  W4Lane w;
  w4_lane_op<AK>(0, wave >> 1, lane, lda, w.a_rd, w.a_sw, w.a_dma);
  w4_lane_op<BKM>(32768, wave & 1, lane, ldb, w.b_rd, w.b_sw, w.b_dma);
  return w;
}

#ifndef W4_CP  // cache-policy A/B builds of the main-loop DMAs (0 default, 1 nt, 2 sc1, 3 sc0 sc1)
#define W4_CP 0
#endif
#if W4_CP == 1
#define W4_DMA_POLICY " nt"
#elif W4_CP == 2
#define W4_DMA_POLICY " sc1"
#elif W4_CP == 3
#define W4_DMA_POLICY " sc0 sc1"
#else
#define W4_DMA_POLICY ""
#endif

// dma16 without its leading s_nop 2 (the wait states after the VALU readfirstlanes that wrote the
// descriptor): inside the main loop the descriptor is built before the half-step's first four
// MFMAs, so only the first piece after a fresh descriptor needs the pad (PAD)
template <bool PAD>
__device__ __forceinline__ void w4_dma(const SRsrc& r, char* lds, int voff) {
  if (PAD) {
    dma16(r, lds, voff);
    return;
  }
  const uint32_t m = (uint32_t)(uintptr_t)LDS_PTR(char, lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen" W4_DMA_POLICY " lds" ::"s"(m),
               "v"(voff), "s"(r.v)
               : "memory");
}

// this wave's DMA piece i (0..7) of one operand's 256x64 tile (image at img + base)
template <bool KMAJ, bool PAD = false>
__device__ __forceinline__ void w4_piece(char* img, int base, const SRsrc& rs, const int (&dma)[2], int ld, int wave,
                                         int i) {
  if (KMAJ) {
    w4_dma<PAD>(rs, img + base + (wave * 8 + i) * 1024, dma[i & 1] + (64 * wave + 8 * i) * ld * 2);
  } else {
    const int jj = (wave & 1) * 8 + i;
    w4_dma<PAD>(rs, img + base + (wave >> 1) * 16384 + jj * 1024, dma[(i >> 1) & 1] + 4 * jj * ld * 2 + (wave >> 1) * 256);
  }
}

__device__ __forceinline__ bf16x8 w4_rd(const char* p) { return *LDS_PTR(const bf16x8, p); }
__device__ __forceinline__ bf16x8 w4_rd_tr(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p + 1024));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
template <bool KMAJ>
__device__ __forceinline__ bf16x8 w4_frag(const char* p, int i, int sw) {
  return KMAJ ? w4_rd(p + i * 2048) : w4_rd_tr(p + ((i << 5) ^ sw));
}

// acc += B-fragment x A-fragment (16x16x32 bf16).  Inline asm with an AGPR "+a" operand keeps
// every accumulator in place in the AGPR file: with the builtin, the register allocator shuffles
// the 256 accumulators between AGPRs and VGPRs across the loop's back edge (hundreds of
// v_accvgpr moves per step) and spills.  Hazards the compiler does not see: accumulators are
// touched once per half-step (64 MFMAs apart), operands come straight from ds_read, and the
// epilogue's first AGPR read follows an explicit s_nop pad (w4_mfma_drain).
__device__ __forceinline__ void w4_mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
// fused bias gradient: accb (VGPRs) += ones x A-fragment.  The leading s_nop 1 covers the
// "VALU wrote an MFMA source VGPR" hazard in case the compiler re-materialises the ones operand
// right before this (invisible-to-it) MFMA; the ones fragment is also laundered once per kernel
// (w4_ones) so it lives in registers of its own.
__device__ __forceinline__ void w4_mfma_v(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ bf16x8 w4_ones() {
  bf16x8 o = bf16x8{(bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f, (bf16)1.f};
  asm volatile("" : "+v"(o));
  return o;
}
__device__ __forceinline__ void w4_mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

// One half-step: 64 MFMAs on the current fragments (fa, fb) in 16 groups of 4; after each group
// one of the next half-step's 16 fragments is read from stage rst, k-half kk (READ) and one of
// this wave's 16 DMA pieces of the stage after next is issued into dimg (DMA).  BG: 8 more MFMAs
// summing the A fragments into the bias-gradient accumulators (waves that own bias rows).
template <bool AK, bool BKM, bool READ, bool DMA, bool BG>
__device__ __forceinline__ void w4_half(f32x4 (&acc)[2][8][4], f32x4 (&accb)[8], bool bias_wave, const bf16x8& ones,
                                        const bf16x8 (&fa)[8], const bf16x8 (&fb)[8], bf16x8 (&na)[8],
                                        bf16x8 (&nb)[8], const char* rst, int kk, const W4Lane& w, int wave,
                                        char* dimg, const SRsrc& ra, const SRsrc& rb, int lda, int ldb) {
  const char* pa = rst + w.a_rd[kk];
  const char* pb = rst + w.b_rd[kk];
  int swa = w.a_sw, swb = w.b_sw;
  asm volatile("" : "+v"(swa), "+v"(swb));  // keep the per-fragment swizzled addresses inside the loop
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int i = g >> 1, h = g & 1;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) w4_mfma(acc[h][i][jj], fb[h * 4 + jj], fa[i]);
    if (BG && h == 1 && bias_wave) w4_mfma_v(accb[i], ones, fa[i]);
    if (READ) {
      if (g < 8) na[g] = w4_frag<AK>(pa, g, swa);
      else nb[g - 8] = w4_frag<BKM>(pb, g - 8, swb);
    }
    if (DMA) {
      if (g == 0) w4_piece<AK, true>(dimg, 0, ra, w.a_dma, lda, wave, 0);
      else if (g < 8) w4_piece<AK>(dimg, 0, ra, w.a_dma, lda, wave, g);
      else w4_piece<BKM>(dimg, 32768, rb, w.b_dma, ldb, wave, g - 8);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// descriptor of one stage's operand tile; an empty one (every DMA reads zeros) when !live
template <bool KMAJ>
__device__ __forceinline__ SRsrc w4_rsrc(const bf16* X, int64_t ld, int row0, int R, int k0, int K, bool live) {
  const bf16* base;
  uint32_t rec;
  extent256<KMAJ>(X, ld, row0, R, live ? k0 : 0, K, base, rec);
  return make_srsrc(base, live ? rec : 0u);
}

// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(0) through the builtin (not asm), so the compiler's own
// waitcnt bookkeeping sees that every fragment read has landed and adds no waits after it
__device__ __forceinline__ void w4_sync() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0070);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(N) lgkmcnt(0) + barrier: retires every VMEM operation but the wave's N youngest.
// (An item-start form that left the previous epilogue's stores in flight, vmcnt(32 / 63), measured
// neutral: profiles/r04_gemm_variants.log.)
template <int N>
__device__ __forceinline__ void w4_sync_n() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0070);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// L2 prefetch of one streamed operand's 256x64 k-stage: one dword per 128-B line of the stage's tile
// (this wave's quarter: 64 lines), LDS-DMA'd into this wave's epilogue staging area, which the main
// loop leaves idle (LDS-DMA needs no destination registers, so no late write can land in a VGPR the
// compiler has reused).  Measured motivation (tools/w4p_stamps.py, profiles/r04_w4p_stamps.log): with
// the activation operand's rows aliased into the CU's own cache the k-step drops from ~3.45k to
// ~2.88k cycles -- the nine CUs that share an activation panel all miss in L2 on the same k-slice at
// the same moment and wait for one HBM fetch; the weights (MALL / L2) are not the bottleneck.
// Two dwords per line (bytes 0 and 64): the L2 allocates 64-B halves on a partial-line miss.
template <bool KMAJ>
__device__ __forceinline__ void w4_prefetch(const SRsrc& r, char* scratch, int wave, int lane, int ld) {
  const int l = wave * 64 + lane;
  const int voff = KMAJ ? l * ld * 2 : (l >> 2) * ld * 2 + (l & 3) * 128;
  const uint32_t m = (uint32_t)(uintptr_t)LDS_PTR(char, scratch);
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\t"
               "buffer_load_dword %1, %2, 0 offen offset:64 lds" ::"s"(m), "v"(voff), "s"(r.v)
               : "memory");
}

template <bool AK, bool BKM>
__device__ __forceinline__ void w4_stage_dma(char* img, const GemmP& p, const W4Lane& w, int wave, int m0, int n0,
                                             int k0, int kend, bool live) {
  const SRsrc ra = w4_rsrc<AK>((const bf16*)p.A, p.lda, m0, p.M, k0, kend, live);
  const SRsrc rb = w4_rsrc<BKM>((const bf16*)p.B, p.ldb, n0, p.N, k0, kend, live);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w4_piece<AK, true>(img, 0, ra, w.a_dma, (int)p.lda, wave, i);
    w4_piece<BKM, true>(img, 32768, rb, w.b_dma, (int)p.ldb, wave, i);
  }
}

template <bool AK, bool BKM>
__device__ __forceinline__ void w4_first_frags(const char* smem, const W4Lane& w, bf16x8 (&a0)[8], bf16x8 (&b0)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = w4_frag<AK>(smem + w.a_rd[0], i, w.a_sw);
#pragma unroll
  for (int j = 0; j < 8; ++j) b0[j] = w4_frag<BKM>(smem + w.b_rd[0], j, w.b_sw);
}

#ifdef CLIPMI_GEMM_EXPERIMENTS  // one tile per workgroup + stamped diagnostic builds (tools/w4_stamps.py)
// ------------------------------------------------------------------ one tile per workgroup
// The first form, kept for its diagnostic builds (ST: s_memtime stamps into LDS past the two
// stages, copied to p.dbg: [0] kernel start, [1] main loop start, [2] main loop end, [3] kernel
// end, [4 + 2s] / [5 + 2s] step s's barrier entry / exit (s < 58), [126] / [127] s_memrealtime at
// kernel start / end; NOLD bit 0: no main-loop DMAs, bit 1: no fragment reads -- timing only).
constexpr int W4_NST = 128;
__device__ __forceinline__ void w4_stamp(char* smem, int wave, int lane, int k, unsigned long long v) {
  if (lane == 0) *LDS_PTR(unsigned long long, smem + 2 * W4_STAGE + (wave * W4_NST + k) * 8) = v;
}

template <bool BKM, typename OutT, int EPI, bool ST = false, int NOLD = 0>
__global__ __launch_bounds__(W4_THR, 1) void gemm_w4_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  unsigned long long st_real0 = 0, st0 = 0;
  if (ST) {
    st_real0 = __builtin_amdgcn_s_memrealtime();
    st0 = __builtin_amdgcn_s_memtime();
  }
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  tile_coords(p, tile, tm, tn);
  const int m0 = tm * BT, n0 = tn * BT;
  const int K = p.K;
  const int ns = (K + 63) / 64;
  const W4Lane w = w4_lane<true, BKM>(wave, lane, p.lda, p.ldb);
  const int lda = (int)p.lda, ldb = (int)p.ldb;

  f32x4 acc[2][8][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];

  // prologue: stages 0 and 1 in flight, stage 0 waited for, first fragments read
  if (ns > 0) w4_stage_dma<true, BKM>(smem, p, w, wave, m0, n0, 0, K, true);
  if (ns > 1) w4_stage_dma<true, BKM>(smem + W4_STAGE, p, w, wave, m0, n0, 64, K, true);
  __builtin_amdgcn_sched_barrier(0);
  if (ns > 1) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (ns > 0) w4_first_frags<true, BKM>(smem, w, a0, b0);

  // One loop body for every step (a single code path keeps the 256 accumulators in place):
  // past the last stage the DMAs get an empty descriptor (the hardware's range check turns them
  // into zero writes of a stage nobody reads) and the reads fetch fragments nobody uses.
  unsigned long long st_loop = 0, st_a = 0, st_b = 0;
  if (ST) st_loop = __builtin_amdgcn_s_memtime();
  const SRsrc none = SRsrc{u32x4{0u, 0u, 0u, 0u}};
  for (int s = 0; s < ns; ++s) {
    char* img = smem + (s & 1) * W4_STAGE;
    char* nxt = smem + ((s + 1) & 1) * W4_STAGE;
    w4_half<true, BKM, !(NOLD & 2), false, false>(acc, accb, false, a0[0], a0, b0, a1, b1, img, 1, w, wave, nullptr, none,
                                                  none, 0, 0);
    if (ST) st_a = __builtin_amdgcn_s_memtime();
    w4_sync();
    if (ST) st_b = __builtin_amdgcn_s_memtime();
    const bool more = s + 2 < ns;
    const SRsrc ra = w4_rsrc<true>((const bf16*)p.A, p.lda, m0, p.M, (s + 2) * 64, K, more);
    const SRsrc rb = w4_rsrc<BKM>((const bf16*)p.B, p.ldb, n0, p.N, (s + 2) * 64, K, more);
    w4_half<true, BKM, !(NOLD & 2), !(NOLD & 1), false>(acc, accb, false, a1[0], a1, b1, a0, b0, nxt, 0, w, wave, img, ra, rb,
                                                        lda, ldb);
    if (ST && s < 58) {
      w4_stamp(smem, wave, lane, 4 + 2 * s, st_a);
      w4_stamp(smem, wave, lane, 5 + 2 * s, st_b);
    }
  }
  w4_mfma_drain();
  unsigned long long st_lend = 0;
  if (ST) st_lend = __builtin_amdgcn_s_memtime();
  // every wave passed the last step's barrier after its last useful LDS read and DMA: the stages
  // are idle, so the epilogue may stage rows in this wave's 16 KiB of them
  char* st = smem + wave * 16384;
  finish256x2<OutT, EPI, true>(p, acc, m0 + wm * 128, n0 + wn * 128, lane, 0, st);
  if (ST) {
    const unsigned long long st_end = __builtin_amdgcn_s_memtime();
    const unsigned long long st_real1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_barrier();
    w4_stamp(smem, wave, lane, 0, st0);
    w4_stamp(smem, wave, lane, 1, st_loop);
    w4_stamp(smem, wave, lane, 3, st_end);
    w4_stamp(smem, wave, lane, 126, st_real0);
    w4_stamp(smem, wave, lane, 127, st_real1);
    __builtin_amdgcn_s_waitcnt(0);
    if (blockIdx.x < 512 && p.dbg) {
      const char* src = smem + 2 * W4_STAGE + wave * W4_NST * 8;
      unsigned long long* dst = p.dbg + ((size_t)blockIdx.x * 4 + wave) * W4_NST;
      for (int k = lane; k < W4_NST; k += 64) dst[k] = k == 2 ? st_lend : *LDS_PTR(const unsigned long long, src + k * 8);
    }
  }
}

#endif  // CLIPMI_GEMM_EXPERIMENTS

// ------------------------------------------------------------------ persistent (production)
// One workgroup per CU walks items i = r * grid + xcd_remap(blockIdx) (item = split * ntiles +
// tile, so each XCD holds a contiguous run of one k-slab's tiles per round).  After an item's
// main loop the next item's first two stages are DMA'd into the (now idle) stage buffers BEFORE
// this item's epilogue runs, so the next prologue's latency hides behind the epilogue's stores;
// the epilogue stages its rows in the 32 KiB past the two stages (8 KiB per wave).
// CLIPMI_W4P_STAMPS (diagnostic build only, tools/w4p_stamps.py): per workgroup < 256, wave and
// item < 20, s_memtime at the item's top, after its start sync, after its main loop, after the next
// item's prologue DMAs and after its epilogue, into p.dbg[(blk * 4 + wave) * 128 + item * 6 + phase];
// [126] / [127] s_memrealtime and [125] / [124] s_memtime at kernel start / end (lane 0, plain
// vector stores).
#ifdef CLIPMI_W4P_STAMPS
#define W4P_ST(ph)                                                                                     \
  do {                                                                                                 \
    if (p.dbg && blockIdx.x < 256 && it_no < 20 && lane == 0)                                          \
      p.dbg[(blockIdx.x * 4 + wave) * 128 + it_no * 6 + (ph)] = __builtin_amdgcn_s_memtime();          \
  } while (0)
#else
#define W4P_ST(ph) do { } while (0)
#endif

// A deferred reduction (internal.h DeferredReduce) shared by the launch's workgroups before their first
// item, with the arithmetic and summation order of the standalone kernels (splitk_reduce4_kernel,
// reduce_partials4_kernel), so the results are bitwise the same.  lds: 4 KiB of scratch (the epilogue
// staging area, idle until the first epilogue).  Every thread of the workgroup calls it.
__device__ __forceinline__ void hosted_reduce(const DeferredReduce& r, char* lds, int wg, int nwg, int t) {
  // One wave per SIMD has little latency hiding of its own: every thread keeps 16 slab loads in flight
  // (4 column groups x 4 splits), then adds them in split order per group, as the standalone kernel does.
  if (r.kind == 1) {
    const int64_t total = (int64_t)r.M * r.N;
    const int n4 = r.N >> 2;
    const int64_t total4 = (int64_t)r.M * n4;
    const int64_t step = (int64_t)nwg * 256;
    for (int64_t i0 = (int64_t)wg * 256 + t; i0 < total4; i0 += 4 * step) {
      int64_t off[4];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = i0 + u * step;
        ok[u] = i < total4;
        const int m = ok[u] ? (int)(i / n4) : 0, n = ok[u] ? (int)(i - (int64_t)m * n4) * 4 : 0;
        off[u] = (int64_t)m * r.N + n;
      }
      float4 sum[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) sum[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      // straight-line loads (invalid groups read offset 0 and are never stored), so all 16 are in flight
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (!ok[u]) off[u] = 0;
      int z = 0;
      for (; z + 4 <= r.splits; z += 4) {
        float4 v[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) v[j][u] = *(const float4*)(r.ws + off[u] + (int64_t)(z + j) * total);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            sum[u].x += v[j][u].x; sum[u].y += v[j][u].y; sum[u].z += v[j][u].z; sum[u].w += v[j][u].w;
          }
      }
      for (; z < r.splits; ++z) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const float4*)(r.ws + off[u] + (int64_t)z * total);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          sum[u].x += v[u].x; sum[u].y += v[u].y; sum[u].z += v[u].z; sum[u].w += v[u].w;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (!ok[u]) continue;
        const int64_t m = off[u] / r.N, n = off[u] - m * r.N;
        float4* c = (float4*)(r.C + m * r.ldc + n);
        float4 o = make_float4(r.alpha * sum[u].x, r.alpha * sum[u].y, r.alpha * sum[u].z, r.alpha * sum[u].w);
        if (r.beta) {
          const float4 q = *c;
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *c = o;
      }
    }
    if (r.bws) {
      for (int m = wg * 256 + t; m < r.M; m += nwg * 256) {
        float acc = 0.f;
        int z = 0;
        for (; z + 8 <= r.splits; z += 8) {  // 8 loads in flight, added in split order
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = r.bws[(int64_t)(z + j) * r.M + m];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += v[j];
        }
        for (; z < r.splits; ++z) acc += r.bws[(int64_t)z * r.M + m];
        r.bias_grad[m] += acc;
      }
    }
    return;
  }
  // kind 2: 16-column chunks (four lanes x four columns; one chunk per workgroup, so 2D / 16 of them share
  // the work); each of the standalone kernel's 64 partial groups ty (partials ty, ty + 64, ..., in order) is
  // one thread here (t >> 2), 8 of its loads in flight, then the kernel's tree: groups of 4, then 16 in order
  const int Dt = r.out2 ? 2 * r.D : r.D;
  const int nch = (Dt + 15) / 16;
  float4* red = (float4*)lds;  // [64 groups][4 lanes]
  const int tx = t & 3, ty = t >> 2;
  for (int ch = wg; ch < nch; ch += nwg) {
    const int c = ch * 16 + tx * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < Dt) {
      const float* src = r.part + c;
      int p = ty;
      for (; p + 7 * 64 < r.P; p += 8 * 64) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(src + (int64_t)(p + j * 64) * r.stride);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w;
        }
      }
      for (; p < r.P; p += 64) {
        const float4 v = *(const float4*)(src + (int64_t)p * r.stride);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    *LDS_PTR(f32x4, (char*)(red + ty * 4 + tx)) = f32x4{acc.x, acc.y, acc.z, acc.w};
    __syncthreads();
    if (ty == 0 && c < Dt) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const f32x4 a0 = *LDS_PTR(const f32x4, (char*)(red + (4 * q) * 4 + tx));
        float4 a = make_float4(a0[0], a0[1], a0[2], a0[3]);
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const f32x4 b = *LDS_PTR(const f32x4, (char*)(red + (4 * q + k) * 4 + tx));
          a.x += b[0]; a.y += b[1]; a.z += b[2]; a.w += b[3];
        }
        if (q == 0) s = a;
        else { s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w; }
      }
      float* o = c < r.D ? r.out + c : r.out2 + (c - r.D);
      if (r.pbeta) {
        s.x += o[0]; s.y += o[1]; s.z += o[2]; s.w += o[3];
      }
      o[0] = s.x; o[1] = s.y; o[2] = s.z; o[3] = s.w;
    }
    __syncthreads();
  }
}

// PF: L2 prefetch of the streamed operands (A always; B too for the weight gradient, whose B is the
// activation X) PF_D stages ahead, issued after each second half-step's DMAs (w4_prefetch); the next
// sync then waits vmcnt(NPF) so the prefetch stays in flight, and a prefetch is required complete
// one step later (it is older than that step's DMAs).  None in the last two steps of an item: the
// epilogue reuses the prefetches' LDS scratch; the next item's stages 0 and 1 are prefetched from
// this item's steps ns - 4 and ns - 3 instead.
constexpr int PF_D = 4;
template <bool AK, bool BKM, typename OutT, int EPI, bool BG, bool PF = false>
__global__ __launch_bounds__(W4_THR, 1) void gemm_w4p_kernel(GemmP p, float* bias_grad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
#ifdef CLIPMI_W4P_STAMPS
  int it_no = 0;
  if (p.dbg && blockIdx.x < 256 && lane == 0) {
    p.dbg[(blockIdx.x * 4 + (t >> 6)) * 128 + 126] = __builtin_amdgcn_s_memrealtime();
    p.dbg[(blockIdx.x * 4 + (t >> 6)) * 128 + 125] = __builtin_amdgcn_s_memtime();
  }
#endif
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = gridDim.x;
  const int splits = (p.K + p.k_per_split - 1) / p.k_per_split;
  const int nitems = p.ntiles * max(1, splits);
  int item = xcd_remap(blockIdx.x, nwg);
  if (item >= nitems && p.red.kind == 0) return;
  const int lda = (int)p.lda, ldb = (int)p.ldb;
  const W4Lane w = w4_lane<AK, BKM>(wave, lane, p.lda, p.ldb);
  auto coords = [&](int it, int& m0, int& n0, int& kz, int& kbeg, int& kend) {
    kz = it / p.ntiles;
    int tm, tn;
    tile_coords(p, it - kz * p.ntiles, tm, tn);
    m0 = tm * BT;
    n0 = tn * BT;
    kbeg = kz * p.k_per_split;
    kend = min(p.K, kbeg + p.k_per_split);
  };
  auto prologue_dma = [&](int it) {  // stages 0 and 1 of item it
    int m0, n0, kz, kbeg, kend;
    coords(it, m0, n0, kz, kbeg, kend);
    const int ns = (kend - kbeg + 63) / 64;
    w4_stage_dma<AK, BKM>(smem, p, w, wave, m0, n0, kbeg, kend, ns > 0);
    w4_stage_dma<AK, BKM>(smem + W4_STAGE, p, w, wave, m0, n0, kbeg + 64, kend, ns > 1);
  };
  if (item < nitems) prologue_dma(item);
  // a deferred reduction (the previous weight gradient's split-K sum or LayerNorm affine sum) while the
  // first stages land
  if (p.red.kind != 0) {
    hosted_reduce(p.red, smem + 2 * W4_STAGE, blockIdx.x, nwg, t);
    if (item >= nitems) return;
  }
  f32x4 acc[2][8][4];
  f32x4 accb[8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  const bf16x8 ones = w4_ones();
  const SRsrc none = SRsrc{u32x4{0u, 0u, 0u, 0u}};
  constexpr bool PFB = PF && !BKM && !AK;  // weight gradient: B is streamed too
  constexpr int NPF = PF ? (PFB ? 4 : 2) : 0;  // prefetch instructions per step
  char* const pf_area = smem + 2 * W4_STAGE + wave * 8192;
  while (true) {
    int m0, n0, kz, kbeg, kend;
    coords(item, m0, n0, kz, kbeg, kend);
    const int ns = (kend - kbeg + 63) / 64;
    int nm0 = 0, nn0 = 0, nkbeg = 0, nkend = 0;
    if (PF && item + nwg < nitems) {
      int nkz;
      coords(item + nwg, nm0, nn0, nkz, nkbeg, nkend);
    }
    const bool bias_wave = BG && n0 == 0 && wn == 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (BG) {
#pragma unroll
      for (int i = 0; i < 8; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // this item's stages 0 and 1 landed (every wave), the previous epilogue's LDS rows consumed
    W4P_ST(0);
    w4_sync();
    W4P_ST(1);
    w4_first_frags<AK, BKM>(smem, w, a0, b0);
    for (int s = 0; s < ns; ++s) {
      char* img = smem + (s & 1) * W4_STAGE;
      char* nxt = smem + ((s + 1) & 1) * W4_STAGE;
      w4_half<AK, BKM, true, false, BG>(acc, accb, bias_wave, ones, a0, b0, a1, b1, img, 1, w, wave, nullptr, none, none, 0,
                                        0);
      if (PF && s >= 1 && s - 1 <= ns - 3) w4_sync_n<NPF>();  // the previous step's prefetch stays in flight
      else w4_sync();
      const bool more = s + 2 < ns;
      const SRsrc ra = w4_rsrc<AK>((const bf16*)p.A, p.lda, m0, p.M, kbeg + (s + 2) * 64, kend, more);
      const SRsrc rb = w4_rsrc<BKM>((const bf16*)p.B, p.ldb, n0, p.N, kbeg + (s + 2) * 64, kend, more);
      w4_half<AK, BKM, true, true, BG>(acc, accb, bias_wave, ones, a1, b1, a0, b0, nxt, 0, w, wave, img, ra, rb, lda, ldb);
      if (PF && s <= ns - 3) {
        // target: stage s + PF_D of this item, else stage s + PF_D - ns of the next one (its stages
        // 0 and 1 from steps ns - 4 and ns - 3); an empty descriptor past either item's end
        const int tj = s + PF_D;
        const bool mine = tj < ns;
        const int pj = mine ? tj : tj - ns;
        const int pm0 = mine ? m0 : nm0, pn0 = mine ? n0 : nn0;
        const int pkb = mine ? kbeg : nkbeg, pke = mine ? kend : nkend;
        const bool live = mine || (pj <= 1 && pke > pkb + pj * 64);
        w4_prefetch<AK>(w4_rsrc<AK>((const bf16*)p.A, p.lda, pm0, p.M, pkb + pj * 64, pke, live), pf_area, wave, lane, lda);
        if (PFB)
          w4_prefetch<BKM>(w4_rsrc<BKM>((const bf16*)p.B, p.ldb, pn0, p.N, pkb + pj * 64, pke, live), pf_area, wave, lane,
                           ldb);
      }
    }
    w4_mfma_drain();
    W4P_ST(2);
    const int next = item + nwg;
    // every wave's last useful stage read came before the last step's barrier (the final
    // half-step's reads fetch fragments nobody uses), so the next item may overwrite both stages
    if (next < nitems) prologue_dma(next);
    W4P_ST(3);
    if (BG && bias_wave && lane < 16) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + wm * 128 + i * 16 + lane;
        if (m < p.M) {
          if (p.bws) p.bws[(int64_t)kz * p.M + m] = accb[i][0];  // summed in split order afterwards
          else atomicAdd(bias_grad + m, accb[i][0]);             // one split: one add per element
        }
      }
    }
    char* st = smem + 2 * W4_STAGE + wave * 8192;
    finish256x2<OutT, EPI, true>(p, acc, m0 + wm * 128, n0 + wn * 128, lane, kz, st);
    W4P_ST(4);
#ifdef CLIPMI_W4P_STAMPS
    ++it_no;
#endif
    if (next >= nitems) break;
    item = next;
  }
#ifdef CLIPMI_W4P_STAMPS
  if (p.dbg && blockIdx.x < 256 && lane == 0) {
    p.dbg[(blockIdx.x * 4 + wave) * 128 + 124] = __builtin_amdgcn_s_memtime();
    p.dbg[(blockIdx.x * 4 + wave) * 128 + 127] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

// persistent grid: one workgroup per CU
template <bool AK, bool BKM, typename OutT, int EPI, bool BG, bool PF = false>
void launch_w4p(const GemmP& p, int splits, hipStream_t s, float* bias_grad) {
  constexpr int L = 2 * W4_STAGE + 4 * 8192;
  (void)lds_optin((const void*)gemm_w4p_kernel<AK, BKM, OutT, EPI, BG, PF>, L);
  int grid = std::min(p.ntiles * splits, num_cus_w4());
  GemmP q = p;
  DeferredReduce* slot = deferred_slot();
  if (slot && slot->kind != 0) {  // host the recorded reduction (every CU's workgroup takes a share)
    q.red = *slot;
    slot->kind = 0;
    grid = num_cus_w4();
  }
  hipLaunchKernelGGL((gemm_w4p_kernel<AK, BKM, OutT, EPI, BG, PF>), dim3(grid), dim3(W4_THR), L, s, q, bias_grad);
}

// dm: 100 persistent, 102 persistent with the L2 prefetch; experiments build only:
// 1 one tile per workgroup, < 0 the stamped diagnostic builds.  Returns false when not built.
template <bool BKM, int EPI>
bool launch_w4(const GemmP& p, hipStream_t s, int dm) {
  if (dm == 100) {
    launch_w4p<true, BKM, bf16, EPI, false>(p, 1, s, nullptr);
    return true;
  }
  if (dm == 102) {  // L2 prefetch of the activation operand
    launch_w4p<true, BKM, bf16, EPI, false, true>(p, 1, s, nullptr);
    return true;
  }
#ifdef CLIPMI_GEMM_EXPERIMENTS
  if (dm < 0) {  // diagnostic stamp builds
    constexpr int L = 2 * W4_STAGE + 4 * W4_NST * 8;
#define W4_ST(n)                                                                                              \
  (void)lds_optin((const void*)gemm_w4_kernel<BKM, bf16, EPI, true, n>, L);                                  \
  hipLaunchKernelGGL((gemm_w4_kernel<BKM, bf16, EPI, true, n>), dim3(p.ntiles), dim3(W4_THR), L, s, p)
    if (dm == -1) { W4_ST(0); }
    else if (dm == -2) { W4_ST(1); }
    else if (dm == -3) { W4_ST(2); }
    else { W4_ST(3); }
#undef W4_ST
    return true;
  }
  (void)lds_optin((const void*)gemm_w4_kernel<BKM, bf16, EPI>, 2 * W4_STAGE);
  hipLaunchKernelGGL((gemm_w4_kernel<BKM, bf16, EPI>), dim3(p.ntiles), dim3(W4_THR), 2 * W4_STAGE, s, p);
  return true;
#else
  return false;
#endif
}


// ------------------------------------------------------------------ MXFP8 (config 5)
// The persistent 4-wave schedule with MXFP8 operands (OCP e4m3, one E8M0 scale per 32 k of a row;
// BASELINE config 5's frozen ViT-L/14@336 towers) on v_mfma_scale_f32_32x32x64_f8f6f4, which runs
// at twice the bf16 rate.  gemm.hip's gemm_fp8_kernel kept the 8-wave ping-pong stage time while
// each stage carried twice the FLOPs (PMC: 24-27 % of the fp8 pipe busy); here a stage is 128 k
// = 256 rows x 128 B per operand, byte for byte the bf16 4-wave kernel's 64-k stage, so the same
// LDS images, DMA pieces and swizzle serve it (the fp8 buffers are addressed as bf16 pairs) and a
// stage carries 2 x 16 MFMAs of 64 cycles per wave = the bf16 kernel's 2048 matrix-pipe cycles
// per 64 KiB.  Per wave 128 x 128 = 4 x 4 blocks of 32 x 32 (16 f32x16 accumulators pinned in the
// AGPRs by inline-asm MFMAs).  Operand map (profiles/r02_f8f6f4_32x32_layout.txt): lane l holds
// row l & 31, bytes 0-15 = k 16h .. 16h + 15 and bytes 16-31 = k 32 + 16h .. of the 64-k step
// (h = l >> 5): two ds_read_b128 per fragment, chunks 4kk + h and 4kk + 2 + h of the 128-B row
// (conflict-free under the bf16 image's c ^ ((r >> 1) & 7)).  Scales: E8M0 bytes of row l & 31,
// block 2kk + h; a stage pair (256 k) is one dwordx2 per row, loaded by asm beside the DMAs of the
// pair's first stage (two steps ahead), retired by the step syncs and copied out by asm after
// them (the compiler does not see the load).  Epilogue: 32 x 32 blocks -> the 16 x 16 fragment
// layout through the wave's 8 KiB of LDS, 32 rows at a time, then the bf16 kernels' finish256
// or the MXFP8 output epilogue on each 128 x 64 half.
constexpr int W8_PAIR = 256;  // k per scale load (8 E8M0 bytes per row)

__device__ __forceinline__ void w8_mfma(f32x16& acc, const i32x8& b, const i32x8& a, int sb, int sa) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0]"
               : "+a"(acc)
               : "v"(b), "v"(a), "v"(sb), "v"(sa));
}
__device__ __forceinline__ u32x2 w8_scale_load(const SRsrc& r, int voff) {
  u32x2 v;
  asm volatile("s_nop 4\n\tbuffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(r.v) : "memory");
  return v;
}
// the loaded words, after a vmcnt wait: this lane's byte (block parity h) moved to bit 0 of each
__device__ __forceinline__ u32x2 w8_scale_take(const u32x2& v, int sh) {
  u32x2 o;
  asm volatile("v_lshrrev_b32 %0, %2, %3\n\tv_lshrrev_b32 %1, %2, %4" : "=&v"(o[0]), "=&v"(o[1]) : "v"(sh), "v"(v[0]),
               "v"(v[1]));
  return o;
}

struct W8Lane {
  int a_rd[2][2], b_rd[2][2];  // [kk][chunk half] byte offsets inside a stage
};
__device__ __forceinline__ W8Lane w8_lane(int wm, int wn, int lane) {
  W8Lane w;
  const int r = lane & 31, h = lane >> 5, sw = (r >> 1) & 7;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int c = 4 * kk + 2 * e + h;
      w.a_rd[kk][e] = (wm * 128 + r) * 128 + ((c ^ sw) << 4);
      w.b_rd[kk][e] = 32768 + (wn * 128 + r) * 128 + ((c ^ sw) << 4);
    }
  return w;
}
__device__ __forceinline__ u32x4 w8_rd(const char* p) { return *LDS_PTR(const u32x4, p); }

// this k-step's scale operands from the stage's words (this lane's byte at bit 0 after
// w8_scale_take): k-step 0 uses byte 0, k-step 1 byte 2; the trailing s_nop 1 covers the "VALU
// wrote an MFMA source" hazard for the asm MFMAs that follow
template <int KK>
__device__ __forceinline__ void w8_kk_scales(const u32x2 (&ca)[4], const u32x2 (&cb)[4], int u, int (&sA)[4],
                                             int (&sB)[4]) {
  const int sh = 16 * KK;
#define W8_S(i)                                                                                                   \
  asm volatile("v_lshrrev_b32 %0, %2, %3\n\tv_lshrrev_b32 %1, %2, %4" : "=&v"(sA[i]), "=&v"(sB[i]) : "v"(sh), \
               "v"(u ? ca[i][1] : ca[i][0]), "v"(u ? cb[i][1] : cb[i][0]))
  W8_S(0);
  W8_S(1);
  W8_S(2);
  W8_S(3);
#undef W8_S
  asm volatile("s_nop 1" : "+v"(sA[0]), "+v"(sA[1]), "+v"(sA[2]), "+v"(sA[3]), "+v"(sB[0]), "+v"(sB[1]), "+v"(sB[2]),
               "+v"(sB[3]));
}

// One half-step (k-step kk of a stage): 16 MFMAs on the current fragments; after MFMA g the next
// half-step's read g (16 ds_read_b128 = 8 fragments, from stage rst, k-step nkk) and, with DMA,
// this wave's DMA piece g of the stage after next.  sA / sB: this k-step's scale operands.
template <bool READ, bool DMA>
__device__ __forceinline__ void w8_half(f32x16 (&acc)[4][4], const i32x8 (&fa)[4], const i32x8 (&fb)[4],
                                        i32x8 (&na)[4], i32x8 (&nb)[4], const int (&sA)[4], const int (&sB)[4],
                                        const char* rst, int nkk, const W8Lane& w8, const W4Lane& w, int wave,
                                        char* dimg, const SRsrc& ra, const SRsrc& rb, int lda2, int ldb2) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int i = g >> 2, j = g & 3;
    w8_mfma(acc[i][j], fb[j], fa[i], sB[j], sA[i]);
    if (READ) {
      const int f = (g & 7) >> 1, e = g & 1;
      const u32x4 v = w8_rd(rst + (g < 8 ? w8.a_rd[nkk][e] : w8.b_rd[nkk][e]) + f * 4096);
      i32x8& d = g < 8 ? na[f] : nb[f];
      d[4 * e] = (int)v[0];
      d[4 * e + 1] = (int)v[1];
      d[4 * e + 2] = (int)v[2];
      d[4 * e + 3] = (int)v[3];
    }
    if (DMA) {
      if (g == 0) w4_piece<true, true>(dimg, 0, ra, w.a_dma, lda2, wave, 0);
      else if (g < 8) w4_piece<true>(dimg, 0, ra, w.a_dma, lda2, wave, g);
      else w4_piece<true>(dimg, 32768, rb, w.b_dma, ldb2, wave, g - 8);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}


template <typename OutT, int EPI>
__global__ __launch_bounds__(W4_THR, 1) void gemm_w4p8_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = gridDim.x, nitems = p.ntiles;
  int item = xcd_remap(blockIdx.x, nwg);
  if (item >= nitems) return;
  // the fp8 buffers addressed as bf16 pairs: a 128-k fp8 stage is a 64-element bf16 stage
  GemmP q = p;
  q.lda = p.lda / 2;
  q.ldb = p.ldb / 2;
  const int lda2 = (int)q.lda, ldb2 = (int)q.ldb;
  const int K2 = p.K / 2, ns = p.K / 128, kb = p.K / 32;
  const W4Lane w = w4_lane<true, true>(wave, lane, q.lda, q.ldb);
  const W8Lane w8 = w8_lane(wm, wn, lane);
  const int h = lane >> 5, hsh = 8 * h;
  const SRsrc rsa = make_srsrc(p.a_scale, (uint32_t)((int64_t)p.M * kb));  // rows past M read 0
  const SRsrc rsb = make_srsrc(p.b_scale, (uint32_t)((int64_t)p.N * kb));
  auto coords = [&](int it, int& m0, int& n0) {
    int tm, tn;
    tile_coords(p, it, tm, tn);
    m0 = tm * BT;
    n0 = tn * BT;
  };
  // this lane's scale rows: A blocks wm*128 + 32i + (l & 31), B blocks wn*128 + 32j + (l & 31)
  auto load_scales = [&](int m0, int n0, int pair, u32x2 (&sa)[4], u32x2 (&sb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sa[i] = w8_scale_load(rsa, ((m0 + wm * 128 + 32 * i + (lane & 31)) * kb + 8 * pair));
      sb[i] = w8_scale_load(rsb, ((n0 + wn * 128 + 32 * i + (lane & 31)) * kb + 8 * pair));
    }
  };
  auto prologue = [&](int it) {  // stages 0, 1 of item it
    int m0, n0;
    coords(it, m0, n0);
    w4_stage_dma<true, true>(smem, q, w, wave, m0, n0, 0, K2, true);
    w4_stage_dma<true, true>(smem + W4_STAGE, q, w, wave, m0, n0, 64, K2, ns > 1);
  };
  u32x2 nsa[4], nsb[4];  // in flight: the next scale pair
  prologue(item);
  f32x16 acc[4][4];
  i32x8 a0[4], b0[4], a1[4], b1[4];
  const SRsrc none = SRsrc{u32x4{0u, 0u, 0u, 0u}};
  while (true) {
    int m0, n0;
    coords(item, m0, n0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    load_scales(m0, n0, 0, nsa, nsb);  // scale pair 0 (not held across the previous epilogue: registers)
    w4_sync();  // stages 0, 1 and scale pair 0 landed (every wave); the previous epilogue's LDS rows consumed
    u32x2 csa[4], csb[4];  // the current scale pair, this lane's bytes at bit 0 of each word's low byte
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      csa[i] = w8_scale_take(nsa[i], hsh);
      csb[i] = w8_scale_take(nsb[i], hsh);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const u32x4 va = w8_rd(smem + w8.a_rd[0][e] + f * 4096), vb = w8_rd(smem + w8.b_rd[0][e] + f * 4096);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a0[f][4 * e + r] = (int)va[r];
          b0[f][4 * e + r] = (int)vb[r];
        }
      }
    // two stages per iteration (ns is even: K % 256 == 0), so the scale word of a stage is static
#pragma unroll 1
    for (int s = 0; s < ns; s += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int st = s + u;
        char* img = smem + u * W4_STAGE;  // stage st lives in slot st & 1 = u
        char* nxt = smem + (u ^ 1) * W4_STAGE;
        if (u == 0 && s >= 2) {  // pair s / 2 (loaded beside stage s's DMAs) landed at stage s - 1's sync
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            csa[i] = w8_scale_take(nsa[i], hsh);
            csb[i] = w8_scale_take(nsb[i], hsh);
          }
        }
        int sA[4], sB[4];
        w8_kk_scales<0>(csa, csb, u, sA, sB);
        w8_half<true, false>(acc, a0, b0, a1, b1, sA, sB, img, 1, w8, w, wave, nullptr, none, none, 0, 0);
        w4_sync();
        w8_kk_scales<1>(csa, csb, u, sA, sB);
        const bool more = st + 2 < ns;
        const SRsrc ra = w4_rsrc<true>((const bf16*)p.A, q.lda, m0, p.M, (st + 2) * 64, K2, more);
        const SRsrc rb = w4_rsrc<true>((const bf16*)p.B, q.ldb, n0, p.N, (st + 2) * 64, K2, more);
        w8_half<true, true>(acc, a1, b1, a0, b0, sA, sB, nxt, 0, w8, w, wave, img, ra, rb, lda2, ldb2);
        if (u == 0 && st + 2 < ns) load_scales(m0, n0, (st + 2) / 2, nsa, nsb);  // pair of stages st + 2, st + 3
      }
    }
    w4_mfma_drain();
    const int next = item + nwg;
    if (next < nitems) prologue(next);
    // epilogue: per 32 x 64 block pair (a, b = 2c, 2c + 1) -> the 16 x 16 fragment layout through
    // this wave's 8 KiB of LDS, then the 16-B-store epilogue on those 32 rows.  (A direct epilogue
    // from the 32 x 32 layout -- permlane32 pairing, bf16 rows staged through LDS per unit -- measured
    // 20-25 % slower per launch: profiles/r04_fp8_gemm.log.)
    char* st_w = smem + 2 * W4_STAGE + wave * 8192;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        f32x4 acc16[2][4];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int r = lane & 31, cc = 8 * b2 + 2 * qq + h;
            const f32x16& v = acc[a][2 * c + b2];
            *LDS_PTR(f32x4, st_w + r * 256 + ((cc ^ (r & 15)) << 4)) =
                f32x4{v[4 * qq], v[4 * qq + 1], v[4 * qq + 2], v[4 * qq + 3]};
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 16 * i2 + (lane & 15), cc = 4 * j + (lane >> 4);
            acc16[i2][j] = *LDS_PTR(const f32x4, st_w + r * 256 + ((cc ^ (r & 15)) << 4));
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int mb = m0 + wm * 128 + 32 * a, nb = n0 + wn * 128 + 64 * c;
        if constexpr (std::is_same<OutT, uint8_t>::value) {
          epilogue_q8<EPI, 2>(p, acc16, mb, nb, lane);
        } else if constexpr (std::is_same<OutT, float>::value) {  // fp32 output: per-fragment generic stores
#pragma unroll
          for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = mb + 16 * i2 + (lane & 15), n = nb + 16 * j + (lane >> 4) * 4;
              float v[4] = {acc16[i2][j][0], acc16[i2][j][1], acc16[i2][j][2], acc16[i2][j][3]};
              if (m < p.M && n < p.N) epilogue4<float, EPI>(p, m, n, v);
            }
        } else {
          epilogue256_w<EPI < 0 ? 0 : EPI, false, 2>(p, acc16, mb, nb, lane);
        }
      }
    if (next >= nitems) break;
    item = next;
  }
}

template <typename OutT, int EPI>
void launch_w4p8(const GemmP& p, hipStream_t s) {
  constexpr int L = 2 * W4_STAGE + 4 * 8192;
  (void)lds_optin((const void*)gemm_w4p8_kernel<OutT, EPI>, L);
  GemmP q = p;
  q.tiles_n = (p.N + BT - 1) / BT;
  q.ntiles = q.tiles_n * ((p.M + BT - 1) / BT);
  const int grid = std::min(q.ntiles, num_cus_w4());
  hipLaunchKernelGGL((gemm_w4p8_kernel<OutT, EPI>), dim3(grid), dim3(W4_THR), L, s, q);
}
}  // namespace

// forward (k-major B) and dgrad (row-major-in-k B) products with bf16 output and one of the
// CLIP path's epilogues; returns the profiler label, or nullptr when not covered.
// dm: 1 one tile per workgroup, 100 persistent, < 0 the stamped diagnostic builds.
const char* dispatch_w4(const GemmP& p, hipStream_t s, bool bkm, int flags, int dm) {
  constexpr int E_B = CLIPMI_EPI_BIAS, E_R = CLIPMI_EPI_RESID, E_Q = CLIPMI_EPI_QGELU;
  constexpr int E_P = CLIPMI_EPI_STORE_PRE, E_DQ = CLIPMI_EPI_DQGELU;
  constexpr int E_DA = CLIPMI_EPI_STORE_DACT, E_MA = CLIPMI_EPI_MUL_AUX;
  if (bkm) {
    switch (flags) {
      case E_B: return launch_w4<true, E_B>(p, s, dm) ? "gemm256_fwd_bias" : nullptr;
      case E_B | E_R: return launch_w4<true, E_B | E_R>(p, s, dm) ? "gemm256_fwd_bias_resid" : nullptr;
      case E_B | E_Q | E_P: return launch_w4<true, E_B | E_Q | E_P>(p, s, dm) ? "gemm256_fwd_bias_qgelu_pre" : nullptr;
      case E_B | E_Q | E_DA: return launch_w4<true, E_B | E_Q | E_DA>(p, s, dm) ? "gemm256_fwd_bias_qgelu_dact" : nullptr;
      case E_B | E_Q: return launch_w4<true, E_B | E_Q>(p, s, dm) ? "gemm256_fwd_bias_qgelu" : nullptr;
      case 0: return launch_w4<true, 0>(p, s, dm) ? "gemm256_fwd" : nullptr;
      default: return nullptr;
    }
  }
  switch (flags) {
    case 0: return launch_w4<false, 0>(p, s, dm) ? "gemm256_dgrad" : nullptr;
    case E_DQ: return launch_w4<false, E_DQ>(p, s, dm) ? "gemm256_dgrad_dqgelu" : nullptr;
    case E_MA: return launch_w4<false, E_MA>(p, s, dm) ? "gemm256_dgrad_mulaux" : nullptr;
    default: return nullptr;
  }
}

// fp32-output forward products (k-major B) on the persistent kernel: the bf16 mode's fp32 residual stream
// (fc2 with bias + residual) and fp32-output bf16 products
const char* dispatch_w4_f32(const GemmP& p, hipStream_t s, int flags, bool bkm) {
  constexpr int E_B = CLIPMI_EPI_BIAS, E_R = CLIPMI_EPI_RESID, E_Q = CLIPMI_EPI_QGELU;
  constexpr int E_DA = CLIPMI_EPI_STORE_DACT, E_MA = CLIPMI_EPI_MUL_AUX;
  if (!bkm) {  // the bf16x3 mode's input gradients (K' = 3K >= 2304), fp32 out or (fc2's, x3o) the image
    if (flags == E_MA && p.x3o) {
      launch_w4p<true, false, float, E_MA, false>(p, 1, s, nullptr);
      return "gemm256_dgrad_mulaux_f32";
    }
    if (flags != 0) return nullptr;
    launch_w4p<true, false, float, 0, false>(p, 1, s, nullptr);
    return "gemm256_dgrad_f32";
  }
  if (p.x3o) {  // the bf16x3 mode's fc1 writing its activation's image (clipmi_gemm_x3out)
    if (flags == (E_B | E_Q | E_DA)) {
      launch_w4p<true, true, float, E_B | E_Q | E_DA, false>(p, 1, s, nullptr);
      return "gemm256_fwd_bias_qgelu_dact_f32";
    }
    if (flags == (E_B | E_Q)) {
      launch_w4p<true, true, float, E_B | E_Q, false>(p, 1, s, nullptr);
      return "gemm256_fwd_bias_qgelu_f32";
    }
    return nullptr;
  }
  switch (flags) {
    case E_B | E_R: launch_w4p<true, true, float, E_B | E_R, false>(p, 1, s, nullptr); return "gemm256_fwd_bias_resid_f32";
    case E_B: launch_w4p<true, true, float, E_B, false>(p, 1, s, nullptr); return "gemm256_fwd_bias_f32";
    case 0: launch_w4p<true, true, float, 0, false>(p, 1, s, nullptr); return "gemm256_fwd_f32";
    default: return nullptr;
  }
}

// weight gradients (both operands row-major in k, fp32 output): split-K slabs (p.ws) or the
// beta epilogue (one split), with the fused bias gradient when bg != nullptr
// MXFP8 forward products on the persistent 4-wave kernel: K % 256 == 0 (whole scale pairs) and at
// least one full tile; nullptr leaves them to gemm.hip's 8-wave fp8 kernel
// Production: every covered shape (round 5).  Round 4 kept the residual / activation epilogues at K = 1024
// (fc1 -> MXFP8, out-proj) on the 8-wave kernel, equal or 5 % slower here in isolation
// (profiles/r04_fp8_gemm.log); in config 5's step this kernel for all of them measured equal throughput
// and a 3.5 % shorter mean fp8 launch (profiles/r05_cfg5_fp8_kernel_ab.log).  40: the 8-wave kernel (A/B).
const char* dispatch_w4_fp8(const GemmP& p, hipStream_t s, bool f32o, bool q8o, int flags) {
  if (p.K % W8_PAIR != 0 || p.M < BT || p.N < BT || p.var == 40) return nullptr;  // 40: the 8-wave kernel (A/B)
  constexpr int B8 = CLIPMI_EPI_BIAS, Q8 = CLIPMI_EPI_QGELU, R8 = CLIPMI_EPI_RESID;
  if (q8o) {
    if (flags != (B8 | Q8)) return nullptr;
    launch_w4p8<uint8_t, B8 | Q8>(p, s);
    return "gemm_fp8_fwd_bias_qgelu_q8";
  }
  if (f32o) {
    launch_w4p8<float, -1>(p, s);
    return "gemm_fp8";
  }
  if (!p.vec8) return nullptr;  // the 16-B-store epilogue needs aligned bf16 rows
  switch (flags) {
    case B8: launch_w4p8<bf16, B8>(p, s); return "gemm_fp8_fwd_bias";
    case B8 | R8: launch_w4p8<bf16, B8 | R8>(p, s); return "gemm_fp8_fwd_bias_resid";
    case B8 | Q8: launch_w4p8<bf16, B8 | Q8>(p, s); return "gemm_fp8_fwd_bias_qgelu";
    case 0: launch_w4p8<bf16, 0>(p, s); return "gemm_fp8";
    default: return nullptr;
  }
}

const char* dispatch_w4_wgrad(const GemmP& p, int splits, hipStream_t s, int flags, float* bg) {
  if (p.ws) {
#ifdef CLIPMI_GEMM_EXPERIMENTS
    if (p.var == 32) {  // L2 prefetch of both operands (measured 5-8 % slower on the CLIP shapes)
      if (bg) launch_w4p<false, false, float, 0, true, true>(p, splits, s, bg);
      else launch_w4p<false, false, float, 0, false, true>(p, splits, s, bg);
      return "gemm256_wgrad_splitk";
    }
#endif
    if (bg) launch_w4p<false, false, float, 0, true>(p, splits, s, bg);
    else launch_w4p<false, false, float, 0, false>(p, splits, s, bg);
    return "gemm256_wgrad_splitk";
  }
  if (flags != CLIPMI_EPI_BETA) return nullptr;
  if (bg) launch_w4p<false, false, float, CLIPMI_EPI_BETA, true>(p, 1, s, bg);
  else launch_w4p<false, false, float, CLIPMI_EPI_BETA, false>(p, 1, s, bg);
  return "gemm256_wgrad";
}

}  // namespace cmg
