// 4-wave 256x256 bf16 GEMM for the forward / dgrad layouts (one wave per SIMD).
//
// Replaces the same nn.Linear products as gemm.hip's ping-pong kernel ([HF] modeling_clip.py
// :313-315,332 q/k/v/out_proj, :348-350 fc1/fc2 and their input gradients) with a schedule
// built around one wave per SIMD instead of two:
//  * 256 threads, 4 waves in 2 (M) x 2 (N); each wave owns a 128x128 block = 8x8 tiles of
//    v_mfma_f32_16x16x32_bf16 (256 fp32 accumulators per lane, in the AGPR half of the unified
//    register file).  Per 64-deep k-step a wave issues 128 MFMAs (2048 matrix-pipe cycles)
//    against 32 fragment reads and 16 LDS-DMA pieces: a quarter of the LDS fragment bytes per
//    FLOP of the 8-wave 128x64 tiling, and no partner wave competing for the SIMD's issue
//    slots or its matrix pipe.
//  * k advances in 64-deep steps through two 64 KiB LDS stages (A [256 rows][128 B] + B);
//    each step is two half-steps of 64 MFMAs (k 0-31, k 32-63).  The fragments of the next
//    half-step are read from LDS between this half-step's MFMAs (double-buffered in
//    registers), so the matrix pipe never waits on a ds_read.
//  * one barrier per step, between its two halves: every wave has retired its reads of the
//    step's stage (lgkmcnt) and its DMAs of the next stage (vmcnt); after it the step's stage
//    is refilled (stage s + 2) by LDS-DMA issued between the second half's MFMAs, while the
//    second half reads the first fragments of stage s + 1.  Every DMA piece is 8 whole 128-B
//    rows (k-major) or 4 whole 256-B k-rows (row-major-in-k), the full-line shape.
//  * epilogues: the 8-wave kernel's finish256 (bias, quick_gelu + pre-activation store,
//    residual, gelu' of the stored pre-activation) on each 128x64 half of the wave's block,
//    bf16 rows staged through the then idle LDS stages so every store instruction writes
//    whole 128-B rows.
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
// computed once; the k-step varies only the stage base (LDS) and the descriptor base (DMA).
struct W4Lane {
  int a_rd[2];  // A fragment i of k-half kk at stage + a_rd[kk] + i * 2048
  int b_rd[2];  // B: k-major as A; row-major-in-k: frag j at stage + b_rd[kk] + ((j << 5) ^ b_sw)
  int b_sw;
  int a_dma[2];  // A piece i: a_dma[i & 1] + (64 wave + 8 i) * lda * 2
  int b_dma[2];  // B piece i: k-major as A; row-major-in-k b_dma[(i >> 1) & 1] + scalar
};

template <bool BKM>
__device__ __forceinline__ W4Lane w4_lane(int wave, int lane, int64_t lda, int64_t ldb) {
  W4Lane w;
  const int wm = wave >> 1, wn = wave & 1;
  const int l15 = lane & 15, l4 = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    w.a_rd[kk] = (wm * 128 + l15) * 128 + (((kk * 4 + l4) ^ ((l15 >> 1) & 7)) << 4);
    if (BKM) {
      w.b_rd[kk] = 32768 + (wn * 128 + l15) * 128 + (((kk * 4 + l4) ^ ((l15 >> 1) & 7)) << 4);
    } else {
      const int q = l15 >> 2, p4 = lane & 3;
      w.b_rd[kk] = 32768 + wn * 16384 + (kk * 32 + 8 * l4 + q) * 256 + (p4 >> 1) * 16 + (p4 & 1) * 8;
    }
  }
  w.b_sw = BKM ? 0 : (2 * (((l15 >> 2) & 3) | ((l4 & 1) << 2))) << 4;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    w.a_dma[p] = (lane >> 3) * (int)lda * 2 + (((lane & 7) ^ (4 * p + (lane >> 4))) << 4);
    if (BKM) w.b_dma[p] = (lane >> 3) * (int)ldb * 2 + (((lane & 7) ^ (4 * p + (lane >> 4))) << 4);
    else w.b_dma[p] = l4 * (int)ldb * 2 + (((lane & 15) ^ (2 * (l4 | (p << 2)))) << 4);
  }
  return w;
}

// dma16 without its leading s_nop 2 (the wait states after the VALU readfirstlanes that wrote the
// descriptor): inside the main loop the descriptor is built before the half-step's first four
// MFMAs, so only the prologue's DMAs need the pad
__device__ __forceinline__ void w4_dma(const SRsrc& r, char* lds, int voff) {
  const uint32_t m = (uint32_t)(uintptr_t)LDS_PTR(char, lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r.v)
               : "memory");
}

template <bool PAD>
__device__ __forceinline__ void w4_dmap(const SRsrc& r, char* lds, int voff) {
  if (PAD) dma16(r, lds, voff);
  else w4_dma(r, lds, voff);
}

// this wave's DMA piece i (0..7) of the A / B operand tile of one stage
template <bool PAD = false>
__device__ __forceinline__ void w4_piece_a(char* img, const SRsrc& rs, const W4Lane& w, int lda, int wave, int i) {
  w4_dmap<PAD>(rs, img + (wave * 8 + i) * 1024, w.a_dma[i & 1] + (64 * wave + 8 * i) * lda * 2);
}
template <bool BKM, bool PAD = false>
__device__ __forceinline__ void w4_piece_b(char* img, const SRsrc& rs, const W4Lane& w, int ldb, int wave, int i) {
  if (BKM) {
    w4_dmap<PAD>(rs, img + 32768 + (wave * 8 + i) * 1024, w.b_dma[i & 1] + (64 * wave + 8 * i) * ldb * 2);
  } else {
    const int jj = (wave & 1) * 8 + i;
    w4_dmap<PAD>(rs, img + 32768 + (wave >> 1) * 16384 + jj * 1024,
           w.b_dma[(i >> 1) & 1] + 4 * jj * ldb * 2 + (wave >> 1) * 256);
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

// acc += B-fragment x A-fragment (16x16x32 bf16).  Inline asm with an AGPR "+a" operand keeps
// every accumulator in place in the AGPR file: with the builtin, the register allocator shuffles
// the 256 accumulators between AGPRs and VGPRs across the loop's back edge (hundreds of
// v_accvgpr moves per step).  Hazards the compiler does not see: accumulators are touched once
// per half-step (64 MFMAs apart), operands come straight from ds_read, and the epilogue's first
// AGPR read follows an explicit s_nop pad (w4_mfma_drain).
__device__ __forceinline__ void w4_mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ void w4_mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

// One half-step: 64 MFMAs on the current fragments (fa, fb), in 16 groups of 4; after each
// group's MFMAs one of the next half-step's 16 fragments is read from stage rst, k-half kk
// (READ) and DM of this wave's 16 DMA pieces of the stage after next are issued into dimg (DMA).
typedef __attribute__((ext_vector_type(16))) float w4f32x16;
__device__ __forceinline__ void w4_mfma32(w4f32x16& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

template <bool BKM, bool READ, bool DMA, int DM, int DMODE = 0, bool M32 = false>
__device__ __forceinline__ void w4_half(f32x4 (&acc)[2][8][4], w4f32x16 (&acc32)[16], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8],
                                        bf16x8 (&na)[8], bf16x8 (&nb)[8], const char* rst, int kk, const W4Lane& w,
                                        int wave, char* dimg, const SRsrc& ra, const SRsrc& rb, int lda, int ldb) {
  const char* pa = rst + w.a_rd[kk];
  const char* pb = rst + w.b_rd[kk];
  int sw = w.b_sw;
  asm volatile("" : "+v"(sw));  // keep the per-fragment swizzled addresses inside the loop
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int i = g >> 1, h = g & 1;
    if (M32) {  // timing experiment: 2 x 32x32x16 (64 cycles) in place of 4 x 16x16x32
      w4_mfma32(acc32[(2 * g) & 15], fb[(2 * g) & 7], fa[i]);
      w4_mfma32(acc32[(2 * g + 1) & 15], fb[(2 * g + 1) & 7], fa[i]);
    } else {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) w4_mfma(acc[h][i][jj], fb[h * 4 + jj], fa[i]);
    }
    if (READ) {
      if (g < 8) na[g] = w4_rd(pa + g * 2048);
      else if (BKM) nb[g - 8] = w4_rd(pb + (g - 8) * 2048);
      else nb[g - 8] = w4_rd_tr(pb + (((g - 8) << 5) ^ sw));
    }
    if (DMA && DMODE == 1) {  // timing experiment: M0 written once per half-step (wrong LDS targets)
      if (g == 0) {
        const uint32_t m = (uint32_t)(uintptr_t)LDS_PTR(char, dimg);
        asm volatile("s_nop 2\n\ts_mov_b32 m0, %0\n\ts_nop 0" ::"s"(m) : "memory");
      }
      const int voff = g < 8 ? w.a_dma[g & 1] + (64 * wave + 8 * g) * lda * 2 : w.b_dma[g & 1] + (64 * wave + 8 * (g - 8)) * ldb * 2;
      asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"((g < 8 ? ra : rb).v) : "memory");
    } else if (DMA) {
#pragma unroll
      for (int d = 0; d < DM; ++d) {
        const int q = g * DM + d;
        if (q == 0) w4_piece_a<true>(dimg, ra, w, lda, wave, q);
        else if (q < 8) w4_piece_a(dimg, ra, w, lda, wave, q);
        else if (q < 16) w4_piece_b<BKM>(dimg, rb, w, ldb, wave, q - 8);
      }
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

// ST (diagnostic build, variant 22): s_memtime stamps into LDS past the two stages, copied to
// p.dbg at the end: [0] kernel start, [1] main loop start, [2] main loop end, [3] kernel end,
// [4 + 2s] / [5 + 2s] step s's barrier entry / exit (s < 58), [126] / [127] s_memrealtime at
// kernel start / end (100 MHz).  Only lane 0 of each wave writes; the stamps' SMEM waits
// perturb the schedule a little (cdna_hip_programming.md §7, in-kernel stamps).
constexpr int W4_NST = 128;
__device__ __forceinline__ void w4_stamp(char* smem, int wave, int lane, int k, unsigned long long v) {
  if (lane == 0) *LDS_PTR(unsigned long long, smem + 2 * W4_STAGE + (wave * W4_NST + k) * 8) = v;
}

template <bool BKM, typename OutT, int EPI, int DM, bool ST = false, int NOLD = 0>
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
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;
  const int lda = (int)p.lda, ldb = (int)p.ldb;
  const W4Lane w = w4_lane<BKM>(wave, lane, p.lda, p.ldb);

  f32x4 acc[2][8][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  w4f32x16 acc32[16];  // timing experiment only (NOLD & 8)
  if (NOLD & 8) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc32[i] = w4f32x16{};
  }

  // prologue: stages 0 and 1 in flight, stage 0 waited for, first fragments read
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (s < ns) {
      char* img = smem + s * W4_STAGE;
      const SRsrc ra = srsrc256<true>(A, p.lda, m0, p.M, s * 64, K);
      const SRsrc rb = srsrc256<BKM>(B, p.ldb, n0, p.N, s * 64, K);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        w4_piece_a<true>(img, ra, w, lda, wave, i);
        w4_piece_b<BKM, true>(img, rb, w, ldb, wave, i);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (ns > 1) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (ns > 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = w4_rd(smem + w.a_rd[0] + i * 2048);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = BKM ? w4_rd(smem + w.b_rd[0] + j * 2048) : w4_rd_tr(smem + w.b_rd[0] + ((j << 5) ^ w.b_sw));
  }

  // One loop body for every step (a single code path keeps the 256 accumulators in place):
  // past the last stage the DMAs get an empty descriptor (the hardware's range check turns them
  // into zero writes of a stage nobody reads) and the reads fetch fragments nobody uses.
  unsigned long long st_loop = 0, st_a = 0, st_b = 0;
  if (ST) st_loop = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < ns; ++s) {
    char* img = smem + (s & 1) * W4_STAGE;
    char* nxt = smem + ((s + 1) & 1) * W4_STAGE;
    const SRsrc none = SRsrc{u32x4{0u, 0u, 0u, 0u}};
    // half 0: k 0-31 of stage s; read k 32-63 of stage s
    w4_half<BKM, !(NOLD & 2), false, DM, 0, (NOLD & 8) != 0>(acc, acc32, a0, b0, a1, b1, img, 1, w, wave, nullptr,
                                                           none, none, 0, 0);
    // stage s retired by every wave's reads, stage s + 1 landed
    if (ST) st_a = __builtin_amdgcn_s_memtime();
    w4_sync();
    if (ST) st_b = __builtin_amdgcn_s_memtime();
    // half 1: k 32-63 of stage s; read k 0-31 of stage s + 1; refill this stage with s + 2
    const bool more = s + 2 < ns;
    const SRsrc ra = w4_rsrc<true>(A, p.lda, m0, p.M, (s + 2) * 64, K, more);
    const SRsrc rb = w4_rsrc<BKM>(B, p.ldb, n0, p.N, (s + 2) * 64, K, more);
    w4_half<BKM, !(NOLD & 2), !(NOLD & 1), DM, (NOLD & 4) ? 1 : 0, (NOLD & 8) != 0>(acc, acc32, a1, b1, a0, b0, nxt, 0,
                                                                                  w, wave, img, ra, rb, lda, ldb);
    if (ST && s < 58) {
      w4_stamp(smem, wave, lane, 4 + 2 * s, st_a);
      w4_stamp(smem, wave, lane, 5 + 2 * s, st_b);
    }
  }
  // every wave passed the last step's barrier after its last LDS read and DMA: the stages are
  // idle, so the epilogue may stage rows in this wave's 16 KiB of them
  w4_mfma_drain();
  if (NOLD & 8) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" ::"a"(acc32[i]));
  }
  unsigned long long st_lend = 0;
  if (ST) st_lend = __builtin_amdgcn_s_memtime();
  char* st = smem + wave * 16384;
  finish256<OutT, EPI, true>(p, acc[0], m0 + wm * 128, n0 + wn * 128, lane, 0, st);
  finish256<OutT, EPI, true>(p, acc[1], m0 + wm * 128, n0 + wn * 128 + 64, lane, 0, st);
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


// Persistent form: one workgroup per CU walks tiles blockIdx' , blockIdx' + grid, ... (the same
// XCD-aware order as the one-tile kernel, round by round).  After a tile's main loop the next
// tile's first two stages are DMA'd into the (now idle) stage buffers BEFORE this tile's
// epilogue runs, so the next tile's prologue latency (~6.7k cycles per tile measured with
// tools/w4_stamps.py) hides behind the epilogue's stores; the epilogue stages its rows in the
// 32 KiB past the two stages (8 KiB per wave).  p.stagger > 0: half the workgroups of every XCD
// start p.stagger x s_sleep(127) later, desynchronising the CUs' epilogue store bursts.
template <bool BKM, typename OutT, int EPI>
__global__ __launch_bounds__(W4_THR, 1) void gemm_w4p_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = gridDim.x;
  int tile = xcd_remap(blockIdx.x, nwg);
  if (tile >= p.ntiles) return;
  const int K = p.K;
  const int ns = (K + 63) / 64;
  const bf16* A = (const bf16*)p.A;
  const bf16* B = (const bf16*)p.B;
  const int lda = (int)p.lda, ldb = (int)p.ldb;
  const W4Lane w = w4_lane<BKM>(wave, lane, p.lda, p.ldb);
  if (p.stagger > 0 && ((blockIdx.x >> 3) & 1)) {
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  auto prologue_dma = [&](int tl) {  // stages 0 and 1 of tile tl
    int tm, tn;
    tile_coords(p, tl, tm, tn);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      char* img = smem + s * W4_STAGE;
      const SRsrc ra = w4_rsrc<true>(A, p.lda, tm * BT, p.M, s * 64, K, s < ns);
      const SRsrc rb = w4_rsrc<BKM>(B, p.ldb, tn * BT, p.N, s * 64, K, s < ns);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        w4_piece_a<true>(img, ra, w, lda, wave, i);
        w4_piece_b<BKM, true>(img, rb, w, ldb, wave, i);
      }
    }
  };
  prologue_dma(tile);
  f32x4 acc[2][8][4];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  w4f32x16 acc32[16];  // unused (w4_half's timing-experiment operand)
  const SRsrc none = SRsrc{u32x4{0u, 0u, 0u, 0u}};
  while (true) {
    int tm, tn;
    tile_coords(p, tile, tm, tn);
    const int m0 = tm * BT, n0 = tn * BT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // this tile's stages 0 and 1 landed (every wave), the previous epilogue's LDS rows consumed
    w4_sync();
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = w4_rd(smem + w.a_rd[0] + i * 2048);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = BKM ? w4_rd(smem + w.b_rd[0] + j * 2048) : w4_rd_tr(smem + w.b_rd[0] + ((j << 5) ^ w.b_sw));
    for (int s = 0; s < ns; ++s) {
      char* img = smem + (s & 1) * W4_STAGE;
      char* nxt = smem + ((s + 1) & 1) * W4_STAGE;
      w4_half<BKM, true, false, 1>(acc, acc32, a0, b0, a1, b1, img, 1, w, wave, nullptr, none, none, 0, 0);
      w4_sync();
      const bool more = s + 2 < ns;
      const SRsrc ra = w4_rsrc<true>(A, p.lda, m0, p.M, (s + 2) * 64, K, more);
      const SRsrc rb = w4_rsrc<BKM>(B, p.ldb, n0, p.N, (s + 2) * 64, K, more);
      w4_half<BKM, true, true, 1>(acc, acc32, a1, b1, a0, b0, nxt, 0, w, wave, img, ra, rb, lda, ldb);
    }
    w4_mfma_drain();
    const int next = tile + nwg;
    // every wave's last useful stage read came before the last step's barrier (the final half-step's
    // reads fetch fragments nobody uses), so the next tile's prologue may overwrite both stages
    if (next < p.ntiles) prologue_dma(next);
    char* st = smem + 2 * W4_STAGE + wave * 8192;
    finish256<OutT, EPI, true>(p, acc[0], m0 + wm * 128, n0 + wn * 128, lane, 0, st);
    finish256<OutT, EPI, true>(p, acc[1], m0 + wm * 128, n0 + wn * 128 + 64, lane, 0, st);
    if (next >= p.ntiles) break;
    tile = next;
  }
}

template <bool BKM, int EPI>
void launch_w4p(const GemmP& p, hipStream_t s) {
  constexpr int L = 2 * W4_STAGE + 4 * 8192;
  (void)lds_optin((const void*)gemm_w4p_kernel<BKM, bf16, EPI>, L);
  const int grid = std::min(p.ntiles, num_cus_w4());
  hipLaunchKernelGGL((gemm_w4p_kernel<BKM, bf16, EPI>), dim3(grid), dim3(W4_THR), L, s, p);
}

template <bool BKM, int EPI>
void launch_w4(const GemmP& p, hipStream_t s, int dm) {
  if (dm == 100) {
    launch_w4p<BKM, EPI>(p, s);
    return;
  }
  if (dm < 0) {
    constexpr int L = 2 * W4_STAGE + 4 * W4_NST * 8;
#define W4_ST(n)                                                                                              \
  (void)lds_optin((const void*)gemm_w4_kernel<BKM, bf16, EPI, 1, true, n>, L);                               \
  hipLaunchKernelGGL((gemm_w4_kernel<BKM, bf16, EPI, 1, true, n>), dim3(p.ntiles), dim3(W4_THR), L, s, p)
    if (dm == -1) { W4_ST(0); }
    else if (dm == -2) { W4_ST(1); }
    else if (dm == -3) { W4_ST(2); }
    else if (dm == -4) { W4_ST(3); }
    else if (dm == -5) { W4_ST(4); }
    else { W4_ST(8); }
#undef W4_ST
    return;
  }
  if (dm == 2) {
    (void)lds_optin((const void*)gemm_w4_kernel<BKM, bf16, EPI, 2>, 2 * W4_STAGE);
    hipLaunchKernelGGL((gemm_w4_kernel<BKM, bf16, EPI, 2>), dim3(p.ntiles), dim3(W4_THR), 2 * W4_STAGE, s, p);
  } else {
    (void)lds_optin((const void*)gemm_w4_kernel<BKM, bf16, EPI, 1>, 2 * W4_STAGE);
    hipLaunchKernelGGL((gemm_w4_kernel<BKM, bf16, EPI, 1>), dim3(p.ntiles), dim3(W4_THR), 2 * W4_STAGE, s, p);
  }
}

}  // namespace

// forward (k-major B) and dgrad (row-major-in-k B) products with bf16 output and one of the
// CLIP path's epilogues; returns the profiler label, or nullptr when not covered.
const char* dispatch_w4(const GemmP& p, hipStream_t s, bool bkm, int flags, int dm) {
  constexpr int E_B = CLIPMI_EPI_BIAS, E_R = CLIPMI_EPI_RESID, E_Q = CLIPMI_EPI_QGELU;
  constexpr int E_P = CLIPMI_EPI_STORE_PRE, E_DQ = CLIPMI_EPI_DQGELU;
  if (bkm) {
    switch (flags) {
      case E_B: launch_w4<true, E_B>(p, s, dm); return "gemm256_fwd_bias";
      case E_B | E_R: launch_w4<true, E_B | E_R>(p, s, dm); return "gemm256_fwd_bias_resid";
      case E_B | E_Q | E_P: launch_w4<true, E_B | E_Q | E_P>(p, s, dm); return "gemm256_fwd_bias_qgelu_pre";
      case E_B | E_Q: launch_w4<true, E_B | E_Q>(p, s, dm); return "gemm256_fwd_bias_qgelu";
      case 0: launch_w4<true, 0>(p, s, dm); return "gemm256_fwd";
      default: return nullptr;
    }
  }
  switch (flags) {
    case 0: launch_w4<false, 0>(p, s, dm); return "gemm256_dgrad";
    case E_DQ: launch_w4<false, E_DQ>(p, s, dm); return "gemm256_dgrad_dqgelu";
    default: return nullptr;
  }
}

}  // namespace cmg
