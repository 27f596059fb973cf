// Device helpers shared by the bf16 GEMM translation units (gemm.hip, gemm4.hip):
// kernel parameters, tile rasterisation, LDS image layouts, LDS-DMA staging and the fused
// epilogues.  Everything here is inline; the kernels live in the .hip files.
#pragma once
#include "common.h"
#include "internal.h"
#include <algorithm>
#include <type_traits>

namespace cmg {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int E8_B = CLIPMI_EPI_BIAS, E8_R = CLIPMI_EPI_RESID, E8_Q = CLIPMI_EPI_QGELU;

struct GemmP {
  int M, N, K;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc;
  const void* bias; const void* res; int64_t ldr;
  void* aux; int64_t ldaux;
  float alpha; int flags; int bias_f32;
  int k_per_split; float* ws;
  int tiles_n, ntiles;
  int vec;  // all leading dimensions multiples of 4 elements
  int var;  // 256-kernel main-loop schedule (0 production)
  int vec8; // bf16 C with N, ldc/ldr/ldaux multiples of 8 and C/res/aux/bias 16-B aligned
  int stagger, first_round;  // s_sleep(127) count for half of the first round's workgroups
  const uint8_t* a_scale; const uint8_t* b_scale;  // MXFP8: E8M0 per 32-element k-block, [rows][K/32]
  uint8_t* c_scale;                                 // MXFP8 output: E8M0 per 32 columns, [M][N/32]
  int raster;  // 0: tiles row-major; g > 0: g tile-rows at a time, column by column (tile_coords)
  float* bws;  // split-K with a fused bias gradient: per-split partial sums [splits][M] (no atomics)
  unsigned long long* dbg;  // diagnostic builds only: in-kernel s_memtime stamps (clipmi_gemm_stamps)
  int* dyn;  // persistent 4-wave kernel: {next-item counter, finished-workgroup counter} (dynamic queue) or null
  // strided batch (clipmi_gemm_batched, f32 SIMT kernel only): blockIdx.z = i1 * nb2 + i2 offsets A / B / C by
  // i1 * s?1 + i2 * s?2 elements (nb2 == 0: no batch)
  int nb2;
  int64_t bsa1, bsa2, bsb1, bsb2, bsc1, bsc2;
  DeferredReduce red;  // persistent 4-wave kernel: a deferred reduction its workgroups run first (kind 0: none)
  // bf16x3 image output (clipmi_gemm_x3out, fp32-epilogue instances): 0 off, 1 pattern 0 (h, h, l), 2 pattern 1
  // (h, l, h); colp: per-128-row column partial sums of the fp32 result [ceil(M / 128)][N], or null
  int x3o;
  float* colp;
};

// host side: the stamp buffer armed by clipmi_gemm_stamps (nullptr when disarmed)
unsigned long long* gemm_stamp_buffer();

// tile -> (tm, tn).  Row-major, or grouped: g tile-rows at a time, walked column by column, so
// the ~32 tiles an XCD holds at once (its contiguous share of the XCD-remapped ids) share g A
// panels and a few B panels in its 4 MB L2 instead of streaming every B panel per tile-row.
__device__ __forceinline__ void tile_coords(const GemmP& p, int tile, int& tm, int& tn) {
  if (p.raster > 0) {
    const int g = p.raster, tiles_m = p.ntiles / p.tiles_n;
    const int grp = tile / (g * p.tiles_n);
    const int rem = tile - grp * g * p.tiles_n;
    const int rows = min(g, tiles_m - grp * g);
    tn = rem / rows;
    tm = grp * g + (rem - tn * rows);
  } else {
    tm = tile / p.tiles_n;
    tn = tile - tm * p.tiles_n;
  }
}

__device__ __forceinline__ float ld_bias(const GemmP& p, int n) {
  return p.bias_f32 ? ((const float*)p.bias)[n] : (float)((const bf16*)p.bias)[n];
}

// v holds C[m][n..n+3] before the epilogue; columns >= N are dropped.  Vector loads and
// stores when the 4 columns are in range and every leading dimension keeps them aligned.
template <typename OutT>
__device__ __forceinline__ void ld4(const OutT* p, float v[4], int nv, bool vec) {
  if (vec) { load4(p, v); return; }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = j < nv ? to_f32(p[j]) : 0.f;
}
template <typename OutT>
__device__ __forceinline__ void st4(OutT* p, const float v[4], int nv, bool vec) {
  if (vec) { store4(p, v); return; }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j < nv) p[j] = from_f32<OutT>(v[j]);
}

template <typename OutT, int EPI>
__device__ __forceinline__ void epilogue4(const GemmP& p, int m, int n, float v[4]) {
  const int f = EPI >= 0 ? EPI : p.flags;  // EPI >= 0: flags folded at compile time
  const int nv = min(4, p.N - n);
  const bool vec = p.vec && nv == 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] *= p.alpha;
  if (f & CLIPMI_EPI_BIAS) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += j < nv ? ld_bias(p, n + j) : 0.f;
  }
  if (f & CLIPMI_EPI_STORE_PRE) st4((OutT*)p.aux + (int64_t)m * p.ldaux + n, v, nv, vec);
  if (f & CLIPMI_EPI_STORE_DACT) {
    float d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = (f & CLIPMI_EPI_QGELU) ? quick_gelu_grad(v[j]) : gelu_erf_grad(v[j]);
    st4((OutT*)p.aux + (int64_t)m * p.ldaux + n, d, nv, vec);
  }
  if (f & CLIPMI_EPI_QGELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = quick_gelu(v[j]);
  } else if (f & CLIPMI_EPI_GELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = gelu_erf(v[j]);
  }
  if (f & (CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU)) {
    float a[4];
    ld4((const OutT*)p.aux + (int64_t)m * p.ldaux + n, a, nv, vec);
    if (f & CLIPMI_EPI_DQGELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= quick_gelu_grad(a[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= gelu_erf_grad(a[j]);
    }
  }
  if (f & CLIPMI_EPI_MUL_AUX) {
    float a[4];
    ld4((const OutT*)p.aux + (int64_t)m * p.ldaux + n, a, nv, vec);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= a[j];
  }
  if (f & CLIPMI_EPI_RESID) {
    float r[4];
    ld4((const OutT*)p.res + (int64_t)m * p.ldr + n, r, nv, vec);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += r[j];
  }
  OutT* c = (OutT*)p.C + (int64_t)m * p.ldc + n;
  if (f & CLIPMI_EPI_BETA) {
    float o[4];
    ld4(c, o, nv, vec);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += o[j];
  }
  st4(c, v, nv, vec);
}

// ---------------------------------------------------------------- LDS images
// k-major image: [128 rows][64 k] bf16, 128-B rows, 16-B chunk c stored at c ^ ((r>>1)&7)
__device__ __forceinline__ int kimg_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// row-major-in-k image: [64 k][128 rows] bf16, 256-B rows, chunk c stored at c ^ 2*g(r)
__device__ __forceinline__ int mimg_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }
__device__ __forceinline__ int mimg_off(int r, int c) { return r * 256 + ((c ^ mimg_swz(r)) << 4); }

// Global -> register staging of one 128x64 operand tile (4 x 16 B per thread).
template <bool KMAJ>
struct Stager {
  const bf16* base[4];  // per pass: k-major -> row start (+chunk), else column chunk start
  int lds_off[4];
  int chunk_k[4];       // k-major: element offset of the chunk within the K step; else k row
  __device__ __forceinline__ void init(const bf16* X, int64_t ld, int row0, int R, int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int id = i * NTHR + t;
      if (KMAJ) {
        int r = id >> 3, c = id & 7;
        int gr = min(row0 + r, R - 1);
        base[i] = X + (int64_t)gr * ld + c * 8;
        chunk_k[i] = c * 8;
        lds_off[i] = kimg_off(r, c);
      } else {
        int kr = id >> 4, c = id & 15;
        int gc = min(row0 + c * 8, R - 8);
        base[i] = X + (int64_t)kr * ld + gc;
        chunk_k[i] = kr;
        lds_off[i] = mimg_off(kr, c);
      }
    }
  }
  __device__ __forceinline__ void load(u32x4 v[4], int k0, int64_t ld, int kvalid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16* g = KMAJ ? base[i] + k0 : base[i] + (int64_t)k0 * ld;
      if (kvalid >= BK || chunk_k[i] < kvalid) v[i] = *(const u32x4*)g;
      else v[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(char* lds, const u32x4 v[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *LDS_PTR(u32x4, lds + lds_off[i]) = v[i];
  }
};

// One 16x32 MFMA operand fragment: rows rb..rb+15 of the tile, k = kk*32 .. kk*32+31.
template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rb, int kk, int lane) {
  if (KMAJ) {
    int r = rb + (lane & 15), c = kk * 4 + (lane >> 4);
    return *LDS_PTR(const bf16x8, lds + kimg_off(r, c));
  } else {
    int q = (lane & 15) >> 2, p4 = lane & 3;
    int m = rb + 4 * p4;
    int r0 = kk * 32 + 8 * (lane >> 4) + q;
    int r1 = r0 + 4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(s16x4, lds + mimg_off(r0, m >> 3) + (m & 7) * 2));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(s16x4, lds + mimg_off(r1, m >> 3) + (m & 7) * 2));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, w);
  }
}

// ------------------------------------------------------------------ 256x256 LDS-DMA path
// 512 threads = 8 waves (2 along M x 4 along N), each wave 128x64 = 8x4 MFMA tiles
// (128 accumulator VGPRs).  Tiles arrive by LDS-DMA (buffer_load ... lds, 16 B per lane,
// 1 KiB per wave-instruction): the LDS images are lane-linear, so the XOR swizzle is
// applied to the per-lane SOURCE address and undone by the same read-side swizzle as the
// 128 kernel.  Two 64 KiB buffers: the DMA of k-step t+1 is in flight while k-step t's
// 64 MFMAs per wave run; one vmcnt(0) + barrier per k-step.  Buffer descriptors are
// rebuilt per k-step at the slab start with exact byte extents, so rows past M/N/K read
// as zero (no clamping, no branches) and offsets stay 32-bit for any tensor size.
// BIASGRAD (wgrad only): waves with wn == 0 of n-tile 0 add one MFMA per A fragment
// against a ones fragment, producing sum_k A(m,k) = the Linear bias gradient.
constexpr int BT = 256, NT2 = 512;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0, 0);
}
// stage one 256x64 operand tile of k-step at k0 into an LDS image (32 KiB)
template <bool KMAJ>
__device__ __forceinline__ void stage256(char* img, const bf16* X, int64_t ld, int row0, int R, int k0, int K,
                                         int wave, int lane) {
  if (KMAJ) {
    // rows row0.. (<=256 valid), k0..k0+63; each wave-instruction fills 8 rows x 128 B
    const int rows = min(BT, R - row0);
    const bf16* base = X + (int64_t)row0 * ld + k0;
    const uint32_t rec = rows > 0 ? (uint32_t)((int64_t)(rows - 1) * ld * 2 + 128) : 0u;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, rec, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wave * 4 + i;
      const int r = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      dma16(rs, img + j * 1024, (int)((int64_t)r * ld * 2 + c * 16));
    }
  } else {
    // k rows k0..k0+63 (<= K), columns row0..row0+255 as two 128-wide half images [64][128]
    const int krows = min(64, K - k0);
    const int cols = min(BT, R - row0);
    const bf16* base = X + (int64_t)k0 * ld + row0;
    const uint32_t rec = krows > 0 ? (uint32_t)((int64_t)(krows - 1) * ld * 2 + (int64_t)cols * 2) : 0u;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, rec, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wave * 4 + i;            // 0..31
      const int half = j >> 4;
      const int kr = 4 * (j & 15) + (lane >> 4);
      const int c = (lane & 15) ^ mimg_swz(kr);
      dma16(rs, img + half * 16384 + (j & 15) * 1024, (int)((int64_t)kr * ld * 2 + (half * 128 + c * 8) * 2));
    }
  }
}

// issue DMA instruction i (0..3) of this wave for one operand tile (same addressing as stage256)
template <bool KMAJ, typename RS>
__device__ __forceinline__ void stage256_one(char* img, RS rs, int64_t ld, int wave, int lane, int i) {
  const int j = wave * 4 + i;
  if (KMAJ) {
    const int r = 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    dma16(rs, img + j * 1024, (int)((int64_t)r * ld * 2 + c * 16));
  } else {
    const int half = j >> 4;
    const int kr = 4 * (j & 15) + (lane >> 4);
    const int c = (lane & 15) ^ mimg_swz(kr);
    dma16(rs, img + half * 16384 + (j & 15) * 1024, (int)((int64_t)kr * ld * 2 + (half * 128 + c * 8) * 2));
  }
}
template <bool KMAJ>
__device__ __forceinline__ void extent256(const bf16* X, int64_t ld, int row0, int R, int k0, int K, const bf16*& base,
                                          uint32_t& rec) {
  if (KMAJ) {
    const int rows = min(BT, R - row0);
    base = X + (int64_t)row0 * ld + k0;
    rec = rows > 0 ? (uint32_t)((int64_t)(rows - 1) * ld * 2 + 128) : 0u;
  } else {
    const int krows = min(64, K - k0);
    const int cols = min(BT, R - row0);
    base = X + (int64_t)k0 * ld + row0;
    rec = krows > 0 ? (uint32_t)((int64_t)(krows - 1) * ld * 2 + (int64_t)cols * 2) : 0u;
  }
}
template <bool KMAJ>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc256(const bf16* X, int64_t ld, int row0, int R, int k0, int K) {
  const bf16* base; uint32_t rec;
  extent256<KMAJ>(X, ld, row0, R, k0, K, base, rec);
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, rec, 0x00020000);
}
template <bool KMAJ>
__device__ __forceinline__ SRsrc srsrc256(const bf16* X, int64_t ld, int row0, int R, int k0, int K) {
  const bf16* base; uint32_t rec;
  extent256<KMAJ>(X, ld, row0, R, k0, K, base, rec);
  return make_srsrc(base, rec);
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag256(const char* img, int rb, int kk, int lane) {
  if (KMAJ) return read_frag<true>(img, rb, kk, lane);
  return read_frag<false>(img + (rb >> 7) * 16384, rb & 127, kk, lane);
}

// AR (accumulators pinned in AGPRs by inline-asm MFMAs, gemm4.hip): an empty asm that needs the
// fragment in its AGPRs right before its first use, so the compiler copies accumulators to VGPRs
// one fragment at a time instead of all 256 at once after the main loop (which spills)
template <bool AR>
__device__ __forceinline__ void acc_pin(f32x4& a) {
  if constexpr (AR) asm volatile("" : "+a"(a));
}

// Batched epilogue for the 256 kernel (vectorisable case): bias preloaded once per lane,
// residual / pre-activation / old-C vectors for half the tile loaded in one burst (clamped
// addresses, no per-element branches), then computed and stored.  The per-subtile
// load->wait->store chain it replaces left the K=768 GEMMs epilogue-latency bound.
template <typename OutT, int EPI, bool AR = false>
__device__ __forceinline__ void epilogue256(const GemmP& p, f32x4 (&acc)[8][4], int mb, int nb, int lane) {
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU, HG = EPI & CLIPMI_EPI_GELU;
  constexpr bool HR = EPI & CLIPMI_EPI_RESID, HDQ = EPI & CLIPMI_EPI_DQGELU, HDG = EPI & CLIPMI_EPI_DGELU;
  constexpr bool HBETA = EPI & CLIPMI_EPI_BETA, HPRE = EPI & CLIPMI_EPI_STORE_PRE;
  constexpr bool HAUX = HDQ || HDG;
  const int nlane = (lane >> 4) * 4, mlane = lane & 15;
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = min(nb + j * 16 + nlane, p.N - 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
    if (HB) {
      if (p.bias_f32) load4((const float*)p.bias + n, bv[j]);
      else load4((const bf16*)p.bias + n, bv[j]);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float xin[4][4][4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int m = min(mb + (h * 4 + ii) * 16 + mlane, p.M - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = min(nb + j * 16 + nlane, p.N - 4);
        if (HR) load4((const OutT*)p.res + (int64_t)m * p.ldr + n, xin[ii][j]);
        else if (HAUX) load4((const OutT*)p.aux + (int64_t)m * p.ldaux + n, xin[ii][j]);
        else if (HBETA) load4((const OutT*)p.C + (int64_t)m * p.ldc + n, xin[ii][j]);
      }
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = h * 4 + ii;
      const int m = mb + i * 16 + mlane;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nb + j * 16 + nlane;
        float v[4];
        acc_pin<AR>(acc[i][j]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][j][r] * p.alpha + bv[j][r];
        }
        const bool ok = m < p.M && n < p.N;
        if (HPRE && ok) store4((OutT*)p.aux + (int64_t)m * p.ldaux + n, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (HQ) v[r] = quick_gelu(v[r]);
          if (HG) v[r] = gelu_erf(v[r]);
          if (HDQ) v[r] *= quick_gelu_grad(xin[ii][j][r]);
          if (HDG) v[r] *= gelu_erf_grad(xin[ii][j][r]);
          if (HR || HBETA) v[r] += xin[ii][j][r];
        }
        if (ok) store4((OutT*)p.C + (int64_t)m * p.ldc + n, v);
      }
    }
  }
}

// 8 consecutive bf16 as float (one 16-B access)
__device__ __forceinline__ void load8(const bf16* p, float v[8]) {
  const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = (float)t[r];
}
__device__ __forceinline__ void store8(bf16* p, const float v[8]) {
  *(bf16x8*)p = bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
}

// bf16-output epilogue with 16-B accesses (cdna_hip_programming.md T21, 16-lane form).  The
// 16x16 accumulator layout gives a lane 4 consecutive columns per fragment, i.e. 8-B stores of
// 16 rows x 32 B per instruction, and those epilogues were store-issue bound.  One
// v_permlane16_swap per accumulator dword pairs fragments (2jp, 2jp+1): afterwards lane
// row-group q = lane>>4 holds 8 consecutive columns, fragment 2jp + (q & 1), columns
// 8*(q >> 1) .. +7, so every residual/aux load and every store is one 16-B access covering
// 16 rows x 64 B per instruction: half the memory instructions for the same bytes.
template <int EPI, bool AR = false, int NI = 8>
__device__ __forceinline__ void epilogue256_w(const GemmP& p, f32x4 (&acc)[NI][4], int mb, int nb, int lane) {
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU, HG = EPI & CLIPMI_EPI_GELU;
  constexpr bool HR = EPI & CLIPMI_EPI_RESID, HDQ = EPI & CLIPMI_EPI_DQGELU, HDG = EPI & CLIPMI_EPI_DGELU;
  constexpr bool HBETA = EPI & CLIPMI_EPI_BETA, HPRE = EPI & CLIPMI_EPI_STORE_PRE;
  constexpr bool HAUX = HDQ || HDG;
  const int q = lane >> 4, mlane = lane & 15;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);  // this lane's column within a fragment pair
  float bv[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const int n = min(nb + 32 * jp + coff, p.N - 8);
#pragma unroll
    for (int r = 0; r < 8; ++r) bv[jp][r] = 0.f;
    if (HB) {
      if (p.bias_f32) {
        load4((const float*)p.bias + n, bv[jp]);
        load4((const float*)p.bias + n + 4, bv[jp] + 4);
      } else {
        load8((const bf16*)p.bias + n, bv[jp]);
      }
    }
  }
  constexpr int NH = NI >= 4 ? NI / 4 : 1, NII = NI >= 4 ? 4 : NI;  // row fragments in groups of <= 4
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    float xin[NII][2][8];
    if (HR || HAUX || HBETA) {
#pragma unroll
      for (int ii = 0; ii < NII; ++ii) {
        const int m = min(mb + (h * NII + ii) * 16 + mlane, p.M - 1);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int n = min(nb + 32 * jp + coff, p.N - 8);
          if (HR) load8((const bf16*)p.res + (int64_t)m * p.ldr + n, xin[ii][jp]);
          else if (HAUX) load8((const bf16*)p.aux + (int64_t)m * p.ldaux + n, xin[ii][jp]);
          else load8((const bf16*)p.C + (int64_t)m * p.ldc + n, xin[ii][jp]);
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < NII; ++ii) {
      const int i = h * NII + ii;
      const int m = mb + i * 16 + mlane;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = nb + 32 * jp + coff;
        float v[8];
        acc_pin<AR>(acc[i][2 * jp]);
        acc_pin<AR>(acc[i][2 * jp + 1]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // swapped right before use: no extra live registers
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                           __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
          v[r] = __uint_as_float(sw[0]) * p.alpha + bv[jp][r];
          v[r + 4] = __uint_as_float(sw[1]) * p.alpha + bv[jp][r + 4];
        }
        const bool ok = m < p.M && n < p.N;
        if (HPRE && ok) store8((bf16*)p.aux + (int64_t)m * p.ldaux + n, v);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (HQ) v[r] = quick_gelu(v[r]);
          if (HG) v[r] = gelu_erf(v[r]);
          if (HDQ) v[r] *= quick_gelu_grad(xin[ii][jp][r]);
          if (HDG) v[r] *= gelu_erf_grad(xin[ii][jp][r]);
          if (HR || HBETA) v[r] += xin[ii][jp][r];
        }
        if (ok) store8((bf16*)p.C + (int64_t)m * p.ldc + n, v);
      }
    }
  }
}

// Full-line stores through LDS: the values of epilogue256_w (same math, same loads) are written
// to the wave's 16 KiB LDS region as a [128 rows][64 cols] bf16 tile (16-B chunk c of row r at
// c ^ (r & 7): conflict-free 8-lane writes and 16-lane reads), then read back row-contiguous so
// each global store instruction covers 8 whole 128-B rows instead of 16 rows x 64 B.  Needs
// the ring idle (after the kernel's final barrier) and is used for the pre-activation store too.
__device__ __forceinline__ int stage_off(int r, int c8) { return r * 128 + ((c8 ^ (r & 7)) << 4); }

__device__ __forceinline__ void stage_store_rows(const GemmP& p, const char* st, bf16* out, int64_t ld, int mb, int nb,
                                                 int lane) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {  // 64 rows, 8 whole rows per instruction
    const int r = it * 8 + (lane >> 3), c8 = lane & 7;
    const u32x4 v = *LDS_PTR(const u32x4, st + stage_off(r, c8));
    const int m = mb + r, n = nb + c8 * 8;
    if (m < p.M && n < p.N) *(u32x4*)(out + (int64_t)m * ld + n) = v;
  }
}

template <int EPI, bool AR = false>
__device__ __forceinline__ void epilogue256_lds(const GemmP& p, f32x4 (&acc)[8][4], int mb, int nb, int lane,
                                                char* st) {
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU, HG = EPI & CLIPMI_EPI_GELU;
  constexpr bool HR = EPI & CLIPMI_EPI_RESID, HDQ = EPI & CLIPMI_EPI_DQGELU, HDG = EPI & CLIPMI_EPI_DGELU;
  constexpr bool HBETA = EPI & CLIPMI_EPI_BETA, HPRE = EPI & CLIPMI_EPI_STORE_PRE;
  constexpr bool HAUX = HDQ || HDG;
  const int q = lane >> 4, mlane = lane & 15;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);
  char* st_out = st;  // [64 rows][64 cols] bf16 = 8 KiB per half of the wave's rows
  float bv[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const int n = min(nb + 32 * jp + coff, p.N - 8);
#pragma unroll
    for (int r = 0; r < 8; ++r) bv[jp][r] = 0.f;
    if (HB) {
      if (p.bias_f32) {
        load4((const float*)p.bias + n, bv[jp]);
        load4((const float*)p.bias + n + 4, bv[jp] + 4);
      } else {
        load8((const bf16*)p.bias + n, bv[jp]);
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float xin[4][2][8];
    if (HR || HAUX || HBETA) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int m = min(mb + (h * 4 + ii) * 16 + mlane, p.M - 1);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int n = min(nb + 32 * jp + coff, p.N - 8);
          if (HR) load8((const bf16*)p.res + (int64_t)m * p.ldr + n, xin[ii][jp]);
          else if (HAUX) load8((const bf16*)p.aux + (int64_t)m * p.ldaux + n, xin[ii][jp]);
          else load8((const bf16*)p.C + (int64_t)m * p.ldc + n, xin[ii][jp]);
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = h * 4 + ii;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        float v[8];
        acc_pin<AR>(acc[i][2 * jp]);
        acc_pin<AR>(acc[i][2 * jp + 1]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                           __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
          v[r] = __uint_as_float(sw[0]) * p.alpha + bv[jp][r];
          v[r + 4] = __uint_as_float(sw[1]) * p.alpha + bv[jp][r + 4];
        }
        const int off = stage_off(ii * 16 + mlane, (32 * jp + coff) >> 3);
        if (HPRE) {  // the pre-activation goes out directly (16 rows x 64 B), overlapping the gelu math
          const int m = mb + i * 16 + mlane, n = nb + 32 * jp + coff;
          if (m < p.M && n < p.N) store8((bf16*)p.aux + (int64_t)m * p.ldaux + n, v);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (HQ) v[r] = quick_gelu(v[r]);
          if (HG) v[r] = gelu_erf(v[r]);
          if (HDQ) v[r] *= quick_gelu_grad(xin[ii][jp][r]);
          if (HDG) v[r] *= gelu_erf_grad(xin[ii][jp][r]);
          if (HR || HBETA) v[r] += xin[ii][jp][r];
        }
        *LDS_PTR(bf16x8, st_out + off) = bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3],
                                                (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staging writes landed
    stage_store_rows(p, st_out, (bf16*)p.C, p.ldc, mb + h * 64, nb, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next half overwrites
  }
}

#ifndef CLIPMI_EPI_PD
#define CLIPMI_EPI_PD 4
#endif
// 16-B output store of the LDS-staged epilogues; CLIPMI_STORE_NT=1 (A/B builds) makes it non-temporal
#ifndef CLIPMI_STORE_NT
#define CLIPMI_STORE_NT 0
#endif
__device__ __forceinline__ void st16_out(u32x4* p, const u32x4& v) {
#if CLIPMI_STORE_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
// 8 bf16 packed in 4 dwords -> float (element 2i in the low half of dword i)
__device__ __forceinline__ void unpack8(const u32x4& x, float v[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(x[i] << 16);
    v[2 * i + 1] = __uint_as_float(x[i] & 0xffff0000u);
  }
}

// Pipelined form of epilogue256_lds over a wave's NC adjacent 128x64 blocks (NC = 1: the 8-wave
// kernels' block, NC = 2: the 4-wave kernel's 128x128), in parts of 64 rows x 64 columns, each
// staged through the wave's 8 KiB of LDS.  Same math and rounding as epilogue256_lds.  Measured
// problem it removes (profiles/r03_epilogue_isa.txt, in-kernel stamps): a part's store chain was
// ds_read -> s_waitcnt lgkmcnt(0) -> global_store per instruction, and every input load issued
// after a store waited for that store's write acknowledgement (vmcnt counts loads and stores in
// issue order), so the epilogue ran ~9 B/clk per CU whether 60 or 256 CUs were storing.  Here:
//  * every bias value is loaded once, before any store, and each part's residual / pre-activation
//    / old-C inputs are loaded before the previous part's stores (double-buffered raw registers);
//  * a part's 8 staged row groups are read back in one batch, then stored;
//  * full tiles (every CLIP shape) store with no per-row exec branches.
template <int EPI, bool AR, int NC>
__device__ __forceinline__ void epilogue_lds_pipe(const GemmP& p, f32x4 (&acc)[NC][8][4], int mb, int nb, int lane,
                                                  char* st) {
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU, HG = EPI & CLIPMI_EPI_GELU;
  constexpr bool HR = EPI & CLIPMI_EPI_RESID, HDQ = EPI & CLIPMI_EPI_DQGELU, HDG = EPI & CLIPMI_EPI_DGELU;
  constexpr bool HBETA = EPI & CLIPMI_EPI_BETA, HPRE = EPI & CLIPMI_EPI_STORE_PRE;
  constexpr bool HDA = EPI & CLIPMI_EPI_STORE_DACT, HMA = EPI & CLIPMI_EPI_MUL_AUX;
  constexpr bool HAUX = HDQ || HDG || HMA;
  constexpr bool HIN = HR || HAUX || HBETA;
  constexpr bool H2 = HPRE || HDA;  // a second output (aux), staged through LDS after the first
  // one input stream (xin: res, else aux, else C) and one aux role per instance
  static_assert(!(HMA && (HR || HBETA)), "MUL_AUX with RESID / BETA would read one input for both");
  static_assert(!(HPRE && HDA), "STORE_PRE and STORE_DACT both write aux");
  static_assert(!(HAUX && H2), "aux is either read or written");
  constexpr int NPART = 2 * NC;
  const int q = lane >> 4, mlane = lane & 15;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);
  const bool full = mb + 128 <= p.M && nb + 64 * NC <= p.N;
  float bv[NC][2][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int n = min(nb + 64 * c + 32 * jp + coff, p.N - 8);
#pragma unroll
      for (int r = 0; r < 8; ++r) bv[c][jp][r] = 0.f;
      if (HB) {
        if (p.bias_f32) {
          load4((const float*)p.bias + n, bv[c][jp]);
          load4((const float*)p.bias + n + 4, bv[c][jp] + 4);
        } else {
          load8((const bf16*)p.bias + n, bv[c][jp]);
        }
      }
    }
  const bf16* src = HR ? (const bf16*)p.res : HAUX ? (const bf16*)p.aux : (const bf16*)p.C;
  const int64_t lds_in = HR ? p.ldr : HAUX ? p.ldaux : p.ldc;
  // inputs PD parts ahead (default: every part, issued before the first store)
  constexpr int PD = CLIPMI_EPI_PD > 0 ? (CLIPMI_EPI_PD < NPART ? CLIPMI_EPI_PD : NPART) : NPART;
  u32x4 xr[PD][4][2];
  auto load_in = [&](int part, u32x4 (&x)[4][2]) {
    const int c = part >> 1, h = part & 1;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int m = min(mb + (h * 4 + ii) * 16 + mlane, p.M - 1);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = min(nb + 64 * c + 32 * jp + coff, p.N - 8);
        x[ii][jp] = *(const u32x4*)(src + (int64_t)m * lds_in + n);
      }
    }
  };
  if (HIN) {
#pragma unroll
    for (int q = 0; q < PD; ++q) load_in(q, xr[q]);
  }
#pragma unroll
  for (int part = 0; part < NPART; ++part) {
    const int c = part >> 1, h = part & 1;
    u32x4 aux2[4][2];  // the part's second output (pre-activation or its derivative), packed bf16
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = h * 4 + ii;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        float v[8];
        // AGPR accumulators (4-wave kernel): a scheduling fence per fragment pair instead of
        // acc_pin, whose "+a" redefinition made the compiler copy every pair into a0..a7 before
        // reading it (56 v_accvgpr_mov per part); the fence alone keeps the reads in place, unspilled
        if constexpr (AR) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[c][i][2 * jp][r]),
                                                           __float_as_uint(acc[c][i][2 * jp + 1][r]), false, false);
          v[r] = __uint_as_float(sw[0]) * p.alpha + bv[c][jp][r];
          v[r + 4] = __uint_as_float(sw[1]) * p.alpha + bv[c][jp][r + 4];
        }
        float xin[8], w2[8];
        if (HIN) unpack8(xr[part % PD][ii][jp], xin);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (HPRE) w2[r] = v[r];
          if (HQ) {
            const float sg = qg_sigmoid(v[r]);  // one exp + rcp for quick_gelu and its derivative
            if (HDA) {  // s + 1.702 x s (1 - s) = s (1 + t - t s), t = 1.702 x
              const float tq = 1.702f * v[r];
              w2[r] = fmaf(sg, fmaf(-tq, sg, tq), sg);
            }
            v[r] *= sg;
          }
          if (HG) {
            if (HDA) w2[r] = gelu_erf_grad(v[r]);
            v[r] = gelu_erf(v[r]);
          }
          if (HDQ) v[r] *= quick_gelu_grad(xin[r]);
          if (HDG) v[r] *= gelu_erf_grad(xin[r]);
          if (HMA) v[r] *= xin[r];
          if (HR || HBETA) v[r] += xin[r];
        }
        if (H2)
          aux2[ii][jp] = __builtin_bit_cast(u32x4, bf16x8{(bf16)w2[0], (bf16)w2[1], (bf16)w2[2], (bf16)w2[3],
                                                           (bf16)w2[4], (bf16)w2[5], (bf16)w2[6], (bf16)w2[7]});
        *LDS_PTR(bf16x8, st + stage_off(ii * 16 + mlane, (32 * jp + coff) >> 3)) =
            bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
      }
    }
    if (HIN && part + PD < NPART) load_in(part + PD, xr[part % PD]);  // before this part's stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                    // this wave's staging writes landed
    u32x4 o[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) o[it] = *LDS_PTR(const u32x4, st + stage_off(it * 8 + (lane >> 3), lane & 7));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read back before the next part overwrites
    if (H2) {  // the second output into the staging buffer, now that its read-back landed
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) *LDS_PTR(u32x4, st + stage_off(ii * 16 + mlane, (32 * jp + coff) >> 3)) = aux2[ii][jp];
    }
    const int r0 = mb + h * 64 + (lane >> 3), col = nb + 64 * c + (lane & 7) * 8;
    auto store_rows = [&](bf16* base, int64_t ld, const u32x4 (&rows)[8]) {
      bf16* out = base + (int64_t)r0 * ld + col;
      const int64_t step = 8 * ld;
      if (full) {
#pragma unroll
        for (int it = 0; it < 8; ++it) st16_out((u32x4*)(out + it * step), rows[it]);
      } else {
#pragma unroll
        for (int it = 0; it < 8; ++it)
          if (r0 + it * 8 < p.M && col < p.N) st16_out((u32x4*)(out + it * step), rows[it]);
      }
    };
    store_rows((bf16*)p.C, p.ldc, o);
    if (H2) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 8; ++it) o[it] = *LDS_PTR(const u32x4, st + stage_off(it * 8 + (lane >> 3), lane & 7));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      store_rows((bf16*)p.aux, p.ldaux, o);
    }
  }
}

// bf16x3 mode (engine.cpp encoder_*_x3): the fp32 result v of the epilogue leaves as its split image instead of
// fp32 -- C bf16 [M][ldc], segments at columns n, N + n, 2N + n: (h, h, l) for x3o == 1 (pattern 0, a forward
// activation) or (h, l, h) for x3o == 2 (pattern 1, an activation gradient), h = bf16(v), l = bf16(v - h): the
// layout and rounding of clipmi_split3_colsum, so the producer's fp32 copy and the split pass over it disappear.
// STORE_DACT's derivative stays fp32 (aux), MUL_AUX reads fp32 aux.  With p.colp (pattern 1: the bias gradient of
// the Linear this is the output gradient of) the column sums of v over the wave's 128 rows go to
// colp[(mb >> 7) * N + n] (rows in order per lane, then a fixed xor tree over the 16 row lanes: deterministic).
// Register layout as epilogue256_w: after v_permlane16_swap lane (q, mlane) holds row mb + 16 i + mlane, columns
// nb + 32 jp + coff .. + 7.  N % 8 == 0, ldc % 8 == 0, C 16-B aligned, aux fp32 16-B aligned (host-checked).
template <int EPI, bool AR = false>
__device__ __forceinline__ void epilogue_x3img(const GemmP& p, f32x4 (&acc)[8][4], int mb, int nb, int lane) {
  // no fma contraction: l = bf16(v - h) of the ROUNDED v (a contracted v * s - h would split the unrounded product
  // and differ from clipmi_split3_colsum's image of the stored fp32 result in l's last bit for ~1 % of elements)
#pragma clang fp contract(off)
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU;
  constexpr bool HDA = EPI & CLIPMI_EPI_STORE_DACT, HMA = EPI & CLIPMI_EPI_MUL_AUX;
  const int q = lane >> 4, mlane = lane & 15;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);
  const int64_t seg = p.N;
  const bool p1 = p.x3o == 2;
  float bv[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const int n = min(nb + 32 * jp + coff, p.N - 8);
#pragma unroll
    for (int r = 0; r < 8; ++r) bv[jp][r] = 0.f;
    if (HB) {
      if (p.bias_f32) {
        load4((const float*)p.bias + n, bv[jp]);
        load4((const float*)p.bias + n + 4, bv[jp] + 4);
      } else {
        load8((const bf16*)p.bias + n, bv[jp]);
      }
    }
  }
  float cs[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int r = 0; r < 8; ++r) cs[jp][r] = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float xin[4][2][8];
    if (HMA) {  // the half's aux rows in one burst (clamped addresses), before its stores
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int m = min(mb + (h * 4 + ii) * 16 + mlane, p.M - 1);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const float* a = (const float*)p.aux + (int64_t)m * p.ldaux + min(nb + 32 * jp + coff, p.N - 8);
          load4(a, xin[ii][jp]);
          load4(a + 4, xin[ii][jp] + 4);
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = h * 4 + ii;
      const int m = mb + i * 16 + mlane;
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int n = nb + 32 * jp + coff;
        float v[8], w2[8];
        // AGPR accumulators (4-wave kernel): a scheduling fence per fragment pair, as epilogue_lds_pipe
        if constexpr (AR) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                           __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
          v[r] = __uint_as_float(sw[0]) * p.alpha + bv[jp][r];
          v[r + 4] = __uint_as_float(sw[1]) * p.alpha + bv[jp][r + 4];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (HQ) {
            const float sg = qg_sigmoid(v[r]);
            if (HDA) {  // s + 1.702 x s (1 - s), as epilogue_lds_pipe
              const float tq = 1.702f * v[r];
              w2[r] = fmaf(sg, fmaf(-tq, sg, tq), sg);
            }
            v[r] *= sg;
          }
          if (HMA) v[r] *= xin[ii][jp][r];
        }
        if (m < p.M && n < p.N) {
          if (HDA) {
            float* a = (float*)p.aux + (int64_t)m * p.ldaux + n;
            store4(a, w2);
            store4(a + 4, w2 + 4);
          }
          bf16x8 hi, lo;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            hi[r] = (bf16)v[r];
            lo[r] = (bf16)(v[r] - (float)hi[r]);
            cs[jp][r] += v[r];
          }
          bf16* o = (bf16*)p.C + (int64_t)m * p.ldc + n;
          *(bf16x8*)o = hi;
          *(bf16x8*)(o + seg) = p1 ? lo : hi;
          *(bf16x8*)(o + 2 * seg) = p1 ? hi : lo;
        }
      }
    }
  }
  if (p.colp && mb < p.M) {
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) cs[jp][r] += __shfl_xor(cs[jp][r], o, 64);
      }
      const int n = nb + 32 * jp + coff;
      if (mlane == 0 && n < p.N) {
        float* c = p.colp + (int64_t)(mb >> 7) * p.N + n;
        store4(c, cs[jp]);
        store4(c + 4, cs[jp] + 4);
      }
    }
  }
}

// Store a wave's 128x64 accumulator block: the specialised batched epilogue when the shape
// allows it (4-aligned columns, aligned leading dims; the 16-B form for bf16 output when
// columns, leading dims and pointers allow 16-B accesses), else the per-subtile generic path
// (split-K slab kz, ragged N, runtime flags).
template <typename OutT, int EPI, bool AR = false>
__device__ __forceinline__ void finish256(const GemmP& p, f32x4 (&acc)[8][4], int mb, int nb, int lane, int kz,
                                          char* stage = nullptr) {
  constexpr bool FAST = EPI >= 0 && !((EPI & CLIPMI_EPI_RESID) && (EPI & (CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU))) &&
                        !((EPI & CLIPMI_EPI_BETA) && (EPI & (CLIPMI_EPI_RESID | CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU)));
  // bf16x3 image output (clipmi_gemm_x3out): the fp32-output instances of fc1 (bias + quick_gelu, with or
  // without the stored derivative) and of fc2's input gradient (the stored-derivative product)
  constexpr int X3E = EPI & ~CLIPMI_EPI_STORE_DACT;
  if constexpr (std::is_same<OutT, float>::value &&
                (X3E == (CLIPMI_EPI_BIAS | CLIPMI_EPI_QGELU) || EPI == CLIPMI_EPI_MUL_AUX)) {
    if (p.x3o) {
      epilogue_x3img<EPI, AR>(p, acc, mb, nb, lane);
      return;
    }
  }
  // the derivative-store / aux-product flags have a fast form only in the pipelined LDS epilogue
  constexpr bool NEWF = EPI >= 0 && (EPI & (CLIPMI_EPI_STORE_DACT | CLIPMI_EPI_MUL_AUX));
  if constexpr (NEWF) {
#if !CLIPMI_OLD_EPI
    if constexpr (std::is_same<OutT, bf16>::value) {
      if (stage && !p.ws && p.vec8) {
        epilogue_lds_pipe<EPI, AR, 1>(p, reinterpret_cast<f32x4(&)[1][8][4]>(acc), mb, nb, lane, stage);
        return;
      }
    }
#endif
  } else if constexpr (FAST && std::is_same<OutT, bf16>::value) {
    if (stage && !p.ws && p.vec8) {
#if CLIPMI_OLD_EPI
      epilogue256_lds<EPI < 0 ? 0 : EPI, AR>(p, acc, mb, nb, lane, stage);
#else
      epilogue_lds_pipe<EPI < 0 ? 0 : EPI, AR, 1>(p, reinterpret_cast<f32x4(&)[1][8][4]>(acc), mb, nb, lane, stage);
#endif
      return;
    }
    if (!p.ws && p.vec8) {
      epilogue256_w<EPI < 0 ? 0 : EPI, AR>(p, acc, mb, nb, lane);
      return;
    }
  }
  if (FAST && !NEWF && !p.ws && p.vec && (p.N & 3) == 0) {
    epilogue256<OutT, EPI < 0 ? 0 : EPI, AR>(p, acc, mb, nb, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mb + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + j * 16 + (lane >> 4) * 4;
      if (n >= p.N) continue;
      acc_pin<AR>(acc[i][j]);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (p.ws) st4(p.ws + (int64_t)kz * p.M * p.N + (int64_t)m * p.N + n, v, min(4, p.N - n), p.vec && n + 4 <= p.N);
      else epilogue4<OutT, EPI>(p, m, n, v);
    }
  }
}

// The 4-wave kernel's 128x128 wave block (two 128x64 halves): one pipelined LDS epilogue over
// both halves where finish256 would stage through LDS (so the second half's bias / input loads
// are not issued behind the first half's stores), else finish256 per half.
template <typename OutT, int EPI, bool AR>
__device__ __forceinline__ void finish256x2(const GemmP& p, f32x4 (&acc)[2][8][4], int mb, int nb, int lane, int kz,
                                            char* stage) {
  constexpr bool FAST = EPI >= 0 && !((EPI & CLIPMI_EPI_RESID) && (EPI & (CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU))) &&
                        !((EPI & CLIPMI_EPI_BETA) && (EPI & (CLIPMI_EPI_RESID | CLIPMI_EPI_DQGELU | CLIPMI_EPI_DGELU)));
#if !CLIPMI_OLD_EPI
  if constexpr (FAST && std::is_same<OutT, bf16>::value) {
    if (stage && !p.ws && p.vec8) {
      epilogue_lds_pipe<EPI < 0 ? 0 : EPI, AR, 2>(p, acc, mb, nb, lane, stage);
      return;
    }
  }
#endif
  finish256<OutT, EPI, AR>(p, acc[0], mb, nb, lane, kz, stage);
  finish256<OutT, EPI, AR>(p, acc[1], mb, nb + 64, lane, kz, stage);
}

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;

// MXFP8 output (fc1 -> fc2 in the fp8 towers) of a wave's NI*16 x 64 block in the 16x16 fragment
// layout: alpha, bias, activation, then per 32-column block of a row -- the 8-column pieces of lanes
// mlane + 16q, q = 0..3 (the permlane16_swap pairing) -- the shared max, its E8M0 scale and the e4m3
// bytes.  The two 8-B pieces a lane quantised (columns coff .. + 7 of the two 32-column blocks) are
// exchanged with lane l ^ 32 (v_permlane32_swap) so each lane holds 16 contiguous bytes of its row --
// lanes q = 0..3 columns 16 q .. 16 q + 15, a whole 64-B row segment per 4 lanes: half the store
// instructions of 8-B pieces -- and the row's two scale bytes go out as one 16-bit store.
template <int EPI, int NI = 8>
__device__ __forceinline__ void epilogue_q8(const GemmP& p, f32x4 (&acc)[NI][4], int mb, int nb, int lane) {
  constexpr bool HB = EPI & CLIPMI_EPI_BIAS, HQ = EPI & CLIPMI_EPI_QGELU, HG = EPI & CLIPMI_EPI_GELU;
  const int q = lane >> 4, mlane = lane & 15;
  const int coff = 16 * (q & 1) + 8 * (q >> 1);
  uint8_t* out = (uint8_t*)p.C;
  const int nsb = p.N >> 5;
  float bv[2][8];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    const int n = min(nb + 32 * jp + coff, p.N - 8);
#pragma unroll
    for (int r = 0; r < 8; ++r) bv[jp][r] = 0.f;
    if (HB) {
      if (p.bias_f32) {
        load4((const float*)p.bias + n, bv[jp]);
        load4((const float*)p.bias + n + 4, bv[jp] + 4);
      } else {
        load8((const bf16*)p.bias + n, bv[jp]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int m = mb + i * 16 + mlane;
    uint32_t w[2][2];
    int ex[2];
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      // the element math in packed fp32 (v_pk_fma / v_pk_mul / v_pk_add: two elements per issue,
      // bitwise the scalar ops' results); only the exp2 / rcp transcendentals stay per element
      f32x2 v2[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][r]),
                                                         __float_as_uint(acc[i][2 * jp + 1][r]), false, false);
        // pairs (r, r + 4): the two 16-column halves the swap returns
        v2[r] = __builtin_elementwise_fma(f32x2{__uint_as_float(sw[0]), __uint_as_float(sw[1])},
                                          f32x2{p.alpha, p.alpha}, f32x2{bv[jp][r], bv[jp][r + 4]});
      }
      float am = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (HQ) {
          const f32x2 z = v2[r] * f32x2{-1.702f * 1.4426950408889634f, -1.702f * 1.4426950408889634f};
          const f32x2 d = f32x2{__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])} + f32x2{1.0f, 1.0f};
          v2[r] = v2[r] * f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
        }
        if (HG) v2[r] = f32x2{gelu_erf(v2[r][0]), gelu_erf(v2[r][1])};
        am = fmaxf(am, fmaxf(fabsf(v2[r][0]), fabsf(v2[r][1])));
      }
      am = fmaxf(am, __shfl_xor(am, 16, 64));
      am = fmaxf(am, __shfl_xor(am, 32, 64));
      ex[jp] = mx_exponent(am);
      const float inv = ldexpf(1.0f, -ex[jp]);
#pragma unroll
      for (int r = 0; r < 4; ++r) v2[r] = v2[r] * f32x2{inv, inv};
      // no clamp: the block's scale makes |v * inv| <= 448 (e4m3's largest normal) exactly, so
      // the round-to-nearest-even conversion cannot leave the range for finite v
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(v2[0][0], v2[1][0], 0, false);
      w[jp][0] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v2[2][0], v2[3][0], pk, true);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(v2[0][1], v2[1][1], 0, false);
      w[jp][1] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v2[2][1], v2[3][1], pk, true);
    }
    // lanes < 32 keep their block-0 piece and take lane l + 32's; lanes >= 32 take lane l - 32's
    // block-1 piece and keep their own
    const auto s0 = __builtin_amdgcn_permlane32_swap(w[0][0], w[1][0], false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(w[0][1], w[1][1], false, false);
    const int col = nb + 16 * q;
    if (m < p.M && col < p.N) *(u32x4*)(out + (int64_t)m * p.ldc + col) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    if (q == 0 && m < p.M) {
      const int sb = (nb >> 5);
      if ((nsb & 1) == 0 && nb + 64 <= p.N) {
        *(uint16_t*)(p.c_scale + (int64_t)m * nsb + sb) = (uint16_t)((ex[0] + 127) | ((ex[1] + 127) << 8));
      } else {
        p.c_scale[(int64_t)m * nsb + sb] = (uint8_t)(ex[0] + 127);
        if (nb + 32 < p.N) p.c_scale[(int64_t)m * nsb + sb + 1] = (uint8_t)(ex[1] + 127);
      }
    }
  }
}

// 4-wave 256x256 kernel (gemm4.hip) for the forward / dgrad layouts; nullptr if not covered
const char* dispatch_w4(const GemmP& p, hipStream_t s, bool bkm, int flags, int dm);
// its fp32-output forward form (flags bias, bias + residual, none); nullptr if not covered
const char* dispatch_w4_f32(const GemmP& p, hipStream_t s, int flags, bool bkm);
// its persistent weight-gradient form (both operands row-major in k, fp32 out, split-K slabs)
const char* dispatch_w4_wgrad(const GemmP& p, int splits, hipStream_t s, int flags, float* bg);
// its MXFP8 form (gemm4.hip gemm_w4p8_kernel); nullptr if the shape or epilogue is not covered
const char* dispatch_w4_fp8(const GemmP& p, hipStream_t s, bool f32o, bool q8o, int flags);

}  // namespace cmg
