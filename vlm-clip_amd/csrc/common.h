// Shared device helpers for libclipmi (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) int i32x4;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// dtype codes shared with include/clipmi.h
enum { DT_F32 = 0, DT_BF16 = 1 };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// sigmoid(1.702 x) through v_exp + v_rcp (1 ulp) instead of an IEEE division sequence:
// these run per output element in the GEMM epilogues
// sigmoid(1.702 x) = 1 / (1 + 2^(x * -1.702 log2 e)): one multiply before v_exp_f32 (the
// epilogues of the quick_gelu GEMMs are VALU-bound on this: profiles/r03_epilogue_stamps.log)
__device__ __forceinline__ float qg_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * (-1.702f * 1.4426950408889634f)));
}
__device__ __forceinline__ float quick_gelu(float x) { return x * qg_sigmoid(x); }
__device__ __forceinline__ float quick_gelu_grad(float x) {
  const float s = qg_sigmoid(x);
  return s + 1.702f * x * s * (1.0f - s);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- MXFP8 (OCP e4m3 + E8M0 per 32-element block), shared by every producer of fp8 operands
// scale exponent: the smallest e with amax / 2^e <= 448 (e4m3's largest normal), clamped to E8M0
__device__ __forceinline__ int mx_exponent(float amax) {
  if (!(amax > 0.f)) return -127;
  int fe;
  const float m = frexpf(amax * (1.0f / 448.0f), &fe);  // amax/448 = m * 2^fe, m in [0.5, 1)
  return max(-127, min(127, m == 0.5f ? fe - 1 : fe));   // ceil(log2(amax / 448))
}
// four values * inv -> four e4m3 bytes (round to nearest even, saturated to +-448), little-endian
__device__ __forceinline__ uint32_t mx_pack4(float a, float b, float c, float d, float inv) {
  int pk = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a * inv, -448.f), 448.f), fminf(fmaxf(b * inv, -448.f), 448.f),
                                           0, false);
  pk = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c * inv, -448.f), 448.f), fminf(fmaxf(d * inv, -448.f), 448.f), pk,
                                       true);
  return (uint32_t)pk;
}

// load/store 4 consecutive elements as float
__device__ __forceinline__ void load4(const float* p, float v[4]) {
  f32x4 t = *(const f32x4*)p; v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
__device__ __forceinline__ void load4(const bf16* p, float v[4]) {
  bf16x4 t = *(const bf16x4*)p; v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
}
__device__ __forceinline__ void store4(float* p, const float v[4]) { *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]}; }
__device__ __forceinline__ void store4(bf16* p, const float v[4]) {
  *(bf16x4*)p = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

#define CLIPMI_CHECK_LAUNCH() do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return clipmi_fail(e_, __FILE__, __LINE__); } while (0)
// LDS-DMA (buffer_load_dwordx4 ... lds: 16 B per lane, 1 KiB per wave-instruction, written
// lane-linearly at the wave-uniform LDS address) issued from inline asm.  hipcc's waitcnt pass treats every
// ds_read_b64_tr_b16 as aliasing any LDS-DMA it can see and puts s_waitcnt vmcnt(0) in
// front of it, which drains the next k-step's prefetch in the middle of the current one;
// DMAs it cannot see are ordered by this kernel's own vmcnt + barrier instead.
struct SRsrc { u32x4 v; };
__device__ __forceinline__ SRsrc make_srsrc(const void* base, uint32_t num_records) {
  const uint64_t b = (uint64_t)base;
  SRsrc r;
  r.v[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
  r.v[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xffffu);
  r.v[2] = __builtin_amdgcn_readfirstlane(num_records);
  r.v[3] = 0x00020000u;
  return r;
}
__device__ __forceinline__ void dma16(SRsrc r, char* lds_wave_base, int voff) {
  const uint32_t m = (uint32_t)(uintptr_t)LDS_PTR(char, lds_wave_base);
  // s_nop 2 + s_mov + s_nop 0: the 5 wait states a buffer instruction needs after a VALU
  // (v_readfirstlane in make_srsrc) wrote its descriptor SGPRs; hipcc pads nothing inside asm
  asm volatile("s_nop 2\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(r.v)
               : "memory");
}

