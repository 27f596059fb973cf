// Fragment helpers shared by the attention kernels (attention.hip: bf16 operands; attention_x3.hip: the
// bf16x3 split operands).  LDS images hold [Npad][64] bf16 rows with 16-B chunk c of row r stored at
// c ^ (r & 6): conflict-free for the ds_read_b128 fragment reads, the ds_read_b64_tr_b16 transposed reads
// and lane-linear DMA writes.
#pragma once
#include "common.h"

namespace {

__device__ __forceinline__ int img_off(int r, int c) { return r * 128 + ((c ^ (r & 6)) << 4); }

__device__ __forceinline__ bf16x8 frag_row(const char* img, int r, int c) {
  return *LDS_PTR(const bf16x8, img + img_off(r, c));
}

// transposed fragment: element j<4 from rows r0+q, j>=4 from rows r0+16+q; column d0 + lane&15
__device__ __forceinline__ bf16x8 frag_tr(const char* img, int r0, int d0, int lane) {
  const int q = (lane & 15) >> 2;
  const int col = d0 + 4 * (lane & 3);
  const int ra = r0 + 4 * (lane >> 4) + q, rb = ra + 16;
  const int c = col >> 3, h = (col & 7) * 2;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, img + img_off(ra, c) + h));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, img + img_off(rb, c) + h));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}

}  // namespace
