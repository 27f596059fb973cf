// Probe: operand / scale lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3, E8M0 scales) on gfx950.
// One wave per experiment.  Each experiment sets one A (or B) byte to 1.0 (0x38) with everything
// else chosen so that the output reveals the (row | col, hardware k-block) that byte belongs to:
//   A one-hot, B all 1.0, B scales 2^(lane >> 4)  ->  C[i][j] = 2^block  at i = row of the byte
//   B one-hot, A all 1.0, A scales 2^(lane >> 4)  ->  C[i][j] = 2^block  at j = col of the byte
// and a scale experiment: A, B all 1.0, A scale of one lane doubled -> which (row, block) it scales.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* out) {
  const int e = blockIdx.x, l = threadIdx.x;
  i32x8 a, b;
  const int* pa = (const int*)(A + ((size_t)e * 64 + l) * 32);
  const int* pb = (const int*)(B + ((size_t)e * 64 + l) * 32);
  for (int i = 0; i < 8; ++i) { a[i] = pa[i]; b[i] = pb[i]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[e * 64 + l], 0, sb[e * 64 + l]);
  for (int r = 0; r < 4; ++r) out[((size_t)e * 64 + l) * 4 + r] = c[r];
}

int main() {
  const int NE = 2048 * 2 + 64;
  std::vector<unsigned char> A((size_t)NE * 64 * 32, 0), B((size_t)NE * 64 * 32, 0);
  std::vector<int> sa((size_t)NE * 64, 127), sb((size_t)NE * 64, 127);
  int e = 0;
  for (int l0 = 0; l0 < 64; ++l0)
    for (int j0 = 0; j0 < 32; ++j0, ++e) {  // A one-hot
      A[((size_t)e * 64 + l0) * 32 + j0] = 0x38;
      for (int l = 0; l < 64; ++l) {
        for (int j = 0; j < 32; ++j) B[((size_t)e * 64 + l) * 32 + j] = 0x38;
        sb[e * 64 + l] = 127 + (l >> 4);
      }
    }
  for (int l0 = 0; l0 < 64; ++l0)
    for (int j0 = 0; j0 < 32; ++j0, ++e) {  // B one-hot
      B[((size_t)e * 64 + l0) * 32 + j0] = 0x38;
      for (int l = 0; l < 64; ++l) {
        for (int j = 0; j < 32; ++j) A[((size_t)e * 64 + l) * 32 + j] = 0x38;
        sa[e * 64 + l] = 127 + (l >> 4);
      }
    }
  for (int l0 = 0; l0 < 64; ++l0, ++e) {  // A scale of lane l0 doubled, A and B all 1.0
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) A[((size_t)e * 64 + l) * 32 + j] = B[((size_t)e * 64 + l) * 32 + j] = 0x38;
    sa[e * 64 + l0] = 128;
  }
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dout;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size());
  hipMalloc(&dsa, sa.size() * 4); hipMalloc(&dsb, sb.size() * 4);
  hipMalloc(&dout, (size_t)NE * 64 * 4 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa.data(), sa.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb.data(), sb.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(NE), dim3(64), 0, 0, dA, dB, dsa, dsb, dout);
  std::vector<float> out((size_t)NE * 64 * 4);
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  // C element (row i, col j) sits in lane (i / 4) * 16 + j ... no: lane l holds D[row 4*(l>>4)+r][col l&15]
  auto C = [&](int ex, int i, int j) { return out[((size_t)ex * 64 + (i / 4) * 16 + j) * 4 + (i % 4)]; };
  e = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int l0 = 0; l0 < 64; ++l0)
      for (int j0 = 0; j0 < 32; ++j0, ++e) {
        int where = -1, blk = -1, cnt = 0;
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            const float v = C(e, i, j);
            if (v != 0.f) {
              ++cnt;
              if (where < 0) { where = pass == 0 ? i : j; blk = v == 1.f ? 0 : v == 2.f ? 1 : v == 4.f ? 2 : v == 8.f ? 3 : -9; }
            }
          }
        printf("%s lane %2d byte %2d -> %s %2d block %d (nonzero %d)\n", pass == 0 ? "A" : "B", l0, j0,
               pass == 0 ? "row" : "col", where, blk, cnt);
      }
  for (int l0 = 0; l0 < 64; ++l0, ++e) {
    printf("Ascale lane %2d ->", l0);
    for (int i = 0; i < 16; ++i) {
      const float v = C(e, i, 0);
      if (v != 128.f) printf(" row %d: %g", i, v);
    }
    printf("\n");
  }
  return 0;
}
