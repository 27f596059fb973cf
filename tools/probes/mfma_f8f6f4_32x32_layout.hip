// Probe: operand / scale lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3, E8M0 scales) on gfx950.
// One wave per experiment.  C/D layout (shape-determined, cdna_hip_programming.md): lane l, reg r
// holds D[row (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col l & 31], row from the A operand, col from B.
//   A one-hot, B all 1.0, B scales 2^(lane >> 5)  ->  D[i][*] = 2^(B block of the byte's k) at the byte's row i
//   B one-hot, A all 1.0, A scales 2^(lane >> 5)  ->  D[*][j] = 2^(A block) at the byte's col j
//   A scale of lane l0 doubled, A, B all 1.0, B scales 2^(lane >> 5): row (l0 & 31) reads 128 if the
//   doubled scale covers block 0, 160 if block 1 (32 k per block).
// Output is compacted to one line per lane: the (row, block) of bytes 0..31 as runs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ void probe(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* out) {
  const int e = blockIdx.x, l = threadIdx.x;
  i32x8 a, b;
  const int* pa = (const int*)(A + ((size_t)e * 64 + l) * 32);
  const int* pb = (const int*)(B + ((size_t)e * 64 + l) * 32);
  for (int i = 0; i < 8; ++i) { a[i] = pa[i]; b[i] = pb[i]; }
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa[e * 64 + l], 0, sb[e * 64 + l]);
  for (int r = 0; r < 16; ++r) out[((size_t)e * 64 + l) * 16 + r] = c[r];
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
        sb[e * 64 + l] = 127 + (l >> 5);
      }
    }
  for (int l0 = 0; l0 < 64; ++l0)
    for (int j0 = 0; j0 < 32; ++j0, ++e) {  // B one-hot
      B[((size_t)e * 64 + l0) * 32 + j0] = 0x38;
      for (int l = 0; l < 64; ++l) {
        for (int j = 0; j < 32; ++j) A[((size_t)e * 64 + l) * 32 + j] = 0x38;
        sa[e * 64 + l] = 127 + (l >> 5);
      }
    }
  for (int l0 = 0; l0 < 64; ++l0, ++e) {  // A scale of lane l0 doubled
    for (int l = 0; l < 64; ++l) {
      for (int j = 0; j < 32; ++j) A[((size_t)e * 64 + l) * 32 + j] = B[((size_t)e * 64 + l) * 32 + j] = 0x38;
      sb[e * 64 + l] = 127 + (l >> 5);
    }
    sa[e * 64 + l0] = 128;
  }
  unsigned char *dA, *dB;
  int *dsa, *dsb;
  float* dout;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size());
  hipMalloc(&dsa, sa.size() * 4); hipMalloc(&dsb, sb.size() * 4);
  hipMalloc(&dout, (size_t)NE * 64 * 16 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa.data(), sa.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb.data(), sb.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(NE), dim3(64), 0, 0, dA, dB, dsa, dsb, dout);
  std::vector<float> out((size_t)NE * 64 * 16);
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  auto D = [&](int ex, int i, int j) {  // row i (A side), col j (B side)
    const int lane = j + 32 * ((i >> 2) & 1), r = (i & 3) + 4 * (i >> 3);
    return out[((size_t)ex * 64 + lane) * 16 + r];
  };
  e = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int l0 = 0; l0 < 64; ++l0) {
      printf("%s lane %2d:", pass == 0 ? "A" : "B", l0);
      for (int j0 = 0; j0 < 32; ++j0, ++e) {
        int where = -1, blk = -1, cnt = 0;
        for (int i = 0; i < 32; ++i)
          for (int j = 0; j < 32; ++j) {
            const float v = D(e, i, j);
            if (v != 0.f) {
              ++cnt;
              if (where < 0) { where = pass == 0 ? i : j; blk = v == 1.f ? 0 : v == 2.f ? 1 : -9; }
            }
          }
        printf(" %d:%d/%d%s", j0, where, blk, cnt == 32 ? "" : "!");
      }
      printf("\n");
    }
  for (int l0 = 0; l0 < 64; ++l0, ++e) {
    printf("Ascale lane %2d ->", l0);
    for (int i = 0; i < 32; ++i) {
      const float v = D(e, i, 0);
      if (v != 96.f) printf(" row %d: %g", i, v);
    }
    printf("\n");
  }
  return 0;
}
