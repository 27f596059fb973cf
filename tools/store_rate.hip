// Global store rate probes (one 512-thread workgroup per CU, forced by 96 KiB of dynamic LDS).
// (1) Per-CU rate vs the number of CUs storing: each workgroup writes its own 256 KiB region 8 times
//     with 16-B stores, contiguous 1 KiB per wave instruction.
// (2) The GEMM epilogue's shape: 256 workgroups each write a 256 x 256 bf16 tile (128 KiB) of a
//     [rows][ld] matrix, one wave instruction covering SEG bytes of each of 1024 / SEG rows (SEG = 128:
//     the LDS-staged epilogue's 8 rows x 128 B; 256; 512: a whole tile row of 4 lines, 2 rows).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__global__ __launch_bounds__(512) void store_kernel(u32x4* out, int per_wg16, int reps) {
  extern __shared__ char lds[];
  if (threadIdx.x == 1023) lds[0] = 0;  // never true: keeps the LDS allocation
  u32x4* base = out + (size_t)blockIdx.x * per_wg16;
  const u32x4 v = u32x4{threadIdx.x, blockIdx.x, 1u, 2u};
  for (int r = 0; r < reps; ++r)
    for (int i = threadIdx.x; i < per_wg16; i += 512) base[i] = v;
}

// tile t of a [tiles_m * 256][ld] bf16 matrix (ld in elements); tiles laid out row-major over
// tiles_n columns of tiles.  Each wave writes 32 rows (8 waves = 256 rows); per instruction SEG-byte
// pieces of 1024 / SEG consecutive rows.
template <int SEG>
__global__ __launch_bounds__(512) void tile_store_kernel(char* out, int64_t ld_bytes, int tiles_n, int reps) {
  extern __shared__ char lds[];
  if (threadIdx.x == 1023) lds[0] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  char* tile = out + (int64_t)tm * 256 * ld_bytes + (int64_t)tn * 512;
  constexpr int LPR = SEG / 16, RPI = 64 / LPR;  // lanes per row piece, rows per instruction
  const u32x4 v = u32x4{threadIdx.x, blockIdx.x, 1u, 2u};
  for (int r = 0; r < reps; ++r)
    for (int c0 = 0; c0 < 512; c0 += SEG)          // column pieces of a tile row
      for (int r0 = 0; r0 < 32; r0 += RPI) {      // this wave's 32 rows
        const int row = wave * 32 + r0 + lane / LPR;
        *(u32x4*)(tile + (int64_t)row * ld_bytes + c0 + (lane % LPR) * 16) = v;
      }
}

template <int SEG>
float time_tiles(char* buf, int64_t ld_bytes, int tiles_n, int tiles, int reps) {
  hipFuncSetAttribute((const void*)tile_store_kernel<SEG>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(tile_store_kernel<SEG>, dim3(tiles), dim3(512), 96 * 1024, 0, buf, ld_bytes, tiles_n, reps);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int t = 0; t < 5; ++t) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(tile_store_kernel<SEG>, dim3(tiles), dim3(512), 96 * 1024, 0, buf, ld_bytes, tiles_n, reps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const int per_wg = 256 * 1024, per_wg16 = per_wg / 16, reps = 8;
  char* buf;
  if (hipMalloc(&buf, (size_t)1536 << 20) != hipSuccess) return 1;
  hipFuncSetAttribute((const void*)store_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int G : {8, 16, 32, 64, 128, 192, 256, 512, 1024}) {
    hipLaunchKernelGGL(store_kernel, dim3(G), dim3(512), 96 * 1024, 0, (u32x4*)buf, per_wg16, reps);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(store_kernel, dim3(G), dim3(512), 96 * 1024, 0, (u32x4*)buf, per_wg16, reps);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double bytes = (double)G * per_wg * reps;
    const int cus = G < 256 ? G : 256;
    printf("WGs %5d: %8.1f us  total %7.0f GB/s  per storing CU %6.1f GB/s\n", G, best * 1e3, bytes / best / 1e6,
           bytes / best / 1e6 / cus);
  }
  // epilogue shape: fc1's output [201728][3072] bf16 region, the first 1024 tiles (4 per CU), 1 rep
  const int64_t ld = 3072 * 2;
  const int tiles_n = 12, tiles = 1024;
  const double tb = (double)tiles * 256 * 512;
  float t128 = time_tiles<128>(buf, ld, tiles_n, tiles, 1), t512 = time_tiles<512>(buf, ld, tiles_n, tiles, 1),
        t256 = time_tiles<256>(buf, ld, tiles_n, tiles, 1);
  printf("tile stores, 8 rows x 128 B per instr: %8.1f us %7.0f GB/s\n", t128 * 1e3, tb / t128 / 1e6);
  printf("tile stores, 4 rows x 256 B per instr: %8.1f us %7.0f GB/s\n", t256 * 1e3, tb / t256 / 1e6);
  printf("tile stores, 2 rows x 512 B per instr: %8.1f us %7.0f GB/s\n", t512 * 1e3, tb / t512 / 1e6);
  hipFree(buf);
  return 0;
}
