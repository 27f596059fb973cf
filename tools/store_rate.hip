// Per-CU global store rate vs the number of CUs storing (one 512-thread workgroup per CU, forced by
// 96 KiB of dynamic LDS).  Each workgroup writes its own 256 KiB region REPS times with 16-B stores,
// 8 whole 128-B rows per wave instruction (the GEMM epilogue's LDS-staged pattern).  Question: is the
// epilogue's ~12.5 B/clk per CU a per-CU limit, or the chip's HBM write rate shared by 256 CUs?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__global__ __launch_bounds__(512) void store_kernel(u32x4* out, int per_wg16, int reps) {
  extern __shared__ char lds[];
  if (threadIdx.x == 1023) lds[0] = 0;  // never true: keeps the LDS allocation
  u32x4* base = out + (size_t)blockIdx.x * per_wg16;
  const u32x4 v = u32x4{threadIdx.x, blockIdx.x, 1u, 2u};
  for (int r = 0; r < reps; ++r)
    for (int i = threadIdx.x; i < per_wg16; i += 512) base[i] = v;
}

int main() {
  const int per_wg = 256 * 1024, per_wg16 = per_wg / 16, reps = 8;
  u32x4* buf;
  if (hipMalloc(&buf, (size_t)1024 * per_wg) != hipSuccess) return 1;
  hipFuncSetAttribute((const void*)store_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int G : {8, 16, 32, 64, 128, 192, 256, 512, 1024}) {
    hipLaunchKernelGGL(store_kernel, dim3(G), dim3(512), 96 * 1024, 0, buf, per_wg16, reps);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(store_kernel, dim3(G), dim3(512), 96 * 1024, 0, buf, per_wg16, reps);
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
  hipFree(buf);
  return 0;
}
