// Probe: does buffer_load ... lds reach LDS offsets >= 64 KiB on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const int* src, int* out, int off) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  for (int i = threadIdx.x; i < 131072 / 4; i += 64) ((int*)lds)[i] = -1;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1024, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + off), 16, threadIdx.x * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  out[threadIdx.x] = ((int*)(lds + off))[threadIdx.x * 4];
  out[64 + threadIdx.x] = ((int*)(lds + (off & 65535)))[threadIdx.x * 4];
}
int main() {
  int h[256]; for (int i = 0; i < 256; ++i) h[i] = i;
  int *src, *out; hipMalloc(&src, 1024); hipMalloc(&out, 512);
  hipMemcpy(src, h, 1024, hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  for (int off : {0, 32768, 65536, 98304}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 131072, 0, src, out, off);
    int o[128]; hipMemcpy(o, out, 512, hipMemcpyDeviceToHost);
    printf("off %6d: at off lane1=%d lane5=%d | at off&0xffff lane1=%d lane5=%d | err=%s\n", off, o[1], o[5], o[65], o[69],
           hipGetErrorString(hipGetLastError()));
  }
  return 0;
}
