// Calibration probe: fixed cost of a launch vs straight-line code size (cold
// instruction cache). Same grid/LDS as the 192x192 conv GEMM (244 x 512 threads,
// 75 KiB LDS). Run under rocprofv3 --kernel-trace --stats for exact durations.
#include <hip/hip_runtime.h>
#include <cstdio>

#define NOP16 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
#define NOP256 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16 NOP16

__global__ __launch_bounds__(512) void k_empty(int* out) {
  __shared__ int sm[19200];
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 511] == -1) out[0] = 1;
}

template <int REP>
__global__ __launch_bounds__(512) void k_straight(int* out) {
  __shared__ int sm[19200];
  sm[threadIdx.x] = threadIdx.x;
#pragma unroll
  for (int i = 0; i < REP; ++i) asm volatile(NOP256);
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 511] == -1) out[0] = 1;
}

template <int REP>
__global__ __launch_bounds__(512) void k_loop(int* out, int n) {
  __shared__ int sm[19200];
  sm[threadIdx.x] = threadIdx.x;
  for (int i = 0; i < n; ++i) asm volatile(NOP256);
  __syncthreads();
  if (sm[(threadIdx.x + 1) & 511] == -1) out[0] = 1;
}

int main() {
  int* out;
  hipMalloc(&out, 64);
  for (int it = 0; it < 20; ++it) {
    hipLaunchKernelGGL(k_empty, dim3(244), dim3(512), 0, 0, out);
    hipLaunchKernelGGL(k_straight<1>, dim3(244), dim3(512), 0, 0, out);     // 1 KiB of nops
    hipLaunchKernelGGL(k_straight<4>, dim3(244), dim3(512), 0, 0, out);     // 4 KiB
    hipLaunchKernelGGL(k_straight<16>, dim3(244), dim3(512), 0, 0, out);    // 16 KiB
    hipLaunchKernelGGL(k_loop<1>, dim3(244), dim3(512), 0, 0, out, 16);     // 16 x 1 KiB loop
  }
  hipDeviceSynchronize();
  printf("ifetch probe done\n");
  return 0;
}
