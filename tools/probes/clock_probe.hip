// Calibration probe: effective shader clock under back-to-back bf16 MFMA load.
// Every wave issues N v_mfma_f32_16x16x32_bf16 on 4 independent accumulators
// (16 cycles each, MI355X_MICROARCH.md cycle constants); wall time from hipEvents,
// and s_memtime / s_memrealtime deltas per wave give the clock the waves saw.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(float* out, unsigned long long* t, int n) {
  s16x8 a = {(short)threadIdx.x, 1, 2, 3, 4, 5, 6, 7}, b = {7, 6, 5, 4, 3, 2, 1, (short)blockIdx.x};
  f32x4 c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; i += 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c[j]) : "v"(a), "v"(b));
  }
  const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) sum += c[j][j & 3];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) { t[blockIdx.x * 2] = m1 - m0; t[blockIdx.x * 2 + 1] = r1 - r0; }
}

int main() {
  const int n = 20000;
  for (int blocks : {1, 256, 1024}) {
    float* out; unsigned long long* t;
    hipMalloc(&out, blocks * 256 * 4); hipMalloc(&t, blocks * 16);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, t, n);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, t, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(blocks * 2);
    hipMemcpy(h.data(), t, blocks * 16, hipMemcpyDeviceToHost);
    // 4 waves per block on 4 SIMDs; per wave 4n MFMAs x 16 cycles (1 wave per SIMD at <=256 blocks)
    const double cyc = 4.0 * n * 16;
    double wpsimd = blocks <= 256 ? 1.0 : blocks / 256.0;
    printf("blocks %5d: %.3f ms -> %.0f MHz (ideal-issue clock); memtime %llu cyc, realtime %llu ticks -> memtime %.0f MHz if realtime=100MHz\n",
           blocks, ms, cyc * wpsimd / (ms * 1e3), h[0], h[1], h[0] / (h[1] / 100.0));
    hipFree(out); hipFree(t);
  }
  return 0;
}
