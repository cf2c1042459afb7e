// Depthwise 3x3 'same' conv (+ optional ReLU on load), NHWC bf16 -> bf16.
// SURVEY.md §2.5 K5. Used by the "split" lowering of SeparableConv2D (dw kernel
// then the MODE_PW GEMM); the autotuner picks split vs fused per layer.
//
// Layout of the work: a wave owns ONE 8-channel chunk for 64 consecutive pixels,
// so the 72 depthwise weights it needs are wave-uniform and come through the
// scalar cache (s_load) instead of 18 vector loads per lane; each lane issues
// its 9 tap loads as 16-byte vectors (neighbouring lanes share rows via L1).
// High occupancy (tiny register footprint) hides the load latency.
#include "common.h"
#include "launch.h"

namespace kdl {

__global__ __launch_bounds__(256) void dw3x3_kernel(DwArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int chunk = blockIdx.y * 4 + wave;
  if (chunk * 8 >= a.C) return;
  const int c0 = chunk * 8;
  const int M = a.B * a.H * a.W;
  const int HW = a.H * a.W;
  int m = blockIdx.x * 64 + lane;
  const bool mvalid = m < M;
  m = mvalid ? m : M - 1;
  const int b = m / HW, rem = m - b * HW;
  const int h = rem / a.W, w = rem - h * a.W;

  u32x4 xv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    int ih = h + tap / 3 - 1, iw = w + tap % 3 - 1;
    ih = ih < 0 ? 0 : (ih >= a.H ? a.H - 1 : ih);
    iw = iw < 0 ? 0 : (iw >= a.W ? a.W - 1 : iw);
    xv[tap] = *(const u32x4*)(a.x + (((long)b * a.H + ih) * a.W + iw) * a.C + c0);
  }
  f32x2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  const float* __restrict__ wq = a.w + c0;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int ih = h + tap / 3 - 1, iw = w + tap % 3 - 1;
    const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    const float* wt = wq + tap * a.C;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t v = ok ? xv[tap][d] : 0u;
      if (a.relu_in) v = relu_bf16x2(v);
      const f32x2 x2 = {bf_lo(v), bf_hi(v)};
      const f32x2 w2 = {wt[2 * d], wt[2 * d + 1]};
      acc[d] = __builtin_elementwise_fma(x2, w2, acc[d]);
    }
  }
  if (mvalid) {
    u32x4 o;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = pack_bf16(acc[d][0], acc[d][1]);
    *(u32x4*)(a.y + (long)m * a.C + c0) = o;
  }
}

hipError_t dw3x3(const DwArgs& a, hipStream_t s) {
  if (a.C % 8 != 0) return hipErrorInvalidValue;
  const long M = (long)a.B * a.H * a.W;
  const dim3 grid((unsigned)((M + 63) / 64), (unsigned)((a.C / 8 + 3) / 4));
  hipLaunchKernelGGL(dw3x3_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
