// Xception stem: block1_conv1 (3x3, stride 2, 'valid', 3 -> 32) + BN + ReLU
// (with K1's normalisation fused).
//
// K = 27 (padded to one 32-deep MFMA step). Each lane gathers its own A fragment
// straight from the image (8 scalars: tap*3 + channel), so there is no LDS at all;
// the whole op is one MFMA per 16x16 output tile. For uint8 input the Xception
// preprocessing x/127.5 - 1 is folded into the weights on the host (exact: the
// conv is 'valid', every tap is in-bounds), so raw pixels are consumed directly
// and the f32 normalised image never exists.
#include "common.h"
#include "launch.h"

namespace kdl {

template <int IN_KIND>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = a.B * a.OH * a.OW;
  const int OHW = a.OH * a.OW;
  const int m_wave = blockIdx.x * 128 + wave * 32;

  s16x8 bw[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bw[j] = *(const s16x8*)(a.wp + (j * 64 + lane) * 8);

  const int kq = 8 * (lane >> 4);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int m = m_wave + f * 16 + (lane & 15);
    const bool mvalid = m < M;
    m = mvalid ? m : M - 1;
    const int b = m / OHW, rem = m - b * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    const long base = ((long)b * a.H + 2 * oh) * a.W + 2 * ow;  // pixel index of tap (0,0)
    s16x8 af;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kq + j;
      float v = 0.f;
      if (k < 27) {
        const int tap = k / 3, c = k - 3 * (k / 3);
        const long p = base + (long)(tap / 3) * a.W + (tap % 3);
        if constexpr (IN_KIND == 0) v = (float)((const uint8_t*)a.x)[p * 3 + c];
        else v = ((const float*)a.x)[p * 3 + c];
      }
      af[j] = (short)f2bf(v);
    }
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = mfma16(bw[j], af, (f32x4){0.f, 0.f, 0.f, 0.f});
    // lane holds Y[m_tile + (lane&15)][16j + 4*(lane>>4) + r]
    const int mo = m_wave + f * 16 + (lane & 15);
    if (mo < M) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 16 * j + 4 * (lane >> 4);
        const float4 bv = *(const float4*)(a.bias + n);
        const float v0 = fmaxf(acc[j][0] + bv.x, 0.f), v1 = fmaxf(acc[j][1] + bv.y, 0.f);
        const float v2 = fmaxf(acc[j][2] + bv.z, 0.f), v3 = fmaxf(acc[j][3] + bv.w, 0.f);
        *(u32x2*)(a.y + (long)mo * a.ldy + n) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
      }
    }
  }
}

hipError_t stem_conv(const StemArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  if (M <= 0 || a.ldy < 32) return hipErrorInvalidValue;
  const dim3 grid((M + 127) / 128);
  if (a.in_kind == 0) hipLaunchKernelGGL(stem_kernel<0>, grid, dim3(256), 0, s, a);
  else if (a.in_kind == 1) hipLaunchKernelGGL(stem_kernel<1>, grid, dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace kdl
