// Image preprocessing on the GPU.
//
// The reference's keras_image_helper resizes with PIL Image.NEAREST and then maps
// x -> x/127.5 - 1 (model_server.py:18,53). PIL's NEAREST source index is a
// double-precision accumulation, not floor((i+0.5)*s), so the row/column tables
// are built on the host (kdl/gateway/preprocess.py) and the kernel is a pure
// table-driven gather. Normalisation is folded into the stem weights for uint8
// batches, so the resized image stays uint8 (4x fewer bytes than f32).
#include "common.h"
#include "launch.h"

namespace kdl {

__global__ __launch_bounds__(256) void resize_nearest_kernel(ResizeArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long plane = (long)a.OH * a.OW;
  const int img = blockIdx.y;
  if (i >= plane) return;
  const int oy = (int)(i / a.OW), ox = (int)(i % a.OW);
  const uint8_t* src = a.src + (long)img * a.SH * a.SW * 3;
  const long sp = ((long)a.ytab[oy] * a.SW + a.xtab[ox]) * 3;
  uint8_t* dst = a.dst + (img * plane + i) * 3;
  dst[0] = src[sp];
  dst[1] = src[sp + 1];
  dst[2] = src[sp + 2];
}

hipError_t resize_nearest_u8(const ResizeArgs& a, hipStream_t s) {
  const long plane = (long)a.OH * a.OW;
  const int n = a.n > 0 ? a.n : 1;
  if (plane <= 0 || a.SH <= 0 || a.SW <= 0 || n > 65535 || !a.src || !a.dst || !a.ytab || !a.xtab)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(resize_nearest_kernel, dim3((unsigned)((plane + 255) / 256), n), dim3(256), 0, s, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void u8_norm_kernel(const uint8_t* x, uint16_t* y, long npix, int ldy) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  uint16_t* o = y + p * ldy;
  for (int c = 0; c < ldy; ++c)
    o[c] = c < 3 ? f2bf((float)x[p * 3 + c] / 127.5f - 1.0f) : (uint16_t)0;
}

hipError_t u8_to_bf16_norm(const uint8_t* x, uint16_t* y, long npix, int ldy, hipStream_t s) {
  if (npix <= 0 || ldy < 3) return hipErrorInvalidValue;
  hipLaunchKernelGGL(u8_norm_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, x, y, npix, ldy);
  return hipGetLastError();
}

}  // namespace kdl
