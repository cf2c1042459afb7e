// Operand-layout probe for the gfx950 block-scaled fp8 MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4, OCP e4m3 A/B, scales 2^0): each lane
// passes its 32 A bytes and 32 B bytes straight from memory, the result is
// written in the standard 16x16 C/D map. tests/test_fp8_gpu.py feeds exact
// small-integer data packed under candidate lane maps and keeps the one that
// reproduces A.B (cdna guide: "Other dtypes: check the map with exact integer
// data before relying on it").
#include "common.h"
#include "launch.h"

namespace kdl {

typedef int v8i __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(64) void mfma_f8_probe_kernel(const v8i* a, const v8i* b, f32x4* d) {
  const int l = threadIdx.x;
  const f32x4 c = {0.f, 0.f, 0.f, 0.f};
  d[l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, 127, 0, 127);
}

hipError_t mfma_f8_probe(const void* a, const void* b, float* d, hipStream_t s) {
  hipLaunchKernelGGL(mfma_f8_probe_kernel, dim3(1), dim3(64), 0, s, (const v8i*)a, (const v8i*)b, (f32x4*)d);
  return hipGetLastError();
}

}  // namespace kdl
