// Shared conv-GEMM epilogue store (conv_gemm / gemm_pipe / sepconv_ws / sepconv_2d):
// residual add, ReLU-after-residual (ResNet), and the zero-bordered output
// layout that lets the following 3x3 'same' conv run as a bounds-check-free
// 'valid' implicit GEMM (the 1-pixel border is zeroed once at allocation).
#pragma once
#include "common.h"
#include "launch.h"

namespace kdl {

__device__ __forceinline__ long out_offset(const ConvGemmArgs& a, int m) {
  if (!a.opad) return (long)m * a.ldy;
  const int OHW = a.OH * a.OW;
  if (a.opad == 2) {
    const int b = m / OHW;
    return ((long)b * (OHW + 1) + 1 + (m - b * OHW)) * a.ldy;
  }
  const int b = m / OHW, rem = m - b * OHW;
  const int oh = rem / a.OW, ow = rem - oh * a.OW;
  return (((long)b * (a.OH + 2) + oh + 1) * (a.OW + 2) + ow + 1) * a.ldy;
}

// Transcendental activations (relu_out 3 exact GELU, 4 SiLU) run here, in the
// store pass over the bf16 C tile (8 values per call, one copy of the code),
// NOT on the MFMA accumulators: expanding erff/expf over every accumulator
// element of every fragment grew the GEMM from ~700 to ~4000 instructions and
// cost 15-30 % on GEMMs that never use them. ReLU (1) stays on the accumulators.
template <int DT = 0>
__device__ __noinline__ u32x4 act_transcendental(int mode, u32x4 v) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    float lo = Elt<DT>::lo(v[d]), hi = Elt<DT>::hi(v[d]);
    if (mode == 3) {
      lo = 0.5f * lo * (1.f + fast_erf(lo * 0.70710678118654752f));
      hi = 0.5f * hi * (1.f + fast_erf(hi * 0.70710678118654752f));
    } else {
      lo = fast_silu(lo);
      hi = fast_silu(hi);
    }
    v[d] = Elt<DT>::pack(lo, hi);
  }
  return v;
}

// v: 8 bf16 / fp16 (DT) values (bias + optional pre-residual ReLU already applied) for
// row m, cols n..n+7
template <int DT = 0>
__device__ __forceinline__ void epi_store(const ConvGemmArgs& a, int m, int n, u32x4 v) {
  using E = Elt<DT>;
  if (a.relu_out >= 3) v = act_transcendental<DT>(a.relu_out, v);
  if (a.res) {
    const u32x4 rv = *(const u32x4*)(a.res + (long)m * a.ldr + n);
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = E::pack(E::lo(v[d]) + E::lo(rv[d]), E::hi(v[d]) + E::hi(rv[d]));
  }
  if (a.relu_out == 2) {
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
  }
  *(u32x4*)(a.y + out_offset(a, m) + n) = v;
}

// epi_store with the residual already loaded (rv; ignored when a.res is null): the caller issued
// the residual loads ahead of the store pass, so no load waits behind the pass's stores in the
// in-order vmcnt
template <int DT = 0>
__device__ __forceinline__ void epi_store_r(const ConvGemmArgs& a, int m, int n, u32x4 v, const u32x4 rv) {
  using E = Elt<DT>;
  if (a.relu_out >= 3) v = act_transcendental<DT>(a.relu_out, v);
  if (a.res) {
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = E::pack(E::lo(v[d]) + E::lo(rv[d]), E::hi(v[d]) + E::hi(rv[d]));
  }
  if (a.relu_out == 2) {
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
  }
  *(u32x4*)(a.y + out_offset(a, m) + n) = v;
}

}  // namespace kdl
