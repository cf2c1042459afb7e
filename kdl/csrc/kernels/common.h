// Shared CDNA4 (gfx950) helpers for the kdl kernel library.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC bf16 with the channel dimension padded to a multiple
//     of 32 ("ldc"); padded channels always hold zeros;
//   * MFMA is v_mfma_f32_16x16x32_bf16 (wave64, 4 fp32 accumulators per lane);
//   * bf16 is carried as raw 16-bit patterns (uint16_t / packed in uint32_t).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdl {

typedef short s16x8 __attribute__((ext_vector_type(8)));   // one MFMA A/B fragment (8 bf16)
typedef float f32x4 __attribute__((ext_vector_type(4)));   // one 16x16 accumulator fragment
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) void lds_void;

// SiLU with a hardware reciprocal: v_exp + v_rcp + v_mul instead of the IEEE division
// sequence (~10 VALU ops) -- the depthwise kernels evaluate it per output element
__device__ __forceinline__ float fast_silu(float v) { return v * __builtin_amdgcn_rcpf(1.f + __expf(-v)); }
// erf to ~1.5e-7 absolute (Abramowitz & Stegun 7.1.26), branch-free: rcp + 5-term Horner + one
// v_exp_f32, ~14 VALU ops against the ~30 of OCML's range-split erff. The GELU epilogue of
// the ViT MLP evaluates it on every element of a 6304 x 3072 tile; its inputs and outputs
// are bf16 (8-bit mantissa), so the approximation error is far below one output ulp.
__device__ __forceinline__ float fast_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-p * t, e, 1.f), x);
}
__device__ __forceinline__ float bf_lo(uint32_t d) { return __uint_as_float(d << 16); }
__device__ __forceinline__ float bf_hi(uint32_t d) { return __uint_as_float(d & 0xffff0000u); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even pack of two floats into bf16x2 (hipcc emits v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ uint16_t f2bf(float x) {
  __bf16 b = (__bf16)x;
  return __builtin_bit_cast(uint16_t, b);
}

// ReLU on two packed bf16 values: a negative bf16 is a negative int16 (sign bit),
// so a signed 16-bit max against 0 is exactly ReLU (v_pk_max_i16).
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t d) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  s2 v = __builtin_bit_cast(s2, d);
  s2 z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, z));
}

// 4 floats -> 4 OCP e4m3 bytes (saturated to +-448; gfx950 v_cvt_pk_fp8_f32 is OCP)
__device__ __forceinline__ uint32_t pack_fp8x4(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f); b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f); d = fminf(fmaxf(d, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16-byte global->LDS DMA. `lds` must be wave-uniform; lane l lands at lds + 16*l.
__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds, 16, 0, 0);
}

// 16-bit activation / weight element type of a kernel instance (DT template parameter,
// runtime field `dt` in the launch args): 0 = bf16 (every model family's default),
// 1 = IEEE fp16 (BASELINE.json's "ResNet-50 fp16" config). Both are 16-bit patterns in
// memory; they differ in the MFMA opcode (v_mfma_f32_16x16x32_{bf16,f16}, same rate on
// gfx950) and in the fp32 <-> 16-bit conversions. The sign bit is bit 15 in both, so
// relu_bf16x2 (signed 16-bit max against 0) is exact for fp16 too.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <int DT>
struct Elt;

template <>
struct Elt<0> {
  static __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) { return mfma16(a, b, c); }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) { return pack_bf16(lo, hi); }
  static __device__ __forceinline__ float lo(uint32_t d) { return bf_lo(d); }
  static __device__ __forceinline__ float hi(uint32_t d) { return bf_hi(d); }
  static __device__ __forceinline__ uint16_t from_f32(float x) { return f2bf(x); }
};

template <>
struct Elt<1> {
  static __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                   0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) {   // round to nearest even
    f16x2 v = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
  static __device__ __forceinline__ float lo(uint32_t d) { return (float)__builtin_bit_cast(f16x2, d)[0]; }
  static __device__ __forceinline__ float hi(uint32_t d) { return (float)__builtin_bit_cast(f16x2, d)[1]; }
  static __device__ __forceinline__ uint16_t from_f32(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }
};

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b, b+8, ... are dispatched to one XCD, so give each XCD a
// contiguous run of logical tiles; neighbouring tiles then share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, local = bid >> 3;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + local;
}

}  // namespace kdl
