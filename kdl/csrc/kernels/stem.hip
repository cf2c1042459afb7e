// Network stems: a KxK / stride / pad conv from 3 input channels + BN + ReLU,
// with the input normalisation fused (SURVEY.md §2.5 K1+K2, §2.6 ResNet 7x7 stem).
//
//   Xception block1_conv1: 3x3 s2 'valid', 3 -> 32 (K = 27 -> one 32-deep step);
//       for uint8 input x/127.5-1 is folded into the weights (exact: 'valid').
//   ResNet-50 conv1:       7x7 s2 pad 3, 3 -> 64 (K = 147 -> 5 steps); the
//       torchvision mean/std normalisation is applied on load (scale/shift per
//       channel) so zero padding stays exact.
//
// Each lane gathers its own A fragment straight from the image (8 scalars:
// k = (ky*KW + kx)*3 + c), so there is no LDS at all. The (ky, kx, c) of a lane's
// 8 k-slots depend only on the k-step, not on the pixel, and are computed once
// per step for both 16-row fragments of the wave.
#include "common.h"
#include "launch.h"

namespace kdl {

// GENERIC=false: 'valid' conv with the normalisation folded into the weights (the
// Xception stem): no bounds checks, no per-element scale/shift.
template <int IN_KIND, int NF, int KW, bool GENERIC, int DT = 0>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  using E = Elt<DT>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = a.B * a.OH * a.OW;
  const int OHW = a.OH * a.OW;
  const int m_wave = blockIdx.x * 128 + wave * 32;
  const int KK = a.KH * KW * 3;
  const int KT = (KK + 31) >> 5;

  long pbase[2];
  int ih0[2], iw0[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int m = m_wave + f * 16 + (lane & 15);
    m = m < M ? m : M - 1;
    const int b = m / OHW, rem = m - b * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    ih0[f] = oh * a.stride - a.pad;
    iw0[f] = ow * a.stride - a.pad;
    pbase[f] = (long)b * a.H * a.W;
  }
  f32x4 acc[2][NF];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int kq = 8 * (lane >> 4);
  for (int ks = 0; ks < KT; ++ks) {
    int dy[8], dx[8], ch[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = ks * 32 + kq + j;
      const int tap = k / 3;
      ch[j] = k < KK ? k - 3 * tap : -1;
      dy[j] = tap / KW;                  // compile-time divisor
      dx[j] = tap - dy[j] * KW;
    }
    s16x8 bw[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) bw[j] = *(const s16x8*)(a.wp + (((long)j * KT + ks) * 64 + lane) * 8);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      s16x8 af;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ih = ih0[f] + dy[j], iw = iw0[f] + dx[j];
        float v = 0.f;
        if (ch[j] >= 0 && (!GENERIC || ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W))) {
          const long p = (pbase[f] + (long)ih * a.W + iw) * 3 + ch[j];
          float raw;
          if constexpr (IN_KIND == 0) raw = (float)((const uint8_t*)a.x)[p];
          else raw = ((const float*)a.x)[p];
          if constexpr (GENERIC) {
            const int c = ch[j];
            v = raw * (c == 0 ? a.scale[0] : c == 1 ? a.scale[1] : a.scale[2]) +
                (c == 0 ? a.shift[0] : c == 1 ? a.shift[1] : a.shift[2]);
          } else {
            v = raw;
          }
        }
        af[j] = (short)E::from_f32(v);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[f][j] = E::mfma(bw[j], af, acc[f][j]);
    }
  }
  // lane holds Y[m_tile + (lane&15)][16j + 4*(lane>>4) + r]. The block's 128 output
  // pixels are consecutive rows of Y: stage the bf16 tile in LDS and write it back
  // with coalesced 16-byte stores (8-byte per-lane stores scattered over 16 rows per
  // instruction made this memory-bound kernel ~4x slower than its write volume).
  __shared__ __attribute__((aligned(16))) uint16_t ys[128 * NF * 16];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int ml = wave * 32 + f * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = 16 * j + 4 * (lane >> 4);
      const float4 bv = *(const float4*)(a.bias + n);
      float v0 = acc[f][j][0] + bv.x, v1 = acc[f][j][1] + bv.y;
      float v2 = acc[f][j][2] + bv.z, v3 = acc[f][j][3] + bv.w;
      if (a.relu == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      } else if (a.relu == 2) {
        v0 = fast_silu(v0); v1 = fast_silu(v1);
        v2 = fast_silu(v2); v3 = fast_silu(v3);
      }
      *(u32x2*)(ys + ml * NF * 16 + n) = (u32x2){E::pack(v0, v1), E::pack(v2, v3)};
    }
  }
  __syncthreads();
  constexpr int CPR = NF * 2;                  // 16-byte chunks per output row
  const int m0 = blockIdx.x * 128;
  for (int c = threadIdx.x; c < 128 * CPR; c += 256) {
    const int r = c / CPR, part = c - r * CPR;
    if (m0 + r < M) *(u32x4*)(a.y + (long)(m0 + r) * a.ldy + part * 8) = *(const u32x4*)(ys + r * NF * 16 + part * 8);
  }
}

// Row-run variant (uint8 input): K is laid out per kernel row, k = ky*RP + kx*3 + c with the
// KW*3 bytes of one kernel row -- contiguous in the NHWC image -- padded to RP (32 for 7x7,
// 16 for 3x3). A lane's 8 k-slots of a step are then 8 CONSECUTIVE image bytes: one aligned
// 12-byte load plus two v_alignbyte per fragment and step, instead of 8 scattered byte loads
// each with its own 64-bit address arithmetic (7x7: 14 loads per lane instead of 80). The
// per-slot channel / column offset / validity depend only on the lane's q, so they are set
// up once. Windows that would start before the tensor or end past it (first / last pixels)
// take a checked byte-wise path.
template <int NF, int KW, int RP, bool GENERIC, int DT = 0>
__global__ __launch_bounds__(256) void stem_rows_kernel(StemArgs a) {
  using E = Elt<DT>;
  constexpr int RUN = KW * 3;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = a.B * a.OH * a.OW;
  const int OHW = a.OH * a.OW;
  const int m_wave = blockIdx.x * 128 + wave * 32;
  const int KT = (a.KH * RP + 31) >> 5;
  const long total = (long)a.B * a.H * a.W * 3;
  const uint8_t* x = (const uint8_t*)a.x;

  long rbase[2];   // byte offset of (b, 0, iw0) -- add ih * W * 3
  int ih0[2], iw0[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int m = m_wave + f * 16 + (lane & 15);
    m = m < M ? m : M - 1;
    const int b = m / OHW, rem = m - b * OHW;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    ih0[f] = oh * a.stride - a.pad;
    iw0[f] = ow * a.stride - a.pad;
    rbase[f] = ((long)b * a.H * a.W + iw0[f]) * 3;
  }
  // the lane's 8 slots within a kernel row: r = rq + j (rq = 8q mod RP), kx = r / 3, c = r % 3
  const int q = lane >> 4;
  const int rq = (8 * q) % RP;
  int kxj[8];
  float scj[8], shj[8];
  bool rv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = rq + j;
    rv[j] = r < RUN;
    kxj[j] = r / 3;
    const int c = r - 3 * (r / 3);
    scj[j] = c == 0 ? a.scale[0] : c == 1 ? a.scale[1] : a.scale[2];
    shj[j] = c == 0 ? a.shift[0] : c == 1 ? a.shift[1] : a.shift[2];
  }
  f32x4 acc[2][NF];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int ks = 0; ks < KT; ++ks) {
    const int ky = (ks * 32 + 8 * q) / RP;
    s16x8 bw[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) bw[j] = *(const s16x8*)(a.wp + (((long)j * KT + ks) * 64 + lane) * 8);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int ih = ih0[f] + ky;
      const bool row_ok = ky < a.KH && (unsigned)ih < (unsigned)a.H && rq < RUN;
      uint32_t w0 = 0u, w1 = 0u;
      if (row_ok) {
        const long p0 = rbase[f] + (long)ih * a.W * 3 + rq;   // first byte of the 8
        const long al = p0 & ~3L;
        if (al >= 0 && al + 12 <= total) {
          const uint32_t* wp = (const uint32_t*)(x + al);
          const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2];
          const uint32_t sh = (uint32_t)(p0 - al);
          w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
          w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const long pj = p0 + j;
            const uint32_t v = (pj >= 0 && pj < total) ? x[pj] : 0u;
            if (j < 4) w0 |= v << (8 * j); else w1 |= v << (8 * (j - 4));
          }
        }
      }
      s16x8 af;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t wd = j < 4 ? w0 : w1;
        const float raw = (float)((wd >> (8 * (j & 3))) & 0xffu);
        const int iw = iw0[f] + kxj[j];
        bool ok = row_ok && rv[j];
        if constexpr (GENERIC) ok = ok && (unsigned)iw < (unsigned)a.W;
        const float v = ok ? (GENERIC ? fmaf(raw, scj[j], shj[j]) : raw) : 0.f;
        af[j] = (short)E::from_f32(v);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[f][j] = E::mfma(bw[j], af, acc[f][j]);
    }
  }
  __shared__ __attribute__((aligned(16))) uint16_t ys[128 * NF * 16];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int ml = wave * 32 + f * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = 16 * j + 4 * (lane >> 4);
      const float4 bv = *(const float4*)(a.bias + n);
      float v0 = acc[f][j][0] + bv.x, v1 = acc[f][j][1] + bv.y;
      float v2 = acc[f][j][2] + bv.z, v3 = acc[f][j][3] + bv.w;
      if (a.relu == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      } else if (a.relu == 2) {
        v0 = fast_silu(v0); v1 = fast_silu(v1);
        v2 = fast_silu(v2); v3 = fast_silu(v3);
      }
      *(u32x2*)(ys + ml * NF * 16 + n) = (u32x2){E::pack(v0, v1), E::pack(v2, v3)};
    }
  }
  __syncthreads();
  constexpr int CPR = NF * 2;
  const int m0 = blockIdx.x * 128;
  for (int c = threadIdx.x; c < 128 * CPR; c += 256) {
    const int r = c / CPR, part = c - r * CPR;
    if (m0 + r < M) *(u32x4*)(a.y + (long)(m0 + r) * a.ldy + part * 8) = *(const u32x4*)(ys + r * NF * 16 + part * 8);
  }
}

template <int KW, int RP>
static hipError_t launch_stem_rows(const StemArgs& a, dim3 grid, bool generic, hipStream_t s) {
  if (a.in_kind != 0) return hipErrorInvalidValue;
#define KDL_SROWS(nf, g, dt) \
  hipLaunchKernelGGL((stem_rows_kernel<nf, KW, RP, g, dt>), grid, dim3(256), 0, s, a); return hipGetLastError();
  if (a.dt == 1) {
    if (a.cout != 64 || !generic) return hipErrorInvalidValue;
    KDL_SROWS(4, true, 1)
  }
  if (a.dt != 0) return hipErrorInvalidValue;
  if (a.cout == 32 && !generic) { KDL_SROWS(2, false, 0) }
  if (a.cout == 32) { KDL_SROWS(2, true, 0) }
  if (a.cout == 64 && !generic) { KDL_SROWS(4, false, 0) }
  if (a.cout == 64) { KDL_SROWS(4, true, 0) }
#undef KDL_SROWS
  return hipErrorInvalidValue;
}

template <int IN_KIND, int KW>
static hipError_t launch_stem(const StemArgs& a, dim3 grid, hipStream_t s) {
  const bool generic = a.pad != 0 || a.scale[0] != 1.f || a.scale[1] != 1.f || a.scale[2] != 1.f ||
                       a.shift[0] != 0.f || a.shift[1] != 0.f || a.shift[2] != 0.f;
  if (a.dt == 1) {   // fp16 (ResNet-50 fp16 config): the 64-channel normalise-on-load stem only
    if (a.cout != 64 || !generic) return hipErrorInvalidValue;
    hipLaunchKernelGGL((stem_kernel<IN_KIND, 4, KW, true, 1>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (a.dt != 0) return hipErrorInvalidValue;
  if (a.cout == 32 && !generic) hipLaunchKernelGGL((stem_kernel<IN_KIND, 2, KW, false>), grid, dim3(256), 0, s, a);
  else if (a.cout == 32) hipLaunchKernelGGL((stem_kernel<IN_KIND, 2, KW, true>), grid, dim3(256), 0, s, a);
  else if (a.cout == 64 && !generic) hipLaunchKernelGGL((stem_kernel<IN_KIND, 4, KW, false>), grid, dim3(256), 0, s, a);
  else if (a.cout == 64) hipLaunchKernelGGL((stem_kernel<IN_KIND, 4, KW, true>), grid, dim3(256), 0, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t stem_conv(const StemArgs& a, hipStream_t s) {
  const int M = a.B * a.OH * a.OW;
  if (M <= 0 || a.ldy < a.cout || a.KH <= 0 || a.KW <= 0 || a.stride <= 0) return hipErrorInvalidValue;
  const dim3 grid((M + 127) / 128);
  if (a.rows) {
    const bool generic = a.pad != 0 || a.scale[0] != 1.f || a.scale[1] != 1.f || a.scale[2] != 1.f ||
                         a.shift[0] != 0.f || a.shift[1] != 0.f || a.shift[2] != 0.f;
    if (a.KW == 7) return launch_stem_rows<7, 32>(a, grid, generic, s);
    if (a.KW == 3) return launch_stem_rows<3, 16>(a, grid, generic, s);
    return hipErrorInvalidValue;
  }
  if (a.KW == 3 && a.in_kind == 0) return launch_stem<0, 3>(a, grid, s);
  if (a.KW == 3 && a.in_kind == 1) return launch_stem<1, 3>(a, grid, s);
  if (a.KW == 7 && a.in_kind == 0) return launch_stem<0, 7>(a, grid, s);
  if (a.KW == 7 && a.in_kind == 1) return launch_stem<1, 7>(a, grid, s);
  return hipErrorInvalidValue;
}

}  // namespace kdl
