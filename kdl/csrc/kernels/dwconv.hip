// Depthwise 3x3 'same' conv (+ optional ReLU on load), NHWC bf16 -> bf16.
// SURVEY.md §2.5 K5. Used by the "split" lowering of SeparableConv2D (dw kernel
// then the MODE_PW GEMM); the autotuner picks split vs fused per layer.
//
// Block tile = one image x RB output rows x CG 8-channel chunks. The RB+2 input
// rows it needs (halo included) are staged ONCE into LDS with coalesced 16-byte
// loads, with a zero column on each side and zero rows outside the image, and the
// ReLU-on-load applied at staging time; the tile's depthwise weights (9 x 8*CG
// fp32) are staged too. Threads then run a register sliding window along W out of
// LDS: each (chunk, row, SEG-column segment) item reads (SEG+2) x 3 16-byte LDS
// vectors and produces SEG outputs, with no bounds checks in the inner loop.
// Every input byte is fetched from L2/HBM (RB+2)/RB times instead of ~9x, which
// is what made the per-pixel tap-gather version L2-miss and latency bound.
#include "common.h"
#include "launch.h"

namespace kdl {

// 5 columns per item: consecutive items start 5 pixels (640 B / 320 B) apart, so
// the 16-lane groups of a ds_read_b128 spread over distinct bank groups (with 4
// the stride is a multiple of the 256-B bank row: 4-way conflicts).
constexpr int DW_SEG = 5;

template <int CG>
__global__ __launch_bounds__(256) void dw3x3_lds_kernel(DwArgs a, int RB) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int C8 = a.C >> 3;
  const int ngroups = (C8 + CG - 1) / CG;
  const int nbands = (a.H + RB - 1) / RB;
  int bid = blockIdx.x;
  const int g = bid % ngroups;
  bid /= ngroups;
  const int band = bid % nbands;
  const int b = bid / nbands;
  const int h0 = band * RB;
  const int WP = a.W + 2;
  const int tid = threadIdx.x;

  float* wsm = (float*)dsm;                                // [9][CG*8]
  uint8_t* xsm = dsm + 9 * CG * 8 * 4;                     // [(RB+2)][WP][CG][16B]
  for (int i = tid; i < 9 * CG * 2; i += 256) {            // 9 taps x CG chunks x 2 float4
    const int tap = i / (CG * 2), rem = i - tap * CG * 2;
    const int c = rem >> 1, half = rem & 1;
    const int ch = (g * CG + c) * 8 + half * 4;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (g * CG + c < C8) v = *(const float4*)(a.w + tap * a.C + ch);
    *(float4*)(wsm + tap * CG * 8 + c * 8 + half * 4) = v;
  }
  const int rows = RB + 2;
  const int nstage = rows * WP * CG;
  for (int i = tid; i < nstage; i += 256) {
    const int c = i % CG;
    const int t = i / CG;
    const int wp = t % WP, r = t / WP;
    const int ih = h0 - 1 + r, iw = wp - 1;
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W && g * CG + c < C8) {
      v = *(const u32x4*)(a.x + (((long)b * a.H + ih) * a.W + iw) * a.C + (g * CG + c) * 8);
      if (a.relu_in) {
#pragma unroll
        for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
      }
    }
    *(u32x4*)(xsm + (long)i * 16) = v;
  }
  __syncthreads();

  const int nseg = (a.W + DW_SEG - 1) / DW_SEG;
  const int nitems = CG * RB * nseg;
  for (int it = tid; it < nitems; it += 256) {
    const int c = it % CG;
    const int t = it / CG;
    const int s = t % nseg, r = t / nseg;
    if (h0 + r >= a.H || g * CG + c >= C8) continue;
    f32x2 wt[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float4 p = *(const float4*)(wsm + tap * CG * 8 + c * 8);
      const float4 q = *(const float4*)(wsm + tap * CG * 8 + c * 8 + 4);
      wt[tap][0] = (f32x2){p.x, p.y};
      wt[tap][1] = (f32x2){p.z, p.w};
      wt[tap][2] = (f32x2){q.x, q.y};
      wt[tap][3] = (f32x2){q.z, q.w};
    }
    f32x2 acc[DW_SEG][4];
#pragma unroll
    for (int o = 0; o < DW_SEG; ++o)
#pragma unroll
      for (int d = 0; d < 4; ++d) acc[o][d] = (f32x2){0.f, 0.f};
    const int w0 = s * DW_SEG;
#pragma unroll
    for (int j = 0; j < DW_SEG + 2; ++j) {          // LDS column w0 + j == input column w0-1+j
      const int lc = min(w0 + j, WP - 1);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const u32x4 v = *(const u32x4*)(xsm + (((long)(r + dy) * WP + lc) * CG + c) * 16);
        f32x2 xv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) xv[d] = (f32x2){bf_lo(v[d]), bf_hi(v[d])};
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int o = j - dx;
          if (o >= 0 && o < DW_SEG) {
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[o][d] = __builtin_elementwise_fma(xv[d], wt[dy * 3 + dx][d], acc[o][d]);
          }
        }
      }
    }
    uint16_t* yb = a.y + (((long)b * a.H + h0 + r) * a.W) * a.C + (g * CG + c) * 8;
#pragma unroll
    for (int o = 0; o < DW_SEG; ++o) {
      if (w0 + o < a.W) {
        u32x4 out;
#pragma unroll
        for (int d = 0; d < 4; ++d) out[d] = pack_bf16(acc[o][d][0], acc[o][d][1]);
        *(u32x4*)(yb + (long)(w0 + o) * a.C) = out;
      }
    }
  }
}

static size_t dw_smem(int CG, int RB, int W) {
  return (size_t)9 * CG * 8 * 4 + (size_t)(RB + 2) * (W + 2) * CG * 16;
}

hipError_t dw3x3(const DwArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.W <= 0 || a.H <= 0) return hipErrorInvalidValue;
  const int C8 = a.C / 8;
  // (CG, RB): tallest row band (halo overhead (RB+2)/RB) that fits 64 KiB of LDS,
  // preferring 8-chunk (128 B) channel groups when the band is as tall.
  constexpr size_t LIM = 64 * 1024;
  int CG = 4, RB = 0;
  for (int cg : {8, 4}) {
    if (cg == 8 && C8 < 8) continue;
    int rb = 8;
    while (rb > 1 && dw_smem(cg, rb, a.W) > LIM) rb >>= 1;
    if (dw_smem(cg, rb, a.W) <= LIM && rb > RB) { CG = cg; RB = rb; }
  }
  if (RB == 0) return hipErrorInvalidValue;
  const long nblk = (long)a.B * ((a.H + RB - 1) / RB) * ((C8 + CG - 1) / CG);
  const size_t smem = dw_smem(CG, RB, a.W);
  if (CG == 8) hipLaunchKernelGGL(dw3x3_lds_kernel<8>, dim3((unsigned)nblk), dim3(256), smem, s, a, RB);
  else hipLaunchKernelGGL(dw3x3_lds_kernel<4>, dim3((unsigned)nblk), dim3(256), smem, s, a, RB);
  return hipGetLastError();
}

}  // namespace kdl
