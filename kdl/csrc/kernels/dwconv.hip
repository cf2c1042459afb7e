// Depthwise 3x3 'same' conv (+ optional ReLU on load), NHWC bf16 -> bf16.
// SURVEY.md §2.5 K5. Used by the "split" lowering of SeparableConv2D (dw kernel
// then the MODE_PW GEMM); the autotuner picks split vs fused per layer.
//
// Block tile = one image x RB output rows x TW output columns x CG 8-channel
// chunks. The (RB+2) x (TW+2) input patch (halo included; zeros outside the
// image, ReLU-on-load applied at staging) is staged ONCE into LDS, then threads
// run a register sliding window along W out of LDS: an item = (chunk, row,
// SEG-column segment) produces SEG outputs from 3 x (SEG+2) 16-byte LDS vectors.
//
// MI355X specifics (measured, profiles/):
//   * staging issues up to MAXL 16-byte loads per thread back to back before the
//     first LDS write (one vmcnt-counted round trip instead of a load->wait->write
//     chain per vector, which is what made the previous version latency bound);
//   * 2-D tiles: at 147x147 a full-width row band only fit RB=1 in LDS (3x halo
//     re-reads); column tiles of 37-49 px keep RB at 4-8;
//   * dy-outer compute: only 3 taps (24 fp32) of weights are live at a time, so
//     the kernel stays near 100 VGPRs (4+ waves/SIMD) instead of 200;
//   * SEG=5/7 columns per item: the 16-lane groups of a ds_read_b128 land 640/896 B
//     apart -> distinct bank halves (SEG=4 would be a 4-way conflict at CG=8).
#include "common.h"
#include "launch.h"

namespace kdl {

constexpr int DW_MAXL = 8;

template <int SEG>
__global__ __launch_bounds__(256) void dw3x3_tile_kernel(DwArgs a, int CG, int RB, int TW) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int C8 = a.C >> 3;
  const int ngroups = (C8 + CG - 1) / CG;
  const int nbands = (a.H + RB - 1) / RB;
  const int ncolt = (a.W + TW - 1) / TW;
  int bid = blockIdx.x;
  const int g = bid % ngroups;
  bid /= ngroups;
  const int ct = bid % ncolt;
  bid /= ncolt;
  const int band = bid % nbands;
  const int b = bid / nbands;
  const int h0 = band * RB, c0 = ct * TW;
  const int TWP = TW + 2;
  const int tid = threadIdx.x;
  const int cbase = g * CG;                                // first chunk of the group

  float* wsm = (float*)dsm;                                // [9][CG*8]
  uint8_t* xsm = dsm + 9 * CG * 8 * 4;                     // [(RB+2)][TWP][CG][16B]
  for (int i = tid; i < 9 * CG * 2; i += 256) {            // 9 taps x CG chunks x 2 float4
    const int tap = i / (CG * 2), rem = i - tap * CG * 2;
    const int c = rem >> 1, half = rem & 1;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (cbase + c < C8) v = *(const float4*)(a.w + tap * a.C + (cbase + c) * 8 + half * 4);
    *(float4*)(wsm + tap * CG * 8 + c * 8 + half * 4) = v;
  }

  // ---- staging: element i = (r, col, c), c fastest. Per-thread coordinates are
  // advanced incrementally by 256 elements (no integer divisions in the loop).
  const int nst = (RB + 2) * TWP * CG;
  const int dc = 256 % CG, dt = 256 / CG;
  const int dcol = dt % TWP, dr = dt / TWP;
  int c = tid % CG, t = tid / CG;
  int col = t % TWP, r = t / TWP;
  const long img = (long)b * a.H;
  for (int base = 0; base < nst; base += 256 * DW_MAXL) {
    u32x4 v[DW_MAXL];
    int cc[DW_MAXL], cl[DW_MAXL], rr[DW_MAXL];
#pragma unroll
    for (int l = 0; l < DW_MAXL; ++l) {
      cc[l] = c; cl[l] = col; rr[l] = r;
      v[l] = (u32x4){0u, 0u, 0u, 0u};
      const int ih = h0 - 1 + r, iw = c0 - 1 + col;
      if (base + tid + l * 256 < nst && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W &&
          cbase + c < C8)
        v[l] = *(const u32x4*)(a.x + ((img + ih) * a.W + iw) * a.C + (cbase + c) * 8);
      // advance by 256 elements
      c += dc;
      int carry = c >= CG;
      c -= carry ? CG : 0;
      col += dcol + carry;
      carry = col >= TWP;
      col -= carry ? TWP : 0;
      r += dr + carry;
    }
#pragma unroll
    for (int l = 0; l < DW_MAXL; ++l) {
      if (base + tid + l * 256 < nst) {
        u32x4 w = v[l];
        if (a.relu_in) {
#pragma unroll
          for (int d = 0; d < 4; ++d) w[d] = relu_bf16x2(w[d]);
        }
        *(u32x4*)(xsm + (((long)rr[l] * TWP + cl[l]) * CG + cc[l]) * 16) = w;
      }
    }
  }
  __syncthreads();

  // ---- compute: item = (c, s, r), c fastest
  const int nseg = (TW + SEG - 1) / SEG;
  const int nitems = CG * RB * nseg;
  for (int it = tid; it < nitems; it += 256) {
    const int ic = it % CG;
    const int tt = it / CG;
    const int s = tt % nseg, ir = tt / nseg;
    const int w0 = s * SEG;
    if (h0 + ir >= a.H || c0 + w0 >= a.W || cbase + ic >= C8) continue;
    f32x2 acc[SEG][4];
#pragma unroll
    for (int o = 0; o < SEG; ++o)
#pragma unroll
      for (int d = 0; d < 4; ++d) acc[o][d] = (f32x2){0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      f32x2 wt[3][4];
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float* wp = wsm + (dy * 3 + dx) * CG * 8 + ic * 8;
        const float4 p = *(const float4*)wp;
        const float4 q = *(const float4*)(wp + 4);
        wt[dx][0] = (f32x2){p.x, p.y};
        wt[dx][1] = (f32x2){p.z, p.w};
        wt[dx][2] = (f32x2){q.x, q.y};
        wt[dx][3] = (f32x2){q.z, q.w};
      }
      const uint8_t* rowp = xsm + ((long)(ir + dy) * TWP * CG + ic) * 16;
#pragma unroll
      for (int j = 0; j < SEG + 2; ++j) {       // LDS column w0+j == input column c0+w0-1+j
        const int lc = min(w0 + j, TWP - 1);   // clamping only feeds outputs that are not stored
        const u32x4 v = *(const u32x4*)(rowp + (long)lc * CG * 16);
        f32x2 xv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) xv[d] = (f32x2){bf_lo(v[d]), bf_hi(v[d])};
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int o = j - dx;
          if (o >= 0 && o < SEG) {
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[o][d] = __builtin_elementwise_fma(xv[d], wt[dx][d], acc[o][d]);
          }
        }
      }
    }
    uint16_t* yb = a.y + ((img + h0 + ir) * a.W + c0 + w0) * a.C + (cbase + ic) * 8;
    const int lim = min(SEG, min(TW - w0, a.W - c0 - w0));
#pragma unroll
    for (int o = 0; o < SEG; ++o) {
      if (o < lim) {
        u32x4 out;
#pragma unroll
        for (int d = 0; d < 4; ++d) out[d] = pack_bf16(acc[o][d][0], acc[o][d][1]);
        *(u32x4*)(yb + (long)o * a.C) = out;
      }
    }
  }
}

static size_t dw_smem(int CG, int RB, int TW) {
  return (size_t)9 * CG * 8 * 4 + (size_t)(RB + 2) * (TW + 2) * CG * 16;
}

// Host tile choice (overridable per call through DwArgs.cg/rb/tw/seg), fitted to
// the batch-32 sweep of tools/dwbench.py on MI355X (profiles/dw_sweep.txt):
//   TW : whole rows up to 40 px, else the narrowest split into <= 49-px tiles;
//   SEG: 5 when it divides TW, else 7;
//   CG : 8 chunks (128 B per pixel) when C/8 allows it, else 4 (728 ch -> 92 = 4*23);
//   RB : tallest band (<= 19 rows) whose LDS image fits 80 KiB.
static void dw_pick(const DwArgs& a, int& CG, int& RB, int& TW, int& SEG) {
  const int C8 = a.C / 8;
  const int ncol = (a.W + 48) / 49;
  TW = a.tw > 0 ? a.tw : (a.W <= 40 ? a.W : (a.W + ncol - 1) / ncol);
  SEG = a.seg > 0 ? a.seg : (TW % 5 == 0 ? 5 : 7);
  CG = a.cg > 0 ? a.cg : (C8 % 8 == 0 ? 8 : (C8 % 4 == 0 ? 4 : (C8 % 2 == 0 ? 2 : 1)));
  if (a.rb > 0) {
    RB = a.rb;
  } else {
    RB = 1;
    while (RB < a.H && RB < 19 && dw_smem(CG, RB + 1, TW) <= 80 * 1024) ++RB;
  }
}

hipError_t dw3x3(const DwArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.W <= 0 || a.H <= 0 || a.B <= 0) return hipErrorInvalidValue;
  int CG, RB, TW, SEG;
  dw_pick(a, CG, RB, TW, SEG);
  const size_t smem = dw_smem(CG, RB, TW);
  if (CG <= 0 || RB <= 0 || TW <= 0 || smem > 160 * 1024 || (SEG != 5 && SEG != 7))
    return hipErrorInvalidValue;
  const long nblk = (long)a.B * ((a.H + RB - 1) / RB) * ((a.W + TW - 1) / TW) * ((a.C / 8 + CG - 1) / CG);
  if (SEG == 7) hipLaunchKernelGGL(dw3x3_tile_kernel<7>, dim3((unsigned)nblk), dim3(256), smem, s, a, CG, RB, TW);
  else hipLaunchKernelGGL(dw3x3_tile_kernel<5>, dim3((unsigned)nblk), dim3(256), smem, s, a, CG, RB, TW);
  return hipGetLastError();
}

}  // namespace kdl
