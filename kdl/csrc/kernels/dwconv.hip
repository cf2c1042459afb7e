// Depthwise 3x3 'same' conv (+ optional ReLU on load), NHWC bf16 -> bf16.
// SURVEY.md §2.5 K5. Used by the "split" lowering of SeparableConv2D (dw kernel
// then the MODE_PW GEMM); the autotuner picks split vs fused per layer. Two kernels:
// the LDS-tiled one below (algo 1) and the direct row-streaming one further down
// (algo 2, the default since it measured faster on every Xception shape).
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

// ---------------------------------------------------------------- direct row-streaming variant
// No LDS, no barrier. A thread owns one 4-channel chunk (8-byte loads) x SEG adjacent output
// columns x an RB-row band, flat-mapped with the chunk fastest: the 64 lanes of a wave read
// 512 contiguous bytes of one pixel row (consecutive chunks), not a CB x segment rectangle,
// so any C % 4 == 0 coalesces (Xception's 736-channel middle flow included). The band's
// input rows stream top to bottom, PD rows in flight ahead of the one being used; each row
// is loaded once, ReLU'd on load, unpacked once and FMA'd (packed fp32) into the
// accumulators of the up-to-3 output rows it feeds; an output row is stored as soon as its
// last input row has passed. The loop is unrolled by 3 input rows so every accumulator slot
// index is a compile-time constant. Workgroups are XCD-remapped so neighbouring bands (which
// share 2 halo rows) run on one XCD's L2. What it replaces: the LDS-tiled kernel above
// stages a patch, syncs, then computes, so one workgroup's loads never overlap its own
// arithmetic (measured 1.8 TB/s on the 19x19x736 middle-flow shape).
template <int SEG, int PD>
__global__ __launch_bounds__(256) void dw3x3_direct_kernel(DwArgs a, int RB, int nseg, int nbands, int nwg) {
  constexpr int NJ = SEG + 2;
  const int C4 = a.C >> 2;
  const long id = (long)xcd_remap(blockIdx.x, nwg) * 256 + threadIdx.x;
  const long total = (long)a.B * nbands * nseg * C4;
  if (id >= total) return;                       // no barrier anywhere below
  const int chunk = (int)(id % C4);
  long r = id / C4;
  const int seg = (int)(r % nseg);
  r /= nseg;
  const int band = (int)(r % nbands);
  const int b = (int)(r / nbands);
  const int ch = chunk * 4;
  const int w0 = seg * SEG, h0 = band * RB;
  const int rows = min(RB, a.H - h0);
  const int vmax = rows + 2;                     // input rows h0-1 .. h0+rows

  f32x2 wt[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float4 q = *(const float4*)(a.w + (long)t * a.C + ch);
    wt[t][0] = (f32x2){q.x, q.y};
    wt[t][1] = (f32x2){q.z, q.w};
  }
  f32x2 acc[3][SEG][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int o = 0; o < SEG; ++o) acc[s][o][0] = acc[s][o][1] = (f32x2){0.f, 0.f};

  const long img = (long)b * a.H;
  const uint16_t* xb = a.x + (img * a.W + (w0 - 1)) * a.C + ch;
  uint16_t* yb = a.y + (img * a.W + w0) * a.C + ch;
  bool cok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cok[j] = (unsigned)(w0 - 1 + j) < (unsigned)a.W;
  const bool relu = a.relu_in != 0;
  auto load = [&](int v, u32x2 (&xr)[NJ]) {
    const int ih = h0 - 1 + v;
    const bool rok = v < vmax && (unsigned)ih < (unsigned)a.H;
    const uint16_t* rp = xb + (long)ih * a.W * a.C;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      xr[j] = (rok && cok[j]) ? *(const u32x2*)(rp + (long)j * a.C) : (u32x2){0u, 0u};
  };
  auto finish = [&](f32x2 (&ac)[SEG][2], int ol) {
    uint16_t* rp = yb + (long)(h0 + ol) * a.W * a.C;
#pragma unroll
    for (int o = 0; o < SEG; ++o) {
      if (w0 + o < a.W)
        *(u32x2*)(rp + (long)o * a.C) = (u32x2){pack_bf16(ac[o][0][0], ac[o][0][1]),
                                                pack_bf16(ac[o][1][0], ac[o][1][1])};
      ac[o][0] = ac[o][1] = (f32x2){0.f, 0.f};
    }
  };

  u32x2 xq[PD + 1][NJ];
#pragma unroll
  for (int k = 0; k < PD; ++k) load(k, xq[k]);
  for (int v0 = 0; v0 < vmax; v0 += 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int v = v0 + u;
      if (v >= vmax) break;
      load(v + PD, xq[PD]);
      f32x2 xf[NJ][2];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        u32x2 d = xq[0][j];
        if (relu) { d[0] = relu_bf16x2(d[0]); d[1] = relu_bf16x2(d[1]); }
        xf[j][0] = (f32x2){bf_lo(d[0]), bf_hi(d[0])};
        xf[j][1] = (f32x2){bf_lo(d[1]), bf_hi(d[1])};
      }
      // input row v feeds output row ol = v - dy with tap row dy
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int ol = v - dy;
        if (ol < 0 || ol >= rows) continue;
        const int slot = (u - dy + 3) % 3;       // == ol % 3 (v0 is a multiple of 3)
#pragma unroll
        for (int o = 0; o < SEG; ++o)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              acc[slot][o][h] = __builtin_elementwise_fma(xf[o + dx][h], wt[dy * 3 + dx][h], acc[slot][o][h]);
        if (dy == 2) finish(acc[slot], ol);
      }
#pragma unroll
      for (int k = 0; k < PD; ++k)
#pragma unroll
        for (int j = 0; j < NJ; ++j) xq[k][j] = xq[k + 1][j];
    }
  }
}

// Direct-variant plan. The Xception shapes take (seg, rb, pd) from the batch-32 sweep of
// tools/dwbench.py --direct on MI355X (profiles/dw_direct_sweep.txt; 1.3-1.9x the tiled
// kernel on every shape); anything else gets SEG 3 and row bands sized for ~2 waves of
// 256-thread workgroups per SIMD over the 256 CUs. a.rb / a.seg / a.pd override.
struct DwdTile { short H, C, seg, rb, pd; };
static const DwdTile kDwdTable[] = {
    {147, 64, 3, 7, 1}, {147, 128, 4, 10, 2}, {74, 128, 3, 5, 1}, {74, 256, 3, 5, 1}, {37, 256, 3, 4, 1},
    {37, 736, 2, 19, 1}, {19, 736, 4, 5, 2},  {10, 1024, 4, 2, 1}, {10, 1536, 2, 5, 2},
};

static void dwd_plan(const DwArgs& a, int* seg, int* rb, int* pd, int* nseg, int* nbands) {
  const DwdTile* t = nullptr;
  for (const DwdTile& e : kDwdTable)
    if (e.H == a.H && e.H == a.W && e.C == a.C) t = &e;
  *seg = a.seg > 0 ? a.seg : t ? t->seg : 3;
  *nseg = (a.W + *seg - 1) / *seg;
  const long per_band = (long)a.B * *nseg * (a.C / 4);
  int R = a.rb > 0 ? a.rb : (t && a.seg <= 0) ? t->rb : 0;
  if (R <= 0) {
    long nb = (2L * 256 * 4 * 64 + per_band - 1) / per_band;
    nb = nb < 1 ? 1 : (nb > a.H ? a.H : nb);
    R = (int)((a.H + nb - 1) / nb);
    if (R < 3 && a.H >= 3) R = 3;
  }
  *rb = R;
  *nbands = (a.H + R - 1) / R;
  *pd = a.pd > 0 ? a.pd : (t && a.seg <= 0 && a.rb <= 0) ? t->pd : 1;
}

static hipError_t dw3x3_direct(const DwArgs& a, hipStream_t s) {
  int seg, rb, pd, nseg, nb;
  dwd_plan(a, &seg, &rb, &pd, &nseg, &nb);
  if (a.C % 4 != 0 || rb <= 0) return hipErrorInvalidValue;
  const long total = (long)a.B * nb * nseg * (a.C / 4);
  const long nblk = (total + 255) / 256;
  if (nblk >= (1L << 31)) return hipErrorInvalidValue;
  const int g = (int)nblk;
#define KDL_DWD(sg, p) \
  if (seg == sg && pd == p) { \
    hipLaunchKernelGGL((dw3x3_direct_kernel<sg, p>), dim3(g), dim3(256), 0, s, a, rb, nseg, nb, g); \
    return hipGetLastError(); }
  KDL_DWD(2, 1) KDL_DWD(2, 2) KDL_DWD(3, 1) KDL_DWD(3, 2) KDL_DWD(4, 1) KDL_DWD(4, 2)
#undef KDL_DWD
  return hipErrorInvalidValue;
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

// a.algo, else KDL_DW_ALGO (A/B runs), else the default below
static int dw_algo(const DwArgs& a) {
  if (a.algo > 0) return a.algo;
  static const int env = [] { const char* e = getenv("KDL_DW_ALGO"); return e ? atoi(e) : 0; }();
  if (env > 0) return env;
  return 2;                                      // direct: faster on every measured shape
}

hipError_t dw3x3(const DwArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.W <= 0 || a.H <= 0 || a.B <= 0) return hipErrorInvalidValue;
  if (dw_algo(a) == 2) return dw3x3_direct(a, s);
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
