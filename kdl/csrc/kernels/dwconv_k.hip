// MBConv depthwise KxK conv (K = 3/5, stride 1/2, symmetric pad) + folded BN bias
// + SiLU, NHWC bf16, with the squeeze-excite average pool AND the squeeze FC fused
// in: each tile reduces its channel sums and projects them on w1 (fc1 is linear in
// the mean), leaving only bias + SiLU + fc2 + sigmoid for se_kernel (SURVEY.md §2.6 EfficientNet-B7: "dw 5x5 (+stride
// 2), squeeze-excite ... SiLU epilogue"; the 600x600 large-activation path).
//
// Same tiling as dw3x3_tile_kernel (dwconv.hip): block = image x RB output rows x
// TW output columns x CG 8-channel chunks; the ((RB-1)S+K) x ((TW-1)S+K) input
// patch is staged once into LDS with all of a thread's loads in flight together;
// an item = (chunk, row, SEG-column segment) slides a register window along W.
// SE partial sums are reduced in a fixed order (deterministic, no atomics):
// CG divides 256, so every item of a thread has the same chunk.
#include <cstdlib>

#include "common.h"
#include "launch.h"

namespace kdl {

constexpr int DWK_MAXL = 8;

__device__ __forceinline__ float silu(float v) { return fast_silu(v); }

// SILU: the activation (DwkArgs.act 2) as a compile-time constant, like the streaming GEMM's: a run-time
// test in the store path splits it into branch blocks the scheduler cannot interleave
template <int K, int S, int SEG, bool SILU>
__global__ __launch_bounds__(256) void dwk_kernel(DwkArgs a, int CG, int RB, int TW) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int C8 = a.C >> 3;
  const int ngroups = C8 / CG;
  const int nbands = (a.OH + RB - 1) / RB;
  const int ncolt = (a.OW + TW - 1) / TW;
  int bid = blockIdx.x;
  const int g = bid % ngroups;
  bid /= ngroups;
  const int ct = bid % ncolt;
  bid /= ncolt;
  const int band = bid % nbands;
  const int b = bid / nbands;
  const int h0 = band * RB, c0 = ct * TW;
  const int PR = (RB - 1) * S + K, PC = (TW - 1) * S + K;
  const int ih0 = h0 * S - a.pad, iw0 = c0 * S - a.pad;
  const int tid = threadIdx.x;
  const int cbase = g * CG;

  float* wsm = (float*)dsm;                                 // [K*K][CG*8]
  uint8_t* xsm = dsm + K * K * CG * 8 * 4;                  // [PR][PC][CG][16B]
  for (int i = tid; i < K * K * CG * 2; i += 256) {
    const int tap = i / (CG * 2), rem = i - tap * CG * 2;
    const int c = rem >> 1, half = rem & 1;
    *(float4*)(wsm + tap * CG * 8 + c * 8 + half * 4) = *(const float4*)(a.w + tap * a.C + (cbase + c) * 8 + half * 4);
  }
  const int nst = PR * PC * CG;
  const int dc = 256 % CG, dt = 256 / CG;
  const int dcol = dt % PC, dr = dt / PC;
  int c = tid % CG, t = tid / CG;
  int col = t % PC, r = t / PC;
  const long img = (long)b * a.H;
  // stride 2: the patch is stored column-deinterleaved (even columns, then odd), so the
  // items of a wave -- SEG*S columns apart -- start on different 16-byte bank slots when
  // SEG is odd (ds_read_b128 conflicts within 16-lane groups otherwise: an even distance
  // puts every item of a chunk on the same slot)
  const int PCe = (PC + 1) >> 1;
  auto pcol = [&](int cc) { return S == 2 ? (cc & 1) * PCe + (cc >> 1) : cc; };
  for (int base = 0; base < nst; base += 256 * DWK_MAXL) {
    u32x4 v[DWK_MAXL];
    int cc[DWK_MAXL], cl[DWK_MAXL], rr[DWK_MAXL];
#pragma unroll
    for (int l = 0; l < DWK_MAXL; ++l) {
      cc[l] = c; cl[l] = col; rr[l] = r;
      v[l] = (u32x4){0u, 0u, 0u, 0u};
      const int ih = ih0 + r, iw = iw0 + col;
      if (base + tid + l * 256 < nst && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        v[l] = *(const u32x4*)(a.x + ((img + ih) * a.W + iw) * a.C + (cbase + c) * 8);
      c += dc;
      int carry = c >= CG;
      c -= carry ? CG : 0;
      col += dcol + carry;
      carry = col >= PC;
      col -= carry ? PC : 0;
      r += dr + carry;
    }
#pragma unroll
    for (int l = 0; l < DWK_MAXL; ++l)
      if (base + tid + l * 256 < nst) *(u32x4*)(xsm + (((long)rr[l] * PC + pcol(cl[l])) * CG + cc[l]) * 16) = v[l];
  }
  __syncthreads();

  const int nseg = (TW + SEG - 1) / SEG;
  const int nitems = CG * RB * nseg;
  const int ic = tid % CG;                 // CG divides 256: fixed chunk per thread
  const float4 bz0 = *(const float4*)(a.bias + (cbase + ic) * 8);
  const float4 bz1 = *(const float4*)(a.bias + (cbase + ic) * 8 + 4);
  const float bias[8] = {bz0.x, bz0.y, bz0.z, bz0.w, bz1.x, bz1.y, bz1.z, bz1.w};
  float psum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int it = tid; it < nitems; it += 256) {
    const int tt = it / CG;
    const int s = tt % nseg, ir = tt / nseg;
    const int w0 = s * SEG;
    if (h0 + ir >= a.OH || c0 + w0 >= a.OW) continue;
    f32x2 acc[SEG][4];
#pragma unroll
    for (int o = 0; o < SEG; ++o)
#pragma unroll
      for (int d = 0; d < 4; ++d) acc[o][d] = (f32x2){0.f, 0.f};
    // dy stays a rolled loop: unrolled, hipcc hoists all K*K taps' weights out of
    // the item loop (200 VGPRs at K=5 -> 512 VGPRs + scratch spills)
#pragma unroll 1
    for (int dy = 0; dy < K; ++dy) {
      f32x2 wt[K][4];
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const float* wp = wsm + (dy * K + dx) * CG * 8 + ic * 8;
        const float4 p = *(const float4*)wp;
        const float4 q = *(const float4*)(wp + 4);
        wt[dx][0] = (f32x2){p.x, p.y};
        wt[dx][1] = (f32x2){p.z, p.w};
        wt[dx][2] = (f32x2){q.x, q.y};
        wt[dx][3] = (f32x2){q.z, q.w};
      }
      const uint8_t* rowp = xsm + ((long)(ir * S + dy) * PC * CG + ic) * 16;
#pragma unroll
      for (int j = 0; j < (SEG - 1) * S + K; ++j) {
        const int lc = min(w0 * S + j, PC - 1);   // clamping only feeds outputs that are not stored
        const u32x4 v = *(const u32x4*)(rowp + (long)pcol(lc) * CG * 16);
        f32x2 xv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) xv[d] = (f32x2){bf_lo(v[d]), bf_hi(v[d])};
#pragma unroll
        for (int o = 0; o < SEG; ++o) {
          const int dx = j - o * S;
          if (dx >= 0 && dx < K) {
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[o][d] = __builtin_elementwise_fma(xv[d], wt[dx][d], acc[o][d]);
          }
        }
      }
    }
    uint16_t* yb = a.y + (((long)b * a.OH + h0 + ir) * a.OW + c0 + w0) * a.C + (cbase + ic) * 8;
    const int lim = min(SEG, min(TW - w0, a.OW - c0 - w0));
#pragma unroll
    for (int o = 0; o < SEG; ++o) {
      if (o < lim) {
        float f[8];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          f[2 * d] = acc[o][d][0] + bias[2 * d];
          f[2 * d + 1] = acc[o][d][1] + bias[2 * d + 1];
        }
        u32x4 out;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if constexpr (SILU) {
            f[2 * d] = silu(f[2 * d]);
            f[2 * d + 1] = silu(f[2 * d + 1]);
          }
          out[d] = pack_bf16(f[2 * d], f[2 * d + 1]);
          // the SE pool sees exactly the stored (bf16-rounded) activations
          psum[2 * d] += bf_lo(out[d]);
          psum[2 * d + 1] += bf_hi(out[d]);
        }
        *(u32x4*)(yb + (long)o * a.C) = out;
      }
    }
  }
  if (a.pool) {
    __syncthreads();                       // staging image no longer needed
    float* red = (float*)dsm;              // [256][8]
#pragma unroll
    for (int d = 0; d < 8; ++d) red[tid * 8 + d] = psum[d];
    __syncthreads();
    float sum = 0.f;
    if (tid < CG * 8) {
      const int rc = tid >> 3, d = tid & 7;
      for (int u = rc; u < 256; u += CG) sum += red[u * 8 + d];
    }
    __syncthreads();
    float* csum = red + 256 * 8;             // [CG*8] channel sums of this tile
    if (tid < CG * 8) csum[tid] = sum;
    __syncthreads();
    // squeeze FC fused: this tile's contribution to h[j] = sum_c w1[j][c] * mean[c]
    // (the mean is linear in the tiles' sums; se_kernel adds the parts up)
    const int part = (band * ncolt + ct) * ngroups + g;
    const int nparts = nbands * ncolt * ngroups;
    for (int j = tid; j < a.Cs; j += 256) {
      const float* w1 = a.w1 + (long)j * a.C + cbase * 8;
      float h = 0.f;
      for (int cc8 = 0; cc8 < CG * 8; ++cc8) h += w1[cc8] * csum[cc8];
      a.pool[((long)b * nparts + part) * a.Cs + j] = h;
    }
  }
}

static size_t dwk_smem(int K, int S, int CG, int RB, int TW) {
  const size_t patch = (size_t)((RB - 1) * S + K) * ((TW - 1) * S + K) * CG * 16;
  const size_t w = (size_t)K * K * CG * 8 * 4;
  const size_t red = (256 * 8 + 64) * 4;
  return w + patch > red ? w + patch : red;
}

// Tile choice. Measured (tools/dwkbench.py --grid, batch 32, profiles/dwk_sweep.txt): the
// EfficientNet-B7 shapes take their best (cg, rb, tw, seg) from the table below; any other
// shape gets the fallback: column tiles of <= 38 outputs (19 at stride 2), for each
// power-of-two chunk group CG in {8, 4, 2, 1} dividing C/8 the tallest row band (<= 8) that
// fits 52 KiB of LDS -- three workgroups per CU, so one tile's staging loads overlap the
// others' arithmetic (the first heuristic filled 96 KiB: one workgroup, one wave per SIMD,
// 25 % slower summed over B7) -- keep the CG with the tallest band, ties -> wider CG.
// SEG odd: the items of a wave then start on different LDS bank slots (stride 2: with the
// patch column-deinterleaved). a.cg/rb/tw/seg override everything.
// 5x5 stride-1 rows at 75x75x480 / 38x38x960 / 38x38x1344 moved to the direct kernel once it took wide
// chunk blocks (profiles/dwv_wide_ab.txt: 203 -> 170, 90 -> 86, 127 -> 106 us)
struct DwkTile { short H, W, C, K, S, algo, cg, rb, tw, seg; };   // algo 2: rb / seg of dwv_kernel, tw = prefetch rows
static const DwkTile kDwkTable[] = {
    {300, 300, 64, 3, 1, 2, 0, 16, 0, 4},   {300, 300, 32, 3, 1, 2, 0, 16, 0, 2},  {300, 300, 192, 3, 2, 2, 0, 6, 0, 2},
    {150, 150, 288, 3, 1, 2, 0, 38, 0, 2},  {150, 150, 288, 5, 2, 2, 0, 16, 0, 4}, {75, 75, 480, 5, 1, 2, 0, 38, 3, 2},
    {75, 75, 480, 3, 2, 2, 0, 38, 0, 2},    {38, 38, 960, 3, 1, 2, 0, 8, 0, 4},    {38, 38, 960, 5, 1, 2, 0, 38, 3, 2},
    {38, 38, 1344, 5, 1, 2, 0, 38, 1, 2},   {38, 38, 1344, 5, 2, 2, 0, 12, 0, 2},  {19, 19, 2304, 5, 1, 1, 8, 12, 19, 5},
    {19, 19, 2304, 3, 1, 1, 8, 8, 19, 5},   {19, 19, 3840, 3, 1, 1, 8, 12, 19, 5},
};

static const DwkTile* dwk_lookup(const DwkArgs& a) {
  for (const DwkTile& t : kDwkTable)
    if (t.H == a.H && t.W == a.W && t.C == a.C && t.K == a.K && t.S == a.S) return &t;
  return nullptr;
}

static void dwt_tiles(const DwkArgs& a, int* cg, int* rb, int* tw, int* ntiles) {
  const int C8 = a.C / 8;
  const DwkTile* t = dwk_lookup(a);
  if (a.cg > 0 && a.rb > 0 && a.tw > 0) {
    *cg = a.cg; *rb = a.rb; *tw = a.tw;
  } else if (t != nullptr && t->algo == 1 && a.lds_kb == 0) {
    *cg = t->cg; *rb = t->rb; *tw = t->tw;
  } else {
    const int budget = (a.lds_kb > 0 ? a.lds_kb : 52) * 1024;
    const int cap = a.S == 1 ? 38 : 19;
    const int ncol = (a.OW + cap - 1) / cap;
    const int TW = (a.OW + ncol - 1) / ncol;
    int bestcg = 1, bestrb = 0;
    for (int CG : {8, 4, 2, 1}) {
      if (C8 % CG != 0) continue;
      int RB = 1;
      while (RB < a.OH && RB < 8 && dwk_smem(a.K, a.S, CG, RB + 1, TW) <= (size_t)budget) ++RB;
      if (dwk_smem(a.K, a.S, CG, RB, TW) > (size_t)budget) continue;
      if (RB > bestrb) { bestrb = RB; bestcg = CG; }
    }
    if (bestrb == 0) bestrb = 1;
    *cg = bestcg; *rb = bestrb; *tw = TW;
  }
  *ntiles = ((a.OH + *rb - 1) / *rb) * ((a.OW + *tw - 1) / *tw) * (C8 / *cg);
}

static int dwt_seg(const DwkArgs& a) {
  if (a.seg > 0) return a.seg;
  const DwkTile* t = dwk_lookup(a);
  if (t != nullptr && t->algo == 1 && a.lds_kb == 0 && a.cg == 0) return t->seg;
  return a.S == 1 ? 5 : 3;
}

static hipError_t dwt(const DwkArgs& a, hipStream_t s) {
  int CG, RB, TW, nt;
  dwt_tiles(a, &CG, &RB, &TW, &nt);
  // CG: a power of two <= 8 dividing C/8 (fixed chunk per thread; the pool reduction's
  // CG*8 channel sums fit the 64-float tail of the reduction buffer)
  if ((CG & (CG - 1)) != 0 || CG > 8 || (a.C / 8) % CG != 0 || RB <= 0 || TW <= 0) return hipErrorInvalidValue;
  const size_t smem = dwk_smem(a.K, a.S, CG, RB, TW);
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const long nblk = (long)a.B * nt;          // nt counts (row band, column tile, channel group)
  if (nblk >= (1L << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk), block(256);
  const int seg = dwt_seg(a);
#define KDL_DWK(k, st, sg) \
  if (a.K == k && a.S == st && seg == sg) { \
    if (a.act == 2) hipLaunchKernelGGL((dwk_kernel<k, st, sg, true>), grid, block, smem, s, a, CG, RB, TW); \
    else hipLaunchKernelGGL((dwk_kernel<k, st, sg, false>), grid, block, smem, s, a, CG, RB, TW); \
    return hipGetLastError(); }
#define KDL_DWK_SEGS(k, st) KDL_DWK(k, st, 3) KDL_DWK(k, st, 4) KDL_DWK(k, st, 5) KDL_DWK(k, st, 7) KDL_DWK(k, st, 8)
  KDL_DWK_SEGS(3, 1) KDL_DWK_SEGS(3, 2) KDL_DWK_SEGS(5, 1) KDL_DWK_SEGS(5, 2)
#undef KDL_DWK_SEGS
#undef KDL_DWK
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------- direct streaming variant
// No LDS staging: a thread owns one 4-channel chunk (8-byte loads, 64 chunk lanes of a
// wave read 512 contiguous bytes) and SEG adjacent output columns of a row band, and
// streams the band's input rows top to bottom. Each input row is loaded once (the next
// one is in flight while this one is used), unpacked once, and scattered into the
// accumulators of the R = ceil(K/S) output rows it feeds; an output row is finished
// (bias, SiLU, bf16 store, SE pool) when its last input row has passed. The row loop is
// unrolled by R*S input rows so every accumulator slot index is a compile-time constant.
// The tap weights live in registers for the whole band. What this replaces: the tiled
// kernel above stages the whole patch, syncs, then computes, so one workgroup's loads never
// overlap its own arithmetic and its LDS budget caps the CU at 1-3 workgroups.
// Workgroup = CB chunk lanes x (256/CB) segment lanes of one (image, row band); the SE
// partials are per workgroup (part = band x segment block x chunk block).
// smallest divisor of P that is >= N (P itself if none is smaller)
template <int P, int N>
constexpr int dwv_ring() {
  for (int d = N; d < P; ++d)
    if (P % d == 0) return d;
  return P;
}

template <int K, int S, int SEG, int CB, int PD, bool SILU>
__global__ __launch_bounds__(256) void dwv_kernel(DwkArgs a, int RB) {
  constexpr int R = (K + S - 1) / S;       // output rows in flight
  constexpr int P = R * S;                 // unroll period (input rows)
  constexpr int NJ = (SEG - 1) * S + K;    // input columns per thread
  constexpr int SL = 256 / CB;             // segment lanes per workgroup
  __shared__ float red[256 * 4 + CB * 4];
  const int C4 = a.C >> 2;
  const int nseg = (a.OW + SEG - 1) / SEG;
  const int nsb = (nseg + SL - 1) / SL;
  const int ncb = C4 / CB;
  const int nbands = (a.OH + RB - 1) / RB;
  int bid = blockIdx.x;
  const int cbk = bid % ncb;
  bid /= ncb;
  const int sb = bid % nsb;
  bid /= nsb;
  const int band = bid % nbands;
  const int b = bid / nbands;
  const int tid = threadIdx.x;
  const int cl = tid % CB, sl = tid / CB;
  const int ch = (cbk * CB + cl) * 4;
  const int seg = sb * SL + sl;
  const bool live = sl < SL && seg < nseg;     // CB not dividing 256: the last 256 % CB lanes idle
  const int w0 = seg * SEG;
  const int h0 = band * RB;
  const int rows = min(RB, a.OH - h0);
  const int iw0 = w0 * S - a.pad, ih0 = h0 * S - a.pad;
  const int vmax = (rows - 1) * S + K;

  f32x2 wt[K * K][2];
#pragma unroll
  for (int t = 0; t < K * K; ++t) {
    const float4 q = *(const float4*)(a.w + (long)t * a.C + ch);
    wt[t][0] = (f32x2){q.x, q.y};
    wt[t][1] = (f32x2){q.z, q.w};
  }
  const float4 bq = *(const float4*)(a.bias + ch);
  f32x2 acc[R][SEG][2];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int o = 0; o < SEG; ++o) acc[r][o][0] = acc[r][o][1] = (f32x2){0.f, 0.f};
  float psum[4] = {0.f, 0.f, 0.f, 0.f};

  const uint16_t* xb = a.x + (long)b * a.H * a.W * a.C + ch;
  uint16_t* yb = a.y + (long)b * a.OH * a.OW * a.C + ch;
  bool cok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cok[j] = live && (unsigned)(iw0 + j) < (unsigned)a.W;
  auto load = [&](int v, u32x2 (&xr)[NJ]) {
    const int ih = ih0 + v;
    const bool rok = v < vmax && (unsigned)ih < (unsigned)a.H;
    const uint16_t* rp = xb + ((long)ih * a.W + iw0) * a.C;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      xr[j] = (rok && cok[j]) ? *(const u32x2*)(rp + (long)j * a.C) : (u32x2){0u, 0u};
  };
  auto finish = [&](f32x2 (&ac)[SEG][2], int ol) {
    uint16_t* rp = yb + ((long)(h0 + ol) * a.OW + w0) * a.C;
#pragma unroll
    for (int o = 0; o < SEG; ++o) {
      float f0 = ac[o][0][0] + bq.x, f1 = ac[o][0][1] + bq.y, f2 = ac[o][1][0] + bq.z, f3 = ac[o][1][1] + bq.w;
      if constexpr (SILU) { f0 = silu(f0); f1 = silu(f1); f2 = silu(f2); f3 = silu(f3); }
      const u32x2 out = {pack_bf16(f0, f1), pack_bf16(f2, f3)};
      if (live && w0 + o < a.OW) {
        *(u32x2*)(rp + (long)o * a.C) = out;
        psum[0] += bf_lo(out[0]); psum[1] += bf_hi(out[0]);
        psum[2] += bf_lo(out[1]); psum[3] += bf_hi(out[1]);
      }
      ac[o][0] = ac[o][1] = (f32x2){0.f, 0.f};
    }
  };

  // Row ring of RS slots, RS the smallest divisor of the unroll period P holding PD + 1 rows: row v
  // lives in slot v % RS (= u % RS, v0 being a multiple of P), and row v + RS - 1 is issued at the
  // top of step v into the slot row v - 1 just left -- every slot index is a compile-time constant,
  // so the ring never moves (the earlier xq[k] = xq[k + 1] rotation cost NJ * PD * 2 moves per row:
  // 36 for the 5x5 kernel against its 100 FMAs). RS - 1 >= PD rows of arithmetic cover each load.
  constexpr int RS = dwv_ring<P, PD + 1>();
  constexpr int LA = RS - 1;                 // look-ahead (rows in flight)
  u32x2 xq[RS][NJ];
#pragma unroll
  for (int k = 0; k < LA; ++k) load(k, xq[k]);
  for (int v0 = 0; v0 < vmax; v0 += P) {
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int v = v0 + u;
      if (v >= vmax) break;
      load(v + LA, xq[(u + LA) % RS]);
      const u32x2 (&xc)[NJ] = xq[u % RS];
      f32x2 xf[NJ][2];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        xf[j][0] = (f32x2){bf_lo(xc[j][0]), bf_hi(xc[j][0])};
        xf[j][1] = (f32x2){bf_lo(xc[j][1]), bf_hi(xc[j][1])};
      }
#pragma unroll
      for (int dy = 0; dy < K; ++dy) {
        if constexpr (true) {
          if (((u - dy) % S + S) % S != 0) continue;
          const int slot = (((u - dy + P) / S) % R);
          const int ol = (v - dy) / S;
          if (v - dy < 0 || ol >= rows) continue;
#pragma unroll
          for (int o = 0; o < SEG; ++o)
#pragma unroll
            for (int dx = 0; dx < K; ++dx)
#pragma unroll
              for (int h = 0; h < 2; ++h)
                acc[slot][o][h] = __builtin_elementwise_fma(xf[o * S + dx][h], wt[dy * K + dx][h], acc[slot][o][h]);
          if (dy == K - 1) finish(acc[slot], ol);
        }
      }
    }
  }

  if (a.pool) {
#pragma unroll
    for (int d = 0; d < 4; ++d) red[tid * 4 + d] = psum[d];
    __syncthreads();
    float* csum = red + 256 * 4;
    if (tid < CB * 4) {
      const int c = tid >> 2, d = tid & 3;
      float sum = 0.f;
      for (int l = 0; l < SL; ++l) sum += red[(l * CB + c) * 4 + d];   // fixed order
      csum[tid] = sum;
    }
    __syncthreads();
    const int part = (band * nsb + sb) * ncb + cbk;
    const int nparts = nbands * nsb * ncb;
    for (int j = tid; j < a.Cs; j += 256) {
      const float* w1 = a.w1 + (long)j * a.C + cbk * CB * 4;
      float h = 0.f;
      for (int c = 0; c < CB * 4; ++c) h += w1[c] * csum[c];
      a.pool[((long)b * nparts + part) * a.Cs + j] = h;
    }
  }
}

// Direct-variant plan: CB = widest chunk block dividing C/4; SEG 2 for 5x5, 4 for 3x3;
// row bands sized for >= 64 workgroups per image (the engine sizes the SE partials per
// image, so the plan must not depend on the batch). When only a 8/16-chunk block divides
// C/4 (64/128 contiguous bytes per pixel: half-used cache lines, e.g. B7's 288 / 960 / 192
// channels), a wider non-power-of-two block (24..48 chunks, the last 256 % CB lanes idle)
// is taken instead (KDL_DWV_WIDE=0 restores the power-of-two rule).
static void dwv_plan(const DwkArgs& a, int* cb, int* rb, int* seg, int* ntiles) {
  const int C4 = a.C / 4;
  *cb = 0;
  for (int c : {64, 32, 16, 8})
    if (C4 % c == 0) { *cb = c; break; }
  static const bool wide = [] { const char* e = getenv("KDL_DWV_WIDE"); return !e || atoi(e) != 0; }();
  // measured (profiles/dwv_wide_ab.txt): 150x150x288 s1 -13 %, 38x38x960 s1 -15 %, 75x75x480 s2
  // -6 %, but 300x300x192 s2 (16 -> 48 chunks) +5 %: a 16-chunk block is widened at stride 1 only
  if (wide && (*cb == 8 || (*cb == 16 && a.S == 1)) && a.cg <= 0)
    for (int c : {48, 40, 36, 24})
      if (C4 % c == 0) { *cb = c; break; }
  if (a.cg > 0 && C4 % a.cg == 0) *cb = a.cg;  // explicit chunk block (sweeps)
  const DwkTile* t = dwk_lookup(a);
  const bool tab = t != nullptr && t->algo == 2;
  *seg = a.seg > 0 ? a.seg : tab ? t->seg : (a.K == 5 ? 2 : 4);
  const int nseg = (a.OW + *seg - 1) / *seg;
  const int SL = *cb > 0 ? 256 / *cb : 1;
  const int nsb = (nseg + SL - 1) / SL, ncb = *cb > 0 ? C4 / *cb : 1;
  int R = a.rb > 0 ? a.rb : tab ? t->rb : 0;
  if (R <= 0) {
    int nb = (64 + nsb * ncb - 1) / (nsb * ncb);
    nb = nb < 1 ? 1 : (nb > a.OH ? a.OH : nb);
    R = (a.OH + nb - 1) / nb;
  }
  *rb = R;
  *ntiles = ((a.OH + R - 1) / R) * nsb * ncb;
}

// Which kernel: a.algo, else KDL_DWK_ALGO (A/B runs), else the measured table's choice,
// else the tiled kernel (tools/dwkbench.py --direct, profiles/dwk_sweep.txt: the direct
// kernel wins the large-map / stride-2 / 3x3 layers, the tiled one the 5x5 stride-1 layers
// with many channels, where 25 taps x 8 channels of weights in registers cost occupancy).
static int dwk_algo(const DwkArgs& a) {
  int al = a.algo;
  if (al == 0 && a.cg == 0) {
    static const int env = [] { const char* e = getenv("KDL_DWK_ALGO"); return e ? atoi(e) : 0; }();
    al = env;
  }
  if (al == 0 && a.cg == 0 && a.lds_kb == 0) {
    const DwkTile* t = dwk_lookup(a);
    if (t != nullptr) al = t->algo;
  }
  if (al == 0) al = 1;
  if (al == 2 && a.C % 32 != 0) al = 1;
  return al;
}

void dwk_tiles(const DwkArgs& a, int* cg, int* rb, int* tw, int* ntiles) {
  if (dwk_algo(a) == 2) {
    int seg;
    dwv_plan(a, cg, rb, &seg, ntiles);
    *tw = 0;
    return;
  }
  dwt_tiles(a, cg, rb, tw, ntiles);
}

int dwk_seg(const DwkArgs& a) {
  if (dwk_algo(a) == 2) {
    int cb, rb, seg, nt;
    dwv_plan(a, &cb, &rb, &seg, &nt);
    return seg;
  }
  return dwt_seg(a);
}

hipError_t dwk(const DwkArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.B <= 0 || (a.K != 3 && a.K != 5) || (a.S != 1 && a.S != 2)) return hipErrorInvalidValue;
  if (dwk_algo(a) != 2) return dwt(a, s);
  int CB, RB, SEG, nt;
  dwv_plan(a, &CB, &RB, &SEG, &nt);
  const DwkTile* tb = dwk_lookup(a);
  const int PDv = a.pd > 0 ? a.pd : (tb != nullptr && tb->algo == 2 && tb->tw > 0) ? tb->tw : 1;
  if (CB == 0 || RB <= 0 || (SEG != 2 && SEG != 4) || (PDv != 1 && PDv != 3)) return hipErrorInvalidValue;
  const long nblk = (long)a.B * nt;
  if (nblk >= (1L << 31)) return hipErrorInvalidValue;
#define KDL_DWV1(k, st, sg, cb, pd)                                                                     \
  if (a.K == k && a.S == st && SEG == sg && CB == cb && PDv == pd) {                                  \
    if (a.act == 2) hipLaunchKernelGGL((dwv_kernel<k, st, sg, cb, pd, true>), dim3((unsigned)nblk), dim3(256), 0, s, a, RB); \
    else hipLaunchKernelGGL((dwv_kernel<k, st, sg, cb, pd, false>), dim3((unsigned)nblk), dim3(256), 0, s, a, RB); \
    return hipGetLastError();                                                                         \
  }
#define KDL_DWV(k, st, sg, cb) KDL_DWV1(k, st, sg, cb, 1) KDL_DWV1(k, st, sg, cb, 3)
#define KDL_DWV_CB(k, st, sg) KDL_DWV(k, st, sg, 8) KDL_DWV(k, st, sg, 16) KDL_DWV(k, st, sg, 32) KDL_DWV(k, st, sg, 64) \
  KDL_DWV(k, st, sg, 24) KDL_DWV(k, st, sg, 36) KDL_DWV(k, st, sg, 40) KDL_DWV(k, st, sg, 48)
#define KDL_DWV_KS(k, st) KDL_DWV_CB(k, st, 2) KDL_DWV_CB(k, st, 4)
  KDL_DWV_KS(3, 1) KDL_DWV_KS(3, 2) KDL_DWV_KS(5, 1) KDL_DWV_KS(5, 2)
#undef KDL_DWV_KS
#undef KDL_DWV_CB
#undef KDL_DWV
#undef KDL_DWV1
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------- squeeze-excite
// grid (image, 256-channel slice). Each workgroup sums the tile partials of the fused
// pool (ntiles x Cs floats) with all 256 threads: G = 256 / Cs thread groups each sum
// every G-th tile of every unit in a fixed order, then one thread per unit adds the G
// group sums in order (deterministic: atomics would make the sums order-dependent, and
// 55 blocks of SiLU amplify that run-to-run); bias + SiLU; then its 256 channels run fc2
// with the TRANSPOSED w2 ([Cs][C]: coalesced across threads) and the sigmoid. The first
// form summed the tiles serially in Cs threads (~35 us per call on B7); one workgroup
// per image then left the 3840 x 160 fc2 of the late stages on 32 CUs.
__global__ __launch_bounds__(256) void se_kernel(SeArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // [256] group sums, [Cs] hidden
  float* part = sm;
  float* hid = sm + 256;
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* pb = a.pool + (long)b * a.ntiles * a.Cs;
  const int G = a.Cs <= 256 ? 256 / a.Cs : 1;
  if (a.Cs <= 256) {
    const int g = tid / a.Cs, j = tid - g * a.Cs;
    if (g < G) {
      float h = 0.f;
      for (int t = g; t < a.ntiles; t += G) h += pb[(long)t * a.Cs + j];
      part[g * a.Cs + j] = h;
    }
  }
  __syncthreads();
  const float inv = 1.f / (float)a.HW;
  for (int j = tid; j < a.Cs; j += 256) {
    float h = 0.f;
    if (a.Cs <= 256) {
      for (int g = 0; g < G; ++g) h += part[g * a.Cs + j];
    } else {
      for (int t = 0; t < a.ntiles; ++t) h += pb[(long)t * a.Cs + j];
    }
    hid[j] = silu(h * inv + a.b1[j]);
  }
  __syncthreads();
  // fc2 for this workgroup's 256-channel slice (grid.y): the hidden vector above is
  // recomputed per slice (ntiles x Cs adds, cheap), so the C x Cs fc2 of the wide late
  // stages (3840 x 160) spreads over C/256 workgroups per image instead of one
  const int c = blockIdx.y * 256 + tid;
  if (c < a.C) {
    float s = a.b2[c];
#pragma unroll 8
    for (int j = 0; j < a.Cs; ++j) s += a.w2t[(long)j * a.C + c] * hid[j];
    a.scale[(long)b * a.C + c] = 1.f / (1.f + __expf(-s));
  }
}

hipError_t squeeze_excite(const SeArgs& a, hipStream_t s) {
  if (a.B <= 0 || a.Cs <= 0 || a.ntiles <= 0 || a.C <= 0 || a.B > 65535) return hipErrorInvalidValue;
  const size_t smem = (size_t)(256 + a.Cs) * sizeof(float);
  hipLaunchKernelGGL(se_kernel, dim3(a.B, (a.C + 255) / 256), dim3(256), smem, s, a);
  return hipGetLastError();
}

// y[b][p][c] *= scale[b][c] (in place, 16-byte vectors); grid (ceil(HW*C/8 / 256), B): the
// image index is blockIdx.y and the channel chunk one 32-bit modulo (the flat 64-bit
// index version spent more VALU on div/mod than on the scaling)
__global__ __launch_bounds__(256) void chscale_kernel(ChScaleArgs a) {
  const int C8 = a.C / 8;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.HW * C8) return;
  const int b = blockIdx.y;
  const int c8 = (int)((unsigned)j % (unsigned)C8);
  uint16_t* p = a.y + ((long)b * a.HW * C8 + j) * 8;
  const float4* sc = (const float4*)(a.scale + (long)b * a.C + c8 * 8);
  const float4 s0 = sc[0], s1 = sc[1];
  u32x4 v = *(const u32x4*)p;
  v[0] = pack_bf16(bf_lo(v[0]) * s0.x, bf_hi(v[0]) * s0.y);
  v[1] = pack_bf16(bf_lo(v[1]) * s0.z, bf_hi(v[1]) * s0.w);
  v[2] = pack_bf16(bf_lo(v[2]) * s1.x, bf_hi(v[2]) * s1.y);
  v[3] = pack_bf16(bf_lo(v[3]) * s1.z, bf_hi(v[3]) * s1.w);
  *(u32x4*)p = v;
}

hipError_t channel_scale(const ChScaleArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.B <= 0 || a.B > 65535 || a.HW <= 0 || (long)a.HW * (a.C / 8) >= (1L << 31))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)(((long)a.HW * (a.C / 8) + 255) / 256), (unsigned)a.B);
  hipLaunchKernelGGL(chscale_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}


}  // namespace kdl
