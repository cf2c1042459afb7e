// Fused SeparableConv2D (+BN)(+ReLU in/out)(+residual) over 2-D SPATIAL tiles, for
// the large-activation early flow of Xception (147x147 and 74x74 feature maps).
//
// Same machinery as sepconv_ws.hip (depthwise 3x3 as a block-diagonal 16x16x144
// GEMM on the matrix cores, pointwise MFMAs, one barrier per 32-channel k-step over an
// LDS-DMA ring), but the M tile is a TH x TW rectangle of output pixels of one image
// instead of BM consecutive raster pixels. Why: a raster tile needs a staged band of
// BM + 2W + 2 pixels (one halo row above and below), i.e. 4-6x the tile at W = 147,
// which does not fit LDS, so sepconv_ws cannot run there at all and the split path
// (dw3x3 kernel -> HBM -> pointwise GEMM) pays a full write + read of the depthwise
// output: ~180 MB per 147x147x128 layer at batch 32. A 2-D tile stages only its
// (TH+2) x (TW+2) halo patch (1.5x for 6x16), so the depthwise output never leaves
// the CU and the layer moves ~x + y bytes.
//
// Patch layout per stage: 4 planes (one per 8-channel chunk of the 32-channel k-step),
// each (TH+2) rows x (TW+2) pixel slots of 16 bytes, row-major, then zero slots up to
// a whole number of 64-slot LDS-DMA instructions. Pixels outside the image are
// staged as zeros (the source pointer of their lane is a zero buffer), so the
// depthwise reads need no bounds logic. A 16-pixel MFMA fragment is one tile row
// segment (TW is a multiple of 16): its 16 lanes read 256 contiguous bytes per tap,
// conflict-free.
#include "common.h"
#include "launch.h"
#include "epilogue.h"

#include <algorithm>

namespace kdl {

__device__ __attribute__((aligned(16))) uint8_t s2d_zeros[16384];   // +64 B per k-step: K <= 8192

template <int N>
__device__ __forceinline__ void s2_wait_barrier() {
  // lgkmcnt(0): this wave's depthwise ds_writes into the next A tile are complete
  // before anyone passes the barrier and reads them
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int TH, int TW>
struct S2dPatch {
  static constexpr int PW = TW + 2;                    // patch row pitch in slots
  static constexpr int PS = (TH + 2) * PW;             // patch slots
  static constexpr int IPP = (PS + 1 + 63) / 64;       // glds instructions per plane (>= 1 zero slot)
  static constexpr int ZSLOT = 64 * IPP - 1;
  static constexpr int XB = 4 * IPP;                   // KiB of patch per stage
};

template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW, bool RELU>
__global__ __launch_bounds__(64 * WGM * WGN) void sepconv_2d_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  static_assert(BM == TH * TW && TW % 16 == 0, "the M tile is TH x TW pixels, 16-pixel row segments");
  static_assert(NW % 2 == 0, "a wave's depthwise units share one channel group");
  using P = S2dPatch<TH, TW>;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int IPP = P::IPP, XB = P::XB;
  constexpr int PL = IPP * 1024;                // bytes per plane
  constexpr int XI = BF + XB + 1;               // 1 KiB glds wave instructions per stage
  constexpr int L = (XI + NW - 1) / NW;
  constexpr int STAGE = XI * 1024;
  constexpr int BAND = BF * 1024, WOFF = (BF + XB) * 1024;
  constexpr int ABUF = AF * 1024;
  constexpr int CS = BN * 2 + 16;
  constexpr int SMEM_PIPE = STAGES * STAGE + 2 * ABUF;
  constexpr int SMEM = SMEM_PIPE > BM * CS ? SMEM_PIPE : BM * CS;
  constexpr int U = 2 * AF;                     // depthwise units (16 pixels x 16 channels)
  constexpr int UPW = (U + NW - 1) / NW;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H;
  const int ntw = (W + TW - 1) / TW, nth = (H + TH - 1) / TH;
  const int nN = (a.NF * 16) / BN;
  const int nM = a.B * nth * ntw;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int n0 = ni * BN;
  const int bimg = mi / (nth * ntw), trem = mi - bimg * (nth * ntw);
  const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
  const int KT = a.K >> 5;

  // ---- per-lane glds sources (the k-step advance is 1 KiB for weights, 64 B for pixels)
  const uint8_t* src[L];
  int kind[L];                                  // 0 = B, 1 = x patch / zeros, 2 = dw weights
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int s = min(wave + i * NW, XI - 1);
    if (s < BF) {
      kind[i] = 0;
      src[i] = (const uint8_t*)(a.wp + ((long)(n0 / 16 + s) * KT) * 512 + lane * 8);
    } else if (s < BF + XB) {
      kind[i] = 1;
      const int q = (s - BF) / IPP, slot = ((s - BF) % IPP) * 64 + lane;
      const int pr = slot / P::PW, pc = slot - pr * P::PW;
      const int h = h0 - 1 + pr, w = w0 - 1 + pc;
      const bool in = slot < P::PS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      src[i] = in ? (const uint8_t*)(a.x + (((long)bimg * H + h) * W + w) * a.ldx + q * 8) : s2d_zeros;
    } else {
      kind[i] = 2;
      src[i] = (const uint8_t*)a.dwk + lane * 16;
    }
  }
  auto issue = [&](int t, int slot) {
    uint8_t* base = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int s = min(wave + i * NW, XI - 1);
      const long step = kind[i] == 1 ? 64 : 1024;
      glds16(src[i] + t * step, base + s * 1024);
    }
  };

  // ---- depthwise units: u = wave + NW*i -> fragment f = u >> 1 (16 tile pixels), channel
  // group g = u & 1 (one g per wave: NW is even)
  const int g = wave & 1;
  const int p16 = lane & 15, kb = lane >> 4;
  const int par = kb >> 1;                      // tap parity: taps par, par+2, .. par+8
  const int qc = 2 * g + (kb & 1);              // 8-channel chunk (patch plane) read
  const int ulast = U - 1 - ((U - 1 - wave) & 1);
  int toff[UPW][5];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = min(wave + NW * i, ulast);
    const int pix = (u >> 1) * 16 + p16;        // tile-local pixel
    const int r = pix / TW, c = pix - r * TW;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int tap = 2 * j + par;
      const int slot = tap < 9 ? (r + tap / 3) * P::PW + c + tap % 3 : P::ZSLOT;
      toff[i][j] = BAND + qc * PL + slot * 16;
    }
  }
  // block-diagonal B operand from a 16-byte weight entry (see the sepconv_ws.hip header)
  const bool wv = (p16 >> 3) == (kb & 1);
  const int e = p16 & 7;
  uint32_t sel[2][4];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t pair = (2u * jp) | ((2u * jp + 1u) << 8);
      const uint32_t val = (e & 1) ? (0x0c0cu | (pair << 16)) : (0x0c0c0000u | pair);
      sel[jp][d] = (wv && (e >> 1) == d) ? val : 0x0c0c0c0cu;
    }
  const int went = WOFF + ((g * 16 + p16) * 2 + par) * 16;
  const int aoffw = (p16 + 16 * (2 * g + (kb >> 1))) * 16 + 8 * (kb & 1);

  auto dw_load = [&](int slot, u32x4 (&xv)[UPW][5]) -> u32x4 {
    const uint8_t* sb = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < UPW; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) xv[i][j] = *(const u32x4*)(sb + toff[i][j]);
    return *(const u32x4*)(sb + went);
  };
  auto dw_mfma = [&](const u32x4 we, u32x4 (&xv)[UPW][5], int abuf) {
    s16x8 wf[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint32_t wd = we[j >> 1];
      u32x4 f;
#pragma unroll
      for (int d = 0; d < 4; ++d) f[d] = __builtin_amdgcn_perm(wd, wd, sel[j & 1][d]);
      wf[j] = __builtin_bit_cast(s16x8, f);
    }
    f32x4 dacc[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) dacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int i = 0; i < UPW; ++i) {
        u32x4 v = xv[i][j];
        if constexpr (RELU) {
#pragma unroll
          for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
        }
        dacc[i] = mfma16(wf[j], __builtin_bit_cast(s16x8, v), dacc[i]);
      }
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int u = min(wave + NW * i, ulast);
      *(u32x2*)(smem + STAGES * STAGE + abuf * ABUF + (u >> 1) * 1024 + aoffw) =
          (u32x2){pack_bf16(dacc[i][0], dacc[i][1]), pack_bf16(dacc[i][2], dacc[i][3])};
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // ---- prologue: stages 0 .. STAGES-2 in flight (clamped to the last k-step so every
  // stage is exactly L DMAs per wave); A(0) = dw(x(0))
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p) issue(min(p, KT - 1), p);
  s2_wait_barrier<(STAGES - 2) * L>();          // stage 0 landed
  {
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load(0, xv);
    dw_mfma(we, xv, 0);
  }

  for (int t = 0; t < KT; ++t) {
    // stage t+1 landed (STAGES-3 younger stages stay in flight); the A tile written by
    // the previous iteration's depthwise is visible after this barrier
    s2_wait_barrier<(STAGES - 3) * L>();
    const uint8_t* As = smem + STAGES * STAGE + (t & 1) * ABUF + lane * 16;
    const uint8_t* Bs = smem + (t % STAGES) * STAGE + lane * 16;
    s16x8 af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + (wm * FM + i) * 1024);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(Bs + (wn * FN + j) * 1024);
    // depthwise inputs of stage t+1 (on the last step a clamped stage whose result
    // goes to an A buffer nobody reads: keeps the loop branch-free)
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load((t + 1) % STAGES, xv);
    // refill the slot of stage t-1 (read by everyone before this barrier)
    issue(min(t + STAGES - 1, KT - 1), (t + STAGES - 1) % STAGES);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    dw_mfma(we, xv, (t + 1) & 1);
    __builtin_amdgcn_s_setprio(0);
  }
  s2_wait_barrier<0>();

  // ---- epilogue: bias (+ReLU) -> bf16 C tile in LDS -> residual / activation store pass
  const int quad = lane >> 4, col = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * FN * 16 + j * 16 + 4 * quad;
    const float4 bv = *(const float4*)(a.bias + n0 + nl);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int mll = wm * FM * 16 + i * 16 + col;
      float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y;
      float v2 = acc[i][j][2] + bv.z, v3 = acc[i][j][3] + bv.w;
      if (a.relu_out == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      *(u32x2*)(smem + mll * CS + nl * 2) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int c = tid; c < BM * CPR; c += NT) {
    const int r = c / CPR, cc = c - r * CPR;
    const int h = h0 + r / TW, w = w0 + r % TW;
    const int n = n0 + cc * 8;
    if (h < H && w < W && n < a.nstore)
      epi_store(a, (bimg * H + h) * W + w, n, *(const u32x4*)(smem + r * CS + cc * 16));
  }
}

// ---------------------------------------------------------------------------
// Persistent variant (ids S2DP_OFFSET..). PMC on the one-shot kernel above at
// 147x147x128 (profiles/sepconv_2d_pmc.txt): MFMA ~2 %, VALU ~5 %, LDS ~4 % busy,
// TA/TCP stalls small -- every workgroup spends its ~20k-cycle life waiting on its
// own short pipeline (KT = 4 k-steps: prologue latency, one stage in flight, C-tile
// epilogue) and only two fit per CU. Here one workgroup per CU walks many tiles:
//   * the pointwise weights of ALL k-steps and the depthwise weight entries are
//     staged once and stay LDS-resident (K x N <= 64 Ki elements);
//   * the LDS-DMA ring runs over the flattened (tile, k-step) sequence, so the next
//     tile's halo patches are in flight while this tile's epilogue runs;
//   * wave roles: waves [0, NW/2) issue every LDS-DMA, waves [NW/2, NW) do every
//     global store. On gfx9 vmcnt counts stores too, and loads and stores retire
//     out of order with respect to each other, so a store in a loader wave would
//     void the counted vmcnt(N) that keeps STAGES-2 patches in flight across the
//     barriers; with split roles the loaders' counters only ever hold DMAs.
// Tiles are dealt out XCD-contiguously (tile = xcd_remap(block) + i * grid): at any
// moment an XCD works on a contiguous band of tiles, so halo rows shared by
// vertically/horizontally adjacent tiles are L2 hits.
template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW, bool RELU>
__global__ __launch_bounds__(64 * WGM * WGN) void sepconv_2dp_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW, NL = NW / 2;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  static_assert(BM == TH * TW && TW % 16 == 0, "the M tile is TH x TW pixels, 16-pixel row segments");
  static_assert(NW % 2 == 0 && STAGES >= 3, "loader/storer halves; >= 1 patch in flight across barriers");
  static_assert(BN <= 256, "the bias is one 1 KiB DMA");
  using P = S2dPatch<TH, TW>;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int IPP = P::IPP, XB = P::XB;
  constexpr int PL = IPP * 1024;
  constexpr int LX = (XB + NL - 1) / NL;        // patch DMAs per loader wave per stage
  constexpr int STAGE = XB * 1024;
  constexpr int ABUF = AF * 1024;
  constexpr int CS = BN * 2 + 16;
  constexpr int U = 2 * AF;
  constexpr int UPW = (U + NW - 1) / NW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H;
  const int KT = a.K >> 5;
  const int ntw = (W + TW - 1) / TW, nth = (H + TH - 1) / TH;
  const int ntiles = a.B * nth * ntw;
  const int G = gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, G);
  const int TWn = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;   // tiles of this workgroup
  const int Q = TWn * KT;                                         // stages
  if (Q == 0) return;                           // uniform per workgroup; nothing issued yet
  // LDS map: [B resident KT*BF KiB][dw entries KT KiB][ring][A x2][C tile][bias 1 KiB]
  uint8_t* const bres = smem;
  uint8_t* const dres = smem + KT * BF * 1024;
  uint8_t* const ring = dres + KT * 1024;
  uint8_t* const abuf = ring + STAGES * STAGE;
  uint8_t* const ctile = abuf + 2 * ABUF;
  uint8_t* const bias = ctile + BM * CS;

  // ---- resident weights (all waves), then the ring prologue (loader waves)
  for (int idx = wave; idx < KT * BF; idx += NW) {
    const int k = idx / BF, f = idx - k * BF;
    glds16(a.wp + ((long)f * KT + k) * 512 + lane * 8, bres + idx * 1024);
  }
  for (int k = wave; k < KT; k += NW) glds16((const uint8_t*)a.dwk + k * 1024 + lane * 16, dres + k * 1024);
  // the bias rides the same DMA path into LDS: a global load of it in the tile epilogue made
  // the compiler put a vmcnt(0) there, which drained the loader waves' whole ring (every
  // in-flight patch) at every tile boundary
  if (wave == NW - 1) glds16((const uint8_t*)(a.bias + min(lane * 4, BN - 4)), bias + lane * 16);

  // loader lanes: patch slot geometry of each of this wave's LX instructions
  int pq[LX], prr[LX], pcc[LX], pis[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int sidx = min(wave + i * NL, XB - 1);
    const int q = sidx / IPP, slot = (sidx % IPP) * 64 + lane;
    pq[i] = q;
    prr[i] = slot / P::PW;
    pcc[i] = slot - prr[i] * P::PW;
    pis[i] = slot < P::PS;
  }
  // issue cursor: stages go out in (tile, k) order, one per call; past the last stage the
  // cursor stays put and re-issues it (keeps every wave's DMA count per stage fixed). The
  // patch sources of a tile are computed once, when the cursor enters it (the divisions
  // per call cost ~70 scalar instructions per k-step).
  int iq = 0, ik = 0, iti = 0;
  const uint8_t* psrc[LX];
  auto enter_tile = [&](int ti) {
    const int tile = t0 + ti * G;
    const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
    const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int h = h0 - 1 + prr[i], w = w0 - 1 + pcc[i];
      const bool in = pis[i] && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      psrc[i] = in ? (const uint8_t*)(a.x + (((long)bimg * H + h) * W + w) * a.ldx + pq[i] * 8) : s2d_zeros;
    }
  };
  auto issue = [&](int slotbuf) {             // the cursor's stage into ring slot slotbuf
    uint8_t* base = ring + slotbuf * STAGE;
#pragma unroll
    for (int i = 0; i < LX; ++i) glds16(psrc[i] + ik * 64, base + min(wave + i * NL, XB - 1) * 1024);
    if (iq + 1 < Q) {
      ++iq;
      if (++ik == KT) {
        ik = 0;
        enter_tile(++iti);
      }
    }
  };
  const bool loader = wave < NL;
  if (loader) {
    enter_tile(0);
    for (int p = 0; p < STAGES - 1; ++p) issue(p);
  }

  // ---- depthwise units (as in sepconv_2d_kernel)
  const int g = wave & 1;
  const int p16 = lane & 15, kb = lane >> 4;
  const int par = kb >> 1;
  const int qc = 2 * g + (kb & 1);
  const int ulast = U - 1 - ((U - 1 - wave) & 1);
  int toff[UPW][5];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = min(wave + NW * i, ulast);
    const int pix = (u >> 1) * 16 + p16;
    const int r = pix / TW, c = pix - r * TW;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int tap = 2 * j + par;
      const int slot = tap < 9 ? (r + tap / 3) * P::PW + c + tap % 3 : P::ZSLOT;
      toff[i][j] = qc * PL + slot * 16;
    }
  }
  const bool wv = (p16 >> 3) == (kb & 1);
  const int e = p16 & 7;
  uint32_t sel[2][4];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t pair = (2u * jp) | ((2u * jp + 1u) << 8);
      const uint32_t val = (e & 1) ? (0x0c0cu | (pair << 16)) : (0x0c0c0000u | pair);
      sel[jp][d] = (wv && (e >> 1) == d) ? val : 0x0c0c0c0cu;
    }
  const int went = ((g * 16 + p16) * 2 + par) * 16;
  const int aoffw = (p16 + 16 * (2 * g + (kb >> 1))) * 16 + 8 * (kb & 1);

  auto dw_load = [&](int slotbuf, int k, u32x4 (&xv)[UPW][5]) -> u32x4 {
    const uint8_t* sb = ring + slotbuf * STAGE;
#pragma unroll
    for (int i = 0; i < UPW; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) xv[i][j] = *(const u32x4*)(sb + toff[i][j]);
    return *(const u32x4*)(dres + k * 1024 + went);
  };
  auto dw_mfma = [&](const u32x4 we, u32x4 (&xv)[UPW][5], int ab) {
    s16x8 wf[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint32_t wd = we[j >> 1];
      u32x4 f;
#pragma unroll
      for (int d = 0; d < 4; ++d) f[d] = __builtin_amdgcn_perm(wd, wd, sel[j & 1][d]);
      wf[j] = __builtin_bit_cast(s16x8, f);
    }
    f32x4 dacc[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) dacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int i = 0; i < UPW; ++i) {
        u32x4 v = xv[i][j];
        if constexpr (RELU) {
#pragma unroll
          for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
        }
        dacc[i] = mfma16(wf[j], __builtin_bit_cast(s16x8, v), dacc[i]);
      }
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int u = min(wave + NW * i, ulast);
      *(u32x2*)(abuf + ab * ABUF + (u >> 1) * 1024 + aoffw) =
          (u32x2){pack_bf16(dacc[i][0], dacc[i][1]), pack_bf16(dacc[i][2], dacc[i][3])};
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // resident weights + stage 0 landed (loads retire in order: the resident DMAs are older)
  if (loader) s2_wait_barrier<(STAGES - 2) * LX>();
  else s2_wait_barrier<0>();
  {
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load(0, 0, xv);
    dw_mfma(we, xv, 0);
  }

  const int quad = lane >> 4, col = lane & 15;
  // bias of this wave's output columns, read once (an LDS read in the tile epilogue got a
  // conservative vmcnt(0) from the compiler: pending LDS-DMAs may alias it)
  float4 bvr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bvr[j] = *(const float4*)(bias + (wn * FN * 16 + j * 16 + 4 * quad) * 4);
  int k = 0, ti = 0;
  for (int q = 0; q < Q; ++q) {
    // stage q+1 landed; STAGES-3 younger patches stay in flight (loaders' counters hold
    // only DMAs); storers hold only stores and may retire them lazily
    if (loader) s2_wait_barrier<(STAGES - 3) * LX>();
    else s2_wait_barrier<63>();
    if (loader) issue((q + STAGES - 1) % STAGES);
    const uint8_t* As = abuf + (q & 1) * ABUF + lane * 16;
    const uint8_t* Bs = bres + k * BF * 1024 + lane * 16;
    s16x8 af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + (wm * FM + i) * 1024);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(Bs + (wn * FN + j) * 1024);
    const int k1 = k + 1 == KT ? 0 : k + 1;
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load((q + 1) % STAGES, k1, xv);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    dw_mfma(we, xv, (q + 1) & 1);
    __builtin_amdgcn_s_setprio(0);
    if (k1 == 0) {
      // ---- tile epilogue: bias (+ReLU) -> bf16 C tile -> storer waves (+residual) -> HBM
      const int tile = t0 + ti * G;
      const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
      const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = wn * FN * 16 + j * 16 + 4 * quad;
        const float4 bv = bvr[j];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int mll = wm * FM * 16 + i * 16 + col;
          float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y;
          float v2 = acc[i][j][2] + bv.z, v3 = acc[i][j][3] + bv.w;
          if (a.relu_out == 1) {
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
          }
          *(u32x2*)(ctile + mll * CS + nl * 2) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
          acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
      s2_wait_barrier<63>();                    // C tile complete (lgkmcnt(0) + barrier, no vmcnt drain)
      if (!loader) {
        constexpr int CPR = BN / 8;
        for (int c = tid - NL * 64; c < BM * CPR; c += NT - NL * 64) {
          const int r = c / CPR, cc = c - r * CPR;
          const int h = h0 + r / TW, w = w0 + r % TW;
          const int n = cc * 8;
          if (h < H && w < W && n < a.nstore)
            epi_store(a, (bimg * H + h) * W + w, n, *(const u32x4*)(ctile + r * CS + cc * 16));
        }
      }
      ++ti;
    }
    k = k1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// Persistent variant with ONE dedicated DMA wave (wave NW) and NW compute waves that
// store their own accumulators (ids S2DW_OFFSET..; same pattern as conv3x3_2dw_kernel,
// which took block1_conv2 from 54.5 to 40.4 us). Versus sepconv_2dp_kernel: no C tile in
// LDS, no storer pass between the epilogue barrier and the next tile, one barrier per
// k-step, and the compute waves' vmcnt only ever holds their own stores (never waited
// for in the loop) while the DMA wave's counted wait stays exact. No padded output or
// transcendental epilogue (the launcher refuses them); a residual is read per lane (8 B).
template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW, bool RELU>
__global__ __launch_bounds__(64 * (WGM * WGN + 1)) void sepconv_2dw_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  static_assert(BM == TH * TW && TW % 16 == 0, "the M tile is TH x TW pixels, 16-pixel row segments");
  static_assert(NW % 2 == 0 && STAGES >= 3, "a wave's depthwise units share one channel group; ring depth");
  using P = S2dPatch<TH, TW>;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int IPP = P::IPP, XB = P::XB;
  constexpr int PL = IPP * 1024;
  constexpr int STAGE = XB * 1024;
  constexpr int ABUF = AF * 1024;
  constexpr int U = 2 * AF;
  constexpr int UPW = (U + NW - 1) / NW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dma = wave == NW;
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H;
  const int KT = a.K >> 5;
  const int ntw = (W + TW - 1) / TW, nth = (H + TH - 1) / TH;
  const int ntiles = a.B * nth * ntw;
  const int G = gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, G);
  const int TWn = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;
  const int Q = TWn * KT;
  if (Q == 0) return;
  // LDS map: [B resident KT*BF KiB][dw entries KT KiB][ring][A x2]
  uint8_t* const bres = smem;
  uint8_t* const dres = smem + KT * BF * 1024;
  uint8_t* const ring = dres + KT * 1024;
  uint8_t* const abuf = ring + STAGES * STAGE;

  // resident weights: every wave helps (older than every ring DMA of the DMA wave)
  for (int idx = wave; idx < KT * BF; idx += NW + 1) {
    const int k = idx / BF, f = idx - k * BF;
    glds16(a.wp + ((long)f * KT + k) * 512 + lane * 8, bres + idx * 1024);
  }
  for (int k = wave; k < KT; k += NW + 1) glds16((const uint8_t*)a.dwk + k * 1024 + lane * 16, dres + k * 1024);

  if (dma) {
    // ---- the DMA wave: XB patch instructions per stage, stages in (tile, k) order
    int iq = 0, ik = 0, iti = 0;
    const uint8_t* psrc[XB];
    auto enter_tile = [&](int ti) {
      const int tile = t0 + ti * G;
      const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
      const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
#pragma unroll
      for (int sidx = 0; sidx < XB; ++sidx) {
        const int q = sidx / IPP, slot = (sidx % IPP) * 64 + lane;
        const int pr = slot / P::PW, pc = slot - pr * P::PW;
        const int h = h0 - 1 + pr, w = w0 - 1 + pc;
        const bool in = slot < P::PS && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        psrc[sidx] = in ? (const uint8_t*)(a.x + (((long)bimg * H + h) * W + w) * a.ldx + q * 8) : s2d_zeros;
      }
    };
    auto issue = [&](int slotbuf) {
      uint8_t* base = ring + slotbuf * STAGE;
#pragma unroll
      for (int sidx = 0; sidx < XB; ++sidx) glds16(psrc[sidx] + ik * 64, base + sidx * 1024);
      if (iq + 1 < Q) {
        ++iq;
        if (++ik == KT) {
          ik = 0;
          enter_tile(++iti);
        }
      }
    };
    enter_tile(0);
    for (int p = 0; p < STAGES - 1; ++p) issue(p);
    s2_wait_barrier<(STAGES - 2) * XB>();       // resident weights + stage 0 landed
    for (int q = 0; q < Q; ++q) {
      s2_wait_barrier<(STAGES - 3) * XB>();     // stage q+1 landed
      issue((q + STAGES - 1) % STAGES);         // slot of stage q-1 (read by the dw of step q-2)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---- compute waves: depthwise units as in sepconv_2d_kernel, pointwise MFMAs, stores
  const int g = wave & 1;
  const int p16 = lane & 15, kb = lane >> 4;
  const int par = kb >> 1;
  const int qc = 2 * g + (kb & 1);
  const int ulast = U - 1 - ((U - 1 - wave) & 1);
  int toff[UPW][5];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = min(wave + NW * i, ulast);
    const int pix = (u >> 1) * 16 + p16;
    const int r = pix / TW, c = pix - r * TW;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int tap = 2 * j + par;
      const int slot = tap < 9 ? (r + tap / 3) * P::PW + c + tap % 3 : P::ZSLOT;
      toff[i][j] = qc * PL + slot * 16;
    }
  }
  const bool wv = (p16 >> 3) == (kb & 1);
  const int e = p16 & 7;
  uint32_t sel[2][4];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t pair = (2u * jp) | ((2u * jp + 1u) << 8);
      const uint32_t val = (e & 1) ? (0x0c0cu | (pair << 16)) : (0x0c0c0000u | pair);
      sel[jp][d] = (wv && (e >> 1) == d) ? val : 0x0c0c0c0cu;
    }
  const int went = ((g * 16 + p16) * 2 + par) * 16;
  const int aoffw = (p16 + 16 * (2 * g + (kb >> 1))) * 16 + 8 * (kb & 1);
  const int quad = lane >> 4, col = lane & 15;
  float4 bvr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bvr[j] = *(const float4*)(a.bias + wn * FN * 16 + j * 16 + 4 * quad);
  int prow[FM], pcol[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int op = (wm * FM + i) * 16 + col;
    prow[i] = op / TW;
    pcol[i] = op - prow[i] * TW;
  }

  auto dw_load = [&](int slotbuf, int k, u32x4 (&xv)[UPW][5]) -> u32x4 {
    const uint8_t* sb = ring + slotbuf * STAGE;
#pragma unroll
    for (int i = 0; i < UPW; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) xv[i][j] = *(const u32x4*)(sb + toff[i][j]);
    return *(const u32x4*)(dres + k * 1024 + went);
  };
  auto dw_mfma = [&](const u32x4 we, u32x4 (&xv)[UPW][5], int ab) {
    s16x8 wf[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint32_t wd = we[j >> 1];
      u32x4 f;
#pragma unroll
      for (int d = 0; d < 4; ++d) f[d] = __builtin_amdgcn_perm(wd, wd, sel[j & 1][d]);
      wf[j] = __builtin_bit_cast(s16x8, f);
    }
    f32x4 dacc[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) dacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int i = 0; i < UPW; ++i) {
        u32x4 v = xv[i][j];
        if constexpr (RELU) {
#pragma unroll
          for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
        }
        dacc[i] = mfma16(wf[j], __builtin_bit_cast(s16x8, v), dacc[i]);
      }
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      const int u = min(wave + NW * i, ulast);
      *(u32x2*)(abuf + ab * ABUF + (u >> 1) * 1024 + aoffw) =
          (u32x2){pack_bf16(dacc[i][0], dacc[i][1]), pack_bf16(dacc[i][2], dacc[i][3])};
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  s2_wait_barrier<0>();                         // own weight DMAs + bias loads; DMA wave: stage 0
  {
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load(0, 0, xv);
    dw_mfma(we, xv, 0);
  }
  int k = 0, ti = 0;
  for (int q = 0; q < Q; ++q) {
    s2_wait_barrier<63>();                      // A(q) written, stage q+1 landed
    const uint8_t* As = abuf + (q & 1) * ABUF + lane * 16;
    const uint8_t* Bs = bres + k * BF * 1024 + lane * 16;
    s16x8 af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + (wm * FM + i) * 1024);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(Bs + (wn * FN + j) * 1024);
    const int k1 = k + 1 == KT ? 0 : k + 1;
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load((q + 1) % STAGES, k1, xv);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    dw_mfma(we, xv, (q + 1) & 1);
    __builtin_amdgcn_s_setprio(0);
    if (k1 == 0) {
      // ---- tile epilogue straight from the accumulators (8-byte stores per lane)
      const int tile = t0 + ti * G;
      const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
      const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int h = h0 + prow[i], w = w0 + pcol[i];
        const bool ok = h < H && w < W;
        uint16_t* yrow = a.y + ((long)(bimg * H + h) * W + w) * a.ldy;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = wn * FN * 16 + j * 16 + 4 * quad;
          float v0 = acc[i][j][0] + bvr[j].x, v1 = acc[i][j][1] + bvr[j].y;
          float v2 = acc[i][j][2] + bvr[j].z, v3 = acc[i][j][3] + bvr[j].w;
          if (a.relu_out == 1) {
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
          }
          u32x2 o = {pack_bf16(v0, v1), pack_bf16(v2, v3)};
          if (a.res && ok) {                    // residual (bf16-rounded output + residual, as epi_store)
            const u32x2 rv = *(const u32x2*)(a.res + ((long)(bimg * H + h) * W + w) * a.ldr + n);
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              o[d] = pack_bf16(bf_lo(o[d]) + bf_lo(rv[d]), bf_hi(o[d]) + bf_hi(rv[d]));
              if (a.relu_out == 2) o[d] = relu_bf16x2(o[d]);
            }
          }
          if (ok && n < a.nstore) *(u32x2*)(yrow + n) = o;
          acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
      ++ti;
    }
    k = k1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// (FM, FN, WGM, WGN, STAGES, TH, TW) of the persistent variant; ids S2D_CFG_BASE + S2DP_OFFSET + i.
constexpr int S2DP_OFFSET = 24;
#define KDL_S2DP_CONFIGS(X)     \
  X(0, 3, 2, 2, 4, 4, 6, 16)    \
  X(1, 2, 2, 2, 4, 4, 4, 16)    \
  X(2, 2, 4, 2, 4, 3, 4, 16)    \
  X(3, 4, 2, 2, 4, 4, 8, 16)    \
  X(4, 3, 2, 2, 4, 6, 6, 16)    \
  X(5, 2, 4, 2, 4, 4, 4, 16)    \
  X(6, 2, 2, 2, 4, 8, 4, 16)    \
  X(7, 2, 2, 2, 4, 11, 4, 16)   \
  X(8, 3, 2, 2, 4, 7, 6, 16)

// (FM, FN, WGM, WGN, STAGES, TH, TW) of the DMA-wave variant; ids S2D_CFG_BASE + S2DW_OFFSET + i
// (host ids 200..204; 205..207 retired: the round-3 pooled variant; C3_CFG_BASE = 208 follows).
constexpr int S2DW_OFFSET = 40;
#define KDL_S2DW_CONFIGS(X)     \
  X(0, 2, 2, 2, 4, 4, 4, 16)    \
  X(1, 4, 2, 2, 4, 4, 8, 16)    \
  X(2, 3, 2, 2, 4, 4, 6, 16)    \
  X(3, 2, 4, 2, 4, 4, 4, 16)    \
  X(4, 4, 2, 2, 4, 6, 8, 16)

static int s2dp_num_cus();

template <int FM, int FN, int WGM, int WGN, int ST, int TH, int TW>
static hipError_t launch_s2dw(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN, NT = 64 * (WGM * WGN + 1);
  using P = S2dPatch<TH, TW>;
  if (a.NF * 16 != BN || a.opad || a.relu_out > 2 || a.dt) return hipErrorInvalidValue;
  const int KT = a.K / 32;
  const size_t smem = (size_t)KT * (BN / 16) * 1024 + (size_t)KT * 1024 + (size_t)ST * P::XB * 1024 + 2 * (BM / 16) * 1024;
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const int ntiles = a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  auto kern = a.relu_in ? sepconv_2dw_kernel<FM, FN, WGM, WGN, ST, TH, TW, true>
                        : sepconv_2dw_kernel<FM, FN, WGM, WGN, ST, TH, TW, false>;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NT, smem) != hipSuccess || per_cu <= 0) per_cu = 1;
  const int grid = std::min(ntiles, s2dp_num_cus() * per_cu);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), smem, s, a);
  return hipGetLastError();
}

template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW>
static size_t s2dp_smem(int K) {
  using P = S2dPatch<TH, TW>;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  const int KT = K / 32;
  return (size_t)KT * (BN / 16) * 1024 + (size_t)KT * 1024 + (size_t)STAGES * P::XB * 1024 + 2 * (BM / 16) * 1024 +
         (size_t)BM * (BN * 2 + 16) + 1024;
}

static int s2dp_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int FM, int FN, int WGM, int WGN, int ST, int TH, int TW>
static hipError_t launch_s2dp(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BN = 16 * FN * WGN;
  if (a.NF * 16 != BN) return hipErrorInvalidValue;      // one N tile: the resident weights are all of N
  const size_t smem = s2dp_smem<FM, FN, WGM, WGN, ST, TH, TW>(a.K);
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const int ntiles = a.B * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  const int per_cu = (int)((160 * 1024) / smem);
  const int grid = std::min(ntiles, s2dp_num_cus() * per_cu);
  if (a.relu_in)
    hipLaunchKernelGGL((sepconv_2dp_kernel<FM, FN, WGM, WGN, ST, TH, TW, true>), dim3(grid), dim3(64 * WGM * WGN), smem, s, a);
  else
    hipLaunchKernelGGL((sepconv_2dp_kernel<FM, FN, WGM, WGN, ST, TH, TW, false>), dim3(grid), dim3(64 * WGM * WGN), smem, s, a);
  return hipGetLastError();
}

// (FM, FN, WGM, WGN, STAGES, TH, TW); ids offset by S2D_CFG_BASE.
#define KDL_S2D_CONFIGS(X)           \
  X(0, 3, 2, 2, 4, 3, 6, 16)         \
  X(1, 4, 2, 2, 4, 3, 8, 16)         \
  X(2, 2, 2, 2, 4, 3, 4, 16)         \
  X(3, 3, 4, 2, 4, 3, 6, 16)         \
  X(4, 4, 4, 2, 4, 3, 8, 16)         \
  X(5, 4, 2, 2, 4, 3, 4, 32)         \
  X(6, 2, 4, 2, 4, 3, 4, 16)         \
  X(7, 3, 2, 2, 4, 4, 6, 16)         \
  X(8, 4, 1, 2, 4, 3, 8, 16)         \
  X(9, 2, 1, 4, 2, 3, 8, 16)         \
  X(10, 3, 2, 2, 4, 5, 6, 16)        \
  X(11, 2, 2, 2, 4, 5, 4, 16)        \
  X(12, 2, 2, 2, 4, 4, 4, 16)        \
  X(13, 3, 4, 2, 4, 4, 6, 16)

int sepconv_2d_config(int cfg, int* bm, int* bn, int* threads) {
  if (cfg >= S2DW_OFFSET) {
    switch (cfg - S2DW_OFFSET) {
#define KDL_S2WINFO(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * (wgm * wgn + 1); return 0;
      KDL_S2DW_CONFIGS(KDL_S2WINFO)
#undef KDL_S2WINFO
      default: return -1;
    }
  }
  if (cfg >= S2DP_OFFSET) {
    switch (cfg - S2DP_OFFSET) {
#define KDL_S2PINFO(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
      KDL_S2DP_CONFIGS(KDL_S2PINFO)
#undef KDL_S2PINFO
      default: return -1;
    }
  }
  switch (cfg) {
#define KDL_S2INFO(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_S2D_CONFIGS(KDL_S2INFO)
#undef KDL_S2INFO
    default: return -1;
  }
}

hipError_t sepconv_2d(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  int bm, bn, th;
  if (sepconv_2d_config(cfg, &bm, &bn, &th) != 0 || a.K % 32 != 0 || a.K > 8192 || (a.NF * 16) % bn != 0 ||
      a.OH != a.H || a.OW != a.W || a.M != a.B * a.H * a.W || a.M <= 0 || a.dwk == nullptr)
    return hipErrorInvalidValue;
  if (cfg >= S2DW_OFFSET) {
    switch (cfg - S2DW_OFFSET) {
#define KDL_S2WCASE(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: return launch_s2dw<fm, fn, wgm, wgn, st, th, tw>(a, s);
      KDL_S2DW_CONFIGS(KDL_S2WCASE)
#undef KDL_S2WCASE
      default: return hipErrorInvalidValue;
    }
  }
  if (cfg >= S2DP_OFFSET) {
    switch (cfg - S2DP_OFFSET) {
#define KDL_S2PCASE(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: return launch_s2dp<fm, fn, wgm, wgn, st, th, tw>(a, s);
      KDL_S2DP_CONFIGS(KDL_S2PCASE)
#undef KDL_S2PCASE
      default: return hipErrorInvalidValue;
    }
  }
  switch (cfg) {
#define KDL_S2CASE(id, fm, fn, wgm, wgn, st, th_, tw)                                                        \
  case id: {                                                                                               \
    const int grid = a.B * ((a.H + th_ - 1) / th_) * ((a.W + tw - 1) / tw) * ((a.NF * 16) / bn);           \
    if (a.relu_in) hipLaunchKernelGGL((sepconv_2d_kernel<fm, fn, wgm, wgn, st, th_, tw, true>), dim3(grid),  \
                                      dim3(th), 0, s, a);                                                  \
    else hipLaunchKernelGGL((sepconv_2d_kernel<fm, fn, wgm, wgn, st, th_, tw, false>), dim3(grid), dim3(th), \
                            0, s, a);                                                                      \
    break;                                                                                                 \
  }
    KDL_S2D_CONFIGS(KDL_S2CASE)
#undef KDL_S2CASE
  }
  return hipGetLastError();
}

}  // namespace kdl
