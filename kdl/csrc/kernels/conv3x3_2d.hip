// 3x3 'valid' stride-1 conv (+BN)(+ReLU) over 2-D spatial tiles with an LDS-staged halo
// patch, for Xception's block1_conv2 (149x149x32 -> 147x147x64).
//
// The implicit GEMM of conv_gemm.hip (MODE_CONV) gathers every A fragment from global
// memory once per tap: each input pixel is fetched 9 times through L1/L2 (~600 MB per
// layer at batch 32 for 133 MB of real traffic) and the kernel runs at ~440 TF/s.
// Here a workgroup stages the (TH+2) x (TW+2) input patch of a TH x TW output tile ONCE
// (LDS-DMA, 4 planes of 8 channels, the sepconv_2d.hip patch layout) and reads each tap's
// A fragment out of it with a slot offset; a 16-pixel fragment is one tile-row segment,
// so its 16 lanes read 256 contiguous bytes: conflict-free.
//
// cin = 32 (one channel chunk): all 9 taps' pointwise weights of a wave's FN output
// fragments (9 x FN x 1 KiB) live in REGISTERS for the whole kernel, so the only LDS
// traffic in the loop is the A reads. Persistent over tiles like sepconv_2dp_kernel:
// loader waves [0, NW/2) issue the patch ring, storer waves [NW/2, NW) do the global
// stores (gfx9 vmcnt counts stores too; split roles keep the loaders' counted waits exact).
#include "common.h"
#include "launch.h"
#include "epilogue.h"

#include <algorithm>

namespace kdl {

__device__ __attribute__((aligned(16))) uint8_t c3_zeros[1024];

template <int N>
__device__ __forceinline__ void c3_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW>
__global__ __launch_bounds__(64 * WGM * WGN) void conv3x3_2d_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW, NL = NW / 2;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  static_assert(BM == TH * TW && TW % 16 == 0, "the M tile is TH x TW pixels, 16-pixel row segments");
  static_assert(NW % 2 == 0 && STAGES >= 3 && BN <= 256, "loader/storer halves; ring depth; bias DMA");
  constexpr int PW = TW + 2, PS = (TH + 2) * PW;
  constexpr int IPP = (PS + 63) / 64;           // glds instructions per plane
  constexpr int XB = 4 * IPP;                   // KiB per patch (4 planes of 8 channels)
  constexpr int PL = IPP * 1024;
  constexpr int LX = (XB + NL - 1) / NL;        // patch DMAs per loader wave
  constexpr int STAGE = XB * 1024;
  constexpr int CS = BN * 2 + 16;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* const ring = smem;
  uint8_t* const ctile = ring + STAGES * STAGE;
  uint8_t* const bias = ctile + BM * CS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H, OH = a.OH, OW = a.OW;
  const int ntw = (OW + TW - 1) / TW, nth = (OH + TH - 1) / TH;
  const int ntiles = a.B * nth * ntw;
  const int G = gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, G);
  const int Q = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;   // tiles (= stages) of this workgroup
  if (Q == 0) return;                           // uniform per workgroup; nothing issued yet
  const bool loader = wave < NL;

  // ---- weights: the 9 taps x FN fragments of this wave's output columns, in registers
  s16x8 bw[9][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bw[t][j] = *(const s16x8*)(a.wp + (((long)(wn * FN + j) * 9 + t) * 64 + lane) * 8);
  if (wave == NW - 1) glds16((const uint8_t*)(a.bias + min(lane * 4, BN - 4)), bias + lane * 16);

  // ---- patch ring: loader lane geometry of each of this wave's LX instructions
  int pq[LX], prr[LX], pcc[LX], pis[LX];
#pragma unroll
  for (int i = 0; i < LX; ++i) {
    const int sidx = min(wave + i * NL, XB - 1);
    const int q = sidx / IPP, slot = (sidx % IPP) * 64 + lane;
    pq[i] = q;
    prr[i] = slot / PW;
    pcc[i] = slot - prr[i] * PW;
    pis[i] = slot < PS;
  }
  int iq = 0;                                   // issue cursor (tile index of this workgroup)
  auto issue = [&](int slotbuf) {
    const int tile = t0 + iq * G;
    const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
    const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
    uint8_t* base = ring + slotbuf * STAGE;
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int sidx = min(wave + i * NL, XB - 1);
      const int h = h0 + prr[i], w = w0 + pcc[i];
      const bool in = pis[i] && h < H && w < W;   // 'valid': patch rows/cols start at the tile origin
      const uint8_t* src = in ? (const uint8_t*)(a.x + (((long)bimg * H + h) * W + w) * a.ldx + pq[i] * 8) : c3_zeros;
      glds16(src, base + sidx * 1024);
    }
    if (iq + 1 < Q) ++iq;                       // past the end: re-issue the last tile
  };
  if (loader)
    for (int p = 0; p < STAGES - 1; ++p) issue(p);

  // A fragment slots: fragment f of this wave = tile row segment; lane -> pixel p16, plane kb
  const int p16 = lane & 15, kb = lane >> 4;
  int aoff[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pix = (wm * FM + i) * 16 + p16;
    const int r = pix / TW, c = pix - r * TW;
    aoff[i] = kb * PL + (r * PW + c) * 16;
  }

  // weights, bias, stage 0 landed (the weight loads are older than every DMA)
  if (loader) c3_wait_barrier<(STAGES - 2) * LX>();
  else c3_wait_barrier<0>();
  const int quad = lane >> 4, col = lane & 15;
  float4 bvr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bvr[j] = *(const float4*)(bias + (wn * FN * 16 + j * 16 + 4 * quad) * 4);

  for (int q = 0; q < Q; ++q) {
    if (q > 0) {
      if (loader) c3_wait_barrier<(STAGES - 2) * LX>();
      else c3_wait_barrier<63>();
    }
    if (loader) issue((q + STAGES - 1) % STAGES);
    const uint8_t* pb = ring + (q % STAGES) * STAGE;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = ((t / 3) * PW + t % 3) * 16;
      s16x8 af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(pb + aoff[i] + toff);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bw[t][j], af[i], acc[i][j]);
    }
    // ---- tile epilogue: bias (+ReLU) -> bf16 C tile -> storer waves -> HBM
    const int tile = t0 + q * G;
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
      }
    }
    // C tile complete; every wave is also done reading this stage's patch
    c3_wait_barrier<63>();
    if (!loader) {
      constexpr int CPR = BN / 8;
      for (int c = tid - NL * 64; c < BM * CPR; c += NT - NL * 64) {
        const int r = c / CPR, cc = c - r * CPR;
        const int h = h0 + r / TW, w = w0 + r % TW;
        const int n = cc * 8;
        if (h < OH && w < OW && n < a.nstore)
          epi_store(a, (bimg * OH + h) * OW + w, n, *(const u32x4*)(ctile + r * CS + cc * 16));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Variant with ONE dedicated DMA wave (wave NW) and NW compute waves that store their
// results straight from the accumulators (no C tile in LDS, no storer role): the compute
// waves' vmcnt then only ever holds their own stores, which nobody waits for inside the
// loop, and the DMA wave's counted wait stays exact. One barrier per tile (stage q landed
// + everybody done with stage q-1, whose slot the DMA wave refills right after it).
// PMC on the first variant (profiles/entry_flow_r2.txt): nothing saturated, ~3 TB/s --
// the storer waves' store pass sat between the epilogue barrier and the next tile.
template <int FM, int FN, int WGM, int WGN, int STAGES, int TH, int TW>
__global__ __launch_bounds__(64 * (WGM * WGN + 1)) void conv3x3_2dw_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  static_assert(BM == TH * TW && TW % 16 == 0, "the M tile is TH x TW pixels, 16-pixel row segments");
  static_assert(STAGES >= 3, "ring depth");
  constexpr int PW = TW + 2, PS = (TH + 2) * PW;
  constexpr int IPP = (PS + 63) / 64;
  constexpr int XB = 4 * IPP;                   // KiB per patch = DMA instructions per stage
  constexpr int PL = IPP * 1024;
  constexpr int STAGE = XB * 1024;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* const ring = smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool dma = wave == NW;
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H, OH = a.OH, OW = a.OW;
  const int ntw = (OW + TW - 1) / TW, nth = (OH + TH - 1) / TH;
  const int ntiles = a.B * nth * ntw;
  const int G = gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, G);
  const int Q = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;
  if (Q == 0) return;

  if (dma) {
    // ---- the DMA wave: patch geometry of its XB instructions (plane sidx / IPP, 64 slots each)
    int iq = 0;
    auto issue = [&](int slotbuf) {
      const int tile = t0 + iq * G;
      const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
      const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
      uint8_t* base = ring + slotbuf * STAGE;
#pragma unroll
      for (int sidx = 0; sidx < XB; ++sidx) {
        const int q = sidx / IPP, slot = (sidx % IPP) * 64 + lane;
        const int pr = slot / PW, pc = slot - pr * PW;
        const int h = h0 + pr, w = w0 + pc;
        const bool in = slot < PS && h < H && w < W;
        const uint8_t* src = in ? (const uint8_t*)(a.x + (((long)bimg * H + h) * W + w) * a.ldx + q * 8) : c3_zeros;
        glds16(src, base + sidx * 1024);
      }
      if (iq + 1 < Q) ++iq;
    };
    for (int p = 0; p < STAGES - 1; ++p) issue(p);
    for (int q = 0; q < Q; ++q) {
      c3_wait_barrier<(STAGES - 2) * XB>();     // stage q landed; publish it
      issue((q + STAGES - 1) % STAGES);         // refill the slot of stage q-1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---- compute waves: the 9 taps x FN weight fragments of this wave's columns, in registers
  s16x8 bw[9][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bw[t][j] = *(const s16x8*)(a.wp + (((long)(wn * FN + j) * 9 + t) * 64 + lane) * 8);
  const int p16 = lane & 15, kb = lane >> 4;
  const int quad = lane >> 4, col = lane & 15;
  float4 bvr[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) bvr[j] = *(const float4*)(a.bias + wn * FN * 16 + j * 16 + 4 * quad);
  int aoff[FM], prow[FM], pcol[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pix = (wm * FM + i) * 16 + p16;
    const int r = pix / TW, c = pix - r * TW;
    aoff[i] = kb * PL + (r * PW + c) * 16;
    const int op = (wm * FM + i) * 16 + col;    // output pixel of this lane's accumulator rows
    prow[i] = op / TW;
    pcol[i] = op - prow[i] * TW;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // weights + bias in registers

  for (int q = 0; q < Q; ++q) {
    c3_wait_barrier<63>();                      // stage q published by the DMA wave
    const uint8_t* pb = ring + (q % STAGES) * STAGE;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = ((t / 3) * PW + t % 3) * 16;
      s16x8 af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(pb + aoff[i] + toff);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bw[t][j], af[i], acc[i][j]);
    }
    // ---- epilogue straight from the accumulators: lane holds 4 consecutive channels of
    // one output pixel per fragment (8-byte stores; the XCD L2 merges the row segments)
    const int tile = t0 + q * G;
    const int bimg = tile / (nth * ntw), trem = tile - bimg * (nth * ntw);
    const int h0 = (trem / ntw) * TH, w0 = (trem % ntw) * TW;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int h = h0 + prow[i], w = w0 + pcol[i];
      if (h < OH && w < OW) {
        uint16_t* yrow = a.y + ((long)(bimg * OH + h) * OW + w) * a.ldy;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = wn * FN * 16 + j * 16 + 4 * quad;
          float v0 = acc[i][j][0] + bvr[j].x, v1 = acc[i][j][1] + bvr[j].y;
          float v2 = acc[i][j][2] + bvr[j].z, v3 = acc[i][j][3] + bvr[j].w;
          if (a.relu_out == 1) {
            v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
          }
          if (n < a.nstore) *(u32x2*)(yrow + n) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// (FM, FN, WGM, WGN, STAGES, TH, TW); ids offset by C3_CFG_BASE.
// ids 4.. (KDL_C3W_CONFIGS): the dedicated-DMA-wave variant, 64 * (WGM * WGN + 1) threads.
#define KDL_C3_CONFIGS(X)          \
  X(0, 2, 2, 4, 2, 4, 8, 16)       \
  X(1, 1, 2, 4, 2, 4, 4, 16)       \
  X(2, 2, 2, 4, 2, 6, 8, 16)       \
  X(3, 3, 2, 4, 2, 4, 12, 16)
#define KDL_C3W_CONFIGS(X)         \
  X(4, 2, 2, 4, 2, 4, 8, 16)       \
  X(5, 1, 2, 4, 2, 4, 4, 16)       \
  X(6, 2, 2, 4, 2, 6, 8, 16)       \
  X(7, 2, 4, 4, 1, 4, 8, 16)

template <int FM, int FN, int WGM, int WGN, int ST, int TH, int TW>
static size_t c3_smem() {
  constexpr int PS = (TH + 2) * (TW + 2), IPP = (PS + 63) / 64;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  return (size_t)ST * 4 * IPP * 1024 + (size_t)BM * (BN * 2 + 16) + 1024;
}

static int c3_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int FM, int FN, int WGM, int WGN, int ST, int TH, int TW>
static hipError_t launch_c3(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BN = 16 * FN * WGN;
  // one N tile holding all outputs, 32 input channels (the register-resident weights),
  // 3x3 'valid' stride 1, no padded output layout
  if (a.NF * 16 != BN || a.K != 9 * 32 || a.cin != 32 || a.ldx < 32 || a.stride != 1 || a.opad ||
      a.OH != a.H - 2 || a.OW != a.W - 2 || a.M != a.B * a.OH * a.OW || a.M <= 0 || a.res || a.dt)
    return hipErrorInvalidValue;
  const size_t smem = c3_smem<FM, FN, WGM, WGN, ST, TH, TW>();
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const int ntiles = a.B * ((a.OH + TH - 1) / TH) * ((a.OW + TW - 1) / TW);
  // resident workgroups per CU from the occupancy API (registers, not only LDS, bound it):
  // the tiles are dealt out statically, so a workgroup that is not resident is pure tail
  static int per_cu = 0;
  if (per_cu == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv3x3_2d_kernel<FM, FN, WGM, WGN, ST, TH, TW>,
                                                     64 * WGM * WGN, smem) != hipSuccess || n <= 0)
      n = 1;
    per_cu = n;
  }
  const int grid = std::min(ntiles, c3_num_cus() * per_cu);
  hipLaunchKernelGGL((conv3x3_2d_kernel<FM, FN, WGM, WGN, ST, TH, TW>), dim3(grid), dim3(64 * WGM * WGN), smem, s, a);
  return hipGetLastError();
}

template <int FM, int FN, int WGM, int WGN, int ST, int TH, int TW>
static hipError_t launch_c3w(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BN = 16 * FN * WGN, NT = 64 * (WGM * WGN + 1);
  if (a.NF * 16 != BN || a.K != 9 * 32 || a.cin != 32 || a.ldx < 32 || a.stride != 1 || a.opad ||
      a.OH != a.H - 2 || a.OW != a.W - 2 || a.M != a.B * a.OH * a.OW || a.M <= 0 || a.res || a.dt ||
      a.relu_out > 1)
    return hipErrorInvalidValue;
  constexpr int PS = (TH + 2) * (TW + 2), IPP = (PS + 63) / 64;
  const size_t smem = (size_t)ST * 4 * IPP * 1024;
  const int ntiles = a.B * ((a.OH + TH - 1) / TH) * ((a.OW + TW - 1) / TW);
  static int per_cu = 0;
  if (per_cu == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv3x3_2dw_kernel<FM, FN, WGM, WGN, ST, TH, TW>, NT,
                                                     smem) != hipSuccess || n <= 0)
      n = 1;
    per_cu = n;
  }
  const int grid = std::min(ntiles, c3_num_cus() * per_cu);
  hipLaunchKernelGGL((conv3x3_2dw_kernel<FM, FN, WGM, WGN, ST, TH, TW>), dim3(grid), dim3(NT), smem, s, a);
  return hipGetLastError();
}

int conv3x3_2d_config(int cfg, int* bm, int* bn, int* threads) {
  switch (cfg) {
#define KDL_C3INFO(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_C3_CONFIGS(KDL_C3INFO)
#undef KDL_C3INFO
#define KDL_C3WINFO(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * (wgm * wgn + 1); return 0;
    KDL_C3W_CONFIGS(KDL_C3WINFO)
#undef KDL_C3WINFO
    default: return -1;
  }
}

hipError_t conv3x3_2d(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  switch (cfg) {
#define KDL_C3CASE(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: return launch_c3<fm, fn, wgm, wgn, st, th, tw>(a, s);
    KDL_C3_CONFIGS(KDL_C3CASE)
#undef KDL_C3CASE
#define KDL_C3WCASE(id, fm, fn, wgm, wgn, st, th, tw) \
  case id: return launch_c3w<fm, fn, wgm, wgn, st, th, tw>(a, s);
    KDL_C3W_CONFIGS(KDL_C3WCASE)
#undef KDL_C3WCASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace kdl
