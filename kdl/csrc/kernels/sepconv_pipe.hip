// Pipelined fused SeparableConv2D (+BN)(+ReLU in/out)(+residual) for CDNA4 with the
// depthwise 3x3 ON THE MATRIX CORES:
//   out[m][n] = sum_c dw3x3(relu?(x))[m][c] * W[n][c] + bias[n]
// SURVEY.md §2.5 K5+K6 / §7.4 hard parts 1-2: the depthwise never leaves the chip.
//
// Why MFMA for a depthwise: the VALU formulation (bf16 -> f32 converts, packed FMAs,
// ReLU, tap masks) costs ~220 VALU instructions per wave per 32-channel k-step and
// made the first version of this kernel VALU/LDS-bound at 1.3x the split path. Here
// a 16-pixel x 16-channel depthwise output fragment is a 16x16x144 GEMM against a
// block-diagonal weight operand (k = (tap, channel)), five v_mfma_f32_16x16x32_bf16:
//   A operand (pixels x k): lane l reads 16 bytes = 8 channels of ONE tap of its pixel
//     straight from the LDS x band (ds_read_b128, no conversion);
//   B operand (k x channels): one non-zero bf16 per lane, built with 4 v_perm_b32
//     from a 16-byte weight entry (5 taps of the lane's channel) staged per k-step.
// That is 42 % more MFMA work than the pointwise alone, on a pipe the split path
// leaves ~75 % idle, and it removes ~85 % of the VALU work.
//
// Staging (one barrier per 32-channel k-step, STAGES-deep LDS ring, all by LDS-DMA):
//   stage t = [ B fragments: pointwise weights BF KiB ]
//             [ x band: XB KiB, 4 planes (one per 8-channel chunk) of 16-byte pixel
//               slots; slots are consecutive raster pixels of rows rlo.., so a 16-lane
//               MFMA read of 16 neighbouring pixels is 256 contiguous bytes
//               (conflict-free); slots past the band load zeros, the last slot of a
//               plane is the target of every out-of-image tap ]
//             [ depthwise weight entries: 1 KiB ]
//   iteration t:  wait(stage t+1) + barrier ; issue stage t+STAGES-1 ;
//                 pointwise MFMAs on A[t&1] x B(t) ; depthwise MFMAs of stage t+1 ->
//                 bf16 -> A[(t+1)&1] (fragment-linear)
// The depthwise output is rounded to bf16 like the split path's dw3x3 output; the
// depthwise weights are bf16 here (fp32 in dw3x3.hip).
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

// zeros for band slots beyond the staged rows (read at +64 B per k-step: K <= 8192)
__device__ __attribute__((aligned(16))) uint8_t sepp_zeros[16384];

template <int N>
__device__ __forceinline__ void sp_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int FM, int FN, int WGM, int WGN, int STAGES, int XB, int ABL, bool RELU>
__global__ __launch_bounds__(64 * WGM * WGN) void sepconv_pipe_kernel(ConvGemmArgs a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int IPP = XB / 4;                   // glds instructions per band plane
  constexpr int PL = IPP * 1024;                // bytes per plane (64*IPP pixel slots)
  constexpr int ZSLOT = 64 * IPP - 1;           // zero slot of each plane
  constexpr int XI = BF + XB + 1;               // 1 KiB glds wave instructions per stage
  constexpr int L = (XI + NW - 1) / NW;         // per wave (surplus re-issues its last slot)
  constexpr int STAGE = XI * 1024;
  constexpr int BAND = BF * 1024, WOFF = (BF + XB) * 1024;
  constexpr int ABUF = AF * 1024;
  constexpr int CS = BN * 2 + 16;
  constexpr int SMEM_PIPE = STAGES * STAGE + 2 * ABUF;
  constexpr int SMEM = SMEM_PIPE > BM * CS ? SMEM_PIPE : BM * CS;
  constexpr int U = 2 * AF;                     // depthwise units (16 pixels x 16 channels)
  constexpr int UPW = (U + NW - 1) / NW;
  static_assert(XB % 4 == 0, "band planes are whole glds instructions");
  static_assert(NW % 2 == 0, "a wave's depthwise units share one channel group");
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H;
  const long NPIX = (long)a.B * H * W;
  const int nN = (a.NF * 16) / BN;
  const int nM = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.K >> 5;
  const int rlo = m0 / W - 1;                   // first staged raster row (may be -1)
  const long P0 = (long)rlo * W;                // its first pixel
  const int mlast = min(m0 + BM, a.M) - 1;
  const int NS = (mlast / W + 2 - rlo) * W;     // band slots used (rows rlo .. last+1)

  // ---- per-lane glds sources (byte pointers; the k-step advance is uniform per kind)
  const uint8_t* src[L];
  int kind[L];                                  // 0 = B, 1 = x band / zeros, 2 = dw weights
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int s = min(wave + i * NW, XI - 1);
    if (s < BF) {
      kind[i] = 0;
      src[i] = (const uint8_t*)(a.wp + ((long)(n0 / 16 + s) * KT) * 512 + lane * 8);
    } else if (s < BF + XB) {
      kind[i] = 1;
      const int q = (s - BF) / IPP, slot = ((s - BF) % IPP) * 64 + lane;
      long p = P0 + slot;
      p = p < 0 ? 0 : (p >= NPIX ? NPIX - 1 : p);
      src[i] = slot < NS ? (const uint8_t*)(a.x + p * a.ldx + q * 8) : sepp_zeros;
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

  // ---- depthwise units of this wave: u = wave + NW*i -> row fragment f = u >> 1,
  // channel group g = u & 1 (the same g for all of a wave's units: NW is even).
  const int g = wave & 1;
  const int p16 = lane & 15, kb = lane >> 4;
  const int par = kb >> 1;                      // tap parity: taps par, par+2, .. par+8
  const int qc = 2 * g + (kb & 1);              // 8-channel chunk (band plane) read
  // waves with fewer than UPW units repeat their last one (same value into the same A slot)
  // so every wave runs the same straight-line code
  const int ulast = U - 1 - ((U - 1 - wave) & 1);
  int toff[UPW][5];                             // band byte offsets (relative to the stage)
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = min(wave + NW * i, ulast);
    int mg = m0 + (u >> 1) * 16 + p16;
    mg = mg < a.M ? mg : a.M - 1;
    const int R = mg / W, w = mg - R * W, h = R % H;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int tap = 2 * j + par;
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bool ok = tap < 9 && (unsigned)(h + dy) < (unsigned)H && (unsigned)(w + dx) < (unsigned)W;
      const int slot = ok ? (R + dy - rlo) * W + w + dx : ZSLOT;
      toff[i][j] = BAND + qc * PL + slot * 16;
    }
  }
  // B-operand builder: lane (n = p16, kb) holds k = 8kb..8kb+7 = channels 16g+8(kb&1)..+7 of
  // one tap; its single non-zero element is e = n - 8(kb&1) (when in 0..7). v_perm_b32
  // selectors move value j (bytes 2(j&1), +1 of entry dword j>>1) to half e&1 of dword e>>1
  // (selector byte 0x0c yields 0x00).
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
  const int went = WOFF + ((g * 16 + p16) * 2 + par) * 16;   // this lane's weight entry
  const int aoffw = (p16 + 16 * (2 * g + (kb >> 1))) * 16 + 8 * (kb & 1);

  // depthwise of one stage: loads (issued early, so their latency hides behind the pointwise
  // MFMAs) and the MFMA part
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
      for (int i = 0; i < UPW; ++i) {             // independent chains interleaved
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

  // ---- prologue: stages 0 .. STAGES-2 in flight; A(0) = dw(x(0))
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < KT) issue(p, p);
  if (STAGES >= 3 && KT > 2) sp_wait_barrier<(STAGES - 2) * L>();   // stage 0 landed
  else sp_wait_barrier<0>();
  {
    u32x4 xv[UPW][5];
    const u32x4 we = dw_load(0, xv);
    dw_mfma(we, xv, 0);
  }

  for (int t = 0; t < KT; ++t) {
    // stage t+1 must have landed; stages issued after it may stay in flight
    const int after = min(KT - 1, t + STAGES - 2) - (t + 1);
    if (t + 1 >= KT || after <= 0) sp_wait_barrier<0>();
    else if (after == 1) sp_wait_barrier<L>();
    else sp_wait_barrier<2 * L>();
    const uint8_t* As = smem + STAGES * STAGE + (t & 1) * ABUF + lane * 16;
    const uint8_t* Bs = smem + (t % STAGES) * STAGE + lane * 16;
    s16x8 af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + (wm * FM + i) * 1024);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(Bs + (wn * FN + j) * 1024);
    // depthwise inputs of stage t+1 (landed). On the last step this reads a retired stage
    // and writes an A buffer nobody reads: harmless, and keeps the loop branch-free.
    u32x4 xv[UPW][5];
    u32x4 we;
    if constexpr (!(ABL & 2)) we = dw_load((t + 1) % STAGES, xv);
    if constexpr (!(ABL & 4))
      if (t + STAGES - 1 < KT) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!(ABL & 8)) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    } else {
      // keep the operand reads live
      acc[0][0][0] += __builtin_bit_cast(float, (int)af[0][0] ^ (int)bf[FN - 1][0]);
    }
    if constexpr (!(ABL & 3)) dw_mfma(we, xv, (t + 1) & 1);
    __builtin_amdgcn_s_setprio(0);
  }
  sp_wait_barrier<0>();

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
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < a.M && n < a.nstore) epi_store(a, m, n, *(const u32x4*)(smem + r * CS + cc * 16));
  }
}

// (FM, FN, WGM, WGN, STAGES, XB = x-band KiB per stage, a multiple of 4, ABL); ids offset by
// SEPP_CFG_BASE. LDS = STAGES * (BN/16 + XB + 1) KiB + 2 * BM/16 KiB <= 160 KiB.
// ABL != 0: timing ablations for tools/kbench.py --cfgs (wrong results by design; never
// autotune candidates): 1 no depthwise MFMA, 2 no depthwise at all, 4 no LDS-DMA in the
// loop, 8 no pointwise MFMA.
#define KDL_SEPP_CONFIGS(X)     \
  X(0, 3, 6, 2, 4, 4, 12, 0)    \
  X(1, 3, 6, 2, 4, 3, 12, 0)    \
  X(2, 3, 3, 2, 4, 4, 12, 0)    \
  X(3, 2, 6, 2, 4, 4, 12, 0)    \
  X(4, 3, 6, 2, 4, 3, 16, 0)    \
  X(5, 3, 3, 2, 4, 4, 16, 0)    \
  X(6, 2, 6, 2, 4, 3, 20, 0)    \
  X(7, 2, 3, 2, 4, 4, 20, 0)    \
  X(8, 3, 3, 2, 4, 3, 12, 0)    \
  X(16, 3, 6, 2, 4, 3, 12, 1)   \
  X(17, 3, 6, 2, 4, 3, 12, 2)   \
  X(18, 3, 6, 2, 4, 3, 12, 6)   \
  X(19, 3, 6, 2, 4, 3, 12, 4)   \
  X(20, 3, 6, 2, 4, 3, 12, 8)   \
  X(21, 3, 6, 2, 4, 3, 12, 14)

// band slots of BM consecutive raster pixels (worst alignment) + one halo row each side,
// plus the zero slot, must fit one plane of 16*XB slots
static int sepp_fits_xb(int BM, int W, int xb) { return ((BM + W - 2) / W + 3) * W + 1 <= 16 * xb; }

// ids >= SEPW_OFFSET: the warp-specialized variant (sepconv_ws.hip)
constexpr int SEPW_OFFSET = 24;

int sepconv_pipe_config(int cfg, int* bm, int* bn, int* threads) {
  if (cfg >= SEPW_OFFSET) return sepconv_ws_config(cfg - SEPW_OFFSET, bm, bn, threads);
  switch (cfg) {
#define KDL_SPINFO(id, fm, fn, wgm, wgn, st, xb, abl) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_SEPP_CONFIGS(KDL_SPINFO)
#undef KDL_SPINFO
    default: return -1;
  }
}

int sepconv_pipe_fits(int cfg, int W) {
  if (cfg >= SEPW_OFFSET) return sepconv_ws_fits(cfg - SEPW_OFFSET, W);
  switch (cfg) {
#define KDL_SPFIT(id, fm, fn, wgm, wgn, st, xb, abl) \
  case id: return sepp_fits_xb(16 * fm * wgm, W, xb);
    KDL_SEPP_CONFIGS(KDL_SPFIT)
#undef KDL_SPFIT
    default: return 0;
  }
}

hipError_t sepconv_pipe(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  if (cfg >= SEPW_OFFSET) return sepconv_ws(cfg - SEPW_OFFSET, a, s);
  int bm, bn, th;
  if (sepconv_pipe_config(cfg, &bm, &bn, &th) != 0 || !sepconv_pipe_fits(cfg, a.W) || a.K % 32 != 0 ||
      a.K > 8192 || (a.NF * 16) % bn != 0 || a.OH != a.H || a.OW != a.W || a.M <= 0 || a.dwk == nullptr)
    return hipErrorInvalidValue;
  const int grid = ((a.M + bm - 1) / bm) * ((a.NF * 16) / bn);
  switch (cfg) {
#define KDL_SPCASE(id, fm, fn, wgm, wgn, st, xb, abl)                                                          \
  case id:                                                                                              \
    if (a.relu_in) hipLaunchKernelGGL((sepconv_pipe_kernel<fm, fn, wgm, wgn, st, xb, abl, true>), dim3(grid),  \
                                      dim3(th), 0, s, a);                                               \
    else hipLaunchKernelGGL((sepconv_pipe_kernel<fm, fn, wgm, wgn, st, xb, abl, false>), dim3(grid), dim3(th), \
                            0, s, a);                                                                   \
    break;
    KDL_SEPP_CONFIGS(KDL_SPCASE)
#undef KDL_SPCASE
  }
  return hipGetLastError();
}

}  // namespace kdl
