// Pipelined fused SeparableConv2D (+BN)(+ReLU in/out)(+residual) for CDNA4:
//   out[m][n] = sum_c dw3x3(relu?(x))[m][c] * W[n][c] + bias[n]
// SURVEY.md §2.5 K5+K6 / §7.4 hard parts 1-2: the depthwise never leaves the chip.
//
// Versus the split lowering (dw3x3 kernel -> 34 MB round trip through MALL/HBM ->
// LDS-DMA GEMM) and the first fused kernel (sepconv_fused.hip: VGPR-staged halo
// rows and B, two barriers per k-step), everything here is LDS-DMA staged:
//
//   stage t (one 32-channel k-step) = { B fragments (pointwise weights, packed)
//                                       x band: the tile's image rows +-1, full width
//                                       depthwise weights of the 32 channels }
//   all three land by global_load_lds_dwordx4 into a STAGES-deep LDS ring with a
//   counted vmcnt + raw barrier (one barrier per k-step), so the x band of k-step
//   t+1 is already in LDS while k-step t's MFMAs run.
//
//   iteration t:  wait(stage t+1) + barrier ; issue stage t+STAGES-1 ;
//                 MFMA(A[t&1], B(t))  ||  depthwise(x(t+1)) -> A[(t+1)&1]
//   Depthwise VALU work of one wave and MFMAs of another overlap on each SIMD
//   (separate pipes); the depthwise output is rounded to bf16 exactly like the
//   split path and written in the fragment-linear A image.
//
// The x band is staged as consecutive raster pixels (rows rlo .. rlo+maxr-1 of the
// flattened B*H image stack), lane-linear, so each 1 KiB glds wave instruction
// covers 16 pixels x 4 quarter-chunks; taps outside the pixel's own image are
// masked at compute time (rows of the neighbouring image are never used).
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

template <int N>
__device__ __forceinline__ void sp_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int FM, int FN, int WGM, int WGN, int STAGES, int XB>
__global__ __launch_bounds__(64 * WGM * WGN) void sepconv_pipe_kernel(ConvGemmArgs a) {
  const float* dwk = a.dwk;
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  constexpr int AF = BM / 16, BF = BN / 16;
  // per-stage layout: [B frags BF KiB][x band XB KiB][dw weights 2 KiB]
  constexpr int XI = BF + XB + 2;              // 1 KiB glds wave instructions per stage
  constexpr int L = (XI + NW - 1) / NW;         // per wave (surplus re-issues its last slot)
  constexpr int STAGE = XI * 1024;
  constexpr int ABUF = AF * 1024;
  constexpr int CS = BN * 2 + 16;
  constexpr int SMEM_PIPE = STAGES * STAGE + 2 * ABUF;
  constexpr int SMEM = SMEM_PIPE > BM * CS ? SMEM_PIPE : BM * CS;
  constexpr int CPW = BM * 4 / NW;              // depthwise chunk-outputs per wave per k-step
  static_assert(CPW <= 64, "one depthwise chunk-output per lane");
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int W = a.W, H = a.H;
  const int TR = a.B * H;
  const int nN = (a.NF * 16) / BN;
  const int nM = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.K >> 5;
  const int rlo = m0 / W - 1;                   // first staged raster row (may be -1)
  const long P0 = (long)rlo * W;                // its first pixel

  // ---- per-lane glds sources
  long src[L];
  int kind[L];                                  // 0 = B, 1 = x band, 2 = dw weights
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int s = min(wave + i * NW, XI - 1);
    if (s < BF) {
      kind[i] = 0;
      src[i] = ((long)(n0 / 16 + s) * KT) * 512 + lane * 8;
    } else if (s < BF + XB) {
      kind[i] = 1;
      const int c = (s - BF) * 64 + lane;       // 16-byte chunk of the band
      long p = P0 + (c >> 2);
      p = p < 0 ? 0 : (p >= (long)TR * W ? (long)TR * W - 1 : p);
      src[i] = p * a.ldx + (c & 3) * 8;
    } else {
      kind[i] = 2;
      const int c = min((s - BF - XB) * 64 + lane, 71);   // 9 taps x 32 ch x 4 B = 72 chunks
      src[i] = (long)c * 4;
    }
  }
  auto issue = [&](int t, int slot) {
    uint8_t* base = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int s = min(wave + i * NW, XI - 1);
      if (kind[i] == 0) glds16(a.wp + src[i] + (long)t * 512, base + s * 1024);
      else if (kind[i] == 1) glds16(a.x + src[i] + t * 32, base + s * 1024);
      else glds16(dwk + src[i] + (long)t * 288, base + s * 1024);
    }
  };

  // ---- depthwise producer: lane owns chunk-output o = wave*CPW + lane (pixel ml, quarter q).
  // Branch-free on purpose: lanes >= CPW duplicate another lane's item (same value to the
  // same LDS slot) and out-of-image taps read the centre pixel and are zeroed by a select.
  // Any branch here puts a block boundary after the in-flight LDS-DMA, where hipcc's
  // waitcnt pass conservatively drains it (s_waitcnt vmcnt(0) before every tap's ds_read).
  const int o = wave * CPW + (lane % CPW);
  const int ml = o >> 2, q = o & 3;
  int mg = m0 + ml;
  mg = mg < a.M ? mg : a.M - 1;
  const int R = mg / W, w = mg - R * W;
  const int h = R % H;
  const int lp = (R - rlo) * W + w;             // local band pixel of the centre tap
  int toff[9];                                  // byte offset of each tap (centre if masked)
  uint32_t tkeep[9];                            // all-ones if the tap is inside the pixel's image
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
    const bool ok = (unsigned)(h + dy) < (unsigned)H && (unsigned)(w + dx) < (unsigned)W;
    toff[tap] = ((ok ? lp + dy * W + dx : lp) * 4 + q) * 16;
    tkeep[tap] = ok ? 0xffffffffu : 0u;
  }
  // fragment-linear A slot of this chunk-output
  const int aoff = ((ml >> 4) * 64 + (ml & 15) + 16 * q) * 16;
  const uint32_t relu_mask = a.relu_in ? 0u : 0xffffffffu;

  auto dw_compute = [&](int slot, int abuf) {
    const uint8_t* xs = smem + slot * STAGE + BF * 1024;
    // dw weights read as u32x4 and bit-cast: float-typed LDS reads here made hipcc drain the
    // in-flight LDS-DMA (s_waitcnt vmcnt(0)) before them; integer-typed reads do not.
    const uint8_t* ws = smem + slot * STAGE + (BF + XB) * 1024;
    f32x2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      u32x4 v = *(const u32x4*)(xs + toff[tap]);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        // ReLU on load (v_pk_max_i16) unless disabled, then the tap mask
        const uint32_t r = relu_bf16x2(v[d]);
        v[d] = ((r & ~relu_mask) | (v[d] & relu_mask)) & tkeep[tap];
      }
      const u32x4 u0 = *(const u32x4*)(ws + tap * 128 + q * 32);
      const u32x4 u1 = *(const u32x4*)(ws + tap * 128 + q * 32 + 16);
      const f32x2 wv[4] = {{__uint_as_float(u0[0]), __uint_as_float(u0[1])},
                           {__uint_as_float(u0[2]), __uint_as_float(u0[3])},
                           {__uint_as_float(u1[0]), __uint_as_float(u1[1])},
                           {__uint_as_float(u1[2]), __uint_as_float(u1[3])}};
#pragma unroll
      for (int d = 0; d < 4; ++d) acc[d] = __builtin_elementwise_fma((f32x2){bf_lo(v[d]), bf_hi(v[d])}, wv[d], acc[d]);
    }
    u32x4 out;
#pragma unroll
    for (int d = 0; d < 4; ++d) out[d] = pack_bf16(acc[d][0], acc[d][1]);
    *(u32x4*)(smem + STAGES * STAGE + abuf * ABUF + aoff) = out;
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
  if (KT > 1) {
    if (STAGES - 2 >= 1 && KT > 2) sp_wait_barrier<(STAGES - 2) * L>();   // stage 0 landed
    else sp_wait_barrier<0>();
  } else {
    sp_wait_barrier<0>();
  }
  dw_compute(0, 0);

  for (int t = 0; t < KT; ++t) {
    // stage t+1 must have landed; stages issued after it may stay in flight
    const int after = min(KT - 1, t + STAGES - 2) - (t + 1);
    if (t + 1 >= KT || after <= 0) sp_wait_barrier<0>();
    else if (after == 1) sp_wait_barrier<L>();
    else sp_wait_barrier<2 * L>();
    if (t + STAGES - 1 < KT) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const uint8_t* As = smem + STAGES * STAGE + (t & 1) * ABUF + lane * 16;
    const uint8_t* Bs = smem + (t % STAGES) * STAGE + lane * 16;
    s16x8 af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + (wm * FM + i) * 1024);
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(Bs + (wn * FN + j) * 1024);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bf[j], af[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (t + 1 < KT) dw_compute((t + 1) % STAGES, (t + 1) & 1);
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

// (FM, FN, WGM, WGN, STAGES, XB = x-band KiB per stage); ids offset by SEPP_CFG_BASE.
#define KDL_SEPP_CONFIGS(X)  \
  X(0, 3, 6, 2, 4, 4, 11)    \
  X(1, 3, 6, 2, 4, 3, 11)    \
  X(2, 3, 3, 2, 4, 4, 11)    \
  X(3, 2, 6, 2, 4, 4, 9)     \
  X(4, 3, 3, 2, 4, 3, 11)    \
  X(5, 2, 3, 2, 4, 4, 9)     \
  X(6, 2, 6, 2, 4, 3, 17)    \
  X(7, 3, 3, 2, 4, 3, 19)    \
  X(8, 2, 3, 2, 4, 3, 17)

// rows touched by BM consecutive raster pixels (worst alignment) + one halo row each side
static int sepp_band_chunks(int BM, int W) { return ((BM + W - 2) / W + 3) * W * 4; }

int sepconv_pipe_config(int cfg, int* bm, int* bn, int* threads) {
  switch (cfg) {
#define KDL_SPINFO(id, fm, fn, wgm, wgn, st, xb) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_SEPP_CONFIGS(KDL_SPINFO)
#undef KDL_SPINFO
    default: return -1;
  }
}

int sepconv_pipe_fits(int cfg, int W) {
  switch (cfg) {
#define KDL_SPFIT(id, fm, fn, wgm, wgn, st, xb) \
  case id: return sepp_band_chunks(16 * fm * wgm, W) <= xb * 64;
    KDL_SEPP_CONFIGS(KDL_SPFIT)
#undef KDL_SPFIT
    default: return 0;
  }
}

hipError_t sepconv_pipe(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  int bm, bn, th;
  if (sepconv_pipe_config(cfg, &bm, &bn, &th) != 0 || !sepconv_pipe_fits(cfg, a.W) || a.K % 32 != 0 ||
      (a.NF * 16) % bn != 0 || a.OH != a.H || a.OW != a.W || a.M <= 0 || a.dwk == nullptr)
    return hipErrorInvalidValue;
  const int grid = ((a.M + bm - 1) / bm) * ((a.NF * 16) / bn);
  switch (cfg) {
#define KDL_SPCASE(id, fm, fn, wgm, wgn, st, xb) \
  case id: hipLaunchKernelGGL((sepconv_pipe_kernel<fm, fn, wgm, wgn, st, xb>), dim3(grid), dim3(th), 0, s, a); break;
    KDL_SEPP_CONFIGS(KDL_SPCASE)
#undef KDL_SPCASE
  }
  return hipGetLastError();
}

}  // namespace kdl
