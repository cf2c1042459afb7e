// Fused Keras SeparableConv2D + BN (+ReLU in/out)(+residual) for CDNA4.
// SURVEY.md §2.5 K5+K6 ("fuse K5 into K6's A-operand producer") and §7.4 hard
// parts 1-2.
//
// out[m][n] = sum_c dw3x3(relu?(x))[m][c] * W[n][c] + bias[n]   (NHWC, bf16)
//
// Design (one block = BM pixels in raster order x BN output channels; BN is
// chosen = all of N for N <= 768 so the depthwise is computed exactly ONCE):
//
//   * per 32-channel k-step the input rows the tile touches (its rows plus one
//     halo row above and below, full width) are register-staged into LDS
//     (16-byte coalesced loads issued one k-step ahead, written after a barrier:
//     the T14 "issue early / write late" split);
//   * the depthwise 3x3 is computed on the VALU out of that LDS image straight
//     into the bf16 A tile in LDS (fragment-linear image, conflict-free);
//   * the MFMA (v_mfma_f32_16x16x32_bf16, operands swapped so a lane holds 4
//     consecutive output channels) consumes the A tile; the weight fragments are
//     streamed global -> VGPR from a host-packed [n_frag][k][lane][8] layout
//     (each weight feeds exactly one wave, so LDS staging would buy nothing);
//   * the depthwise of k-step t+1 and the MFMAs of k-step t sit in the SAME
//     barrier phase, so one wave's VALU work overlaps the other wave's MFMAs on
//     each SIMD (separate pipes).
//
// Tiles that cross an image boundary are handled by staging "global rows"
// (b*H + h) and zeroing taps whose row leaves the pixel's own image.
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

template <int FM, int NFW, int NW, int SPT>
__global__ __launch_bounds__(64 * NW) void sepconv_fused_kernel(ConvGemmArgs a, int maxr) {
  constexpr int NT = 64 * NW;
  constexpr int BM = 16 * FM;
  constexpr int BN = 16 * NFW * NW;
  constexpr int DWS = (BM * 4 + NT - 1) / NT;   // depthwise chunk-outputs per thread per k-step
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int W = a.W, H = a.H;
  const int TR = a.B * H;                      // total rows over the batch
  const int nN = (a.NF * 16) / BN;
  const int nM = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.K >> 5;

  // LDS carve: xs[2][maxr][W][64B] | as[2][BM][64B] | ws[2][9][32] fp32
  const int XS = maxr * W * 64;
  uint8_t* xs0 = smem;
  uint8_t* as0 = smem + 2 * XS;
  float* ws0 = (float*)(as0 + 2 * BM * 64);

  const int R0 = m0 / W;
  const int R1 = min(m0 + BM - 1, a.M - 1) / W;
  const int rlo = R0 - 1;
  const int nrows = R1 - R0 + 3;               // <= maxr (host guarantees)
  const int nchunk = nrows * W * 4;

  // ---- staging: each thread owns SPT 16-byte chunks of the halo'd row band
  long soff[SPT];
  bool sval[SPT];
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int c = tid + i * NT;
    const int rl = c / (W * 4);
    const int rem = c - rl * W * 4;
    const int w = rem >> 2, q = rem & 3;
    const int rg = rlo + rl;
    sval[i] = c < nchunk && rg >= 0 && rg < TR;
    const int rgc = min(max(rg, 0), TR - 1);
    soff[i] = ((long)rgc * W + (c < nchunk ? w : 0)) * a.ldx + q * 8;
  }
  u32x4 xr[SPT];
  auto stage_load = [&](int t) {
#pragma unroll
    for (int i = 0; i < SPT; ++i) xr[i] = *(const u32x4*)(a.x + soff[i] + t * 32);
  };
  auto stage_write = [&](int t, int buf) {
    uint8_t* xs = xs0 + buf * XS;
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int c = tid + i * NT;
      if (c < nchunk) {
        u32x4 v = xr[i];
        if (!sval[i]) v = (u32x4){0u, 0u, 0u, 0u};
        if (a.relu_in) {
#pragma unroll
          for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
        }
        *(u32x4*)(xs + c * 16) = v;
      }
    }
    float* ws = ws0 + buf * 288;
    if (tid < 72) {
      const int tap = tid >> 3, part = tid & 7;
      *(float4*)(ws + tap * 32 + part * 4) = *(const float4*)(a.dww + tap * a.K + t * 32 + part * 4);
    }
  };

  // ---- depthwise producer: chunk-output o -> A-tile fragment-linear slot o*16
  int dpix_l[DWS], dw_w[DWS], dw_h[DWS];
#pragma unroll
  for (int s = 0; s < DWS; ++s) {
    const int o = tid + s * NT;
    const int f = o >> 6, li = o & 63;
    int m = m0 + f * 16 + (li & 15);
    m = min(m, a.M - 1);
    const int R = m / W;
    dw_w[s] = m - R * W;
    dw_h[s] = R % H;
    dpix_l[s] = (R - rlo) * W + dw_w[s];     // local pixel index of the tap (0,0) centre
  }
  auto dw_compute = [&](int buf) {
    const uint8_t* xs = xs0 + buf * XS;
    const float* ws = ws0 + buf * 288;
    uint8_t* as = as0 + buf * BM * 64;
#pragma unroll
    for (int s = 0; s < DWS; ++s) {
      const int o = tid + s * NT;
      if (BM * 4 % NT == 0 || o < BM * 4) {
        const int q = (o & 63) >> 4;
        f32x2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int dy = tap / 3 - 1, dx = tap % 3 - 1;
          const bool ok = (unsigned)(dw_h[s] + dy) < (unsigned)H && (unsigned)(dw_w[s] + dx) < (unsigned)W;
          const int pl = ok ? dpix_l[s] + dy * W + dx : dpix_l[s];
          const u32x4 v = *(const u32x4*)(xs + (pl * 4 + q) * 16);
          const float4 w0 = *(const float4*)(ws + tap * 32 + q * 8);
          const float4 w1 = *(const float4*)(ws + tap * 32 + q * 8 + 4);
          const f32x2 wv[4] = {{w0.x, w0.y}, {w0.z, w0.w}, {w1.x, w1.y}, {w1.z, w1.w}};
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint32_t u = ok ? v[d] : 0u;
            acc[d] = __builtin_elementwise_fma((f32x2){bf_lo(u), bf_hi(u)}, wv[d], acc[d]);
          }
        }
        u32x4 out;
#pragma unroll
        for (int d = 0; d < 4; ++d) out[d] = pack_bf16(acc[d][0], acc[d][1]);
        *(u32x4*)(as + o * 16) = out;
      }
    }
  };

  // ---- B fragments: global -> VGPR (wave w owns n-frags [w*NFW, (w+1)*NFW) of the tile)
  const uint16_t* wb = a.wp + ((long)(n0 / 16 + wave * NFW) * KT) * 512 + lane * 8;
  auto load_b = [&](int t, s16x8 (&bf)[NFW]) {
#pragma unroll
    for (int j = 0; j < NFW; ++j) bf[j] = *(const s16x8*)(wb + ((long)j * KT + t) * 512);
  };

  f32x4 acc[FM][NFW];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < NFW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: xs(0) -> LDS, A(0) = dw(0); xs(1) loads in flight
  s16x8 bc[NFW], bn[NFW];
  stage_load(0);
  load_b(0, bc);
  stage_write(0, 0);
  __syncthreads();
  dw_compute(0);
  if (KT > 1) stage_load(1);
  __syncthreads();
  if (KT > 1) stage_write(1, 1);
  if (KT > 2) stage_load(2);
  __syncthreads();

  for (int t = 0; t < KT; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    // phase A: B(t+1) in flight; MFMA(t) on A[cur] || depthwise(t+1) from xs[nxt] into A[nxt]
    if (t + 1 < KT) load_b(t + 1, bn);
    const uint8_t* As = as0 + cur * BM * 64 + lane * 16;
    s16x8 af[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + i * 1024);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < NFW; ++j) acc[i][j] = mfma16(bc[j], af[i], acc[i][j]);
    if (t + 1 < KT) dw_compute(nxt);
    __syncthreads();
    // phase B: xs(t+2) regs -> xs[cur] (last read by dw(t) one phase ago); issue xs(t+3)
    if (t + 2 < KT) stage_write(t + 2, cur);
    if (t + 3 < KT) stage_load(t + 3);
#pragma unroll
    for (int j = 0; j < NFW; ++j) bc[j] = bn[j];
    __syncthreads();
  }

  // ---- epilogue: bias, ReLU, LDS transpose, residual, 16-byte stores
  constexpr int CS = BN * 2 + 16;
  const int quad = lane >> 4, col = lane & 15;
#pragma unroll
  for (int j = 0; j < NFW; ++j) {
    const int nl = (wave * NFW + j) * 16 + 4 * quad;
    const float4 bv = *(const float4*)(a.bias + n0 + nl);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = i * 16 + col;
      float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y;
      float v2 = acc[i][j][2] + bv.z, v3 = acc[i][j][3] + bv.w;
      if (a.relu_out == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      *(u32x2*)(smem + ml * CS + nl * 2) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int c = tid; c < BM * CPR; c += NT) {
    const int r = c / CPR, cc = c - r * CPR;
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < a.M && n < a.nstore) {
      epi_store(a, m, n, *(const u32x4*)(smem + r * CS + cc * 16));
    }
  }
}

// (FM, NFW, NW, SPT): BM = 16*FM, BN = 16*NFW*NW, SPT = staged chunks per thread.
#define KDL_SEP_CONFIGS(X) \
  X(0, 4, 6, 8, 2)         \
  X(1, 4, 1, 8, 6)         \
  X(2, 4, 2, 8, 3)         \
  X(3, 2, 6, 8, 2)         \
  X(4, 4, 4, 8, 2)         \
  X(5, 4, 3, 8, 2)         \
  X(6, 8, 1, 8, 6)         \
  X(7, 8, 2, 8, 3)         \
  X(8, 2, 3, 8, 2)         \
  X(9, 4, 2, 4, 6)         \
  X(10, 4, 1, 4, 12)

// rows touched by BM consecutive raster pixels, plus one halo row on each side
static int sep_maxr(int BM, int W) { return (BM - 1) / W + 4; }

template <int FM, int NFW, int NW, int SPT>
static hipError_t launch_sep(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BM = 16 * FM, BN = 16 * NFW * NW;
  if ((a.NF * 16) % BN != 0 || a.OH != a.H || a.OW != a.W) return hipErrorInvalidValue;
  const int maxr = sep_maxr(BM, a.W);
  if ((long)maxr * a.W * 4 > (long)SPT * 64 * NW) return hipErrorInvalidValue;  // staging slots
  const size_t pipe = (size_t)2 * maxr * a.W * 64 + 2 * BM * 64 + 2 * 288 * 4;
  const size_t ctile = (size_t)BM * (BN * 2 + 16);
  const size_t smem = pipe > ctile ? pipe : ctile;
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  const int nM = (a.M + BM - 1) / BM, nN = (a.NF * 16) / BN;
  hipLaunchKernelGGL((sepconv_fused_kernel<FM, NFW, NW, SPT>), dim3(nM * nN), dim3(64 * NW), smem, s, a, maxr);
  return hipGetLastError();
}

hipError_t sepconv_fused(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  if (a.K % 32 != 0 || a.M <= 0) return hipErrorInvalidValue;
  switch (cfg) {
#define KDL_SCASE(id, fm, nfw, nw, spt) \
  case id: return launch_sep<fm, nfw, nw, spt>(a, s);
    KDL_SEP_CONFIGS(KDL_SCASE)
#undef KDL_SCASE
    default: return hipErrorInvalidValue;
  }
}

int sepconv_fused_config(int cfg, int* bm, int* bn, int* threads) {
  switch (cfg) {
#define KDL_SINFO(id, fm, nfw, nw, spt) \
  case id: *bm = 16 * fm; *bn = 16 * nfw * nw; *threads = 64 * nw; return 0;
    KDL_SEP_CONFIGS(KDL_SINFO)
#undef KDL_SINFO
    default: return -1;
  }
}

}  // namespace kdl
