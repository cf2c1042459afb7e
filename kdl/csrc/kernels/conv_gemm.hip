// Fused convolution-as-GEMM for NHWC bf16 activations on CDNA4 (gfx950).
//
// One kernel family covers every MFMA-shaped op of the Xception/ResNet graphs
// (SURVEY.md §2.5 K3/K4/K5/K6):
//
//   MODE_PW   1x1 conv (pointwise / residual), optional spatial stride.
//             A rows are gathered per lane and staged global->LDS by LDS-DMA
//             (global_load_lds_dwordx4): no VGPR round trip.
//   MODE_CONV 3x3 'valid' (optionally strided) conv as implicit GEMM; a 'same'
//             conv reads a zero-bordered input (producer wrote it with opad=1).
//             K = 9*cin, one tap per 32-deep
//             k-step, A rows are shifted pixel rows (also LDS-DMA).
//   MODE_DW   Keras SeparableConv2D: depthwise 3x3 'same' (+ optional ReLU on
//             load) is computed by the A-tile *producer* straight into LDS in
//             bf16 and consumed by the pointwise MFMA GEMM.  The depthwise output
//             never touches HBM (SURVEY.md §7.4 hard part 2).
//
// GEMM: Y[m][n] = sum_k A[m][k] * W[n][k] (+bias[n], ReLU, +residual[m][n]).
// The MFMA is issued with operands swapped (W fragment as "A") so each lane's
// accumulator holds 4 *consecutive output channels* of one pixel: the epilogue
// can write 8-byte runs into an LDS C tile and store 16-byte rows to HBM.
//
// Weights are pre-packed on the host into MFMA fragment order
// [n_frag][k_step][lane][8] so each wave's B-fragment load is one fully
// coalesced 1 KiB global_load_dwordx4 straight into VGPRs (each weight is used by
// exactly one wave of the block, so staging it through LDS would buy nothing).
//
// A tile LDS image is "fragment-linear": 16 rows x 32 k = 1 KiB per fragment,
// lane l's 16 bytes at l*16, which is (a) exactly what one LDS-DMA wave
// instruction writes and (b) exactly what ds_read_b128 of the MFMA operand reads:
// bank-conflict free with no swizzle.
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

enum { MODE_PW = 0, MODE_CONV = 1, MODE_DW = 2 };

// DT: element type (common.h Elt): 0 bf16, 1 fp16 (MODE_PW / MODE_CONV only)
template <int MODE, int FM, int FN, int WGM, int WGN, int DT = 0>
__global__ __launch_bounds__(64 * WGM * WGN) void conv_gemm_kernel(ConvGemmArgs a) {
  using E = Elt<DT>;
  static_assert(MODE != MODE_DW || DT == 0, "the fused depthwise producer is bf16-only");
  constexpr int NW = WGM * WGN;
  constexpr int NT = 64 * NW;
  constexpr int BM = 16 * FM * WGM;
  constexpr int BN = 16 * FN * WGN;
  constexpr int AFRAGS = BM / 16;                    // A fragments per stage
  constexpr int STAGE = BM * 64;                     // bytes per A stage
  constexpr int CS = BN * 2 + 16;                    // C tile row stride (bytes)
  constexpr int SMEM_MAIN = 2 * STAGE;
  constexpr int SMEM_C = BM * CS;
  constexpr int SMEM = SMEM_MAIN > SMEM_C ? SMEM_MAIN : SMEM_C;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  const int nN = (a.NF * 16) / BN;
  const int nM = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.K >> 5;

  const int OHW = a.OH * a.OW;

  // ---------------- A producers: per-lane source offsets (elements) ----------
  constexpr int AF_PER_WAVE = (AFRAGS + NW - 1) / NW;
  long aoff[AF_PER_WAVE];
  if constexpr (MODE != MODE_DW) {
#pragma unroll
    for (int s = 0; s < AF_PER_WAVE; ++s) {
      const int f = wave + s * NW;
      int m = m0 + f * 16 + (lane & 15);
      m = m < a.M ? m : a.M - 1;
      const int b = m / OHW, rem = m - b * OHW;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const long pix = ((long)b * a.H + (long)oh * a.stride) * a.W + (long)ow * a.stride;
      aoff[s] = pix * a.ldx + 8 * (lane >> 4);
    }
  }

  // MODE_DW: each thread owns DW_SLOTS 8-channel chunks of the A tile.
  constexpr int DW_CHUNKS = BM * 4;
  constexpr int DW_SLOTS = (DW_CHUNKS + NT - 1) / NT;
  int dw_b[DW_SLOTS], dw_oh[DW_SLOTS], dw_ow[DW_SLOTS];
  if constexpr (MODE == MODE_DW) {
#pragma unroll
    for (int s = 0; s < DW_SLOTS; ++s) {
      const int c = tid + s * NT;
      const int f = c >> 6, li = c & 63;
      int m = m0 + f * 16 + (li & 15);
      m = m < a.M ? m : a.M - 1;
      const int b = m / OHW, rem = m - b * OHW;
      dw_b[s] = b;
      dw_oh[s] = rem / a.OW;
      dw_ow[s] = rem - dw_oh[s] * a.OW;
    }
  }

  auto stage_ptr = [&](int buf) -> uint8_t* { return smem + buf * STAGE; };

  auto issue_a_dma = [&](int t, int buf) {
    long koff;
    if constexpr (MODE == MODE_PW) {
      koff = (long)t * 32;
    } else {
      const int k = t * 32;
      const int tap = k / a.cin, c0 = k - tap * a.cin;
      koff = ((long)(tap / 3) * a.W + (tap % 3)) * a.ldx + c0;
    }
#pragma unroll
    for (int s = 0; s < AF_PER_WAVE; ++s) {
      const int f = wave + s * NW;
      if (AFRAGS % NW == 0 || f < AFRAGS)
        glds16(a.x + aoff[s] + koff, stage_ptr(buf) + f * 1024);
    }
  };

  // Depthwise producer, split in two phases so the tap loads of stage t+1 are
  // in flight while the MFMAs of stage t run.
  u32x4 xr[DW_SLOTS][9];
  auto dw_load = [&](int t) {
#pragma unroll
    for (int s = 0; s < DW_SLOTS; ++s) {
      const int c = tid + s * NT;
      if (DW_CHUNKS % NT == 0 || c < DW_CHUNKS) {
        const int q = (c & 63) >> 4;
        const long cb = (long)t * 32 + 8 * q;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          int ih = dw_oh[s] + tap / 3 - 1, iw = dw_ow[s] + tap % 3 - 1;
          ih = ih < 0 ? 0 : (ih >= a.H ? a.H - 1 : ih);
          iw = iw < 0 ? 0 : (iw >= a.W ? a.W - 1 : iw);
          const long pix = ((long)dw_b[s] * a.H + ih) * a.W + iw;
          xr[s][tap] = *(const u32x4*)(a.x + pix * a.ldx + cb);
        }
      }
    }
  };
  auto dw_compute = [&](int t, int buf) {
#pragma unroll
    for (int s = 0; s < DW_SLOTS; ++s) {
      const int c = tid + s * NT;
      if (DW_CHUNKS % NT == 0 || c < DW_CHUNKS) {
        const int q = (c & 63) >> 4;
        const int kc = t * 32 + 8 * q;
        f32x2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int ih = dw_oh[s] + tap / 3 - 1, iw = dw_ow[s] + tap % 3 - 1;
          const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          const float4 w0 = *(const float4*)(a.dww + tap * a.K + kc);
          const float4 w1 = *(const float4*)(a.dww + tap * a.K + kc + 4);
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            uint32_t v = ok ? xr[s][tap][d] : 0u;
            if (a.relu_in) v = relu_bf16x2(v);
            const f32x2 xv = {bf_lo(v), bf_hi(v)};
            const f32x2 ww = {wv[2 * d], wv[2 * d + 1]};
            acc[d] = __builtin_elementwise_fma(xv, ww, acc[d]);
          }
        }
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = pack_bf16(acc[d][0], acc[d][1]);
        *(u32x4*)(stage_ptr(buf) + c * 16) = o;
      }
    }
  };

  // ---------------- B fragments: direct global -> VGPR -----------------------
  const uint16_t* wbase = a.wp + ((long)(n0 / 16 + wn * FN) * KT) * 512 + lane * 8;
  auto load_b = [&](int t, s16x8 (&bf)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bf[j] = *(const s16x8*)(wbase + ((long)j * KT + t) * 512);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  s16x8 bc[FN], bnx[FN];
  // prologue: stage 0
  load_b(0, bc);
  if constexpr (MODE == MODE_DW) {
    dw_load(0);
    dw_compute(0, 0);
  } else {
    issue_a_dma(0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < KT; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < KT;
    if (more) {
      load_b(t + 1, bnx);
      if constexpr (MODE == MODE_DW) dw_load(t + 1);
      else issue_a_dma(t + 1, cur ^ 1);
    }
    const uint8_t* As = stage_ptr(cur) + (wm * FM) * 1024 + lane * 16;
    s16x8 af[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(As + i * 1024);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = E::mfma(bc[j], af[i], acc[i][j]);
    if constexpr (MODE == MODE_DW) {
      if (more) dw_compute(t + 1, cur ^ 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FN; ++j) bc[j] = bnx[j];
  }

  // ---------------- epilogue: bias, ReLU, LDS transpose, residual, store ----
  const int quad = lane >> 4, col = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * FN * 16 + j * 16 + 4 * quad;
    const float4 bv = *(const float4*)(a.bias + n0 + nl);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = wm * FM * 16 + i * 16 + col;
      float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y;
      float v2 = acc[i][j][2] + bv.z, v3 = acc[i][j][3] + bv.w;
      if (a.relu_out == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      u32x2 pk = {E::pack(v0, v1), E::pack(v2, v3)};
      *(u32x2*)(smem + ml * CS + nl * 2) = pk;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
  for (int c = tid; c < BM * CPR; c += NT) {
    const int r = c / CPR, cc = c - r * CPR;
    const int m = m0 + r, n = n0 + cc * 8;
    if (m < a.M && n < a.nstore) {
      epi_store<DT>(a, m, n, *(const u32x4*)(smem + r * CS + cc * 16));
    }
  }
}

// --------------------------------------------------------------------------
// Config table. Index = config id used by the host (kdl/ops/conv_gemm.py keeps
// the same list).  (FM, FN, WGM, WGN): block tile = (16*FM*WGM) x (16*FN*WGN).
#define KDL_CONFIGS(X)  \
  X(0, 2, 2, 2, 2)      \
  X(1, 4, 2, 2, 2)      \
  X(2, 2, 4, 2, 2)      \
  X(3, 4, 4, 2, 2)      \
  X(4, 4, 6, 1, 8)      \
  X(5, 2, 12, 1, 4)     \
  X(6, 4, 4, 1, 4)      \
  X(7, 2, 6, 1, 8)      \
  X(8, 8, 2, 1, 4)      \
  X(9, 4, 2, 1, 4)

template <int MODE, int FM, int FN, int WGM, int WGN, int DT>
static hipError_t launch_cfg(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  if ((a.NF * 16) % BN != 0) return hipErrorInvalidValue;
  const int nM = (a.M + BM - 1) / BM, nN = (a.NF * 16) / BN;
  hipLaunchKernelGGL((conv_gemm_kernel<MODE, FM, FN, WGM, WGN, DT>), dim3(nM * nN), dim3(64 * WGM * WGN), 0, s, a);
  return hipGetLastError();
}

template <int MODE, int DT = 0>
static hipError_t launch_mode(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  switch (cfg) {
#define KDL_CASE(id, fm, fn, wgm, wgn) \
  case id: return launch_cfg<MODE, fm, fn, wgm, wgn, DT>(a, s);
    KDL_CONFIGS(KDL_CASE)
#undef KDL_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t conv_gemm(int mode, int cfg, const ConvGemmArgs& a, hipStream_t s) {
  if (a.K % 32 != 0 || a.M <= 0 || a.dt < 0 || a.dt > 1) return hipErrorInvalidValue;
  // A-operand channel scales: the LDS-DMA pipelined and streaming GEMMs only (any other kernel
  // would ignore them)
  if (a.ascale && cfg < STREAM_CFG_BASE && (cfg < PIPE_CFG_BASE || cfg >= SEP_CFG_BASE)) return hipErrorInvalidValue;
  if (cfg >= STREAM_CFG_BASE)
    return mode == MODE_PW && cfg <= STREAM_CFG_BASE + 1 ? gemm_stream(a, cfg == STREAM_CFG_BASE + 1, s)
                                                         : hipErrorInvalidValue;
  // split-K: the LDS-DMA pipelined GEMM only
  if (a.ksplit > 1 && (cfg < PIPE_CFG_BASE || cfg >= SEP_CFG_BASE)) return hipErrorInvalidValue;
  if (a.dt == 1) {   // fp16: the pointwise / implicit-3x3 GEMMs only
    if (cfg >= SEP_CFG_BASE) return hipErrorInvalidValue;
    if (cfg >= PIPE_CFG_BASE) return gemm_pipe(mode, cfg - PIPE_CFG_BASE, a, s);
    if (mode == MODE_PW) return launch_mode<MODE_PW, 1>(cfg, a, s);
    if (mode == MODE_CONV) return launch_mode<MODE_CONV, 1>(cfg, a, s);
    return hipErrorInvalidValue;
  }
  if (cfg >= C3_CFG_BASE) return mode == MODE_CONV ? conv3x3_2d(cfg - C3_CFG_BASE, a, s) : hipErrorInvalidValue;
  if (cfg >= S2D_CFG_BASE) return mode == MODE_DW ? sepconv_2d(cfg - S2D_CFG_BASE, a, s) : hipErrorInvalidValue;
  if (cfg >= SEPW_CFG_BASE) return mode == MODE_DW ? sepconv_ws(cfg - SEPW_CFG_BASE, a, s) : hipErrorInvalidValue;
  if (cfg >= SEP_CFG_BASE) return hipErrorInvalidValue;
  if (cfg >= PIPE_CFG_BASE) return gemm_pipe(mode, cfg - PIPE_CFG_BASE, a, s);
  switch (mode) {
    case MODE_PW: return launch_mode<MODE_PW>(cfg, a, s);
    case MODE_CONV: return launch_mode<MODE_CONV>(cfg, a, s);
    case MODE_DW: return launch_mode<MODE_DW>(cfg, a, s);
    default: return hipErrorInvalidValue;
  }
}

int conv_gemm_config(int cfg, int* bm, int* bn, int* threads) {
  if (cfg == STREAM_CFG_BASE || cfg == STREAM_CFG_BASE + 1) { *bm = 16; *bn = 32; *threads = 512; return 0; }   // nominal
  if (cfg > STREAM_CFG_BASE) return -1;
  if (cfg >= C3_CFG_BASE) return conv3x3_2d_config(cfg - C3_CFG_BASE, bm, bn, threads);
  if (cfg >= S2D_CFG_BASE) return sepconv_2d_config(cfg - S2D_CFG_BASE, bm, bn, threads);
  if (cfg >= SEPW_CFG_BASE) return sepconv_ws_config(cfg - SEPW_CFG_BASE, bm, bn, threads);
  if (cfg >= SEP_CFG_BASE) return -1;
  if (cfg >= PIPE_CFG_BASE) return gemm_pipe_config(cfg - PIPE_CFG_BASE, bm, bn, threads);
  switch (cfg) {
#define KDL_INFO(id, fm, fn, wgm, wgn) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_CONFIGS(KDL_INFO)
#undef KDL_INFO
    default: return -1;
  }
}

int conv_gemm_num_configs() {
  int n = 0;
#define KDL_COUNT(id, fm, fn, wgm, wgn) ++n;
  KDL_CONFIGS(KDL_COUNT)
#undef KDL_COUNT
  return n;
}

}  // namespace kdl
