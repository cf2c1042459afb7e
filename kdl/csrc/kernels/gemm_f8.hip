// FP8 (OCP e4m3) GEMM for the transformer linear layers (BASELINE.json "ViT-B/16
// ... pure-GEMM path on CDNA4 fp8 MFMA"):
//   Y[m][n] = act( colscale[n] * sum_k A8[m][k] W8[n][k] + bias[n] ) (+ residual)
// with A8 = activation / s_a, W8 = weight / s_w[n] and colscale[n] = s_a * s_w[n]
// folded on the host; output bf16 or (for a following fp8 GEMM) e4m3 / s_out.
//
// MFMA: v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (e8m0 127) -- the
// 2x-bf16-rate instruction; per-tensor / per-channel scaling is done in fp32 in the
// epilogue. Operand order "contig32": lane l holds row (l & 15), k = 32(l >> 4) ..
// +31 of the 128-deep step, for A and W alike (tests/test_fp8_gpu.py).
//
// Pipeline identical in spirit to gemm_pipe.hip: both operands staged global->LDS
// by LDS-DMA (global_load_lds_dwordx4) into a STAGES-deep ring, counted vmcnt +
// raw barrier, one barrier per 128-deep k-step. A 16x128 fp8 fragment is 2 KiB =
// two lane-linear 1 KiB halves (bytes 0-15 / 16-31 of every lane), so each half is
// exactly one glds wave instruction and one conflict-free ds_read_b128.
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

typedef int v8i __attribute__((ext_vector_type(8)));

template <int N>
__device__ __forceinline__ void f8_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int FM, int FN, int WGM, int WGN, int STAGES>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f8_kernel(GemmF8Args a) {
  constexpr int NW = WGM * WGN;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int HF = 2 * (AF + BF);           // 1 KiB half-fragments per stage
  constexpr int L = (HF + NW - 1) / NW;       // glds per wave per stage (surplus slots re-issue the last)
  constexpr int STAGE = HF * 1024;
  constexpr int CS = BN * 2 + 16;
  constexpr int SMEM = STAGES * STAGE > BM * CS ? STAGES * STAGE : BM * CS;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int nN = (a.NF * 16) / BN;
  const int nM = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, nM * nN);
  const int mi = wg / nN, ni = wg % nN;
  const int m0 = mi * BM, n0 = ni * BN;
  const int KT = a.K >> 7;
  const int krot = a.krot ? (mi * 7) % KT : 0;  // rotated k order: M tiles do not all fetch the same B at once

  long src[L];
  bool isa[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int hf = min(wave + i * NW, HF - 1);
    const int f = hf >> 1, h = hf & 1;
    isa[i] = f < AF;
    if (f < AF) {
      int m = m0 + f * 16 + (lane & 15);
      m = m < a.M ? m : a.M - 1;
      src[i] = (long)m * a.ldx + 32 * (lane >> 4) + 16 * h;
    } else {
      const int nf = n0 / 16 + (f - AF);
      src[i] = ((long)nf * KT * 2 + h) * 1024 + lane * 16;
    }
  }
  auto issue = [&](int t, int buf) {
    uint8_t* base = smem + buf * STAGE;
    t += krot;
    t = t >= KT ? t - KT : t;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int hf = min(wave + i * NW, HF - 1);
      if (isa[i]) glds16(a.x + src[i] + (long)t * 128, base + hf * 1024);
      else glds16(a.wp + src[i] + (long)t * 2048, base + hf * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < KT) issue(p, p);

  for (int t = 0; t < KT; ++t) {
    const int after = min(KT - 1, t + STAGES - 2) - t;
    if (after >= 2) f8_wait_barrier<2 * L>();
    else if (after == 1) f8_wait_barrier<L>();
    else f8_wait_barrier<0>();
    if (t + STAGES - 1 < KT) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const uint8_t* st = smem + (t % STAGES) * STAGE + lane * 16;
    v8i af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const u32x4 lo = *(const u32x4*)(st + ((wm * FM + i) * 2) * 1024);
      const u32x4 hi = *(const u32x4*)(st + ((wm * FM + i) * 2 + 1) * 1024);
      af[i] = (v8i){(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const u32x4 lo = *(const u32x4*)(st + ((AF + wn * FN + j) * 2) * 1024);
      const u32x4 hi = *(const u32x4*)(st + ((AF + wn * FN + j) * 2 + 1) * 1024);
      bf[j] = (v8i){(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[i][j], 0, 0, 0, 127, 0, 127);
    __builtin_amdgcn_s_setprio(0);
  }
  f8_wait_barrier<0>();

  // epilogue: per-column scale + bias (+ReLU) -> bf16 C tile in LDS -> store pass
  const int quad = lane >> 4, col = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * FN * 16 + j * 16 + 4 * quad;
    const float4 bv = *(const float4*)(a.bias + n0 + nl);
    const float4 sv = *(const float4*)(a.colscale + n0 + nl);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = wm * FM * 16 + i * 16 + col;
      float v0 = acc[i][j][0] * sv.x + bv.x, v1 = acc[i][j][1] * sv.y + bv.y;
      float v2 = acc[i][j][2] * sv.z + bv.z, v3 = acc[i][j][3] * sv.w + bv.w;
      if (a.relu_out == 1) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      *(u32x2*)(smem + ml * CS + nl * 2) = (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)};
    }
  }
  // residual rows (ViT out_proj / mlp.3): loaded before the C-tile barrier, not inside the store pass
  // where each load waited behind the earlier stores (in-order vmcnt; cf. gemm_pipe.hip / sepconv_ws.hip):
  // ViT-B/16 fp8 +1.2 % in 3 of 3 interleaved pairs (profiles/epilogue_residual_r6.txt)
  constexpr int CPR = BN / 8;
  constexpr int NIT = (BM * CPR + 64 * NW - 1) / (64 * NW);
  u32x4 rres[NIT];
  if (a.res) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = tid + it * 64 * NW, r = c / CPR, cc = c - r * CPR;
      const int m = min(m0 + r, a.M - 1), n = min(n0 + cc * 8, a.nstore - 8);
      rres[it] = c < BM * CPR ? *(const u32x4*)(a.res + (long)m * a.ldr + n) : (u32x4){0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = tid + it * 64 * NW, r = c / CPR, cc = c - r * CPR;
    const int m = m0 + r, n = n0 + cc * 8;
    if (c < BM * CPR && m < a.M && n < a.nstore) {
      u32x4 v = *(const u32x4*)(smem + r * CS + cc * 16);
      if (a.relu_out >= 3) v = act_transcendental(a.relu_out, v);
      if (a.res) {
        const u32x4 rv = rres[it];
#pragma unroll
        for (int d = 0; d < 4; ++d) v[d] = pack_bf16(bf_lo(v[d]) + bf_lo(rv[d]), bf_hi(v[d]) + bf_hi(rv[d]));
      }
      if (a.y8) {
        const float q = a.out_inv_scale;
        *(u32x2*)(a.y8 + (long)m * a.ldy + n) =
            (u32x2){pack_fp8x4(bf_lo(v[0]) * q, bf_hi(v[0]) * q, bf_lo(v[1]) * q, bf_hi(v[1]) * q),
                    pack_fp8x4(bf_lo(v[2]) * q, bf_hi(v[2]) * q, bf_lo(v[3]) * q, bf_hi(v[3]) * q)};
      } else {
        *(u32x4*)(a.y + (long)m * a.ldy + n) = v;
      }
    }
  }
}

// (FM, FN, WGM, WGN, STAGES)
#define KDL_F8_CONFIGS(X) \
  X(0, 4, 4, 2, 2, 2)     \
  X(1, 4, 4, 2, 2, 3)     \
  X(2, 2, 4, 2, 2, 3)     \
  X(3, 4, 2, 2, 4, 2)     \
  X(4, 3, 3, 2, 4, 2)     \
  X(5, 6, 3, 2, 4, 2)     \
  X(6, 3, 6, 2, 4, 2)     \
  X(7, 4, 4, 2, 4, 2)     \
  X(8, 5, 2, 2, 4, 2)     \
  X(9, 5, 3, 2, 4, 2)     \
  X(10, 5, 4, 2, 4, 2)     \
  X(11, 4, 4, 2, 4, 3)     \
  X(12, 5, 2, 2, 4, 3)     \
  X(13, 4, 2, 2, 4, 3)     \
  X(14, 5, 2, 2, 4, 4)     \
  X(15, 4, 2, 2, 4, 4)     \
  X(16, 8, 4, 2, 4, 2)     \
  X(17, 6, 4, 2, 4, 2)
// 8-10: 160-row tiles, whole waves of 256 CUs at the ViT-B/16 token count (gemm_pipe.hip 45-47);
// 11-15: 3-4 stage rings of the large tiles (2 stages leave one k-step of load latency exposed)
// 16-17: 256 x 256 / 192 x 256 tiles: at 128-deep fp8 k-steps a 160 x 128 tile needs ~57 B/clk per CU
// to keep the MFMAs busy, more than an L2-fed CU takes in (~28-30); 256 x 256 needs ~32 (244 VGPRs;
// the 4-wave 8 x 8-fragment form spills at 256 VGPR + 256 AGPR)

int gemm_f8_config(int cfg, int* bm, int* bn, int* threads) {
  switch (cfg) {
#define KDL_F8INFO(id, fm, fn, wgm, wgn, st) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_F8_CONFIGS(KDL_F8INFO)
#undef KDL_F8INFO
    default: return -1;
  }
}

hipError_t gemm_f8(int cfg, const GemmF8Args& args, hipStream_t s) {
  static const int env_krot = [] { const char* e = getenv("KDL_F8_KROT"); return e ? atoi(e) : -1; }();
  GemmF8Args a = args;
  if (env_krot >= 0) a.krot = env_krot;
  int bm, bn, th;
  if (gemm_f8_config(cfg, &bm, &bn, &th) != 0 || a.K % 128 != 0 || a.ldx % 16 != 0 || (a.NF * 16) % bn != 0 ||
      a.M <= 0)
    return hipErrorInvalidValue;
  const int grid = ((a.M + bm - 1) / bm) * ((a.NF * 16) / bn);
  switch (cfg) {
#define KDL_F8CASE(id, fm, fn, wgm, wgn, st) \
  case id: hipLaunchKernelGGL((gemm_f8_kernel<fm, fn, wgm, wgn, st>), dim3(grid), dim3(th), 0, s, a); break;
    KDL_F8_CONFIGS(KDL_F8CASE)
#undef KDL_F8CASE
  }
  return hipGetLastError();
}

}  // namespace kdl
