// Pipelined conv-GEMM for the pointwise (MODE_PW) and implicit-3x3 (MODE_CONV)
// lowerings: Y[m][n] = sum_k A[m][k] W[n][k] + bias (+ReLU)(+residual), bf16 NHWC.
//
// CDNA4 structure (cdna_hip_programming.md §5, "Pipelining across barriers"):
//   * BOTH operands are staged global->LDS by LDS-DMA (global_load_lds_dwordx4);
//     no VGPR-destination loads in the k-loop, so hipcc never inserts a draining
//     vmcnt(0) (guide §5 trap (b): "go all-glds for both operands").
//   * a STAGES-deep LDS ring; stage t+STAGES-1 is issued while stage t is
//     consumed, and the wait before each barrier is a COUNTED vmcnt that leaves
//     the younger stages in flight across the raw s_barrier.
//   * one barrier per 32-deep k-step; MFMA v_mfma_f32_16x16x32_bf16 with swapped
//     operands so each lane's accumulator holds 4 consecutive output channels
//     (8-byte LDS writes in the epilogue, 16-byte coalesced global stores).
//   * fragment-linear LDS image (1 KiB per 16x32 fragment, lane l at l*16): what
//     one LDS-DMA wave instruction writes is exactly what ds_read_b128 of the MFMA
//     operand reads -> conflict-free without a swizzle.
//   * XCD-aware bijective block remap (T1).
#include "common.h"
#include "launch.h"
#include "epilogue.h"

namespace kdl {

// ASC: one A fragment (8 consecutive k of one row, bf16) times its 8 channel scales (fp32), back to bf16
__device__ __forceinline__ s16x8 pipe_ascale8(const s16x8 v, const f32x4 s0, const f32x4 s1) {
  const u32x4 u = __builtin_bit_cast(u32x4, v);
  u32x4 o;
  o[0] = pack_bf16(bf_lo(u[0]) * s0[0], bf_hi(u[0]) * s0[1]);
  o[1] = pack_bf16(bf_lo(u[1]) * s0[2], bf_hi(u[1]) * s0[3]);
  o[2] = pack_bf16(bf_lo(u[2]) * s1[0], bf_hi(u[2]) * s1[1]);
  o[3] = pack_bf16(bf_lo(u[3]) * s1[2], bf_hi(u[3]) * s1[3]);
  return __builtin_bit_cast(s16x8, o);
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// DT: element type (common.h Elt): 0 bf16, 1 fp16. (Round 2's timing ablations of this
// kernel -- no MFMA / no DMA / no stores / contiguous A -- are in profiles/kernel_ablations_r2.txt.)
// ASC: per-image channel scales on A (ConvGemmArgs.ascale; MODE_PW bf16): each stage gets one more
// 1 KiB DMA slot holding the k-step's 32 scales of the tile's image (128 bytes, repeated), read as
// 2 broadcast ds_read_b128 per lane and applied to the A fragments in registers before the MFMAs.
template <int MODE, int FM, int FN, int WGM, int WGN, int STAGES, int KSUB, int DT = 0, bool ASC = false>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_pipe_kernel(ConvGemmArgs a) {
  using E = Elt<DT>;
  static_assert(!ASC || (MODE == 0 && DT == 0), "A-operand scales: bf16 pointwise only");
  constexpr int NW = WGM * WGN;
  constexpr int BM = 16 * FM * WGM;
  constexpr int BN = 16 * FN * WGN;
  constexpr int AF = BM / 16, BF = BN / 16;
  constexpr int FRD = AF + BF;                // operand fragments per k-step
  constexpr int FR = FRD + (ASC ? 1 : 0);     // 1 KiB DMA slots per k-step (+ the scales)
  // LDS-DMA instructions per wave per stage. When FR does not split evenly, the
  // surplus slots re-issue the last fragment (identical bytes to the identical
  // LDS slot), so every wave issues exactly L and one counted vmcnt fits all.
  constexpr int L = (FR + NW - 1) / NW;
  constexpr int STAGE = FR * 1024 * KSUB;     // KSUB 32-deep k sub-steps per stage
  constexpr int CS = BN * 2 + 16;
  constexpr int SMEM_PIPE = STAGES * STAGE;
  constexpr int SMEM_C = BM * CS;
  constexpr int SMEM = SMEM_PIPE > SMEM_C ? SMEM_PIPE : SMEM_C;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int nN = (a.NF * 16) / BN;
  const int OHW = a.OH * a.OW;
  // A scales (ASC): M tiles are cut per image so a tile has one scale vector
  constexpr bool per_img = ASC;
  const int mpi = per_img ? (OHW + BM - 1) / BM : 0;
  const int nM = per_img ? a.B * mpi : (a.M + BM - 1) / BM;
  // split-K: consecutive logical ids are the splits of one tile (same XCD: their partials meet in L2)
  const int S = a.ksplit > 1 ? a.ksplit : 1;
  const int tiles = nM * nN;
  const int wid = xcd_remap(blockIdx.x, tiles * S);
  const int ksid = wid % S, tile = wid / S;
  const int mi = tile / nN, ni = tile % nN;
  int m0 = mi * BM, mend = a.M;
  int bi = 0;
  if (per_img) {
    bi = mi / mpi;
    m0 = bi * OHW + (mi - bi * mpi) * BM;
    mend = (bi + 1) * OHW;
  }
  const int n0 = ni * BN;
  const int KT32 = (a.K >> 5) / S;           // 32-deep k steps of this split (host: divisible)
  const int kb = ksid * KT32;                 // its first k step
  const int KT = (KT32 + KSUB - 1) / KSUB;    // pipeline stages

  // per-lane source offsets of the fragments this wave stages
  long src[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int f = min(wave + i * NW, FR - 1);
    if (f < AF) {
      int m = m0 + f * 16 + (lane & 15);
      m = m < mend ? m : mend - 1;
      const int b = m / OHW, rem = m - b * OHW;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const long pix = ((long)b * a.H + (long)oh * a.stride) * a.W + (long)ow * a.stride;
      src[i] = pix * a.ldx + 8 * (lane >> 4);
    } else if (f < FRD) {
      const int nf = n0 / 16 + (f - AF);
      src[i] = ((long)nf * (a.K >> 5)) * 512 + lane * 8;
    } else {                                  // ASC: 8 lanes x 16 B = the k-step's 32 scales, repeated
      src[i] = (long)bi * a.ascale_ld + (lane & 7) * 4;
    }
  }

  // Issue stage t (k32 steps t*KSUB .. t*KSUB+KSUB-1). A sub-step past the end
  // of K re-issues the stage's first sub-step into its own slot (its MFMAs are
  // skipped), so every stage has exactly L*KSUB DMAs for the counted vmcnt.
  const int krot = a.krot && S == 1 ? (mi * 7) % KT32 : 0;
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int ks = 0; ks < KSUB; ++ks) {
      int k32 = t * KSUB + ks;
      if (k32 >= KT32) k32 = t * KSUB;
      k32 += krot;                            // uniform: rotated k order (0 = in order)
      k32 = (k32 >= KT32 ? k32 - KT32 : k32) + kb;
      long koff_a;
      if constexpr (MODE == 0) {
        koff_a = (long)k32 * 32;
      } else {
        const int k = k32 * 32;
        const int tap = k / a.cin, c0 = k - tap * a.cin;
        koff_a = ((long)(tap / 3) * a.W + (tap % 3)) * a.ldx + c0;
      }
      uint8_t* base = smem + buf * STAGE + ks * FR * 1024;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int f = min(wave + i * NW, FR - 1);
        if (f < AF) glds16(a.x + src[i] + koff_a, base + f * 1024);
        else if (!ASC || f < FRD) glds16(a.wp + src[i] + (long)k32 * 512, base + f * 1024);
        else glds16(a.ascale + src[i] + (long)k32 * 32, base + f * 1024);
      }
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
    // stages issued after t so far: min(KT-1, t+STAGES-2) - t
    const int after = min(KT - 1, t + STAGES - 2) - t;
    if (after >= 2) wait_vm_barrier<2 * L * KSUB>();
    else if (after == 1) wait_vm_barrier<L * KSUB>();
    else wait_vm_barrier<0>();
    if (t + STAGES - 1 < KT) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
#pragma unroll
    for (int ks = 0; ks < KSUB; ++ks) {
      if (KSUB > 1 && t * KSUB + ks >= KT32) break;
      const uint8_t* st = smem + (t % STAGES) * STAGE + ks * FR * 1024 + lane * 16;
      s16x8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *(const s16x8*)(st + (wm * FM + i) * 1024);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *(const s16x8*)(st + (AF + wn * FN + j) * 1024);
      if constexpr (ASC) {                    // this lane's 8 k (8 * (lane >> 4) ..): 32 bytes of scales
        const uint8_t* sc = st - lane * 16 + FRD * 1024 + (lane >> 4) * 32;
        const f32x4 s0 = *(const f32x4*)sc, s1 = *(const f32x4*)(sc + 16);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = pipe_ascale8(af[i], s0, s1);
      }
      // raise this wave's issue priority while it streams MFMAs (guide §5 T-setprio:
      // the other waves' glds issue / barrier arrival no longer interleave into the
      // MFMA run)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = E::mfma(bf[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  wait_vm_barrier<0>();

  if (S > 1) {
    // fp32 partial of this split, fragment-linear (each wave writes 1 KiB per fragment)
    float4* const part = (float4*)a.ws + (long)tile * (BM * BN / 4);
    const long sstride = (long)tiles * (BM * BN / 4);
    auto pidx = [&](int i, int j) { return ((wave * FM + i) * FN + j) * 64 + lane; };
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        part[ksid * sstride + pidx(i, j)] = (float4){acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
    // publish (every storing wave drains, barrier, agent release, count) and elect the last split
    // the election flag lives in the (idle) pipeline LDS: a second __shared__ object can make hipcc
    // wait vmcnt(0) before every k-step's first LDS read (cdna_hip_programming.md §5 trap (a))
    int& s_last = *(int*)smem;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const int old = __hip_atomic_fetch_add(a.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == S - 1;
      if (s_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const bool last = s_last;
    __syncthreads();                          // every thread read the flag before the C tile reuses the LDS
    if (!last) return;                        // uniform: the whole workgroup leaves
    // every split (this one included) stored its partial: sum them in split order, so the
    // fp32 result does not depend on which split arrived last (bit-identical replays)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float4 v = part[sp * sstride + pidx(i, j)];
          acc[i][j][0] += v.x; acc[i][j][1] += v.y; acc[i][j][2] += v.z; acc[i][j][3] += v.w;
        }
    }
  }

  // epilogue: bias + ReLU -> bf16 C tile in LDS -> (+residual) 16-byte stores
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
      *(u32x2*)(smem + ml * CS + nl * 2) = (u32x2){E::pack(v0, v1), E::pack(v2, v3)};
    }
  }
  // residual rows (ResNet conv3, ViT out_proj / mlp.3): loaded now, with the accumulators already in
  // LDS, instead of inside the store pass where each load waited behind the earlier stores
  // (in-order vmcnt; the same change in sepconv_ws.hip: profiles/middle_flow_r6.txt section 7).
  // Interleaved bench pairs: ResNet-50 +1.6 %, ViT-B/16 bf16 +0.7 % (profiles/epilogue_residual_r6.txt)
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
    if (c < BM * CPR && m < mend && n < a.nstore)
      epi_store_r<DT>(a, m, n, *(const u32x4*)(smem + r * CS + cc * 16), rres[it]);
  }
}

// (FM, FN, WGM, WGN, STAGES); ids are offset by PIPE_CFG_BASE in the host table.
#define KDL_PIPE_CONFIGS(X) \
  X(0, 4, 4, 2, 2, 4, 1)    \
  X(1, 2, 4, 2, 2, 4, 1)    \
  X(2, 4, 2, 2, 2, 4, 1)    \
  X(3, 2, 2, 2, 2, 4, 1)    \
  X(4, 8, 2, 1, 4, 4, 1)    \
  X(5, 4, 4, 1, 4, 4, 1)    \
  X(6, 4, 8, 2, 2, 3, 1)    \
  X(7, 8, 4, 1, 4, 3, 1)    \
  X(8, 3, 6, 2, 4, 3, 1)    \
  X(9, 6, 3, 2, 4, 3, 1)    \
  X(10, 3, 3, 2, 4, 3, 1)   \
  X(11, 4, 4, 2, 2, 3, 1)   \
  X(12, 2, 6, 2, 4, 3, 1)   \
  X(13, 4, 2, 2, 4, 3, 1)   \
  X(14, 3, 3, 2, 4, 2, 2)   \
  X(15, 6, 3, 2, 4, 2, 2)   \
  X(16, 4, 2, 2, 4, 2, 2)   \
  X(17, 4, 4, 2, 2, 3, 2)   \
  X(18, 3, 3, 2, 4, 3, 2)   \
  X(19, 4, 4, 2, 2, 2, 4)   \
  X(20, 2, 4, 2, 2, 3, 2)   \
  X(21, 4, 2, 2, 2, 3, 2)   \
  X(22, 6, 3, 2, 4, 5, 1)   \
  X(23, 3, 6, 2, 4, 5, 1)   \
  X(24, 3, 3, 2, 4, 6, 1)   \
  X(25, 4, 2, 2, 4, 6, 1)   \
  X(26, 6, 3, 2, 4, 3, 2)    \
  X(27, 5, 2, 2, 4, 3, 2)   \
  X(28, 5, 3, 2, 4, 3, 2)   \
  X(29, 5, 4, 2, 4, 2, 2)   \
  X(30, 5, 2, 2, 4, 4, 1)   \
  X(45, 5, 2, 2, 4, 3, 1)   \
  X(46, 5, 3, 2, 4, 3, 1)   \
  X(47, 5, 4, 2, 4, 3, 1)
// 45-47: 160-row tiles (256x256 / 256x192 / 192x256 tiles were tried in round 3 and lost:
// profiles/vit_gemm_tiles256_r3.txt). At the ViT-B/16 shapes (M = 32 x 197 =
// 6304 rows) they fill 256 CUs in whole waves: out_proj / mlp.3 (N 768) 160x128 -> 240
// tiles; QKV (N 2304) 160x192 -> 480; mlp.0 (N 3072) 160x256 -> 480 (vs 192x192: 396 / 528)

template <int MODE, int FM, int FN, int WGM, int WGN, int ST, int KS, int DT = 0, bool ASC = false>
static hipError_t launch_pipe_cfg(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  if ((a.NF * 16) % BN != 0) return hipErrorInvalidValue;
  constexpr bool per_img = ASC;
  if (per_img && (a.M != a.B * a.OH * a.OW || a.B <= 0)) return hipErrorInvalidValue;
  if (ASC && (!a.ascale || a.ascale_ld < a.K || a.ascale_ld % 4 != 0)) return hipErrorInvalidValue;
  const int nM = per_img ? a.B * ((a.OH * a.OW + BM - 1) / BM) : (a.M + BM - 1) / BM, nN = (a.NF * 16) / BN;
  const int S = a.ksplit > 1 ? a.ksplit : 1;
  if (S > 1 && ((a.K / 32) % S != 0 || !a.ws || !a.cnt || per_img || S > 16)) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_pipe_kernel<MODE, FM, FN, WGM, WGN, ST, KS, DT, ASC>), dim3(nM * nN * S),
                     dim3(64 * WGM * WGN), 0, s, a);
  return hipGetLastError();
}

template <int MODE, int DT, bool ASC = false>
static hipError_t launch_pipe_mode(int cfg, const ConvGemmArgs& a, hipStream_t s) {
  switch (cfg) {
#define KDL_PCASE(id, fm, fn, wgm, wgn, st, ks) \
  case id: return launch_pipe_cfg<MODE, fm, fn, wgm, wgn, st, ks, DT, ASC>(a, s);
    KDL_PIPE_CONFIGS(KDL_PCASE)
#undef KDL_PCASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t gemm_pipe(int mode, int cfg, const ConvGemmArgs& args, hipStream_t s) {
  if (args.K % 32 != 0 || args.M <= 0 || args.dt < 0 || args.dt > 1) return hipErrorInvalidValue;
  static const int env_krot = [] { const char* e = getenv("KDL_PIPE_KROT"); return e ? atoi(e) : -1; }();
  ConvGemmArgs a = args;
  if (env_krot >= 0) a.krot = env_krot;
  if (a.ascale) {                             // A-operand channel scales: bf16 pointwise, whole K per tile
    if (mode != 0 || a.dt != 0 || a.ksplit > 1) return hipErrorInvalidValue;
    return launch_pipe_mode<0, 0, true>(cfg, a, s);
  }
  if (mode == 0) return a.dt ? launch_pipe_mode<0, 1>(cfg, a, s) : launch_pipe_mode<0, 0>(cfg, a, s);
  if (mode == 1) return a.dt ? launch_pipe_mode<1, 1>(cfg, a, s) : launch_pipe_mode<1, 0>(cfg, a, s);
  return hipErrorInvalidValue;
}

int gemm_pipe_config(int cfg, int* bm, int* bn, int* threads) {
  switch (cfg) {
#define KDL_PINFO(id, fm, fn, wgm, wgn, st, ks) \
  case id: *bm = 16 * fm * wgm; *bn = 16 * fn * wgn; *threads = 64 * wgm * wgn; return 0;
    KDL_PIPE_CONFIGS(KDL_PINFO)
#undef KDL_PINFO
    default: return -1;
  }
}

}  // namespace kdl
