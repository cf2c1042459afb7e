// EfficientNet MBConv front half in ONE kernel: expand 1x1 (+BN+SiLU) -> KxK/S depthwise
// (+BN+SiLU) -> squeeze-excite pool + fc1 partials (the 600x600
// large-activation path). The expanded tensor E (6x the block input, the largest
// activations of the network: 415 MB per block at 150x150x288, batch 32) never reaches
// HBM -- unfused, the expand conv writes it and the depthwise reads it back.
//
// A workgroup owns one spatial output tile (RB x TW) of one image for ALL expanded channels:
//   * its input patch ((RB-1)S+K) x ((TW-1)S+K) x cin is staged ONCE into LDS, fragment-linear
//     ([fragment][k-step][lane][16 B]: what one LDS-DMA wave instruction writes is what
//     ds_read_b128 of the MFMA operand reads); pixels outside the image are staged as zeros;
//   * per 32-channel block cb: the expand GEMM (M = patch pixels, N = 32, K = cin) on the
//     matrix cores out of the resident patch, + bias + SiLU, forced to 0 outside the image
//     (the depthwise zero padding applies to E), bf16 into an LDS E block [pixel][32 ch];
//     then the depthwise on the VALU from the E block (a register window slides along each
//     output row segment, as dwk_kernel), + bias + SiLU -> D in HBM; the channel sums of the
//     stored values -> this tile's fc1 partial (fc1 is linear in the mean), accumulated over
//     the blocks and written once per tile.
//   * each block's parameters (expand fragments, depthwise weights, biases, fc1 slice) are
//     ONE contiguous host-packed blob, streamed through a MB_RING-deep LDS ring MB_RING-1
//     blocks ahead of use.
// Roles: waves 0-3 compute and store; wave 4 only moves data, so the compute waves never wait
// on vmcnt (their stores are never drained) and the DMA wave's counted wait stays exact; every
// barrier is a raw s_barrier. History (profiles/entry_flow_r2.txt): the first cut fetched each
// block's parameters one block ahead from four scattered places (a memory round trip per block,
// 2x slower than expand conv + dwk); the second gave each workgroup one channel block over many
// tiles and re-read every input patch per block (1.1 GB of L2->LDS traffic per f2 layer).
#include "common.h"
#include "launch.h"

#include <algorithm>

namespace kdl {

constexpr int MB_CB = 32;             // expanded channels per block
constexpr int MB_NPMAX = 576;         // patch pixels (36 fragments: 9 per compute wave)
constexpr int MB_FPW = MB_NPMAX / 64; // fragments per compute wave
constexpr int MB_KTMAX = 5;           // cin <= 160
constexpr int MB_CSMAX = 64;          // squeeze units
constexpr int MB_RING = 4;            // parameter blobs in LDS

__device__ __attribute__((aligned(16))) uint8_t mb_zeros[64];

__device__ __forceinline__ float mb_silu(float v) { return fast_silu(v); }

__device__ __forceinline__ void mb_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void mb_wait_vm(int n) {
  // vmcnt needs an immediate: dispatch over the possible counts
  switch (n) {
#define MBW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MBW(1) MBW(2) MBW(3) MBW(4) MBW(5) MBW(6) MBW(7) MBW(8) MBW(9) MBW(10) MBW(11) MBW(12)
    MBW(13) MBW(14) MBW(15) MBW(16) MBW(17) MBW(18) MBW(19) MBW(20) MBW(21) MBW(22) MBW(23) MBW(24)
    MBW(25) MBW(26) MBW(27) MBW(28) MBW(29) MBW(30) MBW(31) MBW(32) MBW(33) MBW(34) MBW(35) MBW(36)
    MBW(37) MBW(38) MBW(39) MBW(40) MBW(41) MBW(42) MBW(43) MBW(44) MBW(45) MBW(46) MBW(47) MBW(48)
    MBW(49) MBW(50) MBW(51) MBW(52) MBW(53) MBW(54) MBW(55) MBW(56) MBW(57) MBW(58) MBW(59) MBW(60)
    MBW(61) MBW(62) MBW(63)
#undef MBW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Parameter blob of one channel block (host: kdl/engine/efficientnet.py mbconv_blobs), bytes:
//   [0, 2 KT KiB)             expand B fragments (2cb + j, t) at (j KT + t) KiB, lane-linear
//   [WD, WD + K K 128)        depthwise weights [tap][32] fp32
//   [BI, BI + 256)            biases: expand [32] fp32, depthwise [32] fp32
//   [W1, W1 + Cs 128)         fc1 slice [Cs][32] fp32
// padded to whole KiB.
__host__ __device__ inline int mb_wd_off(int KT) { return 2 * KT * 1024; }
__host__ __device__ inline int mb_bias_off(int KT, int K) { return mb_wd_off(KT) + K * K * 128; }
__host__ __device__ inline int mb_w1_off(int KT, int K) { return mb_bias_off(KT, K) + 256; }
__host__ __device__ inline int mb_blob_kib(int KT, int K, int Cs) { return (mb_w1_off(KT, K) + Cs * 128 + 1023) / 1024; }

static size_t mb_smem(int NP, int KT, int K, int Cs) {
  const size_t nfr = (size_t)((NP + 15) / 16);
  return nfr * KT * 1024 + (size_t)MB_RING * mb_blob_kib(KT, K, Cs) * 1024 + (size_t)NP * 64 +
         (16 * 8 + MB_CB + MB_CSMAX) * 4;
}

template <int K, int S, int SEG>
__global__ __launch_bounds__(320) void mbconv_ed_kernel(MbedArgs a, int RB, int TW) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const int PR = (RB - 1) * S + K, PC = (TW - 1) * S + K, NP = PR * PC;
  const int NFR = (NP + 15) >> 4;
  const int KT = a.cin >> 5;
  const int NB = mb_blob_kib(KT, K, a.Cs);                       // DMA instructions per blob
  uint8_t* const xp = sm;                                        // [NFR][KT][64][16 B]
  uint8_t* const ring = xp + NFR * KT * 1024;                    // MB_RING blobs
  uint8_t* const ep = ring + MB_RING * NB * 1024;                // [NP][32] bf16
  float* const red = (float*)(ep + NP * 64);                     // [16][8]
  float* const csum = red + 16 * 8;                              // [32]
  float* const hacc = csum + MB_CB;                              // [Cs]

  const int nbands = (a.OH + RB - 1) / RB, ncolt = (a.OW + TW - 1) / TW;
  int bid = blockIdx.x;
  const int ct = bid % ncolt;
  bid /= ncolt;
  const int band = bid % nbands;
  const int b = bid / nbands;
  const int h0 = band * RB, c0 = ct * TW;
  const int ih0 = h0 * S - a.pad, iw0 = c0 * S - a.pad;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = a.C / MB_CB;

  if (wave == 4) {
    // ================= the data mover
    int ib = 0;                                  // next blob to issue (clamped: re-issues the last)
    auto issue_blob = [&]() {
      const uint8_t* src = (const uint8_t*)a.blob + (long)ib * NB * 1024 + lane * 16;
      uint8_t* dst = ring + (ib % MB_RING) * NB * 1024;
      for (int i = 0; i < NB; ++i) glds16(src + i * 1024, dst + i * 1024);
      if (ib + 1 < ncb) ++ib;
    };
    {
      const int p16 = lane & 15, kb = lane >> 4;
      for (int f = 0; f < NFR; ++f) {
        const int p = f * 16 + p16;
        const int pr = p / PC, pc = p - pr * PC;
        const int ih = ih0 + pr, iw = iw0 + pc;
        const bool in = p < NP && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const uint16_t* src = a.x + (((long)b * a.H + ih) * a.W + iw) * a.ldx + kb * 8;
        for (int t = 0; t < KT; ++t)
          glds16(in ? (const void*)(src + t * 32) : (const void*)mb_zeros, xp + (f * KT + t) * 1024);
      }
    }
    for (int p = 0; p < MB_RING - 1; ++p) issue_blob();
    mb_wait_vm((MB_RING - 2) * NB);              // patch + blob 0 landed
    mb_barrier();                                // P0
    for (int cb = 0; cb < ncb; ++cb) {
      mb_barrier();                              // E1: E block of cb written
      mb_barrier();                              // E2: depthwise done
      mb_barrier();                              // E3: csum ready
      // blobs 0 .. cb + MB_RING - 2 are issued; blob cb+1 (used right after E4) must have
      // landed, the MB_RING - 3 younger ones may stay in flight
      mb_wait_vm((MB_RING - 3) * NB);
      mb_barrier();                              // E4
      issue_blob();                              // blob cb + MB_RING - 1 into the slot of blob cb - 1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ================= compute waves 0-3
  const int p16 = lane & 15;
  const int quad = lane >> 4, col = lane & 15;
  uint32_t inimg = 0;                            // this lane's fragment rows inside the image
#pragma unroll
  for (int i = 0; i < MB_FPW; ++i) {
    const int p = (wave + 4 * i) * 16 + p16;
    const int pr = p / PC, pc = p - pr * PC;
    if (p < NP && (unsigned)(ih0 + pr) < (unsigned)a.H && (unsigned)(iw0 + pc) < (unsigned)a.W) inimg |= 1u << i;
  }
  for (int j = tid; j < a.Cs; j += 256) hacc[j] = 0.f;
  const int ic = tid & 3;                        // depthwise: fixed 8-channel chunk per thread
  const int nseg = (TW + SEG - 1) / SEG;
  const int nitems = 4 * RB * nseg;
  mb_barrier();                                  // P0

  for (int cb = 0; cb < ncb; ++cb) {
    const uint8_t* pb = ring + (cb % MB_RING) * NB * 1024;
    const float* bias = (const float*)(pb + mb_bias_off(KT, K));  // [0,32) expand, [32,64) depthwise
    // ---- expand GEMM for channels [32 cb, 32 cb + 32) of every patch pixel
    f32x4 acc[MB_FPW][2];
#pragma unroll
    for (int i = 0; i < MB_FPW; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < MB_KTMAX; ++t) {
      if (t < KT) {
        const s16x8 b0 = *(const s16x8*)(pb + t * 1024 + lane * 16);
        const s16x8 b1 = *(const s16x8*)(pb + (KT + t) * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < MB_FPW; ++i) {
          const int f = wave + 4 * i;
          if (f < NFR && !(a.abl & 2)) {
            const s16x8 af = *(const s16x8*)(xp + (f * KT + t) * 1024 + lane * 16);
            acc[i][0] = mfma16(b0, af, acc[i][0]);
            acc[i][1] = mfma16(b1, af, acc[i][1]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = j * 16 + 4 * quad;          // channel within the block
      const float4 bz = *(const float4*)(bias + cl);
#pragma unroll
      for (int i = 0; i < MB_FPW; ++i) {
        const int f = wave + 4 * i;
        const int p = f * 16 + col;
        if (f < NFR && p < NP) {
          u32x2 o = {pack_bf16(mb_silu(acc[i][j][0] + bz.x), mb_silu(acc[i][j][1] + bz.y)),
                     pack_bf16(mb_silu(acc[i][j][2] + bz.z), mb_silu(acc[i][j][3] + bz.w))};
          if (!((inimg >> i) & 1u)) o = (u32x2){0u, 0u};
          *(u32x2*)(ep + p * 64 + cl * 2) = o;
        }
      }
    }
    mb_barrier();                                // E1

    // ---- depthwise from the E block: item = (chunk ic, output row, SEG-column segment)
    const float* wsm = (const float*)(pb + mb_wd_off(KT));
    const float4 d0 = *(const float4*)(bias + MB_CB + ic * 8);
    const float4 d1 = *(const float4*)(bias + MB_CB + ic * 8 + 4);
    const float dbias[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
    float psum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int it = (a.abl & 1) ? nitems : tid; it < nitems; it += 256) {
      const int tt = it >> 2;
      const int sg = tt % nseg, ir = tt / nseg;
      const int w0 = sg * SEG;
      if (h0 + ir >= a.OH || c0 + w0 >= a.OW) continue;
      f32x2 dacc[SEG][4];
#pragma unroll
      for (int o = 0; o < SEG; ++o)
#pragma unroll
        for (int d = 0; d < 4; ++d) dacc[o][d] = (f32x2){0.f, 0.f};
#pragma unroll 1
      for (int dy = 0; dy < K; ++dy) {
        f32x2 wt[K][4];
#pragma unroll
        for (int dx = 0; dx < K; ++dx) {
          const float* wp = wsm + (dy * K + dx) * MB_CB + ic * 8;
          const float4 p = *(const float4*)wp;
          const float4 q4 = *(const float4*)(wp + 4);
          wt[dx][0] = (f32x2){p.x, p.y};
          wt[dx][1] = (f32x2){p.z, p.w};
          wt[dx][2] = (f32x2){q4.x, q4.y};
          wt[dx][3] = (f32x2){q4.z, q4.w};
        }
        const uint8_t* rowp = ep + ((ir * S + dy) * PC) * 64 + ic * 16;
#pragma unroll
        for (int j = 0; j < (SEG - 1) * S + K; ++j) {
          const int lc = min(w0 * S + j, PC - 1);   // clamped reads only feed outputs not stored
          const u32x4 v = *(const u32x4*)(rowp + lc * 64);
          f32x2 xv[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) xv[d] = (f32x2){bf_lo(v[d]), bf_hi(v[d])};
#pragma unroll
          for (int o = 0; o < SEG; ++o) {
            const int dx = j - o * S;
            if (dx >= 0 && dx < K) {
#pragma unroll
              for (int d = 0; d < 4; ++d) dacc[o][d] = __builtin_elementwise_fma(xv[d], wt[dx][d], dacc[o][d]);
            }
          }
        }
      }
      uint16_t* yb = a.y + (((long)b * a.OH + h0 + ir) * a.OW + c0 + w0) * a.C + cb * MB_CB + ic * 8;
      const int lim = min(SEG, min(TW - w0, a.OW - c0 - w0));
#pragma unroll
      for (int o = 0; o < SEG; ++o) {
        if (o < lim) {
          u32x4 out;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            out[d] = pack_bf16(mb_silu(dacc[o][d][0] + dbias[2 * d]), mb_silu(dacc[o][d][1] + dbias[2 * d + 1]));
            psum[2 * d] += bf_lo(out[d]);        // the SE pool sees the stored (bf16) values
            psum[2 * d + 1] += bf_hi(out[d]);
          }
          *(u32x4*)(yb + (long)o * a.C) = out;
        }
      }
    }
    // channel sums: butterfly over the lanes of one chunk (lane % 4), then the waves via LDS
#pragma unroll
    for (int off = 4; off < 64; off <<= 1)
#pragma unroll
      for (int d = 0; d < 8; ++d) psum[d] += __shfl_xor(psum[d], off);
    if (lane < 4) {
#pragma unroll
      for (int d = 0; d < 8; ++d) red[(wave * 4 + lane) * 8 + d] = psum[d];
    }
    mb_barrier();                                // E2
    if (tid < MB_CB) {
      const int rc = tid >> 3, d = tid & 7;
      csum[tid] = red[rc * 8 + d] + red[(4 + rc) * 8 + d] + red[(8 + rc) * 8 + d] + red[(12 + rc) * 8 + d];
    }
    mb_barrier();                                // E3
    {
      // fc1 partial: unit j = tid / 8, quarter q8 = tid % 8 (4 channels each), accumulated
      const float* w1s = (const float*)(pb + mb_w1_off(KT, K));   // [Cs][32]
      const int q8 = tid & 7;
      for (int j0 = 0; j0 < a.Cs; j0 += 32) {
        const int j = j0 + (tid >> 3);
        float h = 0.f;
        if (j < a.Cs) {
          const float4 w = *(const float4*)(w1s + j * MB_CB + q8 * 4);
          const float4 c = *(const float4*)(csum + q8 * 4);
          h = w.x * c.x + w.y * c.y + w.z * c.z + w.w * c.w;
        }
        h += __shfl_xor(h, 1);
        h += __shfl_xor(h, 2);
        h += __shfl_xor(h, 4);
        if (q8 == 0 && j < a.Cs) hacc[j] += h;
      }
    }
    mb_barrier();                                // E4: E block, red, csum and blob cb free
  }
  const int part = band * ncolt + ct;
  const int nparts = nbands * ncolt;
  for (int j = tid; j < a.Cs; j += 256) a.pool[((long)b * nparts + part) * a.Cs + j] = hacc[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int mbconv_blob_bytes(int cin, int K, int Cs) { return mb_blob_kib(cin / 32, K, Cs) * 1024; }

// Largest tile (square where the map allows) whose patch fits MB_NPMAX pixels and whose LDS
// keeps two workgroups per CU (<= 78 KiB), else one (<= 150 KiB); ntiles = SE partials per
// image; 0 = not applicable (cin > 160 or Cs > 64: the unfused expand conv + dwk run).
void mbconv_ed_tiles(const MbedArgs& a, int* rb, int* tw, int* ntiles) {
  *rb = *tw = *ntiles = 0;
  if (a.cin % 32 != 0 || a.cin <= 0 || a.cin / 32 > MB_KTMAX || a.C % MB_CB != 0 || a.Cs > MB_CSMAX ||
      a.Cs <= 0)
    return;
  const int KT = a.cin / 32;
  for (int budget : {78 * 1024, 150 * 1024}) {
    for (int r = std::min(a.OH, 32); r >= 4; --r) {
      const int t = std::min(r, a.OW);
      const int PR = (r - 1) * a.S + a.K, PC = (t - 1) * a.S + a.K;
      if (PR * PC > MB_NPMAX || mb_smem(PR * PC, KT, a.K, a.Cs) > (size_t)budget) continue;
      // two workgroups per CU only pays if the tile stays reasonably large
      if (budget < 150 * 1024 && r < std::min(12, a.OH)) break;
      *rb = r;
      *tw = t;
      *ntiles = ((a.OH + r - 1) / r) * ((a.OW + t - 1) / t);
      return;
    }
  }
}

hipError_t mbconv_ed(const MbedArgs& a, hipStream_t s) {
  if (a.B <= 0 || (a.K != 3 && a.K != 5) || (a.S != 1 && a.S != 2) || a.pad != (a.K - 1) / 2 || a.ldx < a.cin ||
      !a.blob)
    return hipErrorInvalidValue;
  int RB, TW, nt;
  mbconv_ed_tiles(a, &RB, &TW, &nt);
  if (nt == 0) return hipErrorInvalidValue;
  const size_t smem = mb_smem(((RB - 1) * a.S + a.K) * ((TW - 1) * a.S + a.K), a.cin / 32, a.K, a.Cs);
  const dim3 grid((unsigned)((long)a.B * nt)), block(320);
  if (a.K == 3 && a.S == 1) hipLaunchKernelGGL((mbconv_ed_kernel<3, 1, 4>), grid, block, smem, s, a, RB, TW);
  else if (a.K == 3 && a.S == 2) hipLaunchKernelGGL((mbconv_ed_kernel<3, 2, 4>), grid, block, smem, s, a, RB, TW);
  else if (a.K == 5 && a.S == 1) hipLaunchKernelGGL((mbconv_ed_kernel<5, 1, 4>), grid, block, smem, s, a, RB, TW);
  else hipLaunchKernelGGL((mbconv_ed_kernel<5, 2, 4>), grid, block, smem, s, a, RB, TW);
  return hipGetLastError();
}

}  // namespace kdl
