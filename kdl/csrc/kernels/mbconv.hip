// EfficientNet MBConv front half in ONE kernel: expand 1x1 (+BN+SiLU) -> KxK/S depthwise
// (+BN+SiLU) -> squeeze-excite pool + fc1 partials (the 600x600
// large-activation path). The expanded tensor E (6x the block input, the largest
// activations of the network: 415 MB per block at 150x150x288, batch 32) never reaches
// HBM -- unfused, the expand conv writes it and the depthwise reads it back.
//
// A workgroup owns one spatial output tile (RB x TW) of one image for ALL expanded
// channels, in 32-channel blocks cb:
//   * its input patch ((RB-1)S+K) x ((TW-1)S+K) pixels x cin is staged ONCE into LDS,
//     fragment-linear ([fragment][k-step][lane][16 B]: what one LDS-DMA wave instruction
//     writes is what ds_read_b128 of the MFMA operand reads, conflict-free); pixels
//     outside the image are staged as zeros;
//   * expand GEMM of block cb (M = patch pixels, N = 32, K = cin) on the matrix cores out
//     of that resident patch, + bias + SiLU, forced to 0 outside the image (the depthwise
//     zero padding applies to E), bf16 into an LDS E block [pixel][32 ch];
//   * the depthwise on the VALU from the E block (a register window slides along each
//     output row segment, as dwk_kernel), + bias + SiLU -> D in HBM; the channel sums of
//     the stored values -> this tile's fc1 partial (fc1 is linear in the mean),
//     accumulated over the blocks and written once per tile.
// Roles: waves 0-3 compute and store; wave 4 only moves data (LDS-DMA of the patch and,
// double-buffered, of block cb+1's expand weights, depthwise weights, biases and fc1
// slice while block cb computes). The compute waves issue no global load at all, so
// their stores are never drained by a vmcnt wait; every barrier is a raw s_barrier.
#include "common.h"
#include "launch.h"

#include <algorithm>

namespace kdl {

constexpr int MB_CB = 32;             // expanded channels per block
constexpr int MB_NPMAX = 576;         // patch pixels (36 fragments: 9 per compute wave)
constexpr int MB_FPW = MB_NPMAX / 64; // fragments per compute wave
constexpr int MB_KTMAX = 5;           // cin <= 160
constexpr int MB_CSMAX = 64;          // squeeze units

__device__ __attribute__((aligned(16))) uint8_t mb_zeros[64];

__device__ __forceinline__ float mb_silu(float v) { return v / (1.f + __expf(-v)); }

__device__ __forceinline__ void mb_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void mb_barrier_vm() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// per-block parameter buffer (double-buffered): expand B fragments | depthwise weights |
// biases (expand, depthwise) | fc1 slice [Cs][32]
struct MbLayout {
  int KT, K, Cs;
  __host__ __device__ int pb_b() const { return 0; }
  __host__ __device__ int pb_wd() const { return 2 * KT * 1024; }
  __host__ __device__ int pb_bias() const { return pb_wd() + ((K * K + 7) / 8) * 1024; }
  __host__ __device__ int pb_w1() const { return pb_bias() + 1024; }
  __host__ __device__ int pb_bytes() const { return pb_w1() + ((Cs + 7) / 8) * 1024; }
};

static size_t mb_smem(int NP, int KT, int K, int Cs) {
  const MbLayout L{KT, K, Cs};
  const size_t nfr = (size_t)((NP + 15) / 16);
  return nfr * KT * 1024 + 2 * (size_t)L.pb_bytes() + (size_t)NP * 64 + (256 * 8 + MB_CB + MB_CSMAX) * 4;
}

template <int K, int S, int SEG>
__global__ __launch_bounds__(320) void mbconv_ed_kernel(MbedArgs a, int RB, int TW) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  const int PR = (RB - 1) * S + K, PC = (TW - 1) * S + K, NP = PR * PC;
  const int NFR = (NP + 15) >> 4;
  const int KT = a.cin >> 5;
  const MbLayout L{KT, K, a.Cs};
  uint8_t* const xp = sm;                                        // [NFR][KT][64][16 B]
  uint8_t* const pbuf = xp + NFR * KT * 1024;                    // 2 x per-block parameters
  uint8_t* const ep = pbuf + 2 * L.pb_bytes();                   // [NP][32] bf16
  float* const red = (float*)(ep + NP * 64);                     // [256][8]
  float* const csum = red + 256 * 8;                             // [32]
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
    auto params = [&](int cb, uint8_t* dst) {
      // expand weights: N fragments 2cb, 2cb+1 for every k-step
      for (int j = 0; j < 2; ++j)
        for (int t = 0; t < KT; ++t)
          glds16(a.we + (((long)(2 * cb + j) * KT + t) * 64 + lane) * 8, dst + L.pb_b() + (j * KT + t) * 1024);
      // depthwise weights [tap][32] fp32: 8 lanes (128 B) per tap
      for (int i = 0; i < (K * K + 7) / 8; ++i) {
        const int tap = min(i * 8 + (lane >> 3), K * K - 1);
        glds16(a.wd + (long)tap * a.C + cb * MB_CB + (lane & 7) * 4, dst + L.pb_wd() + i * 1024);
      }
      // biases: lanes 0-7 expand, 8-15 depthwise (the rest duplicate lane 15's piece)
      {
        const int l = min(lane, 15);
        const float* src = l < 8 ? a.be + cb * MB_CB + l * 4 : a.bd + cb * MB_CB + (l - 8) * 4;
        glds16(src, dst + L.pb_bias());
      }
      // fc1 slice [Cs][32]: 8 lanes per squeeze unit
      for (int i = 0; i < (a.Cs + 7) / 8; ++i) {
        const int j = min(i * 8 + (lane >> 3), a.Cs - 1);
        glds16(a.w1 + (long)j * a.C + cb * MB_CB + (lane & 7) * 4, dst + L.pb_w1() + i * 1024);
      }
    };
    // input patch, fragment-linear
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
    params(0, pbuf);
    mb_barrier_vm();                             // P0: patch + block 0 parameters landed
    for (int cb = 0; cb < ncb; ++cb) {
      if (cb + 1 < ncb) params(cb + 1, pbuf + ((cb + 1) & 1) * L.pb_bytes());
      mb_barrier();                              // E1: E block written
      mb_barrier();                              // E2: depthwise done, channel partials in red
      mb_barrier();                              // E3: csum ready
      mb_barrier_vm();                           // E4: fc1 accumulated; block cb+1 parameters landed
    }
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
    const int ih = ih0 + pr, iw = iw0 + pc;
    if (p < NP && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) inimg |= 1u << i;
  }
  for (int j = tid; j < a.Cs; j += 256) hacc[j] = 0.f;
  const int ic = tid & 3;                        // depthwise: fixed 8-channel chunk per thread
  const int nseg = (TW + SEG - 1) / SEG;
  const int nitems = 4 * RB * nseg;
  mb_barrier();                                  // P0

  for (int cb = 0; cb < ncb; ++cb) {
    const uint8_t* pb = pbuf + (cb & 1) * L.pb_bytes();
    const float* bias = (const float*)(pb + L.pb_bias());       // [0,32) expand, [32,64) depthwise
    // ---- expand GEMM for channels [32 cb, 32 cb + 32) of every patch pixel
    f32x4 acc[MB_FPW][2];
#pragma unroll
    for (int i = 0; i < MB_FPW; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < MB_KTMAX; ++t) {
      if (t < KT) {
        const s16x8 b0 = *(const s16x8*)(pb + L.pb_b() + t * 1024 + lane * 16);
        const s16x8 b1 = *(const s16x8*)(pb + L.pb_b() + (KT + t) * 1024 + lane * 16);
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
    const float* wsm = (const float*)(pb + L.pb_wd());
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
          const float4 q = *(const float4*)(wp + 4);
          wt[dx][0] = (f32x2){p.x, p.y};
          wt[dx][1] = (f32x2){p.z, p.w};
          wt[dx][2] = (f32x2){q.x, q.y};
          wt[dx][3] = (f32x2){q.z, q.w};
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
    // channel sums of the block: butterfly over the lanes of one chunk (lane % 4), then the
    // four waves' partials through LDS (a serial LDS loop here cost ~6k cycles per block)
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
      // fc1 partial: thread (unit j = tid / 8, quarter q = tid % 8) does 4 channels, then a
      // butterfly over the 8 quarters
      const float* w1s = (const float*)(pb + L.pb_w1());        // [Cs][32]
      const int q = tid & 7;
      for (int j0 = 0; j0 < a.Cs; j0 += 32) {
        const int j = j0 + (tid >> 3);
        float h = 0.f;
        if (j < a.Cs) {
          const float4 w = *(const float4*)(w1s + j * MB_CB + q * 4);
          const float4 c = *(const float4*)(csum + q * 4);
          h = w.x * c.x + w.y * c.y + w.z * c.z + w.w * c.w;
        }
        h += __shfl_xor(h, 1);
        h += __shfl_xor(h, 2);
        h += __shfl_xor(h, 4);
        if (q == 0 && j < a.Cs) hacc[j] += h;
      }
    }
    mb_barrier();                                // E4 (E block, red, csum and pb[cb & 1] free again)
  }
  const int part = band * ncolt + ct;
  const int nparts = nbands * ncolt;
  for (int j = tid; j < a.Cs; j += 256) a.pool[((long)b * nparts + part) * a.Cs + j] = hacc[j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Largest tile (square where the map allows) whose patch fits MB_NPMAX pixels and whose LDS
// keeps two workgroups per CU (<= 78 KiB); ntiles = 0: not applicable (cin > 160 or too
// many squeeze units: the unfused expand conv + dwk path is used).
void mbconv_ed_tiles(const MbedArgs& a, int* rb, int* tw, int* ntiles) {
  *rb = *tw = *ntiles = 0;
  if (a.cin % 32 != 0 || a.cin / 32 > MB_KTMAX || a.cin <= 0 || a.C % MB_CB != 0 || a.Cs > MB_CSMAX || a.Cs <= 0)
    return;
  const int KT = a.cin / 32;
  for (int r = std::min(a.OH, 32); r >= 2; --r) {
    const int t = std::min(r, a.OW);
    const int PR = (r - 1) * a.S + a.K, PC = (t - 1) * a.S + a.K;
    if (PR * PC > MB_NPMAX) continue;
    if (mb_smem(PR * PC, KT, a.K, a.Cs) > 78 * 1024) continue;
    *rb = r;
    *tw = t;
    *ntiles = ((a.OH + r - 1) / r) * ((a.OW + t - 1) / t);
    return;
  }
}

hipError_t mbconv_ed(const MbedArgs& a, hipStream_t s) {
  if (a.B <= 0 || (a.K != 3 && a.K != 5) || (a.S != 1 && a.S != 2) || a.pad != (a.K - 1) / 2 || a.ldx < a.cin)
    return hipErrorInvalidValue;
  int RB, TW, nt;
  mbconv_ed_tiles(a, &RB, &TW, &nt);
  if (nt == 0) return hipErrorInvalidValue;
  const size_t smem = mb_smem(((RB - 1) * a.S + a.K) * ((TW - 1) * a.S + a.K), a.cin / 32, a.K, a.Cs);
  const dim3 grid((unsigned)((long)a.B * nt)), block(320);
#define KDL_MBED(k, st) \
  if (a.K == k && a.S == st) { hipLaunchKernelGGL((mbconv_ed_kernel<k, st, 4>), grid, block, smem, s, a, RB, TW); return hipGetLastError(); }
  KDL_MBED(3, 1) KDL_MBED(3, 2) KDL_MBED(5, 1) KDL_MBED(5, 2)
#undef KDL_MBED
  return hipErrorInvalidValue;
}

}  // namespace kdl
