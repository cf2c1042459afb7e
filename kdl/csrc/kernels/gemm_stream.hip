// Streaming pointwise GEMM for small K and large M (EfficientNet-B7's 1x1 expand / project convs on
// its 300x300 / 150x150 / 75x75 maps: K 32-480, N 32-480, M up to 2.9 M rows per batch of 32).
//
// These layers are HBM-bound (a 150x150 expand writes 415 MB for 28 GFLOP), but the tiled GEMMs
// (gemm_pipe / conv_gemm) ran them at 1.7-3.2 TB/s effective: a tile's prologue (operand DMA), a 1-2
// step K loop and its LDS-staged epilogue are paid once per tile of a few dozen KB
// (tools/layer_profile.py --model efficientnet_b7, round 5). Here:
//   * persistent workgroups of 8 or 16 waves, one round of them (occupancy-sized grid); the whole weight matrix (NF fragments x KT k-steps, fragment-
//     linear, <= 90 KiB) and the bias sit in LDS for the kernel's life (reloaded only when a
//     workgroup's row range crosses into the next image's A-operand scales, ConvGemmArgs.ascale);
//   * every wave streams 16-row A fragments straight from HBM into registers, PD fragments ahead
//     (register ring), so each CU keeps ~16 x PD x KT KiB of reads in flight;
//   * per row fragment, the NF output fragments are computed two at a time (MFMA 16x16x32 with the
//     weight fragment as the first operand: each lane holds 4 consecutive output channels of one
//     row) and stored from the accumulators (8 bytes per lane: bias, SiLU / ReLU, residual fused) --
//     no C tile through LDS, no barrier in the loop;
//   * opad 1 (ResNet's conv1 feeding a 'valid' 3x3): rows land in the interior of a zero-bordered buffer.
// Instances per (KT, NF) -- the B7 shapes (bf16) and ResNet-50's layer1 / layer2 1x1 convs (fp16, DT 1);
// any other shape is refused (hipErrorInvalidValue) and the layer keeps its tiled configs.
#include "common.h"
#include "launch.h"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace kdl {

namespace {

// A fragments (and, with RES, the residual rows) each wave keeps in flight: the register ring holds
// PD x (KT A k-steps of 4 VGPRs + NF residual pairs of 2), about 72 VGPRs at most
template <int KT, int NF, bool RES>
constexpr int gs_prefetch() {
  constexpr int per = KT * 4 + (RES ? NF * 2 : 0);
  return per * 3 <= 72 ? 3 : per * 2 <= 72 ? 2 : 1;
}

template <int KT, int NF>
constexpr int gs_lds() { return NF * KT * 1024 + NF * 64; }

// waves per workgroup: 16 when the weights take over a third of the LDS (one workgroup per CU),
// else 8, so the CU's resident waves (set by VGPRs) come in finer steps
template <int KT, int NF>
constexpr int gs_waves() { return gs_lds<KT, NF>() > 53 * 1024 ? 16 : 8; }

// RES: the residual add, its rows prefetched into the ring with the A fragment of the same rows (a
// residual load issued in the epilogue would make the wave wait for every newer A load too: vmcnt
// retires in order)
// ACT: the epilogue activation as a compile-time constant (ConvGemmArgs.relu_out 0 / 1 / 2 / 4): tested at run
// time per element, it compiled to a chain of scalar branches per value that also kept the scheduler from
// overlapping one fragment pair's epilogue with the next pair's LDS reads and MFMAs (2,592 v_mov_b64 and ~650
// branches per loop body of the 150x150 expand instance).
// NT: nontemporal output stores (streaming cache policy). Measured (tools/stream_ab.py, B7 b32): a win for
// outputs well past the 256 MB MALL (the 150x150 expands: 177 -> 138 us), a loss for ones the next layer
// can still find cached (the residual projects: 134 -> 143 us) -- a separate config id, picked by the tuner
// DT: element type of x / weights / residual / y (common.h Elt: 0 bf16, 1 fp16)
template <int KT, int NF, bool RES, bool NT, int ACT, int DT = 0>
__global__ __launch_bounds__((64 * gs_waves<KT, NF>())) void gemm_stream_kernel(ConvGemmArgs a) {
  using E = Elt<DT>;
  constexpr int PD = gs_prefetch<KT, NF, RES>();
  constexpr int GS_NW = gs_waves<KT, NF>();
  __shared__ __attribute__((aligned(16))) uint8_t sB[NF * KT * 1024];
  __shared__ __attribute__((aligned(16))) float sBias[NF * 16];
  // per-image A-operand channel scales of the loaded image (ConvGemmArgs.ascale: EfficientNet's SE
  // scale on the project conv's input), applied to each A fragment in registers before its MFMAs
  __shared__ __attribute__((aligned(16))) float sScale[KT * 32];
  // STG: staged stores (no residual, >= 2 fragment pairs; see the epilogue): a 16 x 144-byte tile per wave
  constexpr bool STG = !RES && NF >= 4;
  constexpr int GS_STG = 16 * 144;
  __shared__ __attribute__((aligned(16))) uint8_t sStg[STG ? GS_NW * GS_STG : 16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int OHW = a.OH * a.OW;
  const int FPI = (OHW + 15) / 16;                   // 16-row fragments per image (the last may be partial)
  const int T = a.B * FPI;
  // A operand: lane = (row, 8-element k chunk); accumulator of fragment pair j: channels
  // 16 j + nq .. + 7 of the same row (the permuted weight columns)
  const int row = lane & 15, kq = lane >> 4;
  const int nq = 8 * (lane >> 4);
  static_assert(NF % 2 == 0, "fragment pairs");
  // Fragment order. Shared weights: workgroups take NW-fragment chunks round-robin, so the resident
  // grid moves through the rows as one window (DRAM pages and TLB reach shared by every CU; a
  // contiguous slice per workgroup made ~800 separate write streams and capped wide outputs at
  // 2.7 TB/s). Per-image weights: a contiguous slice per workgroup, walked image by image, so the
  // weights are reloaded only where the slice crosses an image.
  const bool il = !a.ascale;
  const int f0 = (int)((long)T * blockIdx.x / gridDim.x), f1 = (int)((long)T * (blockIdx.x + 1) / gridDim.x);

  for (int i = tid; i < NF * 16; i += 64 * GS_NW) sBias[i] = a.bias[i];
  int loaded = -1;                                   // image whose weights are in sB (-1: none)
  for (int fb = il ? 0 : f0; il ? fb == 0 : fb < f1;) {
    const int img = il ? 0 : fb / FPI;
    const int fend = il ? T : min(f1, (img + 1) * FPI);
    if (loaded < 0 || (!il && img != loaded)) {
      __syncthreads();                               // the previous segment's waves are done with sB
      const uint16_t* wsrc = a.wp;
      // fragment j, k-step t: KT consecutive KiB per fragment as in the packed [NF_pack][K/32][64][8]
      // layout, but with the output channels permuted inside each fragment pair (j even, j + 1): column
      // c of fragment j + h is channel 16 j + 8 (c / 4) + 4 h + c % 4, so accumulator lane quad g of the
      // pair holds the 8 consecutive channels 16 j + 8 g .. + 7 (one 16-byte store per lane)
      // (per-image scales: the weights are loaded once, only the scales change per image)
      if (loaded < 0)
      for (int i = tid; i < NF * KT * 64; i += 64 * GS_NW) {
        const int l = i & 63, jt = i >> 6, j = jt / KT, t = jt - j * KT, c = l & 15;
        const int ch = (j & ~1) * 16 + (c >> 2) * 8 + (j & 1) * 4 + (c & 3);
        const int src = ((ch >> 4) * KT + t) * 64 + ((ch & 15) | (l & 48));
        *(u32x4*)(sB + i * 16) = *(const u32x4*)(wsrc + (long)src * 8);
      }
      if (a.ascale)
        for (int i = tid; i < KT * 32; i += 64 * GS_NW) sScale[i] = a.ascale[(long)img * a.ascale_ld + i];
      __syncthreads();
      loaded = img;
    }
    // this wave's fragments: fbase + q * fstep, q < mine (wave-uniform)
    const int fbase = il ? blockIdx.x * GS_NW + w : fb + w;
    const int fstep = il ? gridDim.x * GS_NW : GS_NW;
    const int mine = fend > fbase ? (fend - fbase + fstep - 1) / fstep : 0;
    auto row_of = [&](int q, long& mlim) {           // row of this lane in the q-th fragment; image row limit
      const int f = fbase + q * fstep, im = f / FPI;
      mlim = (long)(im + 1) * OHW;
      return (long)im * OHW + (long)(f - im * FPI) * 16 + row;
    };
    s16x8 ar[PD][KT];
    u32x4 rr[PD][RES ? NF / 2 : 1];
    auto fill = [&](s16x8 (&dst)[KT], u32x4 (&rdst)[RES ? NF / 2 : 1], int q) {
      long mlim;
      long m = row_of(q, mlim);
      m = m < mlim ? m : mlim - 1;                   // rows past the image: clamped reads, never stored
      const uint16_t* src = a.x + m * a.ldx + kq * 8;
#pragma unroll
      for (int t = 0; t < KT; ++t) dst[t] = *(const s16x8*)(src + t * 32);
      if constexpr (RES) {
        const uint16_t* r = a.res + m * a.ldr;
#pragma unroll
        for (int j = 0; j < NF / 2; ++j) rdst[j] = *(const u32x4*)(r + min(j * 32 + nq, a.nstore - 8));
      }
    };
#pragma unroll
    for (int p = 0; p < PD; ++p)
      if (p < mine) fill(ar[p], rr[p], p);
    // the ring is unrolled by PD, so every slot index is a compile-time constant (a runtime index into
    // a register array would go through scratch); slot p is refilled after its own MFMAs read it
    for (int q0 = 0; q0 < mine; q0 += PD) {
#pragma unroll
      for (int p = 0; p < PD; ++p) {
        const int q = q0 + p;
        if (q >= mine) break;
        long mlim;
        const long m = row_of(q, mlim);
        const bool mok = m < mlim;
        if (DT == 0 && a.ascale) {                     // uniform: scale this fragment's A in place (bf16)
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            const float* sc = sScale + t * 32 + kq * 8;
            const f32x4 s0 = *(const f32x4*)sc, s1 = *(const f32x4*)(sc + 4);
            const u32x4 u = __builtin_bit_cast(u32x4, ar[p][t]);
            u32x4 o;
            o[0] = pack_bf16(bf_lo(u[0]) * s0[0], bf_hi(u[0]) * s0[1]);
            o[1] = pack_bf16(bf_lo(u[1]) * s0[2], bf_hi(u[1]) * s0[3]);
            o[2] = pack_bf16(bf_lo(u[2]) * s1[0], bf_hi(u[2]) * s1[1]);
            o[3] = pack_bf16(bf_lo(u[3]) * s1[2], bf_hi(u[3]) * s1[3]);
            ar[p][t] = __builtin_bit_cast(s16x8, o);
          }
        }
        // the weight fragments are loop-invariant: an opaque lane offset keeps their LDS reads inside
        // the loop (hoisted, NF x KT fragments would take 4 x NF x KT VGPRs and spill)
        uint32_t boff = lane * 16;
        asm volatile("" : "+v"(boff));
#pragma unroll
        for (int j0 = 0; j0 < NF; j0 += 2) {
          f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int t = 0; t < KT; ++t)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              if (j0 + jj < NF)
                acc[jj] = E::mfma(*(const s16x8*)(sB + ((j0 + jj) * KT + t) * 1024 + boff), ar[p][t], acc[jj]);
          const int n = j0 * 16 + nq;
          if (!STG && (!mok || n >= a.nstore)) continue;   // STG: every lane takes part in the read-back
          const int nb = min(n, NF * 16 - 8);                 // (bias reads stay inside sBias)
          const float4 b0 = *(const float4*)(sBias + nb), b1 = *(const float4*)(sBias + nb + 4);
          float v[8] = {acc[0][0] + b0.x, acc[0][1] + b0.y, acc[0][2] + b0.z, acc[0][3] + b0.w,
                        acc[1][0] + b1.x, acc[1][1] + b1.y, acc[1][2] + b1.z, acc[1][3] + b1.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if constexpr (ACT == 1) v[e] = fmaxf(v[e], 0.f);
            else if constexpr (ACT == 4) v[e] = fast_silu(v[e]);
          }
          if constexpr (RES) {
            const u32x4 r = rr[p][j0 / 2];
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[2 * e] += E::lo(r[e]); v[2 * e + 1] += E::hi(r[e]); }
          }
          if constexpr (ACT == 2)
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          const u32x4 o = {E::pack(v[0], v[1]), E::pack(v[2], v[3]), E::pack(v[4], v[5]), E::pack(v[6], v[7])};
          auto gstore = [&](long mm, int nn, const u32x4& val) {
            if (a.opad == 1) {                                  // into a 1-pixel zero-bordered buffer
              const int b = (int)(mm / OHW), rem = (int)(mm - (long)b * OHW);
              const int oh = rem / a.OW, ow = rem - oh * a.OW;
              mm = ((long)b * (a.OH + 2) + oh + 1) * (a.OW + 2) + ow + 1;
            }
            if constexpr (NT) __builtin_nontemporal_store(val, (u32x4*)(a.y + mm * a.ldy + nn));
            else *(u32x4*)(a.y + mm * a.ldy + nn) = val;
          };
          const int pp = j0 / 2;                                // fragment pair
          if constexpr (STG) {
            if ((NF / 2) % 2 == 1 && pp == NF / 2 - 1) {       // odd pair count: the last pair goes direct
              if (mok && n < a.nstore) gstore(m, n, o);
            } else {
              // two pairs (64 channels) of the wave's 16 rows through its LDS tile (144-byte padded rows),
              // then 2 stores of 8 rows x 128 contiguous bytes each (full cache lines; direct: 16 rows x 64 B)
              uint8_t* stg = sStg + w * GS_STG;
              *(u32x4*)(stg + row * 144 + (pp & 1) * 64 + kq * 16) = o;
              if (pp & 1) {
                asm volatile("" ::: "memory");
                const long mb = m - row;                        // the fragment's first row
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                  const int rr2 = k * 8 + (lane >> 3), c = lane & 7;
                  const u32x4 val = *(const u32x4*)(stg + rr2 * 144 + c * 16);
                  const int nn = (pp - 1) * 32 + c * 8;
                  if (mb + rr2 < mlim && nn < a.nstore) gstore(mb + rr2, nn, val);
                }
                asm volatile("" ::: "memory");
              }
            }
          } else {
            gstore(m, n, o);
          }
        }
        if (q + PD < mine) fill(ar[p], rr[p], q + PD);   // refill slot p: this wave's fragment q + PD
      }
    }
    fb = fend;
  }
}

int num_cus() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return c > 0 ? c : 256;
  }();
  return n;
}

template <int KT, int NF, bool RES, bool NT, int ACT, int DT>
hipError_t launch_act(const ConvGemmArgs& a, hipStream_t s) {
  constexpr int NW = gs_waves<KT, NF>();
  // one round of resident workgroups (by VGPRs and LDS, as the runtime computes it): a grid past
  // that runs its excess as a tail round on a fraction of the CUs
  static const int per_cu = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, gemm_stream_kernel<KT, NF, RES, NT, ACT, DT>, 64 * NW, 0) != hipSuccess)
      return 1;
    return std::max(1, n);
  }();
  const long frags = (long)a.B * ((a.OH * a.OW + 15) / 16);
  const long want = (frags + NW - 1) / NW;
  const int grid = (int)std::max(1L, std::min(want, (long)num_cus() * per_cu));
  hipLaunchKernelGGL((gemm_stream_kernel<KT, NF, RES, NT, ACT, DT>), dim3(grid), dim3(64 * NW), 0, s, a);
  return hipGetLastError();
}

template <int KT, int NF, bool RES, bool NT, int DT>
hipError_t launch_nt(const ConvGemmArgs& a, hipStream_t s) {
  switch (a.relu_out) {
    case 0: return launch_act<KT, NF, RES, NT, 0, DT>(a, s);
    case 1: return launch_act<KT, NF, RES, NT, 1, DT>(a, s);
    case 2: return launch_act<KT, NF, RES, NT, 2, DT>(a, s);
    case 4: return launch_act<KT, NF, RES, NT, 4, DT>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int KT, int NF, bool RES, int DT>
hipError_t launch_stream(const ConvGemmArgs& a, bool nt, hipStream_t s) {
  return nt ? launch_nt<KT, NF, RES, true, DT>(a, s) : launch_nt<KT, NF, RES, false, DT>(a, s);
}

// residual instances up to NF 18 (wider ones would spill the residual ring; no B7 layer has one)
template <int KT, int NF, int DT>
hipError_t launch_res(const ConvGemmArgs& a, bool nt, hipStream_t s) {
  if constexpr (NF <= 18) return launch_stream<KT, NF, true, DT>(a, nt, s);
  else return hipErrorInvalidValue;
}

}  // namespace

// (KT = K / 32, NF = output fragments) instances: EfficientNet-B7's large-map 1x1 convs (bf16) and
// ResNet-50's layer1 / layer2.0 1x1 convs at 56x56 (fp16: 64 -> 64, 64 -> 256, 256 -> 64, 256 -> 128)
#define KDL_STREAM_SHAPES(X) \
  X(1, 2) X(2, 2) X(1, 12) X(6, 4) X(2, 18) X(9, 4) X(9, 6) X(3, 30) X(15, 6)
#define KDL_STREAM_SHAPES_F16(X) \
  X(2, 4) X(2, 16) X(8, 4) X(8, 8)

bool gemm_stream_shape(int K, int nstore, int dt) {
  const int kt = K / 32, nf = (nstore + 15) / 16;
  if (dt == 1) {
    switch (kt * 100 + nf) {
#define KDL_GSHAS(kt_, nf_) case kt_ * 100 + nf_:
      KDL_STREAM_SHAPES_F16(KDL_GSHAS)
      return K % 32 == 0;
      default: return false;
    }
  }
  switch (kt * 100 + nf) {
    KDL_STREAM_SHAPES(KDL_GSHAS)
#undef KDL_GSHAS
    return K % 32 == 0;
    default: return false;
  }
}

hipError_t gemm_stream(const ConvGemmArgs& a, bool nt, hipStream_t s) {
  if (a.dt < 0 || a.dt > 1 || (a.dt == 1 && a.ascale) || (a.opad != 0 && a.opad != 1) || a.stride != 1 || a.ksplit > 1 || a.OH != a.H || a.OW != a.W || a.M <= 0 ||
      a.M != a.B * a.OH * a.OW || a.K % 32 != 0 || a.ldx % 8 != 0 || a.ldy % 8 != 0 || a.nstore % 8 != 0 ||
      (a.res && a.ldr % 8 != 0) || !gemm_stream_shape(a.K, a.nstore, a.dt) ||
      (a.ascale && (a.ascale_ld < a.K || a.ascale_ld % 4 != 0)) ||
      a.relu_out == 3 || a.relu_in || a.NF * 16 < a.nstore)
    return hipErrorInvalidValue;
  if (a.dt == 1) {
    switch ((a.K / 32) * 100 + (a.nstore + 15) / 16) {
#define KDL_GSCASE1(kt_, nf_) \
  case kt_ * 100 + nf_: return a.res ? launch_res<kt_, nf_, 1>(a, nt, s) : launch_stream<kt_, nf_, false, 1>(a, nt, s);
      KDL_STREAM_SHAPES_F16(KDL_GSCASE1)
#undef KDL_GSCASE1
      default: return hipErrorInvalidValue;
    }
  }
  switch ((a.K / 32) * 100 + (a.nstore + 15) / 16) {
#define KDL_GSCASE(kt_, nf_) \
  case kt_ * 100 + nf_: return a.res ? launch_res<kt_, nf_, 0>(a, nt, s) : launch_stream<kt_, nf_, false, 0>(a, nt, s);
    KDL_STREAM_SHAPES(KDL_GSCASE)
#undef KDL_GSCASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace kdl
