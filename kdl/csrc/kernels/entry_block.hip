// Whole Xception entry block in ONE persistent kernel (block2: 147x147x64 -> 74x74x128):
//
//   y1  = ReLU(BN(pw1(dw1(x))))          SeparableConv2D 64 -> 128  (+ReLU)
//   y2  = BN(pw2(dw2(y1)))               SeparableConv2D 128 -> 128
//   out = maxpool3x3/2_same(y2) + BN(conv1x1/2(x))                  (guide.md:222-229 graph)
//
// Unfused, the block moves ~790 MB per batch of 32 through HBM (y1 and y2 are 177 MB each,
// written and read back, plus the pool pass) in four launches (~280 us measured, round 3).
// Here y1 and y2 never leave the CU: the kernel reads x once (88 MB) and writes the pooled
// block output (45 MB).
//
// Tiling: a work item is one POOLED output row k of one image and one strip of PC pooled
// columns. A workgroup walks a run of consecutive rows of a strip (host-built step table,
// `steps`), keeping rolling windows in LDS:
//   x ring   4 rows x (2PC+5) cols x C0   (DMA: two new rows per step)
//   y1 ring  4 rows x (2PC+3) cols x C1   (two new rows per step, written by GEMM1's epilogue)
//   y2       rows 2k, 2k+1 in accumulators; row 2k-1 carried in registers from the previous step
// The 3x3/2 pool needs y2 rows 2k-1..2k+1 (TF 'same', pad 1 for 147 -> 74), so every y1 / y2
// row is computed once per strip; only the 2 halo columns between strips are recomputed
// (~6 %). A run starts with two warm-up steps (y1 only; y1 + y2 without output).
//
// Work split (C1 / 16 waves): wave w owns output channels 16w..16w+15 of EVERY GEMM (pw1, pw2,
// the residual 1x1), so its weights live in registers for the whole kernel and the GEMMs read
// only activations from LDS. The depthwise convs run on the VALU (v_dot2c_f32_bf16 over tap
// pairs, fp32 accumulate), each lane producing the 8 channels of one pixel = exactly its MFMA
// operand fragment, written fragment-linear to an LDS A buffer. Phases per step, separated by
// workgroup barriers: dw1 -> GEMM1 (+ residual GEMM) -> dw2 -> GEMM2 + pool.
//
// LDS activation images are channel-PLANE major (16-byte slot = 8 channels of one pixel, a
// plane = one 8-channel chunk of a row, pitch PLP px, a multiple of 16): a depthwise / MFMA
// fragment read (16 pixels x 4 chunks per wave instruction) then touches all 64 banks once.
#include "common.h"
#include "launch.h"

#include <algorithm>

namespace kdl {

__device__ __attribute__((aligned(16))) uint8_t eb_zeros[256];

constexpr int EB_MAX_STEPS = 128;                  // steps per workgroup (host plan checks it)

// The workgroup's step words in two VGPRs: word i in lane i % 64 of v[i / 64]. A step is decoded with
// v_readlane at its (uniform) index: no LDS round trip at the head of every step's dependency chain
// (address math -> tap reads), which the LDS-resident table put there once per decode.
struct EbStepRegs {
  uint32_t v0 = 0, v1 = 0;
  __device__ __forceinline__ void load(const uint32_t* st, int n, int lane) {
    v0 = lane < n ? st[lane] : 0u;
    v1 = 64 + lane < n ? st[64 + lane] : 0u;
  }
  __device__ __forceinline__ uint32_t get(int i) const {
    i = __builtin_amdgcn_readfirstlane(i);
    return (uint32_t)__builtin_amdgcn_readlane((int)(i < 64 ? v0 : v1), i & 63);
  }
};
static_assert(EB_MAX_STEPS <= 128, "EbStepRegs holds two words per lane");

template <int C0, int C1, int PC, int NFW, bool DWM = false>
struct EbGeom {
  static constexpr int Y2C = 2 * PC + 1;            // y2 columns a strip needs
  static constexpr int Y1C = Y2C + 2;               // y1 columns
  static constexpr int XC = Y1C + 2;                // x columns
  static constexpr int PLP = (XC + 15) / 16 * 16;   // plane pitch (pixels)
  static constexpr int PLB = PLP * 16;              // plane bytes
  static constexpr int XROW = (C0 / 8) * PLB;       // one x ring row
  static constexpr int Y1ROW = (C1 / 8) * PLB;      // one y1 ring row
  static constexpr int KT0 = C0 / 32, KT1 = C1 / 32;
  static constexpr int Y1F = (2 * Y1C + 15) / 16;   // y1 pixel fragments per step (2 rows)
  static constexpr int Y2FR = (Y2C + 15) / 16;      // y2 fragments per row
  static constexpr int Y2F = 2 * Y2FR;
  static constexpr int NW = C1 / (16 * NFW);        // waves (NFW 16-channel output slices each)
  static constexpr int XDMA = XROW / 1024;          // 1 KiB DMA instructions per x row
  static constexpr int ABYTES = (KT0 * Y1F > KT1 * Y2F ? KT0 * Y1F : KT1 * Y2F) * 1024;
  static constexpr int PCOLS = 16 * Y2FR;           // pool row columns
  static constexpr int DWQ = DWM ? 1024 : 640;      // LDS depthwise entries per k-step: 4 lane groups x 40 words
                                                    // (VALU), or pack_dw_entries' 1 KiB (MFMA variant)
  // LDS map: the two depthwise A buffers alias (A1 is read before the barrier that precedes
  // A2's writes, A2 before the next step's first barrier)
  static constexpr int OFF_X = 0;
  static constexpr int OFF_Y1 = OFF_X + 4 * XROW;
  static constexpr int OFF_A = OFF_Y1 + 4 * Y1ROW;
  static constexpr int OFF_P = OFF_A + ABYTES;      // per-wave pool rows [NW][PCOLS][16*NFW] bf16
  static constexpr int OFF_DW = OFF_P + NW * PCOLS * 16 * NFW * 2;
  static constexpr int OFF_B = OFF_DW + (KT0 + KT1) * DWQ;   // biases [3][C1] fp32
  static constexpr int OFF_S = OFF_B + 3 * C1 * 4;  // this workgroup's step table, one packed word per step
  static constexpr int BYTES = OFF_S + 4 * EB_MAX_STEPS;
  static_assert(XROW % 1024 == 0, "whole DMA instructions per x row");
  static_assert(C0 % 32 == 0 && C1 % (16 * NFW) == 0 && NW <= 16, "channel tiling");
  static_assert(BYTES <= 160 * 1024, "LDS");
};

// four bf16 pairs (two 16-B taps a, b of one pixel: channels c..c+7) -> dot2 operands
// (a[c], b[c]) / (a[c+1], b[c+1]) per channel pair
__device__ __forceinline__ uint32_t eb_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ uint32_t eb_hi(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }
__device__ __forceinline__ float eb_dot(uint32_t x, uint32_t w, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, x), __builtin_bit_cast(bf16x2, w), c, false);
}

// depthwise 3x3 of 8 channels of one pixel, tap pair by tap pair (taps 2j, 2j+1; tap 9 = 0) so
// only one pair of 16-B taps and its 8 weight words are live at a time: tap(i) -> the 16-B input
// of tap i (dy*3+dx), wq -> [tap pair j][channel e] bf16x2 words (LDS, broadcast per lane group).
// fp32 accumulation (v_dot2c_f32_bf16); returns the 8 outputs as bf16 = one MFMA operand.
template <bool RELU, class Tap>
__device__ __forceinline__ s16x8 eb_dw8(Tap tap, const uint32_t* wq) {
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    u32x4 a = tap(2 * j);
    u32x4 b = j < 4 ? tap(2 * j + 1) : (u32x4){0u, 0u, 0u, 0u};
    const u32x4 w0 = *(const u32x4*)(wq + 8 * j), w1 = *(const u32x4*)(wq + 8 * j + 4);
    if constexpr (RELU) {
#pragma unroll
      for (int d = 0; d < 4; ++d) { a[d] = relu_bf16x2(a[d]); b[d] = relu_bf16x2(b[d]); }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t wl = d < 2 ? w0[2 * d] : w1[2 * d - 4], wh = d < 2 ? w0[2 * d + 1] : w1[2 * d - 3];
      acc[2 * d] = eb_dot(eb_lo(a[d], b[d]), wl, acc[2 * d]);
      acc[2 * d + 1] = eb_dot(eb_hi(a[d], b[d]), wh, acc[2 * d + 1]);
    }
  }
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = pack_bf16(acc[2 * d], acc[2 * d + 1]);
  return __builtin_bit_cast(s16x8, o);
}

// depthwise 3x3 of a 16-pixel x 32-channel unit on the MATRIX cores (the block-diagonal operand of
// sepconv_ws.hip): per 16-channel group g, 5 MFMAs over tap pairs. Lane (p16, kb) feeds tap
// 2j + (kb >> 1) of chunk 2g + (kb & 1); tap(g, ti) -> that 16-B input; ent(g) -> the 16-B entry
// (pack_dw_entries) of channel 16g + p16, tap parity kb >> 1. The C fragment [16 ch][16 px] is
// written transposed into the unit's lane-linear A fragment at dst.
template <bool RELU, class Tap, class Ent>
__device__ __forceinline__ void eb_dw_mfma_vals(Tap tap, Ent ent, int lane, const uint32_t (&sel)[2][4], u32x2 (&out)[2]) {
  const int kb = lane >> 4, par = kb >> 1;
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const u32x4 we = ent(g);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int ti = 2 * j + par;
      u32x4 v = ti < 9 ? tap(g, ti) : (u32x4){0u, 0u, 0u, 0u};
      if constexpr (RELU) {
#pragma unroll
        for (int d = 0; d < 4; ++d) v[d] = relu_bf16x2(v[d]);
      }
      const uint32_t wd = we[j >> 1];
      u32x4 wf;
#pragma unroll
      for (int d = 0; d < 4; ++d) wf[d] = __builtin_amdgcn_perm(wd, wd, sel[j & 1][d]);
      acc = mfma16(__builtin_bit_cast(s16x8, wf), __builtin_bit_cast(s16x8, v), acc);
    }
    out[g] = (u32x2){pack_bf16(acc[0], acc[1]), pack_bf16(acc[2], acc[3])};
  }
}

// the C fragment [16 ch][16 px] of both channel groups, written transposed into the unit's
// lane-linear A fragment at dst. Kept apart from the MFMAs so a phase can compute all of its
// units before its first store (a later unit's tap reads would otherwise wait behind it)
__device__ __forceinline__ void eb_dw_store(uint8_t* dst, int lane, const u32x2 (&out)[2]) {
  const int p16 = lane & 15, kb = lane >> 4, par = kb >> 1;
#pragma unroll
  for (int g = 0; g < 2; ++g) *(u32x2*)(dst + (p16 + 16 * (2 * g + par)) * 16 + 8 * (kb & 1)) = out[g];
}

// workgroup barrier for LDS hand-offs only: LDS-scoped release / acquire fences around s_barrier, so
// the compiler orders LDS accesses around it and emits only lgkmcnt(0). __syncthreads() (a fence over
// every address space) lowers to s_waitcnt vmcnt(0) lgkmcnt(0) + s_barrier, which drained the next
// step's x-row LDS-DMA at the first phase barrier after its issue (B2) instead of at B0
__device__ __forceinline__ void eb_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// 16-byte global -> LDS DMA as inline asm (M0 = the wave-uniform LDS address; lane l lands at M0 + 16 l).
// The compiler's waitcnt pass cannot tell an LDS-DMA destination from other LDS regions and drains
// (vmcnt(0)) every in-flight DMA before some later LDS stores; asm is invisible to it. CONTRACT: the
// caller waits for the DMA with its own vmcnt, and no compiler-tracked VMEM load is in flight across it.
__device__ __forceinline__ void glds16_asm(const void* g, void* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)lds);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ s16x8 eb_frag(const uint16_t* wp, int nf, int kt, int t, int lane) {
  return *(const s16x8*)(wp + ((long)(nf * kt + t) * 64 + lane) * 8);
}

template <int C0, int C1, int PC, int NFW, int PT, bool RELU1, bool STAMP = false, bool DWM = false, int OCC = 1>
__global__ __launch_bounds__(64 * (C1 / (16 * NFW)), OCC * C1 / (64 * NFW)) void entry_block_kernel(EntryBlockArgs a) {
  using G = EbGeom<C0, C1, PC, NFW, DWM>;
  constexpr int NW = G::NW, KT0 = G::KT0, KT1 = G::KT1;
  constexpr int PLB = G::PLB, XROW = G::XROW, Y1ROW = G::Y1ROW;
  constexpr int Y1C = G::Y1C, Y2C = G::Y2C, XC = G::XC, PLP = G::PLP;
  constexpr int Y1F = G::Y1F, Y2F = G::Y2F, Y2FR = G::Y2FR, PCOLS = G::PCOLS;
  constexpr int U1 = KT0 * Y1F, U2 = KT1 * Y2F;      // depthwise units (fragment x k-step)
  constexpr int U1W = (U1 + NW - 1) / NW, U2W = (U2 + NW - 1) / NW;
  constexpr int PCH = 16 * NFW;                      // channels per wave
  static_assert(NW % KT0 == 0 && NW % KT1 == 0, "a wave's depthwise units share one k-step");
  static_assert(PT == 0 || PT == 1, "TF-'same' 3x3/2 pool: leading pad 1 (odd size) or 0 (even)");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q16 = lane >> 4, p16 = lane & 15;
  const int H = a.H, W = a.W;
  const int s0 = a.step_off[blockIdx.x], s1 = a.step_off[blockIdx.x + 1];
  if (s0 >= s1 || s1 - s0 > EB_MAX_STEPS) return;   // uniform: no work (or a plan the host must reject)

  uint8_t* const xr = smem + G::OFF_X;
  uint8_t* const y1r = smem + G::OFF_Y1;
  uint8_t* const Ab = smem + G::OFF_A;
  uint16_t* const pool = (uint16_t*)(smem + G::OFF_P) + w * (PCOLS * PCH);
  uint32_t* const dwl = (uint32_t*)(smem + G::OFF_DW);
  float* const bl = (float*)(smem + G::OFF_B);
  uint32_t* const stl = (uint32_t*)(smem + G::OFF_S);
  // the step table goes to LDS once: decoding a step from global memory put an L2 round trip
  // on every step's critical path twice (measured ~3k cycles per step, tools/ebbench.py --stamps).
  // One word per step {image 8 | strip 6 | pooled row + 2 9 | mode 2 bits}: a 2-workgroup-per-CU
  // config then fits its 80 KiB (int4 entries took 2 KiB of it)
  for (int i = tid; i < s1 - s0; i += 64 * NW) {
    const int4 e = a.steps[s0 + i];
    stl[i] = (uint32_t)e.x | ((uint32_t)e.y << 8) | ((uint32_t)(e.z + 2) << 14) | ((uint32_t)e.w << 23);
  }

  // ---- depthwise weight entries -> LDS. VALU variant: [k-step][lane group q][tap pair j][channel e]
  // bf16x2; MFMA variant (DWM): pack_dw_entries' [k-step][g][n][parity][8] bf16, 1 KiB per k-step
  if constexpr (DWM) {
    for (int i = tid; i < (KT0 + KT1) * 64; i += 64 * NW) {
      const int t = i / 64;
      const u32x4 v = t < KT0 ? *(const u32x4*)((const uint8_t*)a.dwk1 + t * 1024 + (i % 64) * 16)
                              : *(const u32x4*)((const uint8_t*)a.dwk2 + (t - KT0) * 1024 + (i % 64) * 16);
      *(u32x4*)((uint8_t*)dwl + t * G::DWQ + (i % 64) * 16) = v;
    }
  } else
  for (int i = tid; i < (KT0 + KT1) * 4 * 40; i += 64 * NW) {
    const int t = i / 160, q = (i / 40) % 4, j = (i % 40) / 8, e = i % 8;
    const bool second = t >= KT0;
    const float* wsrc = second ? a.dw2 : a.dw1;
    const int C = second ? C1 : C0, c = 32 * (second ? t - KT0 : t) + 8 * q + e;
    const float wa = wsrc[(2 * j) * C + c];
    const float wb = j < 4 ? wsrc[(2 * j + 1) * C + c] : 0.f;
    dwl[i] = pack_bf16(wa, wb);
  }
  // ---- register-resident pointwise weights of this wave's NFW x 16 output channels
  s16x8 w1[NFW][KT0], w2[NFW][KT1];
#pragma unroll
  for (int n = 0; n < NFW; ++n) {
#pragma unroll
    for (int t = 0; t < KT0; ++t) w1[n][t] = eb_frag(a.w1, NFW * w + n, KT0, t, lane);
#pragma unroll
    for (int t = 0; t < KT1; ++t) w2[n][t] = eb_frag(a.w2, NFW * w + n, KT1, t, lane);
  }
  for (int i = tid; i < 3 * C1; i += 64 * NW) bl[i] = (i < C1 ? a.b1 : i < 2 * C1 ? a.b2 : a.br)[i % C1];
  // this lane's 4 accumulator channels of output slice n: bias (LDS) of GEMM g (0 pw1, 1 pw2, 2 residual)
  // 1-slice configs keep this lane's 3 x 4 biases in registers (read once from global): in LDS a
  // bias read that follows a y1 / pool store cannot be hoisted above it, so every fragment of
  // P2 / P4 re-read it and waited for it
  // 16-wave configs (NW 16: 4 waves per SIMD, <= 128 VGPRs) take none of the register-hungry forms
  constexpr bool WIDE = NFW == 1 && OCC == 1 && NW <= 8;
  constexpr bool BREG = WIDE;
  float4 breg[BREG ? 3 : 1][NFW];
  if constexpr (BREG) {
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int n = 0; n < NFW; ++n)
        breg[g][n] = *(const float4*)((g == 0 ? a.b1 : g == 1 ? a.b2 : a.br) + PCH * w + 16 * n + 4 * q16);
  }
  auto bias = [&](int g, int n) {
    if constexpr (BREG) return breg[g][n];
    else return *(const float4*)(bl + g * C1 + PCH * w + 16 * n + 4 * q16);
  };
  const int t1 = w % KT0, t2 = w % KT1;              // every depthwise unit of this wave uses these k-steps
  uint32_t sel[2][4];                                // DWM: v_perm selectors of the block-diagonal operand
  {
    const bool wv = (p16 >> 3) == (q16 & 1);
    const int e = p16 & 7;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t pair = (2u * jp) | ((2u * jp + 1u) << 8);
        const uint32_t val = (e & 1) ? (0x0c0cu | (pair << 16)) : (0x0c0c0000u | pair);
        sel[jp][d] = (wv && (e >> 1) == d) ? val : 0x0c0c0c0cu;
      }
  }
  // ---- x row DMA: row r of image b, strip columns from global col gx0, into ring slot r & 3
  // (preparing the addresses ahead, before B1, measured slower: the wave runs it in order anyway)
  auto dma_rows = [&](int b, int gx0, int r0, int nr) {
    for (int ii = w; ii < nr * G::XDMA; ii += NW) {
      const int r = r0 + ii / G::XDMA, d = ii % G::XDMA;
      const int slot = d * 64 + lane, plane = slot / PLP, px = slot - plane * PLP;
      const int gx = gx0 + px;
      const bool ok = px < XC && (unsigned)r < (unsigned)H && (unsigned)gx < (unsigned)W;
      const uint8_t* src = ok ? (const uint8_t*)(a.x + (((long)b * H + r) * W + gx) * a.ldx + plane * 8) : eb_zeros;
      glds16(src, xr + (r & 3) * XROW + d * 1024);
    }
  };
  // register-resident step words where the registers are free (1-slice, 1-workgroup-per-CU configs:
  // block3's and the 2-workgroup configs' allocations already spill)
  constexpr bool REG_STEPS = NFW == 1 && OCC == 1;
  EbStepRegs str;                                     // loaded once the table is published (below)
  auto decode = [&](int q, int& b, int& s, int& k, int& mode) {
    const uint32_t e = REG_STEPS ? str.get(q - s0) : stl[q - s0];
    b = e & 255; s = (e >> 8) & 63; k = (int)((e >> 14) & 511) - 2; mode = (e >> 23) & 3;
  };
  // pooled row k pools y2 rows R..R+2, R = 2k - PT; a step computes y1 rows R+2, R+3 from x rows
  // R+1..R+4: the rows its predecessor did not load (a run's first step loads all four)
  auto dma_for = [&](int q) {
    int b, s, k, mode;
    decode(q, b, s, k, mode);
    const int R = 2 * k - PT;
    const int gx0 = 2 * s * PC - PT - 2;
    if (mode == 0) dma_rows(b, gx0, R + 1, 4);
    else dma_rows(b, gx0, R + 3, 2);
  };

  u32x2 carry[NFW][Y2FR];                            // y2 row R+2 of the previous step (= this step's R), bf16
  f32x4 accr[NFW];                                   // residual GEMM of the pooled row it was computed for
  s16x8 wr[NFW][KT0];                                // residual 1x1/2 weights (register-resident)
#pragma unroll
  for (int n = 0; n < NFW; ++n)
#pragma unroll
    for (int t = 0; t < KT0; ++t) wr[n][t] = eb_frag(a.wr, NFW * w + n, KT0, t, lane);
  bool st_pend = false;                              // deferred output store of the previous step
  uint16_t* st_ptr = nullptr;
  u32x2 st_val[NFW];

  // STAMP builds (diagnostics, tools/ebbench.py --stamps): thread 0 of workgroups < 8 records
  // s_memtime after each barrier of its first 64 steps: [wg][step][B0, B1, B2, B3, end]
  auto stamp = [&](int q, int ph) {
    if constexpr (STAMP) {
      if (tid == 0 && blockIdx.x < 8 && q - s0 < 64 && a.stamps)
        a.stamps[((long)blockIdx.x * 64 + (q - s0)) * 5 + ph] = __builtin_amdgcn_s_memtime();
    }
  };
  __syncthreads();                                   // step table, weights, biases in LDS
  if constexpr (REG_STEPS) str.load(stl, s1 - s0, lane);
  dma_for(s0);
  for (int q = s0; q < s1; ++q) {
    int b, s, k, mode;
    decode(q, b, s, k, mode);
    const int R = 2 * k - PT;
    const int pc0 = s * PC;
    // the residual this step's output adds: PT 1 computes it below (x row 2k is in the ring);
    // PT 0 computed it in the previous step (x row 2k has left the ring by now)
    f32x4 acco[NFW];
#pragma unroll
    for (int n = 0; n < NFW; ++n) acco[n] = accr[n];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                 // B0: x rows landed; previous step done

    stamp(q, 0);

    // ---- P1: depthwise 1 -> A (y1 rows R+2, R+3); residual operands: pooled row k (PT 1: x row
    // 2k = R+1) or k+1 (PT 0: x row 2k+2 = R+2; x row 2k is no longer in the ring)
    {
      const uint32_t* wq = dwl + (t1 * 4 + q16) * 40;
      u32x2 dv[U1W][2];                              // every unit's outputs, stored after the loop
      s16x8 vv[U1W];
      uint8_t* ddst[U1W];
#pragma unroll
      for (int i = 0; i < U1W; ++i) ddst[i] = nullptr;
#pragma unroll
      for (int i = 0; i < U1W; ++i) {
        const int u = w + NW * i;
        if (u < U1) {
          const int f = u / KT0;
          int pi = 16 * f + p16;
          pi = pi < 2 * Y1C ? pi : 2 * Y1C - 1;
          const int rr = pi >= Y1C, col = pi - rr * Y1C;
          const int row = R + 2 + rr;
          if constexpr (DWM) {
            const uint8_t* base = xr + (4 * t1 + (q16 & 1)) * PLB + col * 16;
            auto tap = [&](int g, int ti) {
              return *(const u32x4*)(base + 2 * g * PLB + ((row - 1 + ti / 3) & 3) * XROW + (ti % 3) * 16);
            };
            auto ent = [&](int g) {
              return *(const u32x4*)((const uint8_t*)dwl + t1 * G::DWQ + (((g * 16 + p16) * 2) + (q16 >> 1)) * 16);
            };
            eb_dw_mfma_vals<RELU1>(tap, ent, lane, sel, dv[i]);
            ddst[i] = Ab + (t1 * Y1F + f) * 1024;
          } else {
            const uint8_t* base = xr + (4 * t1 + q16) * PLB + col * 16;
            auto tap = [&](int ti) {
              return *(const u32x4*)(base + ((row - 1 + ti / 3) & 3) * XROW + (ti % 3) * 16);
            };
            // 1-slice configs store after the loop (see eb_dw_store); block3's register-bound
            // config stores at once (the deferred form spilled 67 VGPRs there)
            if constexpr (WIDE) {
              vv[i] = eb_dw8<RELU1>(tap, wq);
              ddst[i] = Ab + (t1 * Y1F + f) * 1024 + lane * 16;
            } else {
              *(s16x8*)(Ab + (t1 * Y1F + f) * 1024 + lane * 16) = eb_dw8<RELU1>(tap, wq);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < U1W; ++i) {
        if (!ddst[i]) continue;
        if constexpr (DWM) eb_dw_store(ddst[i], lane, dv[i]);
        else *(s16x8*)ddst[i] = vv[i];
      }
    }
    if (PT == 1 ? mode == 2 : mode >= 1) {           // residual 1x1/2 conv of its pooled row
      const int xrow = R + 2 - PT, xcol = 2 * p16 + PT + 2;
#pragma unroll
      for (int n = 0; n < NFW; ++n) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT0; ++t)
          acc = mfma16(wr[n][t], *(const s16x8*)(xr + (xrow & 3) * XROW + (4 * t + q16) * PLB + xcol * 16), acc);
        accr[n] = acc;
        if (PT == 1) acco[n] = acc;
      }
    }
    eb_lds_barrier();                                // B1: A (y1) complete; x ring free for the next DMA
    stamp(q, 1);

    if (st_pend) {
#pragma unroll
      for (int n = 0; n < NFW; ++n) *(u32x2*)(st_ptr + 16 * n) = st_val[n];
      st_pend = false;
    }
    if (q + 1 < s1) dma_for(q + 1);

    // ---- P2: GEMM1 (+ bias, ReLU) -> y1 ring rows R+2, R+3; residual GEMM
    // HOIST (1-slice configs, registers to spare): every A fragment is read before the first y1
    // store -- the compiler cannot move a read above a store it cannot prove disjoint, which
    // chained each fragment's LDS latency behind the previous fragment's store
    constexpr bool HOIST = WIDE;
    s16x8 a1h[HOIST ? Y1F : 1][KT0];
    if constexpr (HOIST) {
#pragma unroll
      for (int f = 0; f < Y1F; ++f)
#pragma unroll
        for (int t = 0; t < KT0; ++t) a1h[f][t] = *(const s16x8*)(Ab + (t * Y1F + f) * 1024 + lane * 16);
    }
    float4 bz0[NFW];                                 // read before the y1 stores (see BREG)
#pragma unroll
    for (int n = 0; n < NFW; ++n) bz0[n] = bias(0, n);
#pragma unroll
    for (int f = 0; f < Y1F; ++f) {
      const s16x8* af = (const s16x8*)(Ab + f * 1024 + lane * 16);
      const int pi = 16 * f + p16;
      const int rr = pi >= Y1C, col = pi - rr * Y1C;
      const int row = R + 2 + rr, gcol = 2 * pc0 - PT - 1 + col;
      const bool ok = (unsigned)row < (unsigned)H && (unsigned)gcol < (unsigned)W;
#pragma unroll
      for (int n = 0; n < NFW; ++n) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT0; ++t) acc = mfma16(w1[n][t], HOIST ? a1h[HOIST ? f : 0][t] : af[t * Y1F * 64], acc);
        if (pi < 2 * Y1C) {
          const int c = PCH * w + 16 * n + 4 * q16;
          const float4 bv = bz0[n];
          const float v0 = fmaxf(acc[0] + bv.x, 0.f), v1 = fmaxf(acc[1] + bv.y, 0.f);
          const float v2 = fmaxf(acc[2] + bv.z, 0.f), v3 = fmaxf(acc[3] + bv.w, 0.f);
          const u32x2 o = ok ? (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)} : (u32x2){0u, 0u};
          *(u32x2*)(y1r + (row & 3) * Y1ROW + (c / 8) * PLB + col * 16 + (c & 7) * 2) = o;
        }
      }
    }
    eb_lds_barrier();                                // B2: y1 rows R+2, R+3 written; A free
    stamp(q, 2);

    if (mode == 0) continue;                         // warm-up 1: y1 only
    // ---- P3: depthwise 2 -> A (y2 rows R+1, R+2: fragments [row][col / 16])
    {
      const uint32_t* wq = dwl + ((KT0 + t2) * 4 + q16) * 40;
      u32x2 dv2[U2W][2];
      s16x8 vv2[U2W];
      uint8_t* ddst2[U2W];
#pragma unroll
      for (int i = 0; i < U2W; ++i) ddst2[i] = nullptr;
#pragma unroll
      for (int i = 0; i < U2W; ++i) {
        const int u = w + NW * i;
        if (u < U2) {
          const int f = u / KT1;
          const int rr = f / Y2FR, col = (f % Y2FR) * 16 + p16;
          const int row = R + 1 + rr;
          if constexpr (DWM) {
            const uint8_t* base = y1r + (4 * t2 + (q16 & 1)) * PLB + col * 16;
            auto tap = [&](int g, int ti) {
              return *(const u32x4*)(base + 2 * g * PLB + ((row - 1 + ti / 3) & 3) * Y1ROW + (ti % 3) * 16);
            };
            auto ent = [&](int g) {
              return *(const u32x4*)((const uint8_t*)dwl + (KT0 + t2) * G::DWQ + (((g * 16 + p16) * 2) + (q16 >> 1)) * 16);
            };
            eb_dw_mfma_vals<false>(tap, ent, lane, sel, dv2[i]);
            ddst2[i] = Ab + (t2 * Y2F + f) * 1024;
          } else {
            const uint8_t* base = y1r + (4 * t2 + q16) * PLB + col * 16;
            auto tap = [&](int ti) {
              return *(const u32x4*)(base + ((row - 1 + ti / 3) & 3) * Y1ROW + (ti % 3) * 16);
            };
            if constexpr (WIDE) {
              vv2[i] = eb_dw8<false>(tap, wq);
              ddst2[i] = Ab + (t2 * Y2F + f) * 1024 + lane * 16;
            } else {
              *(s16x8*)(Ab + (t2 * Y2F + f) * 1024 + lane * 16) = eb_dw8<false>(tap, wq);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < U2W; ++i) {
        if (!ddst2[i]) continue;
        if constexpr (DWM) eb_dw_store(ddst2[i], lane, dv2[i]);
        else *(s16x8*)ddst2[i] = vv2[i];
      }
    }
    eb_lds_barrier();                                // B3: A (y2) complete
    stamp(q, 3);

    // ---- P4: GEMM2 + bias -> bf16 values; vertical max with the carried row
    const bool r0ok = (unsigned)R < (unsigned)H && mode == 2, r1ok = (unsigned)(R + 1) < (unsigned)H;
    const bool r2ok = (unsigned)(R + 2) < (unsigned)H;
    s16x8 a2h[HOIST ? Y2F : 1][KT1];                 // HOIST: every fragment read before the pool stores
    if constexpr (HOIST) {
#pragma unroll
      for (int f = 0; f < Y2F; ++f)
#pragma unroll
        for (int t = 0; t < KT1; ++t) a2h[f][t] = *(const s16x8*)(Ab + (t * Y2F + f) * 1024 + lane * 16);
    }
    float4 bz1[NFW];                                 // read before the pool stores
#pragma unroll
    for (int n = 0; n < NFW; ++n) bz1[n] = bias(1, n);
#pragma unroll
    for (int fc = 0; fc < Y2FR; ++fc) {
      const s16x8* a0 = (const s16x8*)(Ab + fc * 1024 + lane * 16);
      const s16x8* a1 = (const s16x8*)(Ab + (Y2FR + fc) * 1024 + lane * 16);
      const int col = fc * 16 + p16, gcol = 2 * pc0 - PT + col;
      const bool cok = col < Y2C && (unsigned)gcol < (unsigned)W;
#pragma unroll
      for (int n = 0; n < NFW; ++n) {
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT1; ++t) {
          acc0 = mfma16(w2[n][t], HOIST ? a2h[HOIST ? fc : 0][t] : a0[t * Y2F * 64], acc0);
          acc1 = mfma16(w2[n][t], HOIST ? a2h[HOIST ? Y2FR + fc : 0][t] : a1[t * Y2F * 64], acc1);
        }
        float vm[4];
        const float4 b4 = bz1[n];
        const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
        // bf16 rounding: the values an unfused separable conv would have stored
        const u32x2 y2a = {pack_bf16(acc0[0] + bb[0], acc0[1] + bb[1]), pack_bf16(acc0[2] + bb[2], acc0[3] + bb[3])};
        const u32x2 y2b = {pack_bf16(acc1[0] + bb[0], acc1[1] + bb[1]), pack_bf16(acc1[2] + bb[2], acc1[3] + bb[3])};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t dc = carry[n][fc][e >> 1], da = y2a[e >> 1], db = y2b[e >> 1];
          const float c0 = (e & 1) ? bf_hi(dc) : bf_lo(dc);
          const float v1 = (e & 1) ? bf_hi(da) : bf_lo(da), v2 = (e & 1) ? bf_hi(db) : bf_lo(db);
          float m = r0ok ? c0 : -INFINITY;
          if (r1ok) m = fmaxf(m, v1);
          if (r2ok) m = fmaxf(m, v2);
          vm[e] = cok ? m : -INFINITY;
        }
        carry[n][fc] = y2b;
        if (mode == 2)                               // this wave's pool rows (bf16: lossless here)
          *(u32x2*)(pool + col * PCH + 16 * n + 4 * q16) = (u32x2){pack_bf16(vm[0], vm[1]), pack_bf16(vm[2], vm[3])};
      }
    }
    stamp(q, 4);
    if (mode == 1) continue;                         // warm-up 2: carry (+ PT 0: residual) only
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own pool rows only: no barrier
    // horizontal 3/2 max: pooled column j reads y2 local cols 2j .. 2j+2
    const int j = p16, gj = pc0 + j;
    if (j < PC && gj < a.OW) {
      st_ptr = a.y + (((long)b * a.OH + k) * a.OW + gj) * a.ldy + PCH * w + 4 * q16;
#pragma unroll
      for (int n = 0; n < NFW; ++n) {
        const uint16_t* pp = pool + (2 * j) * PCH + 16 * n + 4 * q16;
        const float4 brv = bias(2, n);
        const float br4[4] = {brv.x, brv.y, brv.z, brv.w};
        const u32x2 c0 = *(const u32x2*)pp, c1 = *(const u32x2*)(pp + PCH), c2 = *(const u32x2*)(pp + 2 * PCH);
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t d0 = c0[e >> 1], d1 = c1[e >> 1], d2 = c2[e >> 1];
          const float m = (e & 1) ? fmaxf(fmaxf(bf_hi(d0), bf_hi(d1)), bf_hi(d2))
                                  : fmaxf(fmaxf(bf_lo(d0), bf_lo(d1)), bf_lo(d2));
          o[e] = m + bf2f(f2bf(acco[n][e] + br4[e]));
        }
        st_val[n] = (u32x2){pack_bf16(o[0], o[1]), pack_bf16(o[2], o[3])};
      }
      st_pend = true;
    }
  }
  if (st_pend) {
#pragma unroll
    for (int n = 0; n < NFW; ++n) *(u32x2*)(st_ptr + 16 * n) = st_val[n];
  }
}

// ===================================================================================================
// Warp-specialized entry block (configs 13 / 113: block2, NWAV = 16). The four dependent stages of a
// step (dw1 -> GEMM1 -> dw2 -> GEMM2 + pool) are split between two wave roles that work on DIFFERENT
// steps at the same time, one workgroup barrier per step:
//   producers (waves NWAV/2..)  iteration i:  dw1(i) -> A1[i&1]   dw2(i-2) -> A2[i&1]   (MFMA depthwise)
//                                             + the x-row DMA of step i+1, + step i's residual input row
//   consumers (waves 0..NWAV/2-1) iteration i: GEMM1(i-1) <- A1 -> y1 ring   GEMM2(i-3) <- A2 + pool
//                                             + residual 1x1/2 GEMM + output of step i-3
// Waves w and w+4 share a SIMD (MI355X_MICROARCH.md: cyclic wave placement), so every SIMD pairs
// depthwise streams with GEMM streams instead of running the phases one after another with every wave
// in the same phase (the round-4 kernel: four barriers per step, ~2k cycles per phase, all of them
// LDS-throughput bound -- profiles/entry_block_ab_r4.txt). Rings: x 8 rows (each step's DMA one
// iteration ahead), y1 6 rows (GEMM1(i-1) writes rows R+4, R+5 of step i-2 while dw2(i-2) reads its
// rows R..R+3), A1 / A2 double-buffered, residual rows in a 4-slot buffer (written by producers at
// step i, read by consumers three iterations later). 13-column strips keep the map at 142 KiB
// (pitch 32 px, no padding). A consumer wave owns 32 output channels of every GEMM (register-resident
// weights); a producer wave owns a quarter of each step's depthwise units.
template <int C0, int C1, int PC, int NWAV, int NCW = NWAV / 2>
struct EbwGeom {
  static constexpr int Y2C = 2 * PC + 1, Y1C = Y2C + 2, XC = Y1C + 2;
  static constexpr int PLP = (XC + 15) / 16 * 16, PLB = PLP * 16;
  static constexpr int XROW = (C0 / 8) * PLB, Y1ROW = (C1 / 8) * PLB;
  static constexpr int KT0 = C0 / 32, KT1 = C1 / 32;
  static constexpr int Y1F = (2 * Y1C + 15) / 16, Y2FR = (Y2C + 15) / 16, Y2F = 2 * Y2FR;
  static constexpr int NC = NCW, NP = NWAV - NCW;  // consumer / producer waves (w, w+4, ... share a SIMD)
  static constexpr int CCH = C1 / NC;                // output channels per consumer wave
  static constexpr int NSL = CCH / 16;               // 16-channel slices per consumer wave
  static constexpr int XDMA = XROW / 1024;
  static constexpr int XR = 8, YR = 6, RS = 4;       // x ring, y1 ring, residual slots
  static constexpr int PCOLS = 16 * Y2FR;
  static constexpr int A1B = KT0 * Y1F * 1024, A2B = KT1 * Y2F * 1024;
  static constexpr int RESB = 16 * C0 * 2;           // one residual input row: 16 strided columns x C0
  static constexpr int BYTES = XR * XROW + YR * Y1ROW + 2 * A1B + 2 * A2B + RS * RESB + NC * PCOLS * CCH * 2 +
                               (KT0 + KT1) * 1024 + 4 * EB_MAX_STEPS;
  static_assert(XROW % 1024 == 0 && RESB % 1024 == 0 && C0 % 32 == 0 && C1 % 64 == 0, "channel tiling");
  static_assert(NP % KT0 == 0 && NP % KT1 == 0, "a producer's depthwise units share one k-step");
  static_assert(BYTES <= 160 * 1024, "LDS");
};

// producers store each depthwise unit as soon as it is computed (true) or after all of the step's
// units (false: more loads in flight, more registers)
#ifndef EBW_EAGER_STORE
#define EBW_EAGER_STORE false
#endif
// CDW: dw2 units per step that every consumer wave computes too (the consumers idle half of an
// iteration while the producers' depthwise is the critical path); the producers keep the rest
template <int C0, int C1, int PC, int NWAV, int NCW, int PT, bool RELU1, bool STAMP, int CDW = 0>
__global__ __launch_bounds__(64 * NWAV, NWAV / 4) void entry_block_ws_kernel(EntryBlockArgs a) {
  using G = EbwGeom<C0, C1, PC, NWAV, NCW>;
  constexpr int KT0 = G::KT0, KT1 = G::KT1, PLB = G::PLB, XROW = G::XROW, Y1ROW = G::Y1ROW, XDMA = G::XDMA;
  constexpr int Y1C = G::Y1C, Y2C = G::Y2C, XC = G::XC, PLP = G::PLP;
  constexpr int Y1F = G::Y1F, Y2F = G::Y2F, Y2FR = G::Y2FR, PCOLS = G::PCOLS;
  constexpr int XR = G::XR, YR = G::YR, RS = G::RS, NC = G::NC, NP = G::NP, CCH = G::CCH, NSL = G::NSL;
  constexpr int U1 = KT0 * Y1F, U2 = KT1 * Y2F;
  constexpr int CU2 = CDW * NC;                      // dw2 units 0..CU2-1: consumers (units w + NC j); the rest: producers
  static_assert(CU2 % KT1 == 0 && CU2 <= U2, "consumer dw2 units keep the producers' k-step per wave");
  constexpr int U1W = (U1 + NP - 1) / NP, U2W = (U2 - CU2 + NP - 1) / NP;
  static_assert(PT == 1, "the residual row 2k is x row R+1 of the step (odd map size: block2)");
  // distinct LDS objects: the compiler may reorder accesses of different regions
  __shared__ __attribute__((aligned(16))) uint8_t s_x[XR * XROW];
  __shared__ __attribute__((aligned(16))) uint8_t s_y1[YR * Y1ROW];
  __shared__ __attribute__((aligned(16))) uint8_t s_a1[2 * G::A1B];
  __shared__ __attribute__((aligned(16))) uint8_t s_a2[2 * G::A2B];
  __shared__ __attribute__((aligned(16))) uint8_t s_res[RS * G::RESB];
  __shared__ __attribute__((aligned(16))) uint16_t s_pool[NC * PCOLS * CCH];
  __shared__ __attribute__((aligned(16))) uint8_t s_dw[(KT0 + KT1) * 1024];
  __shared__ uint32_t s_st[EB_MAX_STEPS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = w < NC;
  const int q16 = lane >> 4, p16 = lane & 15;
  const int H = a.H, W = a.W;
  const int s0 = a.step_off[blockIdx.x], s1 = a.step_off[blockIdx.x + 1];
  if (s0 >= s1 || s1 - s0 > EB_MAX_STEPS) return;

  for (int i = tid; i < s1 - s0; i += 64 * NWAV) {
    const int4 e = a.steps[s0 + i];
    s_st[i] = (uint32_t)e.x | ((uint32_t)e.y << 8) | ((uint32_t)(e.z + 2) << 14) | ((uint32_t)e.w << 23);
  }
  for (int i = tid; i < (KT0 + KT1) * 64; i += 64 * NWAV) {
    const int t = i / 64;
    const u32x4 v = t < KT0 ? *(const u32x4*)((const uint8_t*)a.dwk1 + t * 1024 + (i % 64) * 16)
                            : *(const u32x4*)((const uint8_t*)a.dwk2 + (t - KT0) * 1024 + (i % 64) * 16);
    *(u32x4*)(s_dw + t * 1024 + (i % 64) * 16) = v;
  }
  uint32_t sel[2][4];
  {
    const bool wv = (p16 >> 3) == (q16 & 1);
    const int e = p16 & 7;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t pair = (2u * jp) | ((2u * jp + 1u) << 8);
        const uint32_t val = (e & 1) ? (0x0c0cu | (pair << 16)) : (0x0c0c0000u | pair);
        sel[jp][d] = (wv && (e >> 1) == d) ? val : 0x0c0c0c0cu;
      }
  }
  __syncthreads();
  if (tid == 0) {                                    // ring slot of each step's first x row (rows R+1..R+4)
    int xp = 0, xs = 0;
    for (int i = 0; i < s1 - s0; ++i) {
      const uint32_t e = s_st[i];
      if (((e >> 23) & 3) == 0) { xs = xp; xp += 4; } else { xs += 2; xp += 2; }
      s_st[i] = e | ((uint32_t)(xs & (XR - 1)) << 25);
    }
  }
  EbStepRegs str;                                    // loaded once the ring-slot bits are in (below)
  auto decode = [&](int q, int& b, int& s, int& k, int& mode, int& xs) {
    const uint32_t e = str.get(q - s0);
    b = e & 255; s = (e >> 8) & 63; k = (int)((e >> 14) & 511) - 2; mode = (e >> 23) & 3; xs = (e >> 25) & 7;
  };
  auto dma_for = [&](int q) {                        // producers only: step q's new x rows
    int b, s, k, mode, xs;
    decode(q, b, s, k, mode, xs);
    const int R = 2 * k - PT, gx0 = 2 * s * PC - PT - 2;
    const int r0 = mode == 0 ? R + 1 : R + 3, nr = mode == 0 ? 4 : 2, sl0 = mode == 0 ? xs : xs + 2;
    for (int ii = w - NC; ii < nr * XDMA; ii += NP) {
      const int r = r0 + ii / XDMA, d = ii % XDMA;
      const int slot = d * 64 + lane, plane = slot / PLP, px = slot - plane * PLP;
      const int gx = gx0 + px;
      const bool ok = px < XC && (unsigned)r < (unsigned)H && (unsigned)gx < (unsigned)W;
      const uint8_t* src = ok ? (const uint8_t*)(a.x + (((long)b * H + r) * W + gx) * a.ldx + plane * 8) : eb_zeros;
      glds16_asm(src, s_x + ((sl0 + ii / XDMA) & (XR - 1)) * XROW + d * 1024);
    }
  };
  auto stamp = [&](int it, int ph) {
    if constexpr (STAMP) {
      if (lane == 0 && (w == 0 || w == NC) && blockIdx.x < 8 && it - s0 < 64 && a.stamps)
        a.stamps[((long)blockIdx.x * 64 + (it - s0)) * 5 + ph] = __builtin_amdgcn_s_memtime();
    }
  };

  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));   // prologue loads landed (the waitcnt pass sees it)
  eb_lds_barrier();                                  // ring-slot bits of the step words visible
  str.load(s_st, s1 - s0, lane);

  // The two roles run separate loops with the same trip count and one barrier per iteration (s_barrier
  // counts arrivals, not program counters): each role's registers are live in its own loop only, so
  // the consumers' register-resident weights do not sit in the producers' allocation (and the reverse)
  if (!consumer) {
    dma_for(s0);
    for (int it = s0; it < s1 + 3; ++it) {
      // step `it`'s x rows (their DMA, issued last iteration) must have landed
      __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8));
      eb_lds_barrier();
      stamp(it, 2);
      // =================================================================== producers
      const int pw = w - NC;
      if (it + 1 < s1) dma_for(it + 1);
      u32x2 dv1[U1W][2], dv2[U2W > 0 ? U2W : 1][2];
      uint8_t* d1[U1W];
      uint8_t* d2[U2W > 0 ? U2W : 1];
#pragma unroll
      for (int i = 0; i < U1W; ++i) d1[i] = nullptr;
#pragma unroll
      for (int i = 0; i < U2W; ++i) d2[i] = nullptr;
      if (it < s1) {                                 // dw1(it) -> A1[it & 1]; residual input row of step it
        int b, s, k, mode, xs;
        decode(it, b, s, k, mode, xs);
        const int t1 = pw % KT0;
        uint8_t* const A1 = s_a1 + (it & 1) * G::A1B;
#pragma unroll
        for (int i = 0; i < U1W; ++i) {
          const int u = pw + NP * i;
          if (u < U1) {
            const int f = u / KT0;
            int pi = 16 * f + p16;
            pi = pi < 2 * Y1C ? pi : 2 * Y1C - 1;
            const int rr = pi >= Y1C, col = pi - rr * Y1C;
            const uint8_t* base = s_x + (4 * t1 + (q16 & 1)) * PLB + col * 16;
            auto tap = [&](int g, int ti) {
              return *(const u32x4*)(base + 2 * g * PLB + ((xs + rr + ti / 3) & (XR - 1)) * XROW + (ti % 3) * 16);
            };
            auto ent = [&](int g) {
              return *(const u32x4*)(s_dw + t1 * 1024 + (((g * 16 + p16) * 2) + (q16 >> 1)) * 16);
            };
            eb_dw_mfma_vals<RELU1>(tap, ent, lane, sel, dv1[i]);
            d1[i] = A1 + (t1 * Y1F + f) * 1024;
            if constexpr (EBW_EAGER_STORE) {           // store at once (no deferral)
              eb_dw_store(d1[i], lane, dv1[i]);
              d1[i] = nullptr;
            }
          }
        }
        if (mode == 2) {                             // x row 2k = R + 1 (slot xs), 16 strided columns, C0 channels
          uint8_t* const rs = s_res + (it & (RS - 1)) * G::RESB;
          const int xcol = min(2 * p16 + PT + 2, XC - 1);   // lanes p16 >= PC: unused columns (clamped)
          for (int c = q16 + 4 * pw; c < C0 / 8; c += 4 * NP)   // 16-B chunk c of every column
            *(u32x4*)(rs + (c * 16 + p16) * 16) = *(const u32x4*)(s_x + xs * XROW + c * PLB + xcol * 16);
        }
      }
      if (it - 2 >= s0 && it - 2 < s1) {            // dw2(it - 2) -> A2[it & 1]
        int b, s, k, mode, xs;
        decode(it - 2, b, s, k, mode, xs);
        if (mode >= 1) {
          const int R = 2 * k - PT, t2 = pw % KT1;
          uint8_t* const A2 = s_a2 + (it & 1) * G::A2B;
#pragma unroll
          for (int i = 0; i < U2W; ++i) {
            const int u = CU2 + pw + NP * i;
            if (u < U2) {
              const int f = u / KT1;
              const int rr = f / Y2FR, col = (f % Y2FR) * 16 + p16;
              const int row = R + 1 + rr;
              const uint8_t* base = s_y1 + (4 * t2 + (q16 & 1)) * PLB + col * 16;
              auto tap = [&](int g, int ti) {
                const int yr = row - 1 + ti / 3;
                return *(const u32x4*)(base + 2 * g * PLB + ((yr % YR + YR) % YR) * Y1ROW + (ti % 3) * 16);
              };
              auto ent = [&](int g) {
                return *(const u32x4*)(s_dw + (KT0 + t2) * 1024 + (((g * 16 + p16) * 2) + (q16 >> 1)) * 16);
              };
              eb_dw_mfma_vals<false>(tap, ent, lane, sel, dv2[i]);
              d2[i] = A2 + (t2 * Y2F + f) * 1024;
              if constexpr (EBW_EAGER_STORE) {
                eb_dw_store(d2[i], lane, dv2[i]);
                d2[i] = nullptr;
              }
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < U1W; ++i)
        if (d1[i]) eb_dw_store(d1[i], lane, dv1[i]);
#pragma unroll
      for (int i = 0; i < U2W; ++i)
        if (d2[i]) eb_dw_store(d2[i], lane, dv2[i]);
      stamp(it, 3);
    }
  } else {
    // consumers: this wave's CCH output channels of every GEMM, register-resident
    s16x8 w1[NSL][KT0], w2[NSL][KT1], wr[NSL][KT0];
    float4 bz[3][NSL];
#pragma unroll
    for (int n = 0; n < NSL; ++n) {
#pragma unroll
      for (int t = 0; t < KT0; ++t) {
        w1[n][t] = eb_frag(a.w1, NSL * w + n, KT0, t, lane);
        wr[n][t] = eb_frag(a.wr, NSL * w + n, KT0, t, lane);
      }
#pragma unroll
      for (int t = 0; t < KT1; ++t) w2[n][t] = eb_frag(a.w2, NSL * w + n, KT1, t, lane);
#pragma unroll
      for (int g = 0; g < 3; ++g)
        bz[g][n] = *(const float4*)((g == 0 ? a.b1 : g == 1 ? a.b2 : a.br) + CCH * w + 16 * n + 4 * q16);
    }
    u32x2 carry[NSL][Y2FR];                          // y2 row R+2 of the previous step
    for (int it = s0; it < s1 + 3; ++it) {
      eb_lds_barrier();                              // (no VMEM to wait for: the weights' waits are the compiler's)
      stamp(it, 0);
      if constexpr (CDW > 0) {                       // dw2(it - 2), units w + NC j -> A2[it & 1] (read after the next barrier)
        if (it - 2 >= s0 && it - 2 < s1) {
          int b, s, k, mode, xs;
          decode(it - 2, b, s, k, mode, xs);
          if (mode >= 1) {
            const int R = 2 * k - PT, t2 = w % KT1;
            auto unit = [&](int u) {
              const int f = u / KT1;
              const int rr = f / Y2FR, col = (f % Y2FR) * 16 + p16;
              const int row = R + 1 + rr;
              const uint8_t* base = s_y1 + (4 * t2 + (q16 & 1)) * PLB + col * 16;
              auto tap = [&](int g, int ti) {
                const int yr = row - 1 + ti / 3;
                return *(const u32x4*)(base + 2 * g * PLB + ((yr % YR + YR) % YR) * Y1ROW + (ti % 3) * 16);
              };
              auto ent = [&](int g) {
                return *(const u32x4*)(s_dw + (KT0 + t2) * 1024 + (((g * 16 + p16) * 2) + (q16 >> 1)) * 16);
              };
              u32x2 dv[2];
              eb_dw_mfma_vals<false>(tap, ent, lane, sel, dv);
              eb_dw_store(s_a2 + (it & 1) * G::A2B + (t2 * Y2F + f) * 1024, lane, dv);
            };
            unit(w);
            if constexpr (CDW > 1) unit(w + NC);
          }
        }
      }
      // =================================================================== consumers
      if (it - 1 >= s0 && it - 1 < s1) {             // GEMM1(it - 1) <- A1[(it - 1) & 1] -> y1 ring
        int b, s, k, mode, xs;
        decode(it - 1, b, s, k, mode, xs);
        const int R = 2 * k - PT, pc0 = s * PC;
        const uint8_t* const A1 = s_a1 + ((it - 1) & 1) * G::A1B;
#pragma unroll
        for (int f = 0; f < Y1F; ++f) {
          const int pi = 16 * f + p16;
          const int rr = pi >= Y1C, col = pi - rr * Y1C;
          const int row = R + 2 + rr, gcol = 2 * pc0 - PT - 1 + col;
          const bool ok = (unsigned)row < (unsigned)H && (unsigned)gcol < (unsigned)W;
          s16x8 af[KT0];
#pragma unroll
          for (int t = 0; t < KT0; ++t) af[t] = *(const s16x8*)(A1 + (t * Y1F + f) * 1024 + lane * 16);
#pragma unroll
          for (int n = 0; n < NSL; ++n) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < KT0; ++t) acc = mfma16(w1[n][t], af[t], acc);
            if (pi < 2 * Y1C) {
              const int c = CCH * w + 16 * n + 4 * q16;
              const float4 bv = bz[0][n];
              const float v0 = fmaxf(acc[0] + bv.x, 0.f), v1 = fmaxf(acc[1] + bv.y, 0.f);
              const float v2 = fmaxf(acc[2] + bv.z, 0.f), v3 = fmaxf(acc[3] + bv.w, 0.f);
              const u32x2 o = ok ? (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)} : (u32x2){0u, 0u};
              *(u32x2*)(s_y1 + ((row % YR + YR) % YR) * Y1ROW + (c / 8) * PLB + col * 16 + (c & 7) * 2) = o;
            }
          }
        }
      }
      if (it - 3 >= s0 && it - 3 < s1) {             // GEMM2(it - 3) <- A2[(it - 1) & 1] + pool + residual
        int b, s, k, mode, xs;
        decode(it - 3, b, s, k, mode, xs);
        if (mode >= 1) {
          const int R = 2 * k - PT, pc0 = s * PC;
          const uint8_t* const A2 = s_a2 + ((it - 1) & 1) * G::A2B;
          uint16_t* const pool = s_pool + w * (PCOLS * CCH);
          const bool r0ok = (unsigned)R < (unsigned)H && mode == 2, r1ok = (unsigned)(R + 1) < (unsigned)H;
          const bool r2ok = (unsigned)(R + 2) < (unsigned)H;
#pragma unroll
          for (int fc = 0; fc < Y2FR; ++fc) {
            const int col = fc * 16 + p16, gcol = 2 * pc0 - PT + col;
            const bool cok = col < Y2C && (unsigned)gcol < (unsigned)W;
            s16x8 a0[KT1], a1f[KT1];
#pragma unroll
            for (int t = 0; t < KT1; ++t) {
              a0[t] = *(const s16x8*)(A2 + (t * Y2F + fc) * 1024 + lane * 16);
              a1f[t] = *(const s16x8*)(A2 + (t * Y2F + Y2FR + fc) * 1024 + lane * 16);
            }
#pragma unroll
            for (int n = 0; n < NSL; ++n) {
              f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int t = 0; t < KT1; ++t) {
                acc0 = mfma16(w2[n][t], a0[t], acc0);
                acc1 = mfma16(w2[n][t], a1f[t], acc1);
              }
              const float4 b4 = bz[1][n];
              const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
              const u32x2 y2a = {pack_bf16(acc0[0] + bb[0], acc0[1] + bb[1]), pack_bf16(acc0[2] + bb[2], acc0[3] + bb[3])};
              const u32x2 y2b = {pack_bf16(acc1[0] + bb[0], acc1[1] + bb[1]), pack_bf16(acc1[2] + bb[2], acc1[3] + bb[3])};
              float vm[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const uint32_t dc = carry[n][fc][e >> 1], da = y2a[e >> 1], db = y2b[e >> 1];
                const float c0 = (e & 1) ? bf_hi(dc) : bf_lo(dc);
                const float v1 = (e & 1) ? bf_hi(da) : bf_lo(da), v2 = (e & 1) ? bf_hi(db) : bf_lo(db);
                float m = r0ok ? c0 : -INFINITY;
                if (r1ok) m = fmaxf(m, v1);
                if (r2ok) m = fmaxf(m, v2);
                vm[e] = cok ? m : -INFINITY;
              }
              carry[n][fc] = y2b;
              if (mode == 2)
                *(u32x2*)(pool + col * CCH + 16 * n + 4 * q16) = (u32x2){pack_bf16(vm[0], vm[1]), pack_bf16(vm[2], vm[3])};
            }
          }
          if (mode == 2) {
            // residual 1x1/2 conv of pooled row k from the staged input row (written three iterations ago)
            const uint8_t* const rs = s_res + ((it - 3) & (RS - 1)) * G::RESB;
            f32x4 racc[NSL];
#pragma unroll
            for (int n = 0; n < NSL; ++n) {
              racc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int t = 0; t < KT0; ++t)
                racc[n] = mfma16(wr[n][t], *(const s16x8*)(rs + ((4 * t + q16) * 16 + p16) * 16), racc[n]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own pool rows only
            const int j = p16, gj = pc0 + j;
            if (j < PC && gj < a.OW) {
#pragma unroll
              for (int n = 0; n < NSL; ++n) {
                const uint16_t* pp = pool + (2 * j) * CCH + 16 * n + 4 * q16;
                const float4 brv = bz[2][n];
                const float br4[4] = {brv.x, brv.y, brv.z, brv.w};
                const u32x2 c0 = *(const u32x2*)pp, c1 = *(const u32x2*)(pp + CCH), c2 = *(const u32x2*)(pp + 2 * CCH);
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const uint32_t d0 = c0[e >> 1], d1v = c1[e >> 1], d2v = c2[e >> 1];
                  const float m = (e & 1) ? fmaxf(fmaxf(bf_hi(d0), bf_hi(d1v)), bf_hi(d2v))
                                          : fmaxf(fmaxf(bf_lo(d0), bf_lo(d1v)), bf_lo(d2v));
                  o[e] = m + bf2f(f2bf(racc[n][e] + br4[e]));
                }
                *(u32x2*)(a.y + (((long)b * a.OH + k) * a.OW + gj) * a.ldy + CCH * w + 16 * n + 4 * q16) =
                    (u32x2){pack_bf16(o[0], o[1]), pack_bf16(o[2], o[3])};
              }
            }
          }
        }
      }
      stamp(it, 1);
    }
  }
}

// (C0, C1, PC, NFW, PT, RELU1, DWM, OCC = workgroups per CU) per id: 0 = block2 (147x147x64 -> 74x74x128), 1 = block3
// (74x74x128 -> 37x37x256, the asymmetric 74 -> 37 pool: leading pad 0); 100 + id: the same
// with per-phase s_memtime stamps (EntryBlockArgs.stamps; diagnostics only); 2, 3: 0, 1 with the
// depthwise convs on the matrix cores (block-diagonal operand) instead of the VALU (block2 only:
// block3's LDS map has no room for the larger entries); 4, 5: block2
// with 13-column strips, small enough (LDS, <= 128 VGPRs) for two workgroups per CU. Measured and removed (round 5,
// profiles/entry_block3_r5.txt): block3 as 16 waves of one slice (VALU / MFMA depthwise: 328 / 246 us)
// and block3 with the MFMA depthwise (378 us) against config 1's 188 us -- all spill (78 / 56 / 91 VGPRs)
// 13 / 113: block2 warp-specialized (entry_block_ws_kernel, 16 waves: 8 producers run the depthwise of
// later steps while 8 consumers run the GEMMs of earlier ones; 13-column strips), plain / stamped.
// 210.5 us against config 2's 216.2 / config 5's 208.4 (profiles/entry_block_ab_r4.txt, round 5): the
// producers' LDS-latency-bound depthwise (6,336 cycles per step) stays the critical path, consumers idle
// 37 %. The 8-wave build (4 + 4) ran 280.4 us (producers 10,252 cycles per step) and was removed.
// 15 / 115 (block2's default): config 13 with every consumer wave also computing one of the step's 16
// dw2 units (CDW = 1): 191.8 vs 199.2 us, iteration 7,212 -> 6,636 cycles (consumers busy 4,700,
// producers 5,572), bench +1.0 % in 3 of 3 pairs. Measured and removed (profiles/entry_block_ab_r4.txt):
// 4 consumer + 12 producer waves (227.0 us: the 32-channel consumers spill 32 VGPRs), two dw2 units per
// consumer (215.8 us: consumers 6,168 busy with 14 VGPRs spilled), and the residual-row copy moved to the
// consumers as well (iteration 6,732 vs 6,676, bench -0.2 %).
#define KDL_EBW_CONFIGS(X) \
  X(13, 64, 128, 13, 16, 8, 1, false, 0) \
  X(15, 64, 128, 13, 16, 8, 1, false, 1) \
  X(113, 64, 128, 13, 16, 8, 1, false, 0) \
  X(115, 64, 128, 13, 16, 8, 1, false, 1)

#define KDL_EB_CONFIGS(X)                          \
  X(0, 64, 128, 15, 1, 1, false, false, 1)         \
  X(1, 128, 256, 13, 2, 0, true, false, 1)         \
  X(2, 64, 128, 15, 1, 1, false, true, 1)          \
  X(4, 64, 128, 13, 1, 1, false, false, 2)         \
  X(5, 64, 128, 13, 1, 1, false, true, 2)          \
  X(100, 64, 128, 15, 1, 1, false, false, 1)       \
  X(101, 128, 256, 13, 2, 0, true, false, 1)       \
  X(102, 64, 128, 15, 1, 1, false, true, 1)        \
  X(104, 64, 128, 13, 1, 1, false, false, 2)       \
  X(105, 64, 128, 13, 1, 1, false, true, 2)

int entry_block_config(int cfg, int* c0, int* c1, int* pc, int* lds, int* occ) {
  switch (cfg) {
#define KDL_EBINFO(id, c0_, c1_, pc_, nfw, pt, r_, dwm, occ_) \
  case id: *c0 = c0_; *c1 = c1_; *pc = pc_; *lds = EbGeom<c0_, c1_, pc_, nfw, dwm>::BYTES; *occ = occ_; return 0;
    KDL_EB_CONFIGS(KDL_EBINFO)
#undef KDL_EBINFO
#define KDL_EBWINFO(id, c0_, c1_, pc_, nw, nc, pt, r_, cdw) \
  case id: *c0 = c0_; *c1 = c1_; *pc = pc_; *lds = EbwGeom<c0_, c1_, pc_, nw, nc>::BYTES; *occ = 1; return 0;
    KDL_EBW_CONFIGS(KDL_EBWINFO)
#undef KDL_EBWINFO
    default: return -1;
  }
}

static int eb_pad(int cfg) {
  switch (cfg) {
#define KDL_EBPAD(id, c0_, c1_, pc_, nfw, pt, r_, dwm, occ_) case id: return pt;
    KDL_EB_CONFIGS(KDL_EBPAD)
#undef KDL_EBPAD
#define KDL_EBWPAD(id, c0_, c1_, pc_, nw, nc, pt, r_, cdw) case id: return pt;
    KDL_EBW_CONFIGS(KDL_EBWPAD)
#undef KDL_EBWPAD
    default: return -1;
  }
}

hipError_t entry_block(int cfg, const EntryBlockArgs& a, hipStream_t s) {
  int c0, c1, pc, lds, occ;
  if (entry_block_config(cfg, &c0, &c1, &pc, &lds, &occ) != 0 || a.ldx != c0 || a.ldy != c1 || a.grid < 1 ||
      a.OH != (a.H - 1) / 2 + 1 || a.OW != (a.W - 1) / 2 + 1 || a.H != a.W || !a.steps || !a.step_off ||
      a.B > 256)                                     // the packed LDS step word holds an 8-bit image index
    return hipErrorInvalidValue;
  if (eb_pad(cfg) != (a.H % 2)) return hipErrorInvalidValue;   // TF 'same': leading pad 1 iff odd size
  switch (cfg) {
#define KDL_EBCASE(id, c0_, c1_, pc_, nfw, pt, r_, dwm, occ_)                                               \
  case id:                                                                                                 \
    hipLaunchKernelGGL((entry_block_kernel<c0_, c1_, pc_, nfw, pt, r_, (id >= 100), dwm, occ_>), dim3(a.grid), \
                       dim3(64 * EbGeom<c0_, c1_, pc_, nfw, dwm>::NW), lds, s, a);                               \
    break;
    KDL_EB_CONFIGS(KDL_EBCASE)
#undef KDL_EBCASE
#define KDL_EBWCASE(id, c0_, c1_, pc_, nw, nc, pt, r_, cdw)                                                      \
  case id:                                                                                            \
    hipLaunchKernelGGL((entry_block_ws_kernel<c0_, c1_, pc_, nw, nc, pt, r_, (id >= 100), cdw>), dim3(a.grid),  \
                       dim3(64 * nw), 0, s, a);   /* static LDS */                                   \
    break;
    KDL_EBW_CONFIGS(KDL_EBWCASE)
#undef KDL_EBWCASE
  }
  return hipGetLastError();
}

}  // namespace kdl
