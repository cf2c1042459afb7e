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

template <int C0, int C1, int PC>
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
  static constexpr int NW = C1 / 16;                // waves (one 16-channel output slice each)
  static constexpr int XDMA = XROW / 1024;          // 1 KiB DMA instructions per x row
  // LDS map
  static constexpr int OFF_X = 0;
  static constexpr int OFF_Y1 = OFF_X + 4 * XROW;
  static constexpr int OFF_A1 = OFF_Y1 + 4 * Y1ROW;
  static constexpr int OFF_A2 = OFF_A1 + KT0 * Y1F * 1024;
  static constexpr int OFF_P = OFF_A2 + KT1 * Y2F * 1024;   // per-wave pool rows: [NW][16*Y2FR cols][16 ch] fp32
  static constexpr int BYTES = OFF_P + NW * 16 * Y2FR * 64;
  static_assert(XROW % 1024 == 0, "whole DMA instructions per x row");
  static_assert(C0 % 32 == 0 && C1 % 32 == 0 && NW <= 16, "channel tiling");
};

// four bf16 pairs (two 16-B taps a, b of one pixel: channels c..c+7) -> dot2 operands
// (a[c], b[c]) / (a[c+1], b[c+1]) per channel pair
__device__ __forceinline__ uint32_t eb_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ uint32_t eb_hi(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }
__device__ __forceinline__ float eb_dot(uint32_t x, uint32_t w, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, x), __builtin_bit_cast(bf16x2, w), c, false);
}

// depthwise 3x3 of 8 channels of one pixel: taps t[0..8] (16 B each), weights wq[j][e]: tap pair j
// (taps 2j, 2j+1; tap 9 = 0) for channel e, bf16x2. Returns the 8 outputs as bf16 (MFMA operand).
template <bool RELU>
__device__ __forceinline__ s16x8 eb_dw8(const u32x4 (&t)[9], const uint32_t (&wq)[5][8]) {
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    u32x4 a = t[2 * j];
    u32x4 b = j < 4 ? t[2 * j + 1] : (u32x4){0u, 0u, 0u, 0u};
    if constexpr (RELU) {
#pragma unroll
      for (int d = 0; d < 4; ++d) { a[d] = relu_bf16x2(a[d]); b[d] = relu_bf16x2(b[d]); }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      acc[2 * d] = eb_dot(eb_lo(a[d], b[d]), wq[j][2 * d], acc[2 * d]);
      acc[2 * d + 1] = eb_dot(eb_hi(a[d], b[d]), wq[j][2 * d + 1], acc[2 * d + 1]);
    }
  }
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = pack_bf16(acc[2 * d], acc[2 * d + 1]);
  return __builtin_bit_cast(s16x8, o);
}

// per-lane depthwise weights of channels c..c+7 as tap-pair bf16x2 words (from [9][C] fp32)
__device__ __forceinline__ void eb_load_dw(const float* w, int C, int c, uint32_t (&wq)[5][8]) {
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a = w[(2 * j) * C + c + e];
      const float b = j < 4 ? w[(2 * j + 1) * C + c + e] : 0.f;
      wq[j][e] = pack_bf16(a, b);
    }
}

__device__ __forceinline__ s16x8 eb_frag(const uint16_t* wp, int nf, int kt, int t, int lane) {
  return *(const s16x8*)(wp + ((long)(nf * kt + t) * 64 + lane) * 8);
}

template <int C0, int C1, int PC, bool RELU1>
__global__ __launch_bounds__(64 * (C1 / 16)) void entry_block_kernel(EntryBlockArgs a) {
  using G = EbGeom<C0, C1, PC>;
  constexpr int NW = G::NW, KT0 = G::KT0, KT1 = G::KT1;
  constexpr int PLB = G::PLB, XROW = G::XROW, Y1ROW = G::Y1ROW;
  constexpr int Y1C = G::Y1C, Y2C = G::Y2C, XC = G::XC, PLP = G::PLP;
  constexpr int Y1F = G::Y1F, Y2F = G::Y2F, Y2FR = G::Y2FR;
  constexpr int U1 = KT0 * Y1F, U2 = KT1 * Y2F;      // depthwise units (fragment x k-step)
  constexpr int U1W = (U1 + NW - 1) / NW, U2W = (U2 + NW - 1) / NW;
  static_assert(NW % KT0 == 0 && NW % KT1 == 0, "a wave's depthwise units share one k-step");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q16 = lane >> 4, p16 = lane & 15;
  const int H = a.H, W = a.W;
  const int s0 = a.step_off[blockIdx.x], s1 = a.step_off[blockIdx.x + 1];
  if (s0 >= s1) return;                              // uniform: this workgroup has no work

  // ---- register-resident weights of this wave's 16 output channels
  s16x8 w1[KT0], wr[KT0], w2[KT1];
#pragma unroll
  for (int t = 0; t < KT0; ++t) { w1[t] = eb_frag(a.w1, w, KT0, t, lane); wr[t] = eb_frag(a.wr, w, KT0, t, lane); }
#pragma unroll
  for (int t = 0; t < KT1; ++t) w2[t] = eb_frag(a.w2, w, KT1, t, lane);
  const int nch = 16 * w + 4 * q16;                  // this lane's 4 accumulator channels
  const float4 bias1 = *(const float4*)(a.b1 + nch);
  const float4 bias2 = *(const float4*)(a.b2 + nch);
  const float4 biasr = *(const float4*)(a.br + nch);
  // depthwise weights: every unit of this wave uses k-step w % KT
  const int t1 = w % KT0, t2 = w % KT1;
  uint32_t dq1[5][8], dq2[5][8];
  eb_load_dw(a.dw1, C0, 32 * t1 + 8 * q16, dq1);
  eb_load_dw(a.dw2, C1, 32 * t2 + 8 * q16, dq2);

  uint8_t* const xr = smem + G::OFF_X;
  uint8_t* const y1r = smem + G::OFF_Y1;
  uint8_t* const A1 = smem + G::OFF_A1;
  uint8_t* const A2 = smem + G::OFF_A2;
  float* const pool = (float*)(smem + G::OFF_P) + w * (16 * Y2FR * 16);

  // ---- x row DMA: row r of image b, strip columns starting at global col gx0, into ring slot r & 3
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
  auto decode = [&](int q, int& b, int& s, int& k, int& mode) {
    const int4 e = a.steps[q];
    b = e.x; s = e.y; k = e.z; mode = e.w;
  };
  // rows the step needs that its predecessor did not load: R = 2k-1; y1 rows R+2, R+3 need
  // x rows R+1..R+4 (a run's first step loads all four)
  auto dma_for = [&](int q) {
    int b, s, k, mode;
    decode(q, b, s, k, mode);
    const int R = 2 * k - 1;
    const int gx0 = 2 * s * PC - 3;
    if (mode == 0) dma_rows(b, gx0, R + 1, 4);
    else dma_rows(b, gx0, R + 3, 2);
  };

  // ---- y2 row carried between steps (row 2k-1 of the next step): 2 fragments per row slot
  float carry[Y2FR][4];
  // deferred output store of the previous step
  bool st_pend = false;
  uint16_t* st_ptr = nullptr;
  u32x2 st_val = {0u, 0u};

  dma_for(s0);
  for (int q = s0; q < s1; ++q) {
    int b, s, k, mode;
    decode(q, b, s, k, mode);
    const int R = 2 * k - 1;                         // pooled row k pools y2 rows R, R+1, R+2
    const int pc0 = s * PC;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                 // B0: x rows landed; previous step done

    // ---- P1: depthwise 1 -> A1; residual operands (x row 2k = R+1, columns 2j)
#pragma unroll
    for (int i = 0; i < U1W; ++i) {
      const int u = w + NW * i;
      if (u < U1) {
        const int f = u / KT0;                       // t = u % KT0 == t1
        int pi = 16 * f + p16;
        pi = pi < 2 * Y1C ? pi : 2 * Y1C - 1;
        const int rr = pi >= Y1C, col = pi - rr * Y1C;   // y1 row R+2+rr, local col (x local col+1)
        const int row = R + 2 + rr;
        const uint8_t* base = xr + (32 * t1 / 8 + q16) * PLB + col * 16;
        u32x4 tp[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            tp[dy * 3 + dx] = *(const u32x4*)(base + ((row - 1 + dy) & 3) * XROW + dx * 16);
        *(s16x8*)(A1 + (t1 * Y1F + f) * 1024 + lane * 16) = eb_dw8<RELU1>(tp, dq1);
      }
    }
    s16x8 xres[KT0];
    if (mode == 2) {
#pragma unroll
      for (int t = 0; t < KT0; ++t)
        xres[t] = *(const s16x8*)(xr + ((R + 1) & 3) * XROW + (4 * t + q16) * PLB + (2 * p16 + 3) * 16);
    }
    __syncthreads();                                 // B1: A1 complete; x ring free for the next DMA

    if (st_pend) {
      *(u32x2*)st_ptr = st_val;
      st_pend = false;
    }
    if (q + 1 < s1) dma_for(q + 1);

    // ---- P2: GEMM1 (+ bias, ReLU) -> y1 ring rows R+2, R+3; residual GEMM
    {
#pragma unroll
      for (int f = 0; f < Y1F; ++f) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT0; ++t) acc = mfma16(w1[t], *(const s16x8*)(A1 + (t * Y1F + f) * 1024 + lane * 16), acc);
        const int pi = 16 * f + p16;
        if (pi < 2 * Y1C) {
          const int rr = pi >= Y1C, col = pi - rr * Y1C;
          const int row = R + 2 + rr, gcol = 2 * pc0 - 2 + col;
          const bool ok = (unsigned)row < (unsigned)H && (unsigned)gcol < (unsigned)W;
          const float v0 = fmaxf(acc[0] + bias1.x, 0.f), v1 = fmaxf(acc[1] + bias1.y, 0.f);
          const float v2 = fmaxf(acc[2] + bias1.z, 0.f), v3 = fmaxf(acc[3] + bias1.w, 0.f);
          const u32x2 o = ok ? (u32x2){pack_bf16(v0, v1), pack_bf16(v2, v3)} : (u32x2){0u, 0u};
          *(u32x2*)(y1r + (row & 3) * Y1ROW + (nch / 8) * PLB + col * 16 + (nch & 7) * 2) = o;
        }
      }
    }
    f32x4 accr = {0.f, 0.f, 0.f, 0.f};
    if (mode == 2) {
#pragma unroll
      for (int t = 0; t < KT0; ++t) accr = mfma16(wr[t], xres[t], accr);
    }
    __syncthreads();                                 // B2: y1 rows R+2, R+3 written

    if (mode == 0) continue;                         // warm-up 1: y1 only
    // ---- P3: depthwise 2 -> A2 (y2 rows R+1, R+2: fragments [row][col/16])
#pragma unroll
    for (int i = 0; i < U2W; ++i) {
      const int u = w + NW * i;
      if (u < U2) {
        const int f = u / KT1;                       // t = t2
        const int rr = f / Y2FR, col = (f % Y2FR) * 16 + p16;   // y2 local col (y1 local col+1)
        const int row = R + 1 + rr;
        const uint8_t* base = y1r + (32 * t2 / 8 + q16) * PLB + col * 16;
        u32x4 tp[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx)
            tp[dy * 3 + dx] = *(const u32x4*)(base + ((row - 1 + dy) & 3) * Y1ROW + dx * 16);
        *(s16x8*)(A2 + (t2 * Y2F + f) * 1024 + lane * 16) = eb_dw8<false>(tp, dq2);
      }
    }
    __syncthreads();                                 // B3: A2 complete

    // ---- P4: GEMM2 + bias -> bf16 values; vertical max with the carried row; pool; residual
    float vm[Y2FR][4];
#pragma unroll
    for (int fc = 0; fc < Y2FR; ++fc) {
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KT1; ++t) {
        acc0 = mfma16(w2[t], *(const s16x8*)(A2 + (t * Y2F + fc) * 1024 + lane * 16), acc0);
        acc1 = mfma16(w2[t], *(const s16x8*)(A2 + (t * Y2F + Y2FR + fc) * 1024 + lane * 16), acc1);
      }
      const int col = fc * 16 + p16, gcol = 2 * pc0 - 1 + col;
      const bool cok = col < Y2C && (unsigned)gcol < (unsigned)W;
      const bool r0ok = (unsigned)R < (unsigned)H, r1ok = (unsigned)(R + 1) < (unsigned)H;
      const bool r2ok = (unsigned)(R + 2) < (unsigned)H;
      const float bb[4] = {bias2.x, bias2.y, bias2.z, bias2.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // bf16 round trip: the same values an unfused sepconv would have stored
        const float v1 = bf2f(f2bf(acc0[e] + bb[e])), v2 = bf2f(f2bf(acc1[e] + bb[e]));
        float m = -INFINITY;
        if (r0ok && mode == 2) m = carry[fc][e];
        if (r1ok) m = fmaxf(m, v1);
        if (r2ok) m = fmaxf(m, v2);
        vm[fc][e] = cok ? m : -INFINITY;
        carry[fc][e] = v2;
      }
    }
    if (mode == 1) continue;                         // warm-up 2: carry only
    // vertical maxima -> this wave's pool rows (16 channels x 16*Y2FR cols, fp32), then the
    // horizontal 3/2 max: pooled column j reads y2 local cols 2j .. 2j+2
#pragma unroll
    for (int fc = 0; fc < Y2FR; ++fc)
      *(float4*)(pool + (fc * 16 + p16) * 16 + 4 * q16) = (float4){vm[fc][0], vm[fc][1], vm[fc][2], vm[fc][3]};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own rows only: no barrier
    const int j = p16, gj = pc0 + j;
    if (j < PC && gj < a.OW) {
      float m[4];
      const float4 c0 = *(const float4*)(pool + (2 * j) * 16 + 4 * q16);
      const float4 c1 = *(const float4*)(pool + (2 * j + 1) * 16 + 4 * q16);
      const float4 c2 = *(const float4*)(pool + (2 * j + 2) * 16 + 4 * q16);
      m[0] = fmaxf(fmaxf(c0.x, c1.x), c2.x); m[1] = fmaxf(fmaxf(c0.y, c1.y), c2.y);
      m[2] = fmaxf(fmaxf(c0.z, c1.z), c2.z); m[3] = fmaxf(fmaxf(c0.w, c1.w), c2.w);
      const float r0 = bf2f(f2bf(accr[0] + biasr.x)), r1 = bf2f(f2bf(accr[1] + biasr.y));
      const float r2 = bf2f(f2bf(accr[2] + biasr.z)), r3 = bf2f(f2bf(accr[3] + biasr.w));
      st_val = (u32x2){pack_bf16(m[0] + r0, m[1] + r1), pack_bf16(m[2] + r2, m[3] + r3)};
      st_ptr = a.y + (((long)b * a.OH + k) * a.OW + gj) * a.ldy + nch;
      st_pend = true;
    }
  }
  if (st_pend) *(u32x2*)st_ptr = st_val;
}

// (C0, C1, PC, RELU1) per id
#define KDL_EB_CONFIGS(X) \
  X(0, 64, 128, 15, false)

int entry_block_config(int cfg, int* c0, int* c1, int* pc, int* lds) {
  switch (cfg) {
#define KDL_EBINFO(id, c0_, c1_, pc_, r_) \
  case id: *c0 = c0_; *c1 = c1_; *pc = pc_; *lds = EbGeom<c0_, c1_, pc_>::BYTES; return 0;
    KDL_EB_CONFIGS(KDL_EBINFO)
#undef KDL_EBINFO
    default: return -1;
  }
}

hipError_t entry_block(int cfg, const EntryBlockArgs& a, hipStream_t s) {
  int c0, c1, pc, lds;
  if (entry_block_config(cfg, &c0, &c1, &pc, &lds) != 0 || a.ldx != c0 || a.ldy != c1 || a.grid < 1 ||
      a.OH != (a.H - 1) / 2 + 1 || a.OW != (a.W - 1) / 2 + 1 || (a.H % 2) != 1 || !a.steps || !a.step_off)
    return hipErrorInvalidValue;   // pad 1 on every side (odd H, W): the 147 -> 74 entry block
  switch (cfg) {
#define KDL_EBCASE(id, c0_, c1_, pc_, r_)                                                     \
  case id:                                                                                 \
    hipLaunchKernelGGL((entry_block_kernel<c0_, c1_, pc_, r_>), dim3(a.grid), dim3(64 * (c1_ / 16)), lds, s, a); \
    break;
    KDL_EB_CONFIGS(KDL_EBCASE)
#undef KDL_EBCASE
  }
  return hipGetLastError();
}

}  // namespace kdl
