// Classifier tails for 1000-class heads (ResNet-50 / ViT / EfficientNet):
// global average pool, then a dense layer computed once for the whole batch so
// each weight is read once per 8 images (the per-image fused head of
// pool_head.hip would stream the 8 MB fp32 FC matrix once per image).
#include "common.h"
#include "launch.h"

namespace kdl {

// grid (ceil(F / 8 / GAP_CG), B): a block owns GAP_CG 8-channel chunks of one image; its GAP_PARTS
// thread groups each sum every GAP_PARTS-th pixel (four independent 16-byte loads in flight per
// thread), then the partial sums meet in LDS. The round-1 form (one block per image, every thread
// walking all HW pixels of its chunks in one dependent chain) ran EfficientNet-B7's 19x19x2560 pool
// in 200 us on 32 of the 256 CUs, for 59 MB of reads (tools/layer_profile.py, round 5).
constexpr int GAP_CG = 32, GAP_PARTS = 8;
template <int DT>
__global__ __launch_bounds__(GAP_CG * GAP_PARTS) void gap_kernel(GapArgs a) {
  using E = Elt<DT>;
  __shared__ float red[GAP_PARTS][GAP_CG][9];        // +1: no bank conflicts on the reduction reads
  const int b = blockIdx.y, c = threadIdx.x % GAP_CG, part = threadIdx.x / GAP_CG;
  const int F8 = a.F / 8, c8 = blockIdx.x * GAP_CG + c;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add = [&](const u32x4 v) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      s[2 * d] += E::lo(v[d]);
      s[2 * d + 1] += E::hi(v[d]);
    }
  };
  if (c8 < F8) {
    const uint16_t* xb = a.x + (long)b * a.HW * a.ldx + c8 * 8;
    int p = part;
    for (; p + 3 * GAP_PARTS < a.HW; p += 4 * GAP_PARTS) {
      const u32x4 v0 = *(const u32x4*)(xb + (long)p * a.ldx);
      const u32x4 v1 = *(const u32x4*)(xb + (long)(p + GAP_PARTS) * a.ldx);
      const u32x4 v2 = *(const u32x4*)(xb + (long)(p + 2 * GAP_PARTS) * a.ldx);
      const u32x4 v3 = *(const u32x4*)(xb + (long)(p + 3 * GAP_PARTS) * a.ldx);
      add(v0); add(v1); add(v2); add(v3);
    }
    for (; p < a.HW; p += GAP_PARTS) add(*(const u32x4*)(xb + (long)p * a.ldx));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[part][c][e] = s[e];
  __syncthreads();
  if (part != 0 || c8 >= F8) return;
  const float inv = 1.f / (float)a.HW;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < GAP_PARTS; ++q) t += red[q][c][e];   // fixed order: deterministic
    s[e] = t * inv;
  }
  if (a.y) {
    float4* o = (float4*)(a.y + (long)b * a.F + c8 * 8);
    o[0] = (float4){s[0], s[1], s[2], s[3]};
    o[1] = (float4){s[4], s[5], s[6], s[7]};
  }
  if (a.yb) {
    u32x4 o;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = E::pack(s[2 * d], s[2 * d + 1]);
    *(u32x4*)(a.yb + (long)b * a.F + c8 * 8) = o;
  }
}

hipError_t gap(const GapArgs& a, hipStream_t s) {
  if (a.F % 8 != 0 || a.ldx % 8 != 0 || a.B <= 0 || a.HW <= 0 || a.dt < 0 || a.dt > 1) return hipErrorInvalidValue;
  const dim3 grid((a.F / 8 + GAP_CG - 1) / GAP_CG, a.B);
  if (a.dt) hipLaunchKernelGGL(gap_kernel<1>, grid, dim3(GAP_CG * GAP_PARTS), 0, s, a);
  else hipLaunchKernelGGL(gap_kernel<0>, grid, dim3(GAP_CG * GAP_PARTS), 0, s, a);
  return hipGetLastError();
}

// block = 64 outputs x 4 k-slices, 8 images per block (grid.y over image groups).
constexpr int FC_IMG = 8;
__global__ __launch_bounds__(256) void fc_kernel(FcArgs a) {
  extern __shared__ __attribute__((aligned(16))) float fsm[];   // [FC_IMG][F] then [4][FC_IMG][64]
  const int tid = threadIdx.x;
  const int o = tid & 63, sl = tid >> 6;
  const int n = blockIdx.x * 64 + o;
  const int b0 = blockIdx.y * FC_IMG;
  const int nb = min(FC_IMG, a.B - b0);
  for (int i = tid; i < FC_IMG * a.F; i += 256) {
    const int bi = i / a.F;
    fsm[i] = bi < nb ? a.x[(long)(b0 + bi) * a.F + (i - bi * a.F)] : 0.f;
  }
  __syncthreads();
  float acc[FC_IMG];
#pragma unroll
  for (int i = 0; i < FC_IMG; ++i) acc[i] = 0.f;
  const int klen = (a.F + 3) / 4;
  const int k0 = sl * klen, k1 = min(a.F, k0 + klen);
  if (n < a.N) {
    for (int k = k0; k < k1; ++k) {
      const float w = a.w[(long)k * a.N + n];
#pragma unroll
      for (int i = 0; i < FC_IMG; ++i) acc[i] += fsm[i * a.F + k] * w;
    }
  }
  __syncthreads();
  float* red = fsm;
#pragma unroll
  for (int i = 0; i < FC_IMG; ++i) red[(sl * FC_IMG + i) * 64 + o] = acc[i];
  __syncthreads();
  if (sl == 0 && n < a.N) {
    for (int i = 0; i < nb; ++i) {
      float v = a.bias[n] + red[i * 64 + o] + red[(FC_IMG + i) * 64 + o] + red[(2 * FC_IMG + i) * 64 + o] +
                red[(3 * FC_IMG + i) * 64 + o];
      if (a.relu) v = fmaxf(v, 0.f);
      a.out[(long)(b0 + i) * a.N + n] = v;
    }
  }
}

hipError_t fc(const FcArgs& a, hipStream_t s) {
  if (a.B <= 0 || a.F <= 0 || a.N <= 0) return hipErrorInvalidValue;
  const size_t smem = (size_t)FC_IMG * a.F * sizeof(float);
  if (smem > 160 * 1024 || smem < (size_t)4 * FC_IMG * 64 * sizeof(float)) return hipErrorInvalidValue;
  const dim3 grid((a.N + 63) / 64, (a.B + FC_IMG - 1) / FC_IMG);
  hipLaunchKernelGGL(fc_kernel, grid, dim3(256), smem, s, a);
  return hipGetLastError();
}

// One block = one 16-column N fragment x up to 64 rows (4 M fragments); the 4
// waves split K four ways (each streams its B fragments and the A rows straight
// from global/L2: every operand is used once per block) and the partial
// accumulators are summed through LDS. 63 blocks for a 1000-class head.
template <int DT>
__global__ __launch_bounds__(256) void fc_mfma_kernel(FcMfmaArgs a) {
  using E = Elt<DT>;
  __shared__ __attribute__((aligned(16))) float red[4][4][64][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nf = blockIdx.x, r0 = blockIdx.y * 64;
  const int KT = a.F >> 5;
  const int kt0 = wave * KT / 4, kt1 = (wave + 1) * KT / 4;
  const int rows = min(64, ((a.B + 15) & ~15) - r0);
  const int nm = rows >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const uint16_t* wb = a.wp + ((long)nf * KT) * 512 + lane * 8;
  const uint16_t* xb = a.xb + (long)(r0 + (lane & 15)) * a.F + 8 * (lane >> 4);
#pragma unroll 4
  for (int kt = kt0; kt < kt1; ++kt) {
    const s16x8 bf = *(const s16x8*)(wb + (long)kt * 512);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < nm) {
        const s16x8 af = *(const s16x8*)(xb + (long)i * 16 * a.F + kt * 32);
        acc[i] = E::mfma(bf, af, acc[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) *(f32x4*)&red[wave][i][lane][0] = acc[i];
  __syncthreads();
  if (wave == 0) {
    // lane holds out[row r0 + 16i + (lane&15)][cols 16nf + 4(lane>>4) .. +3]
    const int n0 = nf * 16 + 4 * (lane >> 4);
    for (int i = 0; i < nm; ++i) {
      const int r = r0 + 16 * i + (lane & 15);
      if (r >= a.B) continue;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int n = n0 + d;
        if (n < a.N) {
          float v = red[0][i][lane][d] + red[1][i][lane][d] + red[2][i][lane][d] + red[3][i][lane][d] + a.bias[n];
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[(long)r * a.N + n] = v;
        }
      }
    }
  }
}

hipError_t fc_mfma(const FcMfmaArgs& a, hipStream_t s) {
  if (a.B <= 0 || a.F % 32 != 0 || a.NF * 16 < a.N || a.dt < 0 || a.dt > 1) return hipErrorInvalidValue;
  const dim3 grid(a.NF, ((a.B + 15) / 16 + 3) / 4);
  if (a.dt) hipLaunchKernelGGL(fc_mfma_kernel<1>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(fc_mfma_kernel<0>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
