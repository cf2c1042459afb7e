// Memory-bound tail kernels: TF-'same' max-pool + residual add
// and the fused classifier head GAP -> Dense+ReLU -> Dense (K9).
// Both move bf16 in 16-byte vectors (cdna guide G13).
#include "common.h"
#include "launch.h"

namespace kdl {

// One thread = one output pixel x 8 channels. TF 'same' pads with -inf, i.e.
// out-of-range taps are skipped (the odd pad goes bottom/right: pad_top/left
// are the *leading* pads computed on the host).
__global__ __launch_bounds__(256) void pool_add_kernel(PoolAddArgs a) {
  const int CC = a.C >> 3;
  const long total = (long)a.B * a.OH * a.OW * CC;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % CC);
  const long p = i / CC;  // output pixel
  const int ow = (int)(p % a.OW);
  const long t = p / a.OW;
  const int oh = (int)(t % a.OH);
  const int b = (int)(t / a.OH);
  float mx[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) mx[d] = -INFINITY;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int ih = oh * 2 - a.pad_top + dy;
    if ((unsigned)ih >= (unsigned)a.H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int iw = ow * 2 - a.pad_left + dx;
      if ((unsigned)iw >= (unsigned)a.W) continue;
      const u32x4 v = *(const u32x4*)(a.x + (((long)b * a.H + ih) * a.W + iw) * a.C + cc * 8);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        mx[2 * d] = fmaxf(mx[2 * d], bf_lo(v[d]));
        mx[2 * d + 1] = fmaxf(mx[2 * d + 1], bf_hi(v[d]));
      }
    }
  }
  if (a.res) {
    const u32x4 r = *(const u32x4*)(a.res + p * a.C + cc * 8);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      mx[2 * d] += bf_lo(r[d]);
      mx[2 * d + 1] += bf_hi(r[d]);
    }
  }
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = pack_bf16(mx[2 * d], mx[2 * d + 1]);
  *(u32x4*)(a.y + p * a.C + cc * 8) = o;
}

hipError_t pool_add(const PoolAddArgs& a, hipStream_t s) {
  if (a.C % 8 != 0) return hipErrorInvalidValue;
  const long total = (long)a.B * a.OH * a.OW * (a.C / 8);
  hipLaunchKernelGGL(pool_add_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// One 256-thread block per image. GAP accumulates in fp32; the two dense layers
// are wave-parallel dot products with 64-lane shuffle reductions.
__global__ __launch_bounds__(256) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  float* feat = hsm;           // [F]
  float* hid = hsm + a.F;      // [H1]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint16_t* xb = a.x + (long)b * a.HW * a.ldx;
  const float inv = 1.0f / (float)a.HW;
  for (int c8 = tid; c8 < a.F / 8; c8 += 256) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < a.HW; ++p) {
      const u32x4 v = *(const u32x4*)(xb + (long)p * a.ldx + c8 * 8);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        s[2 * d] += bf_lo(v[d]);
        s[2 * d + 1] += bf_hi(v[d]);
      }
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) feat[c8 * 8 + d] = s[d] * inv;
  }
  __syncthreads();
  for (int o = wave; o < a.H1; o += 4) {
    const float* w = a.w1t + (long)o * a.F;
    float s = 0.f;
    for (int k = lane * 4; k < a.F; k += 256) {
      const float4 wv = *(const float4*)(w + k);
      s += wv.x * feat[k] + wv.y * feat[k + 1] + wv.z * feat[k + 2] + wv.w * feat[k + 3];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) hid[o] = fmaxf(s + a.b1[o], 0.f);
  }
  __syncthreads();
  for (int o = wave; o < a.NC; o += 4) {
    const float* w = a.w2t + (long)o * a.H1;
    float s = 0.f;
    for (int k = lane; k < a.H1; k += 64) s += w[k] * hid[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) a.out[(long)b * a.NC + o] = s + a.b2[o];
  }
}

hipError_t head_dense(const HeadArgs& a, hipStream_t s) {
  if (a.F % 256 != 0 || a.ldx % 8 != 0) return hipErrorInvalidValue;
  const size_t smem = (size_t)(a.F + a.H1) * sizeof(float);
  hipLaunchKernelGGL(head_kernel, dim3(a.B), dim3(256), smem, s, a);
  return hipGetLastError();
}

}  // namespace kdl
