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

// One 1024-thread block per image (the head is latency-bound: parallelise every
// reduction). GAP: 4 pixel groups x 256 channel-chunks, partial sums through LDS.
// Dense1 (Keras [F][H1] layout, coalesced across outputs): 8 k-slices x 128
// outputs, reduced through LDS. Dense2 is tiny.
__global__ __launch_bounds__(1024) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  float* part = hsm;                 // [4][F] GAP partials, later [8][128] dense partials
  float* feat = hsm + 4 * a.F;       // [F]
  float* hid = feat + a.F;           // [H1]
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint16_t* xb = a.x + (long)b * a.HW * a.ldx;
  const int nchunk = a.F / 8;
  for (int i = tid; i < 4 * nchunk; i += 1024) {
    const int c8 = i % nchunk, pg = i / nchunk;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 5
    for (int p = pg; p < a.HW; p += 4) {
      const u32x4 v = *(const u32x4*)(xb + (long)p * a.ldx + c8 * 8);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        s[2 * d] += bf_lo(v[d]);
        s[2 * d + 1] += bf_hi(v[d]);
      }
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) part[pg * a.F + c8 * 8 + d] = s[d];
  }
  __syncthreads();
  const float inv = 1.0f / (float)a.HW;
  for (int k = tid; k < a.F; k += 1024)
    feat[k] = (part[k] + part[a.F + k] + part[2 * a.F + k] + part[3 * a.F + k]) * inv;
  __syncthreads();
  {
    const int o = tid & 127, sl = tid >> 7;   // 8 slices
    const int klen = a.F / 8;
    float s = 0.f;
    if (o < a.H1) {
      const float* w = a.w1 + (long)(sl * klen) * a.H1 + o;
      const float* f = feat + sl * klen;
#pragma unroll 8
      for (int k = 0; k < klen; ++k) s += f[k] * w[(long)k * a.H1];
    }
    part[sl * 128 + o] = s;
  }
  __syncthreads();
  if (tid < a.H1) {
    float s = a.b1[tid];
#pragma unroll
    for (int sl = 0; sl < 8; ++sl) s += part[sl * 128 + tid];
    hid[tid] = fmaxf(s, 0.f);
  }
  __syncthreads();
  if (tid < a.NC) {
    float s = a.b2[tid];
    for (int k = 0; k < a.H1; ++k) s += hid[k] * a.w2[(long)k * a.NC + tid];
    a.out[(long)b * a.NC + tid] = s;
  }
}

hipError_t head_dense(const HeadArgs& a, hipStream_t s) {
  if (a.F % 64 != 0 || a.ldx % 8 != 0 || a.H1 > 128 || a.NC > 1024) return hipErrorInvalidValue;
  const size_t smem = (size_t)(4 * a.F + a.F + a.H1) * sizeof(float);
  hipLaunchKernelGGL(head_kernel, dim3(a.B), dim3(1024), smem, s, a);
  return hipGetLastError();
}

}  // namespace kdl
