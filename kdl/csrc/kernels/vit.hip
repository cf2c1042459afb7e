// Transformer-side elementwise / normalisation kernels for ViT-B/16 (SURVEY.md
// §2.6): patchify with the input normalisation fused, class-token + position
// embedding, and LayerNorm. All move bf16 in 16-byte vectors (cdna guide G13).
#include "common.h"
#include "launch.h"

namespace kdl {

// A[b*np + p][k], k = c*P*P + ky*P + kx (torch conv weight [D][3][P][P] flattened).
// One thread = 8 consecutive k (one channel, one patch row, 8 columns).
__global__ __launch_bounds__(256) void patchify_kernel(PatchifyArgs a) {
  const int K = 3 * a.P * a.P;
  const int npw = a.W / a.P, np = npw * (a.H / a.P);
  const long total = (long)a.B * np * (K / 8);
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int k0 = (int)(i % (K / 8)) * 8;
  const long row = i / (K / 8);
  const int b = (int)(row / np), p = (int)(row % np);
  const int py = p / npw, px = p - py * npw;
  const int c = k0 / (a.P * a.P), rem = k0 - c * a.P * a.P;
  const int ky = rem / a.P, kx = rem - ky * a.P;
  const uint8_t* src = a.x + (((long)b * a.H + py * a.P + ky) * a.W + px * a.P + kx) * 3 + c;
  const float sc = c == 0 ? a.scale[0] : c == 1 ? a.scale[1] : a.scale[2];
  const float sh = c == 0 ? a.shift[0] : c == 1 ? a.shift[1] : a.shift[2];
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d)
    o[d] = pack_bf16((float)src[(2 * d) * 3] * sc + sh, (float)src[(2 * d + 1) * 3] * sc + sh);
  *(u32x4*)(a.y + row * a.ldy + k0) = o;
}

hipError_t patchify(const PatchifyArgs& a, hipStream_t s) {
  if (a.P % 8 != 0 || a.H % a.P != 0 || a.W % a.P != 0) return hipErrorInvalidValue;
  const long total = (long)a.B * (a.H / a.P) * (a.W / a.P) * (3 * a.P * a.P / 8);
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// X[b][0] = cls + pos[0]; X[b][t] += pos[t] for t >= 1 (the patch GEMM wrote rows 1..T-1).
__global__ __launch_bounds__(256) void embed_kernel(EmbedArgs a) {
  const int C8 = a.D / 8;
  const long total = (long)a.B * a.T * C8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int c8 = (int)(i % C8);
  const long r = i / C8;
  const int t = (int)(r % a.T);
  uint16_t* xp = a.x + r * a.D + c8 * 8;
  const float* pp = a.pos + (long)t * a.D + c8 * 8;
  u32x4 v = t == 0 ? (u32x4){0u, 0u, 0u, 0u} : *(const u32x4*)xp;
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    float lo = bf_lo(v[d]) + pp[2 * d], hi = bf_hi(v[d]) + pp[2 * d + 1];
    if (t == 0) {
      lo += a.cls[c8 * 8 + 2 * d];
      hi += a.cls[c8 * 8 + 2 * d + 1];
    }
    o[d] = pack_bf16(lo, hi);
  }
  *(u32x4*)xp = o;
}

hipError_t embed_tokens(const EmbedArgs& a, hipStream_t s) {
  if (a.D % 8 != 0) return hipErrorInvalidValue;
  const long total = (long)a.B * a.T * (a.D / 8);
  hipLaunchKernelGGL(embed_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// One wave per row; each lane owns up to LN_CH 8-element chunks (D <= 64*8*LN_CH).
constexpr int LN_CH = 4;
__global__ __launch_bounds__(256) void layernorm_kernel(LnArgs a) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.rows) return;
  const uint16_t* xr = a.x + r * a.ldx;
  const int C8 = a.D / 8;
  float v[LN_CH][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < LN_CH; ++j) {
    const int c8 = lane + 64 * j;
    if (c8 < C8) {
      const u32x4 u = *(const u32x4*)(xr + c8 * 8);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        v[j][2 * d] = bf_lo(u[d]);
        v[j][2 * d + 1] = bf_hi(u[d]);
      }
    } else {
#pragma unroll
      for (int d = 0; d < 8; ++d) v[j][d] = 0.f;
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) s += v[j][d];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  const float mean = s / (float)a.D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_CH; ++j) {
    if (lane + 64 * j < C8) {
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const float t = v[j][d] - mean;
        q += t * t;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
  const float rstd = rsqrtf(q / (float)a.D + a.eps);
  uint16_t* yr = a.y + r * a.ldy;
#pragma unroll
  for (int j = 0; j < LN_CH; ++j) {
    const int c8 = lane + 64 * j;
    if (c8 < C8) {
      const float4 g0 = *(const float4*)(a.gamma + c8 * 8), g1 = *(const float4*)(a.gamma + c8 * 8 + 4);
      const float4 b0 = *(const float4*)(a.beta + c8 * 8), b1 = *(const float4*)(a.beta + c8 * 8 + 4);
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o8[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) o8[d] = (v[j][d] - mean) * rstd * g[d] + bb[d];
      if (a.y8) {
        const float q = a.inv_scale;
        *(u32x2*)(a.y8 + r * a.ldy + c8 * 8) = (u32x2){pack_fp8x4(o8[0] * q, o8[1] * q, o8[2] * q, o8[3] * q),
                                                        pack_fp8x4(o8[4] * q, o8[5] * q, o8[6] * q, o8[7] * q)};
      } else {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = pack_bf16(o8[2 * d], o8[2 * d + 1]);
        *(u32x4*)(yr + c8 * 8) = o;
      }
    }
  }
}

// Two rows per wave (32 lanes per row, up to 4 chunks of 8 per lane: D <= 1024): every lane
// is busy at D = 768 (the kernel above leaves half its lanes idle for a row's second chunk),
// and sum / sum of squares reduce together in one 5-step butterfly instead of two dependent
// 6-step ones (the row's statistics were a chain of 12 ds_bpermute latencies).
__global__ __launch_bounds__(256) void layernorm2_kernel(LnArgs a) {
  const int lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
  const long r = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + half;
  const bool live = r < a.rows;
  const uint16_t* xr = a.x + (live ? r : 0) * a.ldx;
  const int C8 = a.D / 8;
  float v[LN_CH][8];
  float s = 0.f, ss = 0.f;
#pragma unroll
  for (int j = 0; j < LN_CH; ++j) {
    const int c8 = hl + 32 * j;
    u32x4 u = {0u, 0u, 0u, 0u};
    if (live && c8 < C8) u = *(const u32x4*)(xr + c8 * 8);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      v[j][2 * d] = bf_lo(u[d]);
      v[j][2 * d + 1] = bf_hi(u[d]);
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      s += v[j][d];
      ss += v[j][d] * v[j][d];
    }
  }
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    ss += __shfl_xor(ss, off);
  }
  const float inv_d = 1.f / (float)a.D;
  const float mean = s * inv_d;
  const float var = fmaxf(ss * inv_d - mean * mean, 0.f);
  const float rstd = rsqrtf(var + a.eps);
  if (!live) return;
  uint16_t* yr = a.y + r * a.ldy;
#pragma unroll
  for (int j = 0; j < LN_CH; ++j) {
    const int c8 = hl + 32 * j;
    if (c8 < C8) {
      const float4 g0 = *(const float4*)(a.gamma + c8 * 8), g1 = *(const float4*)(a.gamma + c8 * 8 + 4);
      const float4 b0 = *(const float4*)(a.beta + c8 * 8), b1 = *(const float4*)(a.beta + c8 * 8 + 4);
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o8[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) o8[d] = (v[j][d] - mean) * rstd * g[d] + bb[d];
      if (a.y8) {
        const float q = a.inv_scale;
        *(u32x2*)(a.y8 + r * a.ldy + c8 * 8) = (u32x2){pack_fp8x4(o8[0] * q, o8[1] * q, o8[2] * q, o8[3] * q),
                                                        pack_fp8x4(o8[4] * q, o8[5] * q, o8[6] * q, o8[7] * q)};
      } else {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = pack_bf16(o8[2 * d], o8[2 * d + 1]);
        *(u32x4*)(yr + c8 * 8) = o;
      }
    }
  }
}

hipError_t layernorm(const LnArgs& a, hipStream_t s) {
  if (a.D % 8 != 0 || a.D > 64 * 8 * LN_CH || a.rows <= 0) return hipErrorInvalidValue;
  if (a.D <= 32 * 8 * LN_CH) {
    hipLaunchKernelGGL(layernorm2_kernel, dim3((unsigned)((a.rows + 7) / 8)), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(layernorm_kernel, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
