// Multi-head self-attention for ViT-B/16 (197 tokens, 12 heads x 64), flash-style
// with an online softmax, on v_mfma_f32_16x16x32_bf16 (SURVEY.md §2.6 "fused
// attention ... fits in one workgroup tile set").
//
// Block = (image, head, 64 queries); 4 waves x 16 queries. Per 64-key tile the
// block stages K [key][dim] and V^T [dim][key] in LDS (V transposed once at
// staging). Every wave then computes S^T = K Q^T (A = K rows, B = Q^T kept in
// registers), so a lane holds 16 scores of ONE query (lane & 15): the softmax row
// statistics need only two cross-lane shuffles, and those same registers ARE the
// B operand of O^T = V^T P^T once packed to bf16 -- the key order inside a
// 32-key step is permuted identically in P and in the V^T read (keys 4q..4q+3 and
// 16+4q..16+4q+3 for lane group q), so P never moves through LDS.
#include "common.h"
#include "launch.h"

namespace kdl {

constexpr int AT_Q = 64;
constexpr int AT_KV = 64;
constexpr int AT_DH = 64;
constexpr int AT_ROW = 72;   // LDS row stride (elements): conflict-free 8-byte V^T reads

__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * AT_KV * AT_ROW];
  uint16_t* ks = smem;                  // [key][dim]
  uint16_t* vt = smem + AT_KV * AT_ROW; // [dim][key]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int q = lane >> 4, c = lane & 15;
  const int nqt = (a.T + AT_Q - 1) / AT_Q;
  int bid = blockIdx.x;
  const int qt = bid % nqt;
  bid /= nqt;
  const int h = bid % a.H;
  const int b = bid / a.H;
  const long ld = 3L * a.H * AT_DH;
  const uint16_t* base = a.qkv + (long)b * a.T * ld;
  const int qoff = h * AT_DH, koff = (a.H + h) * AT_DH, voff = (2 * a.H + h) * AT_DH;
  const int qi = qt * AT_Q + wave * 16 + c;
  const bool qvalid = qi < a.T;

  s16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qf[kk] = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    if (qvalid) qf[kk] = *(const s16x8*)(base + (long)qi * ld + qoff + 32 * kk + 8 * q);
  }
  f32x4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;   // fold log2(e): p = exp2(s*sl2 - m)

  const int nkt = (a.T + AT_KV - 1) / AT_KV;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    for (int i = tid; i < AT_KV * 8; i += 256) {
      const int kr = i >> 3, ch = i & 7;
      const int key = kt * AT_KV + kr;
      u32x4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
      if (key < a.T) {
        kv = *(const u32x4*)(base + (long)key * ld + koff + ch * 8);
        vv = *(const u32x4*)(base + (long)key * ld + voff + ch * 8);
      }
      *(u32x4*)(ks + kr * AT_ROW + ch * 8) = kv;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        vt[(ch * 8 + 2 * d) * AT_ROW + kr] = (uint16_t)(vv[d] & 0xffffu);
        vt[(ch * 8 + 2 * d + 1) * AT_ROW + kr] = (uint16_t)(vv[d] >> 16);
      }
    }
    __syncthreads();

    // S^T[key 16kf + 4q + r][query c]
    f32x4 s[4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
      s[kf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const s16x8 kfr = *(const s16x8*)(ks + (16 * kf + c) * AT_ROW + 32 * kk + 8 * q);
        s[kf] = mfma16(kfr, qf[kk], s[kf]);
      }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * AT_KV + 16 * kf + 4 * q + r;
        const float v = key < a.T ? s[kf][r] * sl2 : -INFINITY;
        s[kf][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[kf][r] - mn);
        s[kf][r] = p;
        ls += p;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;
    // O^T[dim 16df + 4q + r][query c] += V^T P^T
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      s16x8 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb[r] = (short)f2bf(s[2 * k2][r]);
        pb[4 + r] = (short)f2bf(s[2 * k2 + 1][r]);
      }
#pragma unroll
      for (int df = 0; df < 4; ++df) {
        const uint16_t* vr = vt + (16 * df + c) * AT_ROW + 32 * k2 + 4 * q;
        const u32x2 lo = *(const u32x2*)vr;
        const u32x2 hi = *(const u32x2*)(vr + 16);
        const u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
        o[df] = mfma16(__builtin_bit_cast(s16x8, w), pb, o[df]);
      }
    }
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  if (qvalid) {
    const float inv = 1.f / l;
    const long off = ((long)b * a.T + qi) * (a.H * AT_DH) + h * AT_DH + 4 * q;
    if (a.out8) {
      const float sc = inv * a.inv_scale;
#pragma unroll
      for (int df = 0; df < 4; ++df)
        *(uint32_t*)(a.out8 + off + 16 * df) = pack_fp8x4(o[df][0] * sc, o[df][1] * sc, o[df][2] * sc, o[df][3] * sc);
    } else {
      uint16_t* op = a.out + off;
#pragma unroll
      for (int df = 0; df < 4; ++df)
        *(u32x2*)(op + 16 * df) = (u32x2){pack_bf16(o[df][0] * inv, o[df][1] * inv),
                                          pack_bf16(o[df][2] * inv, o[df][3] * inv)};
    }
  }
}

hipError_t attention(const AttnArgs& a, hipStream_t s) {
  if (a.dh != AT_DH || a.T <= 0 || a.H <= 0 || a.B <= 0) return hipErrorInvalidValue;
  const int nqt = (a.T + AT_Q - 1) / AT_Q;
  hipLaunchKernelGGL(attn_kernel, dim3((unsigned)(a.B * a.H * nqt)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
