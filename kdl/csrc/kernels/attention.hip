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
#include <cstdlib>

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
  // staging. K: thread = (key kr, 8-dim chunk kc), rows kr and kr + 32: eight lanes read one
  // 128-byte K row (coalesced), written row-major with ds_write_b128. V: thread = (key
  // pair kp, chunk sch), rows 2kp and 2kp + 1, so V^T is written as packed key pairs
  // (ds_write_b32: the 32 lanes of a half-wave hit 32 different banks; per-element
  // ds_write_b16 of the transpose was 8-way conflicted). The next tile's loads are issued
  // before this tile's math.
  const int kp = tid & 31, sch = tid >> 5;
  const int kr = tid >> 3, kc = tid & 7;
  u32x4 kr0, kr1, vr0, vr1;
  auto fetch = [&](int kt) {
    const u32x4 z = {0u, 0u, 0u, 0u};
    const int k0 = kt * AT_KV + kr;
    const uint16_t* kb = base + (long)k0 * ld + koff + kc * 8;
    kr0 = k0 < a.T ? *(const u32x4*)kb : z;
    kr1 = k0 + 32 < a.T ? *(const u32x4*)(kb + 32 * ld) : z;
    const int v0 = kt * AT_KV + 2 * kp;
    const uint16_t* vb = base + (long)v0 * ld + voff + sch * 8;
    vr0 = v0 < a.T ? *(const u32x4*)vb : z;
    vr1 = v0 + 1 < a.T ? *(const u32x4*)(vb + ld) : z;
  };
  fetch(0);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    *(u32x4*)(ks + kr * AT_ROW + kc * 8) = kr0;
    *(u32x4*)(ks + (kr + 32) * AT_ROW + kc * 8) = kr1;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      *(uint32_t*)(vt + (sch * 8 + 2 * d) * AT_ROW + 2 * kp) = (vr0[d] & 0xffffu) | (vr1[d] << 16);
      *(uint32_t*)(vt + (sch * 8 + 2 * d + 1) * AT_ROW + 2 * kp) = (vr0[d] >> 16) | (vr1[d] & 0xffff0000u);
    }
    __syncthreads();
    if (kt + 1 < nkt) fetch(kt + 1);

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
    const bool full = (kt + 1) * AT_KV <= a.T;     // only the last key tile needs the mask
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * AT_KV + 16 * kf + 4 * q + r;
        const float v = (full || key < a.T) ? s[kf][r] * sl2 : -INFINITY;
        s[kf][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(s[kf][r] - mn);
        s[kf][r] = p;
        ls += p;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;
    // O^T[dim 16df + 4q + r][query c] += V^T P^T
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const u32x4 pw = {pack_bf16(s[2 * k2][0], s[2 * k2][1]), pack_bf16(s[2 * k2][2], s[2 * k2][3]),
                        pack_bf16(s[2 * k2 + 1][0], s[2 * k2 + 1][1]),
                        pack_bf16(s[2 * k2 + 1][2], s[2 * k2 + 1][3])};
      const s16x8 pb = __builtin_bit_cast(s16x8, pw);
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

// Whole-head variant (T <= 256): one workgroup per (image, head) with ceil(T/16) waves, so
// K and V^T of the head are staged ONCE (the 64-query-tile kernel above re-stages them per
// query tile: 4x the loads and LDS writes at T = 197, plus a barrier pair per key tile and
// a quarter of its query rows idle in the last tile). All keys live in LDS (K [256][72],
// V^T [64][328]: both row strides keep the 8/16-byte fragment reads conflict-free), one
// barrier, then every wave runs the same online-softmax loop over 64-key tiles.
constexpr int AW_TK = 256;
constexpr int AW_VROW = 264;   // V^T row stride: 132 dwords == 4 (mod 64): the 16 dim rows of a half-wave's
                               // 8-byte reads land 4 banks apart (q adds 2) -> conflict-free

// capped at 64 VGPRs (8 waves per SIMD, no spill) with a 70.7 KB LDS map so two 13-wave heads can
// share a CU: batch-32 ViT-B/16 attention 20.8 -> 19.0 us (profiles/attention_r3.txt)
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void attn_head_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t hsm[];
  uint16_t* ks = hsm;                      // [AW_TK][AT_ROW]
  uint16_t* vt = hsm + AW_TK * AT_ROW;     // [AT_DH][AW_VROW]
  const int tid = threadIdx.x, nth = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  const int h = blockIdx.x % a.H, b = blockIdx.x / a.H;
  const long ld = 3L * a.H * AT_DH;
  const uint16_t* base = a.qkv + (long)b * a.T * ld;
  const int qoff = h * AT_DH, koff = (a.H + h) * AT_DH, voff = (2 * a.H + h) * AT_DH;
  const int nkt = (a.T + AT_KV - 1) / AT_KV;
  const int TK = nkt * AT_KV;
  const u32x4 z = {0u, 0u, 0u, 0u};
  // Staging in chunks: each thread first issues the global loads of up to 4 K rows (2 V key
  // pairs), then writes them to LDS -- one item per loop trip put a full global round trip per
  // item on the critical path (~5 of them at T = 197 with 13 waves)
  // K rows (8 lanes per 128-byte row: coalesced), zero beyond T
  for (int i0 = tid; i0 < TK * 8; i0 += 4 * nth) {
    u32x4 kv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * nth, k = i >> 3, kc = i & 7;
      kv[u] = i < TK * 8 && k < a.T ? *(const u32x4*)(base + (long)k * ld + koff + kc * 8) : z;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * nth;
      if (i < TK * 8) *(u32x4*)(ks + (i >> 3) * AT_ROW + (i & 7) * 8) = kv[u];
    }
  }
  // V^T as packed key pairs: item = (chunk, key pair), pair fastest -> conflict-free b32 writes
  for (int i0 = tid; i0 < (TK / 2) * 8; i0 += 2 * nth) {
    u32x4 v0[2], v1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * nth;
      const int kp = i % (TK / 2), ch = i / (TK / 2), k0 = 2 * kp;
      const bool in = i < (TK / 2) * 8;
      const uint16_t* vb = base + (long)k0 * ld + voff + ch * 8;
      v0[u] = in && k0 < a.T ? *(const u32x4*)vb : z;
      v1[u] = in && k0 + 1 < a.T ? *(const u32x4*)(vb + ld) : z;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + u * nth;
      if (i >= (TK / 2) * 8) continue;
      const int kp = i % (TK / 2), ch = i / (TK / 2), k0 = 2 * kp;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        *(uint32_t*)(vt + (ch * 8 + 2 * d) * AW_VROW + k0) = (v0[u][d] & 0xffffu) | (v1[u][d] << 16);
        *(uint32_t*)(vt + (ch * 8 + 2 * d + 1) * AW_VROW + k0) = (v0[u][d] >> 16) | (v1[u][d] & 0xffff0000u);
      }
    }
  }
  const int qi = wave * 16 + c;
  const bool qvalid = qi < a.T;
  s16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qf[kk] = (s16x8){0, 0, 0, 0, 0, 0, 0, 0};
    if (qvalid) qf[kk] = *(const s16x8*)(base + (long)qi * ld + qoff + 32 * kk + 8 * q);
  }
  __syncthreads();

  f32x4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x4 s[4];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
      s[kf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const s16x8 kfr = *(const s16x8*)(ks + (kt * AT_KV + 16 * kf + c) * AT_ROW + 32 * kk + 8 * q);
        s[kf] = mfma16(kfr, qf[kk], s[kf]);
      }
    }
    float tmax = -INFINITY;
    const bool full = (kt + 1) * AT_KV <= a.T;     // only the last key tile needs the mask
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * AT_KV + 16 * kf + 4 * q + r;
        const float v = (full || key < a.T) ? s[kf][r] * sl2 : -INFINITY;
        s[kf][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
    const float mn = fmaxf(m, tmax);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(s[kf][r] - mn);
        s[kf][r] = p;
        ls += p;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const u32x4 pw = {pack_bf16(s[2 * k2][0], s[2 * k2][1]), pack_bf16(s[2 * k2][2], s[2 * k2][3]),
                        pack_bf16(s[2 * k2 + 1][0], s[2 * k2 + 1][1]),
                        pack_bf16(s[2 * k2 + 1][2], s[2 * k2 + 1][3])};
      const s16x8 pb = __builtin_bit_cast(s16x8, pw);
#pragma unroll
      for (int df = 0; df < 4; ++df) {
        const uint16_t* vr = vt + (16 * df + c) * AW_VROW + kt * AT_KV + 32 * k2 + 4 * q;
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
  static const bool tiled = [] { const char* e = getenv("KDL_ATTN_TILED"); return e && atoi(e) != 0; }();
  if (a.T <= AW_TK && !tiled) {
    const int waves = (a.T + 15) / 16;
    const size_t smem = (size_t)(AW_TK * AT_ROW + AT_DH * AW_VROW) * sizeof(uint16_t);
    hipLaunchKernelGGL(attn_head_kernel, dim3((unsigned)(a.B * a.H)), dim3(64 * waves), smem, s, a);
    return hipGetLastError();
  }
  const int nqt = (a.T + AT_Q - 1) / AT_Q;
  hipLaunchKernelGGL(attn_kernel, dim3((unsigned)(a.B * a.H * nqt)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kdl
