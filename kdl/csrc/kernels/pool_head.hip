// Memory-bound tail kernels: TF-'same' max-pool + residual add
// and the fused classifier head GAP -> Dense+ReLU -> Dense (K9).
// Both move bf16 in 16-byte vectors (cdna guide G13).
#include "common.h"
#include "launch.h"

namespace kdl {

// One thread = one output pixel x 8 channels; grid (ceil(OW*C/8 / 256), B*OH): the output
// row comes from blockIdx.y (scalar), so the only per-thread index math is one 32-bit
// division by C/8. (The flat-index version spent ~200 VALU instructions per thread on
// four 64-bit div/mods -- as much VALU time as the 267 MB it moves at b32 / 147x147.)
// TF 'same' pads with -inf, i.e. out-of-range taps are skipped (the odd pad goes
// bottom/right: pad_top/left are the *leading* pads computed on the host).
template <int DT>
__global__ __launch_bounds__(256) void pool_add_kernel(PoolAddArgs a) {
  using E = Elt<DT>;
  const int CC = a.C >> 3;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.OW * CC) return;
  const int row = blockIdx.y;                   // b * OH + oh
  const int b = row / a.OH, oh = row - b * a.OH;
  const int ow = (unsigned)j / (unsigned)CC, cc = j - ow * CC;
  const long p = (long)row * a.OW + ow;         // output pixel
  float mx[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) mx[d] = -INFINITY;
  const uint16_t* xb = a.x + (long)b * a.H * a.W * a.C + cc * 8;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int ih = oh * 2 - a.pad_top + dy;
    if ((unsigned)ih >= (unsigned)a.H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int iw = ow * 2 - a.pad_left + dx;
      if ((unsigned)iw >= (unsigned)a.W) continue;
      const u32x4 v = *(const u32x4*)(xb + (long)(ih * a.W + iw) * a.C);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        mx[2 * d] = fmaxf(mx[2 * d], E::lo(v[d]));
        mx[2 * d + 1] = fmaxf(mx[2 * d + 1], E::hi(v[d]));
      }
    }
  }
  if (a.res) {
    const u32x4 r = *(const u32x4*)(a.res + p * a.C + cc * 8);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      mx[2 * d] += E::lo(r[d]);
      mx[2 * d + 1] += E::hi(r[d]);
    }
  }
  u32x4 o;
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = E::pack(mx[2 * d], mx[2 * d + 1]);
  *(u32x4*)(a.y + p * a.C + cc * 8) = o;
}

// Row-streaming variant (algo 2): a thread owns one 8-channel chunk x SEG adjacent output
// columns x an RB-row output band, flat-mapped with the chunk fastest (a wave reads 1 KiB
// of contiguous pixel-row bytes). The band's 2*RB+1 input rows stream top to bottom, one
// row in flight ahead: each input row is loaded ONCE per thread (2*SEG+1 pixels), reduced
// horizontally to SEG column maxima, and folded into the single running output row --
// input row 2k+2 both finishes output row k (+ residual, store) and starts row k+1. The
// one-pixel-per-thread kernel above re-reads every input pixel ~2.25x through L1/L2.
template <int DT, int SEG>
__global__ __launch_bounds__(256) void pool_add_rows_kernel(PoolAddArgs a, int RB, int nseg, int nbands) {
  using E = Elt<DT>;
  constexpr int NJ = 2 * SEG + 1;
  const int C8 = a.C >> 3;
  const long id = (long)blockIdx.x * 256 + threadIdx.x;
  if (id >= (long)a.B * nbands * nseg * C8) return;          // no barrier below
  const int cc = (int)(id % C8);
  long r = id / C8;
  const int seg = (int)(r % nseg);
  r /= nseg;
  const int band = (int)(r % nbands);
  const int b = (int)(r / nbands);
  const int ow0 = seg * SEG, oh0 = band * RB;
  const int rows = min(RB, a.OH - oh0);
  const int iw0 = 2 * ow0 - a.pad_left, ih0 = 2 * oh0 - a.pad_top;
  const int vmax = 2 * rows + 1;
  const uint16_t* xb = a.x + ((long)b * a.H * a.W + iw0) * a.C + cc * 8;
  const long obase = ((long)b * a.OH + oh0) * a.OW + ow0;
  bool cok[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) cok[j] = (unsigned)(iw0 + j) < (unsigned)a.W;
  auto load = [&](int v, u32x4 (&xr)[NJ], bool& ok) {
    const int ih = ih0 + v;
    ok = v < vmax && (unsigned)ih < (unsigned)a.H;
    const uint16_t* rp = xb + (long)ih * a.W * a.C;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (ok && cok[j]) xr[j] = *(const u32x4*)(rp + (long)j * a.C);
  };
  float acc[SEG][8];
  u32x4 xq[2][NJ];
  bool okq[2];
  load(0, xq[0], okq[0]);
  for (int v = 0; v < vmax; ++v) {
    load(v + 1, xq[1], okq[1]);
    float hm[SEG][8];
#pragma unroll
    for (int o = 0; o < SEG; ++o)
#pragma unroll
      for (int d = 0; d < 8; ++d) hm[o][d] = -INFINITY;
    if (okq[0]) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (!cok[j]) continue;
        float f[8];
#pragma unroll
        for (int d = 0; d < 4; ++d) { f[2 * d] = E::lo(xq[0][j][d]); f[2 * d + 1] = E::hi(xq[0][j][d]); }
        // input column j feeds output columns o with 2o <= j <= 2o + 2
#pragma unroll
        for (int o = 0; o < SEG; ++o)
          if (j >= 2 * o && j <= 2 * o + 2) {
#pragma unroll
            for (int d = 0; d < 8; ++d) hm[o][d] = fmaxf(hm[o][d], f[d]);
          }
      }
    }
    const int k = v >> 1;
    if ((v & 1) == 0 && k >= 1) {                // row 2k finishes output row k-1
      const long p0 = obase + (long)(k - 1) * a.OW;
#pragma unroll
      for (int o = 0; o < SEG; ++o) {
        if (ow0 + o >= a.OW) continue;
        float m[8];
#pragma unroll
        for (int d = 0; d < 8; ++d) m[d] = fmaxf(acc[o][d], hm[o][d]);
        if (a.res) {
          const u32x4 rr = *(const u32x4*)(a.res + (p0 + o) * a.C + cc * 8);
#pragma unroll
          for (int d = 0; d < 4; ++d) { m[2 * d] += E::lo(rr[d]); m[2 * d + 1] += E::hi(rr[d]); }
        }
        u32x4 out;
#pragma unroll
        for (int d = 0; d < 4; ++d) out[d] = E::pack(m[2 * d], m[2 * d + 1]);
        *(u32x4*)(a.y + (p0 + o) * a.C + cc * 8) = out;
      }
    }
#pragma unroll
    for (int o = 0; o < SEG; ++o)
#pragma unroll
      for (int d = 0; d < 8; ++d) acc[o][d] = (v & 1) ? fmaxf(acc[o][d], hm[o][d]) : hm[o][d];
#pragma unroll
    for (int j = 0; j < NJ; ++j) xq[0][j] = xq[1][j];
    okq[0] = okq[1];
  }
}

static void pool_rows_plan(const PoolAddArgs& a, int* seg, int* rb, int* nseg, int* nb) {
  *seg = a.seg > 0 ? a.seg : 2;
  *nseg = (a.OW + *seg - 1) / *seg;
  const long per_band = (long)a.B * *nseg * (a.C / 8);
  int R = a.rb;
  if (R <= 0) {
    long n = (2L * 256 * 4 * 64 + per_band - 1) / per_band;
    n = n < 1 ? 1 : (n > a.OH ? a.OH : n);
    R = (int)((a.OH + n - 1) / n);
  }
  *rb = R;
  *nb = (a.OH + R - 1) / R;
}

// default: the row-streaming kernel (Xception bench +0.5-1.0 % in three A/B pairs, profiles/pool_algo_ab_r3.txt);
// KDL_POOL_ALGO=1 restores the pixel-per-thread kernel
static int pool_algo(const PoolAddArgs& a) {
  if (a.algo > 0) return a.algo;
  static const int env = [] { const char* e = getenv("KDL_POOL_ALGO"); return e ? atoi(e) : 0; }();
  return env > 0 ? env : 2;
}

hipError_t pool_add(const PoolAddArgs& a, hipStream_t s) {
  if (a.C % 8 != 0 || a.dt < 0 || a.dt > 1 || a.B <= 0 || a.OH <= 0 || a.OW <= 0) return hipErrorInvalidValue;
  // the pixel-per-thread kernel puts B*OH on grid.y (at most 65535): larger batches (e.g. a
  // server's --max_batch_size above ~885 at Xception block2) take the 1-D row-streaming grid
  if (pool_algo(a) == 2 || (long)a.B * a.OH > 65535) {
    int seg, rb, nseg, nb;
    pool_rows_plan(a, &seg, &rb, &nseg, &nb);
    const long nblk = ((long)a.B * nb * nseg * (a.C / 8) + 255) / 256;
    if (rb <= 0 || nblk >= (1L << 31)) return hipErrorInvalidValue;
#define KDL_POOLR(et, sg)                                                                                    \
    if (a.dt == et && seg == sg) {                                                                            \
      hipLaunchKernelGGL((pool_add_rows_kernel<et, sg>), dim3((unsigned)nblk), dim3(256), 0, s, a, rb, nseg, nb); \
      return hipGetLastError();                                                                               \
    }
    KDL_POOLR(0, 1) KDL_POOLR(0, 2) KDL_POOLR(0, 4) KDL_POOLR(1, 1) KDL_POOLR(1, 2) KDL_POOLR(1, 4)
#undef KDL_POOLR
    return hipErrorInvalidValue;
  }
  const dim3 grid((unsigned)((a.OW * (a.C / 8) + 255) / 256), (unsigned)(a.B * a.OH));
  if (a.dt) hipLaunchKernelGGL(pool_add_kernel<1>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(pool_add_kernel<0>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// Classifier head as two small kernels. The head is bound by PER-CU bandwidth, not by the
// chip: a one-block-per-image kernel put the whole 800 KB Dense1 matrix through each of only
// 32 CUs (35-39 us at batch 32). Here
//   gap_dense1_kernel grid (F/64, B/8): GAP of 64 features x 8 images + their K-split dense1
//                     partials [F/64][B][H1];
//   dense2_kernel     one block per image: partials (+b1, ReLU) and w2 in LDS, 16 lanes per logit.
// Every sum is in a fixed order: deterministic logits.
constexpr int D1_K = 64;   // features per K-split block of dense1

// GAP + dense1, K-split: block (kb, image octet) averages features [64kb, 64kb+64) of 8 images
// itself (4 pixel groups per (image, 8-channel chunk), fixed order), stages the w1 slice [H1][64]
// (w1 TRANSPOSED to [H1][F] at load time, so each slice is read by only B/8 blocks) and writes
// partials [F/64][B][H1]; 32 x 4 = 128 blocks at batch 32. Replaced round 2's separate GAP
// (B x F/256 blocks) + dense1 (F/64 blocks) launches: head 22.5 -> 15.4 us, no [B][F] round trip.
__global__ __launch_bounds__(256) void gap_dense1_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float w1s[128][D1_K + 4];
  __shared__ __attribute__((aligned(16))) float gp[4][8][D1_K];   // pixel-group partial sums
  __shared__ __attribute__((aligned(16))) float fs[8][D1_K];
  const int kb = blockIdx.x, k0 = kb * D1_K, tid = threadIdx.x;
  const int ib0 = blockIdx.y * 8, nimg = min(8, a.B - ib0);
  {
    float4 wv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + 256 * j, o = i / (D1_K / 4), c = i - o * (D1_K / 4);
      wv[j] = o < a.H1 ? *(const float4*)(a.w1 + (long)o * a.F + k0 + c * 4) : (float4){0.f, 0.f, 0.f, 0.f};
    }
    const int item = tid & 63, img = item >> 3, c8 = item & 7, pg = tid >> 6;
    float sm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (img < nimg) {
      const uint16_t* xb = a.x + (long)(ib0 + img) * a.HW * a.ldx + k0 + c8 * 8;
#pragma unroll 5
      for (int p = pg; p < a.HW; p += 4) {
        const u32x4 v = *(const u32x4*)(xb + (long)p * a.ldx);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          sm[2 * d] += bf_lo(v[d]);
          sm[2 * d + 1] += bf_hi(v[d]);
        }
      }
    }
#pragma unroll
    for (int d = 0; d < 8; ++d) gp[pg][img][c8 * 8 + d] = sm[d];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + 256 * j, o = i / (D1_K / 4), c = i - o * (D1_K / 4);
      *(float4*)&w1s[o][c * 4] = wv[j];
    }
  }
  __syncthreads();
  const float inv = 1.0f / (float)a.HW;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i = tid + 256 * r, img = i >> 6, c = i & 63;
    fs[img][c] = (gp[0][img][c] + gp[1][img][c] + gp[2][img][c] + gp[3][img][c]) * inv;
  }
  __syncthreads();
  // thread = hidden unit o x 4 images
  const int o = tid & 127, i0 = (tid >> 7) * 4;
  if (o < a.H1) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int k = 0; k < D1_K; k += 4) {
      const float4 w = *(const float4*)&w1s[o][k];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 f = *(const float4*)&fs[i0 + i][k];
        acc[i] += w.x * f.x + w.y * f.y + w.z * f.z + w.w * f.w;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i0 + i < nimg) a.hid[((long)kb * a.B + ib0 + i0 + i) * a.H1 + o] = acc[i];
  }
}

__global__ __launch_bounds__(256) void dense2_kernel(HeadArgs a) {
  // one block per image: reduce dense1's K-split partials (+b1, ReLU) into LDS, then the
  // logits with w2 staged in LDS, 16 lanes per logit
  extern __shared__ __attribute__((aligned(16))) float d2s[];   // [H1] hid + [H1*NC] w2 + [2][128]
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nkb = a.F / D1_K;
  float* hs = d2s;
  float* w2s = d2s + a.H1;
  // partials: 2 slices of the K-split per hidden unit per thread pair, all loads independent
  float* red = w2s + a.H1 * a.NC;               // [2][128]
  {
    const int o = tid & 127, h = tid >> 7;
    float s = 0.f;
    if (o < a.H1) {
#pragma unroll 16
      for (int kb = h; kb < nkb; kb += 2) s += a.hid[((long)kb * a.B + b) * a.H1 + o];
    }
    red[h * 128 + o] = s;
  }
#pragma unroll 4
  for (int i = tid; i < a.H1 * a.NC; i += 256) w2s[i] = a.w2[i];
  __syncthreads();
  for (int o = tid; o < a.H1; o += 256) hs[o] = fmaxf(a.b1[o] + red[o] + red[128 + o], 0.f);
  __syncthreads();
  for (int o0 = 0; o0 < a.NC; o0 += 16) {
    const int o = o0 + (tid >> 4), sl = tid & 15;
    float s = 0.f;
    if (o < a.NC)
      for (int k = sl; k < a.H1; k += 16) s += hs[k] * w2s[k * a.NC + o];
    s += __shfl_xor(s, 1, 16);
    s += __shfl_xor(s, 2, 16);
    s += __shfl_xor(s, 4, 16);
    s += __shfl_xor(s, 8, 16);
    if (o < a.NC && sl == 0) a.out[(long)b * a.NC + o] = s + a.b2[o];
  }
}

hipError_t head_dense(const HeadArgs& a, hipStream_t s) {
  if (a.F % D1_K != 0 || a.ldx % 8 != 0 || a.B <= 0 || a.H1 <= 0 || a.H1 > 128 || a.NC <= 0 ||
      !a.hid)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(gap_dense1_kernel, dim3(a.F / D1_K, (a.B + 7) / 8), dim3(256), 0, s, a);
  hipLaunchKernelGGL(dense2_kernel, dim3(a.B), dim3(256), (size_t)(a.H1 + a.H1 * a.NC + 256) * sizeof(float), s, a);
  return hipGetLastError();
}

}  // namespace kdl
