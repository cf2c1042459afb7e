// Host-side launch API of the kdl HIP kernel library. Every launcher is
// asynchronous on the given stream, allocates nothing and synchronises nothing,
// so any sequence of them can be captured into a hipGraph (cdna guide G9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdl {

struct ConvGemmArgs {
  const uint16_t* x;     // input activations NHWC bf16, channel stride ldx
  const uint16_t* wp;    // packed weights [NF][K/32][64][8] bf16 (BN scale folded)
  const float* bias;     // [NF*16] fp32 (BN shift)
  const float* dww;      // MODE_DW: depthwise weights [9][K] fp32
  const uint16_t* dwk;   // MODE_DW, sepconv_ws / sepconv_2d: the same weights as bf16 entries [K/32][2][16][2][8]
                         //   (k-step, channel group, channel, tap parity, taps parity+2j)
  const uint16_t* res;   // optional residual [M][ldr] bf16
  uint16_t* y;           // output [M][ldy] bf16 (or a zero-bordered [B][OH+2][OW+2][ldy] if opad)
  int B, H, W;           // input spatial dims
  int OH, OW;            // output spatial dims
  int M;                 // B*OH*OW
  int ldx, ldy, ldr;     // channel strides (elements)
  int K;                 // reduction depth (multiple of 32)
  int cin;               // MODE_CONV: padded input channels (multiple of 32)
  int NF;                // 16-wide output-channel fragments in the packed weights
  int nstore;            // output channels written (<= ldy)
  int stride;            // spatial stride (MODE_PW / MODE_CONV)
  int relu_in;
  int relu_out;          // 0 none; 1 ReLU before the residual add (Xception); 2 after it (ResNet);
                         // 3 exact GELU before the residual add (ViT MLP); 4 SiLU before it (EfficientNet)
  unsigned long long* stamps;  // diagnostics only (stamping kernel variants): per-wave s_memtime per k-step
  int opad;              // 1: write into the interior of a 1-pixel zero-bordered output buffer, so the
                         //    next 3x3 'same' conv runs as a 'valid' implicit GEMM with no bounds checks;
                         // 2: token rows behind a class token: row m -> b*(OH*OW+1) + 1 + m%(OH*OW)
  int dt;                // element type of x / wp / res / y: 0 bf16, 1 fp16 (MODE_PW / MODE_CONV GEMMs)
  // LDS-DMA pipelined GEMM (gemm_pipe): 1 = every M tile walks K from its own starting
  // step ((7*mi) mod K/32), so the workgroups sharing the weights do not all fetch the same
  // fragments at launch (env KDL_PIPE_KROT overrides; 0 = in order)
  int krot;
  // split-K (gemm_pipe only; ResNet-50's layer3/4 3x3 convs: M = 6272 / 1568 rows fill a quarter to a
  // half of the 256 CUs with whole-K tiles): ksplit > 1 workgroups per output tile each reduce K/ksplit
  // k-steps into fp32 partials at ws ([ksplit][tiles][BM*BN], fragment-linear); the last of a tile to
  // arrive (per-tile counter cnt, agent-scope release/acquire, reset to 0 by that workgroup) sums
  // them and runs the normal epilogue. K/32 must divide by ksplit.
  int ksplit;
  float* ws;
  int* cnt;
  // per-image channel scales on the A operand (EfficientNet project conv: the SE scale, gemm_pipe
  // MODE_PW bf16 only): A[m][k] is multiplied by ascale[image(m) * ascale_ld + k] on its way from
  // LDS to the MFMA (round 6; it replaced per-image SE-scaled weight copies); M tiles then never
  // straddle two images. nullptr = no scale.
  const float* ascale;
  int ascale_ld;
};

// cfg < PIPE_CFG_BASE: register-B kernel (all modes, incl. fused depthwise);
// cfg >= PIPE_CFG_BASE: LDS-DMA pipelined kernel (MODE_PW / MODE_CONV only).
constexpr int PIPE_CFG_BASE = 16;
// cfg >= SEP_CFG_BASE: fused separable convs (MODE_DW only). Ids 64..119 are retired (the
// round-1/2 sepconv_fused / sepconv_pipe kernels, measured slower than sepconv_ws / sepconv_2d
// on every Xception shape and removed in round 3).
constexpr int SEP_CFG_BASE = 64;
// cfg >= SEPW_CFG_BASE: warp-specialized fused separable conv (sepconv_ws.hip).
constexpr int SEPW_CFG_BASE = 120;
hipError_t sepconv_ws(int cfg, const ConvGemmArgs& a, hipStream_t s);
int sepconv_ws_config(int cfg, int* bm, int* bn, int* threads);
int sepconv_ws_fits(int cfg, int W);

// A whole Xception entry block (SeparableConv -> ReLU -> SeparableConv -> 3x3/2 max-pool, plus
// the 1x1/2 residual conv) in one persistent launch, entry_block.hip. Workgroup g runs the
// host-built steps [step_off[g], step_off[g+1]) of `steps`: int4 {image, strip, pooled row k,
// mode} with mode 0 = warm-up (y1 only), 1 = warm-up (y1 + y2, no output), 2 = output row k.
struct EntryBlockArgs {
  const uint16_t* x;      // block input [B][H][W][ldx] bf16
  uint16_t* y;            // block output [B][OH][OW][ldy] bf16
  const uint16_t* w1;     // sepconv1 pointwise, packed [C1/16][C0/32][64][8] (BN scale folded)
  const float* b1;        // [C1] BN shift
  const float* dw1;       // sepconv1 depthwise [9][C0] fp32
  const uint16_t* w2;     // sepconv2 pointwise, packed [C1/16][C1/32][64][8]
  const float* b2;
  const float* dw2;       // [9][C1]
  const uint16_t* dwk1;   // the same depthwise weights as pack_dw_entries (MFMA depthwise configs)
  const uint16_t* dwk2;
  const uint16_t* wr;     // residual 1x1/2 conv, packed [C1/16][C0/32][64][8]
  const float* br;
  int B, H, W, OH, OW, ldx, ldy;
  int grid;               // workgroups (= len(step_off) - 1)
  const int4* steps;
  const int* step_off;
  unsigned long long* stamps;   // stamping configs (id >= 100) only: [8 wg][64 steps][5 phases]
};
hipError_t entry_block(int cfg, const EntryBlockArgs& a, hipStream_t s);
int entry_block_config(int cfg, int* c0, int* c1, int* pc, int* lds, int* occ);

// cfg >= C3_CFG_BASE: 3x3 'valid' conv over 2-D tiles with an LDS halo patch (MODE_CONV, cin 32 only,
// conv3x3_2d.hip: Xception block1_conv2).
constexpr int C3_CFG_BASE = 208;
hipError_t conv3x3_2d(int cfg, const ConvGemmArgs& a, hipStream_t s);
int conv3x3_2d_config(int cfg, int* bm, int* bn, int* threads);
// cfg >= S2D_CFG_BASE: fused separable conv over 2-D spatial tiles (MODE_DW only, sepconv_2d.hip).
constexpr int S2D_CFG_BASE = 160;
hipError_t sepconv_2d(int cfg, const ConvGemmArgs& a, hipStream_t s);
int sepconv_2d_config(int cfg, int* bm, int* bn, int* threads);
// cfg == STREAM_CFG_BASE (+1: nontemporal output stores): persistent streaming pointwise GEMM, weights
// resident in LDS (MODE_PW, stride 1, small K; the (K, N) shapes of gemm_stream.hip's instance list
// only; per-image weights ok).
constexpr int STREAM_CFG_BASE = 3000;
hipError_t gemm_stream(const ConvGemmArgs& a, bool nt, hipStream_t s);
bool gemm_stream_shape(int K, int nstore, int dt = 0);
hipError_t conv_gemm(int mode, int cfg, const ConvGemmArgs& a, hipStream_t s);
hipError_t gemm_pipe(int mode, int cfg, const ConvGemmArgs& a, hipStream_t s);
int gemm_pipe_config(int cfg, int* bm, int* bn, int* threads);
int conv_gemm_config(int cfg, int* bm, int* bn, int* threads);
int conv_gemm_num_configs();

// Depthwise 3x3 'same' (+ReLU on load): NHWC bf16 [B][H][W][C] -> same layout.
struct DwArgs {
  const uint16_t* x;
  const float* w;         // [9][C] fp32
  uint16_t* y;
  int B, H, W, C;         // C = padded channel stride (multiple of 8)
  int relu_in;
  int cg, rb, tw, seg;    // tile overrides (0 = host heuristic): 8-ch chunks, rows, cols, cols/item
  int algo;               // 0 = auto, 1 = LDS-tiled, 2 = direct row-streaming (rb / seg / pd apply)
  int pd;                 // direct kernel: input rows prefetched ahead (0 = default)
};
hipError_t dw3x3(const DwArgs& a, hipStream_t s);

// Stem: 3x3 stride-2 'valid' conv, 3 input channels -> 32, + bias + ReLU.
// in_kind: 0 = uint8 HWC pixels (Xception normalisation folded into weights),
//          1 = fp32 HWC already preprocessed (TF-Serving compat input).
struct StemArgs {
  const void* x;
  const uint16_t* wp;     // packed [cout/16][K32][64][8], k = (ky*KW+kx)*3 + c
  const float* bias;      // [cout]
  uint16_t* y;            // [B*OH*OW][ldy]
  int B, H, W, OH, OW, ldy;
  int in_kind;
  int KH, KW, stride, pad, cout;  // generic KxK stride/pad conv from 3 channels (cout = 32 or 64)
  float scale[3], shift[3];       // per-channel input normalisation applied on load (zero padding
                                  // stays exact: padded taps are 0 in the normalised space)
  int relu;                       // 0 none, 1 ReLU, 2 SiLU
  int dt;                         // output element type: 0 bf16, 1 fp16
  int rows;                       // 1: row-run K layout (k = ky*RP + kx*3 + c, RP = 32 for 7x7,
                                  // 16 for 3x3; stem_rows_kernel); 0: k = (ky*KW+kx)*3 + c
};
hipError_t stem_conv(const StemArgs& a, hipStream_t s);

// TF-'same' 3x3/2 max-pool of `x` plus `res` (Xception entry/exit block tail).
struct PoolAddArgs {
  const uint16_t* x;      // [B][H][W][C]
  const uint16_t* res;    // [B][OH][OW][C] or null
  uint16_t* y;            // [B][OH][OW][C]
  int B, H, W, OH, OW, C; // C multiple of 8
  int pad_top, pad_left;
  int dt;                 // element type: 0 bf16, 1 fp16
  int algo;               // 0 auto, 1 pixel-per-thread, 2 row-streaming (seg / rb apply)
  int seg, rb;            // row-streaming: output columns per thread, output rows per band (0 = plan)
};
hipError_t pool_add(const PoolAddArgs& a, hipStream_t s);

// Global average pool: x [B][HW][ldx] bf16 -> y [B][F] fp32.
struct GapArgs {
  const uint16_t* x;
  float* y;               // [B][F] fp32 (may be null)
  uint16_t* yb;           // [B][F] bf16 copy for the MFMA classifier (may be null)
  int B, HW, ldx, F;      // F multiple of 8
  int dt;                 // element type of x and yb: 0 bf16, 1 fp16
};
hipError_t gap(const GapArgs& a, hipStream_t s);

// Dense layer on pooled features: out[b][n] = sum_k x[b][k] w[k][n] + bias[n] (+ReLU), fp32.
struct FcArgs {
  const float* x;         // [B][F]
  const float* w;         // [F][N] (Keras Dense / transposed torch Linear layout)
  const float* bias;      // [N]
  float* out;             // [B][N]
  int B, F, N, relu;
};
hipError_t fc(const FcArgs& a, hipStream_t s);

// MFMA classifier: out[b][n] = sum_k xb[b][k] W[n][k] + bias[n] (+ReLU), fp32 out.
// xb: bf16 [rows >= round_up(B,16)][F] (rows >= B zero), wp: packed [NF][F/32][64][8].
struct FcMfmaArgs {
  const uint16_t* xb;
  const uint16_t* wp;
  const float* bias;
  float* out;
  int B, F, N, NF, relu;
  int dt;                 // element type of xb and wp: 0 bf16, 1 fp16
};
hipError_t fc_mfma(const FcMfmaArgs& a, hipStream_t s);

// ViT patch embedding input: uint8 NHWC image -> A [B*np][3*P*P] bf16, k = c*P*P + ky*P + kx,
// normalised on load (per-channel scale/shift).
struct PatchifyArgs {
  const uint8_t* x;
  uint16_t* y;
  int B, H, W, P, ldy;
  float scale[3], shift[3];
};
hipError_t patchify(const PatchifyArgs& a, hipStream_t s);

// Token finalise: x [B][T][D] bf16 (rows 1..T-1 = patch embeddings); row 0 := cls + pos[0],
// rows t >= 1 += pos[t]. cls [D], pos [T][D] fp32.
struct EmbedArgs {
  uint16_t* x;
  const float* cls;
  const float* pos;
  int B, T, D;
};
hipError_t embed_tokens(const EmbedArgs& a, hipStream_t s);

// LayerNorm over the last dim (D <= 2048): y[r][:D] = LN(x[r*ldx .. +D]) * gamma + beta, bf16.
struct LnArgs {
  const uint16_t* x;
  uint16_t* y;
  uint8_t* y8;            // optional e4m3 output (value * inv_scale) instead of y
  float inv_scale;
  const float* gamma;
  const float* beta;
  long rows;
  int D, ldx, ldy;
  float eps;
};
hipError_t layernorm(const LnArgs& a, hipStream_t s);

// Multi-head self-attention (flash-style, online softmax) over a packed QKV buffer:
// qkv [B*T][3*H*dh] bf16 (q | k | v, head-major inside each), out [B*T][H*dh] bf16.
struct AttnArgs {
  const uint16_t* qkv;
  uint16_t* out;
  uint8_t* out8;          // optional e4m3 output (value * inv_scale) instead of out
  float inv_scale;
  int B, T, H, dh;        // dh = 64
  float scale;            // 1/sqrt(dh)
};
hipError_t attention(const AttnArgs& a, hipStream_t s);

// MBConv depthwise KxK (K 3/5, stride S 1/2, symmetric pad) + bias (+SiLU) with the SE
// average pool and squeeze FC fused: pool[b][part][Cs] = sum over the part's channels of
// w1[j][c] * (sum of the part's outputs of channel c); part = (band, column tile, group).
struct DwkArgs {
  const uint16_t* x;      // [B][H][W][C]
  const float* w;         // [K*K][C] fp32 (BN scale folded)
  const float* bias;      // [C]
  uint16_t* y;            // [B][OH][OW][C]
  float* pool;            // null: no SE
  const float* w1;        // SE fc1 [Cs][C]
  int B, H, W, C, OH, OW, K, S, pad, act;   // act: 0 none, 2 SiLU
  int Cs;
  int cg, rb, tw, seg;    // tile override (0: host heuristic; tools/dwkbench.py sweeps these)
  int lds_kb;             // heuristic's LDS budget per workgroup (0: default)
  int algo;               // 0 auto, 1 LDS-tiled, 2 direct streaming (dwv_kernel)
  int pd;                 // dwv_kernel: input rows prefetched ahead (0: table / 1)
};
hipError_t dwk(const DwkArgs& a, hipStream_t s);
void dwk_tiles(const DwkArgs& a, int* cg, int* rb, int* tw, int* ntiles);
int dwk_seg(const DwkArgs& a);

// Squeeze-excite tail: scale[b][c] = sigmoid(W2 SiLU(sum_parts pool / HW + b1) + b2).
struct SeArgs {
  const float* pool;      // [B][ntiles][Cs] fc1 partials from dwk
  const float* b1;        // [Cs]
  const float* w2t;       // [Cs][C] (fc2 transposed)
  const float* b2;        // [C]
  float* scale;           // [B][C]
  int B, ntiles, HW, C, Cs;
};
hipError_t squeeze_excite(const SeArgs& a, hipStream_t s);

struct ChScaleArgs {
  uint16_t* y;            // [B][HW][C] bf16, scaled in place
  const float* scale;     // [B][C]
  int B, HW, C;
};
hipError_t channel_scale(const ChScaleArgs& a, hipStream_t s);

// FP8 (OCP e4m3) GEMM, gemm_f8.hip: y = act(colscale[n] * A8 W8^T + bias[n]) (+res), bf16 or fp8 out.
struct GemmF8Args {
  const uint8_t* x;       // A e4m3 [M][ldx bytes]
  const uint8_t* wp;      // packed e4m3 [NF][K/128][2][64][16]
  const float* bias;      // [NF*16]
  const float* colscale;  // [NF*16] = s_a * s_w[n]
  const uint16_t* res;    // optional bf16 residual [M][ldr]
  uint16_t* y;            // bf16 out [M][ldy] (used when y8 is null)
  uint8_t* y8;            // e4m3 out [M][ldy], value / out_scale
  float out_inv_scale;
  int M, K, ldx, ldy, ldr, NF, nstore, relu_out;
  int krot;               // 1: each M tile starts its K loop at its own 128-deep step (env KDL_F8_KROT overrides)
};
hipError_t gemm_f8(int cfg, const GemmF8Args& a, hipStream_t s);
int gemm_f8_config(int cfg, int* bm, int* bn, int* threads);

// Classifier head: GAP over HW -> dense(F->H1)+ReLU -> dense(H1->NC), fp32 logits.
struct HeadArgs {
  const uint16_t* x;      // [B][HW][ldx] bf16
  const float* w1;        // [H1][F] fp32 (the Keras [F][H1] Dense kernel, transposed at load)
  const float* b1;        // [H1]
  const float* w2;        // [H1][NC]
  const float* b2;        // [NC]
  float* out;             // [B][NC]
  float* feat;            // scratch [B][F] fp32 (pooled features)
  float* hid;             // scratch [F/64][B][H1] fp32 (dense1 K-split partials)
  int B, HW, ldx, F, H1, NC;
};
hipError_t head_dense(const HeadArgs& a, hipStream_t s);

// PIL-exact NEAREST resize of one uint8 HWC RGB image into slot `b` of a
// [B][OH][OW][3] uint8 batch, using host-built index tables.
struct ResizeArgs {
  const uint8_t* src;
  uint8_t* dst;
  const int* ytab;        // [OH] source rows
  const int* xtab;        // [OW] source cols
  int SH, SW, OH, OW;
  int n;                  // images of one source size, packed [n][SH][SW][3] -> [n][OH][OW][3] (0 = 1)
};
hipError_t resize_nearest_u8(const ResizeArgs& a, hipStream_t s);

// Elementwise: uint8 HWC image -> Xception-normalised bf16 NHWC padded to ldy
// (x/127.5 - 1), used by the non-folded path and by tests.
hipError_t u8_to_bf16_norm(const uint8_t* x, uint16_t* y, long npix, int ldy, hipStream_t s);

}  // namespace kdl
