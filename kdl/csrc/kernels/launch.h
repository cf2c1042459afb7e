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
  const uint16_t* res;   // optional residual [M][ldr] bf16 (added after ReLU)
  uint16_t* y;           // output [M][ldy] bf16
  int B, H, W;           // input spatial dims
  int OH, OW;            // output spatial dims
  int M;                 // B*OH*OW
  int ldx, ldy, ldr;     // channel strides (elements)
  int K;                 // reduction depth (multiple of 32)
  int cin;               // MODE_CONV: padded input channels (multiple of 32)
  int NF;                // 16-wide output-channel fragments in the packed weights
  int nstore;            // output channels written (<= ldy)
  int stride;            // MODE_PW spatial stride
  int relu_in, relu_out;
};

// cfg < PIPE_CFG_BASE: register-B kernel (all modes, incl. fused depthwise);
// cfg >= PIPE_CFG_BASE: LDS-DMA pipelined kernel (MODE_PW / MODE_CONV only).
constexpr int PIPE_CFG_BASE = 16;
// cfg >= SEP_CFG_BASE: fused separable conv (MODE_DW only, sepconv_fused.hip).
constexpr int SEP_CFG_BASE = 64;
hipError_t sepconv_fused(int cfg, const ConvGemmArgs& a, hipStream_t s);
int sepconv_fused_config(int cfg, int* bm, int* bn, int* threads);
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
};
hipError_t dw3x3(const DwArgs& a, hipStream_t s);

// Stem: 3x3 stride-2 'valid' conv, 3 input channels -> 32, + bias + ReLU.
// in_kind: 0 = uint8 HWC pixels (Xception normalisation folded into weights),
//          1 = fp32 HWC already preprocessed (TF-Serving compat input).
struct StemArgs {
  const void* x;
  const uint16_t* wp;     // packed [2][1][64][8]
  const float* bias;      // [32]
  uint16_t* y;            // [B*OH*OW][ldy]
  int B, H, W, OH, OW, ldy;
  int in_kind;
};
hipError_t stem_conv(const StemArgs& a, hipStream_t s);

// TF-'same' 3x3/2 max-pool of `x` plus `res` (Xception entry/exit block tail).
struct PoolAddArgs {
  const uint16_t* x;      // [B][H][W][C]
  const uint16_t* res;    // [B][OH][OW][C] or null
  uint16_t* y;            // [B][OH][OW][C]
  int B, H, W, OH, OW, C; // C multiple of 8
  int pad_top, pad_left;
};
hipError_t pool_add(const PoolAddArgs& a, hipStream_t s);

// Classifier head: GAP over HW -> dense(F->H1)+ReLU -> dense(H1->NC), fp32 logits.
struct HeadArgs {
  const uint16_t* x;      // [B][HW][ldx] bf16
  const float* w1;        // [F][H1] fp32 (Keras Dense kernel layout)
  const float* b1;        // [H1]
  const float* w2;        // [H1][NC]
  const float* b2;        // [NC]
  float* out;             // [B][NC]
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
};
hipError_t resize_nearest_u8(const ResizeArgs& a, hipStream_t s);

// Elementwise: uint8 HWC image -> Xception-normalised bf16 NHWC padded to ldy
// (x/127.5 - 1), used by the non-folded path and by tests.
hipError_t u8_to_bf16_norm(const uint8_t* x, uint16_t* y, long npix, int ldy, hipStream_t s);

}  // namespace kdl
