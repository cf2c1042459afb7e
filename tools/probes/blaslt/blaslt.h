// TOOLS-ONLY PROBE (round 5): the hipBLASLt GEMM node that rounds 3-4 offered the engines' tuner.
// It left kdl._C -- every GEMM of the product is a hand-written MFMA kernel -- and is kept here
// as source for vendor comparisons (build it next to a binding of your own; the committed
// vendor yardstick is tools/gemm_vs_vendor.py, which times torch's hipBLASLt path).
//
// Vendor GEMM node (hipBLASLt) for the plain dense linears of the engines.
//
// The task's split: hand-written MFMA kernels for the fused hot ops, hipBLASLt only for
// plain library GEMMs. A linear whose epilogue hipBLASLt expresses natively -- bias, ReLU
// after bias, a residual added as its C operand (beta = 1, in place when C == D) -- is a
// plain GEMM; the engines' graph tuner offers it beside the hand-written tiles (config ids
// >= BLT_BASE in kdl/ops/conv.py, id - BLT_BASE = rank in hipBLASLt's heuristic list) and
// keeps whichever wins the whole captured graph (profiles/vit_blaslt_r3.txt).
//
// Row-major Y[M][N] = X[M][K] W[N][K]^T + bias (+ R) maps onto hipBLASLt's column-major
// "TN" problem m = N, n = M, k = K: A = W^T (K x N, ld K) transposed, B = X^T (K x M, ld
// ldx), C = R^T / D = Y^T (N x M, ld ldr / ldy); the bias runs along m (output channels).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>

namespace kdl {

struct BlasLtPlan;   // descriptors, layouts, chosen algorithm, workspace (blaslt.cpp)

struct BlasLtArgs {
  const void* x = nullptr;      // [M][ldx] activations
  const void* w = nullptr;      // [N][K] row-major weights (unpacked)
  void* y = nullptr;            // [M][ldy]
  const void* res = nullptr;    // [M][ldr] residual (C operand, beta = 1) or null
  const float* bias = nullptr;  // [N] fp32 or null
  int M = 0, N = 0, K = 0, ldx = 0, ldy = 0, ldr = 0;
  int act = 0;                  // applied last, after bias and the residual C: 1 ReLU, 2 GELU (hipBLASLt's)
  int dt = 0;                   // 0 bf16, 1 fp16 (x, w, y, res); 2: x, w OCP e4m3, y / res bf16
  const float* wscale = nullptr;  // dt 2: per-output-channel [N] dequant scale of w (x scale folded in)
  int algo = 0;                 // rank in the heuristic list (clamped to the list's length)
  std::shared_ptr<BlasLtPlan> plan;   // built by blaslt_prepare (Program ops keep theirs)
};

// Build descriptors, query the heuristic, allocate the algorithm's workspace. Throws on a
// shape hipBLASLt rejects. Returns the number of algorithms the heuristic offered.
int blaslt_prepare(BlasLtArgs& a);
// Enqueue the GEMM on s (graph-capturable). Prepares on first use.
hipError_t blaslt_run(BlasLtArgs& a, hipStream_t s);
hipError_t blaslt_run(const BlasLtArgs& a, hipStream_t s);

}  // namespace kdl
