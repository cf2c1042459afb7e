// Native per-GPU executor (the TF-Serving "servable/session run"
// equivalent). A Program is a flat, pre-resolved list of kernel launches with
// every pointer and shape fixed at build time (static memory plan, no allocation
// on the hot path). It can run eagerly, be captured once into a hipGraph and then
// replayed with a single hipGraphLaunch per batch, or be timed op-by-op with HIP
// events (the per-layer trace used by the autotuner and the metrics endpoint).
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/launch.h"

namespace kdl {

enum OpKind { OP_CONV_GEMM = 0, OP_STEM = 1, OP_POOL_ADD = 2, OP_HEAD = 3, OP_RESIZE = 4, OP_MEMSET = 5, OP_DW = 6, OP_GAP = 7, OP_FC = 8, OP_FC_MFMA = 9,
              OP_PATCHIFY = 10, OP_EMBED = 11, OP_LN = 12, OP_ATTN = 13,
              OP_DWK = 14, OP_SE = 15, OP_CHSCALE = 16, OP_GEMM_F8 = 17,
              OP_ENTRY_BLOCK = 21 };   // 18: retired (round 6: the SE weight scale, replaced by the project
                                       // GEMM's A-operand scales); 19: retired (the round-3 chained
                                       // middle-flow launch); 20: retired (round 5: the vendor GEMM node
                                       // left the product, tools/probes/blaslt)

struct Op {
  OpKind kind;
  std::string name;
  int mode = 0, cfg = 0;
  ConvGemmArgs g{};
  StemArgs st{};
  PoolAddArgs pa{};
  HeadArgs hd{};
  ResizeArgs rs{};
  DwArgs dw{};
  GapArgs gp{};
  FcArgs fc{};
  FcMfmaArgs fcm{};
  PatchifyArgs pt{};
  EmbedArgs em{};
  LnArgs ln{};
  AttnArgs at{};
  DwkArgs dk{};
  SeArgs se{};
  ChScaleArgs cs{};
  GemmF8Args f8{};
  EntryBlockArgs eb{};
  void* mem_ptr = nullptr;
  size_t mem_bytes = 0;
};

void check_hip(hipError_t e, const std::string& what);

hipError_t run_op(const Op& op, hipStream_t s);

class Program {
 public:
  Program() = default;
  ~Program();
  Program(const Program&) = delete;
  Program& operator=(const Program&) = delete;

  void add(const Op& op) {
    if (exec_) throw std::runtime_error("Program already captured; reset() first");
    ops_.push_back(op);
  }
  size_t size() const { return ops_.size(); }
  const Op& op(size_t i) const { return ops_.at(i); }
  Op& mutable_op(size_t i) { return ops_.at(i); }

  // Launch every op in order on `s` (no sync).
  void run(hipStream_t s) const;
  // Capture the op list into a hipGraph on `s` (must be a non-default stream).
  void capture(hipStream_t s);
  // Replay the captured graph (or run eagerly when not captured).
  void launch(hipStream_t s) const;
  bool captured() const { return exec_ != nullptr; }
  void reset();
  // Per-op device time in milliseconds, median of `iters` eager runs.
  std::vector<float> profile(hipStream_t s, int iters) const;

 private:
  std::vector<Op> ops_;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace kdl
