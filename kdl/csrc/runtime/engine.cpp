#include "engine.h"

#include <algorithm>

namespace kdl {

void check_hip(hipError_t e, const std::string& what) {
  if (e != hipSuccess) throw std::runtime_error(what + ": " + hipGetErrorString(e));
}

hipError_t run_op(const Op& op, hipStream_t s) {
  switch (op.kind) {
    case OP_CONV_GEMM: return conv_gemm(op.mode, op.cfg, op.g, s);
    case OP_STEM: return stem_conv(op.st, s);
    case OP_POOL_ADD: return pool_add(op.pa, s);
    case OP_HEAD: return head_dense(op.hd, s);
    case OP_RESIZE: return resize_nearest_u8(op.rs, s);
    case OP_MEMSET: return hipMemsetAsync(op.mem_ptr, 0, op.mem_bytes, s);
    case OP_DW: return dw3x3(op.dw, s);
    case OP_GAP: return gap(op.gp, s);
    case OP_FC: return fc(op.fc, s);
    case OP_FC_MFMA: return fc_mfma(op.fcm, s);
    case OP_PATCHIFY: return patchify(op.pt, s);
    case OP_EMBED: return embed_tokens(op.em, s);
    case OP_LN: return layernorm(op.ln, s);
    case OP_ATTN: return attention(op.at, s);
    case OP_DWK: return dwk(op.dk, s);
    case OP_SE: return squeeze_excite(op.se, s);
    case OP_CHSCALE: return channel_scale(op.cs, s);
    case OP_GEMM_F8: return gemm_f8(op.cfg, op.f8, s);
    case OP_ENTRY_BLOCK: return entry_block(op.cfg, op.eb, s);
  }
  return hipErrorInvalidValue;
}

Program::~Program() { reset(); }

void Program::reset() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
}

void Program::run(hipStream_t s) const {
  for (const auto& op : ops_) check_hip(run_op(op, s), "launch " + op.name);
}

void Program::capture(hipStream_t s) {
  reset();
  check_hip(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
  hipError_t err = hipSuccess;
  std::string bad;
  for (const auto& op : ops_) {
    err = run_op(op, s);
    if (err != hipSuccess) { bad = op.name; break; }
  }
  hipGraph_t g = nullptr;
  const hipError_t e2 = hipStreamEndCapture(s, &g);
  if (err != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    check_hip(err, "capture launch " + bad);
  }
  check_hip(e2, "hipStreamEndCapture");
  graph_ = g;
  check_hip(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
}

void Program::launch(hipStream_t s) const {
  if (exec_) check_hip(hipGraphLaunch(exec_, s), "hipGraphLaunch");
  else run(s);
}

std::vector<float> Program::profile(hipStream_t s, int iters) const {
  const size_t n = ops_.size();
  std::vector<hipEvent_t> ev(n + 1);
  for (auto& e : ev) check_hip(hipEventCreate(&e), "hipEventCreate");
  std::vector<std::vector<float>> t(n);
  for (int it = 0; it < iters; ++it) {
    check_hip(hipEventRecord(ev[0], s), "record");
    for (size_t i = 0; i < n; ++i) {
      check_hip(run_op(ops_[i], s), "launch " + ops_[i].name);
      check_hip(hipEventRecord(ev[i + 1], s), "record");
    }
    check_hip(hipEventSynchronize(ev[n]), "sync");
    for (size_t i = 0; i < n; ++i) {
      float ms = 0.f;
      check_hip(hipEventElapsedTime(&ms, ev[i], ev[i + 1]), "elapsed");
      t[i].push_back(ms);
    }
  }
  std::vector<float> med(n, 0.f);
  for (size_t i = 0; i < n; ++i) {
    auto v = t[i];
    if (v.empty()) continue;
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    med[i] = v[v.size() / 2];
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return med;
}

}  // namespace kdl
