// HIP device backend of the native batch executor (exec_backend.h / executor.cpp).
//
// Owns, per in-flight slot, pinned host staging for the batch payload and pinned host
// logits, and drives one GPU: issue() = H2D on the copy stream -> the bucket's captured
// forward (one hipGraph, or the K stage graphs of a stage pipeline on K streams with the
// cross-batch parity waits of kdl/engine/stages.py) -> logits D2H behind the last stage;
// complete() waits for the slot's done event and reports H2D / forward / D2H device times
// from HIP events. Every call is asynchronous except complete(); nothing allocates after
// construction. issue_dev() takes batches with device-resident rows (serving_image requests
// resized on the GPU straight into device memory: no host round trip).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <vector>

#include "engine.h"
#include "exec_backend.h"

namespace kdl {

class HipExecBackend {
 public:
  HipExecBackend(int device, int nslots, size_t item_bytes, int max_batch, int out_cols, hipStream_t copy_stream,
                 bool timing);
  ~HipExecBackend();
  HipExecBackend(const HipExecBackend&) = delete;
  HipExecBackend& operator=(const HipExecBackend&) = delete;

  // Device work of batch bucket `bucket`: K stages on `streams`; stage k also waits for stage
  // wait_for[k] of the batch two back with the same parity when wait_for[k] > k.
  // progs[slot][parity][k]; dev_in[slot] / dev_out[slot]: the engine's input slot and logits.
  void add_recipe(int bucket, const std::vector<hipStream_t>& streams, const std::vector<int>& wait_for,
                  const std::vector<std::vector<std::vector<const Program*>>>& progs,
                  const std::vector<void*>& dev_in, const std::vector<void*>& dev_out);

  const kdl_exec_backend* api() const { return &api_; }
  uint8_t* staging(int slot) { return staging_[slot]; }
  const float* host_out(int slot) const { return out_[slot]; }
  int issue(int slot, int bucket, int n_real);
  // issue() whose rows of `pieces` come from device memory (D2D on the copy stream; the
  // host rows are H2D'd in contiguous runs around them)
  int issue_dev(int slot, int bucket, int n_real, const kdl_dev_piece* pieces, int npieces);
  // the recipe of `bucket` alone (no copies): stage 0 waits `ready`; *last = the last stage's
  // stream (its work is queued behind the forward). For the data-parallel ranks (comm.cpp).
  int launch(int slot, int bucket, hipEvent_t ready, hipStream_t* last);
  void* dev_in(int slot, int bucket) const;
  void* dev_out(int slot, int bucket) const;
  int device() const { return device_; }
  int nslots() const { return nslots_; }
  int max_batch() const { return max_batch_; }
  size_t item_bytes() const { return item_bytes_; }
  int out_cols() const { return out_cols_; }
  hipStream_t copy_stream() const { return copy_; }
  float* host_out_mut(int slot) { return out_[slot]; }
  hipEvent_t done_event(int slot) const { return ev_done_[slot]; }
  int complete(int slot, const float** out, kdl_device_times* t);

 private:
  int finish_issue(int slot, int bucket);      // recipe launch + D2H behind the copies
  struct Recipe {
    int K = 1;
    std::vector<hipStream_t> streams;
    std::vector<int> wait_for;
    std::vector<std::vector<std::vector<const Program*>>> progs;
    std::vector<void*> dev_in, dev_out;
    std::vector<hipEvent_t> done[2];            // [parity][stage]
    long issued = 0;
  };
  int device_;
  int nslots_;
  size_t item_bytes_;
  int max_batch_, out_cols_;
  hipStream_t copy_;
  bool own_copy_ = false, timing_;
  std::vector<uint8_t*> staging_;
  std::vector<float*> out_;
  // per slot: h2d start/end (copy stream), forward start/end, done (after the D2H)
  std::vector<hipEvent_t> ev_h2d0_, ev_h2d1_, ev_fw0_, ev_fw1_, ev_done_;
  std::map<int, Recipe> recipes_;
  std::vector<int> slot_bucket_;
  kdl_exec_backend api_{};
};

}  // namespace kdl
