// C ABI between the native batch executor (kdl._rt, CPU-only: executor.cpp) and a device
// backend (kdl._C: the HIP backend in hip_backend.cpp; tests: the fake backend in
// executor.cpp). Plain C so the two extension modules, built by different compilers
// (g++ for _rt, hipcc/clang for _C), share no C++ ABI: the executor only calls through
// these function pointers.
//
// Slot protocol (one executor thread drives one backend): the executor lets the batcher
// copy a batch into staging(slot), calls issue(slot, ...) -- asynchronous: H2D, the
// bucket's captured forward, D2H of the logits -- and later complete(slot, ...), which
// blocks until that slot's logits are on the host. A slot is reused only after its
// complete() returned.
//
// Device-resident items (batcher.h submit(..., device=true), e.g. serving_image requests
// the GPU already resized): the executor passes them to issue_dev() as pieces; the backend
// copies those rows device-to-device into its input slot and only the other rows from
// staging. A backend without issue_dev (NULL) fails such batches.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// per-batch device-side stage times (HIP event deltas), filled by complete(); -1 = unknown
typedef struct kdl_device_times {
  float h2d_ms, forward_ms, d2h_ms;
} kdl_device_times;

typedef struct kdl_dev_piece {
  int row, n_items;                              // rows [row, row + n_items) of the batch
  const void* src;                               // device memory, n_items x item_bytes
} kdl_dev_piece;

typedef struct kdl_exec_backend {
  void* ctx;
  int nslots;
  int out_cols;                                  // floats per result row
  uint8_t* (*staging)(void* ctx, int slot);      // pinned host staging of `slot`
  // returns 0 on success (non-zero: the batch failed before anything was queued)
  int (*issue)(void* ctx, int slot, int bucket, int n_real);
  // blocks until `slot`'s results are on the host; *out = host logits [bucket][out_cols]
  int (*complete)(void* ctx, int slot, const float** out, kdl_device_times* t);
  // optional: issue() with `npieces` device-resident row ranges (see above)
  int (*issue_dev)(void* ctx, int slot, int bucket, int n_real, const kdl_dev_piece* pieces, int npieces);
} kdl_exec_backend;

#ifdef __cplusplus
}
#endif
