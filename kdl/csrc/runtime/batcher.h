// Deadline-aware dynamic batcher (TF-Serving BasicBatchScheduler equivalent,
// SURVEY.md §2.3 X2 / §2.10 C5, C16).
//
// Producers (gRPC / REST handler threads, GIL released) submit requests of
// n_items fixed-size items and block in wait(). Consumers (one executor thread per
// GPU) call next_batch(), which forms a batch of up to max_batch_size items once
// the queue holds a full batch or the oldest request has waited
// batch_timeout_us, drops requests whose deadline has passed, copies the
// payloads into the consumer's pinned staging buffer and rounds the batch up to
// the smallest allowed bucket (one captured hipGraph per bucket). finish()
// scatters result rows back and wakes the producers.
//
// Knobs mirror TF-Serving's --batching_parameters_file: max_batch_size,
// batch_timeout_micros, max_enqueued_batches, allowed_batch_sizes.
#pragma once
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace kdl {

struct BatcherOptions {
  int max_batch_size = 32;
  int64_t batch_timeout_us = 2000;
  int max_enqueued_batches = 1000;
  std::vector<int> allowed_batch_sizes;      // sorted ascending; empty = exact batch sizes
  size_t item_bytes = 0;
  int out_cols = 0;                          // floats per item result row
  int copy_threads = 4;                      // threads for a batch's payload copy into staging
};

enum BatchStatus { ST_OK = 0, ST_DEADLINE = 1, ST_SHUTDOWN = 2, ST_ERROR = 3, ST_PENDING = 4, ST_QUEUE_FULL = 5 };

struct Batch {
  int64_t id = 0;
  int n_real = 0;                            // real items
  int bucket = 0;                            // padded batch size (graph bucket)
  std::vector<int64_t> tickets;
  std::vector<int> first_item;               // offset of each ticket's items in the batch
  std::vector<int> n_items;
  // per ticket: nullptr = the payload was copied into staging; else a DEVICE pointer the
  // backend copies device-to-device into its input slot (kdl_exec_backend::issue_dev)
  std::vector<const uint8_t*> dev_src;
  int64_t oldest_enqueue_us = 0;
  int64_t formed_us = 0;                     // batch formed (before the payload copy)
};

struct BatcherStats {
  int64_t submitted = 0, completed = 0, expired = 0, rejected = 0, batches = 0, items = 0, padded_items = 0;
  int64_t queue_items = 0;
};

int64_t now_us();

// Persistent pool for the payload copies of formed batches (a full Xception batch is
// 8.6 MB into pinned staging: ~1 ms on one thread). Jobs from concurrent next_batch
// callers (one per GPU executor) share the workers; the caller always works on its own
// job too, so a pool whose threads could not be started degrades to a plain memcpy.
class CopyPool {
 public:
  struct Piece { uint8_t* dst; const uint8_t* src; size_t n; };
  explicit CopyPool(int threads);
  ~CopyPool();
  void run(const std::vector<Piece>& pieces);   // returns when every piece is copied
  int threads() const { return int(workers_.size()); }

 private:
  struct Job {
    const std::vector<Piece>* pieces;
    std::atomic<size_t> next{0}, done{0};
    int users = 0;                              // workers inside drain() (guarded by mu_)
  };
  void worker();
  static void drain(Job& j);
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::deque<Job*> jobs_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
};

class DynamicBatcher {
 public:
  explicit DynamicBatcher(const BatcherOptions& o);
  ~DynamicBatcher();

  // Producer: returns a ticket (> 0) or -ST_QUEUE_FULL / -ST_SHUTDOWN / -ST_ERROR.
  // `data` must stay valid until wait() returns for this ticket. `device`: `data` is device
  // memory (e.g. an image the GPU resized): next_batch does not copy it, the batch lists it in
  // dev_src and the executor's backend copies it on the device; it must then stay valid
  // until the batch's device work is done, not only until wait() (deadline-expired tickets
  // return early), so device payloads come from buffers that are recycled, never freed.
  int64_t submit(const uint8_t* data, int n_items, int64_t deadline_us, bool device = false);
  // Callback form for event-driven producers (the native gRPC front-end, runtime/grpc_front.h):
  // nothing blocks; `done(status, rows, n_floats)` runs exactly once -- on the executor thread
  // that finishes the batch (rows valid only during the call), on the consumer that drops the
  // expired request, or in shutdown() -- never under the batcher's lock. `data` must stay valid
  // until then. Returns the ticket, or -status without calling `done`.
  using DoneFn = std::function<void(int status, const float* rows, size_t n_floats)>;
  int64_t submit_async(const uint8_t* data, int n_items, int64_t deadline_us, DoneFn done);
  // Blocks until the request completes or its deadline passes; copies
  // n_items*out_cols floats into `out`, which holds `out_floats` floats (a smaller
  // buffer is not written and the call returns ST_ERROR). Returns a BatchStatus.
  int wait(int64_t ticket, float* out, size_t out_floats);

  // Consumer: waits up to poll_us for a batch; false on timeout/shutdown. A batch forms
  // when max_batch_size items are queued or the oldest has waited batch_timeout_us; with
  // `eager` (the caller's device is idle) as soon as anything is queued -- work-conserving
  // dispatch: an idle GPU never waits out the timeout, a busy one still gets full batches.
  bool next_batch(uint8_t* staging, int64_t poll_us, Batch* b, bool eager = false);
  void finish(const Batch& b, const float* results, int status);

  void shutdown();
  BatcherStats stats() const;
  int bucket_for(int n) const;
  const BatcherOptions& options() const { return opt_; }

 private:
  enum State { QUEUED, TAKEN, COPIED, DONE, ABANDONED };
  struct Req {
    int64_t ticket;
    const uint8_t* data;
    bool device = false;
    int n_items;
    int64_t enqueue_us, deadline_us;
    State state = QUEUED;
    int status = ST_PENDING;
    std::vector<float> result;
    DoneFn done;                             // submit_async: completion callback (no wait())
  };
  int64_t enqueue_locked(const uint8_t* data, int n_items, int64_t deadline_us, bool device, DoneFn done);
  BatcherOptions opt_;
  mutable std::mutex mu_;
  std::condition_variable cv_consumer_, cv_producer_;
  std::deque<std::shared_ptr<Req>> queue_;
  std::unordered_map<int64_t, std::shared_ptr<Req>> live_;
  std::unordered_map<int64_t, std::shared_ptr<Req>> async_live_;   // submit_async tickets until done
  int64_t next_ticket_ = 1, next_batch_ = 1, queued_items_ = 0;
  bool shutdown_ = false;
  BatcherStats st_;
  std::unique_ptr<CopyPool> pool_;           // copy_threads - 1 persistent workers
};

}  // namespace kdl
