// Native per-device batch executor (TF-Serving's servable session run;
// §5 tracing). One C++ thread per (device, executor) pulls formed batches from the
// DynamicBatcher straight into its backend's pinned staging, issues them (H2D ->
// captured forward -> D2H, asynchronous, kdl_exec_backend::issue) with up to `nslots`
// batches in flight, completes them in order and scatters the logits back to the
// waiting request handlers -- no Python and no GIL anywhere on this path.
//
// Per-device fault isolation: after max_failures consecutive failed batches the
// executor marks itself unhealthy and stops pulling, so the shared batcher routes
// everything to the remaining executors; when the last executor of a group gives up
// the batcher is shut down (queued waiters fail instead of blocking forever).
//
// Tracing: every batch is stamped at formation (batch formed from the queue), after
// the payload copy into staging, after issue, after completion and after finish; the
// backend adds device-side H2D / forward / D2H times from HIP events. Stage histograms
// and a ring of the most recent batch traces are exported (Prometheus + /monitoring).
#pragma once
#include <stdint.h>

#include <atomic>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "batcher.h"
#include "exec_backend.h"

namespace kdl {

// Stage names, in the order of ExecStats::hist / BatchTrace stamps.
enum ExecStage {
  STAGE_QUEUE_WAIT = 0,   // oldest request enqueued -> batch formed
  STAGE_HOST_COPY,        // batch formed -> payloads copied into pinned staging
  STAGE_ISSUE,            // host time of issue() (H2D + graph launch + D2H enqueue)
  STAGE_DEVICE_H2D,       // device: H2D copy            (backend event delta)
  STAGE_DEVICE_FORWARD,   // device: captured forward    (backend event delta)
  STAGE_DEVICE_D2H,       // device: logits D2H          (backend event delta)
  STAGE_IN_FLIGHT,        // issued -> complete() returned (includes waiting behind earlier batches)
  STAGE_BATCH_LATENCY,    // oldest request enqueued -> results scattered (finish)
  N_STAGES
};
const char* exec_stage_name(int s);

// histogram bucket upper bounds in milliseconds (last bucket = +inf)
constexpr int N_BUCKETS = 14;
extern const double kBucketsMs[N_BUCKETS];

struct StageHist {
  int64_t count = 0;
  double sum_ms = 0;
  int64_t buckets[N_BUCKETS] = {0};
  void add(double ms);
};

struct BatchTrace {
  int64_t batch_id = 0;
  int n_real = 0, bucket = 0, slot = 0, status = 0;
  int64_t oldest_enqueue_us = 0, formed_us = 0, copied_us = 0, issued_us = 0, completed_us = 0, finished_us = 0;
  float h2d_ms = -1, forward_ms = -1, d2h_ms = -1;
};

struct ExecStats {
  int64_t batches = 0, items = 0, padded_items = 0, failed_batches = 0;
  bool healthy = true;
  StageHist hist[N_STAGES];
};

// Shared by the executors of one batcher: counts the healthy ones.
class ExecGroup {
 public:
  void join() { healthy_.fetch_add(1); }
  // returns true when the caller was the last healthy executor
  bool leave() { return healthy_.fetch_sub(1) == 1; }
  int healthy() const { return healthy_.load(); }

 private:
  std::atomic<int> healthy_{0};
};

struct ExecOptions {
  std::string name = "exec";
  bool eager = true;            // work-conserving: an idle device takes whatever is queued
  int max_failures = 3;
  int64_t poll_us = 100000;     // batcher poll while idle (wakes for stop())
  // fault injection (tests; KDL_FAULT_INJECT): fail the next `fail_batches` batches (-1 =
  // every batch), delay every batch by `delay_us` before issue
  int fail_batches = 0;
  int64_t delay_us = 0;
  int trace_ring = 256;         // recent batch traces kept
};

class Executor {
 public:
  Executor(DynamicBatcher* batcher, const kdl_exec_backend* backend, ExecGroup* group, const ExecOptions& o);
  ~Executor();
  Executor(const Executor&) = delete;
  Executor& operator=(const Executor&) = delete;

  void start();
  void stop();                  // finishes what is in flight, joins the thread
  bool healthy() const { return healthy_.load(); }
  bool running() const { return running_.load(); }
  ExecStats stats() const;
  std::vector<BatchTrace> recent(int n) const;
  const ExecOptions& options() const { return opt_; }

 private:
  struct Pending {
    Batch batch;
    int slot;
    BatchTrace tr;
  };
  void loop();
  bool fail(Batch& b, BatchTrace& tr);     // true: this executor gives up its device
  void record(const BatchTrace& tr, const Batch& b);

  DynamicBatcher* batcher_;
  kdl_exec_backend be_;
  ExecGroup* group_;
  ExecOptions opt_;
  std::thread th_;
  std::atomic<bool> stop_{false}, healthy_{true}, running_{false};
  int failures_ = 0;
  int fail_left_ = 0;
  mutable std::mutex mu_;
  ExecStats st_;
  std::deque<BatchTrace> ring_;
};

// Fake device backend for CPU tests and the sanitizer stress binary: result row i of a
// batch = {first byte of item i, +1, +2, ...}; `latency_us` of simulated device time per
// batch; fail_every > 0 fails every n-th issue. Its "device" items are host pointers.
struct FakeBackend {
  FakeBackend(int nslots, size_t item_bytes, int max_batch, int out_cols, int64_t latency_us, int fail_every = 0);
  kdl_exec_backend api{};
  std::vector<std::vector<uint8_t>> staging;
  std::vector<std::vector<float>> out;
  std::vector<int64_t> ready_at;
  std::vector<int> bucket;
  size_t item_bytes;
  int out_cols;
  int64_t latency_us;
  int fail_every, issued = 0;
  int dev_pieces = 0;                        // issue_dev calls (device-resident items)
};

}  // namespace kdl
