// Loopback platform for the data-parallel state machine of dp_core.h ("the C++
// comm layer has a backend interface with a loopback/fake implementation"). Everything a GPU
// rank does, in one process, on the CPU:
//
//   Stream   an in-order queue of host operations run by one worker thread (a HIP stream);
//            an operation that fails makes the stream's error sticky, as HIP's is
//   Event    a mark in a stream's queue: done once every earlier operation of that stream ran
//   memory   host memory stands in for device memory
//   Comm     a communicator of `size` ranks sharing one World (looked up by id, like an RCCL
//            unique id): ordered per-(src, dst) queues of posted sends and receives, matched in
//            order with RENDEZVOUS semantics -- a send completes only when its receive is posted,
//            and a size mismatch fails both ends -- so a schedule RCCL would deadlock or
//            mis-deliver on deadlocks or fails here too. Operations between group_start and
//            group_end (per thread, like ncclGroupStart) are posted together as one stream
//            operation, so a group's sends to several peers cannot deadlock on their order.
//   kill     a rank "dies": none of its operations matches any more (a crashed or hung process).
//   abort    fails this rank's pending and later operations (ncclCommAbort).
//   Device   the fake engine (Local): logits row i of a forward = f(first 4 bytes of input row
//            i, model version) after `latency_us`; issue/complete like HipExecBackend.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dp_core.h"
#include "exec_backend.h"

namespace kdl {
namespace loop {

class Stream {
 public:
  Stream();
  ~Stream();                                   // cancels blocked operations, joins the worker
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  void push(std::function<int()> op);
  uint64_t mark();                             // number of operations queued so far
  // blocks until the first n operations ran (0) or the stream failed (-1) or `cancel` is set (-1)
  int wait_reached(uint64_t n, const std::atomic<bool>* cancel);
  int query(uint64_t n);                       // 1 reached, 0 pending, -1 failed
  int sync();
  const std::atomic<bool>& cancelled() const { return cancel_; }

 private:
  void run();
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<int()>> q_;
  uint64_t queued_ = 0, done_ = 0;
  bool error_ = false, stop_ = false;
  std::atomic<bool> cancel_{false};
  std::thread th_;
};

class Event {
 public:
  void record(Stream* s);
  int query();
  // the (stream, mark) pair of the latest record (nullptr: never recorded = complete)
  std::pair<Stream*, uint64_t> get();

 private:
  std::mutex mu_;
  Stream* s_ = nullptr;
  uint64_t mark_ = 0;
};

struct World;

class Comm {
 public:
  Comm(const std::string& id, int nranks, int rank);
  int rank() const { return rank_; }
  int size() const { return size_; }
  void kill();                                 // this rank stops matching (a dead process)
  void abort();                                // fail this rank's pending / later operations
  bool error() const;
  World* world() const { return w_.get(); }

 private:
  std::shared_ptr<World> w_;
  int rank_, size_;
};

std::string unique_id();

// One posted operation of a rendezvous group (one communicator).
struct Op {
  bool send;
  const void* sbuf;
  void* rbuf;
  size_t bytes;
  int peer;
  Comm* comm;
};
// the byte mover of a matched (send, receive) pair, named by the receiving post: 0 = delivered,
// else both ends fail. nullptr: memcpy (host memory). The HIP loopback platform (dp_hiploop.h)
// passes a device-to-device copy.
using CopyFn = int (*)(void* dst, const void* src, size_t n);
// Post every op, then block until each was matched (and copied), this rank aborted, or `cancel`
// is set; 0 = all delivered. Used by both loopback platforms from a stream's worker thread.
int rendezvous(const std::vector<Op>& ops, const std::atomic<bool>& cancel, CopyFn copy);

class Device {
 public:
  Device(int rank, int nslots, size_t item_bytes, int max_batch, int out_cols, std::vector<int> buckets, int version,
         int64_t latency_us);
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;
  int device() const { return rank_; }
  int nslots() const { return nslots_; }
  int max_batch() const { return max_batch_; }
  size_t item_bytes() const { return item_bytes_; }
  int out_cols() const { return out_cols_; }
  uint8_t* staging(int slot) { return staging_[slot].data(); }
  float* host_out_mut(int slot) { return out_[slot].data(); }
  void* dev_in(int slot, int bucket);
  void* dev_out(int slot, int bucket);
  int launch(int slot, int bucket, Event* ready, Stream** last);
  int issue(int slot, int bucket, int n_real);
  int complete(int slot, const float** out, kdl_device_times* t);
  long forwards() const { return forwards_.load(); }
  // fault injection (tests): the next n issue() calls fail before touching anything
  void fail_issues(int n) { fail_issues_.store(n); }
  const kdl_exec_backend* api() const { return &api_; }
  // the value the fake forward gives column k of an input row whose first 4 bytes are `id`
  static float logit(uint32_t id, int k, int version) { return float((id & 0xFFFFF) + 1048576u * (version & 15)) + k; }

 private:
  bool has_bucket(int b) const;
  int rank_, nslots_, max_batch_, out_cols_, version_;
  size_t item_bytes_;
  std::vector<int> buckets_;
  int64_t latency_us_;
  std::vector<std::vector<uint8_t>> staging_, din_;
  std::vector<std::vector<float>> out_, dout_;
  std::vector<Event> ev_h2d_, ev_done_;
  std::atomic<long> forwards_{0};
  std::atomic<int> fail_issues_{0};
  kdl_exec_backend api_{};
  Stream copy_, compute_;                      // last members: joined first on destruction
};

}  // namespace loop

struct LoopPlatform {
  using Stream = loop::Stream*;
  using Event = loop::Event*;
  using Comm = loop::Comm;
  using Local = loop::Device;

  static int select(Local&) { return 0; }
  static Stream new_stream(Local&) { return new loop::Stream(); }
  static void free_stream(Stream s) { delete s; }
  static int sync(Stream s) { return s->sync(); }
  static Event new_event(Local&) { return new loop::Event(); }
  static void free_event(Event e) { delete e; }
  static int record(Event e, Stream s) {
    e->record(s);
    return 0;
  }
  static int wait_event(Stream s, Event e);
  static int query(Event e) { return e->query(); }
  static void* dev_alloc(Local&, size_t n) { return ::operator new(n); }
  static void dev_free(Local&, void* p) { ::operator delete(p); }
  static void* host_alloc(size_t n) { return ::operator new(n); }
  static void host_free(void* p) { ::operator delete(p); }
  static int h2d(void* d, const void* s, size_t n, Stream st);
  static int d2h(void* d, const void* s, size_t n, Stream st) { return h2d(d, s, n, st); }
  static int group_start();
  static int group_end();
  static int send(const void* b, size_t n, int peer, Comm& c, Stream s);
  static int recv(void* b, size_t n, int peer, Comm& c, Stream s);
  static int rank(const Comm& c) { return c.rank(); }
  static int size(const Comm& c) { return c.size(); }
  static void abort(Comm& c) { c.abort(); }
  static bool comm_error(const Comm& c) { return c.error(); }
};

using LoopDpLeader = DpLeaderT<LoopPlatform>;
using LoopDpFollower = DpFollowerT<LoopPlatform>;

}  // namespace kdl
