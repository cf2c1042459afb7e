// HIP loopback platform for the data-parallel state machine of dp_core.h: the REAL device side
// (HIP streams, events, hipMalloc'd control words and send buffers, HipExecBackend engines with
// their captured hipGraphs) with every rank of the world as a thread of ONE process, and the
// transport done by device-to-device copies instead of RCCL.
//
// Why: every builder box has one GPU and RCCL refuses two ranks on one
// device (tools/probes/rccl_dup_probe.py), so HipRcclPlatform has only ever run at world 1. With
// this platform the follower's real HipExecBackend::launch, the per-rank graph buckets, the
// device-side control words, DP_RELOAD and a dying rank run at world 2+ on one MI355X; only the
// byte mover differs from production.
//
//   Stream   a HIP stream plus an in-order worker thread (loop::Stream) that enqueues the
//            stream's HIP operations in post order; a send / receive waits for the stream's
//            earlier HIP work (hipStreamSynchronize on the worker), then meets its peer's post
//            (loop::rendezvous, the loopback's ordered per-(src, dst) matching) and the
//            receiving side copies device to device. The posting thread never blocks, as with
//            ncclSend / ncclRecv. An engine's own stream (HipExecBackend::launch's `last`) is
//            wrapped as an EXTERNAL stream: its operations run inline on the caller's thread.
//   Event    one hipEvent per record (a Rec), plus the worker-queue mark of the record: queried
//            done once the worker enqueued the record AND hipEventQuery says so; a wait captures
//            the record current at post time (a later re-record cannot move it).
//   Comm     loop::Comm: the loopback World (ids, ranks, kill, abort).
//   Local    HipLoopLocal: rank's HipExecBackend, with launch() taking this platform's Event /
//            Stream types.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>

#include "dp_core.h"
#include "dp_loop.h"
#include "hip_backend.h"

namespace kdl {
namespace hl {

struct Stream {
  int device = 0;
  hipStream_t hs = nullptr;
  bool external = false;                         // an engine's stream: ops inline, no worker
  std::unique_ptr<loop::Stream> q;               // the worker (non-external streams)
};

struct Rec {                                     // one record of an Event
  hipEvent_t e = nullptr;
  loop::Stream* q = nullptr;                     // worker that enqueues it (nullptr: enqueued inline)
  uint64_t mark = 0;
  ~Rec() {
    if (e) (void)hipEventDestroy(e);
  }
};

struct Event {
  int device = 0;
  std::mutex mu;
  std::shared_ptr<Rec> last;
  std::shared_ptr<Rec> get() {
    std::lock_guard<std::mutex> lk(mu);
    return last;
  }
};

}  // namespace hl

// the rank's engine (DpLeaderT / DpFollowerT `Local`)
class HipLoopLocal {
 public:
  explicit HipLoopLocal(HipExecBackend* be) : be_(be) {}
  ~HipLoopLocal();
  HipExecBackend* backend() const { return be_; }
  int device() const { return be_->device(); }
  int issue(int slot, int bucket, int n_real) { return be_->issue(slot, bucket, n_real); }
  int complete(int slot, const float** out, kdl_device_times* t) { return be_->complete(slot, out, t); }
  uint8_t* staging(int slot) { return be_->staging(slot); }
  float* host_out_mut(int slot) { return be_->host_out_mut(slot); }
  void* dev_in(int slot, int bucket) const { return be_->dev_in(slot, bucket); }
  void* dev_out(int slot, int bucket) const { return be_->dev_out(slot, bucket); }
  int max_batch() const { return be_->max_batch(); }
  int nslots() const { return be_->nslots(); }
  size_t item_bytes() const { return be_->item_bytes(); }
  int out_cols() const { return be_->out_cols(); }
  // the recipe of `bucket` behind `ready` (its record must have been enqueued: waited for here,
  // bounded); *last = the engine's last-stage stream, wrapped as an external stream
  int launch(int slot, int bucket, hl::Event* ready, hl::Stream** last);

 private:
  HipExecBackend* be_;
  std::mutex mu_;
  std::map<hipStream_t, std::unique_ptr<hl::Stream>> ext_;
};

struct HipLoopPlatform {
  using Stream = hl::Stream*;
  using Event = hl::Event*;
  using Comm = loop::Comm;
  using Local = HipLoopLocal;

  static int select(Local& l) { return hipSetDevice(l.device()) == hipSuccess ? 0 : -1; }
  static Stream new_stream(Local& l);
  static void free_stream(Stream s);
  static int sync(Stream s);
  static Event new_event(Local& l);
  static void free_event(Event e) { delete e; }
  static int record(Event e, Stream s);
  static int wait_event(Stream s, Event e);
  static int query(Event e);
  static void* dev_alloc(Local& l, size_t n);
  static void dev_free(Local&, void* p) { (void)hipFree(p); }
  static void* host_alloc(size_t n);
  static void host_free(void* p) { (void)hipHostFree(p); }
  static int h2d(void* d, const void* s, size_t n, Stream st);
  static int d2h(void* d, const void* s, size_t n, Stream st);
  static int group_start();
  static int group_end();
  static int send(const void* b, size_t n, int peer, Comm& c, Stream s);
  static int recv(void* b, size_t n, int peer, Comm& c, Stream s);
  static int rank(const Comm& c) { return c.rank(); }
  static int size(const Comm& c) { return c.size(); }
  static void abort(Comm& c) { c.abort(); }
  static bool comm_error(const Comm& c) { return c.error(); }
};

using HipLoopDpLeader = DpLeaderT<HipLoopPlatform>;
using HipLoopDpFollower = DpFollowerT<HipLoopPlatform>;

}  // namespace kdl
