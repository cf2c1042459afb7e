#include "dp_hiploop.h"

#include <chrono>
#include <functional>
#include <thread>
#include <vector>

namespace kdl {

namespace {

int ok(hipError_t e) { return e == hipSuccess ? 0 : -1; }

// an operation of stream s, in post order: inline on an external (engine) stream, else queued
// to the stream's worker
int run_on(hl::Stream* s, std::function<int()> op) {
  if (s->external) return op();
  s->q->push(std::move(op));
  return 0;
}

// device-to-device byte mover of a matched pair (runs on the worker thread that completed the
// match): its own non-blocking stream, so the copy never waits on, or is waited for by, any
// engine stream (a legacy-default-stream hipMemcpy could: the engines' work waits on records
// that this very worker enqueues)
int hip_copy(void* dst, const void* src, size_t n) {
  struct CopyStream {
    hipStream_t s = nullptr;
    ~CopyStream() {
      if (s) (void)hipStreamDestroy(s);
    }
  };
  thread_local CopyStream cs;
  if (!cs.s && hipStreamCreateWithFlags(&cs.s, hipStreamNonBlocking) != hipSuccess) return -1;
  if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, cs.s) != hipSuccess) return -1;
  return ok(hipStreamSynchronize(cs.s));
}

// a record's enqueue by its worker, waited for on the host with a deadline (never forever: a
// worker blocked in a rendezvous with a dead peer must not hang the caller)
int wait_enqueued(const hl::Rec& r, double timeout_s) {
  if (!r.q) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    const int q = r.q->query(r.mark);
    if (q != 0) return q > 0 ? 0 : -1;
    if (i > 1000) std::this_thread::sleep_for(std::chrono::microseconds(50));
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return -1;
  }
}

struct HlOp {
  loop::Op op;
  hl::Stream* stream;
};
struct HlGroup {
  int depth = 0;
  std::vector<HlOp> ops;
};
thread_local HlGroup tl_group;

int submit(std::vector<HlOp> ops) {
  if (ops.empty()) return 0;
  hl::Stream* s = ops[0].stream;
  if (s->external) return -1;                    // transport ops run on the platform's own streams
  std::vector<loop::Op> v;
  for (const auto& o : ops) {
    if (o.op.comm != ops[0].op.comm || o.stream != s) return -1;   // one communicator and stream per group
    v.push_back(o.op);
  }
  hipStream_t hs = s->hs;
  loop::Stream* q = s->q.get();
  // the stream's earlier HIP work first (the data to send is written / the receive buffer is
  // free), then the rendezvous; every later operation of the stream runs after the copy
  q->push([v, hs, q] {
    if (hipStreamSynchronize(hs) != hipSuccess) return -1;
    return loop::rendezvous(v, q->cancelled(), &hip_copy);
  });
  return 0;
}

int add_op(const HlOp& o) {
  if (tl_group.depth > 0) {
    tl_group.ops.push_back(o);
    return 0;
  }
  return submit({o});
}

}  // namespace

// --------------------------------------------------------------------------------- Local
HipLoopLocal::~HipLoopLocal() = default;

int HipLoopLocal::launch(int slot, int bucket, hl::Event* ready, hl::Stream** last) {
  const std::shared_ptr<hl::Rec> r = ready ? ready->get() : nullptr;
  if (!r || wait_enqueued(*r, 120.0) != 0) return -1;
  hipStream_t ls = nullptr;
  if (be_->launch(slot, bucket, r->e, &ls) != 0) return -1;
  std::lock_guard<std::mutex> lk(mu_);
  auto& w = ext_[ls];
  if (!w) {
    w = std::make_unique<hl::Stream>();
    w->device = be_->device();
    w->hs = ls;
    w->external = true;
  }
  *last = w.get();
  return 0;
}

// ------------------------------------------------------------------------------ platform
hl::Stream* HipLoopPlatform::new_stream(Local& l) {
  auto s = std::make_unique<hl::Stream>();
  s->device = l.device();
  check_hip(hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking), "hipStreamCreate");
  s->q = std::make_unique<loop::Stream>();
  const int dev = s->device;
  s->q->push([dev] { return ok(hipSetDevice(dev)); });   // the worker's HIP calls target the rank's device
  return s.release();
}

void HipLoopPlatform::free_stream(Stream s) {
  if (!s) return;
  if (!s->external) {
    (void)s->q->sync();
    s->q.reset();                                // cancels anything blocked, joins the worker
    (void)hipStreamSynchronize(s->hs);
    (void)hipStreamDestroy(s->hs);
  }
  delete s;
}

int HipLoopPlatform::sync(Stream s) {
  if (!s->external && s->q->sync() != 0) return -1;
  return ok(hipStreamSynchronize(s->hs));
}

hl::Event* HipLoopPlatform::new_event(Local& l) {
  auto* e = new hl::Event();
  e->device = l.device();
  return e;
}

int HipLoopPlatform::record(Event e, Stream s) {
  auto r = std::make_shared<hl::Rec>();
  if (hipEventCreateWithFlags(&r->e, hipEventDisableTiming) != hipSuccess) {
    r->e = nullptr;
    return -1;
  }
  if (s->external) {
    if (hipEventRecord(r->e, s->hs) != hipSuccess) return -1;
  } else {
    hipStream_t hs = s->hs;
    s->q->push([r, hs] { return ok(hipEventRecord(r->e, hs)); });
    r->q = s->q.get();
    r->mark = s->q->mark();
  }
  std::lock_guard<std::mutex> lk(e->mu);
  e->last = std::move(r);
  return 0;
}

int HipLoopPlatform::wait_event(Stream s, Event e) {
  const std::shared_ptr<hl::Rec> r = e->get();  // the record current at post time
  if (!r) return 0;
  if (s->external) {
    if (wait_enqueued(*r, 120.0) != 0) return -1;
    return ok(hipStreamWaitEvent(s->hs, r->e, 0));
  }
  hipStream_t hs = s->hs;
  loop::Stream* q = s->q.get();
  q->push([r, hs, q] {
    if (r->q && r->q != q && r->q->wait_reached(r->mark, &q->cancelled()) != 0) return -1;
    return ok(hipStreamWaitEvent(hs, r->e, 0));
  });
  return 0;
}

int HipLoopPlatform::query(Event e) {
  const std::shared_ptr<hl::Rec> r = e->get();
  if (!r) return 1;
  if (r->q) {
    const int q = r->q->query(r->mark);
    if (q <= 0) return q;
  }
  const hipError_t st = hipEventQuery(r->e);
  return st == hipSuccess ? 1 : st == hipErrorNotReady ? 0 : -1;
}

void* HipLoopPlatform::dev_alloc(Local& l, size_t n) {
  (void)l;
  void* p = nullptr;
  check_hip(hipMalloc(&p, n), "hipMalloc");
  return p;
}

void* HipLoopPlatform::host_alloc(size_t n) {
  void* p = nullptr;
  check_hip(hipHostMalloc(&p, n, hipHostMallocDefault), "hipHostMalloc");
  return p;
}

int HipLoopPlatform::h2d(void* d, const void* src, size_t n, Stream st) {
  hipStream_t hs = st->hs;
  return run_on(st, [d, src, n, hs] { return ok(hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, hs)); });
}

int HipLoopPlatform::d2h(void* d, const void* src, size_t n, Stream st) {
  hipStream_t hs = st->hs;
  return run_on(st, [d, src, n, hs] { return ok(hipMemcpyAsync(d, src, n, hipMemcpyDeviceToHost, hs)); });
}

int HipLoopPlatform::group_start() {
  ++tl_group.depth;
  return 0;
}

int HipLoopPlatform::group_end() {
  if (tl_group.depth <= 0) return -1;
  if (--tl_group.depth > 0) return 0;
  std::vector<HlOp> ops;
  ops.swap(tl_group.ops);
  return submit(std::move(ops));
}

int HipLoopPlatform::send(const void* b, size_t n, int peer, Comm& c, Stream s) {
  return add_op({{true, b, nullptr, n, peer, &c}, s});
}

int HipLoopPlatform::recv(void* b, size_t n, int peer, Comm& c, Stream s) {
  return add_op({{false, nullptr, b, n, peer, &c}, s});
}

template class DpLeaderT<HipLoopPlatform>;
template class DpFollowerT<HipLoopPlatform>;

}  // namespace kdl
