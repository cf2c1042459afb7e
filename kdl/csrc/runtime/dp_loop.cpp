#include "dp_loop.h"

#include <chrono>
#include <cstring>
#include <random>
#include <stdexcept>

namespace kdl {
namespace loop {

// --------------------------------------------------------------------------------- Stream
Stream::Stream() { th_ = std::thread([this] { run(); }); }

Stream::~Stream() {
  cancel_ = true;                              // blocked operations give up
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

void Stream::push(std::function<int()> op) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(op));
    ++queued_;
  }
  cv_.notify_all();
}

uint64_t Stream::mark() {
  std::lock_guard<std::mutex> lk(mu_);
  return queued_;
}

void Stream::run() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
    if (q_.empty()) return;                    // stop_ and drained
    auto op = std::move(q_.front());
    q_.pop_front();
    const bool skip = error_ || cancel_.load();
    lk.unlock();
    const int r = skip ? -1 : op();
    lk.lock();
    if (r != 0) error_ = true;                 // sticky, like a HIP stream error
    ++done_;
    cv_.notify_all();
  }
}

int Stream::wait_reached(uint64_t n, const std::atomic<bool>* cancel) {
  std::unique_lock<std::mutex> lk(mu_);
  while (done_ < n && !error_) {
    if (cancel && cancel->load()) return -1;
    cv_.wait_for(lk, std::chrono::milliseconds(2));   // `cancel` belongs to another stream
  }
  return error_ ? -1 : 0;
}

int Stream::query(uint64_t n) {
  std::lock_guard<std::mutex> lk(mu_);
  return error_ ? -1 : done_ >= n ? 1 : 0;
}

int Stream::sync() { return wait_reached(mark(), nullptr); }

// ---------------------------------------------------------------------------------- Event
void Event::record(Stream* s) {
  const uint64_t m = s->mark();
  std::lock_guard<std::mutex> lk(mu_);
  s_ = s;
  mark_ = m;
}

std::pair<Stream*, uint64_t> Event::get() {
  std::lock_guard<std::mutex> lk(mu_);
  return {s_, mark_};
}

int Event::query() {
  const auto sm = get();
  return sm.first ? sm.first->query(sm.second) : 1;
}

// ---------------------------------------------------------------------------------- World
struct Post {
  const void* sbuf;
  void* rbuf;
  size_t bytes;
  int state;                                   // 0 pending, 1 delivered, -1 failed
  CopyFn copy;                                 // receiving post: the byte mover (nullptr: memcpy)
};

struct World {
  explicit World(int n) : size(n), dead(n, 0), aborted(n, 0) {}
  std::mutex mu;
  std::condition_variable cv;
  int size;
  std::map<std::pair<int, int>, std::deque<Post*>> sends, recvs;   // key (src, dst), FIFO per pair
  std::vector<char> dead, aborted;

  // pair posted sends with posted receives, per (src, dst) in order (caller holds mu)
  void match() {
    for (auto& kv : sends) {
      auto& sq = kv.second;
      auto it = recvs.find(kv.first);
      if (it == recvs.end() || dead[kv.first.first] || dead[kv.first.second]) continue;
      auto& rq = it->second;
      while (!sq.empty() && !rq.empty()) {
        Post* s = sq.front();
        Post* r = rq.front();
        sq.pop_front();
        rq.pop_front();
        if (s->bytes != r->bytes) {
          s->state = r->state = -1;            // RCCL would mis-deliver or hang: fail both ends
        } else if (s->bytes && r->copy) {
          s->state = r->state = r->copy(r->rbuf, s->sbuf, s->bytes) == 0 ? 1 : -1;
        } else {
          if (s->bytes) std::memcpy(r->rbuf, s->sbuf, s->bytes);
          s->state = r->state = 1;
        }
      }
    }
  }
};

namespace {
std::mutex g_reg_mu;
std::map<std::string, std::weak_ptr<World>> g_reg;
}  // namespace

std::string unique_id() {
  static std::atomic<uint64_t> n{0};
  std::random_device rd;
  return "loop-" + std::to_string(rd()) + "-" + std::to_string(n.fetch_add(1));
}

Comm::Comm(const std::string& id, int nranks, int rank) : rank_(rank), size_(nranks) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("LoopComm: bad rank");
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto& slot = g_reg[id];
  w_ = slot.lock();
  if (!w_) {
    w_ = std::make_shared<World>(nranks);
    slot = w_;
  }
  if (w_->size != nranks) throw std::invalid_argument("LoopComm: size differs from the other ranks'");
}

void Comm::kill() {
  {
    std::lock_guard<std::mutex> lk(w_->mu);
    w_->dead[rank_] = 1;
  }
  w_->cv.notify_all();
}

void Comm::abort() {
  {
    std::lock_guard<std::mutex> lk(w_->mu);
    w_->aborted[rank_] = 1;
  }
  w_->cv.notify_all();
}

bool Comm::error() const {
  std::lock_guard<std::mutex> lk(w_->mu);
  return w_->aborted[rank_] != 0;
}

// --------------------------------------------------------------------------------- Device
Device::Device(int rank, int nslots, size_t item_bytes, int max_batch, int out_cols, std::vector<int> buckets,
               int version, int64_t latency_us)
    : rank_(rank), nslots_(nslots), max_batch_(max_batch), out_cols_(out_cols), version_(version),
      item_bytes_(item_bytes), buckets_(std::move(buckets)), latency_us_(latency_us),
      staging_(nslots, std::vector<uint8_t>(item_bytes * max_batch)),
      din_(nslots, std::vector<uint8_t>(item_bytes * max_batch)),
      out_(nslots, std::vector<float>(size_t(out_cols) * max_batch)),
      dout_(nslots, std::vector<float>(size_t(out_cols) * max_batch)), ev_h2d_(nslots), ev_done_(nslots) {
  if (nslots < 1 || max_batch < 1 || out_cols < 1 || item_bytes < 4) throw std::invalid_argument("LoopDevice: geometry");
  for (int b : buckets_)
    if (b < 1 || b > max_batch) throw std::invalid_argument("LoopDevice: bucket > max_batch");
  api_.ctx = this;
  api_.nslots = nslots;
  api_.out_cols = out_cols;
  api_.staging = [](void* c, int s) { return static_cast<Device*>(c)->staging(s); };
  api_.issue = [](void* c, int s, int b, int n) { return static_cast<Device*>(c)->issue(s, b, n); };
  api_.complete = [](void* c, int s, const float** o, kdl_device_times* t) {
    return static_cast<Device*>(c)->complete(s, o, t);
  };
}

Device::~Device() {
  (void)compute_.sync();
  (void)copy_.sync();
}

bool Device::has_bucket(int b) const {
  for (int x : buckets_)
    if (x == b) return true;
  return false;
}

void* Device::dev_in(int slot, int bucket) {
  return slot >= 0 && slot < nslots_ && has_bucket(bucket) ? din_[slot].data() : nullptr;
}

void* Device::dev_out(int slot, int bucket) {
  return slot >= 0 && slot < nslots_ && has_bucket(bucket) ? dout_[slot].data() : nullptr;
}

int Device::launch(int slot, int bucket, Event* ready, Stream** last) {
  if (!dev_in(slot, bucket)) return -1;
  if (LoopPlatform::wait_event(&compute_, ready) != 0) return -1;
  compute_.push([this, slot, bucket] {
    if (latency_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(latency_us_));
    for (int i = 0; i < bucket; ++i) {
      uint32_t id;
      std::memcpy(&id, din_[slot].data() + size_t(i) * item_bytes_, 4);
      for (int k = 0; k < out_cols_; ++k) dout_[slot][size_t(i) * out_cols_ + k] = logit(id, k, version_);
    }
    forwards_.fetch_add(1);
    return 0;
  });
  *last = &compute_;
  return 0;
}

int Device::issue(int slot, int bucket, int n_real) {
  (void)n_real;
  if (fail_issues_.load() > 0 && fail_issues_.fetch_sub(1) > 0) return -1;
  if (!dev_in(slot, bucket)) return -1;
  if (LoopPlatform::h2d(din_[slot].data(), staging_[slot].data(), item_bytes_ * bucket, &copy_) != 0) return -1;
  ev_h2d_[slot].record(&copy_);
  Stream* last = nullptr;
  if (launch(slot, bucket, &ev_h2d_[slot], &last) != 0) return -1;
  if (LoopPlatform::d2h(out_[slot].data(), dout_[slot].data(), sizeof(float) * out_cols_ * bucket, last) != 0) return -1;
  ev_done_[slot].record(last);
  return 0;
}

int Device::complete(int slot, const float** out, kdl_device_times* t) {
  if (slot < 0 || slot >= nslots_) return -1;
  if (dp_poll<LoopPlatform>(&ev_done_[slot], 60.0, [] { return false; }) != 0) return -1;
  *out = out_[slot].data();
  if (t) {
    t->h2d_ms = 0.f;
    t->forward_ms = latency_us_ * 1e-3f;
    t->d2h_ms = 0.f;
  }
  return 0;
}

}  // namespace loop

// ------------------------------------------------------------------------------- platform
namespace loop {
int rendezvous(const std::vector<Op>& ops, const std::atomic<bool>& cancel, CopyFn copy) {
  World* w = ops[0].comm->world();
  const int me = ops[0].comm->rank();
  std::vector<Post> posts(ops.size());
  std::unique_lock<std::mutex> lk(w->mu);
  if (w->aborted[me]) return -1;
  for (size_t i = 0; i < ops.size(); ++i) {
    const Op& o = ops[i];
    if (o.peer < 0 || o.peer >= w->size || o.peer == me) return -1;
    posts[i] = Post{o.sbuf, o.rbuf, o.bytes, 0, copy};
    if (o.send)
      w->sends[{me, o.peer}].push_back(&posts[i]);
    else
      w->recvs[{o.peer, me}].push_back(&posts[i]);
  }
  w->match();
  w->cv.notify_all();
  int rc = 0;
  for (;;) {
    bool pending = false, failed = false;
    for (const auto& p : posts) {
      pending |= p.state == 0;
      failed |= p.state < 0;
    }
    if (failed) rc = -1;
    if (!pending) break;
    if (failed || w->aborted[me] || cancel.load()) {
      rc = -1;
      break;
    }
    w->cv.wait_for(lk, std::chrono::milliseconds(2));
  }
  // withdraw whatever is still queued (it points into this frame)
  for (size_t i = 0; i < ops.size(); ++i) {
    if (posts[i].state != 0) continue;
    auto& q = ops[i].send ? w->sends[{me, ops[i].peer}] : w->recvs[{ops[i].peer, me}];
    for (auto it = q.begin(); it != q.end(); ++it)
      if (*it == &posts[i]) {
        q.erase(it);
        break;
      }
  }
  return rc;
}
}  // namespace loop

namespace {
struct LoopOp {
  loop::Op op;
  loop::Stream* stream;
};
struct LoopGroup {
  int depth = 0;
  std::vector<LoopOp> ops;
};
thread_local LoopGroup tl_group;

int submit(std::vector<LoopOp> ops) {
  if (ops.empty()) return 0;
  std::vector<loop::Op> v;
  for (const auto& o : ops) {
    if (o.op.comm != ops[0].op.comm || o.stream != ops[0].stream) return -1;   // one communicator and stream per group
    v.push_back(o.op);
  }
  loop::Stream* st = ops[0].stream;
  // one stream operation: post every op of the group, then wait (rendezvous) until each was
  // matched, this rank aborted, or its stream was cancelled
  st->push([v, st] { return loop::rendezvous(v, st->cancelled(), nullptr); });
  return 0;
}

int add_op(const LoopOp& o) {
  if (tl_group.depth > 0) {
    tl_group.ops.push_back(o);
    return 0;
  }
  return submit({o});
}
}  // namespace

int LoopPlatform::wait_event(Stream s, Event e) {
  const auto sm = e->get();
  if (!sm.first) return 0;
  loop::Stream* es = sm.first;
  const uint64_t m = sm.second;
  s->push([es, m, s] { return es->wait_reached(m, &s->cancelled()); });
  return 0;
}

int LoopPlatform::h2d(void* d, const void* src, size_t n, Stream st) {
  st->push([d, src, n] {
    if (n) std::memcpy(d, src, n);
    return 0;
  });
  return 0;
}

int LoopPlatform::group_start() {
  ++tl_group.depth;
  return 0;
}

int LoopPlatform::group_end() {
  if (tl_group.depth <= 0) return -1;
  if (--tl_group.depth > 0) return 0;
  std::vector<LoopOp> ops;
  ops.swap(tl_group.ops);
  return submit(std::move(ops));
}

int LoopPlatform::send(const void* b, size_t n, int peer, Comm& c, Stream s) {
  return add_op({{true, b, nullptr, n, peer, &c}, s});
}

int LoopPlatform::recv(void* b, size_t n, int peer, Comm& c, Stream s) {
  return add_op({{false, nullptr, b, n, peer, &c}, s});
}

template class DpLeaderT<LoopPlatform>;
template class DpFollowerT<LoopPlatform>;

}  // namespace kdl
