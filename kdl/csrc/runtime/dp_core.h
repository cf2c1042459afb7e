// Data-parallel serving state machine, written ONCE against a platform
// policy P so the same leader / follower code runs over
//   * RCCL + HIP   (comm.h: HipRcclPlatform; the real one-process-per-GPU topology), and
//   * a loopback   (dp_loop.h: LoopPlatform; threads as "streams", host memory as "device"
//                   memory, ordered per-(channel, peer) rendezvous queues as the transport),
// which is how CPU tests and ThreadSanitizer drive world 2/4/8 without a GPU (SURVEY.md §4.2:
// "the C++ comm layer has a backend interface with a loopback/fake implementation").
//
// The reference scales by Deployment replicas behind a ClusterIP Service
// (/root/reference/tf-serving-clothing-model-deployment.yaml:8,
//  /root/reference/tf-serving-clothing-model-service.yaml:8-14); here one front-end feeds every
// GPU of the node as one collective step per batch (message lists: dp_schedule.h).
//
// Policy P (all static; every int-returning call: 0 = ok, non-zero = failed):
//   types   Stream, Event (copyable handles), Comm, Local (the rank's device backend)
//   select(Local&)                              make the rank's device current (this thread)
//   new_stream(Local&) / free_stream(Stream) / sync(Stream)
//   new_event(Local&) / free_event(Event) / record(Event, Stream) / wait_event(Stream, Event)
//   query(Event) -> 1 done, 0 pending, < 0 error
//   dev_alloc(Local&, n) / dev_free(Local&, p) / host_alloc(n) / host_free(p)
//   h2d(dst, src, n, Stream) / d2h(dst, src, n, Stream)
//   group_start() / group_end() / send(buf, n, peer, Comm&, Stream) / recv(buf, n, peer, Comm&, Stream)
//   rank(Comm&) / size(Comm&) / abort(Comm&) (unblocks every pending op of this rank) /
//   comm_error(Comm&) (asynchronous error reported by the transport)
// Local (leader): issue / complete / staging / host_out_mut / dev_in / max_batch / nslots /
//   item_bytes / out_cols; (follower): dev_in / dev_out / launch(slot, bucket, Event, Stream*).
//
// Liveness (every wait is bounded):
//   leader    each step's scatter / gather completion is polled for at most timeout_s; on
//             expiry (a follower died or hung) or a communicator error the leader aborts both
//             communicators (under its mutex: no other thread is inside a post) and fails every
//             later batch -> the executor marks itself unhealthy (executor.cpp). While idle it
//             sends a DP_PING every ping_s.
//   follower  waits at most liveness_s for the next control word (a ping, a batch or a command);
//             silence or a communicator error -> it aborts its communicators and throws, so the
//             rank's process exits non-zero and is restarted (serving/dp.py).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "dp_schedule.h"
#include "exec_backend.h"

namespace kdl {

// Posts `msgs` (all on one communicator) as sends / receives, one transport group per
// DpMsg::group value, in order. buf(msg) -> device pointer of that message.
template <class P, class F>
int dp_post(const std::vector<DpMsg>& msgs, typename P::Comm& c, typename P::Stream s, F buf) {
  size_t i = 0;
  while (i < msgs.size()) {
    const int g = msgs[i].group;
    if (P::group_start() != 0) return -1;
    int r = 0;
    for (; i < msgs.size() && msgs[i].group == g; ++i) {
      const DpMsg& m = msgs[i];
      if (r == 0) r = m.send ? P::send(buf(m), m.bytes, m.peer, c, s) : P::recv(buf(m), m.bytes, m.peer, c, s);
    }
    if (P::group_end() != 0 || r != 0) return -1;
  }
  return 0;
}

// Poll an event: spin briefly (a step's control word usually lands within microseconds of the
// previous one), then sleep between queries so an idle rank does not burn a core. Every ~64
// queries: the deadline and bad() (e.g. a communicator error). 0 = done, -1 = error / timeout / bad.
template <class P, class Bad>
int dp_poll(typename P::Event e, double timeout_s, Bad bad) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int i = 0;; ++i) {
    const int q = P::query(e);
    if (q > 0) return 0;
    if (q < 0) return -1;
    if (i > 2000) usleep(50);
    if (i % 64 == 63) {
      if (bad()) return -1;
      if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) return -1;
    }
  }
}

inline void dp_check(int r, const char* what) {
  if (r != 0) throw std::runtime_error(std::string("dp: ") + what + " failed");
}

// ------------------------------------------------------------------------------------ leader
// Rank 0. Wraps rank 0's own device backend as a kdl_exec_backend (executor.cpp drives it): per
// batch of world x shard images it H2Ds its own shard straight into its engine's input slot (the
// local forward starts at once) and the other shards into a send buffer, then posts the step of
// dp_schedule.h on the two communicators and D2Hs the followers' logits behind its own.
template <class P>
class DpLeaderT {
 public:
  using Local = typename P::Local;
  using Comm = typename P::Comm;
  using Stream = typename P::Stream;
  using Event = typename P::Event;

  // local: rank 0's backend, built with max_batch >= world x the largest rank bucket and one
  // recipe per rank bucket. ping_s <= 0: no heartbeat.
  DpLeaderT(Local* local, Comm* scatter, Comm* gather, std::vector<int> rank_buckets, double timeout_s,
            double ping_s = 0)
      : L_(local), S_(scatter), G_(gather), world_(P::size(*scatter)), buckets_(std::move(rank_buckets)),
        timeout_s_(timeout_s > 0 ? timeout_s : 120.0), ping_s_(ping_s) {
    if (P::size(*G_) != world_ || P::rank(*S_) != 0 || P::rank(*G_) != 0 || buckets_.empty())
      throw std::invalid_argument("DpLeader: rank 0 of two equal-size communicators, >= 1 bucket");
    max_shard_ = *std::max_element(buckets_.begin(), buckets_.end());
    for (int b : buckets_)
      if (!L_->dev_in(0, b)) throw std::invalid_argument("DpLeader: no local recipe for a rank bucket");
    if (L_->max_batch() < world_ * max_shard_) throw std::invalid_argument("DpLeader: local staging < world x bucket");
    dp_check(P::select(*L_), "select device");
    cs_ = P::new_stream(*L_);
    ss_ = P::new_stream(*L_);
    gs_ = P::new_stream(*L_);
    const int ns = L_->nslots();
    for (int s = 0; s < ns + 2; ++s) {           // slot ns: STOP / RELOAD, ns + 1: pings
      d_ctrl_.push_back(static_cast<DpCtrl*>(P::dev_alloc(*L_, sizeof(DpCtrl))));
      h_ctrl_.push_back(static_cast<DpCtrl*>(P::host_alloc(sizeof(DpCtrl))));
    }
    for (int s = 0; s < ns; ++s) {
      d_send_.push_back(world_ > 1 ? static_cast<uint8_t*>(P::dev_alloc(*L_, L_->item_bytes() * (world_ - 1) * max_shard_))
                                   : nullptr);
      d_gather_.push_back(static_cast<float*>(P::dev_alloc(*L_, sizeof(float) * L_->out_cols() * world_ * max_shard_)));
      ev_in_.push_back(P::new_event(*L_));
      ev_sent_.push_back(P::new_event(*L_));
      ev_gdone_.push_back(P::new_event(*L_));
    }
    ev_ping_ = P::new_event(*L_);
    ev_ctl_ = P::new_event(*L_);
    last_ctrl_ = now();
    api_.ctx = this;
    api_.nslots = ns;
    api_.out_cols = L_->out_cols();
    api_.staging = [](void* ctx, int slot) { return static_cast<DpLeaderT*>(ctx)->L_->staging(slot); };
    api_.issue = [](void* ctx, int slot, int bucket, int n) { return static_cast<DpLeaderT*>(ctx)->issue(slot, bucket, n); };
    api_.complete = [](void* ctx, int slot, const float** out, kdl_device_times* t) {
      return static_cast<DpLeaderT*>(ctx)->complete(slot, out, t);
    };
    if (world_ > 1 && ping_s_ > 0) hb_ = std::thread([this] { heartbeat(); });
  }

  ~DpLeaderT() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      hb_stop_ = true;
    }
    hb_cv_.notify_all();
    if (hb_.joinable()) hb_.join();
    (void)P::select(*L_);
    // drain what is queued; a peer that never answers is cut loose by aborting the communicators
    for (Stream s : {cs_, ss_, gs_}) {
      if (P::record(ev_ctl_, s) != 0 || wait(ev_ctl_) != 0) break;
    }
    for (Stream s : {cs_, ss_, gs_}) (void)P::sync(s);
    for (auto* v : {&ev_in_, &ev_sent_, &ev_gdone_})
      for (auto e : *v) P::free_event(e);
    P::free_event(ev_ping_);
    P::free_event(ev_ctl_);
    for (auto p : d_send_)
      if (p) P::dev_free(*L_, p);
    for (auto p : d_gather_) P::dev_free(*L_, p);
    for (auto p : d_ctrl_) P::dev_free(*L_, p);
    for (auto p : h_ctrl_) P::host_free(p);
    for (Stream s : {cs_, ss_, gs_}) P::free_stream(s);
  }
  DpLeaderT(const DpLeaderT&) = delete;
  DpLeaderT& operator=(const DpLeaderT&) = delete;

  const kdl_exec_backend* api() const { return &api_; }
  int world() const { return world_; }
  long steps() const { return steps_.load(); }
  bool broken() const {
    std::lock_guard<std::mutex> lk(mu_);
    return broken_;
  }

  // bucket = world x a rank bucket. Asynchronous; 0 = queued.
  int issue(int slot, int bucket, int n_real) {
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_ || closed_ || slot < 0 || slot >= L_->nslots() || bucket % world_ != 0) return -1;
    const int shard = bucket / world_;
    if (std::find(buckets_.begin(), buckets_.end(), shard) == buckets_.end()) return -1;
    if (P::select(*L_) != 0) return -1;
    const DpGeometry g{world_, L_->item_bytes(), L_->out_cols()};
    const size_t ib = L_->item_bytes();
    // rank 0's own shard first: rows [0, shard) of the staging, straight into its engine's input
    // slot. A local failure here fails this batch only: no control word has used a sequence
    // number yet, so the followers' next word is still in sequence (advisor r5)
    if (L_->issue(slot, shard, std::min(n_real, shard)) != 0) return -1;
    // from here on every failure breaks the group (a word may be half-posted)
    *h_ctrl_[slot] = DpCtrl{DP_BATCH, shard, n_real, seq_++, 0, {0, 0, 0}};
    last_ctrl_ = now();
    if (world_ > 1) {
      if (P::h2d(d_ctrl_[slot], h_ctrl_[slot], sizeof(DpCtrl), cs_) != 0 ||
          P::h2d(d_send_[slot], L_->staging(slot) + ib * shard, ib * shard * (world_ - 1), cs_) != 0 ||
          P::record(ev_in_[slot], cs_) != 0)
        return fail_locked();
    }
    if (world_ > 1) {
      const auto msgs = dp_leader_step(g, DP_BATCH, shard);
      std::vector<DpMsg> sc, ga;
      for (const auto& m : msgs) (m.channel == DP_SCATTER ? sc : ga).push_back(m);
      if (P::wait_event(ss_, ev_in_[slot]) != 0) return fail_locked();
      if (dp_post<P>(sc, *S_, ss_, [&](const DpMsg& m) -> void* {
            return m.what == 0 ? static_cast<void*>(d_ctrl_[slot])
                               : static_cast<void*>(d_send_[slot] + ib * shard * (m.peer - 1));
          }) != 0)
        return fail_locked();
      if (P::record(ev_sent_[slot], ss_) != 0) return fail_locked();
      if (dp_post<P>(ga, *G_, gs_, [&](const DpMsg& m) -> void* {
            return static_cast<void*>(d_gather_[slot] + (size_t)g.out_cols * shard * m.peer);
          }) != 0)
        return fail_locked();
      if (P::d2h(L_->host_out_mut(slot) + (size_t)g.out_cols * shard, d_gather_[slot] + (size_t)g.out_cols * shard,
                 sizeof(float) * g.out_cols * shard * (world_ - 1), gs_) != 0 ||
          P::record(ev_gdone_[slot], gs_) != 0)
        return fail_locked();
    }
    steps_.fetch_add(1);
    return 0;
  }

  // blocks (bounded) until `slot`'s global logits are on the host
  int complete(int slot, const float** out, kdl_device_times* t) {
    if (slot < 0 || slot >= L_->nslots()) return -1;
    if (L_->complete(slot, out, t) != 0) return -1;
    if (world_ > 1) {
      if (P::select(*L_) != 0 || wait(ev_gdone_[slot]) != 0 || wait(ev_sent_[slot]) != 0) return -1;
    }
    return 0;
  }

  // DP_STOP / DP_RELOAD to every follower; synchronous (bounded). No batch after it.
  int send_ctrl(int cmd, int version) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (broken_ || closed_ || cmd == DP_BATCH || cmd == DP_PING) return -1;
      closed_ = true;
      if (world_ == 1) return 0;
      if (post_ctrl_locked(L_->nslots(), cmd, version, ev_ctl_) != 0) return fail_locked();
    }
    return wait(ev_ctl_);
  }

  // one DP_PING now, synchronous (bounded); the heartbeat thread calls it while idle
  int ping() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (broken_ || closed_) return -1;
      if (world_ == 1) return 0;
      if (post_ctrl_locked(L_->nslots() + 1, DP_PING, 0, ev_ping_) != 0) return fail_locked();
    }
    return wait(ev_ping_);
  }

 private:
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  // control word `cmd` (no batch) from buffer x on the scatter channel; `done` marks it sent
  int post_ctrl_locked(int x, int cmd, int version, Event done) {
    if (P::select(*L_) != 0) return -1;
    *h_ctrl_[x] = DpCtrl{cmd, 0, 0, seq_++, version, {0, 0, 0}};
    last_ctrl_ = now();
    if (P::h2d(d_ctrl_[x], h_ctrl_[x], sizeof(DpCtrl), ss_) != 0) return -1;
    const DpGeometry g{world_, L_->item_bytes(), L_->out_cols()};
    if (dp_post<P>(dp_leader_step(g, cmd, 0), *S_, ss_, [&](const DpMsg&) -> void* { return d_ctrl_[x]; }) != 0)
      return -1;
    return P::record(done, ss_);
  }

  // a follower died or stalled, or the transport failed: unblock the communicators so no later
  // step hangs on them, and fail every later batch. Caller holds mu_ (no other thread is
  // inside a post, so the abort cannot free a communicator under it).
  int fail_locked() {
    if (!broken_) {
      broken_ = true;
      P::abort(*S_);
      P::abort(*G_);
    }
    return -1;
  }

  // bounded wait (timeout_s_) for a step's transfers; called without mu_
  int wait(Event e) {
    const int r = dp_poll<P>(e, timeout_s_, [&] {
      std::lock_guard<std::mutex> lk(mu_);
      return broken_ || P::comm_error(*S_) || P::comm_error(*G_);
    });
    if (r == 0) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    return fail_locked();
  }

  void heartbeat() {
    std::unique_lock<std::mutex> lk(mu_);
    const auto period = std::chrono::duration<double>(std::max(ping_s_ / 4, 1e-3));
    while (!hb_stop_) {
      hb_cv_.wait_for(lk, period);
      if (hb_stop_ || broken_ || closed_ || now() - last_ctrl_ < ping_s_) continue;
      lk.unlock();
      (void)ping();              // a failure marks the leader broken (the executor then fails its batches)
      lk.lock();
    }
  }

  Local* L_;
  Comm *S_, *G_;
  int world_;
  std::vector<int> buckets_;
  int max_shard_ = 0;
  double timeout_s_, ping_s_;
  Stream cs_{}, ss_{}, gs_{};                    // follower-shard H2D, scatter, gather
  std::vector<uint8_t*> d_send_;
  std::vector<float*> d_gather_;
  std::vector<DpCtrl*> d_ctrl_, h_ctrl_;
  std::vector<Event> ev_in_, ev_sent_, ev_gdone_;
  Event ev_ping_{}, ev_ctl_{};
  int seq_ = 0;
  std::atomic<long> steps_{0};
  double last_ctrl_ = 0;
  bool broken_ = false;
  bool closed_ = false;                          // a DP_STOP / DP_RELOAD went out: no more batches
  bool hb_stop_ = false;
  mutable std::mutex mu_;                        // every communicator use and the abort
  std::condition_variable hb_cv_;
  std::thread hb_;
  kdl_exec_backend api_{};
};

// ---------------------------------------------------------------------------------- follower
// Ranks >= 1: a C++ loop (the GIL released by the binding): receive the control word (it carries
// the per-rank bucket, so the follower picks the captured graph) and the shard into the
// engine's input slot, launch the forward, send the logits, and already post the next step's
// control receive. Steps stay in flight on `nslots` slots, as on the leader.
template <class P>
class DpFollowerT {
 public:
  using Local = typename P::Local;
  using Comm = typename P::Comm;
  using Stream = typename P::Stream;
  using Event = typename P::Event;

  DpFollowerT(Local* local, Comm* scatter, Comm* gather) : L_(local), S_(scatter), G_(gather), nslots_(local->nslots()) {
    if (P::rank(*S_) == 0 || P::rank(*G_) != P::rank(*S_) || P::size(*G_) != P::size(*S_))
      throw std::invalid_argument("DpFollower: a rank >= 1 of two matching communicators");
    dp_check(P::select(*L_), "select device");
    ss_ = P::new_stream(*L_);
    gs_ = P::new_stream(*L_);
    for (int s = 0; s < nslots_; ++s) {
      d_ctrl_.push_back(static_cast<DpCtrl*>(P::dev_alloc(*L_, sizeof(DpCtrl))));
      h_ctrl_.push_back(static_cast<DpCtrl*>(P::host_alloc(sizeof(DpCtrl))));
      for (auto* v : {&ev_ctrl_, &ev_in_, &ev_fw_, &ev_free_}) v->push_back(P::new_event(*L_));
      dp_check(P::record(ev_free_.back(), gs_), "record");
    }
  }

  ~DpFollowerT() {
    (void)P::select(*L_);
    for (Stream s : {ss_, gs_}) (void)P::sync(s);
    for (auto* v : {&ev_ctrl_, &ev_in_, &ev_fw_, &ev_free_})
      for (auto e : *v) P::free_event(e);
    for (auto p : d_ctrl_) P::dev_free(*L_, p);
    for (auto p : h_ctrl_) P::host_free(p);
    for (Stream s : {ss_, gs_}) P::free_stream(s);
  }
  DpFollowerT(const DpFollowerT&) = delete;
  DpFollowerT& operator=(const DpFollowerT&) = delete;

  // Serve rank 0's steps until a DP_STOP / DP_RELOAD control word arrives; returns it. Throws
  // (after aborting both communicators) when no control word arrives within liveness_s or a
  // communicator reports an error.
  DpCtrl run(double liveness_s) {
    try {
      return loop(liveness_s > 0 ? liveness_s : 30.0);
    } catch (...) {
      P::abort(*S_);               // pending receives must not outlive this rank's loop
      P::abort(*G_);
      throw;
    }
  }
  long steps() const { return steps_.load(); }

 private:
  void post_ctrl_recv(int slot) {
    dp_check(P::recv(d_ctrl_[slot], sizeof(DpCtrl), 0, *S_, ss_), "recv(ctrl)");
    dp_check(P::d2h(h_ctrl_[slot], d_ctrl_[slot], sizeof(DpCtrl), ss_), "D2H ctrl");
    dp_check(P::record(ev_ctrl_[slot], ss_), "record");
  }

  DpCtrl loop(double liveness_s) {
    dp_check(P::select(*L_), "select device");
    const DpGeometry g{P::size(*S_), L_->item_bytes(), L_->out_cols()};
    (void)dp_follower_prologue();
    int slot = (int)(steps_.load() % nslots_);
    post_ctrl_recv(slot);
    for (;;) {
      if (dp_poll<P>(ev_ctrl_[slot], liveness_s, [&] { return P::comm_error(*S_) || P::comm_error(*G_); }) != 0)
        throw std::runtime_error("DpFollower: no control word from rank 0 within the liveness window "
                                 "(leader dead or hung) or a communicator error");
      const DpCtrl c = *h_ctrl_[slot];
      if (c.seq != seq_) throw std::runtime_error("DpFollower: control word out of sequence");
      ++seq_;
      if (c.cmd == DP_PING) {                    // heartbeat: same slot, next control word
        post_ctrl_recv(slot);
        continue;
      }
      if (c.cmd != DP_BATCH) {
        dp_check(P::sync(gs_), "drain gather");
        dp_check(P::sync(ss_), "drain scatter");
        return c;
      }
      const int shard = c.shard;
      void* din = L_->dev_in(slot, shard);
      void* dout = L_->dev_out(slot, shard);
      if (!din || !dout) throw std::runtime_error("DpFollower: no captured graph for the shard size");
      const int next = (slot + 1) % nslots_;
      // the shard lands in the engine's input slot once its previous batch has been sent back;
      // the compute waits for the shard only, never for the next control word
      const auto msgs = dp_follower_step(g, DP_BATCH, shard, true);
      dp_check(P::wait_event(ss_, ev_free_[slot]), "wait slot free");
      for (const auto& m : msgs) {
        if (m.channel == DP_SCATTER && m.what == 1) {
          dp_check(P::recv(din, m.bytes, 0, *S_, ss_), "recv(shard)");
          dp_check(P::record(ev_in_[slot], ss_), "record");
        } else if (m.channel == DP_SCATTER && m.what == 0) {
          post_ctrl_recv(next);
        }
      }
      Stream last{};
      if (L_->launch(slot, shard, ev_in_[slot], &last) != 0) throw std::runtime_error("DpFollower: launch failed");
      dp_check(P::record(ev_fw_[slot], last), "record");
      dp_check(P::wait_event(gs_, ev_fw_[slot]), "wait forward");
      for (const auto& m : msgs)
        if (m.channel == DP_GATHER) dp_check(P::send(dout, m.bytes, 0, *G_, gs_), "send(logits)");
      dp_check(P::record(ev_free_[slot], gs_), "record");
      steps_.fetch_add(1);
      slot = next;
    }
  }

  Local* L_;
  Comm *S_, *G_;
  int nslots_;
  Stream ss_{}, gs_{};
  std::vector<DpCtrl*> d_ctrl_, h_ctrl_;
  std::vector<Event> ev_ctrl_, ev_in_, ev_fw_, ev_free_;
  std::atomic<long> steps_{0};
  int seq_ = 0;
};

}  // namespace kdl
