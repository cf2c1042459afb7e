#include "executor.h"

#include <algorithm>
#include <cstring>

namespace kdl {

const double kBucketsMs[N_BUCKETS] = {0.05, 0.1, 0.25, 0.5, 1, 2, 4, 8, 16, 32, 64, 128, 512, 1e30};

static const char* kStageNames[N_STAGES] = {"queue_wait", "host_copy", "issue", "device_h2d",
                                            "device_forward", "device_d2h", "in_flight", "batch_latency"};

const char* exec_stage_name(int s) { return s >= 0 && s < N_STAGES ? kStageNames[s] : "?"; }

void StageHist::add(double ms) {
  if (!(ms >= 0)) return;          // unknown (-1) or NaN: not recorded
  ++count;
  sum_ms += ms;
  for (int i = 0; i < N_BUCKETS; ++i)
    if (ms <= kBucketsMs[i]) { ++buckets[i]; break; }
}

Executor::Executor(DynamicBatcher* batcher, const kdl_exec_backend* backend, ExecGroup* group, const ExecOptions& o)
    : batcher_(batcher), be_(*backend), group_(group), opt_(o), fail_left_(o.fail_batches) {
  if (be_.nslots < 1) be_.nslots = 1;
  if (group_) group_->join();
}

Executor::~Executor() { stop(); }

void Executor::start() {
  if (th_.joinable()) return;
  stop_ = false;
  running_ = true;
  th_ = std::thread([this] { loop(); });
}

void Executor::stop() {
  stop_ = true;
  if (th_.joinable()) th_.join();
  running_ = false;
}

ExecStats Executor::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  ExecStats s = st_;
  s.healthy = healthy_.load();
  return s;
}

std::vector<BatchTrace> Executor::recent(int n) const {
  std::lock_guard<std::mutex> lk(mu_);
  const int k = std::min<int>(n, int(ring_.size()));
  return std::vector<BatchTrace>(ring_.end() - k, ring_.end());
}

void Executor::record(const BatchTrace& tr, const Batch& b) {
  std::lock_guard<std::mutex> lk(mu_);
  if (tr.status == ST_OK) {
    ++st_.batches;
    st_.items += b.n_real;
    st_.padded_items += b.bucket - b.n_real;
    const double ms = 1e-3;
    st_.hist[STAGE_QUEUE_WAIT].add((tr.formed_us - tr.oldest_enqueue_us) * ms);
    st_.hist[STAGE_HOST_COPY].add((tr.copied_us - tr.formed_us) * ms);
    st_.hist[STAGE_ISSUE].add((tr.issued_us - tr.copied_us) * ms);
    st_.hist[STAGE_DEVICE_H2D].add(tr.h2d_ms);
    st_.hist[STAGE_DEVICE_FORWARD].add(tr.forward_ms);
    st_.hist[STAGE_DEVICE_D2H].add(tr.d2h_ms);
    st_.hist[STAGE_IN_FLIGHT].add((tr.completed_us - tr.issued_us) * ms);
    st_.hist[STAGE_BATCH_LATENCY].add((tr.finished_us - tr.oldest_enqueue_us) * ms);
  } else {
    ++st_.failed_batches;
  }
  ring_.push_back(tr);
  while (int(ring_.size()) > std::max(1, opt_.trace_ring)) ring_.pop_front();
}

bool Executor::fail(Batch& b, BatchTrace& tr) {
  batcher_->finish(b, nullptr, ST_ERROR);
  tr.status = ST_ERROR;
  tr.finished_us = now_us();
  record(tr, b);
  if (++failures_ < opt_.max_failures) return false;
  healthy_ = false;
  if (group_ && group_->leave()) batcher_->shutdown();   // nobody left to drain the queue
  return true;
}

void Executor::loop() {
  std::deque<Pending> pending;
  std::vector<kdl_dev_piece> pieces;
  int slot = 0;
  bool gave_up = false;
  while (!stop_.load() && !gave_up) {
    // with work in flight never sleep in the batcher; an idle device dispatches whatever is
    // queued (eager) instead of waiting out the batch timeout
    const int64_t poll = pending.empty() ? opt_.poll_us : 0;
    Pending p;
    p.slot = slot;
    const bool got = batcher_->next_batch(be_.staging(be_.ctx, slot), poll, &p.batch, opt_.eager && pending.empty());
    if (got) {
      p.tr.batch_id = p.batch.id;
      p.tr.n_real = p.batch.n_real;
      p.tr.bucket = p.batch.bucket;
      p.tr.slot = slot;
      p.tr.oldest_enqueue_us = p.batch.oldest_enqueue_us;
      p.tr.formed_us = p.batch.formed_us;
      p.tr.copied_us = now_us();
      if (opt_.delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(opt_.delay_us));
      int rc = 0;
      if (fail_left_ != 0) {
        if (fail_left_ > 0) --fail_left_;
        rc = -1;                                            // injected fault
      } else {
        pieces.clear();
        for (size_t i = 0; i < p.batch.dev_src.size(); ++i)
          if (p.batch.dev_src[i]) pieces.push_back({p.batch.first_item[i], p.batch.n_items[i], p.batch.dev_src[i]});
        if (pieces.empty())
          rc = be_.issue(be_.ctx, slot, p.batch.bucket, p.batch.n_real);
        else if (be_.issue_dev)
          rc = be_.issue_dev(be_.ctx, slot, p.batch.bucket, p.batch.n_real, pieces.data(), int(pieces.size()));
        else
          rc = -1;                                          // this backend takes host payloads only
      }
      if (rc != 0) {
        gave_up = fail(p.batch, p.tr);
      } else {
        p.tr.issued_us = now_us();
        pending.push_back(std::move(p));
        slot = (slot + 1) % be_.nslots;
      }
    }
    if (!pending.empty() && (!got || int(pending.size()) >= be_.nslots || gave_up)) {
      Pending d = std::move(pending.front());
      pending.pop_front();
      const float* out = nullptr;
      kdl_device_times t{-1.f, -1.f, -1.f};
      const int rc = be_.complete(be_.ctx, d.slot, &out, &t);
      d.tr.completed_us = now_us();
      d.tr.h2d_ms = t.h2d_ms;
      d.tr.forward_ms = t.forward_ms;
      d.tr.d2h_ms = t.d2h_ms;
      if (rc != 0 || out == nullptr) {
        gave_up = fail(d.batch, d.tr) || gave_up;
      } else {
        batcher_->finish(d.batch, out, ST_OK);
        d.tr.finished_us = now_us();
        d.tr.status = ST_OK;
        failures_ = 0;
        record(d.tr, d.batch);
      }
    }
  }
  // leaving (stop or give-up): drain what is in flight
  while (!pending.empty()) {
    Pending d = std::move(pending.front());
    pending.pop_front();
    const float* out = nullptr;
    kdl_device_times t{-1.f, -1.f, -1.f};
    const int rc = gave_up ? -1 : be_.complete(be_.ctx, d.slot, &out, &t);
    if (rc == 0 && out) {
      batcher_->finish(d.batch, out, ST_OK);
    } else {
      if (gave_up) (void)be_.complete(be_.ctx, d.slot, &out, &t);   // device work must end first
      batcher_->finish(d.batch, nullptr, gave_up ? ST_ERROR : ST_SHUTDOWN);
    }
  }
  running_ = false;
}

// --------------------------------------------------------------------------- fake backend
namespace {
uint8_t* fake_staging(void* ctx, int slot) { return static_cast<FakeBackend*>(ctx)->staging[slot].data(); }

int fake_issue(void* ctx, int slot, int bucket, int n_real) {
  auto* f = static_cast<FakeBackend*>(ctx);
  ++f->issued;
  if (f->fail_every > 0 && f->issued % f->fail_every == 0) return -1;
  for (int i = 0; i < bucket; ++i)
    for (int k = 0; k < f->out_cols; ++k)
      f->out[slot][size_t(i) * f->out_cols + k] =
          i < n_real ? float(f->staging[slot][size_t(i) * f->item_bytes]) + float(k) : -1.f;
  f->ready_at[slot] = now_us() + f->latency_us;
  f->bucket[slot] = bucket;
  return 0;
}

int fake_issue_dev(void* ctx, int slot, int bucket, int n_real, const kdl_dev_piece* pc, int np) {
  auto* f = static_cast<FakeBackend*>(ctx);   // "device" memory is host memory here
  for (int i = 0; i < np; ++i)
    std::memcpy(f->staging[slot].data() + size_t(pc[i].row) * f->item_bytes, pc[i].src,
                size_t(pc[i].n_items) * f->item_bytes);
  ++f->dev_pieces;
  return fake_issue(ctx, slot, bucket, n_real);
}

int fake_complete(void* ctx, int slot, const float** out, kdl_device_times* t) {
  auto* f = static_cast<FakeBackend*>(ctx);
  const int64_t wait = f->ready_at[slot] - now_us();
  if (wait > 0) std::this_thread::sleep_for(std::chrono::microseconds(wait));
  *out = f->out[slot].data();
  if (t) { t->h2d_ms = 0.f; t->forward_ms = f->latency_us * 1e-3f; t->d2h_ms = 0.f; }
  return 0;
}
}  // namespace

FakeBackend::FakeBackend(int nslots, size_t item_bytes_, int max_batch, int out_cols_, int64_t latency_us_,
                         int fail_every_)
    : staging(nslots, std::vector<uint8_t>(item_bytes_ * max_batch)),
      out(nslots, std::vector<float>(size_t(out_cols_) * max_batch)),
      ready_at(nslots, 0), bucket(nslots, 0), item_bytes(item_bytes_), out_cols(out_cols_),
      latency_us(latency_us_), fail_every(fail_every_) {
  api.ctx = this;
  api.nslots = nslots;
  api.out_cols = out_cols_;
  api.staging = fake_staging;
  api.issue = fake_issue;
  api.complete = fake_complete;
  api.issue_dev = fake_issue_dev;
}

}  // namespace kdl
