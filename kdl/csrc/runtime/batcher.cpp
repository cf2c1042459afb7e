#include "batcher.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

namespace kdl {

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

CopyPool::CopyPool(int threads) {
  try {
    for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { worker(); });
  } catch (const std::system_error&) {
    // fewer (or no) helper threads: run() still completes every job on the calling thread
  }
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_work_.notify_all();
  for (auto& t : workers_) t.join();
}

void CopyPool::drain(Job& j) {
  const auto& p = *j.pieces;
  for (size_t k; (k = j.next.fetch_add(1)) < p.size();) {
    std::memcpy(p[k].dst, p[k].src, p[k].n);
    j.done.fetch_add(1, std::memory_order_release);
  }
}

void CopyPool::worker() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_work_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
    if (stop_) return;
    Job* j = jobs_.front();
    ++j->users;                                 // the owner keeps the job alive while users > 0
    lk.unlock();
    drain(*j);
    lk.lock();
    --j->users;
    if (!jobs_.empty() && jobs_.front() == j) jobs_.pop_front();   // every piece is claimed
    cv_done_.notify_all();
  }
}

void CopyPool::run(const std::vector<Piece>& pieces) {
  if (pieces.empty()) return;
  Job j;
  j.pieces = &pieces;
  const bool helpers = !workers_.empty() && pieces.size() > 1;
  if (helpers) {
    std::lock_guard<std::mutex> lk(mu_);
    jobs_.push_back(&j);
  }
  if (helpers) cv_work_.notify_all();
  drain(j);
  if (!helpers) return;
  std::unique_lock<std::mutex> lk(mu_);
  cv_done_.wait(lk, [&] { return j.done.load(std::memory_order_acquire) == pieces.size() && j.users == 0; });
  // unlink before the job leaves this frame (a worker may not have popped it yet)
  for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
    if (*it == &j) { jobs_.erase(it); break; }
}

DynamicBatcher::DynamicBatcher(const BatcherOptions& o) : opt_(o) {
  std::sort(opt_.allowed_batch_sizes.begin(), opt_.allowed_batch_sizes.end());
  if (!opt_.allowed_batch_sizes.empty() && opt_.allowed_batch_sizes.back() != opt_.max_batch_size)
    opt_.allowed_batch_sizes.push_back(opt_.max_batch_size);  // TF-Serving requires last == max
  if (opt_.copy_threads > 1 && opt_.item_bytes) pool_ = std::make_unique<CopyPool>(opt_.copy_threads - 1);
}

DynamicBatcher::~DynamicBatcher() { shutdown(); }

int DynamicBatcher::bucket_for(int n) const {
  for (int b : opt_.allowed_batch_sizes)
    if (b >= n) return b;
  return n;
}

int64_t DynamicBatcher::submit(const uint8_t* data, int n_items, int64_t deadline_us, bool device) {
  std::lock_guard<std::mutex> lk(mu_);
  return enqueue_locked(data, n_items, deadline_us, device, nullptr);
}

int64_t DynamicBatcher::submit_async(const uint8_t* data, int n_items, int64_t deadline_us, DoneFn done) {
  if (!done) return -ST_ERROR;
  std::lock_guard<std::mutex> lk(mu_);
  return enqueue_locked(data, n_items, deadline_us, false, std::move(done));
}

int64_t DynamicBatcher::enqueue_locked(const uint8_t* data, int n_items, int64_t deadline_us, bool device,
                                       DoneFn done) {
  if (n_items <= 0 || n_items > opt_.max_batch_size) return -ST_ERROR;
  if (shutdown_) return -ST_SHUTDOWN;
  if (queued_items_ + n_items > int64_t(opt_.max_enqueued_batches) * opt_.max_batch_size) {
    ++st_.rejected;
    return -ST_QUEUE_FULL;
  }
  auto r = std::make_shared<Req>();
  r->ticket = next_ticket_++;
  r->data = data;
  r->device = device;
  r->n_items = n_items;
  r->enqueue_us = now_us();
  r->deadline_us = deadline_us;
  r->done = std::move(done);
  queue_.push_back(r);
  (r->done ? async_live_ : live_)[r->ticket] = r;   // async requests are never wait()ed
  queued_items_ += n_items;
  ++st_.submitted;
  cv_consumer_.notify_one();
  return r->ticket;
}

int DynamicBatcher::wait(int64_t ticket, float* out, size_t out_floats) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = live_.find(ticket);
  if (it == live_.end()) return ST_ERROR;
  auto r = it->second;
  for (;;) {
    if (r->state == DONE || r->state == ABANDONED) break;   // ABANDONED: expired by next_batch
    if (shutdown_ && r->state != TAKEN) {   // TAKEN: payload copy in flight, wait for it
      if (r->state == QUEUED) {
        auto q = std::find(queue_.begin(), queue_.end(), r);
        if (q != queue_.end()) { queue_.erase(q); queued_items_ -= r->n_items; }
      }
      r->state = ABANDONED;
      r->status = ST_SHUTDOWN;
      break;
    }
    const int64_t now = now_us();
    if (r->deadline_us > 0 && now >= r->deadline_us && r->state != TAKEN) {
      // expired: a QUEUED request is removed here; a COPIED one is abandoned
      // (its payload is no longer referenced, finish() will skip it)
      if (r->state == QUEUED) {
        auto q = std::find(queue_.begin(), queue_.end(), r);
        if (q != queue_.end()) { queue_.erase(q); queued_items_ -= r->n_items; }
      }
      r->state = ABANDONED;
      r->status = ST_DEADLINE;
      ++st_.expired;
      break;
    }
    if (r->deadline_us > 0 && r->state != TAKEN)
      cv_producer_.wait_for(lk, std::chrono::microseconds(std::max<int64_t>(1, r->deadline_us - now)));
    else
      cv_producer_.wait(lk);
  }
  int status = r->status;
  if (status == ST_OK && out) {
    if (r->result.size() > out_floats) status = ST_ERROR;   // caller's buffer too small: never overrun it
    else std::memcpy(out, r->result.data(), r->result.size() * sizeof(float));
  }
  live_.erase(ticket);
  return status;
}

bool DynamicBatcher::next_batch(uint8_t* staging, int64_t poll_us, Batch* b, bool eager) {
  std::vector<std::shared_ptr<Req>> take, expired;
  struct Fire {                              // async callbacks of expired requests, outside the lock
    std::vector<std::shared_ptr<Req>>& v;
    ~Fire() { for (auto& r : v) r->done(ST_DEADLINE, nullptr, 0); }
  } fire{expired};
  {
    std::unique_lock<std::mutex> lk(mu_);
    const int64_t give_up = now_us() + poll_us;
    for (;;) {
      if (shutdown_) return false;
      // drop expired requests at the head of the queue
      const int64_t now = now_us();
      for (auto q = queue_.begin(); q != queue_.end();) {
        if ((*q)->deadline_us > 0 && now >= (*q)->deadline_us) {
          (*q)->state = ABANDONED;
          (*q)->status = ST_DEADLINE;
          queued_items_ -= (*q)->n_items;
          ++st_.expired;
          if ((*q)->done) {
            async_live_.erase((*q)->ticket);
            expired.push_back(*q);
          }
          q = queue_.erase(q);
          cv_producer_.notify_all();
        } else {
          ++q;
        }
      }
      if (!queue_.empty()) {
        const bool full = queued_items_ >= opt_.max_batch_size;
        const bool timed_out = now - queue_.front()->enqueue_us >= opt_.batch_timeout_us;
        if (full || timed_out || eager) break;
        const int64_t wake = std::min(give_up, queue_.front()->enqueue_us + opt_.batch_timeout_us);
        if (now >= give_up) return false;
        cv_consumer_.wait_for(lk, std::chrono::microseconds(std::max<int64_t>(1, wake - now)));
      } else {
        if (now >= give_up) return false;
        cv_consumer_.wait_for(lk, std::chrono::microseconds(give_up - now));
      }
    }
    // greedily pack whole requests in FIFO order
    int n = 0;
    b->tickets.clear(); b->first_item.clear(); b->n_items.clear(); b->dev_src.clear();
    b->oldest_enqueue_us = queue_.front()->enqueue_us;
    while (!queue_.empty() && n + queue_.front()->n_items <= opt_.max_batch_size) {
      auto r = queue_.front();
      queue_.pop_front();
      queued_items_ -= r->n_items;
      r->state = TAKEN;
      b->tickets.push_back(r->ticket);
      b->first_item.push_back(n);
      b->n_items.push_back(r->n_items);
      b->dev_src.push_back(r->device ? r->data : nullptr);
      n += r->n_items;
      take.push_back(r);
    }
    b->id = next_batch_++;
    b->formed_us = now_us();
    b->n_real = n;
    b->bucket = bucket_for(n);
    ++st_.batches;
    st_.items += n;
    st_.padded_items += b->bucket - n;
  }
  // payload copies outside the lock (producers stay blocked in wait() on TAKEN). A full
  // Xception batch is 8.6 MB into pinned memory: ~1 ms for one thread, which is most of a
  // 1.45 ms GPU batch, so large batches are cut into ~1 MiB pieces copied by the
  // persistent pool (copy_threads - 1 workers) and the caller; small ones stay on the caller
  if (staging && opt_.item_bytes) {
    std::vector<CopyPool::Piece> pieces;
    size_t total = 0;
    constexpr size_t kPiece = size_t(1) << 20;
    for (size_t i = 0; i < take.size(); ++i) {
      if (take[i]->device) continue;         // copied on the device by the backend
      uint8_t* dst = staging + size_t(b->first_item[i]) * opt_.item_bytes;
      const uint8_t* src = take[i]->data;
      const size_t n = size_t(take[i]->n_items) * opt_.item_bytes;
      for (size_t o = 0; o < n; o += kPiece) pieces.push_back({dst + o, src + o, std::min(kPiece, n - o)});
      total += n;
    }
    if (pool_ && total >= 2 * kPiece) {
      pool_->run(pieces);
    } else {
      for (const auto& p : pieces) std::memcpy(p.dst, p.src, p.n);
    }
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& r : take)
      if (r->state == TAKEN) r->state = COPIED;
  }
  cv_producer_.notify_all();
  return true;
}

void DynamicBatcher::finish(const Batch& b, const float* results, int status) {
  std::vector<std::pair<std::shared_ptr<Req>, size_t>> async;   // (request, its batch index)
  {
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < b.tickets.size(); ++i) {
    auto it = live_.find(b.tickets[i]);
    if (it == live_.end()) {
      auto a = async_live_.find(b.tickets[i]);
      if (a != async_live_.end()) {
        a->second->state = DONE;
        ++st_.completed;
        async.emplace_back(std::move(a->second), i);
        async_live_.erase(a);
      }
      continue;
    }
    auto& r = it->second;
    if (r->state == ABANDONED) continue;
    r->status = status;
    if (status == ST_OK && results) {
      const size_t n = size_t(b.n_items[i]) * opt_.out_cols;
      r->result.assign(results + size_t(b.first_item[i]) * opt_.out_cols,
                       results + size_t(b.first_item[i]) * opt_.out_cols + n);
    }
    r->state = DONE;
    ++st_.completed;
  }
  cv_producer_.notify_all();
  }
  for (auto& [r, i] : async) {
    const bool rows = status == ST_OK && results;
    r->done(rows ? status : (status == ST_OK ? ST_ERROR : status),
            rows ? results + size_t(b.first_item[i]) * opt_.out_cols : nullptr,
            rows ? size_t(b.n_items[i]) * opt_.out_cols : 0);
  }
}

void DynamicBatcher::shutdown() {
  std::vector<std::shared_ptr<Req>> dropped;   // queued async requests: answered here
  {
    std::lock_guard<std::mutex> lk(mu_);
    shutdown_ = true;
    for (auto q = queue_.begin(); q != queue_.end();) {
      if ((*q)->done) {
        (*q)->state = ABANDONED;
        queued_items_ -= (*q)->n_items;
        async_live_.erase((*q)->ticket);
        dropped.push_back(*q);
        q = queue_.erase(q);
      } else {
        ++q;
      }
    }
    cv_consumer_.notify_all();
    cv_producer_.notify_all();
  }
  for (auto& r : dropped) r->done(ST_SHUTDOWN, nullptr, 0);
}

BatcherStats DynamicBatcher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  BatcherStats s = st_;
  s.queue_items = queued_items_;
  return s;
}

}  // namespace kdl
