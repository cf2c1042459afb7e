#include "hip_backend.h"

#include <stdexcept>

namespace kdl {

namespace {
uint8_t* be_staging(void* ctx, int slot) { return static_cast<HipExecBackend*>(ctx)->staging(slot); }
int be_issue(void* ctx, int slot, int bucket, int n_real) {
  return static_cast<HipExecBackend*>(ctx)->issue(slot, bucket, n_real);
}
int be_issue_dev(void* ctx, int slot, int bucket, int n_real, const kdl_dev_piece* pc, int np) {
  return static_cast<HipExecBackend*>(ctx)->issue_dev(slot, bucket, n_real, pc, np);
}
int be_complete(void* ctx, int slot, const float** out, kdl_device_times* t) {
  return static_cast<HipExecBackend*>(ctx)->complete(slot, out, t);
}
#define KDL_TRY(expr)                          \
  do {                                         \
    if ((expr) != hipSuccess) return -1;       \
  } while (0)
}  // namespace

HipExecBackend::HipExecBackend(int device, int nslots, size_t item_bytes, int max_batch, int out_cols,
                               hipStream_t copy_stream, bool timing)
    : device_(device), nslots_(nslots), item_bytes_(item_bytes), max_batch_(max_batch), out_cols_(out_cols),
      copy_(copy_stream), timing_(timing) {
  if (nslots < 1 || max_batch < 1 || out_cols < 1) throw std::invalid_argument("HipExecBackend: bad geometry");
  check_hip(hipSetDevice(device), "hipSetDevice");
  if (!copy_) {
    check_hip(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "hipStreamCreate(copy)");
    own_copy_ = true;
  }
  const unsigned evf = timing ? hipEventDefault : hipEventDisableTiming;
  for (int s = 0; s < nslots; ++s) {
    void* p = nullptr;
    check_hip(hipHostMalloc(&p, item_bytes * max_batch, hipHostMallocDefault), "hipHostMalloc(staging)");
    staging_.push_back(static_cast<uint8_t*>(p));
    check_hip(hipHostMalloc(&p, sizeof(float) * out_cols * max_batch, hipHostMallocDefault), "hipHostMalloc(out)");
    out_.push_back(static_cast<float*>(p));
    for (auto* v : {&ev_h2d0_, &ev_h2d1_, &ev_fw0_, &ev_fw1_, &ev_done_}) {
      hipEvent_t e;
      check_hip(hipEventCreateWithFlags(&e, evf), "hipEventCreate");
      v->push_back(e);
    }
  }
  slot_bucket_.assign(nslots, 0);
  api_.ctx = this;
  api_.nslots = nslots;
  api_.out_cols = out_cols;
  api_.staging = be_staging;
  api_.issue = be_issue;
  api_.complete = be_complete;
  api_.issue_dev = be_issue_dev;
}

HipExecBackend::~HipExecBackend() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(copy_);
  for (auto& kv : recipes_) {
    for (auto s : kv.second.streams) (void)hipStreamSynchronize(s);
    for (auto& v : kv.second.done)
      for (auto e : v) (void)hipEventDestroy(e);
  }
  for (auto* v : {&ev_h2d0_, &ev_h2d1_, &ev_fw0_, &ev_fw1_, &ev_done_})
    for (auto e : *v) (void)hipEventDestroy(e);
  for (auto p : staging_) (void)hipHostFree(p);
  for (auto p : out_) (void)hipHostFree(p);
  if (own_copy_) (void)hipStreamDestroy(copy_);
}

void HipExecBackend::add_recipe(int bucket, const std::vector<hipStream_t>& streams, const std::vector<int>& wait_for,
                                const std::vector<std::vector<std::vector<const Program*>>>& progs,
                                const std::vector<void*>& dev_in, const std::vector<void*>& dev_out) {
  const int K = int(streams.size());
  if (K < 1 || int(wait_for.size()) != K || int(progs.size()) != nslots_ || int(dev_in.size()) != nslots_ ||
      int(dev_out.size()) != nslots_ || bucket < 1 || bucket > max_batch_)
    throw std::invalid_argument("add_recipe: shape mismatch");
  for (const auto& ps : progs) {
    if (ps.size() != 2) throw std::invalid_argument("add_recipe: one program list per parity");
    for (const auto& pk : ps)
      if (int(pk.size()) != K) throw std::invalid_argument("add_recipe: one program per stage");
  }
  Recipe r;
  r.K = K;
  r.streams = streams;
  r.wait_for = wait_for;
  r.progs = progs;
  r.dev_in = dev_in;
  r.dev_out = dev_out;
  check_hip(hipSetDevice(device_), "hipSetDevice");
  for (auto& v : r.done)
    for (int k = 0; k < K; ++k) {
      hipEvent_t e;
      check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      v.push_back(e);
    }
  auto it = recipes_.find(bucket);
  if (it != recipes_.end()) {
    for (auto& v : it->second.done)
      for (auto e : v) (void)hipEventDestroy(e);
    recipes_.erase(it);
  }
  recipes_.emplace(bucket, std::move(r));
}

int HipExecBackend::launch(int slot, int bucket, hipEvent_t ready, hipStream_t* last) {
  if (slot < 0 || slot >= nslots_) return -1;
  auto it = recipes_.find(bucket);
  if (it == recipes_.end()) return -1;
  Recipe& r = it->second;
  const int p = int(r.issued & 1);
  ++r.issued;
  for (int k = 0; k < r.K; ++k) {
    hipStream_t st = r.streams[k];
    KDL_TRY(hipStreamWaitEvent(st, k == 0 ? ready : r.done[p][k - 1], 0));
    if (r.wait_for[k] > k) KDL_TRY(hipStreamWaitEvent(st, r.done[p][r.wait_for[k]], 0));
    if (k == 0 && timing_) KDL_TRY(hipEventRecord(ev_fw0_[slot], st));
    try {
      r.progs[slot][p][k]->launch(st);
    } catch (const std::exception&) {
      return -1;
    }
    KDL_TRY(hipEventRecord(r.done[p][k], st));
  }
  *last = r.streams[r.K - 1];
  return 0;
}

void* HipExecBackend::dev_in(int slot, int bucket) const {
  auto it = recipes_.find(bucket);
  return it == recipes_.end() || slot < 0 || slot >= nslots_ ? nullptr : it->second.dev_in[slot];
}

void* HipExecBackend::dev_out(int slot, int bucket) const {
  auto it = recipes_.find(bucket);
  return it == recipes_.end() || slot < 0 || slot >= nslots_ ? nullptr : it->second.dev_out[slot];
}

int HipExecBackend::issue(int slot, int bucket, int n_real) {
  return issue_dev(slot, bucket, n_real, nullptr, 0);
}

int HipExecBackend::issue_dev(int slot, int bucket, int n_real, const kdl_dev_piece* pieces, int npieces) {
  (void)n_real;                               // padding rows are computed and ignored
  if (slot < 0 || slot >= nslots_) return -1;
  auto it = recipes_.find(bucket);
  if (it == recipes_.end()) return -1;
  uint8_t* din = static_cast<uint8_t*>(it->second.dev_in[slot]);
  KDL_TRY(hipSetDevice(device_));
  if (timing_) KDL_TRY(hipEventRecord(ev_h2d0_[slot], copy_));
  // host rows: H2D in contiguous runs between the (row-sorted) device pieces; device rows: D2D
  // (hipMemcpyDefault: a piece resized on another GPU of the node comes over xGMI)
  int row = 0;
  for (int i = 0; i <= npieces; ++i) {
    const int end = i < npieces ? pieces[i].row : bucket;
    if (end < row || end > bucket) return -1;
    if (end > row)
      KDL_TRY(hipMemcpyAsync(din + item_bytes_ * row, staging_[slot] + item_bytes_ * row, item_bytes_ * (end - row),
                             hipMemcpyHostToDevice, copy_));
    if (i == npieces) break;
    const int n = pieces[i].n_items;
    if (n < 1 || end + n > bucket || !pieces[i].src) return -1;
    KDL_TRY(hipMemcpyAsync(din + item_bytes_ * end, pieces[i].src, item_bytes_ * n, hipMemcpyDefault, copy_));
    row = end + n;
  }
  KDL_TRY(hipEventRecord(ev_h2d1_[slot], copy_));
  return finish_issue(slot, bucket);
}

int HipExecBackend::finish_issue(int slot, int bucket) {
  Recipe& r = recipes_.find(bucket)->second;
  hipStream_t last = nullptr;
  if (launch(slot, bucket, ev_h2d1_[slot], &last) != 0) return -1;
  if (timing_) KDL_TRY(hipEventRecord(ev_fw1_[slot], last));
  KDL_TRY(hipMemcpyAsync(out_[slot], r.dev_out[slot], sizeof(float) * out_cols_ * bucket, hipMemcpyDeviceToHost, last));
  KDL_TRY(hipEventRecord(ev_done_[slot], last));
  slot_bucket_[slot] = bucket;
  return 0;
}

int HipExecBackend::complete(int slot, const float** out, kdl_device_times* t) {
  if (slot < 0 || slot >= nslots_) return -1;
  KDL_TRY(hipSetDevice(device_));
  KDL_TRY(hipEventSynchronize(ev_done_[slot]));
  *out = out_[slot];
  if (t) {
    t->h2d_ms = t->forward_ms = t->d2h_ms = -1.f;
    if (timing_) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, ev_h2d0_[slot], ev_h2d1_[slot]) == hipSuccess) t->h2d_ms = ms;
      if (hipEventElapsedTime(&ms, ev_fw0_[slot], ev_fw1_[slot]) == hipSuccess) t->forward_ms = ms;
      if (hipEventElapsedTime(&ms, ev_fw1_[slot], ev_done_[slot]) == hipSuccess) t->d2h_ms = ms;
    }
  }
  return 0;
}

}  // namespace kdl
