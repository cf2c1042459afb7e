#include "comm.h"

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace kdl {

namespace {
void check_nccl(ncclResult_t r, const std::string& what) {
  if (r != ncclSuccess) throw std::runtime_error(what + ": " + ncclGetErrorString(r));
}
#define KDL_TRY(expr)                    \
  do {                                   \
    if ((expr) != hipSuccess) return -1; \
  } while (0)
#define KDL_NTRY(expr)                     \
  do {                                     \
    if ((expr) != ncclSuccess) return -1;  \
  } while (0)

int be_issue(void* ctx, int slot, int bucket, int n_real) {
  return static_cast<DpLeader*>(ctx)->issue(slot, bucket, n_real);
}
int be_complete(void* ctx, int slot, const float** out, kdl_device_times* t) {
  return static_cast<DpLeader*>(ctx)->complete(slot, out, t);
}

hipEvent_t new_event() {
  hipEvent_t e;
  check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  return e;
}

// poll an event: spin briefly (a step's control word usually lands within microseconds of the
// previous one), then sleep between queries so an idle rank does not burn a CPU core
bool poll_event(hipEvent_t e, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) return false;
    if (i > 2000) usleep(50);
    if (timeout_s > 0 && i % 64 == 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return false;
  }
}
}  // namespace

std::string rccl_unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

RcclComm::RcclComm(const std::string& id, int nranks, int rank, int device) : rank_(rank), size_(nranks), device_(device) {
  if (id.size() != NCCL_UNIQUE_ID_BYTES || nranks < 1 || rank < 0 || rank >= nranks)
    throw std::invalid_argument("RcclComm: bad id / rank");
  ncclUniqueId u;
  std::memcpy(u.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
  check_hip(hipSetDevice(device), "hipSetDevice");
  check_nccl(ncclCommInitRank(&comm_, nranks, u, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  if (comm_) {
    (void)hipSetDevice(device_);
    (void)ncclCommDestroy(comm_);
  }
}

void RcclComm::abort() {
  if (comm_) {
    (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }
}

bool RcclComm::async_error() const {
  if (!comm_) return true;
  ncclResult_t r = ncclSuccess;
  return ncclCommGetAsyncError(comm_, &r) != ncclSuccess || (r != ncclSuccess && r != ncclInProgress);
}

// ------------------------------------------------------------------------------------ leader
DpLeader::DpLeader(HipExecBackend* local, RcclComm* scatter, RcclComm* gather, std::vector<int> rank_buckets,
                   double timeout_s)
    : L_(local), S_(scatter), G_(gather), world_(scatter->size()), buckets_(std::move(rank_buckets)),
      timeout_s_(timeout_s) {
  if (G_->size() != world_ || S_->rank() != 0 || G_->rank() != 0 || buckets_.empty())
    throw std::invalid_argument("DpLeader: rank 0 of two equal-size communicators, >= 1 bucket");
  max_shard_ = *std::max_element(buckets_.begin(), buckets_.end());
  for (int b : buckets_)
    if (!L_->dev_in(0, b)) throw std::invalid_argument("DpLeader: no local recipe for a rank bucket");
  if (L_->max_batch() < world_ * max_shard_) throw std::invalid_argument("DpLeader: local staging < world x bucket");
  check_hip(hipSetDevice(L_->device()), "hipSetDevice");
  for (auto* s : {&cs_, &ss_, &gs_}) check_hip(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate");
  const int ns = L_->nslots();
  for (int s = 0; s <= ns; ++s) {              // slot ns: control words outside batches
    void* p = nullptr;
    check_hip(hipMalloc(&p, sizeof(DpCtrl)), "hipMalloc(ctrl)");
    d_ctrl_.push_back(static_cast<DpCtrl*>(p));
    check_hip(hipHostMalloc(&p, sizeof(DpCtrl), hipHostMallocDefault), "hipHostMalloc(ctrl)");
    h_ctrl_.push_back(static_cast<DpCtrl*>(p));
    if (s == ns) break;
    p = nullptr;
    if (world_ > 1) check_hip(hipMalloc(&p, L_->item_bytes() * (world_ - 1) * max_shard_), "hipMalloc(send)");
    d_send_.push_back(static_cast<uint8_t*>(p));
    check_hip(hipMalloc(&p, sizeof(float) * L_->out_cols() * world_ * max_shard_), "hipMalloc(gather)");
    d_gather_.push_back(static_cast<float*>(p));
    ev_in_.push_back(new_event());
    ev_sent_.push_back(new_event());
    ev_gdone_.push_back(new_event());
  }
  slot_shard_.assign(ns, 0);
  api_.ctx = this;
  api_.nslots = ns;
  api_.out_cols = L_->out_cols();
  api_.staging = [](void* ctx, int slot) { return static_cast<DpLeader*>(ctx)->L_->staging(slot); };
  api_.issue = be_issue;
  api_.complete = be_complete;
}

DpLeader::~DpLeader() {
  (void)hipSetDevice(L_->device());
  for (auto s : {cs_, ss_, gs_})
    if (s) (void)hipStreamSynchronize(s);
  for (auto* v : {&ev_in_, &ev_sent_, &ev_gdone_})
    for (auto e : *v) (void)hipEventDestroy(e);
  for (auto p : d_send_) (void)hipFree(p);
  for (auto p : d_gather_) (void)hipFree(p);
  for (auto p : d_ctrl_) (void)hipFree(p);
  for (auto p : h_ctrl_) (void)hipHostFree(p);
  for (auto s : {cs_, ss_, gs_})
    if (s) (void)hipStreamDestroy(s);
}

int DpLeader::wait(hipEvent_t e) {
  if (poll_event(e, timeout_s_)) return 0;
  // a follower died or stalled: unblock the communicators so no later step hangs on them
  broken_ = true;
  S_->abort();
  G_->abort();
  return -1;
}

int DpLeader::issue(int slot, int bucket, int n_real) {
  std::lock_guard<std::mutex> lk(mu_);
  if (broken_ || closed_ || slot < 0 || slot >= L_->nslots() || bucket % world_ != 0) return -1;
  const int shard = bucket / world_;
  if (std::find(buckets_.begin(), buckets_.end(), shard) == buckets_.end()) return -1;
  KDL_TRY(hipSetDevice(L_->device()));
  const DpGeometry g{world_, L_->item_bytes(), L_->out_cols()};
  const size_t ib = L_->item_bytes();
  *h_ctrl_[slot] = DpCtrl{DP_BATCH, shard, n_real, seq_++, 0, {0, 0, 0}};
  if (world_ > 1) {
    KDL_TRY(hipMemcpyAsync(d_ctrl_[slot], h_ctrl_[slot], sizeof(DpCtrl), hipMemcpyHostToDevice, cs_));
    KDL_TRY(hipMemcpyAsync(d_send_[slot], L_->staging(slot) + ib * shard, ib * shard * (world_ - 1),
                           hipMemcpyHostToDevice, cs_));
    KDL_TRY(hipEventRecord(ev_in_[slot], cs_));
  }
  // rank 0's own shard: rows [0, shard) of the staging, straight into its engine's input slot
  if (L_->issue(slot, shard, std::min(n_real, shard)) != 0) return -1;
  if (world_ > 1) {
    const auto msgs = dp_leader_step(g, DP_BATCH, shard);
    std::vector<DpMsg> sc, ga;
    for (const auto& m : msgs) (m.channel == DP_SCATTER ? sc : ga).push_back(m);
    KDL_TRY(hipStreamWaitEvent(ss_, ev_in_[slot], 0));
    KDL_NTRY(dp_post(sc, *S_, ss_, [&](const DpMsg& m) -> void* {
      return m.what == 0 ? static_cast<void*>(d_ctrl_[slot])
                         : static_cast<void*>(d_send_[slot] + ib * shard * (m.peer - 1));
    }));
    KDL_TRY(hipEventRecord(ev_sent_[slot], ss_));
    KDL_NTRY(dp_post(ga, *G_, gs_, [&](const DpMsg& m) -> void* {
      return static_cast<void*>(d_gather_[slot] + (size_t)g.out_cols * shard * m.peer);
    }));
    KDL_TRY(hipMemcpyAsync(L_->host_out_mut(slot) + (size_t)g.out_cols * shard, d_gather_[slot] + (size_t)g.out_cols * shard,
                           sizeof(float) * g.out_cols * shard * (world_ - 1), hipMemcpyDeviceToHost, gs_));
    KDL_TRY(hipEventRecord(ev_gdone_[slot], gs_));
  }
  slot_shard_[slot] = shard;
  return 0;
}

int DpLeader::complete(int slot, const float** out, kdl_device_times* t) {
  if (slot < 0 || slot >= L_->nslots()) return -1;
  if (L_->complete(slot, out, t) != 0) return -1;
  if (world_ > 1) {
    KDL_TRY(hipSetDevice(L_->device()));
    if (wait(ev_gdone_[slot]) != 0 || wait(ev_sent_[slot]) != 0) return -1;
  }
  return 0;
}

int DpLeader::send_ctrl(int cmd, int version) {
  std::lock_guard<std::mutex> lk(mu_);
  if (broken_ || closed_ || cmd == DP_BATCH) return -1;
  closed_ = true;
  if (world_ == 1) return 0;
  KDL_TRY(hipSetDevice(L_->device()));
  const int x = L_->nslots();
  *h_ctrl_[x] = DpCtrl{cmd, 0, 0, seq_++, version, {0, 0, 0}};
  KDL_TRY(hipMemcpyAsync(d_ctrl_[x], h_ctrl_[x], sizeof(DpCtrl), hipMemcpyHostToDevice, ss_));
  const DpGeometry g{world_, L_->item_bytes(), L_->out_cols()};
  KDL_NTRY(dp_post(dp_leader_step(g, cmd, 0), *S_, ss_, [&](const DpMsg&) -> void* { return d_ctrl_[x]; }));
  hipEvent_t e = new_event();
  const hipError_t r = hipEventRecord(e, ss_);
  const int ok = r == hipSuccess ? wait(e) : -1;
  (void)hipEventDestroy(e);
  return ok;
}

// ---------------------------------------------------------------------------------- follower
DpFollower::DpFollower(HipExecBackend* local, RcclComm* scatter, RcclComm* gather)
    : L_(local), S_(scatter), G_(gather), nslots_(local->nslots()) {
  if (S_->rank() == 0 || G_->rank() != S_->rank() || G_->size() != S_->size())
    throw std::invalid_argument("DpFollower: a rank >= 1 of two matching communicators");
  check_hip(hipSetDevice(L_->device()), "hipSetDevice");
  for (auto* s : {&ss_, &gs_}) check_hip(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate");
  for (int s = 0; s < nslots_; ++s) {
    void* p = nullptr;
    check_hip(hipMalloc(&p, sizeof(DpCtrl)), "hipMalloc(ctrl)");
    d_ctrl_.push_back(static_cast<DpCtrl*>(p));
    check_hip(hipHostMalloc(&p, sizeof(DpCtrl), hipHostMallocDefault), "hipHostMalloc(ctrl)");
    h_ctrl_.push_back(static_cast<DpCtrl*>(p));
    for (auto* v : {&ev_ctrl_, &ev_in_, &ev_fw_, &ev_free_}) v->push_back(new_event());
    check_hip(hipEventRecord(ev_free_.back(), gs_), "hipEventRecord");
  }
}

DpFollower::~DpFollower() {
  (void)hipSetDevice(L_->device());
  for (auto s : {ss_, gs_})
    if (s) (void)hipStreamSynchronize(s);
  for (auto* v : {&ev_ctrl_, &ev_in_, &ev_fw_, &ev_free_})
    for (auto e : *v) (void)hipEventDestroy(e);
  for (auto p : d_ctrl_) (void)hipFree(p);
  for (auto p : h_ctrl_) (void)hipHostFree(p);
  for (auto s : {ss_, gs_})
    if (s) (void)hipStreamDestroy(s);
}

DpCtrl DpFollower::run() {
  check_hip(hipSetDevice(L_->device()), "hipSetDevice");
  const DpGeometry g{S_->size(), L_->item_bytes(), L_->out_cols()};
  auto post_ctrl_recv = [&](int slot) {
    check_nccl(ncclRecv(d_ctrl_[slot], sizeof(DpCtrl), ncclUint8, 0, S_->get(), ss_), "ncclRecv(ctrl)");
    check_hip(hipMemcpyAsync(h_ctrl_[slot], d_ctrl_[slot], sizeof(DpCtrl), hipMemcpyDeviceToHost, ss_), "D2H ctrl");
    check_hip(hipEventRecord(ev_ctrl_[slot], ss_), "hipEventRecord");
  };
  (void)dp_follower_prologue();
  int slot = (int)(steps_ % nslots_);
  post_ctrl_recv(slot);
  for (;;) {
    if (!poll_event(ev_ctrl_[slot], 0)) throw std::runtime_error("DpFollower: control receive failed");
    const DpCtrl c = *h_ctrl_[slot];
    if (c.seq != seq_) throw std::runtime_error("DpFollower: control word out of sequence");
    ++seq_;
    if (c.cmd != DP_BATCH) {
      check_hip(hipStreamSynchronize(gs_), "drain gather");
      check_hip(hipStreamSynchronize(ss_), "drain scatter");
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
    check_hip(hipStreamWaitEvent(ss_, ev_free_[slot], 0), "wait slot free");
    for (const auto& m : msgs) {
      if (m.channel == DP_SCATTER && m.what == 1) {
        check_nccl(ncclRecv(din, m.bytes, ncclUint8, 0, S_->get(), ss_), "ncclRecv(shard)");
        check_hip(hipEventRecord(ev_in_[slot], ss_), "hipEventRecord");
      } else if (m.channel == DP_SCATTER && m.what == 0) {
        post_ctrl_recv(next);
      }
    }
    hipStream_t last = nullptr;
    if (L_->launch(slot, shard, ev_in_[slot], &last) != 0) throw std::runtime_error("DpFollower: launch failed");
    check_hip(hipEventRecord(ev_fw_[slot], last), "hipEventRecord");
    check_hip(hipStreamWaitEvent(gs_, ev_fw_[slot], 0), "wait forward");
    for (const auto& m : msgs)
      if (m.channel == DP_GATHER)
        check_nccl(ncclSend(dout, m.bytes, ncclUint8, 0, G_->get(), gs_), "ncclSend(logits)");
    check_hip(hipEventRecord(ev_free_[slot], gs_), "hipEventRecord");
    ++steps_;
    slot = next;
  }
}

}  // namespace kdl
