// RCCL over xGMI for data-parallel serving on one node (SURVEY.md §2.4 "comm.cpp", §2.8 C2/C3).
//
// One process per GPU. Rank 0 (the front-end) drives its native executor through DpLeader, a
// kdl_exec_backend that wraps rank 0's own HipExecBackend: per batch of world x shard images it
// H2Ds its own shard straight into its engine's input slot (the local forward starts at once)
// and the other shards into a send buffer, then posts the step of dp_schedule.h on two
// communicators -- SCATTER: control word + uint8 shard to every follower; GATHER: the
// followers' fp32 logits -- and D2Hs them behind its own. Followers (ranks >= 1) run
// DpFollower::run(), a C++ loop with the GIL released: receive the control word (it carries
// the per-rank bucket, so the follower picks the captured graph) and the shard into the
// engine's input slot, launch the stage-pipelined graphs, send the logits, and already post
// the next step's control receive. Steps stay in flight on `nslots` slots on both ends, as the
// single-GPU backend does.
//
// The RCCL library is the one torch loaded (same soname librccl.so.1, like libamdhip64), so
// our communicators live beside torch.distributed's in one RCCL instance.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>
#include <vector>

#include "dp_schedule.h"
#include "exec_backend.h"
#include "hip_backend.h"

namespace kdl {

std::string rccl_unique_id();                  // NCCL_UNIQUE_ID_BYTES opaque bytes (rank 0 creates)

class RcclComm {
 public:
  RcclComm(const std::string& id, int nranks, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;
  ncclComm_t get() const { return comm_; }
  int rank() const { return rank_; }
  int size() const { return size_; }
  void abort();                                // unblock every pending operation (a peer died)
  bool async_error() const;

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, size_, device_;
};

// Posts the given messages (all of one channel) as ncclSend / ncclRecv, one RCCL group per
// DpMsg::group value, in order. buf(msg) -> device pointer of that message.
template <class F>
ncclResult_t dp_post(const std::vector<DpMsg>& msgs, RcclComm& c, hipStream_t s, F buf) {
  size_t i = 0;
  while (i < msgs.size()) {
    const int g = msgs[i].group;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return r;
    for (; i < msgs.size() && msgs[i].group == g; ++i) {
      const DpMsg& m = msgs[i];
      r = m.send ? ncclSend(buf(m), m.bytes, ncclUint8, m.peer, c.get(), s)
                 : ncclRecv(buf(m), m.bytes, ncclUint8, m.peer, c.get(), s);
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return r;
      }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) return r;
  }
  return ncclSuccess;
}

class DpLeader {
 public:
  // local: rank 0's backend, built with max_batch = world x the largest rank bucket (its pinned
  // staging / logits hold the whole global batch) and one recipe per per-rank bucket
  DpLeader(HipExecBackend* local, RcclComm* scatter, RcclComm* gather, std::vector<int> rank_buckets,
           double timeout_s);
  ~DpLeader();
  DpLeader(const DpLeader&) = delete;
  DpLeader& operator=(const DpLeader&) = delete;
  const kdl_exec_backend* api() const { return &api_; }
  int world() const { return world_; }
  int issue(int slot, int bucket, int n_real);   // bucket = world x a rank bucket
  int complete(int slot, const float** out, kdl_device_times* t);
  int send_ctrl(int cmd, int version);           // DP_STOP / DP_RELOAD to every follower (synchronous)
  long steps() const { return seq_; }

 private:
  HipExecBackend* L_;
  RcclComm *S_, *G_;
  int world_;
  std::vector<int> buckets_;
  int max_shard_;
  double timeout_s_;
  hipStream_t cs_ = nullptr, ss_ = nullptr, gs_ = nullptr;   // follower-shard H2D, scatter, gather
  std::vector<uint8_t*> d_send_;
  std::vector<float*> d_gather_;
  std::vector<DpCtrl*> d_ctrl_, h_ctrl_;
  std::vector<hipEvent_t> ev_in_, ev_sent_, ev_gdone_;
  std::vector<int> slot_shard_;
  int seq_ = 0;
  bool broken_ = false;
  bool closed_ = false;                          // a DP_STOP / DP_RELOAD went out: no more batches
  std::mutex mu_;                                // issue() (executor thread) vs send_ctrl() (reload)
  kdl_exec_backend api_{};
  int wait(hipEvent_t e);                        // bounded wait (timeout_s_), aborts the comms on expiry
};

class DpFollower {
 public:
  DpFollower(HipExecBackend* local, RcclComm* scatter, RcclComm* gather);
  ~DpFollower();
  DpFollower(const DpFollower&) = delete;
  DpFollower& operator=(const DpFollower&) = delete;
  // serve rank 0's steps until a control word other than DP_BATCH arrives; returns it
  DpCtrl run();
  long steps() const { return steps_; }

 private:
  HipExecBackend* L_;
  RcclComm *S_, *G_;
  int nslots_;
  hipStream_t ss_ = nullptr, gs_ = nullptr;
  std::vector<DpCtrl*> d_ctrl_, h_ctrl_;
  std::vector<hipEvent_t> ev_ctrl_, ev_in_, ev_fw_, ev_free_;
  long steps_ = 0;
  int seq_ = 0;
};

}  // namespace kdl
