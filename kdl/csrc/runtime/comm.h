// RCCL over xGMI for data-parallel serving on one node (SURVEY.md §2.4 "comm.cpp", §2.8 C2/C3).
//
// One process per GPU. Rank 0 (the front-end) drives its native executor through DpLeader, a
// kdl_exec_backend that wraps rank 0's own HipExecBackend; followers (ranks >= 1) run
// DpFollower::run(). The protocol, the slot pipelining and every bounded wait live in
// dp_core.h, written once against a platform policy: HipRcclPlatform below (HIP streams /
// events, hipMalloc'd buffers, ncclSend / ncclRecv on two communicators) is the production
// instance; dp_loop.h's LoopPlatform runs the SAME state machine over threads and host memory
// so CPU tests drive world 2/4/8, reload and rank death without GPUs.
//
// The RCCL library is the one torch loaded (same soname librccl.so.1, like libamdhip64), so
// our communicators live beside torch.distributed's in one RCCL instance.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "dp_core.h"
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

// gather of equal-size byte blocks to rank 0 on `stream` (rank r >= 1's block -> recv + r x bytes;
// rank 0's own block is NOT copied: the caller reads it where it is -- a 1 KB device-to-device
// hipMemcpyAsync there cost the bench 17 % at world 1, profiles/dist_path_r5.txt), posted directly on the caller's stream: no
// extra internal stream (torch.distributed's NCCL process group adds one per device), so a
// stage-pipelined bench rank keeps compute stages + H2D + comm within GPU_MAX_HW_QUEUES = 4.
int rccl_gather(RcclComm& c, const void* send, void* recv, size_t bytes, hipStream_t stream);

struct HipRcclPlatform {
  using Stream = hipStream_t;
  using Event = hipEvent_t;
  using Comm = RcclComm;
  using Local = HipExecBackend;

  static int ok(hipError_t e) { return e == hipSuccess ? 0 : -1; }
  static int nok(ncclResult_t r) { return r == ncclSuccess ? 0 : -1; }
  static int select(Local& l) { return ok(hipSetDevice(l.device())); }
  static Stream new_stream(Local&) {
    hipStream_t s;
    check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    return s;
  }
  static void free_stream(Stream s) { (void)hipStreamDestroy(s); }
  static int sync(Stream s) { return ok(hipStreamSynchronize(s)); }
  static Event new_event(Local&) {
    hipEvent_t e;
    check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  static void free_event(Event e) { (void)hipEventDestroy(e); }
  static int record(Event e, Stream s) { return ok(hipEventRecord(e, s)); }
  static int wait_event(Stream s, Event e) { return ok(hipStreamWaitEvent(s, e, 0)); }
  static int query(Event e) {
    const hipError_t q = hipEventQuery(e);
    return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : -1;
  }
  static void* dev_alloc(Local&, size_t n) {
    void* p = nullptr;
    check_hip(hipMalloc(&p, n), "hipMalloc");
    return p;
  }
  static void dev_free(Local&, void* p) { (void)hipFree(p); }
  static void* host_alloc(size_t n) {
    void* p = nullptr;
    check_hip(hipHostMalloc(&p, n, hipHostMallocDefault), "hipHostMalloc");
    return p;
  }
  static void host_free(void* p) { (void)hipHostFree(p); }
  static int h2d(void* d, const void* s, size_t n, Stream st) { return ok(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, st)); }
  static int d2h(void* d, const void* s, size_t n, Stream st) { return ok(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, st)); }
  static int group_start() { return nok(ncclGroupStart()); }
  static int group_end() { return nok(ncclGroupEnd()); }
  static int send(const void* b, size_t n, int peer, Comm& c, Stream s) {
    return c.get() ? nok(ncclSend(b, n, ncclUint8, peer, c.get(), s)) : -1;
  }
  static int recv(void* b, size_t n, int peer, Comm& c, Stream s) {
    return c.get() ? nok(ncclRecv(b, n, ncclUint8, peer, c.get(), s)) : -1;
  }
  static int rank(const Comm& c) { return c.rank(); }
  static int size(const Comm& c) { return c.size(); }
  static void abort(Comm& c) { c.abort(); }
  static bool comm_error(const Comm& c) { return c.async_error(); }
};

using DpLeader = DpLeaderT<HipRcclPlatform>;
using DpFollower = DpFollowerT<HipRcclPlatform>;

}  // namespace kdl
