#include "comm.h"

#include <cstring>
#include <stdexcept>

namespace kdl {

namespace {
void check_nccl(ncclResult_t r, const std::string& what) {
  if (r != ncclSuccess) throw std::runtime_error(what + ": " + ncclGetErrorString(r));
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

int rccl_gather(RcclComm& c, const void* send, void* recv, size_t bytes, hipStream_t stream) {
  if (!c.get()) return -1;
  if (c.size() == 1) return 0;
  if (ncclGroupStart() != ncclSuccess) return -1;
  ncclResult_t r = ncclSuccess;
  if (c.rank() == 0) {
    for (int p = 1; p < c.size() && r == ncclSuccess; ++p)
      r = ncclRecv(static_cast<uint8_t*>(recv) + bytes * p, bytes, ncclUint8, p, c.get(), stream);
  } else {
    r = ncclSend(send, bytes, ncclUint8, 0, c.get(), stream);
  }
  const ncclResult_t e = ncclGroupEnd();
  return r == ncclSuccess && e == ncclSuccess ? 0 : -1;
}

// the two class templates are instantiated once, here, for the HIP / RCCL platform
template class DpLeaderT<HipRcclPlatform>;
template class DpFollowerT<HipRcclPlatform>;

}  // namespace kdl
