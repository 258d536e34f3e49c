// Framework-owned RCCL communicator (see rccl_comm.cc).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>

#include "common.h"

namespace rmm::hip {

int rccl_load(const std::string& path);  // returns the RCCL version code
std::string rccl_unique_id();            // 128 opaque bytes, made by rank 0

class RcclComm {
 public:
  RcclComm(const std::string& uid, int nranks, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // enqueue on `stream` (legal inside HIP stream capture); in-place when send == recv
  void AllReduce(uint64_t send, uint64_t recv, uint64_t count, int dtype, int op, uint64_t stream);
  void Broadcast(uint64_t send, uint64_t recv, uint64_t count, int dtype, int root, uint64_t stream);
  std::string AsyncError();
  void Abort();
  void Destroy();
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
};

}  // namespace rmm::hip
