// Peer-memory all-reduce over xGMI for co-located ranks (one process per GPU, or several
// processes sharing one GPU in the 1-GPU rehearsal). See peer_allreduce.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

namespace rmm::hip {

constexpr int kPeerMaxRanks = 16;

// How many workgroups of the peer kernels one CU holds at once (hipOccupancyMaxActiveBlocksPerMultiprocessor)
// and the device's CU count: a launch whose workgroups wait on their peers' same-index workgroups must have
// ALL of them resident together (with every rank sharing the GPU, and beside concurrent kernels), so the
// communicators derive their workgroup counts from this instead of a constant.
struct PeerOccupancy {
  int cus;
  int allreduce_per_cu;
  int zero1_per_cu;
};
PeerOccupancy PeerKernelOccupancy(int device);

class PeerAllReduce {
 public:
  // `cap_bytes`: largest payload one kernel reduces (larger calls are split into several launches);
  // `nblocks`: workgroups per launch (fixed for the communicator's lifetime: every launch uses all of
  // them, which is what lets the staging buffers be reused after two launches, see the .hip file).
  PeerAllReduce(int rank, int world, int device, uint64_t cap_bytes, int nblocks, double timeout_s);
  ~PeerAllReduce();
  PeerAllReduce(const PeerAllReduce&) = delete;
  PeerAllReduce& operator=(const PeerAllReduce&) = delete;

  // 2 x 64-byte hipIpcMemHandle_t (data region, signal region) to publish to the peers
  std::string Handles() const;
  // open every peer's regions (handles[r] for r != rank is mapped; handles[rank] is ignored)
  void Open(const std::vector<std::string>& handles);
  // in-place sum of `count` elements (dtype 0 = bf16, 1 = fp32) on `stream`; legal inside capture.
  // algo: 0 = auto, 1 = one-shot, 2 = two-shot
  void AllReduce(uint64_t buf, uint64_t count, int dtype, uint64_t stream, int algo);
  // ZeRO-1 step in ONE launch per `cap / 4` elements: reduce-scatter the gradient (dtype 0 = bf16, 1 =
  // fp32; fp32 sum in rank order, bf16 gradients rounded once as AllReduce does), K6's Adam on the
  // chunk this rank owns (master / m1 / m2 and the bf16 weight planes), all-gather of the updated fp32
  // masters; every rank re-derives the weight planes from the gathered masters with the owner's
  // rounding, so weights and masters are bit-identical everywhere; m1 / m2 are current on the owner
  // only (MaskUnowned + AllReduce replicates them). Counters as adam_flat: the step from step_ctr,
  // `bump` advanced by the last launch (ticket `done`, or parity `bump_next`); bump = null: no advance.
  struct AdamArgs {
    float* master;
    float* m1;
    float* m2;
    void* whi;  // bf16 weights (hi plane)
    void* wlo;  // optional split-pair lo plane
    const float* hp;
    float grad_scale;
    const int64_t* step_ctr;
    int64_t* bump;
    int nbump;
    uint32_t* done;
    int64_t* bump_next;
  };
  void AllReduceAdam(uint64_t grad, uint64_t count, int dtype, uint64_t stream, const AdamArgs& z);
  // zero the fp32 `buf[0, count)` elements this rank does NOT own under AllReduceAdam(count, dtype)
  void MaskUnowned(uint64_t buf, uint64_t count, int dtype, uint64_t stream);
  // 0 = healthy; otherwise 1 + the rank whose flag timed out (+ block in the upper bits)
  int64_t Error() const;
  void ClearError();
  uint64_t launches() const { return launches_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  int nblocks() const { return nblocks_; }
  uint64_t cap_bytes() const { return cap_; }
  bool uncached_signals() const { return sig_uncached_; }
  int alloc_attempts() const { return alloc_attempts_; }
  void set_timeout(double s) { timeout_ticks_ = uint64_t(s > 0 ? s * 1e8 : 1e8); }
  void Close();

 private:
  int rank_, world_, device_, nblocks_;
  uint64_t cap_;
  uint64_t timeout_ticks_;
  char* data_ = nullptr;       // [in0 | in1 | red0 | red1], cap bytes each (exported)
  uint64_t* sig_ = nullptr;    // flags [2 phases][nblocks][kPeerMaxRanks] (exported)
  uint64_t* epochs_ = nullptr; // per-block epoch counters (local)
  int64_t* err_host_ = nullptr;  // mapped pinned host word the kernel reports timeouts to
  int64_t* err_dev_ = nullptr;
  bool sig_uncached_ = false;
  int alloc_attempts_ = 0;
  bool open_ = false;
  char* peer_data_[kPeerMaxRanks] = {};
  uint64_t* peer_sig_[kPeerMaxRanks] = {};
  uint64_t launches_ = 0;
};

}  // namespace rmm::hip
