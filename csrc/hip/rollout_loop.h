// Native hybrid rollout loop (see rollout_loop.cc).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

#include "../rl/synth_env.h"
#include "kernels.h"

namespace rmm {
namespace hip {

struct RolloutGroup {
  hipGraphExec_t exec = nullptr;  // one policy step (instantiated HIP graph)
  hipStream_t stream = nullptr;
  rl::SynthAtariState env;        // the group's native envs
  const int64_t* act = nullptr;   // pinned host [n]: the graph stores the step's actions here
  uint8_t* new_frames = nullptr;  // pinned host [n][84*84]: the graph reads the newest frames from here
  float* rew = nullptr;           // pinned host [T][n]
  float* done = nullptr;          // pinned host [T][n]
  double* ep_rew = nullptr;       // [n] running episode returns
  int64_t* ep_len = nullptr;      // [n] running episode lengths
  // step gate (optional): the graph starts with a device-side wait until *release passes its
  // sequence number, so step t+1 is launched BEFORE step t's env step and only released after it
  int64_t* release = nullptr;     // pinned host release counter (null: no gate)
  // the envs are stepped in `gate_parts` ranges with a release after each (the counter advances
  // gate_parts per step), and each K10x workgroup waits for its own range only
  int gate_parts = 1;
  // direct launches (optional): the policy step as its three kernel launches (K10 push → K13s →
  // K16 with the step advance) from this thread instead of a graph launch; `exec` is then unused
  const RolloutServerArgs* direct = nullptr;
  unsigned int* k16_done = nullptr;  // K16's zero-initialised completion counter (advances t / ctr)
  // completion word (direct launches, optional): pinned host int64 and its device view; K16 stores
  // row + 1 there with a system-scope release after the step's actions, and the loop polls it
  // instead of recording / waiting on an event
  int64_t* host_seq = nullptr;
  int64_t* host_seq_dev = nullptr;
};

// host µs per empty-kernel launch, per hipEventRecord, per 200x512 launch + error check (n of each)
std::vector<double> launch_overhead_probe(int n, hipStream_t stream);
// One policy step of `a` as direct launches on `stream` (the kernels a captured step graph holds).
void rollout_step_direct(const RolloutServerArgs& a, unsigned int* k16_done, hipStream_t stream,
                         int64_t* host_seq_dev = nullptr, int64_t gate_want = 0, int gate_parts = 1);

// Launch step 0 of every group, then for t < T and each group: wait for its step (poll when
// `spin`), step its envs (actions → newest frames, rewards, dones at row t) on `threads` CPU threads,
// and launch its next step. Blocking; returns the episodes that finished as (return, length).
std::vector<std::pair<double, int64_t>> hybrid_rollout(const std::vector<RolloutGroup>& G, int64_t T,
                                                       int threads = 1, bool spin = false);
// µs the last hybrid_rollout call spent {waiting for policy steps, in env steps, launching steps}
std::vector<double> hybrid_rollout_phases();

// The same loop over ONE group with the K21 persistent rollout server: one kernel launch for the
// fragment; per step the host releases the step (`go`), waits for the server's `done_seq` (spin,
// bounded), steps the envs. `a` carries the weights / buffers; its sync words are filled in here.
// Throws (after aborting and draining the kernel) on a server timeout or a host-side failure.
std::vector<std::pair<double, int64_t>> hybrid_rollout_server(const RolloutGroup& g, RolloutServerArgs a, int64_t T,
                                                              int threads = 1, double wait_timeout_s = 30.0);

}  // namespace hip
}  // namespace rmm
