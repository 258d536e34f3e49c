// Native hybrid rollout loop (see rollout_loop.cc).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

#include "../rl/synth_env.h"

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
};

// Launch step 0 of every group, then for t < T and each group: wait for its step, step its envs
// (actions → newest frames, rewards, dones at row t), and launch its next step. Blocking; returns
// the episodes that finished as (return, length).
std::vector<std::pair<double, int64_t>> hybrid_rollout(const std::vector<RolloutGroup>& G, int64_t T);

}  // namespace hip
}  // namespace rmm
