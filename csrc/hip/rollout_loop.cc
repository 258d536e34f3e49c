// Native rollout loop of a hybrid rollout worker (rllib/evaluation/gpu_rollout_worker.py:
// HybridRolloutWorker) over native synthetic Atari envs.
//
// Reference role: the sampler loop of rllib/evaluation/sampler.py / rollout_worker.py — step the
// vector env, run the policy, record the transition — which the reference drives from Python with
// the policy on the worker's GPU (num_gpus_per_worker > 0). MI355X design: every policy step is ONE
// HIP-graph launch (K10 trunk reading the envs' newest frames straight from mapped pinned memory →
// K13s → K16 sampling, actions stored into mapped pinned memory), and the envs are split into
// groups that are double-buffered (group A's env step on the CPU overlaps group B's policy step on
// the GPU). With the whole T-step loop here, a group step costs an event wait, the native env step
// and a graph launch — no Python, no per-step torch wrappers — so the loop runs at the GPU's pace.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <utility>
#include <vector>

#include "../rl/synth_env.h"
#include "common.h"
#include "rollout_loop.h"

namespace rmm {
namespace hip {

std::vector<std::pair<double, int64_t>> hybrid_rollout(const std::vector<RolloutGroup>& G, int64_t T) {
  if (T <= 0 || G.empty()) return {};
  for (const auto& g : G)
    if (!g.exec || !g.env.pools || !g.act || !g.new_frames || !g.rew || !g.done || !g.ep_rew || !g.ep_len)
      throw std::invalid_argument("hybrid_rollout: incomplete group");
  std::vector<hipEvent_t> ev(G.size(), nullptr);
  std::vector<std::pair<double, int64_t>> completed;
  auto launch = [&](size_t i) {
    RMM_HIP_CHECK(hipGraphLaunch(G[i].exec, G[i].stream));
    RMM_HIP_CHECK(hipEventRecord(ev[i], G[i].stream));
  };
  try {
    for (auto& e : ev) RMM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (size_t i = 0; i < G.size(); i++) launch(i);
    for (int64_t t = 0; t < T; t++) {
      for (size_t i = 0; i < G.size(); i++) {  // group i's env step overlaps the other groups' policy steps
        const RolloutGroup& g = G[i];
        RMM_HIP_CHECK(hipEventSynchronize(ev[i]));  // step t's actions are in g.act
        float* rew = g.rew + t * g.env.n;
        float* done = g.done + t * g.env.n;
        rl::synth_step(g.env, g.act, g.new_frames, false, rew, done);
        rl::episode_update(g.env.n, rew, done, g.ep_rew, g.ep_len, completed);
        if (t + 1 < T) launch(i);
      }
    }
  } catch (...) {
    for (const auto& g : G) (void)hipStreamSynchronize(g.stream);  // no launch may outlive the buffers
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    throw;
  }
  for (auto e : ev) RMM_HIP_CHECK(hipEventDestroy(e));
  return completed;
}

}  // namespace hip
}  // namespace rmm
