// Native core of the synthetic Atari vector env (CPUSyntheticAtariVectorEnv, rllib/env.py).
//
// Reference role: the emulator behind a RolloutWorker's vector env — ALE is C++ under gym's
// Python wrapper (rllib/env/vector_env.py, rllib/env/wrappers/atari_wrappers.py). Here a step of
// n envs is one call: per env, pick a pooled 84x84 frame (the pool is pre-rolled per action, so the
// action shifts the image), append it to the env's frame stack (or emit only the newest frame when
// the consumer keeps the stacks in HBM), sparse Bernoulli(0.05) reward, truncation at episode_len.
// All randomness comes from a counter-based hash of (seed, global step, env), so the numpy
// fallback in env.py reproduces the native stream exactly.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace rmm {
namespace rl {

constexpr int64_t kFrameHW = 84 * 84;
constexpr int64_t kPoolFrames = 64;
constexpr uint32_t kRewardThresh = 838861;  // P(reward) = 0.05 over 24 hash bits

struct SynthAtariState {
  const uint8_t* pools = nullptr;  // [num_actions][64][84*84]: the frame pool pre-rolled per action
  int64_t* t = nullptr;            // [n] episode step counters
  uint64_t* step = nullptr;        // [1] global step counter (position in the random stream)
  uint64_t seed = 0;
  int64_t n = 0, num_actions = 4, episode_len = 1000;
};

inline uint64_t mix64(uint64_t seed, uint64_t step, uint64_t env) {
  uint64_t z = seed ^ (step * 0x9E3779B97F4A7C15ull) ^ ((env + 1) * 0xD1B54A32D192ED03ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Envs [i0, i1) of one step at random-stream position `step` (threads split a step by env range).
// act: [n] int64 (taken mod num_actions). stacks = false: out is [n][84*84] and receives each env's
// NEWEST frame only; stacks = true: out is [n][4][84*84], shifted by one frame in place with the
// newest appended. rew / done: [n] float (0/1).
inline void synth_step_range(const SynthAtariState& s, uint64_t step, int64_t i0, int64_t i1, const int64_t* act,
                             uint8_t* out, bool stacks, float* rew, float* done) {
  for (int64_t i = i0; i < i1; i++) {
    int64_t a = act[i] % s.num_actions;
    if (a < 0) a += s.num_actions;
    const uint64_t h = mix64(s.seed, step, uint64_t(i));
    const uint8_t* src = s.pools + (a * kPoolFrames + int64_t(h & 63)) * kFrameHW;
    if (stacks) {
      uint8_t* st = out + i * 4 * kFrameHW;
      std::memmove(st, st + kFrameHW, 3 * kFrameHW);
      std::memcpy(st + 3 * kFrameHW, src, kFrameHW);
    } else {
      std::memcpy(out + i * kFrameHW, src, kFrameHW);
    }
    rew[i] = uint32_t((h >> 32) & 0xFFFFFFu) < kRewardThresh ? 1.f : 0.f;
    const bool d = ++s.t[i] >= s.episode_len;
    if (d) s.t[i] = 0;
    done[i] = d ? 1.f : 0.f;
  }
}

// One step of all n envs (advances the random-stream position).
inline void synth_step(const SynthAtariState& s, const int64_t* act, uint8_t* out, bool stacks, float* rew,
                       float* done) {
  synth_step_range(s, s.step[0]++, 0, s.n, act, out, stacks, rew, done);
}

// Episode bookkeeping of a rollout worker after a step: running return / length per env, and the
// finished episodes as (return, length).
inline void episode_update(int64_t n, const float* rew, const float* done, double* ep_rew, int64_t* ep_len,
                           std::vector<std::pair<double, int64_t>>& completed) {
  for (int64_t i = 0; i < n; i++) {
    ep_rew[i] += rew[i];
    ep_len[i] += 1;
    if (done[i] != 0.f) {
      completed.emplace_back(ep_rew[i], ep_len[i]);
      ep_rew[i] = 0.0;
      ep_len[i] = 0;
    }
  }
}

}  // namespace rl
}  // namespace rmm
