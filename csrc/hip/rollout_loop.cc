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

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <string>
#include <chrono>
#include <stdexcept>
#include <thread>
#include <utility>
#include <vector>

#include "../rl/synth_env.h"
#include "common.h"
#include "rollout_loop.h"

namespace rmm {
namespace hip {

namespace {

inline void cpu_relax() { __builtin_ia32_pause(); }

// Helper threads that split each env step by env range (rollout_env_threads > 1). They spin on a
// job sequence number for the duration of one hybrid_rollout call (a fragment, a few ms), so handing
// out a step costs two cache-line transfers instead of a futex wake-up. For the synthetic env (4 µs
// per 50-env step) this measured neutral; it is meant for envs whose step dominates.
class EnvThreads {
 public:
  explicit EnvThreads(int n) : n_(std::max(0, n - 1)) {
    for (int k = 0; k < n_; k++) th_.emplace_back([this, k] { run(k + 1); });
  }
  ~EnvThreads() {
    stop_.store(true, std::memory_order_release);
    seq_.fetch_add(1, std::memory_order_acq_rel);
    for (auto& t : th_) t.join();
  }
  // env step of group g at row t in `parts` consecutive env ranges on the calling thread, `after(p)`
  // once range p is written (the gated K10x workgroups of that range may start reading its frames).
  // With helper threads the ranges are not ordered: one full step, then every after(p).
  template <typename F>
  void step_parts(const RolloutGroup& g, uint64_t step, int64_t t, int parts, F&& after) {
    if (n_ > 0 || parts <= 1) {
      this->step(g, step, t);
      for (int p = 0; p < std::max(1, parts); p++) after(p);
      return;
    }
    const int64_t n = g.env.n;
    for (int p = 0; p < parts; p++) {
      const int64_t i0 = n * p / parts, i1 = n * (p + 1) / parts;
      rl::synth_step_range(g.env, step, i0, i1, g.act, g.new_frames, false, g.rew + t * n, g.done + t * n);
      after(p);
    }
  }
  // env step of group g at row t, split over all threads (the caller takes part)
  void step(const RolloutGroup& g, uint64_t step, int64_t t) {
    job_ = Job{&g, step, t};
    if (n_ == 0) {
      work(0);
      return;
    }
    done_.store(0, std::memory_order_relaxed);
    seq_.fetch_add(1, std::memory_order_release);
    work(0);
    while (done_.load(std::memory_order_acquire) != n_) cpu_relax();
  }

 private:
  struct Job {
    const RolloutGroup* g;
    uint64_t step;
    int64_t t;
  };
  void work(int k) {
    const RolloutGroup& g = *job_.g;
    const int64_t n = g.env.n, parts = n_ + 1;
    const int64_t i0 = n * k / parts, i1 = n * (k + 1) / parts;
    rl::synth_step_range(g.env, job_.step, i0, i1, g.act, g.new_frames, false, g.rew + job_.t * n, g.done + job_.t * n);
  }
  void run(int k) {
    uint64_t seen = seq_.load(std::memory_order_acquire);
    for (;;) {
      uint64_t s;
      while ((s = seq_.load(std::memory_order_acquire)) == seen) cpu_relax();
      seen = s;
      if (stop_.load(std::memory_order_acquire)) return;
      work(k);
      done_.fetch_add(1, std::memory_order_acq_rel);
    }
  }
  int n_;
  std::vector<std::thread> th_;
  Job job_{};
  alignas(64) std::atomic<uint64_t> seq_{0};
  alignas(64) std::atomic<int> done_{0};
  alignas(64) std::atomic<bool> stop_{false};
};

// Wait for a step's event. `spin`: poll for up to kSpinUs (a policy step takes ~30-40 µs; a blocking
// wait adds a wake-up), then block — on a host whose CPUs are shared, an unbounded poll that loses its
// core costs more than it saves (measured outliers, profiles/native_rollout_r3.txt).
constexpr double kSpinUs = 150.0;
void wait_event(hipEvent_t e, bool spin) {
  if (spin) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; k++) {
      const hipError_t r = hipEventQuery(e);
      if (r == hipSuccess) return;
      if (r != hipErrorNotReady) RMM_HIP_CHECK(r);
      cpu_relax();
      if ((k & 15) == 15 &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kSpinUs)
        break;
    }
  }
  RMM_HIP_CHECK(hipEventSynchronize(e));
}

using Clock = std::chrono::steady_clock;
double g_phase_us[3] = {0, 0, 0};  // last call: time waiting for steps, in env steps, in launches

inline double us_since(Clock::time_point a) {
  return std::chrono::duration<double, std::micro>(Clock::now() - a).count();
}

}  // namespace

std::vector<double> hybrid_rollout_phases() { return {g_phase_us[0], g_phase_us[1], g_phase_us[2]}; }

namespace {
__global__ void k_launch_probe(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}
}  // namespace

std::vector<double> launch_overhead_probe(int n, hipStream_t stream) {
  // host µs per {empty kernel launch, hipEventRecord, rollout-step-sized kernel argument block launch}
  hipEvent_t e;
  RMM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::vector<double> out;
  auto t0 = Clock::now();
  for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_launch_probe, dim3(1), dim3(64), 0, stream, nullptr);
  out.push_back(us_since(t0) / n);
  RMM_HIP_CHECK(hipStreamSynchronize(stream));
  t0 = Clock::now();
  for (int i = 0; i < n; i++) RMM_HIP_CHECK(hipEventRecord(e, stream));
  out.push_back(us_since(t0) / n);
  RMM_HIP_CHECK(hipStreamSynchronize(stream));
  t0 = Clock::now();
  for (int i = 0; i < n; i++) {
    hipLaunchKernelGGL(k_launch_probe, dim3(200), dim3(512), 0, stream, nullptr);
    RMM_HIP_CHECK(hipGetLastError());
  }
  out.push_back(us_since(t0) / n);
  RMM_HIP_CHECK(hipStreamSynchronize(stream));
  RMM_HIP_CHECK(hipEventDestroy(e));
  return out;
}

void rollout_step_direct(const RolloutServerArgs& a, unsigned int* k16_done, hipStream_t stream,
                         int64_t* host_seq_dev, int64_t gate_want, int gate_parts) {
  // ctr_t = {rng counter, rollout row}: K10 stores row *t, K16 samples with the counter and advances both
  if (a.x3) {  // fp32 policy: the split-bf16 twins (K10x push -> K13x -> K16x)
    const X3Out h2{a.h2, a.h2lo};
    x3_trunk_fwd_push(a.stack, a.nf, a.rows, a.ctr_t + 1, a.B, X3In{a.W1, a.W1lo}, a.w1s, X3In{a.b1, a.b1lo},
                      X3In{a.W2, a.W2lo}, a.w2s, X3In{a.b2, a.b2lo}, h2, stream, a.gate, gate_want, a.gate_err,
                      gate_parts, a.gate_timeout_ms);
    if (a.fused_heads) {
      x3_dense_heads_sample(X3In{a.h2, a.h2lo}, X3In{a.Wd, a.Wdlo}, a.B, 3872, a.hpart, a.S, X3In{a.bd, a.bdlo},
                            X3In{a.Wh, a.Whlo}, X3In{a.bh, a.bhlo}, a.ctr_t + 1, a.ctr_t, a.seed, a.act, a.logp, a.vf,
                            a.lout, a.act_now, a.A1, stream, k16_done, host_seq_dev);
    } else {
      x3_dense_fwd_part(X3In{a.h2, a.h2lo}, X3In{a.Wd, a.Wdlo}, a.B, 3872, 256, a.hpart, a.S, stream);
      x3_heads_sample(a.hpart, a.S, X3In{a.bd, a.bdlo}, X3In{a.Wh, a.Whlo}, X3In{a.bh, a.bhlo}, a.ctr_t + 1, a.ctr_t,
                      a.seed, a.act, a.logp, a.vf, a.lout, a.act_now, a.B, a.A1, stream, k16_done, host_seq_dev);
    }
    return;
  }
  nature_trunk_fwd_push(a.stack, a.nf, a.rows, a.ctr_t + 1, a.B, a.W1, a.w1s, a.b1, a.W2, a.w2s, a.b2, a.h2, stream);
  dense_fwd_part(a.h2, a.Wd, a.B, 3872, 256, a.hpart, a.S, stream);
  dense_heads_sample(nullptr, a.Wh, a.bh, a.ctr_t + 1, a.ctr_t, a.seed, a.act, a.logp, a.vf, a.lout, a.act_now, a.B,
                     a.A1, stream, k16_done, a.hpart, a.S, a.bd, host_seq_dev);
}

namespace {
// Poll a step's completion word (pinned host memory written by K16 with a system-scope release): the
// CPU sees the step ~1 µs after its last store instead of after an event's interrupt + wake-up.
// Bounded: a step that never completes (device fault, hung kernel) fails the fragment after `limit_s`.
void wait_seq(const int64_t* seq, int64_t want, double limit_s = 10.0) {
  if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) >= want) return;
  const auto t0 = Clock::now();
  for (int k = 0;; k++) {
    for (int i = 0; i < 64; i++) {
      if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) >= want) return;
      cpu_relax();
    }
    if ((k & 63) == 63) {
      if (std::chrono::duration<double>(Clock::now() - t0).count() > limit_s)
        throw std::runtime_error("hybrid_rollout: a policy step did not complete (completion word timeout)");
      std::this_thread::yield();
    }
  }
}
}  // namespace

std::vector<std::pair<double, int64_t>> hybrid_rollout(const std::vector<RolloutGroup>& G, int64_t T, int threads,
                                                       bool spin) {
  if (T <= 0 || G.empty()) return {};
  for (const auto& g : G)
    if ((!g.exec && !g.direct) || (g.direct && !g.k16_done) || !g.env.pools || !g.act || !g.new_frames || !g.rew ||
        !g.done || !g.ep_rew || !g.ep_len)
      throw std::invalid_argument("hybrid_rollout: incomplete group");
  // two events per group: with the gate, steps t and t+1 are in flight together
  std::vector<hipEvent_t> ev(2 * G.size(), nullptr);
  std::vector<std::pair<double, int64_t>> completed;
  auto launch = [&](size_t i, int64_t step) {
    if (G[i].direct) {
      // gated direct launches: step s waits in K10x until the release counter reaches s + 1
      // step s opens at release count s P + 1 (P = gate_parts; range p of it at s P + 1 + p)
      const int P = G[i].release ? std::max(1, G[i].gate_parts) : 1;
      rollout_step_direct(*G[i].direct, G[i].k16_done, G[i].stream, G[i].host_seq_dev,
                          G[i].release ? step * P + 1 : 0, P);
      if (G[i].host_seq) return;  // completion comes through the host word
    } else {
      RMM_HIP_CHECK(hipGraphLaunch(G[i].exec, G[i].stream));
    }
    RMM_HIP_CHECK(hipEventRecord(ev[2 * i + (step & 1)], G[i].stream));
  };
  // test hook: a host that stalls before opening each gate (RMM_TEST_GATE_DELAY_US), to exercise the gate's
  // timeout and the worker's ungated re-run (tests/test_rllib_runtime_gpu.py)
  const long delay_us = [] {
    const char* e = std::getenv("RMM_TEST_GATE_DELAY_US");
    return e ? std::atol(e) : 0L;
  }();
  auto release = [&](size_t i, int64_t k = 1) {  // frames of the next step (range) are written: open its gate
    if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
    __atomic_fetch_add(G[i].release, k, __ATOMIC_RELEASE);
  };
  try {
    EnvThreads pool(std::max(1, std::min(threads, 16)));
    for (auto& e : ev) RMM_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (size_t i = 0; i < G.size(); i++) {
      if (G[i].host_seq) __atomic_store_n(G[i].host_seq, int64_t(0), __ATOMIC_RELEASE);  // rows restart at 0
      // the in-kernel gate of direct launches counts from 0 each fragment (nothing is in flight here)
      if (G[i].direct && G[i].release) __atomic_store_n(G[i].release, int64_t(0), __ATOMIC_RELEASE);
      launch(i, 0);
      if (G[i].release) {
        release(i, G[i].direct ? std::max(1, G[i].gate_parts) : 1);  // step 0's frames are already staged
        if (T > 1) launch(i, 1);     // step 1 waits on the device for its frames
      }
    }
    double ph[3] = {0, 0, 0};
    for (int64_t t = 0; t < T; t++) {
      for (size_t i = 0; i < G.size(); i++) {  // group i's env step overlaps the other groups' policy steps
        const RolloutGroup& g = G[i];
        auto c0 = Clock::now();
        if (g.host_seq)
          wait_seq(g.host_seq, t + 1);  // step t (row t) stored its actions, then row + 1 here
        else
          wait_event(ev[2 * i + (t & 1)], spin);  // step t's actions are in g.act
        ph[0] += us_since(c0);
        c0 = Clock::now();
        const int P = g.release && g.direct ? std::max(1, g.gate_parts) : 1;
        if (g.release && P > 1) {  // open step t+1 range by range as the envs are stepped
          pool.step_parts(g, g.env.step[0]++, t, P, [&](int) {
            if (t + 1 < T) release(i);
          });
        } else {
          pool.step(g, g.env.step[0]++, t);
        }
        rl::episode_update(g.env.n, g.rew + t * g.env.n, g.done + t * g.env.n, g.ep_rew, g.ep_len, completed);
        ph[1] += us_since(c0);
        c0 = Clock::now();
        if (g.release) {
          // gate: step t+1 is already enqueued (its launch latency hid behind step t); open it, then
          // enqueue step t+2 while step t+1 runs
          if (t + 1 < T && P == 1) release(i);
          if (t + 2 < T) launch(i, t + 2);
        } else if (t + 1 < T) {
          launch(i, t + 1);
        }
        ph[2] += us_since(c0);
      }
    }
    for (int k = 0; k < 3; k++) g_phase_us[k] = ph[k];
  } catch (...) {
    for (const auto& g : G) (void)hipStreamSynchronize(g.stream);  // no launch may outlive the buffers
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    throw;
  }
  for (auto e : ev) RMM_HIP_CHECK(hipEventDestroy(e));
  return completed;
}

namespace {
// Host words the rollout server synchronises through (pinned, device-mapped) and its device words,
// allocated once per process (one hybrid worker runs one fragment at a time).
struct ServerSync {
  int64_t* host = nullptr;       // [0] go, [8] done_seq, [16] err  (separate 64-B lines)
  int64_t* host_dev = nullptr;   // device view of `host`
  unsigned int* bar = nullptr;   // 10 device words
  int64_t* err_dev = nullptr;
};
ServerSync& server_sync() {
  static ServerSync s;
  static std::once_flag once;
  std::call_once(once, [] {
    RMM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s.host), 256, hipHostMallocMapped));
    RMM_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.host_dev), s.host, 0));
    void* d = nullptr;
    RMM_HIP_CHECK(hipMalloc(&d, 128));
    s.bar = static_cast<unsigned int*>(d);  // 10 counters (40 B)
    s.err_dev = reinterpret_cast<int64_t*>(static_cast<char*>(d) + 64);
  });
  return s;
}
}  // namespace

std::vector<std::pair<double, int64_t>> hybrid_rollout_server(const RolloutGroup& g, RolloutServerArgs a, int64_t T,
                                                              int threads, double wait_timeout_s) {
  if (T <= 0) return {};
  if (!g.env.pools || !g.act || !g.new_frames || !g.rew || !g.done || !g.ep_rew || !g.ep_len)
    throw std::invalid_argument("hybrid_rollout_server: incomplete group");
  ServerSync& sy = server_sync();
  volatile int64_t* go = sy.host;
  volatile int64_t* done_seq = sy.host + 8;
  volatile int64_t* err = sy.host + 16;
  *go = 0;
  *done_seq = 0;
  *err = 0;
  a.T = T;
  a.go = sy.host_dev;
  a.done_seq = sy.host_dev + 8;
  a.err_host = sy.host_dev + 16;
  a.bar = sy.bar;
  a.err_dev = sy.err_dev;
  std::vector<std::pair<double, int64_t>> completed;
  rollout_server_launch(a, g.stream);
  double ph[3] = {0, 0, 0};
  try {
    EnvThreads pool(std::max(1, std::min(threads, 16)));
    for (int64_t t = 0; t < T; t++) {
      auto c0 = Clock::now();
      __atomic_store_n(const_cast<int64_t*>(go), t + 1, __ATOMIC_RELEASE);  // step t's frames are staged
      for (uint64_t k = 0;; k++) {  // the server stores step t's actions, then done_seq = t + 1
        if (__atomic_load_n(const_cast<int64_t*>(done_seq), __ATOMIC_ACQUIRE) >= t + 1) break;
        cpu_relax();
        if ((k & 1023) == 1023) {
          if (*err) throw std::runtime_error("rollout server error " + std::to_string(*err));
          if (us_since(c0) > wait_timeout_s * 1e6) throw std::runtime_error("rollout server: step timed out");
        }
      }
      ph[0] += us_since(c0);
      c0 = Clock::now();
      pool.step(g, g.env.step[0]++, t);
      rl::episode_update(g.env.n, g.rew + t * g.env.n, g.done + t * g.env.n, g.ep_rew, g.ep_len, completed);
      ph[1] += us_since(c0);
    }
    RMM_HIP_CHECK(hipStreamSynchronize(g.stream));
    if (*err) throw std::runtime_error("rollout server error " + std::to_string(*err));
  } catch (...) {
    __atomic_store_n(const_cast<int64_t*>(go), int64_t(-1), __ATOMIC_RELEASE);  // abort: every wait exits
    (void)hipStreamSynchronize(g.stream);
    throw;
  }
  for (int k = 0; k < 3; k++) g_phase_us[k] = ph[k];
  return completed;
}

}  // namespace hip
}  // namespace rmm
