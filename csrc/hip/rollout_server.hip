// K21 — persistent rollout server: a hybrid rollout worker's whole T-step policy loop in ONE launch.
//
// Role parity: the sampler loop of rllib/evaluation/sampler.py / rollout_worker.py (step the vector
// env, run the policy, record the transition) with the policy on the worker's GPU
// (num_gpus_per_worker > 0). The graph-per-step design (rollout_loop.cc: event wait → CPU env step →
// hipGraphLaunch of K10 push → K13s → K16) pays, per env step, a graph launch, three kernel
// boundaries and a completion signal — ~20 µs of the ~50 µs step with the GPU idle
// (profiles/native_rollout_r3.txt). Here the kernel stays resident for the fragment and talks to
// the host through words in pinned, device-mapped host memory:
//
//   host:  env step t-1 → newest frames → go = t+1 ─────────────┐            ┌→ env step t ...
//   GPU:   ...wait go ≥ t+1 → A: K10 trunk per env (frame stack shift + row t store, u8 frame from
//          host memory) ─grid barrier─ B: K13s split-K dense partials ─grid barrier─ C: K16 heads +
//          Gumbel sampling (actions → host memory, rollout-row stores) → done_seq = t+1 ┘
//
// Phases reuse the standalone kernels' device code (trunk_device.h, dense_device.h) with the same
// weights, split-K slicing and sampling counters, so a fragment is bit-identical to the graph path.
// Weights are staged into LDS once per fragment. Grid: one workgroup per CU (G <= #CUs, G >= B);
// workgroup b < B owns env b in phase A; phase B spreads the K13s units over every wave; phase C
// uses ceil(B / 8) workgroups (one wave per env row).
//
// Safety: every wait is bounded (s_memrealtime, 100 MHz): the host's `go` (also -1 = abort), the
// grid barriers; a timeout records an error code into a device word and a mapped host word and
// every workgroup leaves the kernel at its next wait, so the grid always drains. The host side
// (rollout_loop.cc: hybrid_rollout_server) bounds its own wait for `done_seq` the same way and
// aborts the kernel (go = -1) on any host-side failure before synchronising.
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "common.h"
#include "dense_device.h"
#include "kernels.h"
#include "trunk_device.h"

namespace rmm {
namespace hip {
namespace server {

using trunk::C0;
using trunk::C1;
using trunk::C2;
using trunk::FrameRegs;
using trunk::H0;
using trunk::NP2;

constexpr int NT = 512;
constexpr int KDENSE = 11 * 11 * 32;  // 3872: trunk output width = dense input width

struct Args {
  const unsigned short* W1;
  trunk::WStrides w1;
  const unsigned short* b1;
  const unsigned short* W2;
  trunk::WStrides w2;
  const unsigned short* b2;
  const unsigned short* Wd;  // dense [256, 3872] row-major
  const unsigned short* bd;
  const unsigned short* Wh;  // heads [A1, 256]
  const unsigned short* bh;
  int64_t B, T;
  int S;                     // K13s slices (dense_fwd_part_slices(B, 3872, 256))
  uint32_t seed;
  uint8_t* stack;            // [B, 4, 84, 84] device frame stacks (shifted in place)
  const uint8_t* nf;         // [B, 84, 84] newest frames (device-mapped pinned host)
  uint8_t* rows;             // [T, B, 4, 84, 84] rollout rows
  unsigned short* h2;        // [B, 3872] scratch
  float* hpart;              // [S, B, 256] scratch
  int64_t* act;              // [T, B]
  float* logp;               // [T, B]
  float* vf;                 // [T, B]
  float* lout;               // [T, B, A]
  int64_t* act_now;          // [B] device-mapped pinned host (the env reads the actions here)
  int64_t* ctr_t;            // device {rng counter, row}: read at start, advanced by T at the end
  const int64_t* go;         // mapped host: step t may run once *go >= t + 1; *go < 0 aborts
  int64_t* done_seq;         // mapped host: t + 1 once step t's actions are stored
  unsigned int* bar;         // device: [0] global barrier arrivals, [2..9] per-XCD arrivals (zeroed at launch)
  unsigned int* cdone;       // device: phase-C completion counter (zeroed before the launch)
  int64_t* err_dev;          // device error word (first error wins)
  int64_t* err_host;         // mapped host error word
  uint64_t go_ticks, bar_ticks;  // wait bounds in s_memrealtime ticks
  uint64_t* prof;            // optional [T][5] s_memrealtime stamps of workgroup 0 (phase timing)
};

// error codes (err = code | step << 8)
constexpr int64_t kErrGoTimeout = 1, kErrAbort = 2, kErrBarrierTimeout = 3;

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void fail(const Args& a, int64_t code) {
  int64_t expected = 0;
  if (__hip_atomic_compare_exchange_strong(a.err_dev, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT))
    __hip_atomic_store(a.err_host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool failed(const Args& a) {
  return __hip_atomic_load(a.err_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// thread 0 waits until the host releases step t (its frames are staged); false: leave the kernel
__device__ __forceinline__ bool wait_go(const Args& a, int64_t t) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    const uint64_t t0 = now_ticks();
    for (;;) {
      const int64_t g = __hip_atomic_load(const_cast<int64_t*>(a.go), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (g >= t + 1) break;
      if (g < 0) {
        fail(a, kErrAbort | (t << 8));
        ok = 0;
        break;
      }
      if (failed(a)) {
        ok = 0;
        break;
      }
      if (now_ticks() - t0 > a.go_ticks) {
        fail(a, kErrGoTimeout | (t << 8));
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the host wrote the frames before `go`
  }
  __syncthreads();
  return ok != 0;
}

// XCC (XCD) this workgroup runs on: hardware register XCC_ID (gfx940+: HW_REG id 20, bits [3:0])
__device__ __forceinline__ int xcc_id() {
  return int(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20)) & 15;
}

// Grid barrier number k (1-based): hierarchical over the 8 XCDs. A workgroup's global stores
// reach its XCD's L2 (s_barrier drains vmcnt); the L2s of different XCDs are not coherent, so the
// stores must be written back before workgroups elsewhere read them — but ONE write-back per XCD
// suffices: workgroups arrive on a per-XCD counter (blockIdx % 8 = the dispatcher's round-robin
// XCD; a workgroup whose hardware XCC_ID differs writes back its own L2 first), the last arriver
// of each XCD group writes that L2 back and arrives on the global counter. Everyone waits for 8 k
// global arrivals, then invalidates (acquire) before reading other workgroups' results. A
// per-workgroup write-back (64-128 of them serialised per XCD) measured ~5-8 µs per barrier.
__device__ __forceinline__ bool grid_barrier(const Args& a, uint32_t k, int64_t t) {
  __shared__ int ok;
  __syncthreads();  // every wave's global stores have reached the L2
  if (threadIdx.x == 0) {
    ok = 1;
    const int G = int(gridDim.x), grp = int(blockIdx.x) & 7;
    const uint32_t members = uint32_t((G - grp + 7) / 8);  // workgroups with blockIdx % 8 == grp
    if (xcc_id() != grp) __threadfence();                  // not where the grouping assumed: own write-back
    if (atomicAdd(&a.bar[2 + grp], 1u) == members * k - 1) {
      __threadfence();  // release: write back this XCD's L2 (every member's stores are in it)
      atomicAdd(a.bar, 1u);
    }
    const uint32_t target = uint32_t(G < 8 ? G : 8) * k;
    const uint64_t t0 = now_ticks();
    while (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (failed(a)) {
        ok = 0;
        break;
      }
      if (now_ticks() - t0 > a.bar_ticks) {
        fail(a, kErrBarrierTimeout | (t << 8));
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __threadfence();  // acquire: drop stale lines before reading the other workgroups' results
  }
  __syncthreads();
  return ok != 0;
}

template <int A1>
__global__ __launch_bounds__(NT) void k_rollout_server(const Args a) {
  using namespace trunk;
  __shared__ __attribute__((aligned(16))) unsigned short fh[HF_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short h1p[H1P_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short w1s[C1 * W1_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w2s[C2 * W2_PITCH];
  __shared__ __attribute__((aligned(16))) float whs[A1 * dense::H];
  __shared__ float bhs[A1];
  __shared__ dense::f32x4 red[2][3][1][64];  // K13s unit reductions, one per 4-wave half
  const int G = int(gridDim.x), wg = int(blockIdx.x), tid = int(threadIdx.x), wave = tid >> 6, lane = tid & 63;
  const int64_t B = a.B, T = a.T;
  const int64_t ctr0 = a.ctr_t[0];
  const bool trunk_wg = wg < B;
  const bool head_wg = int64_t(wg) * 8 < B;
  const int nC = int((B + 7) / 8);
  constexpr int64_t FB = C0 * H0 * H0;

  // ---- once per fragment: weights into LDS, h1 tile padding
  TrunkBias tb{0.f, 0.f, 0.f};
  if (trunk_wg) {
    stage_weight<NT, C1, C0, 8>(a.W1, a.w1, w1s, W1_PITCH);
    stage_weight<NT, C2, C1, 4>(a.W2, a.w2, w2s, W2_PITCH);
    zero_lds(h1p, H1P_ELEMS * 2);
    tb = trunk_bias(a.b1, a.b2);
  }
  if (head_wg) {
    for (int e = tid; e < A1 * dense::H; e += NT) whs[e] = dense::bf2f(a.Wh[e]);
    if (tid < A1) bhs[tid] = dense::bf2f(a.bh[tid]);
  }
  __syncthreads();

  const int64_t mt = (B + 15) / 16;
  const int64_t tiles = mt * (dense::H / 16), units = tiles * a.S;
  uint32_t nbar = 0;
  for (int64_t t = 0; t < T; t++) {
    // ---- A: K10 trunk of env `wg` (push mode: stack shift + new frame + row t store)
    uint64_t* pr = (a.prof && wg == 0 && tid == 0) ? a.prof + t * 5 : nullptr;
    if (trunk_wg) {
      if (!wait_go(a, t)) return;
      if (pr) pr[0] = now_ticks();
      FrameRegs<NT> fr;
      frame_issue_push<NT>(a.stack + wg * FB, a.nf + wg * (H0 * H0), fr);
      zero_half_frame_border(fh);  // the previous step's h2 staging overwrote part of it
      frame_push_store<NT>(fr, a.stack + wg * FB, a.rows + (t * B + wg) * FB);
      trunk_convs<NT>(fr, fh, h1p, w1s, w2s, tb, nullptr, a.h2 + wg * NP2 * C2, 0);
    }
    if (pr) pr[1] = now_ticks();
    if (!grid_barrier(a, ++nbar, t)) return;
    if (pr) pr[2] = now_ticks();
    // ---- B: K13s split-K dense partials over all waves (two 4-wave units per workgroup pass)
    for (int64_t u0 = 2 * int64_t(wg); u0 < units; u0 += 2 * int64_t(G)) {
      const int64_t u = u0 + (wave >> 2);
      const bool valid = u < units;
      const int64_t uu = valid ? u : 0, sl = uu / tiles, rem = uu % tiles, tm = rem / 16, tn = rem % 16;
      dense::dense_part_unit<1, 1, 1, 1>(a.h2, a.Wd, B, KDENSE, dense::H, a.S, a.hpart, sl, tm, tn, wave & 3, valid,
                                         red[wave >> 2]);
    }
    if (!grid_barrier(a, ++nbar, t)) return;
    if (pr) pr[3] = now_ticks();
    // ---- C: K16 heads + sampling, one wave per env row; the last workgroup to finish signals the host
    if (head_wg) {
      const int64_t b = int64_t(wg) * 8 + wave;
      if (b < B)
        dense::heads_sample_row<A1>(nullptr, whs, bhs, t, uint32_t(ctr0 + t), a.seed, a.act, a.logp, a.vf, a.lout,
                                    a.act_now, B, b, lane, a.hpart, a.S, a.bd);
      __syncthreads();
      if (tid == 0) {
        // system-scope release per workgroup: an acknowledged host-memory store is not yet visible
        // to the CPU, and stores from different CUs may overtake each other in the fabric (a relaxed
        // done_seq after the arrival count let the host read stale actions: parity test failed)
        __threadfence_system();
        if (atomicAdd(a.cdone, 1u) == unsigned(nC - 1)) {
          __hip_atomic_store(a.cdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.done_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (pr) pr[4] = now_ticks();
      }
    }
  }
  if (wg == 0 && tid == 0) {  // every workgroup read ctr_t[0] before the first barrier
    a.ctr_t[0] = ctr0 + T;
    a.ctr_t[1] = T;
  }
}

}  // namespace server

int rollout_server_launch(const RolloutServerArgs& r, hipStream_t stream) {
  if (r.B < 1 || r.B > 64) throw std::invalid_argument("rollout server: 1 <= B <= 64 envs");
  if (r.A1 < 3 || r.A1 > 16) throw std::invalid_argument("rollout server: 2 <= A <= 15 actions");
  if (r.T < 1) throw std::invalid_argument("rollout server: T >= 1");
  if (r.S != dense_fwd_part_slices(r.B, server::KDENSE, dense::H))
    throw std::invalid_argument("rollout server: S must be dense_fwd_part_slices(B, 3872, 256)");
  int dev = 0, cus = 0;
  RMM_HIP_CHECK(hipGetDevice(&dev));
  RMM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int G = r.workgroups > 0 ? r.workgroups : cus;
  G = std::min(G, cus);  // one resident workgroup per CU (~100 KB of LDS each)
  if (G < r.B) throw std::invalid_argument("rollout server: needs at least one workgroup per env");
  server::Args a;
  a.W1 = static_cast<const unsigned short*>(r.W1);
  a.w1 = trunk::WStrides{r.w1s[0], r.w1s[1], r.w1s[2], r.w1s[3]};
  a.b1 = static_cast<const unsigned short*>(r.b1);
  a.W2 = static_cast<const unsigned short*>(r.W2);
  a.w2 = trunk::WStrides{r.w2s[0], r.w2s[1], r.w2s[2], r.w2s[3]};
  a.b2 = static_cast<const unsigned short*>(r.b2);
  a.Wd = static_cast<const unsigned short*>(r.Wd);
  a.bd = static_cast<const unsigned short*>(r.bd);
  a.Wh = static_cast<const unsigned short*>(r.Wh);
  a.bh = static_cast<const unsigned short*>(r.bh);
  a.B = r.B;
  a.T = r.T;
  a.S = r.S;
  a.seed = r.seed;
  a.stack = r.stack;
  a.nf = r.nf;
  a.rows = r.rows;
  a.h2 = static_cast<unsigned short*>(r.h2);
  a.hpart = r.hpart;
  a.act = r.act;
  a.logp = r.logp;
  a.vf = r.vf;
  a.lout = r.lout;
  a.act_now = r.act_now;
  a.ctr_t = r.ctr_t;
  a.go = r.go;
  a.done_seq = r.done_seq;
  a.bar = r.bar;
  a.cdone = r.bar + 1;  // bar[0] global, bar[1] phase C, bar[2..9] per XCD
  a.err_dev = r.err_dev;
  a.err_host = r.err_host;
  a.go_ticks = uint64_t(r.go_timeout_s * 1e8);
  a.bar_ticks = uint64_t(r.barrier_timeout_s * 1e8);
  a.prof = r.prof;
  RMM_HIP_CHECK(hipMemsetAsync(r.bar, 0, 10 * sizeof(unsigned int), stream));
  RMM_HIP_CHECK(hipMemsetAsync(r.err_dev, 0, sizeof(int64_t), stream));
#define RMM_K21(N)                                                                                 \
  case N:                                                                                          \
    hipLaunchKernelGGL(server::k_rollout_server<N>, dim3(uint32_t(G)), dim3(server::NT), 0, stream, a); \
    break;
  switch (r.A1) {
    RMM_K21(3) RMM_K21(4) RMM_K21(5) RMM_K21(6) RMM_K21(7) RMM_K21(8) RMM_K21(9)
    RMM_K21(10) RMM_K21(11) RMM_K21(12) RMM_K21(13) RMM_K21(14) RMM_K21(15) RMM_K21(16)
  }
#undef RMM_K21
  RMM_HIP_CHECK(hipGetLastError());
  return G;
}

}  // namespace hip
}  // namespace rmm
