// K17: sample-batch ingest on the learner GPU.
//
// Rollout workers ship each fragment as one packed fp32 row table raw[rows, A+5] =
// [logits(A) | logp | vf | reward | done | action] (time-major rows: row = t*n + env) plus the
// bootstrap values V(s_T) of their n envs. The learner DMAs every worker's table straight from the
// shared-memory object store into one device table (the concat happens in the DMA: each block
// lands at its row offset) and this kernel turns it into the PPO loss-column table
//   cols[rows, A+4] = [old logits(A) | old logp | advantage | value target | action]
// computing GAE per (block, env) column on the way. Parity: reference
// rllib/evaluation/postprocessing.py:compute_gae_for_sample_batch (GAE with the bootstrapped value
// on truncation) + rllib/algorithms/ppo/ppo.py:training_step (standardize_fields: advantages).
//
// One workgroup per rollout block. The block's reward / value / done columns are staged through
// LDS in env chunks (coalesced loads), each lane then runs the backward recursion of one env over
// T from LDS; the advantage sum / sum of squares feed K17b's standardisation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

namespace {
constexpr int kIngestThreads = 256;
constexpr int kIngestLds = 2048;  // staged rows per env chunk (5 fp32 columns -> 40 KB LDS)

__global__ __launch_bounds__(kIngestThreads) void k_ingest_gae(const float* __restrict__ raw,
                                                               const float* __restrict__ boot,
                                                               const IngestBlock* __restrict__ blocks, int A,
                                                               float gamma, float gl, float* __restrict__ cols,
                                                               double* __restrict__ stats) {
  __shared__ float s_rew[kIngestLds], s_val[kIngestLds], s_done[kIngestLds], s_adv[kIngestLds];
  __shared__ double s_red[2][kIngestThreads / kWave];
  const IngestBlock b = blocks[blockIdx.x];
  const int R = A + 5, C = A + 4;
  const int64_t T = b.T, n = b.n;
  const int tid = threadIdx.x;
  double sum = 0.0, sq = 0.0;
  // 1) straight column copies (logits, logp, action) for every row of the block
  for (int64_t k = tid; k < T * n * int64_t(A + 2); k += kIngestThreads) {
    const int64_t r = k / (A + 2);
    const int j = int(k % (A + 2));
    const int64_t row = b.row0 + r;
    const int src = j < A + 1 ? j : A + 4;  // logits.., logp | action
    const int dst = j < A + 1 ? j : A + 3;
    cols[row * C + dst] = raw[row * R + src];
  }
  // 2) GAE over env chunks staged in LDS
  const int64_t nc = T <= kIngestLds ? std::max<int64_t>(1, std::min<int64_t>(n, kIngestLds / T)) : 0;
  if (nc > 0) {
    for (int64_t e0 = 0; e0 < n; e0 += nc) {
      const int64_t ne = std::min<int64_t>(nc, n - e0);
      __syncthreads();
      for (int64_t k = tid; k < T * ne; k += kIngestThreads) {
        const int64_t t = k / ne, e = k % ne;
        const int64_t row = b.row0 + t * n + e0 + e;
        s_rew[k] = raw[row * R + A + 2];
        s_val[k] = raw[row * R + A + 1];
        s_done[k] = raw[row * R + A + 3];
      }
      __syncthreads();
      for (int64_t e = tid; e < ne; e += kIngestThreads) {
        float adv = 0.f, vnext = boot[b.boot0 + e0 + e];
        for (int64_t t = T - 1; t >= 0; --t) {
          const int64_t k = t * ne + e;
          const float nd = 1.f - s_done[k], v = s_val[k];
          adv = s_rew[k] + gamma * vnext * nd - v + gl * nd * adv;
          s_adv[k] = adv;
          vnext = v;
        }
      }
      __syncthreads();
      for (int64_t k = tid; k < T * ne; k += kIngestThreads) {
        const int64_t t = k / ne, e = k % ne;
        const int64_t row = b.row0 + t * n + e0 + e;
        const float a = s_adv[k];
        cols[row * C + A + 1] = a;
        cols[row * C + A + 2] = a + s_val[k];
        sum += double(a);
        sq += double(a) * double(a);
      }
    }
  } else {  // T > LDS rows: one lane per env straight from global memory
    for (int64_t e = tid; e < n; e += kIngestThreads) {
      float adv = 0.f, vnext = boot[b.boot0 + e];
      for (int64_t t = T - 1; t >= 0; --t) {
        const int64_t row = b.row0 + t * n + e;
        const float nd = 1.f - raw[row * R + A + 3], v = raw[row * R + A + 1];
        adv = raw[row * R + A + 2] + gamma * vnext * nd - v + gl * nd * adv;
        cols[row * C + A + 1] = adv;
        cols[row * C + A + 2] = adv + v;
        sum += double(adv);
        sq += double(adv) * double(adv);
        vnext = v;
      }
    }
  }
  // 3) block reduction of the advantage moments -> two device atomics
  for (int o = kWave / 2; o > 0; o >>= 1) {
    sum += __shfl_xor(sum, o, kWave);
    sq += __shfl_xor(sq, o, kWave);
  }
  __syncthreads();
  if ((tid & (kWave - 1)) == 0) {
    s_red[0][tid / kWave] = sum;
    s_red[1][tid / kWave] = sq;
  }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, q = 0.0;
    for (int w = 0; w < kIngestThreads / kWave; w++) a += s_red[0][w], q += s_red[1][w];
    atomicAdd(stats, a);
    atomicAdd(stats + 1, q);
  }
}

// K17b: cols[:, A+1] = (adv - mean) / max(std, 1e-4) (population std, as the reference's
// rllib/utils/numpy.py standardized()).
__global__ __launch_bounds__(256) void k_standardize_col(float* __restrict__ cols, int64_t N, int C, int col,
                                                        const double* __restrict__ stats) {
  const double mean = stats[0] / double(N);
  const double var = fmax(stats[1] / double(N) - mean * mean, 0.0);
  const float inv = 1.f / fmaxf(float(sqrt(var)), 1e-4f);
  const float m = float(mean);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x)
    cols[i * C + col] = (cols[i * C + col] - m) * inv;
}

// Chunked hipHostRegister of one shared-memory segment: the first DMA from a region pins the
// 64 MB chunk(s) covering it; later DMAs from the (recycled) store arena are straight page-locked
// transfers. Chunks are aligned to the segment base and never extend past its mapping.
struct HostRegistry {
  std::mutex mu;
  std::map<uintptr_t, std::pair<uintptr_t, uint64_t>> segs;  // base -> (base, size)
  std::map<uintptr_t, bool> chunks;                          // chunk start -> registered ok
};
HostRegistry& Registry() {
  static HostRegistry r;
  return r;
}
constexpr uint64_t kRegChunk = 64ull << 20;
}  // namespace

void ingest_gae(const float* raw, const float* boot, const IngestBlock* blocks_dev, int nblocks, int A, float gamma,
                float lam, float* cols, double* stats, hipStream_t stream) {
  if (nblocks <= 0) return;
  if (A < 1 || A > 64) throw std::invalid_argument("ingest_gae: 1 <= A <= 64");
  hipLaunchKernelGGL(k_ingest_gae, dim3(uint32_t(nblocks)), dim3(kIngestThreads), 0, stream, raw, boot, blocks_dev,
                     A, gamma, gamma * lam, cols, stats);
  RMM_HIP_CHECK(hipGetLastError());
}

void standardize_col(float* cols, int64_t N, int C, int col, const double* stats, hipStream_t stream) {
  if (N <= 0) return;
  const int blocks = int(std::min<int64_t>(1024, (N + 255) / 256));
  hipLaunchKernelGGL(k_standardize_col, dim3(blocks), dim3(256), 0, stream, cols, N, C, col, stats);
  RMM_HIP_CHECK(hipGetLastError());
}

void host_register_segment(uintptr_t base, uint64_t size) {
  std::lock_guard<std::mutex> g(Registry().mu);
  Registry().segs[base] = {base, size};
}

namespace {
std::string g_reg_error;
struct H2DStats {  // updated from several threads (learner ingest, spill / restore of each GpuStore)
  std::atomic<uint64_t> direct{0}, staged{0}, chunks_ok{0}, chunks_failed{0};
} g_h2d;

// Page-locked bounce buffers for ranges the registry could not pin (e.g. pages another process on
// the same GPU already registered): host memcpy into buffer k while buffer k^1 is in flight.
// Shared by every thread of the process: `mu` is held for a whole staged transfer, and each buffer's
// event orders its reuse after the DMA that last read / wrote it (whatever stream that was on).
struct Staging {
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::mutex mu;
  static constexpr uint64_t kBytes = 32ull << 20;
};
Staging& Stage() {
  static Staging s;
  static std::once_flag once;
  std::call_once(once, [] {
    for (int k = 0; k < 2; k++) {
      RMM_HIP_CHECK(hipHostMalloc(&s.buf[k], Staging::kBytes, hipHostMallocDefault));
      RMM_HIP_CHECK(hipEventCreateWithFlags(&s.ev[k], hipEventDisableTiming));
    }
  });
  return s;
}

void staged_copy(void* dst, const void* src, uint64_t n, hipStream_t stream) {
  Staging& st = Stage();
  std::lock_guard<std::mutex> g(st.mu);
  const uint8_t* s8 = static_cast<const uint8_t*>(src);
  uint8_t* d8 = static_cast<uint8_t*>(dst);
  int k = 0;
  for (uint64_t off = 0; off < n; off += Staging::kBytes, k ^= 1) {
    const uint64_t len = std::min<uint64_t>(Staging::kBytes, n - off);
    RMM_HIP_CHECK(hipEventSynchronize(st.ev[k]));  // the DMA that last read buffer k is done
    memcpy(st.buf[k], s8 + off, len);
    RMM_HIP_CHECK(hipMemcpyAsync(d8 + off, st.buf[k], len, hipMemcpyHostToDevice, stream));
    RMM_HIP_CHECK(hipEventRecord(st.ev[k], stream));
  }
}
}  // namespace

bool host_pin_range(const void* src, uint64_t n, uint64_t* newly_out) {
  auto& R = Registry();
  const uintptr_t s = reinterpret_cast<uintptr_t>(src);
  uint64_t newly = 0;
  bool all_ok = false;
  {
    std::lock_guard<std::mutex> g(R.mu);
    auto it = R.segs.upper_bound(s);
    if (it != R.segs.begin()) {
      --it;
      const uintptr_t base = it->second.first, end = base + it->second.second;
      if (s >= base && s + n <= end) {
        all_ok = true;
        for (uintptr_t c = base + ((s - base) / kRegChunk) * kRegChunk; c < s + n; c += kRegChunk) {
          auto ck = R.chunks.find(c);
          if (ck == R.chunks.end()) {
            const uint64_t len = std::min<uint64_t>(kRegChunk, end - c);
            const hipError_t re = hipHostRegister(reinterpret_cast<void*>(c), len, hipHostRegisterDefault);
            const bool ok = re == hipSuccess;
            if (!ok) {
              (void)hipGetLastError();
              g_reg_error = std::string(hipGetErrorString(re)) + " registering " + std::to_string(len) + " B at +" +
                            std::to_string(c - base);
            }
            ck = R.chunks.emplace(c, ok).first;
            if (ok) {
              newly += len;
              g_h2d.chunks_ok++;
            } else {
              g_h2d.chunks_failed++;
            }
          }
          all_ok &= ck->second;
        }
      }
    }
  }
  if (newly_out) *newly_out += newly;
  return all_ok;
}

namespace {
// D2H through the bounce buffers (host side is not page-locked).
void staged_copy_d2h(void* dst, const void* src, uint64_t n, hipStream_t stream) {
  Staging& st = Stage();
  std::lock_guard<std::mutex> g(st.mu);
  const uint8_t* s8 = static_cast<const uint8_t*>(src);
  uint8_t* d8 = static_cast<uint8_t*>(dst);
  for (uint64_t off = 0; off < n; off += Staging::kBytes) {
    const uint64_t len = std::min<uint64_t>(Staging::kBytes, n - off);
    RMM_HIP_CHECK(hipEventSynchronize(st.ev[0]));
    RMM_HIP_CHECK(hipMemcpyAsync(st.buf[0], s8 + off, len, hipMemcpyDeviceToHost, stream));
    RMM_HIP_CHECK(hipStreamSynchronize(stream));
    memcpy(d8 + off, st.buf[0], len);
  }
}
}  // namespace

void dma_host_segment(void* host, void* dev, uint64_t n, bool to_device, hipStream_t stream) {
  auto& R = Registry();
  const uintptr_t h = reinterpret_cast<uintptr_t>(host);
  uintptr_t base = 0, end = 0;
  {
    std::lock_guard<std::mutex> g(R.mu);
    auto it = R.segs.upper_bound(h);
    if (it != R.segs.begin()) {
      --it;
      if (h >= it->second.first && h + n <= it->second.first + it->second.second) {
        base = it->second.first;
        end = base + it->second.second;
      }
    }
  }
  auto piece = [&](uintptr_t p, uint64_t len, bool pinned) {
    void* hp = reinterpret_cast<void*>(p);
    uint8_t* dp = static_cast<uint8_t*>(dev) + (p - h);
    if (pinned) {
      if (to_device) RMM_HIP_CHECK(hipMemcpyAsync(dp, hp, len, hipMemcpyHostToDevice, stream));
      else RMM_HIP_CHECK(hipMemcpyAsync(hp, dp, len, hipMemcpyDeviceToHost, stream));
      g_h2d.direct += len;
    } else {
      if (to_device) staged_copy(dp, hp, len, stream);
      else staged_copy_d2h(hp, dp, len, stream);
      g_h2d.staged += len;
    }
  };
  if (!base) {  // not inside a registered segment
    piece(h, n, false);
    return;
  }
  // never let one copy straddle a pinned and an unpinned chunk: split at chunk boundaries
  for (uintptr_t p = h; p < h + n;) {
    const uintptr_t c = base + ((p - base) / kRegChunk) * kRegChunk;
    const uintptr_t cend = std::min<uintptr_t>(std::min<uintptr_t>(c + kRegChunk, end), h + n);
    const bool ok = host_pin_range(reinterpret_cast<const void*>(p), cend - p, nullptr);
    piece(p, cend - p, ok);
    p = cend;
  }
}

std::string host_register_last_error() {
  std::lock_guard<std::mutex> g(Registry().mu);
  return g_reg_error;
}

uint64_t h2d_from_segment(void* dst, const void* src, uint64_t n, hipStream_t stream) {
  uint64_t newly = 0;
  host_pin_range(src, n, &newly);
  dma_host_segment(const_cast<void*>(src), dst, n, true, stream);
  return newly;
}

std::vector<uint64_t> h2d_stats() {
  return {g_h2d.direct.load(), g_h2d.staged.load(), g_h2d.chunks_ok.load(), g_h2d.chunks_failed.load()};
}

void host_prepin(uintptr_t base, uint64_t bytes, const std::atomic<bool>* stop, std::atomic<uint64_t>* done_bytes) {
  for (uint64_t off = 0; off < bytes; off += kRegChunk) {
    if (stop && stop->load()) return;
    const uint64_t len = std::min<uint64_t>(kRegChunk, bytes - off);
    host_pin_range(reinterpret_cast<const void*>(base + off), len, nullptr);
    if (done_bytes) done_bytes->fetch_add(len);
  }
}

void host_unregister_segment(uintptr_t base) {
  auto& R = Registry();
  std::lock_guard<std::mutex> g(R.mu);
  auto it = R.segs.find(base);
  if (it == R.segs.end()) return;
  const uintptr_t end = base + it->second.second;
  for (auto c = R.chunks.lower_bound(base); c != R.chunks.end() && c->first < end;) {
    if (c->second) (void)hipHostUnregister(reinterpret_cast<void*>(c->first));
    c = R.chunks.erase(c);
  }
  R.segs.erase(it);
}

void host_unregister_all() {
  auto& R = Registry();
  std::lock_guard<std::mutex> g(R.mu);
  for (auto& kv : R.chunks)
    if (kv.second) (void)hipHostUnregister(reinterpret_cast<void*>(kv.first));
  R.chunks.clear();
  R.segs.clear();
}

}  // namespace hip
}  // namespace rmm
