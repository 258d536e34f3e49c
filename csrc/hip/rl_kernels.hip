// Fused RL kernels for the PPO learner on CDNA4 (gfx950).
//
//  K5b ppo_cat_fwd / ppo_cat_bwd — the WHOLE categorical PPO loss head in two launches:
//        log-softmax, log p(a), entropy, KL(old||new), ratio, clipped surrogate, clipped value
//        loss, stats reduction (fwd) and d/dlogits, d/dvalue scaled by the upstream gradient read
//        from device memory (bwd). Replaces ~30 PyTorch elementwise/reduction launches per step.
//        Parity: reference rllib/algorithms/ppo/ppo_torch_policy.py:loss (+ TorchCategorical).
//  K6  adam_flat — Adam over ONE flat fp32 master buffer with bf16 gradients in, bf16 weights
//        out (the compute copy the model reads), bias correction from a device step counter:
//        the whole optimizer step is one launch and graph-capturable.
//  K7  sample_store — Gumbel-max categorical sampling with a stateless counter-based hash RNG,
//        writes action / log p(a) / value / logits straight into the rollout buffers at row t
//        read from device memory (HIP-graph friendly).
//
// Small-A categorical heads (A <= 32): one thread per sample, logits held in registers.
#include <hip/hip_bf16.h>

#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "adam_device.h"
#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

constexpr int kMaxA = 32;

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<__hip_bfloat16>(const __hip_bfloat16* p, int64_t i) {
  return __bfloat162float(p[i]);
}
template <typename T>
__device__ __forceinline__ void stf(T* p, int64_t i, float v);
template <>
__device__ __forceinline__ void stf<float>(float* p, int64_t i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void stf<__hip_bfloat16>(__hip_bfloat16* p, int64_t i, float v) {
  p[i] = __float2bfloat16(v);
}

// coef layout (device): [clip, vf_clip, vf_coeff, ent_coeff, kl_coeff]
// stats layout: [sum(-surr), sum(vf_clipped), sum(entropy), sum(kl), sum(clipped), sum(total)]
template <typename TL, typename TV>
__global__ __launch_bounds__(256) void k_ppo_cat_fwd(const TL* __restrict__ logits, const float* __restrict__ old_logits,
                                                    const int64_t* __restrict__ actions,
                                                    const float* __restrict__ old_logp, const float* __restrict__ adv,
                                                    const TV* __restrict__ values, const float* __restrict__ vtgt,
                                                    const float* __restrict__ coef, float* __restrict__ stats,
                                                    int64_t N, int A) {
  const float clip = coef[0], vf_clip = coef[1], vf_coeff = coef[2], ent_coeff = coef[3], kl_coeff = coef[4];
  float s[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    float l[kMaxA], lo[kMaxA];
    float mx = -INFINITY, mxo = -INFINITY;
    for (int j = 0; j < A; j++) {
      l[j] = ldf(logits, i * A + j);
      lo[j] = old_logits[i * A + j];
      mx = fmaxf(mx, l[j]);
      mxo = fmaxf(mxo, lo[j]);
    }
    float se = 0.f, seo = 0.f;
    for (int j = 0; j < A; j++) {
      se += __expf(l[j] - mx);
      seo += __expf(lo[j] - mxo);
    }
    const float lse = mx + __logf(se), lseo = mxo + __logf(seo);
    float m = 0.f, kl = 0.f;
    for (int j = 0; j < A; j++) {
      const float p = __expf(l[j] - lse), po = __expf(lo[j] - lseo);
      m += p * l[j];
      kl += po * ((lo[j] - lseo) - (l[j] - lse));
    }
    const float ent = lse - m;
    const int a = int(actions[i]);
    const float logp = l[a] - lse;
    const float r = __expf(logp - old_logp[i]);
    const float ad = adv[i];
    const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
    const float surr = fminf(r * ad, rc * ad);
    const float d = ldf(values, i) - vtgt[i];
    const float vf = fminf(d * d, vf_clip);
    s[0] += -surr;
    s[1] += vf;
    s[2] += ent;
    s[3] += kl;
    s[4] += (fabsf(r - 1.f) > clip) ? 1.f : 0.f;
    s[5] += -surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl;
  }
#pragma unroll
  for (int k = 0; k < 6; k++)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
  __shared__ float red[6][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0)
    for (int k = 0; k < 6; k++) red[k][w] = s[k];
  __syncthreads();
  if (threadIdx.x < 6) {
    float t = 0.f;
    for (int k = 0; k < int(blockDim.x >> 6); k++) t += red[threadIdx.x][k];
    atomicAdd(&stats[threadIdx.x], t);
  }
}

template <typename TL, typename TV>
__global__ __launch_bounds__(256) void k_ppo_cat_bwd(const TL* __restrict__ logits, const float* __restrict__ old_logits,
                                                    const int64_t* __restrict__ actions,
                                                    const float* __restrict__ old_logp, const float* __restrict__ adv,
                                                    const TV* __restrict__ values, const float* __restrict__ vtgt,
                                                    const float* __restrict__ coef, const float* __restrict__ gout,
                                                    TL* __restrict__ g_logits, TV* __restrict__ g_values, int64_t N,
                                                    int A) {
  const float clip = coef[0], vf_clip = coef[1], vf_coeff = coef[2], ent_coeff = coef[3], kl_coeff = coef[4];
  const float gs = gout[0] / float(N);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    float l[kMaxA], lo[kMaxA];
    float mx = -INFINITY, mxo = -INFINITY;
    for (int j = 0; j < A; j++) {
      l[j] = ldf(logits, i * A + j);
      lo[j] = old_logits[i * A + j];
      mx = fmaxf(mx, l[j]);
      mxo = fmaxf(mxo, lo[j]);
    }
    float se = 0.f, seo = 0.f;
    for (int j = 0; j < A; j++) {
      se += __expf(l[j] - mx);
      seo += __expf(lo[j] - mxo);
    }
    const float lse = mx + __logf(se), lseo = mxo + __logf(seo);
    float m = 0.f;
    for (int j = 0; j < A; j++) m += __expf(l[j] - lse) * l[j];
    const int a = int(actions[i]);
    const float logp = l[a] - lse;
    const float r = __expf(logp - old_logp[i]);
    const float ad = adv[i];
    const bool unclipped = r * ad <= fminf(fmaxf(r, 1.f - clip), 1.f + clip) * ad;
    const bool inside = (r >= 1.f - clip) && (r <= 1.f + clip);
    const float spg = (unclipped || inside) ? -(r * ad) : 0.f;  // d(-surr)/d logp
    for (int j = 0; j < A; j++) {
      const float p = __expf(l[j] - lse), po = __expf(lo[j] - lseo);
      const float g = spg * ((j == a ? 1.f : 0.f) - p) + ent_coeff * p * (l[j] - m) + kl_coeff * (p - po);
      stf(g_logits, i * A + j, g * gs);
    }
    const float d = ldf(values, i) - vtgt[i];
    stf(g_values, i, (d * d < vf_clip) ? vf_coeff * 2.f * d * gs : 0.f);
  }
}

void ppo_cat_loss(bool fwd, const void* logits, bool logits_bf16, const float* old_logits, const int64_t* actions,
                  const float* old_logp, const float* adv, const void* values, bool values_bf16, const float* vtgt,
                  const float* coef, float* stats, const float* gout, void* g_logits, void* g_values, int64_t N,
                  int A, hipStream_t stream) {
  if (A > kMaxA) throw std::invalid_argument("ppo_cat_loss: at most 32 actions");
  if (N <= 0) return;
  int64_t blocks = std::min<int64_t>((N + 255) / 256, 1024);
  using bf = __hip_bfloat16;
#define RMM_PPO_LAUNCH(TL, TV)                                                                                    \
  if (fwd)                                                                                                       \
    hipLaunchKernelGGL((k_ppo_cat_fwd<TL, TV>), dim3(uint32_t(blocks)), dim3(256), 0, stream,                   \
                       static_cast<const TL*>(logits), old_logits, actions, old_logp, adv,                       \
                       static_cast<const TV*>(values), vtgt, coef, stats, N, A);                                 \
  else                                                                                                           \
    hipLaunchKernelGGL((k_ppo_cat_bwd<TL, TV>), dim3(uint32_t(blocks)), dim3(256), 0, stream,                   \
                       static_cast<const TL*>(logits), old_logits, actions, old_logp, adv,                       \
                       static_cast<const TV*>(values), vtgt, coef, gout, static_cast<TL*>(g_logits),             \
                       static_cast<TV*>(g_values), N, A);
  if (logits_bf16 && values_bf16) {
    RMM_PPO_LAUNCH(bf, bf)
  } else if (logits_bf16) {
    RMM_PPO_LAUNCH(bf, float)
  } else if (values_bf16) {
    RMM_PPO_LAUNCH(float, bf)
  } else {
    RMM_PPO_LAUNCH(float, float)
  }
#undef RMM_PPO_LAUNCH
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K5c merged-head PPO loss

// heads[N, A+1] (bf16): logits in columns [0, A), value in column A (one Linear for both heads).
// cols[N, A+4] (f32): old logits [0, A), old logp A, advantage A+1, value target A+2, action A+3.
// fwd: atomically accumulates the 6 stats sums into acc[0..5] (zeroed by the caller per update).
// bwd: g_heads[N, A+1] = d(total)/d(heads) * (*gout) / N.
template <int kMode>  // 0: stats (fwd), 1: grads (bwd), 2: both in one pass
__global__ __launch_bounds__(256) void k_ppo_heads(const __hip_bfloat16* __restrict__ heads,
                                                  const float* __restrict__ cols, const float* __restrict__ coef,
                                                  float* __restrict__ acc, const float* __restrict__ gout,
                                                  __hip_bfloat16* __restrict__ g_heads, int64_t N, int A) {
  const float clip = coef[0], vf_clip = coef[1], vf_coeff = coef[2], ent_coeff = coef[3], kl_coeff = coef[4];
  const int lh = A + 1, lc = A + 4;
  float s[6] = {0, 0, 0, 0, 0, 0};
  constexpr bool kStats = kMode != 1, kGrads = kMode != 0;
  const float gs = kGrads ? gout[0] / float(N) : 0.f;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += int64_t(gridDim.x) * blockDim.x) {
    const __hip_bfloat16* hrow = heads + i * lh;
    const float* crow = cols + i * lc;
    float l[kMaxA], lo[kMaxA];
    float mx = -INFINITY, mxo = -INFINITY;
    for (int j = 0; j < A; j++) {
      l[j] = __bfloat162float(hrow[j]);
      lo[j] = crow[j];
      mx = fmaxf(mx, l[j]);
      mxo = fmaxf(mxo, lo[j]);
    }
    float se = 0.f, seo = 0.f;
    for (int j = 0; j < A; j++) {
      se += __expf(l[j] - mx);
      seo += __expf(lo[j] - mxo);
    }
    const float lse = mx + __logf(se), lseo = mxo + __logf(seo);
    float m = 0.f, kl = 0.f;
    for (int j = 0; j < A; j++) {
      const float p = __expf(l[j] - lse), po = __expf(lo[j] - lseo);
      m += p * l[j];
      kl += po * ((lo[j] - lseo) - (l[j] - lse));
    }
    const int a = min(max(int(crow[A + 3]), 0), A - 1);
    const float logp = l[a] - lse;
    const float r = __expf(logp - crow[A]);
    const float ad = crow[A + 1];
    const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
    const float d = __bfloat162float(hrow[A]) - crow[A + 2];
    if constexpr (kStats) {
      const float ent = lse - m;
      const float surr = fminf(r * ad, rc * ad);
      const float vf = fminf(d * d, vf_clip);
      s[0] += -surr;
      s[1] += vf;
      s[2] += ent;
      s[3] += kl;
      s[4] += (fabsf(r - 1.f) > clip) ? 1.f : 0.f;
      s[5] += -surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl;
    }
    if constexpr (kGrads) {
      const bool unclipped = r * ad <= rc * ad;
      const bool inside = (r >= 1.f - clip) && (r <= 1.f + clip);
      const float spg = (unclipped || inside) ? -(r * ad) : 0.f;
      __hip_bfloat16* grow = g_heads + i * lh;
      for (int j = 0; j < A; j++) {
        const float p = __expf(l[j] - lse), po = __expf(lo[j] - lseo);
        const float g = spg * ((j == a ? 1.f : 0.f) - p) + ent_coeff * p * (l[j] - m) + kl_coeff * (p - po);
        grow[j] = __float2bfloat16(g * gs);
      }
      grow[A] = __float2bfloat16((d * d < vf_clip) ? vf_coeff * 2.f * d * gs : 0.f);
    }
  }
  if constexpr (kStats) {
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
    __shared__ float red[6][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0)
      for (int k = 0; k < 6; k++) red[k][w] = s[k];
    __syncthreads();
    if (threadIdx.x < 6) {
      float t = 0.f;
      for (int k = 0; k < int(blockDim.x >> 6); k++) t += red[threadIdx.x][k];
      atomicAdd(&acc[threadIdx.x], t);
    }
  }
}

void ppo_heads_loss(bool bwd, const void* heads, const float* cols, const float* coef, float* acc, const float* gout,
                    void* g_heads, int64_t N, int A, hipStream_t stream) {
  if (A > kMaxA) throw std::invalid_argument("ppo_heads_loss: at most 32 actions");
  if (N <= 0) return;
  int64_t blocks = std::min<int64_t>((N + 255) / 256, 1024);
  auto* h = static_cast<const __hip_bfloat16*>(heads);
  if (bwd && acc)  // stats + grads in one pass (the upstream gradient is known at forward time)
    hipLaunchKernelGGL(k_ppo_heads<2>, dim3(uint32_t(blocks)), dim3(256), 0, stream, h, cols, coef, acc, gout,
                       static_cast<__hip_bfloat16*>(g_heads), N, A);
  else if (bwd)
    hipLaunchKernelGGL(k_ppo_heads<1>, dim3(uint32_t(blocks)), dim3(256), 0, stream, h, cols, coef, acc, gout,
                       static_cast<__hip_bfloat16*>(g_heads), N, A);
  else
    hipLaunchKernelGGL(k_ppo_heads<0>, dim3(uint32_t(blocks)), dim3(256), 0, stream, h, cols, coef, acc, gout,
                       static_cast<__hip_bfloat16*>(nullptr), N, A);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K6 flat Adam (fp32 master -> bf16 weights)

// hp layout (device): [lr, beta1, beta2, eps, weight_decay, step]; the step comes from the device
// counter when given. The per-element pass is adam_span (adam_device.h), shared with the Adam
// workgroups of the trunk-reduce launch.
// Each thread updates U groups of 4 consecutive elements with 16-B fp32 and 8-B bf16 accesses (the
// step is HBM / Infinity-Cache bound: 28 B/param), issuing every group's loads before the first
// update so U x 4 vector loads are in flight per lane; the n % 4 tail is done by the first threads
// of the grid. Requires the host-checked alignment of every pointer (adam_flat falls back to
// vec=false otherwise).
template <typename TG, bool VEC, int U>
__global__ __launch_bounds__(256) void k_adam_flat(float* __restrict__ master, float* __restrict__ m1,
                                                  float* __restrict__ m2, const TG* __restrict__ grad,
                                                  __hip_bfloat16* __restrict__ wbf16, const float* __restrict__ hp,
                                                  float grad_scale, int64_t n, const int64_t* __restrict__ step_ctr,
                                                  int64_t* bump, int nbump, uint32_t* done,
                                                  const float* __restrict__ scale_ptr, int64_t* bump_next,
                                                  __hip_bfloat16* __restrict__ wlo) {
  // step: hp[5], or (device step counter + 1) when the counter is given (graph-friendly)
  // scale_ptr (optional): a device-side factor, e.g. the global-norm clip coefficient of K6b
  if (scale_ptr) grad_scale *= scale_ptr[0];
  const AdamCoef c = adam_coef(hp, step_ctr);
  if (bump_next) {
    // parity counters: this step's kernels read `bump`, the next step's read `bump_next`, so one lane
    // writes the advanced values straight away — no ticket, nothing waits for the other workgroups
    // (every reader of `bump_next` runs after this kernel's boundary; `bump` is rewritten only by
    // the following step's K6, after every reader of this step has finished)
    if (blockIdx.x == 0 && threadIdx.x == 0)
      for (int k = 0; k < nbump; k++) bump_next[k] = bump[k] + 1;
    bump = nullptr;
  }
  const int64_t tid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x, nthr = int64_t(gridDim.x) * blockDim.x;
  adam_span<TG, VEC, U>(master, m1, m2, grad, wbf16, grad_scale, c, tid, nthr, n, wlo);
  last_block_bump(bump, nbump, done);
}

int bump_done_words() { return kBumpWords; }

void adam_flat(float* master, float* m1, float* m2, const void* grad, bool grad_bf16, void* wbf16, const float* hp,
               float grad_scale, int64_t n, hipStream_t stream, const int64_t* step_ctr, int64_t* bump, int nbump,
               uint32_t* done, const float* scale_ptr, int max_blocks, int64_t* bump_next, void* wlo) {
  if (n <= 0) return;
  if (wlo && !wbf16) throw std::invalid_argument("adam_flat: the split lo plane needs the hi plane (wbf16)");
  if (bump_next && (!bump || nbump <= 0)) throw std::invalid_argument("adam_flat: bump_next needs bump / nbump");
  auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
  const bool vec = al(master, 16) && al(m1, 16) && al(m2, 16) && al(grad, grad_bf16 ? 8 : 16) &&
                   (wbf16 == nullptr || al(wbf16, 8)) && (wlo == nullptr || al(wlo, 8));
  // groups of 4 per lane per loop trip (vector path), RMM_ADAM_UNROLL=1/2/4, read once. Default 2:
  // 7.8-8.0 us vs 8.8 us per launch at 1M params with U=1 on MI355X (benchmarks/bench_adam.py,
  // profiles/adam_unroll_r3.txt: half the workgroups, two groups of loads in flight per lane);
  // the per-element math is unchanged, so every U gives bit-identical results
  static const int unroll = [] {
    const char* e = getenv("RMM_ADAM_UNROLL");
    const int u = e ? atoi(e) : 2;
    return u == 1 || u == 4 ? u : 2;
  }();
  const int u = vec ? unroll : 1;
  const int64_t work = vec ? ((n + 3) / 4 + u - 1) / u : n;
  // max_blocks > 0 caps the grid (an Adam that runs BESIDE another kernel takes few wave slots)
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, max_blocks > 0 ? max_blocks : 256 * 8));
  auto go = [&](auto kern, const auto* g) {
    hipLaunchKernelGGL(kern, dim3(uint32_t(blocks)), dim3(256), 0, stream, master, m1, m2, g,
                       static_cast<__hip_bfloat16*>(wbf16), hp, grad_scale, n, step_ctr, bump, nbump, done,
                       scale_ptr, bump_next, static_cast<__hip_bfloat16*>(wlo));
  };
  auto dispatch = [&](const auto* g) {
    using TG = std::remove_const_t<std::remove_pointer_t<decltype(g)>>;
    if (!vec) go(k_adam_flat<TG, false, 1>, g);
    else if (u == 4) go(k_adam_flat<TG, true, 4>, g);
    else if (u == 2) go(k_adam_flat<TG, true, 2>, g);
    else go(k_adam_flat<TG, true, 1>, g);
  };
  if (grad_bf16)
    dispatch(static_cast<const __hip_bfloat16*>(grad));
  else
    dispatch(static_cast<const float*>(grad));
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K6b global-norm clip coefficient

// out[0] = min(1, max_norm / (||grad * grad_scale||_2 + 1e-6)) (torch.nn.utils.clip_grad_norm_
// semantics), computed on the device so it can feed K6's scale_ptr inside a HIP graph. Per-block
// fp32 partial sums of squares, the last block (ticket) reduces them in fixed order: deterministic.
constexpr int kNormBlocks = 256;
template <typename TG>
__global__ __launch_bounds__(256) void k_grad_clip_coef(const TG* __restrict__ g, int64_t n, float grad_scale,
                                                       float max_norm, float* __restrict__ partial,
                                                       uint32_t* __restrict__ ticket, float* __restrict__ out) {
  __shared__ float red[256 / kWave];
  float s = 0.f;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const float v = ldf(g, i);
    s += v * v;
  }
  for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
    for (int w = 0; w < int(blockDim.x / kWave); w++) b += red[w];
    partial[blockIdx.x] = b;
    __threadfence();
    if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __threadfence();
      double tot = 0.0;
      for (uint32_t k = 0; k < gridDim.x; k++) tot += double(__hip_atomic_load(partial + k, __ATOMIC_RELAXED,
                                                                                __HIP_MEMORY_SCOPE_AGENT));
      const float norm = float(sqrt(tot)) * fabsf(grad_scale);
      out[0] = fminf(1.f, max_norm / (norm + 1e-6f));
      out[1] = norm;
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int64_t grad_clip_workspace_floats() { return kNormBlocks + 1; }

void grad_clip_coef(const void* grad, bool grad_bf16, int64_t n, float grad_scale, float max_norm, float* workspace,
                    float* out, hipStream_t stream) {
  // workspace: kNormBlocks partial floats followed by one zero-initialised u32 ticket
  const int blocks = int(std::max<int64_t>(1, std::min<int64_t>(kNormBlocks, (n + 255) / 256)));
  uint32_t* ticket = reinterpret_cast<uint32_t*>(workspace + kNormBlocks);
  if (grad_bf16)
    hipLaunchKernelGGL(k_grad_clip_coef<__hip_bfloat16>, dim3(blocks), dim3(256), 0, stream,
                       static_cast<const __hip_bfloat16*>(grad), n, grad_scale, max_norm, workspace, ticket, out);
  else
    hipLaunchKernelGGL(k_grad_clip_coef<float>, dim3(blocks), dim3(256), 0, stream, static_cast<const float*>(grad),
                       n, grad_scale, max_norm, workspace, ticket, out);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K7 sample + store


// logits [B, A] (TL, row stride ldl), values [B] (TV, stride ldv — both may view one merged
// [B, A+1] head output); writes row t (=*t_ptr) of act [T,B], logp [T,B], vf [T,B],
// logits_out [T,B,A]; rng: uniform from hash(seed, counter, b*A+j); counter = *ctr (advanced by caller).
template <typename TL, typename TV>
__global__ __launch_bounds__(256) void k_sample_store(const TL* __restrict__ logits, const TV* __restrict__ values,
                                                     const int64_t* __restrict__ t_ptr, const int64_t* __restrict__ ctr,
                                                     uint32_t seed, int64_t* __restrict__ act, float* __restrict__ logp,
                                                     float* __restrict__ vf, float* __restrict__ lout,
                                                     int64_t* __restrict__ act_now, int64_t B, int A, int64_t ldl,
                                                     int64_t ldv) {
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  for (int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; b < B; b += int64_t(gridDim.x) * blockDim.x) {
    float best = -INFINITY, mx = -INFINITY;
    int arg = 0;
    float l[kMaxA];
    for (int j = 0; j < A; j++) {
      l[j] = ldf(logits, b * ldl + j);
      mx = fmaxf(mx, l[j]);
      const uint32_t h = hash3(seed, c, uint32_t(b * A + j));
      const float u = (float(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float gmb = l[j] - __logf(-__logf(u));
      if (gmb > best) {
        best = gmb;
        arg = j;
      }
    }
    float se = 0.f;
    for (int j = 0; j < A; j++) se += __expf(l[j] - mx);
    const int64_t o = t * B + b;
    act[o] = arg;
    act_now[b] = arg;
    logp[o] = l[arg] - mx - __logf(se);
    vf[o] = ldf(values, b * ldv);
    for (int j = 0; j < A; j++) lout[o * A + j] = l[j];
  }
}

void sample_store(const void* logits, bool logits_bf16, const void* values, bool values_bf16, const int64_t* t_ptr,
                  const int64_t* ctr, uint32_t seed, int64_t* act, float* logp, float* vf, float* lout,
                  int64_t* act_now, int64_t B, int A, hipStream_t stream, int64_t ldl, int64_t ldv) {
  if (A > kMaxA) throw std::invalid_argument("sample_store: at most 32 actions");
  if (ldl <= 0) ldl = A;
  if (ldv <= 0) ldv = 1;
  int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((B + 255) / 256, 1024));
  using bf = __hip_bfloat16;
#define RMM_SS(TL, TV)                                                                                          \
  hipLaunchKernelGGL((k_sample_store<TL, TV>), dim3(uint32_t(blocks)), dim3(256), 0, stream,                   \
                     static_cast<const TL*>(logits), static_cast<const TV*>(values), t_ptr, ctr, seed, act, logp, vf, \
                     lout, act_now, B, A, ldl, ldv);
  if (logits_bf16 && values_bf16) {
    RMM_SS(bf, bf)
  } else if (logits_bf16) {
    RMM_SS(bf, float)
  } else if (values_bf16) {
    RMM_SS(float, bf)
  } else {
    RMM_SS(float, float)
  }
#undef RMM_SS
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K9 synthetic Atari env step

// One thread per (env, pixel): stores the CURRENT observation into the rollout buffer row *t_ptr,
// shifts the 4-frame stack in place and writes the new frame (pooled frame chosen by a counter
// hash, shifted by 3*(action%4) columns); the (0,0) thread of each env also writes the reward
// (Bernoulli 0.05), advances the episode clock and writes done. Replaces ~12 PyTorch launches and
// the observation index_copy of a rollout step.
__global__ __launch_bounds__(256) void k_synth_env_step(uint8_t* __restrict__ frames, const uint8_t* __restrict__ pool,
                                                       const int64_t* __restrict__ actions, int32_t* __restrict__ tenv,
                                                       const int64_t* __restrict__ ctr_t, uint8_t* __restrict__ buf_obs,
                                                       float* __restrict__ buf_rew, float* __restrict__ buf_done,
                                                       uint32_t seed, int episode_len, int64_t B,
                                                       int64_t* bump, uint32_t* done_ctr) {
  constexpr int H = 84, W = 84, HW = H * W, C = 4;
  const uint32_t ctr = uint32_t(ctr_t[0]);
  const int64_t trow = ctr_t[1];
  const int64_t total = B * HW;
  for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < total; p += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = p / HW;
    const int s = int(p - b * HW);
    const int h = s / W, w = s - h * W;
    uint8_t* f = frames + b * C * HW + s;
    const uint8_t f0 = f[0], f1 = f[HW], f2 = f[2 * HW], f3 = f[3 * HW];
    if (buf_obs) {
      uint8_t* o = buf_obs + (trow * B + b) * C * HW + s;
      o[0] = f0;
      o[HW] = f1;
      o[2 * HW] = f2;
      o[3 * HW] = f3;
    }
    const uint32_t pidx = hash3(seed, ctr, uint32_t(b) * 2u) & 63u;
    const int shift = int(actions[b] & 3) * 3;
    int src_w = w - shift;
    if (src_w < 0) src_w += W;
    const uint8_t nf = pool[pidx * HW + h * W + src_w];
    f[0] = f1;
    f[HW] = f2;
    f[2 * HW] = f3;
    f[3 * HW] = nf;
    if (s == 0) {
      const uint32_t hr = hash3(seed, ctr, uint32_t(b) * 2u + 1u);
      const float u = float(hr >> 8) * (1.0f / 16777216.0f);
      int32_t t = tenv[b] + 1;
      const bool ended = t >= episode_len;
      tenv[b] = ended ? 0 : t;
      buf_rew[trow * B + b] = u < 0.05f ? 1.f : 0.f;
      buf_done[trow * B + b] = ended ? 1.f : 0.f;
    }
  }
  last_block_bump(bump, 2, done_ctr);
}

void synth_env_step(uint8_t* frames, const uint8_t* pool, const int64_t* actions, int32_t* tenv, const int64_t* ctr_t,
                    uint8_t* buf_obs, float* buf_rew, float* buf_done, uint32_t seed, int episode_len, int64_t B,
                    hipStream_t stream, int64_t* bump, uint32_t* done) {
  int64_t total = B * 84 * 84;
  int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(k_synth_env_step, dim3(uint32_t(blocks)), dim3(256), 0, stream, frames, pool, actions, tenv,
                     ctr_t, buf_obs, buf_rew, buf_done, seed, episode_len, B, bump, done);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K8 conv epilogue: bias + ReLU

// y[M, C] (NHWC conv output, bf16) <- relu(y + bias). 8 channels (16 B) per thread.
__global__ __launch_bounds__(256) void k_bias_relu_fwd(__hip_bfloat16* __restrict__ y, const __hip_bfloat16* __restrict__ bias,
                                                      int64_t M, int C, int relu) {
  const int groups = C / 8;
  const int64_t total = M * groups;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
    const int g = int(e % groups);
    uint4 v = reinterpret_cast<uint4*>(y)[e];
    const uint4 bv = reinterpret_cast<const uint4*>(bias)[g];
    uint32_t* pv = reinterpret_cast<uint32_t*>(&v);
    const uint32_t* pb = reinterpret_cast<const uint32_t*>(&bv);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      float lo = __uint_as_float(pv[k] << 16) + __uint_as_float(pb[k] << 16);
      float hi = __uint_as_float(pv[k] & 0xFFFF0000u) + __uint_as_float(pb[k] & 0xFFFF0000u);
      if (relu) {
        lo = fmaxf(lo, 0.f);
        hi = fmaxf(hi, 0.f);
      }
      __hip_bfloat16 l = __float2bfloat16(lo), h = __float2bfloat16(hi);
      pv[k] = uint32_t(*reinterpret_cast<unsigned short*>(&l)) | (uint32_t(*reinterpret_cast<unsigned short*>(&h)) << 16);
    }
    reinterpret_cast<uint4*>(y)[e] = v;
  }
}

// dpre = dy * (y > 0) (relu) and per-workgroup channel partial sums of dpre (deterministic: no
// atomics, no cross-workgroup hand-off; k_colsum_partials finishes the reduction).
constexpr int kBRThreads = 256;
__global__ __launch_bounds__(kBRThreads) void k_bias_relu_bwd(const __hip_bfloat16* __restrict__ dy,
                                                             const __hip_bfloat16* __restrict__ y,
                                                             __hip_bfloat16* __restrict__ dpre, float* __restrict__ partial,
                                                             int64_t M, int C, int relu, int64_t rows_per_wg) {
  const int groups = C / 8;                  // channel groups of 8
  const int rpi = kBRThreads / groups;       // rows per iteration of the workgroup
  const int g = threadIdx.x % groups;
  const int r0 = threadIdx.x / groups;
  const int64_t row_begin = int64_t(blockIdx.x) * rows_per_wg;
  const int64_t row_end = min(M, row_begin + rows_per_wg);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r0 < rpi) {
    for (int64_t r = row_begin + r0; r < row_end; r += rpi) {
      const int64_t e = r * groups + g;
      uint4 d = reinterpret_cast<const uint4*>(dy)[e];
      uint32_t* pd = reinterpret_cast<uint32_t*>(&d);
      if (relu) {
        const uint4 yv = reinterpret_cast<const uint4*>(y)[e];
        const uint32_t* py = reinterpret_cast<const uint32_t*>(&yv);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t mlo = (py[k] & 0x7FFFu) && !(py[k] & 0x8000u) ? 0x0000FFFFu : 0u;
          const uint32_t mhi = (py[k] & 0x7FFF0000u) && !(py[k] & 0x80000000u) ? 0xFFFF0000u : 0u;
          pd[k] &= (mlo | mhi);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        acc[2 * k] += __uint_as_float(pd[k] << 16);
        acc[2 * k + 1] += __uint_as_float(pd[k] & 0xFFFF0000u);
      }
      reinterpret_cast<uint4*>(dpre)[e] = d;
    }
  }
  // reduce threads sharing a channel group through LDS
  __shared__ float red[kBRThreads][9];
#pragma unroll
  for (int k = 0; k < 8; k++) red[threadIdx.x][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < groups * 8) {
    const int gg = threadIdx.x / 8, k = threadIdx.x % 8;
    float s = 0.f;
    for (int t = gg; t < rpi * groups; t += groups) s += red[t][k];
    partial[int64_t(blockIdx.x) * C + gg * 8 + k] = s;
  }
}

// Column sums of partial[G, C]: blockIdx.x owns channels [c0, c0 + cb) with cb = min(C, 64);
// the 256 threads form (256 / cb) row slots x cb channels, each slot sums a strided subset of the
// G rows (independent loads in flight), then slots combine through LDS in a fixed order =>
// deterministic. (One slot per wave was latency bound: ~30 us for G ~ 900 on gfx950.)
__global__ __launch_bounds__(256) void k_colsum_partials(const float* __restrict__ partial, int64_t G, int C,
                                                        __hip_bfloat16* __restrict__ out_bf16, float* __restrict__ out_f32) {
  __shared__ float red[256];
  const int cb = C < 64 ? C : 64;
  const int nslots = 256 / cb;
  const int slot = threadIdx.x / cb, lc = threadIdx.x % cb;
  const int c = blockIdx.x * 64 + lc;
  float s = 0.f;
  if (slot < nslots && c < C) {
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t g = slot;
    for (; g + 3 * nslots < G; g += 4 * nslots) {
      s += partial[g * C + c];
      s1 += partial[(g + nslots) * C + c];
      s2 += partial[(g + 2 * nslots) * C + c];
      s3 += partial[(g + 3 * nslots) * C + c];
    }
    for (; g < G; g += nslots) s += partial[g * C + c];
    s = (s + s1) + (s2 + s3);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < cb && c < C) {
    float t = 0.f;
    for (int k = 0; k < nslots; k++) t += red[k * cb + threadIdx.x];
    if (out_bf16) out_bf16[c] = __float2bfloat16(t);
    if (out_f32) out_f32[c] = t;
  }
}

void bias_relu_fwd(void* y, const void* bias, int64_t M, int C, bool relu, hipStream_t stream) {
  if (C % 8) throw std::invalid_argument("bias_relu_fwd: C must be a multiple of 8");
  int64_t total = M * (C / 8);
  if (total <= 0) return;
  int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(k_bias_relu_fwd, dim3(uint32_t(blocks)), dim3(256), 0, stream, static_cast<__hip_bfloat16*>(y),
                     static_cast<const __hip_bfloat16*>(bias), M, C, relu ? 1 : 0);
  RMM_HIP_CHECK(hipGetLastError());
}

int64_t bias_relu_bwd_partials(int64_t M) {
  // one workgroup per CU at most (256 CUs), each streaming >= 512 rows: enough bytes in flight
  // for HBM while keeping the second-pass column sum short
  return std::max<int64_t>(1, std::min<int64_t>(256, (M + 511) / 512));
}

void bias_relu_bwd(const void* dy, const void* y, void* dpre, void* dbias_bf16, float* partial, int64_t M, int C,
                   bool relu, hipStream_t stream) {
  if (C % 8 || C > 8 * kBRThreads) throw std::invalid_argument("bias_relu_bwd: bad C");
  const int64_t G = bias_relu_bwd_partials(M);
  const int64_t rows_per_wg = (M + G - 1) / G;
  hipLaunchKernelGGL(k_bias_relu_bwd, dim3(uint32_t(G)), dim3(kBRThreads), 0, stream,
                     static_cast<const __hip_bfloat16*>(dy), static_cast<const __hip_bfloat16*>(y),
                     static_cast<__hip_bfloat16*>(dpre), partial, M, C, relu ? 1 : 0, rows_per_wg);
  hipLaunchKernelGGL(k_colsum_partials, dim3(uint32_t((C + 63) / 64)), dim3(256), 0, stream, partial, G, C,
                     static_cast<__hip_bfloat16*>(dbias_bf16), static_cast<float*>(nullptr));
  RMM_HIP_CHECK(hipGetLastError());
}

// K8b: dense-layer epilogue backward for small M (a PPO minibatch): dpre = dy * [y > 0] (or dy)
// and db = column sums, ONE launch, deterministic. Workgroup = V adjacent columns x all rows
// (256 threads stride the rows, fixed-order LDS tree for the sum).
template <int V>
__global__ __launch_bounds__(256) void k_mask_colsum(const unsigned short* __restrict__ dy,
                                                     const unsigned short* __restrict__ y,
                                                     unsigned short* __restrict__ dpre,
                                                     unsigned short* __restrict__ db, int64_t M, int C, int relu) {
  __shared__ float red[V][256];
  const int col0 = blockIdx.x * V;
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; v++) acc[v] = 0.f;
  for (int64_t m = threadIdx.x; m < M; m += 256) {
    unsigned short g[V], h[V];
    if constexpr (V == 8) {
      *reinterpret_cast<uint4*>(g) = *reinterpret_cast<const uint4*>(&dy[m * C + col0]);
      if (relu) *reinterpret_cast<uint4*>(h) = *reinterpret_cast<const uint4*>(&y[m * C + col0]);
    } else {
#pragma unroll
      for (int v = 0; v < V; v++) {
        g[v] = dy[m * C + col0 + v];
        h[v] = relu ? y[m * C + col0 + v] : static_cast<unsigned short>(0);
      }
    }
#pragma unroll
    for (int v = 0; v < V; v++) {
      if (relu && (h[v] == 0 || (h[v] & 0x8000))) g[v] = 0;
      acc[v] += __uint_as_float(uint32_t(g[v]) << 16);
    }
    if (dpre) {
      if constexpr (V == 8) {
        *reinterpret_cast<uint4*>(&dpre[m * C + col0]) = *reinterpret_cast<const uint4*>(g);
      } else {
#pragma unroll
        for (int v = 0; v < V; v++) dpre[m * C + col0 + v] = g[v];
      }
    }
  }
#pragma unroll
  for (int v = 0; v < V; v++) red[v][threadIdx.x] = acc[v];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
#pragma unroll
      for (int v = 0; v < V; v++) red[v][threadIdx.x] += red[v][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x < V) {
    uint32_t u = __float_as_uint(red[threadIdx.x][0]);
    u += 0x7fffu + ((u >> 16) & 1u);
    db[col0 + threadIdx.x] = static_cast<unsigned short>(u >> 16);
  }
}

void mask_colsum(const void* dy, const void* y, void* dpre, void* db, int64_t M, int C, bool relu,
                 hipStream_t stream) {
  if (M <= 0 || C <= 0) return;
  auto* g = static_cast<const unsigned short*>(dy);
  auto* h = static_cast<const unsigned short*>(y);
  auto* d = static_cast<unsigned short*>(dpre);
  auto* b = static_cast<unsigned short*>(db);
  if (C % 8 == 0)
    hipLaunchKernelGGL(k_mask_colsum<8>, dim3(uint32_t(C / 8)), dim3(256), 0, stream, g, h, d, b, M, C, relu ? 1 : 0);
  else
    hipLaunchKernelGGL(k_mask_colsum<1>, dim3(uint32_t(C)), dim3(256), 0, stream, g, h, d, b, M, C, relu ? 1 : 0);
  RMM_HIP_CHECK(hipGetLastError());
}


// ---------------------------------------------------------------------------------------------
// K19: device-resident frame stacks for hybrid rollout workers. The CPU env uploads only the
// newest frame per env ([B, HW] u8, pinned H2D); this kernel shifts the HBM stack [B, 4, HW] one
// frame, appends the new frame and stores the resulting observation as rollout row t of buf_obs
// ([T, B, 4, HW]; row index read on the device so the step can live in a HIP graph). One thread
// owns a 16-byte pixel chunk of one env across all 4 channels, so the in-place shift is race free.
// Replaces: full-stack numpy shift on the CPU + 4x larger H2D copy + a separate row-store launch.
__global__ void __launch_bounds__(256) k_frame_push(uint8_t* __restrict__ stack, const uint8_t* __restrict__ nf,
                                                    uint8_t* __restrict__ buf_obs, const int64_t* __restrict__ t_ptr,
                                                    int64_t B, int64_t chunks) {
  const int64_t total = B * chunks;
  const int64_t trow = buf_obs ? *t_ptr : 0;
  const int64_t HW = chunks * 16;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = i / chunks, c = i - b * chunks;
    uint4* s = reinterpret_cast<uint4*>(stack + b * 4 * HW) + c;
    const int64_t cs = chunks;  // channel stride in uint4
    const uint4 f1 = s[cs], f2 = s[2 * cs], f3 = s[3 * cs];
    const uint4 n = reinterpret_cast<const uint4*>(nf + b * HW)[c];
    s[0] = f1;
    s[cs] = f2;
    s[2 * cs] = f3;
    s[3 * cs] = n;
    if (buf_obs) {
      uint4* o = reinterpret_cast<uint4*>(buf_obs + (trow * B + b) * 4 * HW) + c;
      o[0] = f1;
      o[cs] = f2;
      o[2 * cs] = f3;
      o[3 * cs] = n;
    }
  }
}

// Rollout step gate: lets the host enqueue step t+1 (a HIP-graph replay) BEFORE its CPU env step
// has produced the frames, so the launch latency overlaps the env step. The first node of the step
// waits until the host's release counter (device-mapped pinned memory, bumped by the CPU after
// writing the frames) reaches this step's sequence number, then publishes it in *dev_seq. Bounded:
// after `max_polls` polls (~s_sleep-paced) it gives up, flags *err and lets the step run, so a host
// that dies mid-fragment can never leave a wave spinning.
__global__ void __launch_bounds__(64) k_step_gate(const int64_t* host_release, int64_t* __restrict__ dev_seq,
                                                  int64_t max_polls, int* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const int64_t want = dev_seq[0] + 1;
  int64_t n = 0;
  while (__hip_atomic_load(host_release, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if (++n >= max_polls) {
      err[0] = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  dev_seq[0] = want;
}

void step_gate(const int64_t* host_release, int64_t* dev_seq, int64_t max_polls, int* err, hipStream_t stream) {
  if (host_release == nullptr || dev_seq == nullptr || err == nullptr) throw std::invalid_argument("step_gate: null pointer");
  if (max_polls < 1) max_polls = 1;
  hipLaunchKernelGGL(k_step_gate, dim3(1), dim3(64), 0, stream, host_release, dev_seq, max_polls, err);
  RMM_HIP_CHECK(hipGetLastError());
}

void frame_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* buf_obs, const int64_t* t_ptr, int64_t B,
                int64_t hw, hipStream_t stream) {
  if (hw % 16 != 0) throw std::runtime_error("frame_push: frame bytes must be a multiple of 16");
  if ((reinterpret_cast<uintptr_t>(stack) | reinterpret_cast<uintptr_t>(new_frames) |
       reinterpret_cast<uintptr_t>(buf_obs)) & 15)
    throw std::runtime_error("frame_push: buffers must be 16-byte aligned");
  const int64_t chunks = hw / 16, total = B * chunks;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 2048));
  hipLaunchKernelGGL(k_frame_push, dim3(uint32_t(blocks)), dim3(256), 0, stream, stack, new_frames, buf_obs, t_ptr,
                     B, chunks);
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
