// Shared helpers for the CDNA4 (gfx950) HIP code of ray_memory_management_amd.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#define RMM_HIP_CHECK(expr)                                                                 \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);     \
  } while (0)

namespace rmm {
namespace hip {

constexpr int kWave = 64;  // CDNA wavefront width

// K6 folded into a gradient epilogue (K12 dense tail, K10 trunk reduce; world of one, no global-norm
// clip). Instead of storing the bf16 gradient at address g inside the flat gradient bucket, the
// kernel rounds it to bf16 (bit-identical to the unfused K6 input) and applies Adam to element
// (g - grad_base) of the flat fp32 master / moment buffers, writing the new bf16 weight. A kernel
// given `bump` advances the device step counters from its last workgroup (as K6 does).
struct FusedAdam {
  const void* grad_base = nullptr;  // null: plain gradient stores
  float* master = nullptr;
  float* m1 = nullptr;
  float* m2 = nullptr;
  void* wbf16 = nullptr;
  const float* hp = nullptr;         // [lr, beta1, beta2, eps, weight_decay, step]
  const int64_t* step_ctr = nullptr; // Adam step = *step_ctr + 1
  int64_t* bump = nullptr;
  int nbump = 0;
  uint32_t* done = nullptr;
};

// K6 folded into the K10 trunk-reduce LAUNCH (world of one, no global-norm clip): extra workgroups
// beside the partial-sum workgroups run K6's pass over the dense + heads range of the flat
// buffers (the trunk range goes through FusedAdam in the reduce epilogue), so the SGD step loses
// the K6 launch and the two latency-bound passes overlap. Pointers are already offset to the range
// start; `bump_next` set = parity step counters (one lane writes the advanced copy), else the
// FusedAdam ticket bump advances them in place.
struct AdamTail {
  float* master = nullptr;  // null: no Adam workgroups
  float* m1 = nullptr;
  float* m2 = nullptr;
  const void* grad = nullptr;  // bf16
  void* wbf16 = nullptr;
  int64_t n = 0;
  const float* hp = nullptr;
  const int64_t* step_ctr = nullptr;
  float grad_scale = 1.f;
  int64_t* bump = nullptr;
  int nbump = 0;
  int64_t* bump_next = nullptr;
  // K12 row split with a deferred finalize: the range is the dense weight [256][K] and each gradient
  // is the sum of the rs fp32 member partials (workspace [groups][rs][20][512], see
  // dense_device.h:split_finalize_elem), rounded to bf16 — read 4 consecutive elements at a time
  const float* part = nullptr;
  int rs = 0;
  int64_t K = 0;
};

// Adam folded into the x3 (fp32 learner) trunk-reduce launch: the flat fp32 buffers (param memory
// order; the trunk range [0, n_trunk) is reduced in this launch, [n_trunk, n) holds the final dense +
// heads gradients), the split-pair weight planes, and the step counters (bump_next set = parity
// counters, else `done` tickets the last workgroup, which advances them in place).
struct X3Adam {
  float* master = nullptr;  // null: gradients only (Adam runs as K6 afterwards)
  float* m1 = nullptr;
  float* m2 = nullptr;
  const float* grad = nullptr;
  void* whi = nullptr;
  void* wlo = nullptr;
  int64_t n_trunk = 0;
  int64_t n = 0;
  const float* hp = nullptr;
  const int64_t* step_ctr = nullptr;
  float grad_scale = 1.f;
  int64_t* bump = nullptr;
  int nbump = 0;
  uint32_t* done = nullptr;
  int64_t* bump_next = nullptr;
  // K12x row parts (rs = 2): the second part's dense + heads gradients, element n_trunk + i at grad2[i];
  // the Adam workgroups use grad[n_trunk + i] + grad2[i]
  const float* grad2 = nullptr;
};

// XCD-aware remap of a linear workgroup id (bijective for any grid size): consecutive
// logical ids land on the same XCD so neighbouring tiles share an L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  const uint32_t kXcd = 8;
  if (nwg < kXcd) return orig;
  uint32_t q = nwg / kXcd, r = nwg % kXcd;
  uint32_t xcd = orig % kXcd;
  uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / kXcd;
}

}  // namespace hip
}  // namespace rmm

#if defined(__HIPCC__)
namespace rmm {
namespace hip {
// counter-based mix (murmur3 finaliser over three words); shared by the samplers and the synthetic env
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Device step counters advanced by the LAST workgroup of the kernel that reads them, instead of a
// separate 1-element add launch per step (~4 µs each in a HIP graph). Every workgroup reads the
// counters at its start, so once all of them have drawn a ticket nobody reads them any more;
// the kernel boundary publishes the new values to the next launch. Tickets are relaxed (nothing
// is published between workgroups; an acq_rel agent-scope atomic costs an L2 writeback per
// workgroup) and two-level: 16 sub-counters on separate 128-B lines, then one top counter, so
// ~2000 workgroups do not serialise on a single address (one address cost ~2 µs/1000 WGs).
// `done` = kBumpWords zero-initialised u32 owned by the call site; counters reset themselves.
// Every thread of the workgroup must reach it (it holds a workgroup barrier).
constexpr int kBumpSubs = 16, kBumpStride = 32, kBumpWords = (kBumpSubs + 1) * kBumpStride;
__device__ __forceinline__ void last_block_bump(int64_t* bump, int nbump, uint32_t* done) {
  if (!bump) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t G = gridDim.x, sub = blockIdx.x % kBumpSubs;
    const uint32_t members = (G - sub + kBumpSubs - 1) / kBumpSubs;
    uint32_t* sc = done + sub * kBumpStride;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t* top = done + kBumpSubs * kBumpStride;
      const uint32_t nsubs = G < uint32_t(kBumpSubs) ? G : uint32_t(kBumpSubs);
      if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsubs - 1) {
        for (int k = 0; k < nbump; k++) bump[k] += 1;
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

struct AdamCoef {
  float lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt;
};

// hp = [lr, beta1, beta2, eps, weight_decay, step]; the step comes from the device counter when given
__device__ __forceinline__ AdamCoef adam_coef(const float* hp, const int64_t* step_ctr) {
#pragma clang fp contract(off)
  AdamCoef c;
  c.lr = hp[0], c.b1 = hp[1], c.b2 = hp[2], c.eps = hp[3], c.wd = hp[4];
  const float step = step_ctr ? float(step_ctr[0] + 1) : hp[5];
  const float bc1 = 1.f - __powf(c.b1, step), bc2 = 1.f - __powf(c.b2, step);
  c.step_size = c.lr / bc1;
  c.inv_bc2_sqrt = 1.f / sqrtf(bc2);
  return c;
}

// No FMA contraction: K6 and the fused epilogues (K12, K10 trunk reduce) inline this into different
// code, and contraction choices made per call site would break their bit-identical results.
__device__ __forceinline__ float adam_one(float w, float g, float& a, float& b, const AdamCoef& c) {
#pragma clang fp contract(off)
  if (c.wd != 0.f) w -= c.lr * c.wd * w;  // decoupled (AdamW) decay
  a = c.b1 * a + (1.f - c.b1) * g;
  b = c.b2 * b + (1.f - c.b2) * g * g;
  return w - c.step_size * a / (sqrtf(b) * c.inv_bc2_sqrt + c.eps);
}

__device__ __forceinline__ unsigned short bf16_bits_rn(float f) {  // round-to-nearest-even (finite f)
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<unsigned short>(u >> 16);
}

// Fused-Adam state of one element, loaded ahead of the epilogue (kernels issue these loads before
// their main loop so the HBM latency hides behind it instead of serialising the epilogue).
struct AdamState {
  float w, a, b;
};
__device__ __forceinline__ AdamState adam_prefetch(const FusedAdam& fa, const unsigned short* g) {
  if (fa.grad_base == nullptr) return AdamState{0.f, 0.f, 0.f};
  const int64_t i = g - static_cast<const unsigned short*>(fa.grad_base);
  return AdamState{fa.master[i], fa.m1[i], fa.m2[i]};
}
// Epilogue store with prefetched state: the bf16 gradient at g, or the Adam update of that element.
__device__ __forceinline__ void grad_store_pf(const FusedAdam& fa, const AdamCoef& c, unsigned short* g, float v,
                                              AdamState s) {
  const unsigned short gb = bf16_bits_rn(v);
  if (fa.grad_base == nullptr) {
    *g = gb;
    return;
  }
  const int64_t i = g - static_cast<const unsigned short*>(fa.grad_base);
  const float w = adam_one(s.w, __uint_as_float(uint32_t(gb) << 16), s.a, s.b, c);
  fa.m1[i] = s.a;
  fa.m2[i] = s.b;
  fa.master[i] = w;
  static_cast<unsigned short*>(fa.wbf16)[i] = bf16_bits_rn(w);
}

// Gradient epilogue store: the bf16 gradient at g, or (FusedAdam) the Adam update of that element.
__device__ __forceinline__ void grad_store(const FusedAdam& fa, const AdamCoef& c, unsigned short* g, float v) {
  const unsigned short gb = bf16_bits_rn(v);
  if (fa.grad_base == nullptr) {
    *g = gb;
    return;
  }
  const int64_t i = g - static_cast<const unsigned short*>(fa.grad_base);
  float a = fa.m1[i], b = fa.m2[i];
  const float w = adam_one(fa.master[i], __uint_as_float(uint32_t(gb) << 16), a, b, c);
  fa.m1[i] = a;
  fa.m2[i] = b;
  fa.master[i] = w;
  static_cast<unsigned short*>(fa.wbf16)[i] = bf16_bits_rn(w);
}
}  // namespace hip
}  // namespace rmm
#endif
