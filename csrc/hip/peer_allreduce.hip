// Peer-memory all-reduce for the PPO learner's gradient bucket (and any small bf16 / fp32 buffer)
// between co-located ranks, one process per MI355X.
//
// Why not RCCL for this: the learner all-reduces a ~1.3 MB bf16 bucket once per SGD minibatch step,
// 100 times per update. An RCCL ring over xGMI pays 2(W-1) dependent link hops per call and, on
// ROCm, cannot be captured reliably inside the learner's chained HIP graph (profiles/
// rccl_native_r3.txt). xGMI is point-to-point: every GPU has a direct link to every other, so each
// rank can READ all of its peers' buckets at once. Here:
//
//  * every rank hipMallocs one data region [in0 | in1 | red0 | red1] and one small signal region
//    (uncached) and exports both once through hipIPC; every rank maps every peer's regions;
//  * one kernel launch = one all-reduce, on the caller's stream, graph-capturable (no host
//    involvement: a device-side per-workgroup epoch counter numbers the launches);
//  * workgroup b owns a 128-B-aligned slice of the buffer. It stages its slice into its exported
//    in[epoch & 1], then signals "slice b of epoch e staged" to every peer with a system-scope
//    release store (the L2 write-back that publishes the staged data), and waits for the same flag
//    from every peer (acquire, system scope). Workgroups only wait on the SAME workgroup index of
//    their peers, so there is no grid-wide barrier;
//  * one-shot (W == 2 or small payloads): every rank reads slice b from all W staging buffers and
//    sums in fp32 in rank order 0..W-1, rounding once to the output dtype: every rank computes the
//    same bits. Two-shot (reduce-scatter + all-gather, larger W): rank r reduces chunk r of the
//    slice into its exported red[e & 1], signals phase 2, then gathers the other chunks from their
//    owners. Each rank moves 2(W-1)/W of the payload over its links instead of (W-1)x;
//  * staging buffers alternate with the epoch parity. A launch uses EVERY workgroup, so when rank A
//    starts launch e+2 it has finished launch e+1, whose barriers saw every peer start launch e+1,
//    i.e. finish reading launch e's staging: buffer e & 1 is free again without an end barrier;
//  * bounded: a flag that does not arrive within `timeout` (s_memrealtime, 100 MHz) sets an error
//    word (device copy + mapped host copy the host polls) and the workgroup gives up; later launches
//    see the device error word and return at once, so a dead peer never leaves a wave spinning.
//
// Reference parity: the tower-gradient averaging of rllib/execution/multi_gpu_learner_thread.py:20
// and rllib/execution/train_ops.py:98 (multi_gpu_train_one_step), re-designed for xGMI peers.
#include "peer_allreduce.h"

#include <cstring>

#include "adam_device.h"
#include <stdexcept>
#include <vector>

namespace rmm::hip {
namespace {

constexpr int kThreads = 512;
constexpr int kUnitVecs = 8;  // 8 x 16 B = one 128-B line: slice / chunk granularity

struct PeerArgs {
  const char* data[kPeerMaxRanks];
  uint64_t* sig[kPeerMaxRanks];
  uint64_t* epochs;
  int64_t* err_dev;
  int64_t* err_host;
  uint64_t cap;
  uint64_t timeout_ticks;
  int rank, world, nblocks;
};

__device__ __forceinline__ uint64_t* flag_at(uint64_t* sig, int phase, int nblocks, int block, int src) {
  return sig + (size_t(phase) * size_t(nblocks) + size_t(block)) * kPeerMaxRanks + size_t(src);
}

// 16-byte vector <-> 8 bf16 or 4 fp32 lanes in fp32
template <bool BF16>
struct V;
template <>
struct V<true> {
  static constexpr int N = 8;
  __device__ static void unpack(const uint4& u, float* f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static uint32_t rn(float x) {  // RNE; a NaN stays a NaN (v_cvt_pk_bf16_f32)
    return uint32_t(__builtin_bit_cast(unsigned short, __float2bfloat16(x)));
  }
  __device__ static uint4 pack(const float* f) {
    uint4 u;
    u.x = rn(f[0]) | (rn(f[1]) << 16);
    u.y = rn(f[2]) | (rn(f[3]) << 16);
    u.z = rn(f[4]) | (rn(f[5]) << 16);
    u.w = rn(f[6]) | (rn(f[7]) << 16);
    return u;
  }
  __device__ static float elem(const void* p, int64_t i) {
    return __uint_as_float(uint32_t(static_cast<const unsigned short*>(p)[i]) << 16);
  }
  __device__ static void store_elem(void* p, int64_t i, float x) {
    static_cast<unsigned short*>(p)[i] = static_cast<unsigned short>(rn(x));
  }
};
template <>
struct V<false> {
  static constexpr int N = 4;
  __device__ static void unpack(const uint4& u, float* f) {
    f[0] = __uint_as_float(u.x);
    f[1] = __uint_as_float(u.y);
    f[2] = __uint_as_float(u.z);
    f[3] = __uint_as_float(u.w);
  }
  __device__ static uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
  __device__ static float elem(const void* p, int64_t i) { return static_cast<const float*>(p)[i]; }
  __device__ static void store_elem(void* p, int64_t i, float x) { static_cast<float*>(p)[i] = x; }
};

// vector v of the user buffer (n elements); the last vector may be partial (zero padded)
template <bool BF16>
__device__ __forceinline__ uint4 load_user(const void* buf, int64_t v, int64_t n) {
  constexpr int N = V<BF16>::N;
  if ((v + 1) * N <= n) return reinterpret_cast<const uint4*>(buf)[v];
  float f[N];
#pragma unroll
  for (int i = 0; i < N; i++) f[i] = (v * N + i < n) ? V<BF16>::elem(buf, v * N + i) : 0.f;
  return V<BF16>::pack(f);
}
template <bool BF16>
__device__ __forceinline__ void store_user(void* buf, int64_t v, int64_t n, const uint4& u) {
  constexpr int N = V<BF16>::N;
  if ((v + 1) * N <= n) {
    reinterpret_cast<uint4*>(buf)[v] = u;
    return;
  }
  float f[N];
  V<BF16>::unpack(u, f);
  for (int i = 0; i < N; i++)
    if (v * N + i < n) V<BF16>::store_elem(buf, v * N + i, f[i]);
}

// Signal `phase` of epoch e to every rank, then wait for every rank's. False: timed out.
__device__ bool block_barrier(const PeerArgs& a, int phase, uint64_t e) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = 1;
  __syncthreads();  // every wave's staging stores are issued before lane t publishes them
  const int t = threadIdx.x;
  if (t < a.world) {
    __hip_atomic_store(flag_at(a.sig[t], phase, a.nblocks, blockIdx.x, a.rank), e, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t* f = flag_at(a.sig[a.rank], phase, a.nblocks, blockIdx.x, t);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // relaxed polls (each a coherent system-scope load), ONE acquire fence after the flag arrived:
    // an acquire per poll would invalidate this XCD's L2 on every iteration, under the feet of
    // whatever else runs there
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        const int64_t code = 1 + int64_t(t) + (int64_t(blockIdx.x) << 8) + (int64_t(phase) << 24);
        __hip_atomic_store(a.err_dev, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.err_host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' staged data is visible
  }
  __syncthreads();
  return s_ok != 0;
}

template <bool BF16, bool TWO_SHOT>
__global__ void __launch_bounds__(kThreads) k_peer_allreduce(PeerArgs a, void* buf, int64_t n) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_dead;
  constexpr int N = V<BF16>::N;
  const int tid = threadIdx.x, b = blockIdx.x;
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1;
    s_dead = __hip_atomic_load(a.err_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  }
  // slice of this workgroup, in 16-B vectors, 128-B aligned (no two workgroups share a line)
  const int64_t nv = (n + N - 1) / N;
  const int64_t nu = (nv + kUnitVecs - 1) / kUnitVecs;
  const int64_t ub = (nu + a.nblocks - 1) / a.nblocks;
  const int64_t u0 = min(nu, int64_t(b) * ub), u1 = min(nu, u0 + ub);
  const int64_t lo = u0 * kUnitVecs, hi = min(nv, u1 * kUnitVecs);
  __syncthreads();
  if (s_dead) return;
  const uint64_t e = s_epoch;
  const uint64_t par = e & 1ull;
  uint4* mine = reinterpret_cast<uint4*>(const_cast<char*>(a.data[a.rank]) + par * a.cap);
  for (int64_t v = lo + tid; v < hi; v += kThreads) mine[v] = load_user<BF16>(buf, v, n);
  bool ok = block_barrier(a, 0, e);
  if (ok) {
    if (!TWO_SHOT) {
      for (int64_t v = lo + tid; v < hi; v += kThreads) {
        uint4 x[kPeerMaxRanks];
#pragma unroll
        for (int r = 0; r < kPeerMaxRanks; r++)
          if (r < a.world) x[r] = reinterpret_cast<const uint4*>(a.data[r] + par * a.cap)[v];
        float acc[N], f[N];
        V<BF16>::unpack(x[0], acc);
#pragma unroll
        for (int r = 1; r < kPeerMaxRanks; r++) {
          if (r < a.world) {
            V<BF16>::unpack(x[r], f);
#pragma unroll
            for (int i = 0; i < N; i++) acc[i] += f[i];
          }
        }
        store_user<BF16>(buf, v, n, V<BF16>::pack(acc));
      }
    } else {
      // reduce-scatter: chunk `rank` of the slice, summed in rank order, into red[par] and the output
      const int64_t su = u1 - u0, cu = (su + a.world - 1) / a.world;
      const int64_t c0 = lo + min(su, int64_t(a.rank) * cu) * kUnitVecs;
      const int64_t c1 = min(hi, lo + min(su, int64_t(a.rank + 1) * cu) * kUnitVecs);
      uint4* red = reinterpret_cast<uint4*>(const_cast<char*>(a.data[a.rank]) + (2 + par) * a.cap);
      for (int64_t v = c0 + tid; v < c1; v += kThreads) {
        uint4 x[kPeerMaxRanks];
#pragma unroll
        for (int r = 0; r < kPeerMaxRanks; r++)
          if (r < a.world) x[r] = reinterpret_cast<const uint4*>(a.data[r] + par * a.cap)[v];
        float acc[N], f[N];
        V<BF16>::unpack(x[0], acc);
#pragma unroll
        for (int r = 1; r < kPeerMaxRanks; r++) {
          if (r < a.world) {
            V<BF16>::unpack(x[r], f);
#pragma unroll
            for (int i = 0; i < N; i++) acc[i] += f[i];
          }
        }
        const uint4 o = V<BF16>::pack(acc);
        red[v] = o;
        store_user<BF16>(buf, v, n, o);
      }
      ok = block_barrier(a, 1, e);
      if (ok) {
        // all-gather: every other chunk from its owner's red[par]
        for (int c = 0; c < a.world; c++) {
          if (c == a.rank) continue;
          const int64_t g0 = lo + min(su, int64_t(c) * cu) * kUnitVecs;
          const int64_t g1 = min(hi, lo + min(su, int64_t(c + 1) * cu) * kUnitVecs);
          const uint4* src = reinterpret_cast<const uint4*>(a.data[c] + (2 + par) * a.cap);
          for (int64_t v = g0 + tid; v < g1; v += kThreads) store_user<BF16>(buf, v, n, src[v]);
        }
      }
    }
  }
  if (tid == 0) a.epochs[b] = e;
}

// ---------------------------------------------------------------- ZeRO-1: reduce-scatter + Adam + all-gather
// The partition is AllReduce's two-shot one: workgroup b owns a 128-B-line slice of the staged
// gradient vectors, rank r chunk r of it. Red regions hold fp32 masters (4 B per element, so a launch
// covers at most cap / 4 elements whatever the gradient dtype).
struct Part {
  int64_t c0, c1;  // this rank's chunk, in gradient vectors
  int64_t lo, hi, su, cu;
};
template <int N>
__device__ __forceinline__ Part zero1_part(int64_t n, int nblocks, int b, int rank, int world) {
  Part p;
  const int64_t nv = (n + N - 1) / N;
  const int64_t nu = (nv + kUnitVecs - 1) / kUnitVecs;
  const int64_t ub = (nu + nblocks - 1) / nblocks;
  const int64_t u0 = min(nu, int64_t(b) * ub), u1 = min(nu, u0 + ub);
  p.lo = u0 * kUnitVecs;
  p.hi = min(nv, u1 * kUnitVecs);
  p.su = u1 - u0;
  p.cu = (p.su + world - 1) / world;
  p.c0 = p.lo + min(p.su, int64_t(rank) * p.cu) * kUnitVecs;
  p.c1 = min(p.hi, p.lo + min(p.su, int64_t(rank + 1) * p.cu) * kUnitVecs);
  return p;
}

struct Zero1Dev {
  float* master;
  float* m1;
  float* m2;
  __hip_bfloat16* whi;
  __hip_bfloat16* wlo;
  const float* hp;
  float grad_scale;
  const int64_t* step_ctr;
  int64_t* bump;
  int nbump;
  uint32_t* done;
  int64_t* bump_next;
};

// the weight planes of element e from its fp32 master (adam_span's rounding: hi = RNE(w), lo = RNE(w - hi))
__device__ __forceinline__ void zero1_planes4(const Zero1Dev& z, int64_t e, const float4& w) {
  *reinterpret_cast<uint2*>(z.whi + e) = make_uint2(bf16x2_rn(w.x, w.y), bf16x2_rn(w.z, w.w));
  if (z.wlo) *reinterpret_cast<uint2*>(z.wlo + e) = make_uint2(bf16x2_lo(w.x, w.y), bf16x2_lo(w.z, w.w));
}
__device__ __forceinline__ void zero1_planes1(const Zero1Dev& z, int64_t e, float w) {
  z.whi[e] = __float2bfloat16(w);
  if (z.wlo) z.wlo[e] = __float2bfloat16(w - __bfloat162float(__float2bfloat16(w)));
}

// <= 128 VGPRs (two workgroups per CU): the peers' same-index workgroups must be able to run at once,
// and ranks sharing a GPU (or a concurrent kernel) compete for the same slots
constexpr int kZThreads = 512, kZU = 4;  // kZU vectors in flight per lane in the copy loops
template <bool BF16>
__global__ void __launch_bounds__(kZThreads) __attribute__((amdgpu_waves_per_eu(4)))
k_peer_zero1(PeerArgs a, const void* grad, int64_t n, Zero1Dev z) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_dead;
  constexpr int N = V<BF16>::N;
  const int tid = threadIdx.x, b = blockIdx.x;
  if (tid == 0) {
    s_epoch = a.epochs[b] + 1;
    s_dead = __hip_atomic_load(a.err_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  }
  const AdamCoef c = adam_coef(z.hp, z.step_ctr);  // every workgroup reads the step before any bump
  int64_t* bump = z.bump;
  if (z.bump_next) {  // parity counters (k_adam_flat): one lane writes the next copy, no ticket
    if (b == 0 && tid == 0)
      for (int k = 0; k < z.nbump; k++) z.bump_next[k] = z.bump[k] + 1;
    bump = nullptr;
  }
  const Part p = zero1_part<N>(n, a.nblocks, b, a.rank, a.world);
  __syncthreads();
  if (!s_dead) {
    const uint64_t e = s_epoch, par = e & 1ull;
    uint4* mine = reinterpret_cast<uint4*>(const_cast<char*>(a.data[a.rank]) + par * a.cap);
    for (int64_t v0 = p.lo + tid; v0 < p.hi; v0 += kZThreads * kZU) {  // loads first: kZU in flight
      uint4 t[kZU];
#pragma unroll
      for (int u = 0; u < kZU; u++)
        if (v0 + u * kZThreads < p.hi) t[u] = load_user<BF16>(grad, v0 + u * kZThreads, n);
#pragma unroll
      for (int u = 0; u < kZU; u++)
        if (v0 + u * kZThreads < p.hi) mine[v0 + u * kZThreads] = t[u];
    }
    bool ok = a.world == 1 || block_barrier(a, 0, e);
    if (ok) {
      float* red = reinterpret_cast<float*>(const_cast<char*>(a.data[a.rank]) + (2 + par) * a.cap);
      for (int64_t v = p.c0 + tid; v < p.c1; v += kZThreads) {
        uint4 x[kPeerMaxRanks];
#pragma unroll
        for (int r = 0; r < kPeerMaxRanks; r++)
          if (r < a.world) x[r] = reinterpret_cast<const uint4*>(a.data[r] + par * a.cap)[v];
        // this slot's master / moments loaded with the peers' slices, before the sum waits for them (loaded
        // after it, they cost a second round trip per slot); clamped to the last whole quad, used only when
        // the quad is whole
        constexpr int NQ = N / 4;
        float4 wq[NQ], mq[NQ], sq[NQ];
        if (n >= 4) {
          const int64_t lastq = ((n >> 2) - 1) << 2;
#pragma unroll
          for (int q = 0; q < NQ; q++) {
            const int64_t el = min(v * N + 4 * q, lastq);
            wq[q] = *reinterpret_cast<const float4*>(z.master + el);
            mq[q] = *reinterpret_cast<const float4*>(z.m1 + el);
            sq[q] = *reinterpret_cast<const float4*>(z.m2 + el);
          }
        }
        float acc[N], f[N];
        V<BF16>::unpack(x[0], acc);
#pragma unroll
        for (int r = 1; r < kPeerMaxRanks; r++) {
          if (r < a.world) {
            V<BF16>::unpack(x[r], f);
#pragma unroll
            for (int i = 0; i < N; i++) acc[i] += f[i];
          }
        }
        if constexpr (BF16) V<BF16>::unpack(V<BF16>::pack(acc), acc);  // the all-reduce's single rounding
#pragma unroll
        for (int q = 0; q < N / 4; q++) {
          const int64_t e0 = v * N + 4 * q;
          if (e0 + 4 <= n) {
            float4 w = wq[q], m = mq[q], s2 = sq[q];
            w.x = adam_one(w.x, acc[4 * q] * z.grad_scale, m.x, s2.x, c);
            w.y = adam_one(w.y, acc[4 * q + 1] * z.grad_scale, m.y, s2.y, c);
            w.z = adam_one(w.z, acc[4 * q + 2] * z.grad_scale, m.z, s2.z, c);
            w.w = adam_one(w.w, acc[4 * q + 3] * z.grad_scale, m.w, s2.w, c);
            *reinterpret_cast<float4*>(z.master + e0) = w;
            *reinterpret_cast<float4*>(z.m1 + e0) = m;
            *reinterpret_cast<float4*>(z.m2 + e0) = s2;
            *reinterpret_cast<float4*>(red + e0) = w;
            zero1_planes4(z, e0, w);
          } else {
            for (int i = 0; i < 4; i++) {
              const int64_t ei = e0 + i;
              if (ei < n) {
                float m = z.m1[ei], s2 = z.m2[ei];
                const float w = adam_one(z.master[ei], acc[4 * q + i] * z.grad_scale, m, s2, c);
                z.master[ei] = w;
                z.m1[ei] = m;
                z.m2[ei] = s2;
                red[ei] = w;
                zero1_planes1(z, ei, w);
              }
            }
          }
        }
      }
      ok = a.world == 1 || block_barrier(a, 1, e);
      if (ok) {  // all-gather the other chunks' fp32 masters; the planes follow with the same rounding
        for (int cc = 0; cc < a.world; cc++) {
          if (cc == a.rank) continue;
          const int64_t g0 = p.lo + min(p.su, int64_t(cc) * p.cu) * kUnitVecs;
          const int64_t g1 = min(p.hi, p.lo + min(p.su, int64_t(cc + 1) * p.cu) * kUnitVecs);
          const float* src = reinterpret_cast<const float*>(a.data[cc] + (2 + par) * a.cap);
          // groups of 4 masters; whole groups (all but possibly the last) kZU at a time, loads first
          const int64_t q0 = g0 * (N / 4), q1 = min(g1 * (N / 4), n / 4);
          for (int64_t j0 = q0 + tid; j0 < q1; j0 += kZThreads * kZU) {
            float4 w[kZU];
#pragma unroll
            for (int u = 0; u < kZU; u++)
              if (j0 + u * kZThreads < q1) w[u] = *reinterpret_cast<const float4*>(src + 4 * (j0 + u * kZThreads));
#pragma unroll
            for (int u = 0; u < kZU; u++)
              if (j0 + u * kZThreads < q1) {
                const int64_t e0 = 4 * (j0 + u * kZThreads);
                *reinterpret_cast<float4*>(z.master + e0) = w[u];
                zero1_planes4(z, e0, w[u]);
              }
          }
          if (tid == 0)  // n % 4 tail inside this chunk
            for (int64_t e1 = max(4 * q1, g0 * N); e1 < min(g1 * N, n); e1++) {
              const float w = src[e1];
              z.master[e1] = w;
              zero1_planes1(z, e1, w);
            }
        }
      }
    }
    if (tid == 0) a.epochs[b] = e;
  }
  last_block_bump(bump, z.nbump, z.done);  // every workgroup, dead or not, so the tickets stay whole
}

template <int N>
__global__ void __launch_bounds__(256) k_zero1_mask(float* buf, int64_t n, int nblocks, int rank, int world) {
  for (int b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const Part p = zero1_part<N>(n, nblocks, b, rank, world);
    for (int64_t v = p.lo + threadIdx.x; v < p.hi; v += blockDim.x) {
      if (v >= p.c0 && v < p.c1) continue;
      for (int i = 0; i < N; i++)
        if (v * N + i < n) buf[v * N + i] = 0.f;
    }
  }
}

}  // namespace

PeerOccupancy PeerKernelOccupancy(int device) {
  int prev = 0;
  RMM_HIP_CHECK(hipGetDevice(&prev));
  RMM_HIP_CHECK(hipSetDevice(device));
  PeerOccupancy o{};
  RMM_HIP_CHECK(hipDeviceGetAttribute(&o.cus, hipDeviceAttributeMultiprocessorCount, device));
  RMM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &o.allreduce_per_cu, reinterpret_cast<const void*>(&k_peer_allreduce<false, false>), kThreads, 0));
  RMM_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &o.zero1_per_cu, reinterpret_cast<const void*>(&k_peer_zero1<false>), kZThreads, 0));
  RMM_HIP_CHECK(hipSetDevice(prev));
  return o;
}

PeerAllReduce::PeerAllReduce(int rank, int world, int device, uint64_t cap_bytes, int nblocks, double timeout_s)
    : rank_(rank), world_(world), device_(device), nblocks_(nblocks) {
  if (world < 1 || world > kPeerMaxRanks || rank < 0 || rank >= world)
    throw std::invalid_argument("PeerAllReduce: bad rank / world (max 16 ranks)");
  if (nblocks < 1 || nblocks > 1024) throw std::invalid_argument("PeerAllReduce: nblocks in [1, 1024]");
  cap_ = (cap_bytes + 255) & ~uint64_t(255);
  if (cap_ < 4096) cap_ = 4096;
  timeout_ticks_ = uint64_t(timeout_s > 0 ? timeout_s * 1e8 : 1e8);
  RMM_HIP_CHECK(hipSetDevice(device));
  // The data region must be exportable: a process's first allocation has been seen to come back
  // non-exportable (hipIpcGetMemHandle: invalid argument, 1 of 3 ranks sharing one MI355X), so
  // probe the export here and retry with a fresh allocation (keeping the failed one until the end
  // so the allocator cannot hand the same range back) before giving up.
  {
    std::vector<void*> rejected;
    for (int attempt = 0; attempt < 4 && !data_; attempt++) {
      void* p = nullptr;
      const size_t bytes = size_t(4 * cap_) + (attempt ? (size_t(2) << 20) * size_t(attempt) : 0);
      hipError_t e = attempt % 2 ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocDefault) : hipMalloc(&p, bytes);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      hipIpcMemHandle_t probe;
      if (hipIpcGetMemHandle(&probe, p) == hipSuccess) {
        data_ = static_cast<char*>(p);
        alloc_attempts_ = attempt + 1;
      } else {
        (void)hipGetLastError();
        rejected.push_back(p);
      }
    }
    for (void* p : rejected) (void)hipFree(p);
    if (!data_) throw std::runtime_error("PeerAllReduce: no IPC-exportable device allocation");
  }
  const size_t sig_bytes = size_t(2) * size_t(nblocks) * kPeerMaxRanks * sizeof(uint64_t);
  // flags in uncached (fine-grained) device memory: peers' remote stores and the local spin meet in
  // HBM, not in an XCD's L2
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sig_bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t probe;
    if (hipIpcGetMemHandle(&probe, sig_) == hipSuccess) {
      sig_uncached_ = true;
    } else {  // not exportable on this driver: ordinary device memory (system-scope atomics still order it)
      (void)hipGetLastError();
      (void)hipFree(sig_);
      sig_ = nullptr;
    }
  } else {
    (void)hipGetLastError();
  }
  if (!sig_) RMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&sig_), sig_bytes));
  RMM_HIP_CHECK(hipMemset(sig_, 0, sig_bytes));
  RMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&epochs_), size_t(nblocks) * sizeof(uint64_t) + sizeof(int64_t)));
  RMM_HIP_CHECK(hipMemset(epochs_, 0, size_t(nblocks) * sizeof(uint64_t) + sizeof(int64_t)));
  err_dev_ = reinterpret_cast<int64_t*>(epochs_ + nblocks);
  RMM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), 64, hipHostMallocMapped));
  *err_host_ = 0;
  RMM_HIP_CHECK(hipDeviceSynchronize());
  peer_data_[rank] = data_;
  peer_sig_[rank] = sig_;
}

PeerAllReduce::~PeerAllReduce() {
  try {
    Close();
  } catch (...) {
  }
}

std::string PeerAllReduce::Handles() const {
  hipIpcMemHandle_t h[2];
  RMM_HIP_CHECK(hipIpcGetMemHandle(&h[0], data_));
  RMM_HIP_CHECK(hipIpcGetMemHandle(&h[1], sig_));
  return std::string(reinterpret_cast<const char*>(h), sizeof(h));
}

void PeerAllReduce::Open(const std::vector<std::string>& handles) {
  if (int(handles.size()) != world_) throw std::invalid_argument("PeerAllReduce::Open: one handle blob per rank");
  RMM_HIP_CHECK(hipSetDevice(device_));
  for (int r = 0; r < world_; r++) {
    if (r == rank_) continue;
    if (handles[size_t(r)].size() != 2 * sizeof(hipIpcMemHandle_t))
      throw std::invalid_argument("PeerAllReduce::Open: bad handle blob");
    hipIpcMemHandle_t h[2];
    memcpy(h, handles[size_t(r)].data(), sizeof(h));
    void* p = nullptr;
    RMM_HIP_CHECK(hipIpcOpenMemHandle(&p, h[0], hipIpcMemLazyEnablePeerAccess));
    peer_data_[r] = static_cast<char*>(p);
    RMM_HIP_CHECK(hipIpcOpenMemHandle(&p, h[1], hipIpcMemLazyEnablePeerAccess));
    peer_sig_[r] = static_cast<uint64_t*>(p);
  }
  open_ = true;
}

void PeerAllReduce::AllReduce(uint64_t buf, uint64_t count, int dtype, uint64_t stream, int algo) {
  if (!open_ && world_ > 1) throw std::runtime_error("PeerAllReduce: Open() the peers first");
  if (dtype != 0 && dtype != 1) throw std::invalid_argument("PeerAllReduce: dtype 0 (bf16) or 1 (fp32)");
  if (buf % 16) throw std::invalid_argument("PeerAllReduce: buffer must be 16-byte aligned");
  if (count == 0 || world_ == 1) return;
  const uint64_t esz = dtype == 0 ? 2 : 4;
  const uint64_t per = (cap_ / esz) & ~uint64_t(127);  // elements per launch (whole 128-B lines)
  PeerArgs a{};
  for (int r = 0; r < world_; r++) {
    a.data[r] = peer_data_[r];
    a.sig[r] = peer_sig_[r];
  }
  a.epochs = epochs_;
  a.err_dev = err_dev_;
  void* dh = nullptr;
  RMM_HIP_CHECK(hipHostGetDevicePointer(&dh, err_host_, 0));
  a.err_host = static_cast<int64_t*>(dh);
  a.cap = cap_;
  a.timeout_ticks = timeout_ticks_;
  a.rank = rank_;
  a.world = world_;
  a.nblocks = nblocks_;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (uint64_t off = 0; off < count; off += per) {
    const uint64_t n = count - off < per ? count - off : per;
    void* p = reinterpret_cast<void*>(buf + off * esz);
    // one-shot reads (W-1) x n per rank in one phase; two-shot 2(W-1)/W x n in two phases: two-shot
    // once the payload per link is large enough to outweigh the second barrier
    const bool two = algo == 2 || (algo == 0 && world_ > 2 && n * esz >= (uint64_t(256) << 10));
    const dim3 g(nblocks_), blk(kThreads);
    if (dtype == 0) {
      if (two)
        hipLaunchKernelGGL((k_peer_allreduce<true, true>), g, blk, 0, s, a, p, int64_t(n));
      else
        hipLaunchKernelGGL((k_peer_allreduce<true, false>), g, blk, 0, s, a, p, int64_t(n));
    } else {
      if (two)
        hipLaunchKernelGGL((k_peer_allreduce<false, true>), g, blk, 0, s, a, p, int64_t(n));
      else
        hipLaunchKernelGGL((k_peer_allreduce<false, false>), g, blk, 0, s, a, p, int64_t(n));
    }
    RMM_HIP_CHECK(hipGetLastError());
    launches_++;
  }
}

void PeerAllReduce::AllReduceAdam(uint64_t grad, uint64_t count, int dtype, uint64_t stream, const AdamArgs& z) {
  if (!open_ && world_ > 1) throw std::runtime_error("PeerAllReduce: Open() the peers first");
  if (dtype != 0 && dtype != 1) throw std::invalid_argument("AllReduceAdam: dtype 0 (bf16) or 1 (fp32)");
  if (grad % 16 || reinterpret_cast<uintptr_t>(z.master) % 16 || reinterpret_cast<uintptr_t>(z.m1) % 16 ||
      reinterpret_cast<uintptr_t>(z.m2) % 16 || reinterpret_cast<uintptr_t>(z.whi) % 8 ||
      reinterpret_cast<uintptr_t>(z.wlo) % 8)
    throw std::invalid_argument("AllReduceAdam: 16-B aligned gradient / master / moments, 8-B aligned planes");
  if (!z.master || !z.m1 || !z.m2 || !z.whi || !z.hp) throw std::invalid_argument("AllReduceAdam: buffers");
  if (z.bump_next && (!z.bump || z.nbump <= 0)) throw std::invalid_argument("AllReduceAdam: bump_next needs bump");
  if (z.bump && !z.bump_next && !z.done) throw std::invalid_argument("AllReduceAdam: in-place bump needs done");
  if (count == 0) return;
  const uint64_t esz = dtype == 0 ? 2 : 4;
  const uint64_t per = (cap_ / 4) & ~uint64_t(127);  // the red regions hold fp32 masters
  PeerArgs a{};
  for (int r = 0; r < world_; r++) {
    a.data[r] = peer_data_[r];
    a.sig[r] = peer_sig_[r];
  }
  a.epochs = epochs_;
  a.err_dev = err_dev_;
  void* dh = nullptr;
  RMM_HIP_CHECK(hipHostGetDevicePointer(&dh, err_host_, 0));
  a.err_host = static_cast<int64_t*>(dh);
  a.cap = cap_;
  a.timeout_ticks = timeout_ticks_;
  a.rank = rank_;
  a.world = world_;
  a.nblocks = nblocks_;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (uint64_t off = 0; off < count; off += per) {
    const uint64_t n = count - off < per ? count - off : per;
    const bool last = off + per >= count;
    Zero1Dev d{z.master + off, z.m1 + off, z.m2 + off, static_cast<__hip_bfloat16*>(z.whi) + off,
               z.wlo ? static_cast<__hip_bfloat16*>(z.wlo) + off : nullptr, z.hp, z.grad_scale, z.step_ctr,
               last ? z.bump : nullptr, z.nbump, z.done, last ? z.bump_next : nullptr};
    const void* g = reinterpret_cast<const void*>(grad + off * esz);
    if (dtype == 0)
      hipLaunchKernelGGL((k_peer_zero1<true>), dim3(nblocks_), dim3(kZThreads), 0, s, a, g, int64_t(n), d);
    else
      hipLaunchKernelGGL((k_peer_zero1<false>), dim3(nblocks_), dim3(kZThreads), 0, s, a, g, int64_t(n), d);
    RMM_HIP_CHECK(hipGetLastError());
    launches_++;
  }
}

void PeerAllReduce::MaskUnowned(uint64_t buf, uint64_t count, int dtype, uint64_t stream) {
  if (dtype != 0 && dtype != 1) throw std::invalid_argument("MaskUnowned: dtype 0 (bf16) or 1 (fp32)");
  const uint64_t per = (cap_ / 4) & ~uint64_t(127);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (uint64_t off = 0; off < count && world_ > 1; off += per) {
    const uint64_t n = count - off < per ? count - off : per;
    float* p = reinterpret_cast<float*>(buf) + off;
    if (dtype == 0)
      hipLaunchKernelGGL(k_zero1_mask<8>, dim3(64), dim3(256), 0, s, p, int64_t(n), nblocks_, rank_, world_);
    else
      hipLaunchKernelGGL(k_zero1_mask<4>, dim3(64), dim3(256), 0, s, p, int64_t(n), nblocks_, rank_, world_);
    RMM_HIP_CHECK(hipGetLastError());
  }
}

int64_t PeerAllReduce::Error() const { return err_host_ ? *reinterpret_cast<volatile int64_t*>(err_host_) : 0; }

void PeerAllReduce::ClearError() {
  RMM_HIP_CHECK(hipSetDevice(device_));
  RMM_HIP_CHECK(hipDeviceSynchronize());
  if (err_host_) *err_host_ = 0;
  RMM_HIP_CHECK(hipMemset(err_dev_, 0, sizeof(int64_t)));
}

void PeerAllReduce::Close() {
  if (!data_) return;
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (int r = 0; r < world_; r++) {
    if (r == rank_) continue;
    if (peer_data_[r]) (void)hipIpcCloseMemHandle(peer_data_[r]);
    if (peer_sig_[r]) (void)hipIpcCloseMemHandle(peer_sig_[r]);
    peer_data_[r] = nullptr;
    peer_sig_[r] = nullptr;
  }
  (void)hipFree(data_);
  (void)hipFree(sig_);
  (void)hipFree(epochs_);
  (void)hipHostFree(err_host_);
  data_ = nullptr;
  sig_ = nullptr;
  epochs_ = nullptr;
  err_host_ = nullptr;
  err_dev_ = nullptr;
  open_ = false;
}

}  // namespace rmm::hip
