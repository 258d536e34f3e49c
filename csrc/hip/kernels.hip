// CDNA4 (gfx950) kernels for ray_memory_management_amd.
//
//  K1/K2 multi_copy   — many-segment copy in ONE launch (tensor pack/unpack for serialization,
//                       sample-batch concat). Workgroups walk 256 KiB chunks; 16 B per lane.
//  K2    gather_rows  — minibatch row gather by index (SGD minibatch sampling).
//  K3    gae          — generalised advantage estimation as a chunked two-level backward affine
//                       scan: per-(env, chunk) affine maps in LDS, carry combine, re-sweep.
//                       Parity: reference rllib/evaluation/postprocessing.py:compute_advantages
//                       (discount_cumsum over delta_t with gamma*lambda).
//  K4    compress     — lossless spill compression: rotate sign to the LSB, per-256-element block
//                       frame-of-reference bit-packing of the exponent byte, raw mantissa planes,
//                       zero-block elision. One wave per block; bit-packing through LDS atomics.
//  K5    ppo_loss     — fused PPO clipped-surrogate / clipped-value / entropy loss: forward value
//                       and analytic gradient in one pass (reference
//                       rllib/algorithms/ppo/ppo_torch_policy.py:loss).
//
// All kernels use 64-lane waves; block sizes are multiples of 64.
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace rmm {
namespace hip {

// ============================================================== K1 multi_copy

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMaxSegs = 64;
constexpr uint64_t kChunk = 256 * 1024;  // bytes per workgroup
constexpr int kCopyThreads = 256;

struct SegTable {
  CopySeg seg[kMaxSegs];
  uint64_t chunk_prefix[kMaxSegs + 1];  // first chunk index of each segment
  int nseg;
};

// U independent 16 B loads in flight per lane, then U nontemporal stores; NTL: nontemporal loads too
// (the source is read once: keep it out of the L2 / MALL). RMM_COPY_VARIANT picks (U, NTL):
// 2 = (4, yes) default: 2.74 TB/s vs 2.69 for the round-3 loop 0 = (4, no) on MI355X (profiles/copy_r4.txt);
// 1 = (8, yes), 3 = (8, no).
template <int U, bool NTL>
__device__ __forceinline__ void copy_range(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                           uint64_t n) {
  const int tid = threadIdx.x;
  uint64_t s = reinterpret_cast<uint64_t>(src), d = reinterpret_cast<uint64_t>(dst);
  if (((s ^ d) & 15) == 0) {
    // byte head up to 16 B alignment
    uint64_t head = (16 - (s & 15)) & 15;
    if (head > n) head = n;
    if (tid < int(head)) dst[tid] = src[tid];
    const u32x4* vs = reinterpret_cast<const u32x4*>(src + head);
    u32x4* vd = reinterpret_cast<u32x4*>(dst + head);
    uint64_t nv = (n - head) >> 4;
    uint64_t i = tid;
    const uint64_t step = kCopyThreads;
    for (; i + (U - 1) * step < nv; i += U * step) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = NTL ? __builtin_nontemporal_load(vs + i + u * step) : vs[i + u * step];
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_nontemporal_store(v[u], vd + i + u * step);
    }
    for (; i < nv; i += step) __builtin_nontemporal_store(vs[i], vd + i);
    uint64_t tail0 = head + (nv << 4);
    for (uint64_t t = tail0 + tid; t < n; t += step) dst[t] = src[t];
  } else if (((s ^ d) & 3) == 0) {
    uint64_t head = (4 - (s & 3)) & 3;
    if (head > n) head = n;
    if (tid < int(head)) dst[tid] = src[tid];
    const uint32_t* vs = reinterpret_cast<const uint32_t*>(src + head);
    uint32_t* vd = reinterpret_cast<uint32_t*>(dst + head);
    uint64_t nv = (n - head) >> 2;
    for (uint64_t i = tid; i < nv; i += kCopyThreads) vd[i] = vs[i];
    for (uint64_t t = head + (nv << 2) + tid; t < n; t += kCopyThreads) dst[t] = src[t];
  } else {
    for (uint64_t t = tid; t < n; t += kCopyThreads) dst[t] = src[t];
  }
}

template <int U, bool NTL>
__global__ __launch_bounds__(kCopyThreads) void k_multi_copy(SegTable tab) {
  const uint64_t chunk = blockIdx.x;
  // wave-uniform binary search for the owning segment
  int lo = 0, hi = tab.nseg - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (tab.chunk_prefix[mid] <= chunk) lo = mid;
    else hi = mid - 1;
  }
  const CopySeg sg = tab.seg[lo];
  uint64_t off = (chunk - tab.chunk_prefix[lo]) * kChunk;
  if (off >= sg.nbytes) return;
  uint64_t n = sg.nbytes - off;
  if (n > kChunk) n = kChunk;
  copy_range<U, NTL>(reinterpret_cast<const uint8_t*>(sg.src) + off, reinterpret_cast<uint8_t*>(sg.dst) + off, n);
}

void multi_copy(const std::vector<CopySeg>& segs, hipStream_t stream) {
  size_t i = 0;
  while (i < segs.size()) {
    SegTable tab;
    memset(&tab, 0, sizeof(tab));
    uint64_t chunks = 0;
    int k = 0;
    for (; i < segs.size() && k < kMaxSegs; i++) {
      if (segs[i].nbytes == 0) continue;
      tab.seg[k] = segs[i];
      tab.chunk_prefix[k] = chunks;
      chunks += (segs[i].nbytes + kChunk - 1) / kChunk;
      k++;
    }
    tab.chunk_prefix[k] = chunks;
    tab.nseg = k;
    if (k == 0 || chunks == 0) continue;
    // grid is bounded by 2^31-1 blocks; 256 KiB chunks => > 500 TB per launch.
    static const int variant = [] {
      const char* e = getenv("RMM_COPY_VARIANT");
      return e ? atoi(e) : 2;
    }();
    const dim3 grid{uint32_t(chunks)}, block{uint32_t(kCopyThreads)};
    switch (variant) {
      case 0: hipLaunchKernelGGL((k_multi_copy<4, false>), grid, block, 0, stream, tab); break;
      case 1: hipLaunchKernelGGL((k_multi_copy<8, true>), grid, block, 0, stream, tab); break;
      case 3: hipLaunchKernelGGL((k_multi_copy<8, false>), grid, block, 0, stream, tab); break;
      default: hipLaunchKernelGGL((k_multi_copy<4, true>), grid, block, 0, stream, tab); break;
    }
    RMM_HIP_CHECK(hipGetLastError());
  }
}

// ============================================================== K2 gather_rows

// idx may be offset by a device counter: rows are taken from idx + (ctr[0] % period) * rows, so a
// HIP graph can walk a whole epoch's permutation without any host-side copies between replays.
__device__ __forceinline__ const int64_t* offset_idx(const int64_t* idx, const int64_t* ctr, int64_t period,
                                                     int64_t rows) {
  return (ctr && idx) ? idx + (ctr[0] % period) * rows : idx;
}

__global__ __launch_bounds__(256) void k_gather_rows16(const uint4* __restrict__ in,
                                                      const int64_t* __restrict__ idx0,
                                                      uint4* __restrict__ out, int64_t rows,
                                                      int64_t row_vec, const int64_t* __restrict__ ctr,
                                                      int64_t period) {
  const int64_t* idx = offset_idx(idx0, ctr, period, rows);
  const int64_t total = rows * row_vec;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
       e += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = e / row_vec, c = e - r * row_vec;
    out[e] = in[idx[r] * row_vec + c];
  }
}

__global__ __launch_bounds__(256) void k_gather_rows1(const uint8_t* __restrict__ in,
                                                     const int64_t* __restrict__ idx0,
                                                     uint8_t* __restrict__ out, int64_t rows,
                                                     int64_t row_bytes, const int64_t* __restrict__ ctr,
                                                     int64_t period) {
  const int64_t* idx = offset_idx(idx0, ctr, period, rows);
  const int64_t total = rows * row_bytes;
  for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
       e += int64_t(gridDim.x) * blockDim.x) {
    int64_t r = e / row_bytes, c = e - r * row_bytes;
    out[e] = in[idx[r] * row_bytes + c];
  }
}

void gather_rows(const void* in, const int64_t* idx, void* out, int64_t rows, int64_t row_bytes,
                 hipStream_t stream, const int64_t* ctr, int64_t period) {
  if (rows <= 0 || row_bytes <= 0) return;
  bool vec = (row_bytes % 16 == 0) && (reinterpret_cast<uintptr_t>(in) % 16 == 0) &&
             (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  int64_t units = vec ? rows * (row_bytes / 16) : rows * row_bytes;
  int64_t blocks = std::min<int64_t>((units + 255) / 256, 256 * 16);
  if (period <= 0) period = 1;
  if (vec)
    hipLaunchKernelGGL(k_gather_rows16, dim3(uint32_t(blocks)), dim3(256), 0, stream,
                       static_cast<const uint4*>(in), idx, static_cast<uint4*>(out), rows, row_bytes / 16, ctr,
                       period);
  else
    hipLaunchKernelGGL(k_gather_rows1, dim3(uint32_t(blocks)), dim3(256), 0, stream,
                       static_cast<const uint8_t*>(in), idx, static_cast<uint8_t*>(out), rows, row_bytes, ctr, period);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K2b frames -> NHWC bf16

// dst[b, h, w, c] = bf16(src[idx ? idx[b] : b, c, h, w] * scale). One thread per pixel, C <= 8.
// Reads are coalesced per channel plane (consecutive w), writes are one 8/16-byte vector per pixel.
template <int C>
__global__ __launch_bounds__(256) void k_frames_nhwc(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx0,
                                                    __hip_bfloat16* __restrict__ dst, int64_t B, int64_t HW,
                                                    float scale, const int64_t* __restrict__ ctr, int64_t period);

// fp32 twin of K2b for the precision-matched (fp32) learner: one float4 store per 4-channel pixel.
template <int C>
__global__ __launch_bounds__(256) void k_frames_nhwc_f32(const uint8_t* __restrict__ src,
                                                        const int64_t* __restrict__ idx0, float* __restrict__ dst,
                                                        int64_t B, int64_t HW, float scale,
                                                        const int64_t* __restrict__ ctr, int64_t period) {
  const int64_t* idx = offset_idx(idx0, ctr, period, B);
  const int64_t total = B * HW;
  for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < total;
       p += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = p / HW, s = p - b * HW;
    const int64_t sb = idx ? idx[b] : b;
    const uint8_t* in = src + sb * C * HW + s;
    if constexpr (C == 4) {
      *reinterpret_cast<float4*>(dst + p * 4) =
          make_float4(float(in[0]) * scale, float(in[HW]) * scale, float(in[2 * HW]) * scale, float(in[3 * HW]) * scale);
    } else {
#pragma unroll
      for (int c = 0; c < C; c++) dst[p * C + c] = float(in[c * HW]) * scale;
    }
  }
}

void frames_to_nhwc_f32(const uint8_t* src, const int64_t* idx, float* dst, int64_t B, int64_t C, int64_t H,
                        int64_t W, float scale, hipStream_t stream, const int64_t* ctr, int64_t period) {
  int64_t total = B * H * W;
  if (total <= 0) return;
  if (period <= 0) period = 1;
  int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 32);
  switch (C) {
    case 1: hipLaunchKernelGGL(k_frames_nhwc_f32<1>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, dst, B, H * W, scale, ctr, period); break;
    case 3: hipLaunchKernelGGL(k_frames_nhwc_f32<3>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, dst, B, H * W, scale, ctr, period); break;
    case 4: hipLaunchKernelGGL(k_frames_nhwc_f32<4>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, dst, B, H * W, scale, ctr, period); break;
    default: throw std::invalid_argument("frames_to_nhwc_f32: C must be 1, 3 or 4");
  }
  RMM_HIP_CHECK(hipGetLastError());
}

template <int C>
__global__ __launch_bounds__(256) void k_frames_nhwc(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx0,
                                                    __hip_bfloat16* __restrict__ dst, int64_t B, int64_t HW,
                                                    float scale, const int64_t* __restrict__ ctr, int64_t period) {
  const int64_t* idx = offset_idx(idx0, ctr, period, B);
  const int64_t total = B * HW;
  for (int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; p < total;
       p += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = p / HW, s = p - b * HW;
    const int64_t sb = idx ? idx[b] : b;
    const uint8_t* in = src + sb * C * HW + s;
    unsigned short v[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      __hip_bfloat16 h = __float2bfloat16(float(in[c * HW]) * scale);
      v[c] = *reinterpret_cast<unsigned short*>(&h);
    }
    unsigned short* o = reinterpret_cast<unsigned short*>(dst) + p * C;
    if constexpr (C == 4) {
      uint2 w;
      w.x = uint32_t(v[0]) | (uint32_t(v[1]) << 16);
      w.y = uint32_t(v[2]) | (uint32_t(v[3]) << 16);
      *reinterpret_cast<uint2*>(o) = w;
    } else {
#pragma unroll
      for (int c = 0; c < C; c++) o[c] = v[c];
    }
  }
}

void frames_to_nhwc_bf16(const uint8_t* src, const int64_t* idx, void* dst, int64_t B, int64_t C, int64_t H,
                         int64_t W, float scale, hipStream_t stream, const int64_t* ctr, int64_t period) {
  int64_t total = B * H * W;
  if (total <= 0) return;
  if (period <= 0) period = 1;
  int64_t blocks = std::min<int64_t>((total + 255) / 256, 256 * 32);
  auto* d = static_cast<__hip_bfloat16*>(dst);
  switch (C) {
    case 1: hipLaunchKernelGGL(k_frames_nhwc<1>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, d, B, H * W, scale, ctr, period); break;
    case 3: hipLaunchKernelGGL(k_frames_nhwc<3>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, d, B, H * W, scale, ctr, period); break;
    case 4: hipLaunchKernelGGL(k_frames_nhwc<4>, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, idx, d, B, H * W, scale, ctr, period); break;
    default: throw std::invalid_argument("frames_to_nhwc_bf16: C must be 1, 3 or 4");
  }
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K3 GAE

// Workgroup = 64 envs (one per lane) x C chunks (one wave per chunk), C <= 16.
__global__ __launch_bounds__(1024) void k_gae(const float* __restrict__ rew, const float* __restrict__ val,
                                             const float* __restrict__ done, const float* __restrict__ last_val,
                                             float* __restrict__ adv, float* __restrict__ ret, int64_t T,
                                             int64_t B, int C, int L, float gamma, float gl) {
  __shared__ float sa[16][64];
  __shared__ float sb[16][64];
  __shared__ float carry[16][64];
  const int lane = threadIdx.x & 63;
  const int ch = threadIdx.x >> 6;
  const int64_t env = int64_t(blockIdx.x) * 64 + lane;
  const bool active = env < B;
  const int64_t t0 = int64_t(ch) * L;
  const int64_t t1 = std::min<int64_t>(T, t0 + L);
  // phase 1: affine map of this chunk, A(t0) = a + b * A(t1)
  float a = 0.f, b = 1.f;
  if (active) {
    float vnext = (t1 < T) ? val[t1 * B + env] : last_val[env];
    for (int64_t t = t1 - 1; t >= t0; --t) {
      const int64_t o = t * B + env;
      const float nd = 1.f - done[o];
      const float v = val[o];
      const float delta = rew[o] + gamma * vnext * nd - v;
      a = delta + gl * nd * a;
      b = gl * nd * b;
      vnext = v;
    }
  }
  sa[ch][lane] = a;
  sb[ch][lane] = b;
  __syncthreads();
  // phase 2: carries, sequential over chunks (C <= 16) by the first wave
  if (ch == 0) {
    float c = 0.f;
    for (int k = C - 1; k >= 0; --k) {
      carry[k][lane] = c;  // advantage at the END of chunk k (start of chunk k+1)
      c = sa[k][lane] + sb[k][lane] * c;
    }
  }
  __syncthreads();
  // phase 3: re-sweep with the carry-in
  if (active && t0 < T) {
    float A = carry[ch][lane];
    float vnext = (t1 < T) ? val[t1 * B + env] : last_val[env];
    for (int64_t t = t1 - 1; t >= t0; --t) {
      const int64_t o = t * B + env;
      const float nd = 1.f - done[o];
      const float v = val[o];
      const float delta = rew[o] + gamma * vnext * nd - v;
      A = delta + gl * nd * A;
      adv[o] = A;
      ret[o] = A + v;
      vnext = v;
    }
  }
}

void gae(const float* rewards, const float* values, const float* dones, const float* last_values,
         float* adv, float* ret, int64_t T, int64_t B, float gamma, float lam, hipStream_t stream) {
  if (T <= 0 || B <= 0) return;
  int C = int(std::min<int64_t>(16, std::max<int64_t>(1, T / 8)));
  int L = int((T + C - 1) / C);
  C = int((T + L - 1) / L);
  dim3 grid(uint32_t((B + 63) / 64)), block(uint32_t(64 * C));
  hipLaunchKernelGGL(k_gae, grid, block, 0, stream, rewards, values, dones, last_values, adv, ret, T, B,
                     C, L, gamma, gamma * lam);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== scan (u16 -> u64 exclusive)

constexpr int kScanThreads = 256;
constexpr int kScanPer = 8;
constexpr int kScanTile = kScanThreads * kScanPer;  // 2048 elements per workgroup

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t n = __shfl_up(v, o, 64);
    if (lane >= o) v += n;
  }
  return v;
}

// block-wide exclusive scan of one value per thread; returns exclusive prefix, total in *tot
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* tot) {
  __shared__ uint64_t wsum[kScanThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint64_t pre = 0, total = 0;
  for (int i = 0; i < kScanThreads / 64; i++) {
    if (i < w) pre += wsum[i];
    total += wsum[i];
  }
  __syncthreads();
  *tot = total;
  return pre + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint16_t* __restrict__ in, uint64_t n,
                                                             uint64_t* __restrict__ partial) {
  uint64_t base = uint64_t(blockIdx.x) * kScanTile + uint64_t(threadIdx.x) * kScanPer;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; k++)
    if (base + k < n) s += in[base + k];
  uint64_t tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_partials(uint64_t* __restrict__ partial, uint64_t np,
                                                               uint64_t* __restrict__ total_out) {
  uint64_t carry = 0;
  for (uint64_t base = 0; base < np; base += kScanThreads) {
    uint64_t i = base + threadIdx.x;
    uint64_t v = i < np ? partial[i] : 0;
    uint64_t tot;
    uint64_t ex = block_excl_scan(v, &tot);
    if (i < np) partial[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *total_out = carry;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_down(const uint16_t* __restrict__ in, uint64_t n,
                                                           const uint64_t* __restrict__ partial,
                                                           uint64_t* __restrict__ out) {
  uint64_t base = uint64_t(blockIdx.x) * kScanTile + uint64_t(threadIdx.x) * kScanPer;
  uint64_t vals[kScanPer];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    vals[k] = (base + k < n) ? in[base + k] : 0;
    s += vals[k];
  }
  uint64_t tot;
  uint64_t ex = block_excl_scan(s, &tot) + partial[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    if (base + k < n) out[base + k] = ex;
    ex += vals[k];
  }
}

// workspace layout: [partials: nparts u64]; out has n+1 entries (out[n] = total)
void scan_u16(const uint16_t* in, uint64_t* out, uint64_t n, void* workspace, hipStream_t stream) {
  uint64_t nparts = (n + kScanTile - 1) / kScanTile;
  if (nparts == 0) {
    RMM_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(uint64_t), stream));
    return;
  }
  uint64_t* partial = static_cast<uint64_t*>(workspace);
  hipLaunchKernelGGL(k_scan_reduce, dim3(uint32_t(nparts)), dim3(kScanThreads), 0, stream, in, n, partial);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kScanThreads), 0, stream, partial, nparts, out + n);
  hipLaunchKernelGGL(k_scan_down, dim3(uint32_t(nparts)), dim3(kScanThreads), 0, stream, in, n, partial, out);
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K4 compress / decompress

constexpr uint32_t kCMagic = 0x434d4d52u;  // "RMMC"
constexpr int kCBlock = 256;               // elements per compression block
constexpr int kCWavesPerWG = 4;

struct CHeader {
  uint32_t magic;
  uint32_t elem_bits;
  uint64_t n_elems;
  uint64_t n_blocks;
  uint64_t payload_bytes;
};

__host__ __device__ inline uint64_t c_sizes_off() { return sizeof(CHeader); }
__host__ __device__ inline uint64_t c_payload_off(uint64_t nb) {
  return (sizeof(CHeader) + nb * 2 + 15) & ~uint64_t(15);
}

template <int BITS>
struct ElemT;
template <>
struct ElemT<16> {
  using T = uint16_t;
  using V = uint2;  // 4 elements per lane
  static constexpr int kLowBytes = 1;
};
template <>
struct ElemT<32> {
  using T = uint32_t;
  using V = uint4;
  static constexpr int kLowBytes = 3;
};

template <int BITS>
__device__ __forceinline__ uint32_t rotl1(uint32_t x) {
  if constexpr (BITS == 16) return ((x << 1) | (x >> 15)) & 0xFFFFu;
  else return (x << 1) | (x >> 31);
}
template <int BITS>
__device__ __forceinline__ uint32_t rotr1(uint32_t x) {
  if constexpr (BITS == 16) return ((x >> 1) | (x << 15)) & 0xFFFFu;
  else return (x >> 1) | (x << 31);
}

// Load this lane's 4 elements of block `blk` (zero past n), rotated.
template <int BITS>
__device__ __forceinline__ void load4(const typename ElemT<BITS>::T* src, uint64_t n, uint64_t blk, int lane,
                                      uint32_t v[4]) {
  uint64_t e0 = blk * kCBlock + uint64_t(lane) * 4;
  if (e0 + 4 <= n) {
    using V = typename ElemT<BITS>::V;
    V x = *reinterpret_cast<const V*>(src + e0);
    if constexpr (BITS == 16) {
      v[0] = x.x & 0xFFFFu; v[1] = x.x >> 16; v[2] = x.y & 0xFFFFu; v[3] = x.y >> 16;
    } else {
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = (e0 + k < n) ? uint32_t(src[e0 + k]) : 0u;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = rotl1<BITS>(v[k]);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

template <int BITS>
__device__ __forceinline__ void block_params(const uint32_t v[4], uint32_t* mn, uint32_t* w, uint32_t* zero,
                                             uint32_t* size) {
  constexpr int kShift = BITS - 8;
  uint32_t lmin = 255, lmax = 0, lor = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t e = v[k] >> kShift;
    lmin = min(lmin, e);
    lmax = max(lmax, e);
    lor |= v[k];
  }
  lmin = wave_min(lmin);
  lmax = wave_max(lmax);
  lor = wave_or(lor);
  uint32_t range = lmax - lmin;
  uint32_t width = range == 0 ? 0 : 32 - __builtin_clz(range);
  *mn = lmin;
  *w = width;
  *zero = lor == 0;
  *size = lor == 0 ? 4u : 4u + 32u * width + uint32_t(kCBlock * ElemT<BITS>::kLowBytes);
}

template <int BITS>
__global__ __launch_bounds__(64 * kCWavesPerWG) void k_compress_sizes(const typename ElemT<BITS>::T* __restrict__ src,
                                                                       uint64_t n, uint64_t nb,
                                                                       uint16_t* __restrict__ sizes) {
  const int lane = threadIdx.x & 63;
  const uint64_t blk = uint64_t(blockIdx.x) * kCWavesPerWG + (threadIdx.x >> 6);
  if (blk >= nb) return;
  uint32_t v[4];
  load4<BITS>(src, n, blk, lane, v);
  uint32_t mn, w, z, sz;
  block_params<BITS>(v, &mn, &w, &z, &sz);
  if (lane == 0) sizes[blk] = uint16_t(sz);
}

template <int BITS>
__global__ __launch_bounds__(64 * kCWavesPerWG) void k_compress_write(const typename ElemT<BITS>::T* __restrict__ src,
                                                                       uint64_t n, uint64_t nb,
                                                                       const uint64_t* __restrict__ offs,
                                                                       uint8_t* __restrict__ payload) {
  __shared__ uint32_t bits[kCWavesPerWG][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t blk = uint64_t(blockIdx.x) * kCWavesPerWG + wv;
  bits[wv][lane] = 0;
  __syncthreads();
  uint32_t v[4] = {0, 0, 0, 0};
  uint32_t mn = 0, w = 0, z = 1, sz = 0;
  if (blk < nb) {
    load4<BITS>(src, n, blk, lane, v);
    block_params<BITS>(v, &mn, &w, &z, &sz);
  }
  uint8_t* out = payload + (blk < nb ? offs[blk] : 0);
  if (blk < nb && lane == 0) *reinterpret_cast<uint32_t*>(out) = mn | (w << 8) | (z << 16);
  constexpr int kShift = BITS - 8;
  if (blk < nb && !z && w > 0) {
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) packed |= ((v[k] >> kShift) - mn) << (k * w);
    uint32_t bitoff = 4u * w * uint32_t(lane);
    uint32_t wi = bitoff >> 5, sh = bitoff & 31;
    atomicOr(&bits[wv][wi], packed << sh);
    if (sh + 4 * w > 32) atomicOr(&bits[wv][wi + 1], packed >> (32 - sh));
  }
  __syncthreads();
  if (blk < nb && !z) {
    uint32_t* o32 = reinterpret_cast<uint32_t*>(out + 4);
    if (uint32_t(lane) < 8 * w) o32[lane] = bits[wv][lane];
    uint8_t* low = out + 4 + 32 * w;
    if constexpr (BITS == 16) {
      uint32_t lb = (v[0] & 0xFF) | ((v[1] & 0xFF) << 8) | ((v[2] & 0xFF) << 16) | ((v[3] & 0xFF) << 24);
      reinterpret_cast<uint32_t*>(low)[lane] = lb;
    } else {
#pragma unroll
      for (int p = 0; p < 3; p++) {
        uint32_t lb = ((v[0] >> (8 * p)) & 0xFF) | (((v[1] >> (8 * p)) & 0xFF) << 8) |
                      (((v[2] >> (8 * p)) & 0xFF) << 16) | (((v[3] >> (8 * p)) & 0xFF) << 24);
        reinterpret_cast<uint32_t*>(low + p * kCBlock)[lane] = lb;
      }
    }
  }
}

template <int BITS>
__global__ __launch_bounds__(64 * kCWavesPerWG) void k_decompress(const uint8_t* __restrict__ payload,
                                                                   const uint64_t* __restrict__ offs, uint64_t n,
                                                                   uint64_t nb, typename ElemT<BITS>::T* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const uint64_t blk = uint64_t(blockIdx.x) * kCWavesPerWG + (threadIdx.x >> 6);
  if (blk >= nb) return;
  const uint8_t* in = payload + offs[blk];
  uint32_t h = *reinterpret_cast<const uint32_t*>(in);
  uint32_t mn = h & 0xFF, w = (h >> 8) & 0xFF, z = (h >> 16) & 1;
  uint32_t v[4] = {0, 0, 0, 0};
  constexpr int kShift = BITS - 8;
  if (!z) {
    uint32_t e[4] = {mn, mn, mn, mn};
    if (w > 0) {
      const uint32_t* b32 = reinterpret_cast<const uint32_t*>(in + 4);
      uint32_t bitoff = 4u * w * uint32_t(lane);
      uint32_t wi = bitoff >> 5, sh = bitoff & 31;
      uint64_t both = uint64_t(b32[wi]);
      if (sh + 4 * w > 32) both |= uint64_t(b32[wi + 1]) << 32;
      uint32_t packed = uint32_t(both >> sh);
      uint32_t mask = (w >= 32) ? 0xFFFFFFFFu : ((1u << w) - 1u);
#pragma unroll
      for (int k = 0; k < 4; k++) e[k] = mn + ((packed >> (k * w)) & mask);
    }
    const uint8_t* low = in + 4 + 32 * w;
    if constexpr (BITS == 16) {
      uint32_t lb = reinterpret_cast<const uint32_t*>(low)[lane];
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = (e[k] << kShift) | ((lb >> (8 * k)) & 0xFF);
    } else {
      uint32_t l0 = reinterpret_cast<const uint32_t*>(low)[lane];
      uint32_t l1 = reinterpret_cast<const uint32_t*>(low + kCBlock)[lane];
      uint32_t l2 = reinterpret_cast<const uint32_t*>(low + 2 * kCBlock)[lane];
#pragma unroll
      for (int k = 0; k < 4; k++)
        v[k] = (e[k] << kShift) | ((l0 >> (8 * k)) & 0xFF) | (((l1 >> (8 * k)) & 0xFF) << 8) |
               (((l2 >> (8 * k)) & 0xFF) << 16);
    }
  }
  uint64_t e0 = blk * kCBlock + uint64_t(lane) * 4;
  using T = typename ElemT<BITS>::T;
  if (e0 + 4 <= n) {
    if constexpr (BITS == 16) {
      uint2 x;
      x.x = rotr1<16>(v[0]) | (rotr1<16>(v[1]) << 16);
      x.y = rotr1<16>(v[2]) | (rotr1<16>(v[3]) << 16);
      *reinterpret_cast<uint2*>(dst + e0) = x;
    } else {
      uint4 x;
      x.x = rotr1<32>(v[0]); x.y = rotr1<32>(v[1]); x.z = rotr1<32>(v[2]); x.w = rotr1<32>(v[3]);
      *reinterpret_cast<uint4*>(dst + e0) = x;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (e0 + k < n) dst[e0 + k] = T(rotr1<BITS>(v[k]));
  }
}

__global__ void k_write_header(uint8_t* dst, uint32_t bits, uint64_t n, uint64_t nb, const uint64_t* total) {
  CHeader* h = reinterpret_cast<CHeader*>(dst);
  h->magic = kCMagic;
  h->elem_bits = bits;
  h->n_elems = n;
  h->n_blocks = nb;
  h->payload_bytes = *total;
}

uint64_t compress_bound(uint64_t n_elems, int elem_bits) {
  uint64_t nb = (n_elems + kCBlock - 1) / kCBlock;
  uint64_t per = 4 + 256 + uint64_t(kCBlock) * (elem_bits == 16 ? 1 : 3);
  return c_payload_off(nb) + nb * per;
}

uint64_t compress_workspace(uint64_t n_elems) {
  uint64_t nb = (n_elems + kCBlock - 1) / kCBlock;
  uint64_t nparts = (nb + kScanTile - 1) / kScanTile;
  // offsets (nb+1) + partials
  return ((nb + 1) * 8 + 255) / 256 * 256 + (nparts + 1) * 8 + 256;
}

uint64_t compress(const void* src, uint64_t n, int elem_bits, void* dst, void* workspace, hipStream_t stream,
                  bool readback) {
  if (elem_bits != 16 && elem_bits != 32) throw std::invalid_argument("compress: elem_bits must be 16 or 32");
  uint64_t nb = (n + kCBlock - 1) / kCBlock;
  uint8_t* d = static_cast<uint8_t*>(dst);
  uint16_t* sizes = reinterpret_cast<uint16_t*>(d + c_sizes_off());
  uint8_t* payload = d + c_payload_off(nb);
  uint64_t* offs = static_cast<uint64_t*>(workspace);
  void* scan_ws = static_cast<uint8_t*>(workspace) + ((nb + 1) * 8 + 255) / 256 * 256;
  uint32_t grid = uint32_t((nb + kCWavesPerWG - 1) / kCWavesPerWG);
  if (nb > 0) {
    if (elem_bits == 16)
      hipLaunchKernelGGL(k_compress_sizes<16>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream,
                         static_cast<const uint16_t*>(src), n, nb, sizes);
    else
      hipLaunchKernelGGL(k_compress_sizes<32>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream,
                         static_cast<const uint32_t*>(src), n, nb, sizes);
  }
  scan_u16(sizes, offs, nb, scan_ws, stream);
  if (nb > 0) {
    if (elem_bits == 16)
      hipLaunchKernelGGL(k_compress_write<16>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream,
                         static_cast<const uint16_t*>(src), n, nb, offs, payload);
    else
      hipLaunchKernelGGL(k_compress_write<32>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream,
                         static_cast<const uint32_t*>(src), n, nb, offs, payload);
  }
  hipLaunchKernelGGL(k_write_header, dim3(1), dim3(1), 0, stream, d, uint32_t(elem_bits), n, nb, offs + nb);
  RMM_HIP_CHECK(hipGetLastError());
  if (!readback) return 0;  // the size stays on the device (CHeader::payload_bytes)
  uint64_t total = 0;
  RMM_HIP_CHECK(hipMemcpyAsync(&total, offs + nb, sizeof(total), hipMemcpyDeviceToHost, stream));
  RMM_HIP_CHECK(hipStreamSynchronize(stream));
  return c_payload_off(nb) + total;
}

// ---- device-placed spill (GpuStore::SpillTransfer): chunk c of a spill is written by a copy kernel straight into
// the registered host arena at a device-resident offset, so the host never waits for a chunk's compressed size.
// The chunk goes compressed when its stream (header + sizes + payload, read from the compress() output on the
// device) saves at least len / 16, else raw; every chunk starts 64-byte aligned.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t spill_chunk_bytes(const uint8_t* scratch, uint64_t len, bool try_c, bool* comp) {
  uint64_t t = len;
  *comp = false;
  if (try_c) {
    const CHeader* h = reinterpret_cast<const CHeader*>(scratch);
    t = c_payload_off(h->n_blocks) + h->payload_bytes;
    *comp = t < len - len / 16;
  }
  return *comp ? t : len;
}

__global__ __launch_bounds__(256) void k_spill_commit(const uint8_t* __restrict__ scratch, const uint8_t* __restrict__ raw,
                                                      uint64_t len, int try_c, uint8_t* host, const uint64_t* base) {
  bool comp;
  const uint64_t n = spill_chunk_bytes(scratch, len, try_c != 0, &comp);
  const uint8_t* src = comp ? scratch : raw;
  uint8_t* dst = host + *base;  // 64-byte aligned
  const uint64_t nv = n / 16;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nv; i += stride)
    __builtin_nontemporal_store(reinterpret_cast<const u32x4v*>(src)[i], reinterpret_cast<u32x4v*>(dst) + i);
  if (blockIdx.x == 0 && threadIdx.x < n % 16) dst[nv * 16 + threadIdx.x] = src[nv * 16 + threadIdx.x];
}

__global__ void k_spill_advance(const uint8_t* __restrict__ scratch, uint64_t len, int try_c, uint64_t* base,
                                uint64_t* csize) {
  bool comp;
  const uint64_t n = spill_chunk_bytes(scratch, len, try_c != 0, &comp);
  *csize = comp ? n : 0;
  *base += (n + 63) & ~uint64_t(63);
}

void spill_commit(const void* scratch, const void* raw, uint64_t len, bool try_compressed, void* host_dev,
                  uint64_t* base_dev, uint64_t* csize_dev, hipStream_t stream) {
  if ((reinterpret_cast<uintptr_t>(raw) | reinterpret_cast<uintptr_t>(scratch) | reinterpret_cast<uintptr_t>(host_dev)) & 15)
    throw std::invalid_argument("spill_commit: 16-byte aligned source, scratch and host mapping");
  const uint32_t grid = uint32_t(std::min<uint64_t>(1024, std::max<uint64_t>(1, (len / 16 + 255) / 256)));
  hipLaunchKernelGGL(k_spill_commit, dim3(grid), dim3(256), 0, stream, static_cast<const uint8_t*>(scratch),
                     static_cast<const uint8_t*>(raw), len, int(try_compressed), static_cast<uint8_t*>(host_dev),
                     base_dev);
  hipLaunchKernelGGL(k_spill_advance, dim3(1), dim3(1), 0, stream, static_cast<const uint8_t*>(scratch), len,
                     int(try_compressed), base_dev, csize_dev);
  RMM_HIP_CHECK(hipGetLastError());
}

void decompress(const void* src, void* dst, uint64_t n, int elem_bits, void* workspace, hipStream_t stream) {
  uint64_t nb = (n + kCBlock - 1) / kCBlock;
  if (nb == 0) return;
  const uint8_t* s = static_cast<const uint8_t*>(src);
  const uint16_t* sizes = reinterpret_cast<const uint16_t*>(s + c_sizes_off());
  const uint8_t* payload = s + c_payload_off(nb);
  uint64_t* offs = static_cast<uint64_t*>(workspace);
  void* scan_ws = static_cast<uint8_t*>(workspace) + ((nb + 1) * 8 + 255) / 256 * 256;
  scan_u16(sizes, offs, nb, scan_ws, stream);
  uint32_t grid = uint32_t((nb + kCWavesPerWG - 1) / kCWavesPerWG);
  if (elem_bits == 16)
    hipLaunchKernelGGL(k_decompress<16>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream, payload, offs, n, nb,
                       static_cast<uint16_t*>(dst));
  else
    hipLaunchKernelGGL(k_decompress<32>, dim3(grid), dim3(64 * kCWavesPerWG), 0, stream, payload, offs, n, nb,
                       static_cast<uint32_t*>(dst));
  RMM_HIP_CHECK(hipGetLastError());
}

// ============================================================== K5 fused PPO loss

// stats[0..5] = sum(-surr), sum(vf_clipped), sum(entropy), sum(clipped?1:0), sum(total), sum(vf_explained num)
constexpr int kLossThreads = 256;

__global__ __launch_bounds__(kLossThreads) void k_ppo_loss(const float* __restrict__ logp_new,
                                                          const float* __restrict__ logp_old,
                                                          const float* __restrict__ adv,
                                                          const float* __restrict__ v_new,
                                                          const float* __restrict__ v_tgt,
                                                          const float* __restrict__ ent,
                                                          float* __restrict__ g_logp, float* __restrict__ g_v,
                                                          float* __restrict__ g_ent, float* __restrict__ stats,
                                                          int64_t n, float clip, float vf_clip, float vf_coeff,
                                                          float ent_coeff) {
  float s_pol = 0.f, s_vf = 0.f, s_ent = 0.f, s_clip = 0.f;
  const float inv_n = 1.f / float(n);
  for (int64_t i = int64_t(blockIdx.x) * kLossThreads + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * kLossThreads) {
    const float r = __expf(logp_new[i] - logp_old[i]);
    const float a = adv[i];
    const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
    const float s1 = r * a, s2 = rc * a;
    const bool take_unclipped = s1 <= s2;
    const float surr = take_unclipped ? s1 : s2;
    // d(-surr)/dlogp_new: the chosen branch's derivative (clamp passes grad inside the range)
    const bool inside = (r >= 1.f - clip) && (r <= 1.f + clip);
    const float dsurr = (take_unclipped || inside) ? r * a : 0.f;
    g_logp[i] = -dsurr * inv_n;
    const float d = v_new[i] - v_tgt[i];
    const float vf = d * d;
    const bool vf_in = vf < vf_clip;
    g_v[i] = vf_in ? vf_coeff * 2.f * d * inv_n : 0.f;
    g_ent[i] = -ent_coeff * inv_n;
    s_pol += -surr;
    s_vf += vf_in ? vf : vf_clip;
    s_ent += ent[i];
    s_clip += (fabsf(r - 1.f) > clip) ? 1.f : 0.f;
  }
  // wave reduce then LDS across the 4 waves, one atomic per workgroup per stat
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s_pol += __shfl_xor(s_pol, o, 64);
    s_vf += __shfl_xor(s_vf, o, 64);
    s_ent += __shfl_xor(s_ent, o, 64);
    s_clip += __shfl_xor(s_clip, o, 64);
  }
  __shared__ float red[4][kLossThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = s_pol;
    red[1][w] = s_vf;
    red[2][w] = s_ent;
    red[3][w] = s_clip;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float t = 0.f;
    for (int k = 0; k < kLossThreads / 64; k++) t += red[threadIdx.x][k];
    atomicAdd(&stats[threadIdx.x], t);
  }
}

void ppo_loss_fwd(const float* logp_new, const float* logp_old, const float* adv, const float* v_new,
                  const float* /*v_old*/, const float* v_tgt, const float* ent, float* grad_logp, float* grad_v,
                  float* grad_ent, float* stats, int64_t n, float clip, float vf_clip, float vf_coeff,
                  float ent_coeff, hipStream_t stream) {
  if (n <= 0) return;
  RMM_HIP_CHECK(hipMemsetAsync(stats, 0, 4 * sizeof(float), stream));
  int64_t blocks = std::min<int64_t>((n + kLossThreads - 1) / kLossThreads, 1024);
  hipLaunchKernelGGL(k_ppo_loss, dim3(uint32_t(blocks)), dim3(kLossThreads), 0, stream, logp_new, logp_old, adv,
                     v_new, v_tgt, ent, grad_logp, grad_v, grad_ent, stats, n, clip, vf_clip, vf_coeff, ent_coeff);
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
