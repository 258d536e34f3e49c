// K11 — key partitioning for the GPU all-to-all shuffle (experimental/gpu_shuffle.py).
//
// One shuffle round on one MI355X: every row (int64 key + fixed-size payload) goes to destination
// dest(key) = splitmix64(key) % R ("hash"), key mod R ("mod") or floor(key·R / 2^64) with the key read
// as unsigned ("range": R equal key ranges, what a distributed sort needs). Rows are reordered so each
// destination's rows are contiguous — exactly the layout `all_to_all_single` with split sizes
// sends over RCCL/xGMI. Two launches and a tiny scan:
//   k_part_hist    — per-workgroup destination histogram in LDS (workgroup w owns rows
//                    [w*chunk, (w+1)*chunk)) → counts[w][R];
//   (host-side torch scan over the [W, R] matrix → per-(workgroup, destination) offsets)
//   k_part_scatter — the same rows again; LDS cursors hand out slots, key and payload (16-B vector
//                    copies when the row size allows) land at their final position.
// Order inside a destination block is not stable (LDS atomics): a shuffle does not need it.
#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

__device__ __forceinline__ uint32_t part_dest(int64_t key, int R, int mode) {
  if (mode == 2) return uint32_t(__umul64hi(uint64_t(key), uint64_t(R)));  // range: R equal slices of the u64 keys
  if (mode == 1) {  // mod
    const int64_t m = key % R;
    return uint32_t(m < 0 ? m + R : m);
  }
  uint64_t x = uint64_t(key);  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return uint32_t(x % uint64_t(R));
}

constexpr int kPartMaxR = 1024;

__global__ __launch_bounds__(256) void k_part_hist(const int64_t* __restrict__ keys, int64_t n, int64_t chunk, int R,
                                                   int mode, int64_t* __restrict__ counts) {
  __shared__ uint32_t hist[kPartMaxR];
  for (int r = threadIdx.x; r < R; r += blockDim.x) hist[r] = 0;
  __syncthreads();
  const int64_t lo = int64_t(blockIdx.x) * chunk, hi = min(n, lo + chunk);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&hist[part_dest(keys[i], R, mode)], 1u);
  __syncthreads();
  for (int r = threadIdx.x; r < R; r += blockDim.x) counts[int64_t(blockIdx.x) * R + r] = hist[r];
}

__global__ __launch_bounds__(256) void k_part_scatter(const int64_t* __restrict__ keys, const uint8_t* __restrict__ vals,
                                                      int64_t n, int64_t chunk, int64_t row_bytes, int R, int mode,
                                                      const int64_t* __restrict__ offsets,
                                                      int64_t* __restrict__ out_keys, uint8_t* __restrict__ out_vals) {
  __shared__ unsigned long long cursor[kPartMaxR];
  for (int r = threadIdx.x; r < R; r += blockDim.x) cursor[r] = uint64_t(offsets[int64_t(blockIdx.x) * R + r]);
  __syncthreads();
  const int64_t lo = int64_t(blockIdx.x) * chunk, hi = min(n, lo + chunk);
  const bool vec = (row_bytes & 15) == 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const int64_t k = keys[i];
    const int64_t pos = int64_t(atomicAdd(&cursor[part_dest(k, R, mode)], 1ull));
    out_keys[pos] = k;
    if (row_bytes) {
      const uint8_t* s = vals + i * row_bytes;
      uint8_t* d = out_vals + pos * row_bytes;
      if (vec) {
        for (int64_t b = 0; b < row_bytes; b += 16)
          *reinterpret_cast<uint4*>(d + b) = *reinterpret_cast<const uint4*>(s + b);
      } else {
        for (int64_t b = 0; b < row_bytes; b++) d[b] = s[b];
      }
    }
  }
}

int64_t partition_groups(int64_t n) { return std::max<int64_t>(1, std::min<int64_t>((n + 4095) / 4096, 2048)); }

void partition_hist(const int64_t* keys, int64_t n, int R, int mode, int64_t* counts, hipStream_t stream) {
  if (R <= 0 || R > kPartMaxR) throw std::invalid_argument("partition: 1 <= R <= 1024");
  const int64_t G = partition_groups(n), chunk = std::max<int64_t>((n + G - 1) / G, 1);
  hipLaunchKernelGGL(k_part_hist, dim3(uint32_t(G)), dim3(256), 0, stream, keys, n, chunk, R, mode, counts);
  RMM_HIP_CHECK(hipGetLastError());
}

void partition_scatter(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, int R, int mode,
                       const int64_t* offsets, int64_t* out_keys, void* out_vals, hipStream_t stream) {
  if (R <= 0 || R > kPartMaxR) throw std::invalid_argument("partition: 1 <= R <= 1024");
  const int64_t G = partition_groups(n), chunk = std::max<int64_t>((n + G - 1) / G, 1);
  hipLaunchKernelGGL(k_part_scatter, dim3(uint32_t(G)), dim3(256), 0, stream, keys, static_cast<const uint8_t*>(vals),
                     n, chunk, row_bytes, R, mode, offsets, out_keys, static_cast<uint8_t*>(out_vals));
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
