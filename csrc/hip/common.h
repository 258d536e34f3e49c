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
}  // namespace hip
}  // namespace rmm
#endif
