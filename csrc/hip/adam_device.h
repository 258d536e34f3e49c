// K6's per-element Adam pass as a device function: the flat Adam kernel (rl_kernels.hip) and the
// trunk-reduce launch (conv_kernels.hip, Adam workgroups beside the partial-sum workgroups) run the
// SAME code over their thread ranges, so the two layouts give bit-identical parameters.
#pragma once
#include <hip/hip_bf16.h>

#include "common.h"

namespace rmm {
namespace hip {

__device__ __forceinline__ void adam_load4(const float* g, int64_t i, float (&o)[4]) {
  const float4 v = *reinterpret_cast<const float4*>(g + i);
  o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
}
__device__ __forceinline__ void adam_load4(const __hip_bfloat16* g, int64_t i, float (&o)[4]) {
  const uint2 v = *reinterpret_cast<const uint2*>(g + i);  // 4 bf16 = 8 B
  o[0] = __uint_as_float(v.x << 16), o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16), o[3] = __uint_as_float(v.y & 0xffff0000u);
}
__device__ __forceinline__ float adam_ld1(const float* g, int64_t i) { return g[i]; }
__device__ __forceinline__ float adam_ld1(const __hip_bfloat16* g, int64_t i) { return __bfloat162float(g[i]); }
__device__ __forceinline__ uint32_t bf16x2_rn(float a, float b) {
  const uint32_t lo = __bfloat16_as_ushort(__float2bfloat16(a)), hi = __bfloat16_as_ushort(__float2bfloat16(b));
  return lo | (hi << 16);
}

// Elements [0, n) of the flat buffers over threads tid = 0 .. nthr-1. VEC: each thread updates U
// groups of 4 consecutive elements with 16-B fp32 and 8-B bf16 accesses (the pass is HBM / Infinity
// Cache bound: 28 B/param), issuing every group's loads before the first update so U x 4 vector
// loads are in flight per lane; the n % 4 tail is done by the first threads. VEC requires 16-B
// aligned fp32 and 8-B aligned bf16 pointers (checked by the host).
template <typename TG, bool VEC, int U>
__device__ __forceinline__ void adam_span(float* __restrict__ master, float* __restrict__ m1, float* __restrict__ m2,
                                          const TG* __restrict__ grad, __hip_bfloat16* __restrict__ wbf16,
                                          float grad_scale, const AdamCoef& c, int64_t tid, int64_t nthr, int64_t n) {
  int64_t scalar_from = 0;
  if constexpr (VEC) {
    const int64_t nv = n >> 2;
    for (int64_t v0 = tid; v0 < nv; v0 += nthr * U) {
      float g[U][4];
      float4 w[U], a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t v = v0 + u * nthr;
        if (v < nv) {
          const int64_t i = v << 2;
          adam_load4(grad, i, g[u]);
          w[u] = *reinterpret_cast<const float4*>(master + i);
          a[u] = *reinterpret_cast<const float4*>(m1 + i);
          b[u] = *reinterpret_cast<const float4*>(m2 + i);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t v = v0 + u * nthr;
        if (v < nv) {
          const int64_t i = v << 2;
          w[u].x = adam_one(w[u].x, g[u][0] * grad_scale, a[u].x, b[u].x, c);
          w[u].y = adam_one(w[u].y, g[u][1] * grad_scale, a[u].y, b[u].y, c);
          w[u].z = adam_one(w[u].z, g[u][2] * grad_scale, a[u].z, b[u].z, c);
          w[u].w = adam_one(w[u].w, g[u][3] * grad_scale, a[u].w, b[u].w, c);
          *reinterpret_cast<float4*>(master + i) = w[u];
          *reinterpret_cast<float4*>(m1 + i) = a[u];
          *reinterpret_cast<float4*>(m2 + i) = b[u];
          if (wbf16)
            *reinterpret_cast<uint2*>(wbf16 + i) = make_uint2(bf16x2_rn(w[u].x, w[u].y), bf16x2_rn(w[u].z, w[u].w));
        }
      }
    }
    scalar_from = nv << 2;
  }
  for (int64_t i = scalar_from + tid; i < n; i += nthr) {
    float a = m1[i], b = m2[i];
    const float w = adam_one(master[i], adam_ld1(grad, i) * grad_scale, a, b, c);
    m1[i] = a;
    m2[i] = b;
    master[i] = w;
    if (wbf16) wbf16[i] = __float2bfloat16(w);
  }
}

}  // namespace hip
}  // namespace rmm
