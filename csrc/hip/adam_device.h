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
// wlo (optional, the split-bf16 fp32 learner, x3_device.h): wbf16 receives hi = RNE(w) and wlo the
// residual lo = RNE(w - hi), so the kernels read the fp32 master as the pair hi + lo.
__device__ __forceinline__ uint32_t bf16x2_lo(float a, float b) {
  const float ra = a - __bfloat162float(__float2bfloat16(a)), rb = b - __bfloat162float(__float2bfloat16(b));
  return bf16x2_rn(ra, rb);
}
template <typename TG, bool VEC, int U>
__device__ __forceinline__ void adam_span(float* __restrict__ master, float* __restrict__ m1, float* __restrict__ m2,
                                          const TG* __restrict__ grad, __hip_bfloat16* __restrict__ wbf16,
                                          float grad_scale, const AdamCoef& c, int64_t tid, int64_t nthr, int64_t n,
                                          __hip_bfloat16* __restrict__ wlo = nullptr,
                                          const float* __restrict__ grad2 = nullptr) {
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
          if (grad2) {  // a second partial of the same gradient (K12x row parts), added in a fixed order
            const float4 q = *reinterpret_cast<const float4*>(grad2 + i);
            g[u][0] += q.x, g[u][1] += q.y, g[u][2] += q.z, g[u][3] += q.w;
          }
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
          if (wlo)
            *reinterpret_cast<uint2*>(wlo + i) = make_uint2(bf16x2_lo(w[u].x, w[u].y), bf16x2_lo(w[u].z, w[u].w));
        }
      }
    }
    scalar_from = nv << 2;
  }
  for (int64_t i = scalar_from + tid; i < n; i += nthr) {
    float a = m1[i], b = m2[i];
    const float w = adam_one(master[i], (grad2 ? adam_ld1(grad, i) + grad2[i] : adam_ld1(grad, i)) * grad_scale, a, b, c);
    m1[i] = a;
    m2[i] = b;
    master[i] = w;
    if (wbf16) wbf16[i] = __float2bfloat16(w);
    if (wlo) wlo[i] = __float2bfloat16(w - __bfloat162float(__float2bfloat16(w)));
  }
}

// adam_span's vector pass over the dense weight [256][K] of a K12 row split whose finalize was deferred:
// each group of 4 gradients (same row m, columns k..k+3 of one 32-column K12 group) is a float4 at the
// same place of every member's partial block; the members are summed in order and rounded to bf16
// exactly as k_dense_split_finalize does, so the update is bit-identical to finalize -> K6.
__device__ __forceinline__ int64_t k12_part_index(int64_t e, int64_t K, int rs, int h) {
  const int64_t m = e / K, k = e - m * K;
  const int64_t group = k >> 5;
  const int c = int(k & 31), jt = c >> 4, r = c & 15;
  const int hi = int(m >> 7), wave = int((m >> 4) & 7), g = int((m & 15) >> 2), i = int(m & 3);
  const int slot = (hi * 2 + jt) * 4 + i, tid = wave * 64 + g * 16 + r;
  return ((group * rs + h) * 20 + slot) * 512 + tid;
}
template <int U>
__device__ __forceinline__ void adam_span_split(float* __restrict__ master, float* __restrict__ m1,
                                                float* __restrict__ m2, const float* __restrict__ part, int rs,
                                                int64_t K, __hip_bfloat16* __restrict__ wbf16, float grad_scale,
                                                const AdamCoef& c, int64_t tid, int64_t nthr, int64_t n) {
  const int64_t nv = n >> 2;  // n = 256 K, K % 32 == 0: whole groups of 4 in one 32-column K12 group
  for (int64_t v0 = tid; v0 < nv; v0 += nthr * U) {
    float g[U][4];
    float4 w[U], a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t v = v0 + u * nthr;
      if (v < nv) {
        const int64_t i = v << 2;
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int h = 0; h < rs; h++) {
          const float4 p = *reinterpret_cast<const float4*>(part + k12_part_index(i, K, rs, h));
          t.x += p.x, t.y += p.y, t.z += p.z, t.w += p.w;
        }
        g[u][0] = __uint_as_float(uint32_t(bf16_bits_rn(t.x)) << 16);
        g[u][1] = __uint_as_float(uint32_t(bf16_bits_rn(t.y)) << 16);
        g[u][2] = __uint_as_float(uint32_t(bf16_bits_rn(t.z)) << 16);
        g[u][3] = __uint_as_float(uint32_t(bf16_bits_rn(t.w)) << 16);
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
        *reinterpret_cast<uint2*>(wbf16 + i) = make_uint2(bf16x2_rn(w[u].x, w[u].y), bf16x2_rn(w[u].z, w[u].w));
      }
    }
  }
}

}  // namespace hip
}  // namespace rmm
