// Split-bf16 ("bf16x3") arithmetic for the precision-matched (fp32) learner and rollout policy.
//
// gfx950 has no TF32 / xf32 MFMA, and v_mfma_f32_16x16x4_f32 runs at 1/16 of the bf16 MFMA rate
// (MI355X_MICROARCH.md constants table: 32 cycles per 2,048 FLOP vs 16 cycles per 16,384). So the fp32
// path carries every fp32 operand as an unevaluated pair x = hi + lo of two bf16 values
// (hi = RNE(x), lo = RNE(x - hi); ~17 significant bits, |x - hi - lo| <= 2^-17 |x|) and multiplies
// pairs with THREE bf16 MFMAs, hi*hi + hi*lo + lo*hi, accumulating in fp32 (the dropped lo*lo term is
// <= 2^-16 relative). One fp32-equivalent product costs 48 cycles per 16x16x32 block instead of 256
// with the fp32 MFMA. Frames are integers 0..255, exact in bf16: frame products need two MFMAs.
// Master weights, Adam moments, gradient reductions, loss math and every accumulator are fp32; the
// optimizer writes the split pair of each weight next to the fp32 master (adam_device.h).
// Storage: a split tensor is two bf16 planes of the same shape (hi plane, lo plane).
#pragma once
#include <hip/hip_bf16.h>

#include "common.h"

namespace rmm {
namespace hip {
namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// a read-only split tensor (hi / lo planes) and its writable twin
struct CPair {
  const unsigned short* hi = nullptr;
  const unsigned short* lo = nullptr;
};
struct Pair {
  unsigned short* hi = nullptr;
  unsigned short* lo = nullptr;
};

__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ bf16x8 as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// x -> (hi, lo) bf16 bits (hardware v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ void split(float x, unsigned short& hi, unsigned short& lo) {
  const __bf16 h = static_cast<__bf16>(x);
  const float r = x - static_cast<float>(h);
  hi = __builtin_bit_cast(unsigned short, h);
  lo = __builtin_bit_cast(unsigned short, static_cast<__bf16>(r));
}
__device__ __forceinline__ float join(unsigned short hi, unsigned short lo) { return bf2f(hi) + bf2f(lo); }
__device__ __forceinline__ float join(const CPair& p, int64_t i) { return bf2f(p.hi[i]) + bf2f(p.lo[i]); }

// store one fp32 value as its split pair
__device__ __forceinline__ void store1(const Pair& p, int64_t i, float x) {
  unsigned short h, l;
  split(x, h, l);
  p.hi[i] = h;
  p.lo[i] = l;
}
// 4 consecutive values (8-B aligned index) as two 8-byte stores
__device__ __forceinline__ void store4(const Pair& p, int64_t i, const float (&v)[4]) {
  unsigned short h[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; k++) split(v[k], h[k], l[k]);
  *reinterpret_cast<uint2*>(p.hi + i) =
      make_uint2(uint32_t(h[0]) | (uint32_t(h[1]) << 16), uint32_t(h[2]) | (uint32_t(h[3]) << 16));
  *reinterpret_cast<uint2*>(p.lo + i) =
      make_uint2(uint32_t(l[0]) | (uint32_t(l[1]) << 16), uint32_t(l[2]) | (uint32_t(l[3]) << 16));
}

// The product of two split fragments accumulates into two chains: `hh` (hi*hi) and `x` (the cross
// terms, smaller by 2^-8): two independent MFMA dependency chains instead of one of length 3.
struct Acc {
  f32x4 hh, x;
};
__device__ __forceinline__ Acc acc0() { return Acc{f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}}; }
__device__ __forceinline__ void mma3(Acc& c, bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl) {
  c.x = mfma(al, bh, c.x);
  c.x = mfma(ah, bl, c.x);
  c.hh = mfma(ah, bh, c.hh);
}
// one operand exact in bf16 (frames, the ones row of a bias reduction): two MFMAs
__device__ __forceinline__ void mma2a(Acc& c, bf16x8 a, bf16x8 bh, bf16x8 bl) {
  c.x = mfma(a, bl, c.x);
  c.hh = mfma(a, bh, c.hh);
}
__device__ __forceinline__ f32x4 total(const Acc& c) { return c.x + c.hh; }

__device__ __forceinline__ bf16x8 ld8(const unsigned short* p) { return as_bf(*reinterpret_cast<const u16x8*>(p)); }

}  // namespace x3
}  // namespace hip
}  // namespace rmm
