// Device helpers of the dense-tail kernels (dense_kernels.hip) shared with the persistent rollout
// server (rollout_server.hip): bf16 / MFMA helpers, the K13s split-K unit, the K16 head + sampling row.
#pragma once
#include <hip/hip_bf16.h>

#include "common.h"

namespace rmm {
namespace hip {
namespace dense {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int H = 256;       // hidden width
constexpr int AMAX = 16;     // head width (A+1) limit

__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<unsigned short>(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ bf16x8 as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// One K13s unit (a WM x WN-wave tile of FM x FN 16x16 fragments over K slice `sl`, KW = 4 / (WM WN)
// waves splitting its k-steps and combining through LDS), executed by the 4 waves wave0 .. wave0+3 of
// the calling workgroup. `red` holds (KW-1) x FM*FN x 64 f32x4. Every wave of the workgroup must
// call it the same number of times (it holds a workgroup barrier when KW > 1); a call with
// valid == false computes nothing and stores nothing. Shared by k_dense_fwd_part and the
// persistent rollout server (rollout_server.hip): identical arithmetic → identical partials.
template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void dense_part_unit(const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
                                                int64_t M, int64_t K, int N, int S, float* __restrict__ part,
                                                int64_t sl, int64_t tm, int64_t tn, int wave, bool valid,
                                                f32x4 (*red)[FM * FN][64]) {
  constexpr int KW = 4 / (WM * WN);
  static_assert(WM * WN * KW == 4, "4 waves per unit");
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int sub = wave / KW, kw = wave % KW;
  const int64_t m0 = tm * 16 * FM * WM + (sub / WN) * 16 * FM, n0 = tn * 16 * FN * WN + (sub % WN) * 16 * FN;
  const int64_t steps = K / 32, lo = valid ? steps * sl / S : 0, hi = valid ? steps * (sl + 1) / S : 0;
  const unsigned short* xa[FM];
  const unsigned short* wb[FN];
#pragma unroll
  for (int i = 0; i < FM; i++) xa[i] = x + min(m0 + 16 * i + r, M - 1) * K + 8 * g;
#pragma unroll
  for (int j = 0; j < FN; j++) wb[j] = w + (valid ? (n0 + 16 * j + r) : 0) * K + 8 * g;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // D of this wave's k-steps per batch: D (FM + FN) loads in flight per lane, then D FM FN MFMAs in
  // k order (the same accumulation order for any D). D = 4 (8 at FM = FN = 1) measured slower on
  // MI355X (K13s at M = 500: 8.0 -> 8.6 us; M = 50 unchanged): the loads of one batch already cover
  // the L2 latency with 1024 waves resident
  constexpr int D = 2;
  int64_t k = lo + kw;
  for (; k + (D - 1) * KW < hi; k += D * KW) {
    u16x8 av[D][FM], bv[D][FN];
#pragma unroll
    for (int c = 0; c < D; c++) {
#pragma unroll
      for (int i = 0; i < FM; i++) av[c][i] = *reinterpret_cast<const u16x8*>(xa[i] + (k + KW * c) * 32);
#pragma unroll
      for (int j = 0; j < FN; j++) bv[c][j] = *reinterpret_cast<const u16x8*>(wb[j] + (k + KW * c) * 32);
    }
#pragma unroll
    for (int c = 0; c < D; c++)
#pragma unroll
      for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = mfma(as_bf(av[c][i]), as_bf(bv[c][j]), acc[i][j]);
  }
  if (k < hi) {  // the last < D k-steps: one more batch, loads clamped to a valid step, MFMAs in k order
    u16x8 av[D][FM], bv[D][FN];
#pragma unroll
    for (int c = 0; c < D; c++) {
      const int64_t kc = (k + KW * c < hi) ? k + KW * c : k;
#pragma unroll
      for (int i = 0; i < FM; i++) av[c][i] = *reinterpret_cast<const u16x8*>(xa[i] + kc * 32);
#pragma unroll
      for (int j = 0; j < FN; j++) bv[c][j] = *reinterpret_cast<const u16x8*>(wb[j] + kc * 32);
    }
#pragma unroll
    for (int c = 0; c < D; c++)
      if (k + KW * c < hi)  // wave-uniform
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
          for (int j = 0; j < FN; j++) acc[i][j] = mfma(as_bf(av[c][i]), as_bf(bv[c][j]), acc[i][j]);
  }
  if constexpr (KW > 1) {
    if (kw > 0) {
#pragma unroll
      for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) red[kw - 1][i * FN + j][lane] = acc[i][j];
    }
    __syncthreads();
    if (kw == 0) {
#pragma unroll
      for (int q = 0; q < KW - 1; q++)
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
          for (int j = 0; j < FN; j++) acc[i][j] += red[q][i * FN + j][lane];
    }
    __syncthreads();  // red is free for the next unit
    if (kw != 0) return;
  }
  if (!valid) return;
  float* out = part + (sl * M) * N + n0 + r;
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t row = m0 + 16 * i + 4 * g + e;
      if (row < M)
#pragma unroll
        for (int j = 0; j < FN; j++) out[row * N + 16 * j] = acc[i][j][e];
    }
}

// Consumer prologue of K13s: a lane's 4 hidden values of row rr = bf16(ReLU(Σ_s part[s] + b)),
// summed in slice order (deterministic), rounded exactly like K13's epilogue. Without partials
// (hpart == nullptr) the bf16 hidden row is read as before.
__device__ __forceinline__ void load_hidden4(const unsigned short* __restrict__ hid, const float* __restrict__ hpart,
                                             int S, const unsigned short* __restrict__ hb, int64_t M, int64_t rr,
                                             int lane, float hv[4], uint2& bits) {
  if (hpart == nullptr) {
    bits = *reinterpret_cast<const uint2*>(&hid[rr * H + 4 * lane]);
  } else {
    const uint2 bb = *reinterpret_cast<const uint2*>(&hb[4 * lane]);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* p = hpart + rr * H + 4 * lane;
    // slices loaded 8 at a time before any is summed (a load -> add loop waits out each round trip)
    for (int s0 = 0; s0 < S; s0 += 8) {
      float4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = *reinterpret_cast<const float4*>(p + int64_t(min(s0 + j, S - 1)) * M * H);
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (s0 + j < S) a.x += v[j].x, a.y += v[j].y, a.z += v[j].z, a.w += v[j].w;
    }
    const unsigned short o0 = f2bf(fmaxf(a.x + __uint_as_float(bb.x << 16), 0.f));
    const unsigned short o1 = f2bf(fmaxf(a.y + __uint_as_float(bb.x & 0xffff0000u), 0.f));
    const unsigned short o2 = f2bf(fmaxf(a.z + __uint_as_float(bb.y << 16), 0.f));
    const unsigned short o3 = f2bf(fmaxf(a.w + __uint_as_float(bb.y & 0xffff0000u), 0.f));
    bits = make_uint2(uint32_t(o0) | (uint32_t(o1) << 16), uint32_t(o2) | (uint32_t(o3) << 16));
  }
  hv[0] = __uint_as_float(bits.x << 16), hv[1] = __uint_as_float(bits.x & 0xffff0000u);
  hv[2] = __uint_as_float(bits.y << 16), hv[3] = __uint_as_float(bits.y & 0xffff0000u);
}

// one env row of K16 (one wave): head GEMV + bias, bf16 rounding, Gumbel-max draw, row stores
template <int A1, bool ROUND = true>
__device__ __forceinline__ void heads_sample_row_pre(const float (&hv)[4], const float* whs, const float* bhs,
                                                     const int64_t t, const uint32_t c, uint32_t seed,
                                                     int64_t* __restrict__ act, float* __restrict__ logp,
                                                     float* __restrict__ vf, float* __restrict__ lout,
                                                     int64_t* __restrict__ act_now, int64_t B, int64_t b, int lane);
template <int A1>
__device__ __forceinline__ void heads_sample_row(const unsigned short* __restrict__ hid, const float* whs,
                                                 const float* bhs, const int64_t t, const uint32_t c, uint32_t seed,
                                                 int64_t* __restrict__ act, float* __restrict__ logp,
                                                 float* __restrict__ vf, float* __restrict__ lout,
                                                 int64_t* __restrict__ act_now, int64_t B, int64_t b, int lane,
                                                 const float* __restrict__ hpart, int S,
                                                 const unsigned short* __restrict__ hb) {
  float hv[4];
  uint2 hbits;
  load_hidden4(hid, hpart, S, hb, B, b, lane, hv, hbits);
  heads_sample_row_pre<A1>(hv, whs, bhs, t, c, seed, act, logp, vf, lout, act_now, B, b, lane);
}

// heads_sample_row with this lane's 4 hidden values already loaded (load_hidden4): kernels issue those
// loads before staging Wh into LDS, so the partial-sum round trip overlaps the staging.
// ROUND: the bf16 policy rounds the head row to bf16 (as K14 stores it); the fp32 policy keeps fp32.
template <int A1, bool ROUND>
__device__ __forceinline__ void heads_sample_row_pre(const float (&hv)[4], const float* whs, const float* bhs,
                                                     const int64_t t, const uint32_t c, uint32_t seed,
                                                     int64_t* __restrict__ act, float* __restrict__ logp,
                                                     float* __restrict__ vf, float* __restrict__ lout,
                                                     int64_t* __restrict__ act_now, int64_t B, int64_t b, int lane) {
  constexpr int A = A1 - 1;
  const float h0 = hv[0], h1 = hv[1], h2 = hv[2], h3 = hv[3];
  float hd[A1];
#pragma unroll
  for (int a = 0; a < A1; a++) {
    const float4 w = *reinterpret_cast<const float4*>(&whs[a * H + 4 * lane]);
    hd[a] = h0 * w.x + h1 * w.y + h2 * w.z + h3 * w.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < A1; a++) hd[a] += __shfl_xor(hd[a], o, 64);
#pragma unroll
  for (int a = 0; a < A1; a++) hd[a] = ROUND ? bf2f(f2bf(hd[a] + bhs[a])) : hd[a] + bhs[a];
  const int64_t o = t * B + b;
  if (lane < A) {
    float l = hd[0];
#pragma unroll
    for (int j = 1; j < A; j++)
      if (lane == j) l = hd[j];
    lout[o * A + lane] = l;
  }
  if (lane == 0) {
    float best = -INFINITY, mx = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int j = 0; j < A; j++) {
      mx = fmaxf(mx, hd[j]);
      const uint32_t hh = hash3(seed, c, uint32_t(b * A + j));
      const float u = (float(hh >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float gmb = hd[j] - __logf(-__logf(u));
      if (gmb > best) {
        best = gmb;
        arg = j;
      }
    }
    float se = 0.f, la = hd[0];
#pragma unroll
    for (int j = 0; j < A; j++) {
      se += __expf(hd[j] - mx);
      if (j == arg) la = hd[j];
    }
    act[o] = arg;
    act_now[b] = arg;
    logp[o] = la - mx - __logf(se);
    vf[o] = hd[A];
  }
}

// The categorical PPO loss of one row given its head row hd = [logits (A) | value] (every lane of the
// row's wave holds the whole row and evaluates it redundantly: no broadcast). cv = the row's packed
// loss columns [old logits (A) | old logp | advantage | value target | action]. Returns the 6 loss
// statistics (meaningful on `stat_lane`) and g = d(loss)/d(heads) scaled by gs (= upstream / M).
// ROUND: the bf16 learner rounds g to bf16 (what K12 reads); the split-bf16 (fp32) learner keeps fp32.
// Shared by K15 (bf16) and K15x (x3_kernels.hip): the same loss code on both paths.
template <int A1, bool ROUND>
__device__ __forceinline__ void ppo_loss_row(const float (&hd)[A1], const float* cv, float clip, float vf_clip,
                                             float vf_coeff, float ent_coeff, float kl_coeff, float gs,
                                             bool stat_lane, float (&s)[6], float (&g)[A1]) {
  constexpr int A = A1 - 1;
  float mx = -INFINITY, mxo = -INFINITY, lo[A > 0 ? A : 1];
#pragma unroll
  for (int j = 0; j < A; j++) {
    lo[j] = cv[j];
    mx = fmaxf(mx, hd[j]);
    mxo = fmaxf(mxo, lo[j]);
  }
  float se = 0.f, seo = 0.f;
#pragma unroll
  for (int j = 0; j < A; j++) {
    se += __expf(hd[j] - mx);
    seo += __expf(lo[j] - mxo);
  }
  const float lse = mx + __logf(se), lseo = mxo + __logf(seo);
  float m = 0.f, kl = 0.f, p[A > 0 ? A : 1], po[A > 0 ? A : 1];
#pragma unroll
  for (int j = 0; j < A; j++) {
    p[j] = __expf(hd[j] - lse);
    po[j] = __expf(lo[j] - lseo);
    m += p[j] * hd[j];
    kl += po[j] * ((lo[j] - lseo) - (hd[j] - lse));
  }
  const int act = min(max(int(cv[A + 3]), 0), A - 1);
  float la = hd[0];
#pragma unroll
  for (int j = 1; j < A; j++)
    if (j == act) la = hd[j];
  const float r = __expf((la - lse) - cv[A]);
  const float ad = cv[A + 1];
  const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
  const float d = hd[A] - cv[A + 2];
#pragma unroll
  for (int k = 0; k < 6; k++) s[k] = 0.f;
  if (stat_lane) {
    const float ent = lse - m, surr = fminf(r * ad, rc * ad), vf = fminf(d * d, vf_clip);
    s[0] = -surr;
    s[1] = vf;
    s[2] = ent;
    s[3] = kl;
    s[4] = (fabsf(r - 1.f) > clip) ? 1.f : 0.f;
    s[5] = -surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl;
  }
  const bool unclipped = r * ad <= rc * ad;
  const bool inside = (r >= 1.f - clip) && (r <= 1.f + clip);
  const float spg = (unclipped || inside) ? -(r * ad) : 0.f;
#pragma unroll
  for (int j = 0; j < A; j++) {
    const float v = (spg * ((j == act ? 1.f : 0.f) - p[j]) + ent_coeff * p[j] * (hd[j] - m) + kl_coeff * (p[j] - po[j])) * gs;
    g[j] = ROUND ? bf2f(f2bf(v)) : v;
  }
  const float gv = (d * d < vf_clip) ? vf_coeff * 2.f * d * gs : 0.f;
  g[A] = ROUND ? bf2f(f2bf(gv)) : gv;
}

// One gradient element of the K12 row split's deferred finalize: (group, slot, lane-of-K12) → the
// element's destination in dW / db / dWh / dbh; sums the rs member partials (workspace
// [groups][rs][kK12PSlots][kK12NT]). Used by k_dense_split_finalize and by the finalize-Adam
// workgroups of the K10 trunk-reduce launch.
constexpr int kK12JB = 32, kK12NT = 512, kK12PSlots = 20;
__device__ __forceinline__ void split_finalize_elem(const float* __restrict__ part, int rs, int64_t K, int A1,
                                                    unsigned short* dw, unsigned short* db, unsigned short* dwh,
                                                    unsigned short* dbh, int group, int slot, const FusedAdam& fa,
                                                    const AdamCoef& ac) {

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, g = lane >> 4;
  const bool head = int64_t(group) * kK12JB == K;
  if (!head && slot >= 16) return;
  unsigned short* dst = nullptr;
  if (!head) {  // slot = (hi * 2 + jt) * 4 + i  →  dW[16 (wave + 8 hi) + 4 g + i][J0 + 16 jt + r]
    const int hi = slot >> 3, jt = (slot >> 2) & 1, i = slot & 3;
    dst = &dw[int64_t(16 * (wave + 8 * hi) + 4 * g + i) * K + int64_t(group) * kK12JB + 16 * jt + r];
  } else {
    const int i = slot & 3, q = slot >> 2;  // q: 0,1 dWh (hi), 2,3 db (hi), 4 dbh
    if (q < 2) {
      if (4 * g + i < A1) dst = &dwh[(4 * g + i) * H + 16 * (wave + 8 * q) + r];
    } else if (q < 4) {
      if (g == 0 && i == 0) dst = &db[16 * (wave + 8 * (q - 2)) + r];
    } else if (wave == 0 && r == 0 && 4 * g + i < A1) {
      dst = &dbh[4 * g + i];
    }
  }
  if (dst == nullptr) return;
  float t = 0.f;
  for (int h = 0; h < rs; h++) t += part[((int64_t(group) * rs + h) * kK12PSlots + slot) * kK12NT + tid];
  // the members' partials in member order (deterministic), rounded to bf16: stored, or (FusedAdam)
  // applied to the parameter — bit-identical to storing and running K6 on the bf16 gradient
  if (fa.grad_base) {
    grad_store(fa, ac, dst, t);
  } else {
    *dst = f2bf(t);
  }
}

}  // namespace dense
}  // namespace hip
}  // namespace rmm
