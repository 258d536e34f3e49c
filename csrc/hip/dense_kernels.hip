// K12 — fused backward of the PPO dense tail: hidden = ReLU(x Wᵀ + b) [M, 256], heads = hidden Whᵀ + bh
// [M, A1]. Given dheads (the fused PPO loss gradient, K5c), ONE launch produces
//   dx  = dpre W            [M, K]        dW  = dpreᵀ x   [256, K]       db  = Σ_m dpre
//   dWh = dheadsᵀ hidden    [A1, 256]     dbh = Σ_m dheads
// with dpre = (dheads Wh) ⊙ [hidden > 0] (k_dense_dpre, or written by the fused loss kernel K15).
// It replaces four hipBLASLt GEMMs (two of them 5-wide) and two bias/mask reductions (~45 µs at
// M = 500, K = 3872 on MI355X) — at this size every one of them is latency-bound.
//
// Decomposition (k_dense_heads_bwd2 below): workgroup j owns the 32 input columns J = [32j, 32j+32) of
// x / W (K/32 of them) and streams the batch in 64-row chunks; one extra workgroup carries the head
// gradients (dWh, db, dbh). dpre comes from k_dense_dpre (or the fused loss kernel K15). Every
// reduction over rows happens inside one workgroup in a fixed order: deterministic, no atomics.
//
// MFMA 16x16x32 bf16 maps: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// C/D col l&15, row 4(l>>4)+i.
#include <hip/hip_bf16.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "dense_device.h"
#include "kernels.h"

namespace rmm {
namespace hip {
namespace dense {


constexpr int MC = 32;       // rows per chunk
constexpr int JB = 32;       // columns of x / W per workgroup
constexpr int NT = 512;      // 8 waves
constexpr int HP = H + 8;    // padded pitches (bank spread, keep 16-B alignment)
constexpr int MP = MC + 8;
constexpr int MMAX = 640;    // batch rows held in LDS (dheads and the dx output block)
static_assert(MC * JB / 2 == NT, "x staging: one (row, column pair) per thread");

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but NOT for
// its outstanding global loads, so the next chunk's prefetch stays in flight across it.
// (__syncthreads() carries a workgroup fence that drains vmcnt to 0 first.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// dpre = (dheads · Wh) ⊙ [hidden > 0], computed ONCE for the batch (32 rows per workgroup) and
// read by every column-block workgroup of k_dense_heads_bwd. Recomputing it inside each of those
// 121 workgroups made that kernel VALU-bound (PMC: ~5.3k VALU instructions per wave, 40 µs).
template <int A1>
__global__ __launch_bounds__(NT) void k_dense_dpre(const unsigned short* __restrict__ dz,
                                                   const unsigned short* __restrict__ wh,
                                                   const unsigned short* __restrict__ y, int64_t M,
                                                   unsigned short* __restrict__ dpre) {
  __shared__ __attribute__((aligned(16))) unsigned short whs[A1 * H];
  const int tid = threadIdx.x;
  const int pm = tid & (MC - 1), hb = (tid / MC) * 16;
  const int64_t row = int64_t(blockIdx.x) * MC + pm, rc = row < M ? row : M - 1;
  const uint4 y0 = *reinterpret_cast<const uint4*>(&y[rc * H + hb]);
  const uint4 y1 = *reinterpret_cast<const uint4*>(&y[rc * H + hb + 8]);
  unsigned short rdz[A1];
#pragma unroll
  for (int a = 0; a < A1; a++) rdz[a] = dz[rc * A1 + a];
  for (int e = tid; e < A1 * H; e += NT) whs[e] = wh[e];
  __syncthreads();
  if (row >= M) return;
  float dyv[16];
#pragma unroll
  for (int i = 0; i < 16; i++) dyv[i] = 0.f;
#pragma unroll
  for (int a = 0; a < A1; a++) {
    const float za = bf2f(rdz[a]);
    const u16x8 w0 = *reinterpret_cast<const u16x8*>(&whs[a * H + hb]);
    const u16x8 w1 = *reinterpret_cast<const u16x8*>(&whs[a * H + hb + 8]);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      dyv[i] += za * bf2f(w0[i]);
      dyv[8 + i] += za * bf2f(w1[i]);
    }
  }
  unsigned short yv[16];
  *reinterpret_cast<uint4*>(&yv[0]) = y0;
  *reinterpret_cast<uint4*>(&yv[8]) = y1;
  u16x8 o0, o1;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const unsigned short yi = yv[i];
    const unsigned short dp = (yi != 0 && !(yi & 0x8000)) ? f2bf(dyv[i]) : static_cast<unsigned short>(0);
    if (i < 8) o0[i] = dp; else o1[i - 8] = dp;
  }
  *reinterpret_cast<u16x8*>(&dpre[row * H + hb]) = o0;
  *reinterpret_cast<u16x8*>(&dpre[row * H + hb + 8]) = o1;
}

// (The first K12, which transposed dpre / x into LDS with VALU scatters and had workgroup 0 carry the
// head gradients on top of its column block, was ~1.8 us per 32-row chunk; superseded by the form below,
// profiles/ppo_kernels_r2.txt -> k12 notes.)

// ---------------------------------------------------------------- K12 (transposed-read form)
// Same outputs as above, restructured after PMC + phase timing showed the per-chunk critical
// path (u16 scatter transposes into LDS, two barriers per 32-row chunk, and workgroup 0 carrying
// the head gradients on top of its column block) set the time: ~1.8 µs per chunk.
//  * Operands that must be reduced over rows (dpreᵀ, xᵀ, dzᵀ, hiddenᵀ) are read from ROW-MAJOR LDS
//    images with gfx950's ds_read_b64_tr_b16 (a 4-row x 16-column block per 16-lane group,
//    delivered column-wise): staging is plain coalesced 16-B loads + ds_write_b128, no VALU
//    transposes. The k order inside a step is permuted (lane group g takes rows 4g..4g+3 and
//    16+4g..16+4g+3) identically for both operands: a 32-lane half then reads 8 consecutive rows,
//    conflict-free at row pitch 272 (136 dwords ≡ 8 mod 64).
//  * 64-row chunks, double-buffered LDS, ONE barrier per chunk; next-next chunk's loads in flight.
//  * dx is computed as dxᵀ tiles (A = Wᵀ fragments kept in registers for the whole launch), so a
//    lane's 4 outputs are 4 consecutive columns: one 8-byte LDS store.
//  * The head gradients (dWh, db, dbh) run in their own extra workgroup (index K/32).
constexpr int MC2 = 64;       // rows per chunk
constexpr int DMP = H + 16;   // dpre / hidden image row pitch (b128 row reads P=2 slots, tr reads conflict-free)
constexpr int DXP = JB + 8;   // dx block pitch (8-byte stores: 2-way at most, 16-B aligned rows)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr4(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
// A/B fragment from two transposed reads: elements 0-3 from block p0, 4-7 from block p1
__device__ __forceinline__ bf16x8 tr8(const unsigned short* p0, const unsigned short* p1) {
  const s16x4 a = tr4(p0), b = tr4(p1);
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// ok ? v : 0 per component (a ternary on the uint4 struct is lowered through a stack copy: scratch)
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}

constexpr int K12_LDS_DM = 2 * MC2 * DMP;                 // elements, both roles
constexpr int K12_WS = 2 * H * 16, K12_XS = 2 * 2 * MC2 * 16, K12_DXS = MMAX * DXP;
constexpr int K12_YS = 2 * MC2 * DMP, K12_DZS = MMAX * 16;
constexpr int K12_RB = (K12_WS + K12_XS + K12_DXS) > (K12_YS + K12_DZS) ? (K12_WS + K12_XS + K12_DXS)
                                                                       : (K12_YS + K12_DZS);
static_assert((K12_LDS_DM + K12_RB) * 2 <= 160 * 1024, "K12 LDS");

// Row split of K12 (RMM_K12_SPLIT=2): each column block (and the head role) runs as RS workgroups
// over disjoint chunk ranges of the batch — 244 instead of 122 workgroups at M = 500, half the
// serial chunk chain each. dx rows are independent; the dW / head partials (fp32, 16-20 per lane,
// lane-major so the stores coalesce) go to a workspace that k_dense_split_finalize sums in member
// order (deterministic) into the gradients. A last-arriver combine inside K12 measured 2x SLOWER:
// each workgroup's agent-scope release fence wrote back its XCD's whole L2 (dx included).
constexpr int K12_PSLOTS = 20;  // partial floats per lane (head role: 8 dWh + 8 db + 4 dbh)
static_assert(K12_PSLOTS == kK12PSlots && JB == kK12JB && NT == kK12NT, "split_finalize_elem layout");
struct RowSplit {
  float* part = nullptr;  // [groups][rs][K12_PSLOTS][NT]
  int rs = 1, h = 0, group = 0;
};
__device__ __forceinline__ void k12_publish(const RowSplit& rsp, const float* v, int n) {
  float* my = rsp.part + ((int64_t(rsp.group) * rsp.rs + rsp.h) * K12_PSLOTS) * NT + threadIdx.x;
  for (int i = 0; i < n; i++) my[i * NT] = v[i];
}

// grid (groups, K12_PSLOTS) x NT: thread = (group, slot, lane-of-K12) → one gradient element
__global__ __launch_bounds__(NT) void k_dense_split_finalize(const float* __restrict__ part, int rs, int64_t K, int A1,
                                                             unsigned short* __restrict__ dw,
                                                             unsigned short* __restrict__ db,
                                                             unsigned short* __restrict__ dwh,
                                                             unsigned short* __restrict__ dbh) {
  split_finalize_elem(part, rs, K, A1, dw, db, dwh, dbh, blockIdx.x, blockIdx.y, FusedAdam{}, AdamCoef{});
}

// column-block role: dx[:, J] and dW[:, J] for J = [J0, J0+32)
__device__ __forceinline__ void k12_cols(const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
                                         const unsigned short* __restrict__ dpre, int64_t M, int64_t K, int64_t J0,
                                         unsigned short* __restrict__ dx, unsigned short* __restrict__ dw,
                                         unsigned short* dm, unsigned short* rb, const FusedAdam& fa, int c0, int c1,
                                         const RowSplit& rsp) {
  unsigned short* ws = rb;                    // [jt][h][16]  W[:, J] (setup only)
  unsigned short* xs = rb + K12_WS;           // [buf][jt][m][16]
  unsigned short* dxs = rb + K12_WS + K12_XS; // [m][DXP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int q = r >> 2, p = r & 3;
  const int NC = int((M + MC2 - 1) / MC2);

  uint4 sd[4], sx;
  auto load = [&](int c) {  // unconditional clamped loads (rows >= M are zeroed at the LDS store)
    const int64_t m0 = int64_t(c) * MC2;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      const int64_t rr = min(m0 + row, M - 1);
      sd[k] = *reinterpret_cast<const uint4*>(&dpre[rr * H + 8 * pc]);
    }
    const int row = (tid >> 2) & (MC2 - 1), pc = tid & 3;  // threads 256.. duplicate 0..255 (not stored)
    sx = *reinterpret_cast<const uint4*>(&x[min(m0 + row, M - 1) * K + J0 + 8 * pc]);
  };
  auto store = [&](int c) {
    const int64_t m0 = int64_t(c) * MC2;
    unsigned short* d = dm + (c & 1) * MC2 * DMP;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      *reinterpret_cast<uint4*>(&d[row * DMP + 8 * pc]) = keep_if(m0 + row < M, sd[k]);
    }
    if (tid < MC2 * 4) {
      const int row = tid >> 2, pc = tid & 3;
      *reinterpret_cast<uint4*>(&xs[(((c & 1) * 2 + (pc >> 1)) * MC2 + row) * 16 + 8 * (pc & 1)]) =
          keep_if(m0 + row < M, sx);
    }
  };

  {  // W[:, J] → ws (two 16-column halves, row-major over h)
    uint4 wv[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int v = tid + NT * k, h = v >> 2, pc = v & 3;
      wv[k] = *reinterpret_cast<const uint4*>(&w[int64_t(h) * K + J0 + 8 * pc]);
    }
    load(c0);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int v = tid + NT * k, h = v >> 2, pc = v & 3;
      *reinterpret_cast<uint4*>(&ws[((pc >> 1) * H + h) * 16 + 8 * (pc & 1)]) = wv[k];
    }
  }
  store(c0);
  if (c0 + 1 < c1) load(c0 + 1);
  lds_barrier();

  // Wᵀ fragments for this wave's column tile nt: A[row j = 16nt + r][k = h = 32s + 8g + e]
  const int mt = wave >> 1, nt = wave & 1;
  bf16x8 wf[H / 32];
#pragma unroll
  for (int s = 0; s < H / 32; s++) {
    const unsigned short* p0 = &ws[(nt * H + 32 * s + 8 * g + q) * 16 + 4 * p];
    wf[s] = tr8(p0, p0 + 4 * 16);
  }
  f32x4 adw[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++) adw[i][0] = adw[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused Adam: this lane's 16 dW elements' master / moments, in flight during the chunk loop
  auto dw_at = [&](int hi, int jt, int i) { return &dw[int64_t(16 * (wave + 8 * hi) + 4 * g + i) * K + J0 + 16 * jt + r]; };
  AdamState ast[2][2][4];
#pragma unroll
  for (int hi = 0; hi < 2; hi++)
#pragma unroll
    for (int jt = 0; jt < 2; jt++)
#pragma unroll
      for (int i = 0; i < 4; i++) ast[hi][jt][i] = adam_prefetch(fa, dw_at(hi, jt, i));

  for (int c = c0; c < c1; c++) {
    const unsigned short* d = dm + (c & 1) * MC2 * DMP;
    const unsigned short* xb = xs + (c & 1) * 2 * MC2 * 16;
    {  // dxᵀ tile: D[j][m] = Σ_h Wᵀ[j][h] · dpre[m][h]  (B = dpre row reads)
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      const unsigned short* drow = d + (16 * mt + r) * DMP + 8 * g;
#pragma unroll
      for (int s = 0; s < H / 32; s += 2) {
        a0 = mfma(wf[s], as_bf(*reinterpret_cast<const u16x8*>(drow + 32 * s)), a0);
        a1 = mfma(wf[s + 1], as_bf(*reinterpret_cast<const u16x8*>(drow + 32 * s + 32)), a1);
      }
      const f32x4 t = a0 + a1;
      const uint2 o = make_uint2(uint32_t(f2bf(t[0])) | (uint32_t(f2bf(t[1])) << 16),
                                 uint32_t(f2bf(t[2])) | (uint32_t(f2bf(t[3])) << 16));
      *reinterpret_cast<uint2*>(&dxs[(c * MC2 + 16 * mt + r) * DXP + 16 * nt + 4 * g]) = o;
    }
    // dW[h][j] += Σ_m dpre[m][h] x[m][j]: both operands by transposed reads (permuted k order)
#pragma unroll
    for (int ks = 0; ks < MC2 / 32; ks++) {
      bf16x8 bx[2];
#pragma unroll
      for (int jt = 0; jt < 2; jt++) {
        const unsigned short* p0 = &xb[(jt * MC2 + 32 * ks + 4 * g + q) * 16 + 4 * p];
        bx[jt] = tr8(p0, p0 + 16 * 16);
      }
#pragma unroll
      for (int hi = 0; hi < 2; hi++) {
        const unsigned short* p0 = &d[(32 * ks + 4 * g + q) * DMP + 16 * (wave + 8 * hi) + 4 * p];
        const bf16x8 ad = tr8(p0, p0 + 16 * DMP);
        adw[hi][0] = mfma(ad, bx[0], adw[hi][0]);
        adw[hi][1] = mfma(ad, bx[1], adw[hi][1]);
      }
    }
    if (c + 1 < c1) store(c + 1);  // loaded one chunk ago
    if (c + 2 < c1) load(c + 2);   // in flight across the barrier and the next chunk's MFMAs
    lds_barrier();
  }
  (void)NC;

  const int r0 = c0 * MC2, r1 = int(min(int64_t(c1) * MC2, M));
  for (int v = tid + r0 * (JB / 8); v < r1 * (JB / 8); v += NT) {
    const int row = v >> 2, pc = v & 3;
    *reinterpret_cast<uint4*>(&dx[int64_t(row) * K + J0 + 8 * pc]) = *reinterpret_cast<const uint4*>(&dxs[row * DXP + 8 * pc]);
  }
  if (rsp.rs > 1) {  // dW[:, J] over this workgroup's rows only: the group's last finisher sums them
    float pv[16];
#pragma unroll
    for (int hi = 0; hi < 2; hi++)
#pragma unroll
      for (int jt = 0; jt < 2; jt++)
#pragma unroll
        for (int i = 0; i < 4; i++) pv[(hi * 2 + jt) * 4 + i] = adw[hi][jt][i];
    k12_publish(rsp, pv, 16);  // k_dense_split_finalize sums the members' partials
    return;
  }
  // dW[:, J] is final here (every row reduced): store it, or apply Adam to it
  const AdamCoef ac = fa.grad_base ? adam_coef(fa.hp, fa.step_ctr) : AdamCoef{};
#pragma unroll
  for (int hi = 0; hi < 2; hi++)
#pragma unroll
    for (int jt = 0; jt < 2; jt++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        grad_store_pf(fa, ac, dw_at(hi, jt, i), adw[hi][jt][i], ast[hi][jt][i]);
}

// head role: dWh = dheadsᵀ hidden [A1, 256], db = Σ_m dpre, dbh = Σ_m dheads
template <int A1>
__device__ __forceinline__ void k12_head(const unsigned short* __restrict__ dz, const unsigned short* __restrict__ y,
                                         const unsigned short* __restrict__ dpre, int64_t M,
                                         unsigned short* __restrict__ db, unsigned short* __restrict__ dwh,
                                         unsigned short* __restrict__ dbh, unsigned short* dm, unsigned short* rb,
                                         const FusedAdam& fa, int c0, int c1, const RowSplit& rsp) {
  unsigned short* ys = rb;            // [buf][m][DMP]
  unsigned short* dzs = rb + K12_YS;  // [m][16] (a >= A1 and rows >= M zero)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int q = r >> 2, p = r & 3;
  const int NC = int((M + MC2 - 1) / MC2);

  uint4 sd[4], sy[4];
  auto load = [&](int c) {
    const int64_t m0 = int64_t(c) * MC2;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      const int64_t rr = min(m0 + row, M - 1);
      sd[k] = *reinterpret_cast<const uint4*>(&dpre[rr * H + 8 * pc]);
      sy[k] = *reinterpret_cast<const uint4*>(&y[rr * H + 8 * pc]);
    }
  };
  auto store = [&](int c) {
    const int64_t m0 = int64_t(c) * MC2;
    const int o = (c & 1) * MC2 * DMP;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      const bool ok = m0 + row < M;
      *reinterpret_cast<uint4*>(&dm[o + row * DMP + 8 * pc]) = keep_if(ok, sd[k]);
      *reinterpret_cast<uint4*>(&ys[o + row * DMP + 8 * pc]) = keep_if(ok, sy[k]);
    }
  };
  {
    constexpr int PZ = MMAX * 16 / NT;  // 20
    unsigned short zv[PZ];
#pragma unroll
    for (int k = 0; k < PZ; k++) {
      const int e = tid + NT * k, m = e >> 4, a = e & 15;
      zv[k] = dz[int64_t(min(int64_t(m), M - 1)) * A1 + min(a, A1 - 1)];
    }
    load(c0);
#pragma unroll
    for (int k = 0; k < PZ; k++) {
      const int e = tid + NT * k, m = e >> 4, a = e & 15;
      dzs[e] = (m < M && a < A1) ? zv[k] : static_cast<unsigned short>(0);
    }
  }
  store(c0);
  if (c0 + 1 < c1) load(c0 + 1);
  lds_barrier();
  (void)NC;

  u16x8 onev;
#pragma unroll
  for (int j = 0; j < 8; j++) onev[j] = (r == 0) ? static_cast<unsigned short>(0x3f80) : static_cast<unsigned short>(0);
  const bf16x8 ones = as_bf(onev);  // as A: row 0 all ones; as B: column 0 all ones
  f32x4 awh[2], adb[2], abh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; i++) awh[i] = adb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused Adam: prefetch this lane's dWh / db / dbh elements' state (clamped addresses; unused if out of range)
  AdamState swh[2][4], sdb[2], sbh[4];
#pragma unroll
  for (int hi = 0; hi < 2; hi++) {
    const int h = 16 * (wave + 8 * hi) + r;
#pragma unroll
    for (int i = 0; i < 4; i++) swh[hi][i] = adam_prefetch(fa, &dwh[min(4 * g + i, A1 - 1) * H + h]);
    sdb[hi] = adam_prefetch(fa, &db[h]);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) sbh[i] = adam_prefetch(fa, &dbh[min(4 * g + i, A1 - 1)]);

  for (int c = c0; c < c1; c++) {
    const int o = (c & 1) * MC2 * DMP;
#pragma unroll
    for (int ks = 0; ks < MC2 / 32; ks++) {
      const unsigned short* pz = &dzs[(c * MC2 + 32 * ks + 4 * g + q) * 16 + 4 * p];
      const bf16x8 az = tr8(pz, pz + 16 * 16);  // A[row a = r][k = m]
#pragma unroll
      for (int hi = 0; hi < 2; hi++) {
        const int off = o + (32 * ks + 4 * g + q) * DMP + 16 * (wave + 8 * hi) + 4 * p;
        const bf16x8 by = tr8(&ys[off], &ys[off + 16 * DMP]);
        const bf16x8 bd = tr8(&dm[off], &dm[off + 16 * DMP]);
        awh[hi] = mfma(az, by, awh[hi]);
        adb[hi] = mfma(ones, bd, adb[hi]);
      }
      if (wave == 0) abh = mfma(az, ones, abh);
    }
    if (c + 1 < c1) store(c + 1);
    if (c + 2 < c1) load(c + 2);
    lds_barrier();
  }
  if (rsp.rs > 1) {  // partial over this workgroup's rows: the group's last finisher sums them
    float pv[K12_PSLOTS];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      pv[i] = awh[0][i], pv[4 + i] = awh[1][i], pv[8 + i] = adb[0][i], pv[12 + i] = adb[1][i], pv[16 + i] = abh[i];
    }
    k12_publish(rsp, pv, K12_PSLOTS);
    return;
  }
  const AdamCoef ac = fa.grad_base ? adam_coef(fa.hp, fa.step_ctr) : AdamCoef{};
#pragma unroll
  for (int hi = 0; hi < 2; hi++) {
    const int h = 16 * (wave + 8 * hi) + r;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * g + i < A1) grad_store_pf(fa, ac, &dwh[(4 * g + i) * H + h], awh[hi][i], swh[hi][i]);
    if (g == 0) grad_store_pf(fa, ac, &db[h], adb[hi][0], sdb[hi]);
  }
  if (wave == 0 && r == 0) {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * g + i < A1) grad_store_pf(fa, ac, &dbh[4 * g + i], abh[i], sbh[i]);
  }
}

template <int A1>
__global__ __launch_bounds__(NT) void k_dense_heads_bwd2(
    const unsigned short* __restrict__ dz, const unsigned short* __restrict__ y, const unsigned short* __restrict__ x,
    const unsigned short* __restrict__ w, const unsigned short* __restrict__ dpre, int64_t M, int64_t K,
    unsigned short* __restrict__ dx, unsigned short* __restrict__ dw, unsigned short* __restrict__ db,
    unsigned short* __restrict__ dwh, unsigned short* __restrict__ dbh, const FusedAdam fa, float* __restrict__ rs_part,
    int rs) {
  __shared__ __attribute__((aligned(16))) unsigned short dm[K12_LDS_DM];
  __shared__ __attribute__((aligned(16))) unsigned short rb[K12_RB];
  // block = (role group, row split h); the RS members of a group are consecutive blocks
  RowSplit rsp;
  rsp.part = rs_part, rsp.rs = rs, rsp.h = int(blockIdx.x) % rs, rsp.group = int(blockIdx.x) / rs;
  const int NC = int((M + MC2 - 1) / MC2);
  const int c0 = NC * rsp.h / rs, c1 = NC * (rsp.h + 1) / rs;
  if (int64_t(rsp.group) * JB == K)
    k12_head<A1>(dz, y, dpre, M, db, dwh, dbh, dm, rb, fa, c0, c1, rsp);
  else
    k12_cols(x, w, dpre, M, K, int64_t(rsp.group) * JB, dx, dw, dm, rb, fa, c0, c1, rsp);
}

// K13: hidden = ReLU(x Wᵀ + b) for small M (PPO minibatch / rollout batch). One 4-wave workgroup
// per 16x16 output tile, K split over the waves and streamed straight from L2 with 4 independent
// accumulator chains and 8 x 16-B loads in flight per lane. A (16 rows of x) and B (16 rows of W) fragments are both contiguous
// 16-B runs along K in row-major storage, so no LDS is needed. Grid = (M/16) x (256/16) waves:
// spreading W and x reads over many CUs is the point — a 16-row block reading all of W through
// one CU is per-CU-L2-bandwidth bound (~14 µs for W = 2 MB, like the library kernel it replaces).
__global__ __launch_bounds__(256) void k_dense_fwd(const unsigned short* __restrict__ x,
                                                   const unsigned short* __restrict__ w,
                                                   const unsigned short* __restrict__ b, int64_t M, int64_t K, int N,
                                                   unsigned short* __restrict__ y, int xcd_remap) {
  // 4 waves split K (wave w takes k-steps s ≡ w mod 4), 4 accumulator chains each, partial tiles
  // combined through LDS in a fixed order: the serial L2-latency chain per wave is K/128 deep.
  __shared__ f32x4 part[3][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  // 1-D grid of (M/16) x (N/16) tiles. XCD-aware order (guide §5.5 T1): blocks id, id+8, ... share
  // an XCD (and its 4 MB L2), so give each XCD a CONTIGUOUS run of tiles = a few 16-row x slices
  // against all of W. Its L2 then holds ~2.5 MB (W + its x rows) instead of the whole 6 MB
  // working set every XCD touches in raster order (which streams from the Infinity Cache).
  const int nn = N / 16;
  const int64_t total = gridDim.x;
  int64_t id = blockIdx.x;
  if (xcd_remap && (total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  const int64_t m0 = (id / nn) * 16, n0 = (id % nn) * 16;
  const int64_t xr = min(m0 + r, M - 1);
  const unsigned short* xa = x + xr * K + 8 * g;
  const unsigned short* wb = w + (n0 + r) * K + 8 * g;
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; c++) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t steps = K / 32;
  int64_t s = wave;
  for (; s + 12 < steps; s += 16) {  // 4 of this wave's k-steps per batch: 8 x 16-B loads in flight
    u16x8 av[4], bv[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      av[c] = *reinterpret_cast<const u16x8*>(xa + (s + 4 * c) * 32);
      bv[c] = *reinterpret_cast<const u16x8*>(wb + (s + 4 * c) * 32);
    }
#pragma unroll
    for (int c = 0; c < 4; c++) acc[c] = mfma(as_bf(av[c]), as_bf(bv[c]), acc[c]);
  }
  for (; s < steps; s += 4) {
    const u16x8 av = *reinterpret_cast<const u16x8*>(xa + s * 32);
    const u16x8 bv = *reinterpret_cast<const u16x8*>(wb + s * 32);
    acc[0] = mfma(as_bf(av), as_bf(bv), acc[0]);
  }
  f32x4 t = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (wave > 0) part[wave - 1][lane] = t;
  __syncthreads();
  if (wave != 0) return;
  t = ((t + part[0][lane]) + part[1][lane]) + part[2][lane];
  const float bias = bf2f(b[n0 + r]);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int64_t row = m0 + 4 * g + i;
    if (row < M) y[row * N + n0 + r] = f2bf(fmaxf(t[i] + bias, 0.f));
  }
}


// K13s — split-K form of K13 for the fused paths: the K10 → K13 → K15/K16 chain already has a
// kernel boundary between the dense layer and its consumer, so the cross-workgroup reduction of a
// split-K GEMM can happen in the CONSUMER's prologue (load_hidden4) instead of in-kernel (an
// agent-scope release/acquire = L2 write-back across XCDs, 4x slower, round 2) or in an extra
// reduce launch (+1 boundary, round 2). Output: fp32 partials part[S][M][N], no bias / ReLU.
// Workgroup = WM x WN waves side by side, each owning FM x FN 16x16 fragments (register blocking:
// FM + FN fragment loads feed FM*FN MFMAs — K13 issues 2 loads per MFMA, and at M = 500 the CU's
// vector-load path, hits included, is what bounds it), the remaining KW = 4 / (WM WN) waves split
// the slice's k-steps and combine through LDS; S contiguous K slices are separate workgroups.
// Block order: slice slowest, then row tiles, then column tiles, XCD-aware (blocks id, id+8, ... on
// one XCD get a contiguous run: same K slice, neighbouring tiles → shared x rows / W rows in its L2).
template <int FM, int FN, int WM, int WN>
__global__ __launch_bounds__(256) void k_dense_fwd_part(const unsigned short* __restrict__ x,
                                                        const unsigned short* __restrict__ w, int64_t M, int64_t K,
                                                        int N, int S, float* __restrict__ part) {
  constexpr int KW = 4 / (WM * WN);
  __shared__ f32x4 red[KW > 1 ? KW - 1 : 1][FM * FN][64];
  const int wave = threadIdx.x >> 6;
  const int nt = N / (16 * FN * WN);
  const int64_t mt = (M + 16 * FM * WM - 1) / (16 * FM * WM);
  const int64_t tiles = mt * nt, total = gridDim.x;
  int64_t id = blockIdx.x;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  const int64_t sl = id / tiles, rem = id % tiles, tm = rem / nt, tn = rem % nt;
  dense_part_unit<FM, FN, WM, WN>(x, w, M, K, N, S, part, sl, tm, tn, wave, true, red);
}



// K14 — the A1-wide head GEMM heads[M, A1] = hidden[M, 256] Whᵀ + bh (bf16 in/out, fp32 accumulate).
// Too narrow for MFMA or hipBLASLt to pay (a 16x256 macro tile for 5 useful columns, ~5-6 µs): one
// wave per row, each lane a 4-element slice of the row (8-B load) dotted against all A1 head rows
// (Wh, bias staged once per workgroup in LDS), then A1 butterfly reductions across the wave.
template <int A1>
__global__ __launch_bounds__(256) void k_heads_fwd(const unsigned short* __restrict__ hid,
                                                   const unsigned short* __restrict__ wh,
                                                   const unsigned short* __restrict__ bh, int64_t M,
                                                   unsigned short* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  for (int e = threadIdx.x; e < A1 * H; e += blockDim.x) whs[e] = bf2f(wh[e]);
  if (threadIdx.x < A1) bhs[threadIdx.x] = bf2f(bh[threadIdx.x]);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;  // whole wave exits together (row is wave-uniform)
  const uint2 v = *reinterpret_cast<const uint2*>(&hid[row * H + 4 * lane]);
  const float h0 = __uint_as_float(v.x << 16), h1 = __uint_as_float(v.x & 0xffff0000u);
  const float h2 = __uint_as_float(v.y << 16), h3 = __uint_as_float(v.y & 0xffff0000u);
  float acc[A1];
#pragma unroll
  for (int a = 0; a < A1; a++) {
    const float4 w = *reinterpret_cast<const float4*>(&whs[a * H + 4 * lane]);
    acc[a] = h0 * w.x + h1 * w.y + h2 * w.z + h3 * w.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < A1; a++) acc[a] += __shfl_xor(acc[a], o, 64);
  if (lane < A1) {
    float r = acc[0];
#pragma unroll
    for (int a = 1; a < A1; a++)
      if (lane == a) r = acc[a];
    out[row * A1 + lane] = f2bf(r + bhs[lane]);
  }
}


// K15 — the SGD step's head layer + PPO loss in ONE launch (replaces K14 + K5c + the K12 dpre
// pre-kernel). One wave per row as in K14; after the butterfly every lane holds the full head row,
// so every lane evaluates the (A ≤ 15 wide) categorical PPO loss of its row redundantly (no
// broadcast), lanes < A1 store d(loss)/d(heads) (bf16, scaled by *gout / M), and each lane turns
// its 4 hidden elements into dpre = (dheads Wh) ⊙ [hidden > 0] — exactly what K12 needs, while the
// row is still in registers. Loss statistics: lane 0 per row → workgroup sum → 6 atomics.
// cols[M, A+4] (f32): old logits [0, A), old logp A, advantage A+1, value target A+2, action A+3.
// coef: [clip, vf_clip, vf_coeff, entropy_coeff, kl_coeff]; acc[6] as K5c (zeroed per update).
template <int A1>
__global__ __launch_bounds__(256) void k_heads_ppo(const unsigned short* __restrict__ hid,
                                                   const unsigned short* __restrict__ wh,
                                                   const unsigned short* __restrict__ bh,
                                                   const float* __restrict__ cols, const float* __restrict__ coef,
                                                   float* __restrict__ acc, const float* __restrict__ gout, int64_t M,
                                                   unsigned short* __restrict__ dz,
                                                   unsigned short* __restrict__ dpre,
                                                   const int64_t* __restrict__ cidx,
                                                   const int64_t* __restrict__ ctr, int64_t period,
                                                   const float* __restrict__ hpart, int S,
                                                   const unsigned short* __restrict__ hb,
                                                   unsigned short* __restrict__ hid_out) {
  constexpr int A = A1 - 1;
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  __shared__ float red[6][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x >> 6) + wave;
  const bool valid = row < M;  // wave-uniform
  const int64_t rr = valid ? row : M - 1;
  // the cols row (ctr → index window → row: three dependent loads) and the hidden partials go out
  // first, so their round trips overlap the head-weight staging below instead of following it
  const int64_t crr = cidx ? (ctr ? cidx[(ctr[0] % period) * M + rr] : cidx[rr]) : rr;
  const float* crow = cols + crr * (A + 4);
  float cv[A + 4];
#pragma unroll
  for (int j = 0; j < A + 4; j++) cv[j] = crow[j];
  float hv[4];
  uint2 hbits;
  load_hidden4(hid, hpart, S, hb, M, rr, lane, hv, hbits);
  for (int e = threadIdx.x; e < A1 * H; e += blockDim.x) whs[e] = bf2f(wh[e]);
  if (threadIdx.x < A1) bhs[threadIdx.x] = bf2f(bh[threadIdx.x]);
  __syncthreads();
  const float clip = coef[0], vf_clip = coef[1], vf_coeff = coef[2], ent_coeff = coef[3], kl_coeff = coef[4];
  const float gs = gout[0] / float(M);
  if (hid_out != nullptr && valid) *reinterpret_cast<uint2*>(&hid_out[row * H + 4 * lane]) = hbits;  // for K12
  float hd[A1];
#pragma unroll
  for (int a = 0; a < A1; a++) {
    const float4 w = *reinterpret_cast<const float4*>(&whs[a * H + 4 * lane]);
    hd[a] = hv[0] * w.x + hv[1] * w.y + hv[2] * w.z + hv[3] * w.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int a = 0; a < A1; a++) hd[a] += __shfl_xor(hd[a], o, 64);
#pragma unroll
  for (int a = 0; a < A1; a++) hd[a] = bf2f(f2bf(hd[a] + bhs[a]));  // the bf16 head output
  // cols row (loaded above): gathered through the minibatch index window (as K2) when cidx is given;
  // statistics from lane 0 of each valid row, d(loss)/d(heads) rounded to bf16 (what K12 reads)
  float s[6], g[A1];
  ppo_loss_row<A1, true>(hd, cv, clip, vf_clip, vf_coeff, ent_coeff, kl_coeff, gs, valid && lane == 0, s, g);
  if (valid) {
    if (lane < A1) {
      float gl = g[0];
#pragma unroll
      for (int j = 1; j < A1; j++)
        if (lane == j) gl = g[j];
      dz[row * A1 + lane] = f2bf(gl);
    }
    float dp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < A1; a++) {
      const float4 w = *reinterpret_cast<const float4*>(&whs[a * H + 4 * lane]);
      dp[0] += g[a] * w.x, dp[1] += g[a] * w.y, dp[2] += g[a] * w.z, dp[3] += g[a] * w.w;
    }
    unsigned short o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) o[k] = hv[k] > 0.f ? f2bf(dp[k]) : static_cast<unsigned short>(0);
    *reinterpret_cast<uint2*>(&dpre[row * H + 4 * lane]) =
        make_uint2(uint32_t(o[0]) | (uint32_t(o[1]) << 16), uint32_t(o[2]) | (uint32_t(o[3]) << 16));
  }
  if (lane == 0)
    for (int k = 0; k < 6; k++) red[k][wave] = s[k];
  __syncthreads();
  if (threadIdx.x < 6) {
    float t = 0.f;
    for (int k = 0; k < int(blockDim.x >> 6); k++) t += red[threadIdx.x][k];
    atomicAdd(&acc[threadIdx.x], t);
  }
}


// K16 — the rollout step's head layer + action sampling in ONE launch (replaces K14 + K7). One wave
// per env row as in K14; after the butterfly every lane holds the bf16-rounded head row; lane 0
// draws the Gumbel-max action (same counter hash and stream as K7, so the two paths sample
// identically) and writes act/logp/vf of rollout row t = *t_ptr, lanes < A write the logits row.
// With `done` set the launch also ADVANCES the step: the last workgroup to finish (device-scope
// completion counter) bumps *t_ptr and *ctr and re-arms the counter, so a rollout step needs no
// separate counter-increment kernel after it. Every block has consumed t / ctr before it arrives.
template <int A1>
__global__ __launch_bounds__(256) void k_heads_sample(const unsigned short* __restrict__ hid,
                                                      const unsigned short* __restrict__ wh,
                                                      const unsigned short* __restrict__ bh,
                                                      const int64_t* t_ptr, const int64_t* ctr, uint32_t seed,
                                                      int64_t* __restrict__ act, float* __restrict__ logp,
                                                      float* __restrict__ vf, float* __restrict__ lout,
                                                      int64_t* __restrict__ act_now, int64_t B,
                                                      unsigned int* __restrict__ done,
                                                      const float* __restrict__ hpart, int S,
                                                      const unsigned short* __restrict__ hb, int64_t* host_seq) {
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  const int lane = threadIdx.x & 63;
  const int64_t b = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  // the row's hidden partials and the step counters load first: their round trips overlap the Wh staging
  float hv[4] = {0.f, 0.f, 0.f, 0.f};
  uint2 hbits;
  if (b < B) load_hidden4(hid, hpart, S, hb, B, b, lane, hv, hbits);  // wave-uniform
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  for (int e = threadIdx.x; e < A1 * H; e += blockDim.x) whs[e] = bf2f(wh[e]);
  if (threadIdx.x < A1) bhs[threadIdx.x] = bf2f(bh[threadIdx.x]);
  __syncthreads();
  if (b < B) heads_sample_row_pre<A1>(hv, whs, bhs, t, c, seed, act, logp, vf, lout, act_now, B, b, lane);
  if (done) {
    __shared__ unsigned int last;
    if (host_seq) __threadfence_system();  // this wave's action stores to host memory, visible to the CPU
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
      int64_t* tw = const_cast<int64_t*>(t_ptr);
      int64_t* cw = const_cast<int64_t*>(ctr);
      *tw += 1;
      if (cw != tw) *cw += 1;
      atomicExch(done, 0u);
      // host_seq: the step's completion word in mapped host memory (the native loop polls it instead of
      // recording and waiting on an event); every workgroup's actions were made system-visible above
      if (host_seq) __hip_atomic_store(host_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// K16 for a small rollout batch with the step advance (B <= 16 R): ONE workgroup of 16 waves, wave w
// takes rows w, w + 16, ... (at most R); every row's hidden partials are loaded before the Wh staging,
// so the R round trips overlap each other and the staging. Then thread 0 bumps *t_ptr / *ctr after a
// workgroup barrier — no device-scope fence and completion atomic (an L2 write-back across XCDs) as
// the multi-workgroup K16 needs. Same per-row code as K16, so the two launches are bit-identical.
template <int A1, int R>
__global__ __launch_bounds__(1024) void k_heads_sample1(const unsigned short* __restrict__ hid,
                                                        const unsigned short* __restrict__ wh,
                                                        const unsigned short* __restrict__ bh, int64_t* t_ptr,
                                                        int64_t* ctr, uint32_t seed, int64_t* __restrict__ act,
                                                        float* __restrict__ logp, float* __restrict__ vf,
                                                        float* __restrict__ lout, int64_t* __restrict__ act_now,
                                                        int64_t B, const float* __restrict__ hpart, int S,
                                                        const unsigned short* __restrict__ hb, int64_t* host_seq) {
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  constexpr int kWaves = 16;
  const int lane = threadIdx.x & 63;
  const int64_t b0 = threadIdx.x >> 6;
  float hv[R][4];
  uint2 hbits;
#pragma unroll
  for (int r = 0; r < R; r++)  // wave-uniform
    if (b0 + r * kWaves < B) load_hidden4(hid, hpart, S, hb, B, b0 + r * kWaves, lane, hv[r], hbits);
  for (int e = threadIdx.x; e < A1 * H; e += blockDim.x) whs[e] = bf2f(wh[e]);
  if (threadIdx.x < A1) bhs[threadIdx.x] = bf2f(bh[threadIdx.x]);
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; r++)
    if (b0 + r * kWaves < B) heads_sample_row_pre<A1>(hv[r], whs, bhs, t, c, seed, act, logp, vf, lout, act_now, B,
                                                      b0 + r * kWaves, lane);
  if (host_seq) __threadfence_system();  // this wave's action stores to host memory, visible to the CPU
  __syncthreads();  // every wave has read t / ctr
  if (threadIdx.x == 0) {
    *t_ptr = t + 1;
    if (ctr != t_ptr) *ctr = int64_t(c) + 1;
    if (host_seq) __hip_atomic_store(host_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// K12 row-split workspace (partials), one per (device, groups, rs),
// allocated on first use (outside any graph capture: the learner's eager warm-up steps come first)
// and kept for the process lifetime.
void k12_split_ws(int groups, int rs, hipStream_t stream, float** part) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int>, float*> cache;
  int dev = 0;
  RMM_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_tuple(dev, groups, rs);
  auto it = cache.find(key);
  if (it == cache.end()) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    RMM_HIP_CHECK(hipStreamIsCapturing(stream, &cs));
    if (cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("dense_heads_bwd: run one step eagerly before capturing (K12 row-split workspace)");
    float* p = nullptr;
    RMM_HIP_CHECK(hipMalloc(&p, sizeof(float) * size_t(groups) * rs * K12_PSLOTS * NT));
    it = cache.emplace(key, p).first;
  }
  *part = it->second;
}
}  // namespace dense

void dense_heads_fwd(const void* hidden, const void* wh, const void* bh, int64_t M, int A1, void* heads,
                     hipStream_t stream) {
  if (M <= 0) return;
  if (A1 < 1 || A1 > dense::AMAX) throw std::invalid_argument("dense_heads_fwd: 1 <= A+1 <= 16");
  const dim3 grid(uint32_t((M + 3) / 4)), block(256);
  auto U = [](const void* p) { return static_cast<const unsigned short*>(p); };
  auto* o = static_cast<unsigned short*>(heads);
#define RMM_K14(N)                                                                                   \
  case N:                                                                                            \
    hipLaunchKernelGGL(dense::k_heads_fwd<N>, grid, block, 0, stream, U(hidden), U(wh), U(bh), M, o); \
    break;
  switch (A1) {
    RMM_K14(1) RMM_K14(2) RMM_K14(3) RMM_K14(4) RMM_K14(5) RMM_K14(6) RMM_K14(7) RMM_K14(8)
    RMM_K14(9) RMM_K14(10) RMM_K14(11) RMM_K14(12) RMM_K14(13) RMM_K14(14) RMM_K14(15) RMM_K14(16)
  }
#undef RMM_K14
  RMM_HIP_CHECK(hipGetLastError());
}

void dense_heads_ppo(const void* hidden, const void* wh, const void* bh, const float* cols, const float* coef,
                     float* acc, const float* gout, int64_t M, int A1, void* dz, void* dpre, hipStream_t stream,
                     const int64_t* cidx, const int64_t* ctr, int64_t period, const float* hpart, int S,
                     const void* hb, void* hid_out) {
  if (hpart != nullptr && (S < 1 || hb == nullptr)) throw std::invalid_argument("dense_heads_ppo: partials need S >= 1 and the dense bias");
  if (M <= 0) return;
  if (period < 1) period = 1;
  if (A1 < 3 || A1 > dense::AMAX) throw std::invalid_argument("dense_heads_ppo: 2 <= A <= 15 actions");
  const dim3 grid(uint32_t((M + 3) / 4)), block(256);
  auto U = [](const void* p) { return static_cast<const unsigned short*>(p); };
  auto V = [](void* p) { return static_cast<unsigned short*>(p); };
#define RMM_K15(N)                                                                                        \
  case N:                                                                                                 \
    hipLaunchKernelGGL(dense::k_heads_ppo<N>, grid, block, 0, stream, U(hidden), U(wh), U(bh), cols, coef, \
                       acc, gout, M, V(dz), V(dpre), cidx, ctr, period, hpart, S, U(hb), V(hid_out));     \
    break;
  switch (A1) {
    RMM_K15(3) RMM_K15(4) RMM_K15(5) RMM_K15(6) RMM_K15(7) RMM_K15(8) RMM_K15(9)
    RMM_K15(10) RMM_K15(11) RMM_K15(12) RMM_K15(13) RMM_K15(14) RMM_K15(15) RMM_K15(16)
  }
#undef RMM_K15
  RMM_HIP_CHECK(hipGetLastError());
}

void dense_heads_sample(const void* hidden, const void* wh, const void* bh, const int64_t* t_ptr, const int64_t* ctr,
                        uint32_t seed, int64_t* act, float* logp, float* vf, float* lout, int64_t* act_now, int64_t B,
                        int A1, hipStream_t stream, unsigned int* done, const float* hpart, int S, const void* hb,
                        int64_t* host_seq) {
  if (B <= 0) return;
  if (host_seq != nullptr && done == nullptr) throw std::invalid_argument("dense_heads_sample: host_seq needs done");
  if (hpart != nullptr && (S < 1 || hb == nullptr)) throw std::invalid_argument("dense_heads_sample: partials need S >= 1 and the dense bias");
  if (A1 < 3 || A1 > dense::AMAX) throw std::invalid_argument("dense_heads_sample: 2 <= A <= 15 actions");
  auto U = [](const void* p) { return static_cast<const unsigned short*>(p); };
  // one-workgroup K16 up to one_wg_rows rows (RMM_K16_ONE_WG_ROWS: 32 or 64, default 32; RMM_K16_MULTI=1:
  // always the multi-workgroup K16 + completion counter, for A/B). 64 measured 13 us/step SLOWER at 50
  // rows (profiles/k16_layout_r4.txt): each wave runs its 4 rows (GEMV, butterfly, host stores) back to back
  static const int64_t one_wg_rows = [] {
    const char* m = std::getenv("RMM_K16_MULTI");
    if (m && m[0] == '1') return int64_t(0);
    return int64_t(32);
  }();
  if (done != nullptr && B <= one_wg_rows) {
    auto* tw = const_cast<int64_t*>(t_ptr);
    auto* cw = const_cast<int64_t*>(ctr);
#define RMM_K16S(N)                                                                                                 \
  case N:                                                                                                           \
    if (B <= 32)                                                                                                    \
      hipLaunchKernelGGL((dense::k_heads_sample1<N, 2>), dim3(1), dim3(1024), 0, stream, U(hidden), U(wh), U(bh), tw, \
                         cw, seed, act, logp, vf, lout, act_now, B, hpart, S, U(hb), host_seq);                    \
    else                                                                                                            \
      hipLaunchKernelGGL((dense::k_heads_sample1<N, 4>), dim3(1), dim3(1024), 0, stream, U(hidden), U(wh), U(bh), tw, \
                         cw, seed, act, logp, vf, lout, act_now, B, hpart, S, U(hb), host_seq);                    \
    break;
    switch (A1) {
      RMM_K16S(3) RMM_K16S(4) RMM_K16S(5) RMM_K16S(6) RMM_K16S(7) RMM_K16S(8) RMM_K16S(9)
      RMM_K16S(10) RMM_K16S(11) RMM_K16S(12) RMM_K16S(13) RMM_K16S(14) RMM_K16S(15) RMM_K16S(16)
    }
#undef RMM_K16S
    RMM_HIP_CHECK(hipGetLastError());
    return;
  }
  // waves (= rows) per workgroup of the multi-workgroup K16 (RMM_K16_WPW: 1, 2 or 4, default 4)
  static const int wpw = [] {
    const char* e = std::getenv("RMM_K16_WPW");
    const int v = e ? std::atoi(e) : 4;
    return (v == 1 || v == 2) ? v : 4;
  }();
  const dim3 grid(uint32_t((B + wpw - 1) / wpw)), block(uint32_t(64 * wpw));
#define RMM_K16(N)                                                                                          \
  case N:                                                                                                   \
    hipLaunchKernelGGL(dense::k_heads_sample<N>, grid, block, 0, stream, U(hidden), U(wh), U(bh), t_ptr, ctr, \
                       seed, act, logp, vf, lout, act_now, B, done, hpart, S, U(hb), host_seq);             \
    break;
  switch (A1) {
    RMM_K16(3) RMM_K16(4) RMM_K16(5) RMM_K16(6) RMM_K16(7) RMM_K16(8) RMM_K16(9)
    RMM_K16(10) RMM_K16(11) RMM_K16(12) RMM_K16(13) RMM_K16(14) RMM_K16(15) RMM_K16(16)
  }
#undef RMM_K16
  RMM_HIP_CHECK(hipGetLastError());
}

void dense_relu_fwd(const void* x, const void* w, const void* b, int64_t M, int64_t K, int N, void* y,
                    hipStream_t stream) {
  if (M <= 0) return;
  if (K % 32 != 0 || N % 16 != 0) throw std::invalid_argument("dense_relu_fwd: K % 32 == 0 and N % 16 == 0");
  const int remap = 1;  // grouped tile order (raster order measured slower)
  hipLaunchKernelGGL(dense::k_dense_fwd, dim3(uint32_t(((M + 15) / 16) * (N / 16))), dim3(256), 0, stream,
                     static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(w),
                     static_cast<const unsigned short*>(b), M, K, N, static_cast<unsigned short*>(y), remap);
  RMM_HIP_CHECK(hipGetLastError());
}

// K13s configurations (FM, FN, WM, WN): 0 = 16x16 tile, 4 waves split K (small M);
// 1 = 32x32 tile of 4 16x16 waves; 2 = 32x32 per wave, 4 waves split K; 3 = 64x32 per wave, 4 waves
// split K; 4 = 64x64 tile of 4 32x32 waves; 5 = 64x64 per wave, 6 = 32x64 per wave (4 waves split K).
struct PartCfg {
  int fm, fn, wm, wn;
};
static constexpr PartCfg kPartCfgs[] = {{1, 1, 1, 1}, {1, 1, 2, 2}, {2, 2, 1, 1}, {4, 2, 1, 1},
                                        {2, 2, 2, 2}, {4, 4, 1, 1}, {2, 4, 1, 1}};

static void dense_part_cfg(int64_t M, int64_t K, int N, int* cfg, int* S) {
  // default: by M; slices for ~512-1024 workgroups with >= 4 k-steps each, at most 16 (the
  // consumer sums S partial rows per lane). RMM_K13S_CFG / RMM_K13S_S override (tuning).
  static const int force_c = [] {
    const char* e = std::getenv("RMM_K13S_CFG");
    return e ? std::atoi(e) : -1;
  }();
  static const int force_s = [] {
    const char* e = std::getenv("RMM_K13S_S");
    return e ? std::atoi(e) : 0;
  }();
  int c = M <= 64 ? 0 : 6;
  if (force_c >= 0 && force_c < 7) c = force_c;
  const PartCfg& p = kPartCfgs[c];
  const int64_t tiles = ((M + 16 * p.fm * p.wm - 1) / (16 * p.fm * p.wm)) * (N / (16 * p.fn * p.wn));
  const int64_t steps = K / 32;
  int64_t s = M <= 64 ? 8 : (256 + tiles - 1) / tiles;
  s = std::min<int64_t>(s, std::max<int64_t>(1, steps / 4));
  s = std::max<int64_t>(1, std::min<int64_t>(s, 16));
  if (force_s > 0) s = std::min<int64_t>(force_s, steps);
  *cfg = c;
  *S = int(s);
}

int dense_fwd_part_slices(int64_t M, int64_t K, int N) {
  int c, S;
  dense_part_cfg(M, K, N, &c, &S);
  return S;
}

void dense_fwd_part(const void* x, const void* w, int64_t M, int64_t K, int N, float* part, int S,
                    hipStream_t stream) {
  if (M <= 0) return;
  if (K % 32 != 0 || N % 64 != 0) throw std::invalid_argument("dense_fwd_part: K % 32 == 0 and N % 64 == 0");
  int c, s_cfg;
  dense_part_cfg(M, K, N, &c, &s_cfg);
  if (S != s_cfg) throw std::invalid_argument("dense_fwd_part: S must be dense_fwd_part_slices(M, K, N)");
  const PartCfg& p = kPartCfgs[c];
  const int64_t tiles = ((M + 16 * p.fm * p.wm - 1) / (16 * p.fm * p.wm)) * (N / (16 * p.fn * p.wn));
  const dim3 grid(uint32_t(tiles * S)), block(256);
  auto U = [](const void* q) { return static_cast<const unsigned short*>(q); };
  switch (c) {
    case 0: hipLaunchKernelGGL((dense::k_dense_fwd_part<1, 1, 1, 1>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    case 1: hipLaunchKernelGGL((dense::k_dense_fwd_part<1, 1, 2, 2>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    case 2: hipLaunchKernelGGL((dense::k_dense_fwd_part<2, 2, 1, 1>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    case 3: hipLaunchKernelGGL((dense::k_dense_fwd_part<4, 2, 1, 1>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    case 4: hipLaunchKernelGGL((dense::k_dense_fwd_part<2, 2, 2, 2>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    case 5: hipLaunchKernelGGL((dense::k_dense_fwd_part<4, 4, 1, 1>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
    default: hipLaunchKernelGGL((dense::k_dense_fwd_part<2, 4, 1, 1>), grid, block, 0, stream, U(x), U(w), M, K, N, S, part); break;
  }
  RMM_HIP_CHECK(hipGetLastError());
}

static int k12_split_env() {
  static const int v = [] {
    const char* e = std::getenv("RMM_K12_SPLIT");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

DenseSplitPlan dense_split_plan(int64_t M, int64_t K, int split, hipStream_t stream) {
  DenseSplitPlan p;
  const int nc = int((M + dense::MC2 - 1) / dense::MC2);
  p.rs = std::max(1, std::min(split >= 1 ? split : k12_split_env(), nc));
  p.groups = int(K / dense::JB + 1);
  if (p.rs > 1) dense::k12_split_ws(p.groups, p.rs, stream, &p.part);
  return p;
}

void dense_heads_bwd(const void* dz, int A1, const void* wh, const void* y, const void* x, const void* w, int64_t M,
                     int64_t K, void* dx, void* dw, void* db, void* dwh, void* dbh, void* dpre_scratch,
                     hipStream_t stream, bool dpre_ready, const FusedAdam& fa, bool defer_finalize, int split) {
  if (M <= 0) return;
  if (K % dense::JB != 0) throw std::invalid_argument("dense_heads_bwd: K must be a multiple of 32");
  if (A1 < 1 || A1 > dense::AMAX) throw std::invalid_argument("dense_heads_bwd: 1 <= A+1 <= 16");
  if (M > dense::MMAX) throw std::invalid_argument("dense_heads_bwd: at most 640 rows per call");
  auto U = [](const void* p) { return static_cast<const unsigned short*>(p); };
  auto V = [](void* p) { return static_cast<unsigned short*>(p); };
  const dim3 block(dense::NT);
  if (fa.grad_base && fa.bump) throw std::invalid_argument("dense_heads_bwd: the step counters advance in the trunk reduce");
  const dim3 pgrid(uint32_t((M + dense::MC - 1) / dense::MC));
  auto* dp = V(dpre_scratch);
  // K12 row split + finalize kernel (split >= 1 explicit, else RMM_K12_SPLIT; plain gradients only, not
  // the fused-Adam epilogues). A deferred finalize must use the same `split` in dense_split_plan.
  const int nc = int((M + dense::MC2 - 1) / dense::MC2);
  const int rs = !fa.grad_base ? std::max(1, std::min(split >= 1 ? split : k12_split_env(), nc)) : 1;
  if (defer_finalize && rs < 2) throw std::invalid_argument("dense_heads_bwd: a deferred finalize needs the row split");
  const int groups = int(K / dense::JB + 1);
  float* rs_part = nullptr;
  if (rs > 1) dense::k12_split_ws(groups, rs, stream, &rs_part);
  const dim3 grid3(uint32_t(groups * rs));
#define RMM_K12(N)                                                                                               \
  case N:                                                                                                        \
    if (!dpre_ready)                                                                                             \
      hipLaunchKernelGGL(dense::k_dense_dpre<N>, pgrid, block, 0, stream, U(dz), U(wh), U(y), M, dp);            \
    hipLaunchKernelGGL(dense::k_dense_heads_bwd2<N>, grid3, block, 0, stream, U(dz), U(y), U(x), U(w), dp, M,   \
                       K, V(dx), V(dw), V(db), V(dwh), V(dbh), fa, rs_part, rs);                                  \
    break;
  switch (A1) {
    RMM_K12(1) RMM_K12(2) RMM_K12(3) RMM_K12(4) RMM_K12(5) RMM_K12(6) RMM_K12(7) RMM_K12(8)
    RMM_K12(9) RMM_K12(10) RMM_K12(11) RMM_K12(12) RMM_K12(13) RMM_K12(14) RMM_K12(15) RMM_K12(16)
  }
#undef RMM_K12
  RMM_HIP_CHECK(hipGetLastError());
  if (rs > 1 && !defer_finalize) {  // deferred: the K10 trunk-reduce launch finalizes (+ Adam)
    hipLaunchKernelGGL(dense::k_dense_split_finalize, dim3(uint32_t(groups), uint32_t(dense::K12_PSLOTS)), block, 0,
                       stream, rs_part, rs, K, A1, V(dw), V(db), V(dwh), V(dbh));
    RMM_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace hip
}  // namespace rmm
