// K12 — fused backward of the PPO dense tail: hidden = ReLU(x Wᵀ + b) [M, 256], heads = hidden Whᵀ + bh
// [M, A1]. Given dheads (the fused PPO loss gradient, K5c), ONE launch produces
//   dx  = dpre W            [M, K]        dW  = dpreᵀ x   [256, K]       db  = Σ_m dpre
//   dWh = dheadsᵀ hidden    [A1, 256]     dbh = Σ_m dheads
// with dpre = (dheads Wh) ⊙ [hidden > 0] recomputed on the fly (never stored in HBM).
// It replaces four hipBLASLt GEMMs (two of them 5-wide) and two bias/mask reductions (~45 µs at
// M = 500, K = 3872 on MI355X) — at this size every one of them is latency-bound.
//
// Decomposition: workgroup j owns the 32 input columns J = [32j, 32j+32) of x / W (K/32 of them),
// streams the batch in chunks of 32 rows and, per chunk, (a) recomputes dpre[32, 256] into LDS in
// both orientations, (b) stages x[chunk, J]ᵀ, then (c) waves 0-3 compute dx[chunk, J] (MFMA
// M=32 N=32 K=256) while waves 4-7 accumulate dW[:, J] += dpreᵀ x (M=256 N=32 K=32) in registers.
// Workgroup 0 also accumulates dWh, db (MFMA with a ones row) and dbh. Every reduction over rows
// happens inside one workgroup in a fixed order: deterministic, no atomics.
//
// MFMA 16x16x32 bf16 maps: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// C/D col l&15, row 4(l>>4)+i.
#include <hip/hip_bf16.h>

#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {
namespace dense {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int H = 256;       // hidden width
constexpr int MC = 32;       // rows per chunk
constexpr int JB = 32;       // columns of x / W per workgroup
constexpr int AMAX = 16;     // head width (A+1) limit
constexpr int NT = 512;      // 8 waves
constexpr int HP = H + 8;    // padded pitches (bank spread, keep 16-B alignment)
constexpr int MP = MC + 8;
constexpr int MMAX = 640;    // batch rows held in LDS (dheads and the dx output block)
static_assert(MC * JB / 2 == NT, "x staging: one (row, column pair) per thread");

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but NOT for
// its outstanding global loads, so the next chunk's prefetch stays in flight across it.
// (__syncthreads() carries a workgroup fence that drains vmcnt to 0 first.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

// A1 is a template parameter: a runtime `if (a < A1)` around the per-element Wh reads made hipcc
// branch around each LDS load and wait for it (measured 128 µs per call; see the dispatch below).
template <int A1>
__global__ __launch_bounds__(NT) void k_dense_heads_bwd(
    const unsigned short* __restrict__ dz, const unsigned short* __restrict__ wh,
    const unsigned short* __restrict__ y, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    const unsigned short* __restrict__ dpre, int64_t M, int64_t K, unsigned short* __restrict__ dx,
    unsigned short* __restrict__ dw,
    unsigned short* __restrict__ db, unsigned short* __restrict__ dwh, unsigned short* __restrict__ dbh) {
  __shared__ __attribute__((aligned(16))) unsigned short wt[JB * HP];   // W[:, J]ᵀ  [j][h]
  __shared__ __attribute__((aligned(16))) unsigned short whs[AMAX * H]; // Wh [a][h]
  __shared__ __attribute__((aligned(16))) unsigned short dm[MC * HP];   // dpre [m][h]
  __shared__ __attribute__((aligned(16))) unsigned short dt[H * MP];    // dpre [h][m]
  __shared__ __attribute__((aligned(16))) unsigned short xt[JB * MP];   // x[chunk, J]ᵀ [j][m]
  __shared__ __attribute__((aligned(16))) unsigned short yt[H * MP];    // hidden [h][m] (wg 0)
  __shared__ __attribute__((aligned(16))) unsigned short dzt[AMAX * MP];// dheads [a][m] (wg 0)
  // The whole dheads [M, A1] and this workgroup's dx block [M, 32] live in LDS: the chunk loop then
  // issues no global stores and no dependent global loads, so the only vmcnt waits are for the
  // prefetched hidden / x rows of the NEXT chunk (in-order vmcnt: an in-loop dx store or an eagerly
  // unpacked 10-byte dheads row made every chunk wait for all its loads and stores).
  __shared__ __attribute__((aligned(16))) unsigned short dzs[MMAX * A1];
  __shared__ __attribute__((aligned(16))) unsigned short dxs[MMAX * JB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t J0 = int64_t(blockIdx.x) * JB;
  const bool head_wg = blockIdx.x == 0;

  // ---- setup: W[:, J]ᵀ and Wh into LDS (loads batched ahead of the LDS writes), zero dzt
  {
    constexpr int PW = JB * H / NT;  // 16 per thread
    unsigned short wv[PW];
#pragma unroll
    for (int k = 0; k < PW; k++) {
      const int e = tid + NT * k, h = e / JB, j = e - h * JB;  // consecutive threads: consecutive j
      wv[k] = w[int64_t(h) * K + J0 + j];
    }
    constexpr int PH = AMAX * H / NT;  // 8 per thread
    unsigned short hv[PH];
#pragma unroll
    for (int k = 0; k < PH; k++) {
      const int e = tid + NT * k;
      hv[k] = wh[e < A1 * H ? e : 0];
    }
#pragma unroll
    for (int k = 0; k < PW; k++) {
      const int e = tid + NT * k, h = e / JB, j = e - h * JB;
      wt[j * HP + h] = wv[k];
    }
#pragma unroll
    for (int k = 0; k < PH; k++) {
      const int e = tid + NT * k;
      whs[e] = (e < A1 * H) ? hv[k] : static_cast<unsigned short>(0);
    }
    for (int e = tid; e < AMAX * MP; e += NT) dzt[e] = 0;
    constexpr int PZ = (MMAX * A1 + NT - 1) / NT;
    unsigned short zv[PZ];
    const int nz = int(M) * A1;
#pragma unroll
    for (int k = 0; k < PZ; k++) zv[k] = dz[min(tid + NT * k, nz - 1)];
#pragma unroll
    for (int k = 0; k < PZ; k++)
      if (tid + NT * k < nz) dzs[tid + NT * k] = zv[k];
  }

  f32x4 acc_dw[4][2];   // waves 4-7: h tiles (w-4)+4i, j tiles 0/1
  f32x4 acc_h[4][2];    // wg 0, waves 0-3: h tiles w+4i; [0] dWh, [1] db
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 2; k++) {
      acc_dw[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc_h[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  f32x4 acc_bh = {0.f, 0.f, 0.f, 0.f};  // wg 0, wave 0: dbh in column 0 (rows a = 4g+e)

  // per-thread staging registers, refilled for chunk c+1 while chunk c's MFMAs run
  // (a): row pm of the chunk, h in [hb, hb+16). Consecutive lanes take consecutive ROWS so the
  // transposed dpre/hidden stores ([h][m]) are conflict-free and Wh reads broadcast.
  const int pm = tid & (MC - 1), hb = (tid / MC) * 16;
  const int xm = tid >> 4, xj = (tid & 15) * 2;  // (b): row xm (0..31), cols xj, xj+1 (512 threads)
  uint4 rp0, rp1, ry0 = make_uint4(0, 0, 0, 0), ry1 = make_uint4(0, 0, 0, 0);
  uint32_t rx;
  auto stage = [&](int64_t m0) {  // unconditional clamped loads (see load_frame in K10)
    const int64_t row = m0 + pm, rc = row < M ? row : M - 1;
    rp0 = *reinterpret_cast<const uint4*>(&dpre[rc * H + hb]);
    rp1 = *reinterpret_cast<const uint4*>(&dpre[rc * H + hb + 8]);
    if (head_wg) {
      ry0 = *reinterpret_cast<const uint4*>(&y[rc * H + hb]);
      ry1 = *reinterpret_cast<const uint4*>(&y[rc * H + hb + 8]);
    }
    const int64_t xr = m0 + xm, xc = xr < M ? xr : M - 1;
    rx = *reinterpret_cast<const uint32_t*>(&x[xc * K + J0 + xj]);
  };
  stage(0);
  __syncthreads();

  for (int64_t m0 = 0; m0 < M; m0 += MC) {
    // ---- (a) dpre chunk from the staged registers (and wg 0: hidden / dheads transposed)
    {
      const bool valid = m0 + pm < M;
      u16x8 o0 = __builtin_bit_cast(u16x8, rp0), o1 = __builtin_bit_cast(u16x8, rp1);
      if (!valid) {
        o0 = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        o1 = o0;
      }
#pragma unroll
      for (int i = 0; i < 16; i++) dt[(hb + i) * MP + pm] = i < 8 ? o0[i] : o1[i - 8];
      *reinterpret_cast<u16x8*>(&dm[pm * HP + hb]) = o0;
      *reinterpret_cast<u16x8*>(&dm[pm * HP + hb + 8]) = o1;
      if (head_wg) {
        u16x8 h0 = __builtin_bit_cast(u16x8, ry0), h1 = __builtin_bit_cast(u16x8, ry1);
#pragma unroll
        for (int i = 0; i < 16; i++)
          yt[(hb + i) * MP + pm] = valid ? (i < 8 ? h0[i] : h1[i - 8]) : static_cast<unsigned short>(0);
        if (hb == 0) {
          const int zrow = int(valid ? m0 + pm : 0) * A1;
#pragma unroll
          for (int a = 0; a < A1; a++) dzt[a * MP + pm] = valid ? dzs[zrow + a] : static_cast<unsigned short>(0);
        }
      }
      // ---- (b) x[chunk, J]ᵀ
      {  // MC * JB / 2 == NT pairs: every thread writes one
        const bool xv = m0 + xm < M;
        xt[xj * MP + xm] = xv ? static_cast<unsigned short>(rx & 0xffffu) : static_cast<unsigned short>(0);
        xt[(xj + 1) * MP + xm] = xv ? static_cast<unsigned short>(rx >> 16) : static_cast<unsigned short>(0);
      }
    }
    if (m0 + MC < M) stage(m0 + MC);  // next chunk's loads fly during this chunk's MFMAs
    lds_barrier();

    if (wave < 4) {
      // ---- (c) dx[chunk, J] tile (mt, nt) = dm[32 x 256] · W[:, J]
      const int mt = wave >> 1, nt = wave & 1;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};  // two chains: half the MFMA latency
#pragma unroll
      for (int s = 0; s < H / 32; s += 2) {
        const bf16x8 a = as_bf(*reinterpret_cast<const u16x8*>(&dm[(mt * 16 + r) * HP + 32 * s + 8 * g]));
        const bf16x8 b = as_bf(*reinterpret_cast<const u16x8*>(&wt[(nt * 16 + r) * HP + 32 * s + 8 * g]));
        const bf16x8 a2 = as_bf(*reinterpret_cast<const u16x8*>(&dm[(mt * 16 + r) * HP + 32 * s + 32 + 8 * g]));
        const bf16x8 b2 = as_bf(*reinterpret_cast<const u16x8*>(&wt[(nt * 16 + r) * HP + 32 * s + 32 + 8 * g]));
        acc = mfma(a, b, acc);
        acc2 = mfma(a2, b2, acc2);
      }
      acc += acc2;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int64_t row = m0 + mt * 16 + 4 * g + i;
        if (row < M) dxs[row * JB + nt * 16 + r] = f2bf(acc[i]);
      }
      if (head_wg) {
        // dWh[a][h] += Σ_m dheads[m][a] hidden[m][h];  db[h] += Σ_m dpre[m][h] (A row 0 = ones)
        const bf16x8 az = as_bf(*reinterpret_cast<const u16x8*>(&dzt[r * MP + 8 * g]));
        u16x8 ones;
#pragma unroll
        for (int j = 0; j < 8; j++) ones[j] = (r == 0) ? static_cast<unsigned short>(0x3f80) : static_cast<unsigned short>(0);
        const bf16x8 a1 = as_bf(ones);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int ht = wave + 4 * i;
          const bf16x8 by = as_bf(*reinterpret_cast<const u16x8*>(&yt[(ht * 16 + r) * MP + 8 * g]));
          const bf16x8 bd = as_bf(*reinterpret_cast<const u16x8*>(&dt[(ht * 16 + r) * MP + 8 * g]));
          acc_h[i][0] = mfma(az, by, acc_h[i][0]);
          acc_h[i][1] = mfma(a1, bd, acc_h[i][1]);
        }
        if (wave == 0) {  // dbh[a] = Σ_m dheads[m][a]: dheadsᵀ times a ones column (col 0)
          u16x8 onec;
#pragma unroll
          for (int j = 0; j < 8; j++) onec[j] = (r == 0) ? static_cast<unsigned short>(0x3f80) : static_cast<unsigned short>(0);
          acc_bh = mfma(az, as_bf(onec), acc_bh);
        }
      }
    } else {
      // ---- (d) dW[:, J] += dpreᵀ[256 x 32] · x[chunk, J]   (K = the 32 chunk rows)
      const int w4 = wave - 4;
      const bf16x8 b0 = as_bf(*reinterpret_cast<const u16x8*>(&xt[r * MP + 8 * g]));
      const bf16x8 b1 = as_bf(*reinterpret_cast<const u16x8*>(&xt[(16 + r) * MP + 8 * g]));
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int ht = w4 + 4 * i;
        const bf16x8 a = as_bf(*reinterpret_cast<const u16x8*>(&dt[(ht * 16 + r) * MP + 8 * g]));
        acc_dw[i][0] = mfma(a, b0, acc_dw[i][0]);
        acc_dw[i][1] = mfma(a, b1, acc_dw[i][1]);
      }
    }
    lds_barrier();
  }

  // ---- epilogue: dx block out with 16-B stores (the loop ended on a barrier: dxs is complete)
  for (int v = tid; v < int(M) * (JB / 8); v += NT) {
    const int row = v / (JB / 8), c = v - row * (JB / 8);
    *reinterpret_cast<uint4*>(&dx[int64_t(row) * K + J0 + 8 * c]) = *reinterpret_cast<const uint4*>(&dxs[row * JB + 8 * c]);
  }
  if (wave >= 4) {
    const int w4 = wave - 4;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int ht = w4 + 4 * i;
#pragma unroll
      for (int nt = 0; nt < 2; nt++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int h = ht * 16 + 4 * g + e;
          dw[int64_t(h) * K + J0 + nt * 16 + r] = f2bf(acc_dw[i][nt][e]);
        }
    }
  } else if (head_wg) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int h = (wave + 4 * i) * 16 + r;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int a = 4 * g + e;
        if (a < A1) dwh[a * H + h] = f2bf(acc_h[i][0][e]);
      }
      if (g == 0) db[h] = f2bf(acc_h[i][1][0]);  // row 0 of the ones-row product
    }
  }
  if (head_wg && wave == 0 && r == 0) {
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (4 * g + e < A1) dbh[4 * g + e] = f2bf(acc_bh[e]);
  }
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
                                                   unsigned short* __restrict__ y) {
  // 4 waves split K (wave w takes k-steps s ≡ w mod 4), 4 accumulator chains each, partial tiles
  // combined through LDS in a fixed order: the serial L2-latency chain per wave is K/128 deep.
  __shared__ f32x4 part[3][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int64_t m0 = int64_t(blockIdx.x) * 16, n0 = int64_t(blockIdx.y) * 16;
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

}  // namespace dense

void dense_relu_fwd(const void* x, const void* w, const void* b, int64_t M, int64_t K, int N, void* y,
                    hipStream_t stream) {
  if (M <= 0) return;
  if (K % 32 != 0 || N % 16 != 0) throw std::invalid_argument("dense_relu_fwd: K % 32 == 0 and N % 16 == 0");
  hipLaunchKernelGGL(dense::k_dense_fwd, dim3(uint32_t((M + 15) / 16), uint32_t(N / 16)), dim3(256), 0, stream,
                     static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(w),
                     static_cast<const unsigned short*>(b), M, K, N, static_cast<unsigned short*>(y));
  RMM_HIP_CHECK(hipGetLastError());
}

void dense_heads_bwd(const void* dz, int A1, const void* wh, const void* y, const void* x, const void* w, int64_t M,
                     int64_t K, void* dx, void* dw, void* db, void* dwh, void* dbh, void* dpre_scratch,
                     hipStream_t stream) {
  if (M <= 0) return;
  if (K % dense::JB != 0) throw std::invalid_argument("dense_heads_bwd: K must be a multiple of 32");
  if (A1 < 1 || A1 > dense::AMAX) throw std::invalid_argument("dense_heads_bwd: 1 <= A+1 <= 16");
  if (M > dense::MMAX) throw std::invalid_argument("dense_heads_bwd: at most 640 rows per call");
  auto U = [](const void* p) { return static_cast<const unsigned short*>(p); };
  auto V = [](void* p) { return static_cast<unsigned short*>(p); };
  const dim3 grid(uint32_t(K / dense::JB)), block(dense::NT);
  const dim3 pgrid(uint32_t((M + dense::MC - 1) / dense::MC));
  auto* dp = V(dpre_scratch);
#define RMM_K12(N)                                                                                               \
  case N:                                                                                                        \
    hipLaunchKernelGGL(dense::k_dense_dpre<N>, pgrid, block, 0, stream, U(dz), U(wh), U(y), M, dp);              \
    hipLaunchKernelGGL(dense::k_dense_heads_bwd<N>, grid, block, 0, stream, U(dz), U(wh), U(y), U(x), U(w), dp,  \
                       M, K, V(dx), V(dw), V(db), V(dwh), V(dbh));                                               \
    break;
  switch (A1) {
    RMM_K12(1) RMM_K12(2) RMM_K12(3) RMM_K12(4) RMM_K12(5) RMM_K12(6) RMM_K12(7) RMM_K12(8)
    RMM_K12(9) RMM_K12(10) RMM_K12(11) RMM_K12(12) RMM_K12(13) RMM_K12(14) RMM_K12(15) RMM_K12(16)
  }
#undef RMM_K12
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
