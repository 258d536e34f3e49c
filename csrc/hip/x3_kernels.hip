// Precision-matched (fp32-level) twins of the PPO SGD-step and rollout-step kernels, on the bf16 MFMA
// through split-bf16 operands (x3_device.h): K10x (Nature-CNN trunk fwd / bwd), K13x (split-K dense),
// K15x (heads + PPO loss + dheads + dpre), K12x (dense + heads backward), K16x (heads + sampling).
//
// Parity target: the reference trains PPO in fp32 torch (rllib/algorithms/ppo/ppo_torch_policy.py:70,
// rllib/models/torch/visionnet.py). Here every tensor is fp32-equivalent: weights are the fp32 master
// (carried to the kernels as its split pair), activations / activation gradients are split pairs
// (≈17 significant bits), products use hi*hi + hi*lo + lo*hi with fp32 accumulation, gradients are
// reduced and stored in fp32, the loss and the optimizer run in fp32. The bf16 learner rounds
// activations, gradients and head outputs to 8 significant bits instead.
//
// Layout changes vs the bf16 kernels (the split pairs double the LDS images):
//   * K10x fwd: one workgroup of 8 waves per CU loops over frames (the full bf16 frame image,
//     h1 hi/lo, W1 hi/lo and W2 hi/lo = 149 KB of LDS), next frame's loads in flight;
//   * K10x bwd: conv2's backward (dW2, db2, dh1 -> dpre1, db1; 76 KB, two workgroups per CU) and
//     conv1's weight gradient (space-to-depth frame + dpre1; 145 KB) are two launches; dpre1 goes
//     through HBM as a split pair;
//   * K12x: 64-row chunks single-buffered in LDS with the next chunk's loads in registers (the bf16
//     K12 double-buffers and keeps the whole dx block in LDS), dx stored per chunk.
// MFMA 16x16x32 bf16 maps: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15];
// C/D col l&15, row 4(l>>4)+i.
#include <hip/hip_bf16.h>

#include "adam_device.h"
#include "common.h"
#include "dense_device.h"
#include "kernels.h"
#include "trunk_device.h"
#include "x3_device.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace rmm {
namespace hip {
namespace x3 {

using trunk::C0;
using trunk::C1;
using trunk::C2;
using trunk::FrameRegs;
using trunk::H0;
using trunk::H1;
using trunk::H1P_ELEMS;
using trunk::H2;
using trunk::NP1;
using trunk::NP2;
using trunk::NP2P;
using trunk::P0;
using trunk::P1;
using trunk::W1_PITCH;
using trunk::W2_PITCH;
using trunk::WeightRegs;
using trunk::WStrides;

// ---------------------------------------------------------------- phase probe (opt-in, x3_probe_set)
// When a buffer is set (before the learner captures its SGD graphs: the pointer is a kernel argument), thread 0
// of every workgroup stores the 100 MHz real-time counter at the kernels' phase boundaries:
// ts[(kernel * 1024 + workgroup) * 16 + slot] (benchmarks/x3_phase_probe.py reads it). The sites compile to
// nothing unless the extension is built with RMM_X3_PROBE=1 (build_native.py): even a null-pointer test per
// site measured +0.3 us on kernels that had only two (same-box A/B), and a device-global pointer cost a load
// whose wait drained every memory op in flight at each site.
uint64_t* g_x3_probe = nullptr;  // host side: the buffer the launchers pass
enum : int { TS_FWD = 0, TS_C2B = 1, TS_C1W = 2, TS_K12 = 3, TS_RED = 4, TS_K13L = 5, TS_K15 = 6 };
__device__ __forceinline__ void x3_ts(uint64_t* ts, int k, int slot) {
#ifdef RMM_X3_PROBE
  if (ts != nullptr && threadIdx.x == 0 && blockIdx.x < 1024 && slot < 16)
    ts[(int64_t(k) * 1024 + blockIdx.x) * 16 + slot] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ================================================================ K10x forward
constexpr int NTF = 512;  // 8 waves (1024 threads cap a lane at 128 VGPRs: the W1 / W2 pair fragments spilled)
constexpr int FIMG = P0 * P0 * C0;  // the whole padded HWC frame as bf16 (exact for 0..255)

// frame words in registers -> bf16 HWC image interior (padded row y+2, column x+2)
template <int NT>
__device__ __forceinline__ void frame_image_store(const FrameRegs<NT>& f, unsigned short* img) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
      const int y = o / 21, xw = o - y * 21;
      uint32_t w[8];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t c0 = __float_as_uint(float((f.v[k][0] >> (8 * q)) & 0xffu));
        const uint32_t c1 = __float_as_uint(float((f.v[k][1] >> (8 * q)) & 0xffu));
        const uint32_t c2 = __float_as_uint(float((f.v[k][2] >> (8 * q)) & 0xffu));
        const uint32_t c3 = __float_as_uint(float((f.v[k][3] >> (8 * q)) & 0xffu));
        w[2 * q] = trunk::bf16pair(c0, c1);
        w[2 * q + 1] = trunk::bf16pair(c2, c3);
      }
      uint4* d = reinterpret_cast<uint4*>(img + ((y + 2) * P0 + 4 * xw + 2) * C0);
      d[0] = make_uint4(w[0], w[1], w[2], w[3]);
      d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
  }
}
// zero the 2-pixel border of the bf16 image (rows 0, 1, 86, 87; columns 0, 1, 86, 87)
__device__ __forceinline__ void zero_image_border(unsigned short* img) {
  uint2* f = reinterpret_cast<uint2*>(img);  // one uint2 = one pixel (4 bf16)
  constexpr int NROW = 4 * P0, NCOL = (P0 - 4) * 4;
  for (int i = threadIdx.x; i < NROW + NCOL; i += blockDim.x) {
    int y, x;
    if (i < NROW) {
      const int r = i / P0;
      y = r < 2 ? r : r + (P0 - 4);
      x = i - r * P0;
    } else {
      const int j = i - NROW, c = j & 3;
      y = 2 + (j >> 2);
      x = c < 2 ? c : c + (P0 - 4);
    }
    f[y * P0 + x] = make_uint2(0u, 0u);
  }
}

// grid = G workgroups, each loops over frames b = blockIdx.x, +G, ... (push mode: G = B, one frame each)
__global__ __launch_bounds__(NTF) void k_trunk_fwd_x3(
    const uint8_t* __restrict__ obs, const int64_t* __restrict__ idx0, const int64_t* __restrict__ ctr, int64_t period,
    int64_t B, CPair W1, WStrides w1, CPair b1, CPair W2, WStrides w2, CPair b2, Pair h1_out, Pair h2_out,
    uint8_t* push_stack, const uint8_t* __restrict__ push_new, uint8_t* push_rows, const int64_t* __restrict__ push_t,
    const int64_t* gate, int64_t gate_want, int* gate_err, int gate_parts, int gate_timeout_ms,
    const float* __restrict__ cols, float* __restrict__ cols_out, int ncols, uint64_t* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) unsigned short img[FIMG];
  __shared__ __attribute__((aligned(16))) unsigned short h1h[H1P_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short h1l[H1P_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short w1h[C1 * W1_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w1l[C1 * W1_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w2h[C2 * W2_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w2l[C2 * W2_PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t G = gridDim.x;
  const int64_t* idx = trunk::window(idx0, ctr, period, B);
  constexpr int64_t FB = C0 * H0 * H0;
  x3_ts(ts, TS_FWD, 0);

  // prologue: weight loads (L2), then the first frame's HBM loads, then zeroing and staging
  WeightRegs<NTF, C1, C0, 8> r1h, r1l;
  WeightRegs<NTF, C2, C1, 4> r2h, r2l;
  trunk::weight_issue(W1.hi, w1, r1h);
  trunk::weight_issue(W1.lo, w1, r1l);
  trunk::weight_issue(W2.hi, w2, r2h);
  trunk::weight_issue(W2.lo, w2, r2l);
  FrameRegs<NTF> fr;
  int64_t b = blockIdx.x;
  if (gate) {
    // step gate: this launch was enqueued before the host stepped the envs; wait for the release counter
    // (mapped pinned memory, bumped after the new frames are written) before reading them. With
    // gate_parts P the host steps the envs in P ranges and bumps the counter after each, so frame b waits
    // only for its own range: the first ranges' frames cross PCIe and their conv1
    // runs while the host still steps the rest. Bounded by wall clock (gate_timeout_ms on the 100 MHz
    // real-time counter): a host that died mid-fragment can never leave a wave spinning (*gate_err is
    // set; the worker then re-runs the fragment ungated instead of using stale frames)
    if (threadIdx.x == 0) {
      // range of frame b under the host's split [B p / P, B (p + 1) / P): p = ((b + 1) P - 1) / B
      const int64_t want = gate_want + (gate_parts > 1 ? ((b + 1) * gate_parts - 1) / B : 0);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      const uint64_t limit = uint64_t(gate_timeout_ms > 0 ? gate_timeout_ms : 2000) * 100000ull;
      while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
          if (gate_err) __hip_atomic_store(gate_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
  }
  if (push_stack)
    trunk::frame_issue_push<NTF>(push_stack + b * FB, push_new + b * (H0 * H0), fr);
  else
    trunk::frame_issue<NTF>(obs + (idx ? idx[b] : b) * FB, fr);
  const float bias1 = join(b1, r), bias2[2] = {join(b2, r), join(b2, 16 + r)};
  zero_image_border(img);
  trunk::zero_lds(h1h, H1P_ELEMS * 2);
  trunk::zero_lds(h1l, H1P_ELEMS * 2);
  trunk::weight_store(r1h, W1.hi, w1, w1h, W1_PITCH);
  trunk::weight_store(r1l, W1.lo, w1, w1l, W1_PITCH);
  trunk::weight_store(r2h, W2.hi, w2, w2h, W2_PITCH);
  trunk::weight_store(r2l, W2.lo, w2, w2l, W2_PITCH);
  if (push_stack)
    trunk::frame_push_store<NTF>(fr, push_stack + b * FB, push_rows ? push_rows + (push_t[0] * B + b) * FB : nullptr);
  // every B fragment a wave multiplies is the same for all its tiles and frames: conv1's depends on the
  // k-step only (N = 16), conv2's on the k-step and the wave's N tile (jobs step by 8 waves, so a wave's
  // nt = wave & 1 never changes) — read them from LDS once (128 VGPRs) instead of 2 of every 3 (conv1) /
  // 4 (conv2) LDS reads per MFMA group
  __syncthreads();  // weights staged
  x3_ts(ts, TS_FWD, 1);
  bf16x8 w1fh[8], w1fl[8], w2fh[8], w2fl[8];
  {
    const int nt = wave & 1;
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const int wo1 = r * W1_PITCH + (s * 8 + 2 * g) * 4;
      w1fh[s] = ld8(&w1h[wo1]), w1fl[s] = ld8(&w1l[wo1]);
      const int pp = 2 * s + (g >> 1);
      const int wo2 = (nt * 16 + r) * W2_PITCH + pp * 16 + 8 * (g & 1);
      w2fh[s] = ld8(&w2h[wo2]), w2fl[s] = ld8(&w2l[wo2]);
    }
  }

  for (; b < B; b += G) {
    // the frame's PPO loss columns, gathered through the same index window, so the loss kernel (K15x)
    // reads its row directly instead of a step counter -> index -> row chain of dependent loads
    if (cols_out != nullptr && int(threadIdx.x) < ncols)
      cols_out[b * ncols + threadIdx.x] = cols[(idx ? idx[b] : b) * ncols + threadIdx.x];
    frame_image_store<NTF>(fr, img);
    __syncthreads();  // image (+ first frame: border / h1 zeros, weights); the previous conv2 is done
    const int fi = int((b - blockIdx.x) / G);
    x3_ts(ts, TS_FWD, 2 + 3 * fi);
    if (b + G < B) trunk::frame_issue<NTF>(obs + (idx ? idx[b + G] : b + G) * FB, fr);  // in flight meanwhile

    // ---- conv1: M = 441 positions (28 tiles) x N = 16 x K = 256 (k = ky, kx, ci); frame exact -> 2 MFMAs
    for (int mt = wave; mt < 28; mt += NTF / 64) {
      const int p = min(mt * 16 + r, NP1 - 1);
      const int oy = p / H1, ox = p - oy * H1;
      Acc acc = acc0();
#pragma unroll
      for (int s = 0; s < 8; s++) mma2a(acc, ld8(&img[((4 * oy + s) * P0 + 4 * ox + 2 * g) * C0]), w1fh[s], w1fl[s]);
      const f32x4 t = total(acc);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int q = mt * 16 + 4 * g + i;
        if (q < NP1) {
          const float v = fmaxf(t[i] * (1.0f / 255.0f) + bias1, 0.f);
          const int y = q / H1, x = q - y * H1;
          unsigned short hh, hl;
          split(v, hh, hl);
          const int o = ((y + 2) * P1 + (x + 2)) * C1 + r;
          h1h[o] = hh;
          h1l[o] = hl;
          if (h1_out.hi) {
            const int64_t go = (b * NP1 + q) * C1 + r;
            h1_out.hi[go] = hh;
            h1_out.lo[go] = hl;
          }
        }
      }
    }
    __syncthreads();
    x3_ts(ts, TS_FWD, 3 + 3 * fi);

    // ---- conv2: 8 M-tiles x 2 N-tiles = 16 jobs over the waves, K = 256 (pixel pp = 2s + (g>>1), ci half g&1)
    static_assert(NTF / 64 % 2 == 0, "a wave's conv2 N tile (job & 1) must not change");
    for (int job = wave; job < 16; job += NTF / 64) {
      const int mt = job >> 1, nt = job & 1;
      const int q = min(mt * 16 + r, NP2 - 1);
      const int oy = q / H2, ox = q - oy * H2;
      Acc acc = acc0();
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int pp = 2 * s + (g >> 1), ky = pp >> 2, kx = pp & 3;
        const int ao = ((2 * oy + ky) * P1 + (2 * ox + kx)) * C1 + 8 * (g & 1);
        mma3(acc, ld8(&h1h[ao]), ld8(&h1l[ao]), w2fh[s], w2fl[s]);
      }
      const f32x4 t = total(acc);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int qq = mt * 16 + 4 * g + i;
        if (qq < NP2) store1(h2_out, (b * NP2 + qq) * C2 + nt * 16 + r, fmaxf(t[i] + bias2[nt], 0.f));
      }
    }
    x3_ts(ts, TS_FWD, 4 + 3 * fi);
  }
  x3_ts(ts, TS_FWD, 15);
}

// ================================================================ K10x backward, launch 1: conv2
// Per frame: dpre2 = dh2 * [h2 > 0] (db2), dW2 += dpre2ᵀ im2col(h1), dh1 = conv2ᵀ(dpre2) by stride-parity
// class, dpre1 = dh1 * [h1 > 0] (db1) -> HBM (split pair [B][441][16], read by launch 2).
// Per-workgroup fp32 partial: [dW2 32x256 (k = ky, kx, ci)][db2 32][db1 16].
constexpr int NTB = 512;
constexpr int DP2_PITCH = NP2P + 8, D2W = 12;
constexpr int PART2 = C2 * 256 + C2 + C1;
constexpr int B1_NH1 = NP1 * 2, B1_PH1 = (B1_NH1 + NTB - 1) / NTB;  // 882 x 16 B per plane
constexpr int B1_NH2 = NP2 * 4, B1_PH2 = (B1_NH2 + NTB - 1) / NTB;  // 484 x 16 B per plane
static_assert(B1_PH2 == 1, "one h2 / dh2 chunk per thread");

struct B1Regs {
  u16x8 h1h[B1_PH1], h1l[B1_PH1], h2[B1_PH2], dh[B1_PH2], dl[B1_PH2];
};
__device__ __forceinline__ void b1_issue(int64_t bb, CPair h1, const unsigned short* __restrict__ h2hi, CPair dh2,
                                         B1Regs& R) {
#pragma unroll
  for (int k = 0; k < B1_PH1; k++) {
    const int v = min(int(threadIdx.x) + NTB * k, B1_NH1 - 1);
    const int64_t o = (bb * NP1 + (v >> 1)) * C1 + 8 * (v & 1);
    R.h1h[k] = *reinterpret_cast<const u16x8*>(&h1.hi[o]);
    R.h1l[k] = *reinterpret_cast<const u16x8*>(&h1.lo[o]);
  }
  const int v = min(int(threadIdx.x), B1_NH2 - 1);
  const int64_t o = (bb * NP2 + (v >> 2)) * C2 + 8 * (v & 3);
  R.h2[0] = *reinterpret_cast<const u16x8*>(&h2hi[o]);
  R.dh[0] = *reinterpret_cast<const u16x8*>(&dh2.hi[o]);
  R.dl[0] = *reinterpret_cast<const u16x8*>(&dh2.lo[o]);
}

__global__ __launch_bounds__(NTB) void k_conv2_bwd_x3(int64_t B, CPair W2, WStrides w2, CPair h1,
                                                      const unsigned short* __restrict__ h2hi, CPair dh2,
                                                      Pair dpre1, float* __restrict__ partial,
                                                      int dbg /* timing probes: bit 1 skips dW2, bit 2 dh1 */,
                                                      uint64_t* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) unsigned short h1s[2 * H1P_ELEMS];      // hi plane, lo plane
  __shared__ __attribute__((aligned(16))) unsigned short dp2[2 * D2W * D2W * C2];   // [plane][oy*12+ox][co2]
  __shared__ __attribute__((aligned(16))) unsigned short dp2t[2 * C2 * DP2_PITCH];  // [plane][co2][kperm(q)]
  __shared__ float red[8 * 64];
  // the frame's dpre1 pair, staged so it leaves in coalesced 16-B stores (scattered 2-B stores measured 7.9 us
  // of the launch's 23.5; one workgroup per CU leaves the LDS for it)
  __shared__ __attribute__((aligned(16))) unsigned short dq[2 * NP1 * C1];
  static_assert(2 * C2 * W2_PITCH <= 2 * H1P_ELEMS, "W2 staging aliases the h1 tile");
  unsigned short* h1hs = h1s;
  unsigned short* h1ls = h1s + H1P_ELEMS;
  unsigned short* w2hs = h1s;                   // staging only (read into registers before the loop)
  unsigned short* w2ls = h1s + C2 * W2_PITCH;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  constexpr int DPL = D2W * D2W * C2, DTL = C2 * DP2_PITCH;
  x3_ts(ts, TS_C2B, 0);

  WeightRegs<NTB, C2, C1, 4> wrh, wrl;
  trunk::weight_issue(W2.hi, w2, wrh);
  trunk::weight_issue(W2.lo, w2, wrl);
  B1Regs R;
  if (int64_t(blockIdx.x) < B) b1_issue(blockIdx.x, h1, h2hi, dh2, R);
  trunk::zero_lds(dp2, 2 * DPL * 2);
  trunk::zero_lds(dp2t, 2 * DTL * 2);
  trunk::weight_store(wrh, W2.hi, w2, w2hs, W2_PITCH);
  trunk::weight_store(wrl, W2.lo, w2, w2ls, W2_PITCH);
  // dh1 = conv2ᵀ(dpre2): waves 2c, 2c+1 own stride-parity class c = (py, px); taps t = (ty, tx)
  const int cls = wave >> 1, half = wave & 1;
  const int py = cls >> 1, px = cls & 1;
  const int nrow = py ? 10 : 11, ncol = px ? 10 : 11, ncls = nrow * ncol;
  const uint32_t cdiv = px ? 6554u : 5958u;  // m / ncol for m < 200 as multiply-shift
  __syncthreads();
  bf16x8 wth[4], wtl[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
    u16x8 vh, vl;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      vh[j] = w2hs[(8 * g + j) * W2_PITCH + (ky * 4 + kx) * 16 + r];
      vl[j] = w2ls[(8 * g + j) * W2_PITCH + (ky * 4 + kx) * 16 + r];
    }
    wth[t] = as_bf(vh);
    wtl[t] = as_bf(vl);
  }
  __syncthreads();  // the W2 staging (aliasing the h1 tile) is read
  trunk::zero_lds(h1s, 2 * H1P_ELEMS * 2);
  Acc aw2[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++) aw2[0][i] = aw2[1][i] = acc0();
  float db1 = 0.f, db2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  __syncthreads();
  x3_ts(ts, TS_C2B, 1);

  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    const int fi = int((b - blockIdx.x) / gridDim.x);
    // ---- P0: h1 -> padded tile planes, dpre2 (both layouts, both planes) + db2
#pragma unroll
    for (int k = 0; k < B1_PH1; k++) {
      const int v = threadIdx.x + NTB * k;
      if (v < B1_NH1) {
        const int p = v >> 1, y = p / H1, x = p - y * H1;
        const int o = ((y + 2) * P1 + (x + 2)) * C1 + 8 * (v & 1);
        *reinterpret_cast<u16x8*>(&h1hs[o]) = R.h1h[k];
        *reinterpret_cast<u16x8*>(&h1ls[o]) = R.h1l[k];
      }
    }
    if (int(threadIdx.x) < B1_NH2) {
      const int v = threadIdx.x;
      const int q = v >> 2, c0 = 8 * (v & 3), oy = q / H2, ox = q - oy * H2;
      u16x8 oh, ol;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const unsigned short hj = R.h2[0][j];
        const bool on = hj != 0 && !(hj & 0x8000);
        oh[j] = on ? R.dh[0][j] : static_cast<unsigned short>(0);
        ol[j] = on ? R.dl[0][j] : static_cast<unsigned short>(0);
        db2[j] += bf2f(oh[j]) + bf2f(ol[j]);
        dp2t[(c0 + j) * DP2_PITCH + trunk::kperm(q)] = oh[j];
        dp2t[DTL + (c0 + j) * DP2_PITCH + trunk::kperm(q)] = ol[j];
      }
      *reinterpret_cast<u16x8*>(&dp2[(oy * D2W + ox) * C2 + c0]) = oh;
      *reinterpret_cast<u16x8*>(&dp2[DPL + (oy * D2W + ox) * C2 + c0]) = ol;
    }
    __syncthreads();
    x3_ts(ts, TS_C2B, 2 + 4 * fi);
    if (b + gridDim.x < B) b1_issue(b + gridDim.x, h1, h2hi, dh2, R);  // next frame: in flight through P1

    // ---- P1a: dW2[co2][k = (ky, kx, ci)] += Σ_q dpre2[q][co2] · h1[2oy+ky][2ox+kx][ci]
#pragma unroll
    for (int s = 0; s < ((dbg & 1) ? 0 : NP2P / 32); s++) {
      const int ao0 = r * DP2_PITCH + 32 * s + 8 * g, ao1 = (16 + r) * DP2_PITCH + 32 * s + 8 * g;
      const bf16x8 a0h = ld8(&dp2t[ao0]), a0l = ld8(&dp2t[DTL + ao0]);
      const bf16x8 a1h = ld8(&dp2t[ao1]), a1l = ld8(&dp2t[DTL + ao1]);
      int qoff[8];
      {
        const int q0 = 32 * s + g;
        int oy = q0 / H2, ox = q0 - oy * H2;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          qoff[j] = (q0 + 4 * j < NP2) ? (oy * 2 * P1 + ox * 2) * C1 : 0;  // dpre2 is 0 there
          ox += 4;
          if (ox >= H2) {
            ox -= H2;
            oy++;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int k = (wave + 8 * i) * 16 + r;
        const int ky = k >> 6, kx = (k >> 4) & 3, ci = k & 15;
        const int base = (ky * P1 + kx) * C1 + ci;
        u16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          bh[j] = h1hs[base + qoff[j]];
          bl[j] = h1ls[base + qoff[j]];
        }
        mma3(aw2[0][i], a0h, a0l, as_bf(bh), as_bf(bl));
        mma3(aw2[1][i], a1h, a1l, as_bf(bh), as_bf(bl));
      }
    }
    x3_ts(ts, TS_C2B, 3 + 4 * fi);
    // ---- P1b: dh1 for this wave's parity class, masked by h1 > 0 -> dpre1 (HBM), db1
    for (int mt = half; mt * 16 < ((dbg & 2) ? 0 : ncls); mt += 2) {
      const int m = min(mt * 16 + r, ncls - 1);
      const int a = int((uint32_t(m) * cdiv) >> 16), c = m - a * ncol;
      Acc acc = acc0();
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int oy = a + 1 - (t >> 1), ox = c + 1 - (t & 1);
        const int o = (oy * D2W + ox) * C2 + 8 * g;
        mma3(acc, ld8(&dp2[o]), ld8(&dp2[DPL + o]), wth[t], wtl[t]);
      }
      const f32x4 tt = total(acc);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int mm = mt * 16 + 4 * g + i;
        if (mm < ncls) {
          const int aa = int((uint32_t(mm) * cdiv) >> 16), cc = mm - aa * ncol;
          const int y = 2 * aa + py, x = 2 * cc + px;
          const unsigned short hv = h1hs[((y + 2) * P1 + (x + 2)) * C1 + r];
          const float d = (hv != 0 && !(hv & 0x8000)) ? tt[i] : 0.f;
          unsigned short dh, dl;
          split(d, dh, dl);
          db1 += bf2f(dh) + bf2f(dl);
          const int lo_ = (y * H1 + x) * C1 + r;
          dq[lo_] = dh;
          dq[NP1 * C1 + lo_] = dl;
        }
      }
    }
    __syncthreads();  // tiles free for the next frame; dq complete
    x3_ts(ts, TS_C2B, 4 + 4 * fi);
    {  // dpre1 pair of frame b: 2 x 441 x 16 bf16 -> HBM in 16-B vectors
      constexpr int NV = NP1 * C1 / 8;  // vectors per plane
      const int64_t go = b * NP1 * C1;
      for (int v = threadIdx.x; v < 2 * NV; v += NTB) {
        const int pl = v >= NV, vv = v - pl * NV;
        const u16x8 d = *reinterpret_cast<const u16x8*>(&dq[pl * NP1 * C1 + 8 * vv]);
        *reinterpret_cast<u16x8*>(&(pl ? dpre1.lo : dpre1.hi)[go + 8 * vv]) = d;
      }
    }
    x3_ts(ts, TS_C2B, 5 + 4 * fi);
  }

  float* out = partial + int64_t(blockIdx.x) * PART2;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int col = (wave + 8 * i) * 16 + r;
    const f32x4 t0 = total(aw2[0][i]), t1 = total(aw2[1][i]);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int row = 4 * g + e;
      out[row * 256 + col] = t0[e];
      out[(16 + row) * 256 + col] = t1[e];
    }
  }
  // db2: thread t holds co2 = 8(t&3)+j (threads < 484 only touched it); db1: lanes r, r+16.. share ci = r
#pragma unroll
  for (int j = 0; j < 8; j++) {
    float v = db2[j];
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 4) red[wave * 64 + lane * 8 + j] = v;
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int co = threadIdx.x, q4 = co >> 3, j = co & 7;
    float s = 0.f;
    for (int w = 0; w < 8; w++) s += red[w * 64 + q4 * 8 + j];
    out[C2 * 256 + co] = s;
  }
  __syncthreads();
  db1 += __shfl_xor(db1, 16);
  db1 += __shfl_xor(db1, 32);
  if (lane < 16) red[wave * 16 + lane] = db1;
  __syncthreads();
  if (threadIdx.x < 16) {
    float s = 0.f;
    for (int w = 0; w < 8; w++) s += red[w * 16 + threadIdx.x];
    out[C2 * 256 + C2 + threadIdx.x] = s;
  }
  x3_ts(ts, TS_C2B, 15);
}

// ================================================================ K10x backward, launch 2: conv1 dW1
// dW1 in space-to-depth form (see conv_kernels.hip P2): D[(a, b, c)][co] = Σ_t st[c][t] · dpre1_b[co][t + (1-a)*24]
// with the frame exact in bf16 (2 MFMAs) and dpre1 a split pair (two shifted copies b = 0, 1 per plane).
using trunk::ST_C;
using trunk::ST_CP;
using trunk::ST_W;
constexpr int DB_CP = 24 * ST_W + 8, DB_B = 16 * DB_CP;
constexpr int KSTEPS1 = (22 * ST_W + 31) / 32;
constexpr int PART1 = C1 * 256;
constexpr int B2_N = NP1 * 2, B2_PER = (B2_N + NTB - 1) / NTB;  // 882 x 16 B per plane

__global__ __launch_bounds__(NTB) void k_conv1_wgrad_x3(const uint8_t* __restrict__ obs,
                                                        const int64_t* __restrict__ idx0,
                                                        const int64_t* __restrict__ ctr, int64_t period, int64_t B,
                                                        CPair dpre1, float* __restrict__ partial,
                                                        uint64_t* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) unsigned short st[trunk::ST_ELEMS];  // space-to-depth frame (exact)
  __shared__ __attribute__((aligned(16))) unsigned short dp[4 * DB_B];        // [hi b0][hi b1][lo b0][lo b1]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t* idx = trunk::window(idx0, ctr, period, B);
  FrameRegs<NTB> fr;
  u16x8 vh[B2_PER], vl[B2_PER];
  auto issue = [&](int64_t bb) {
    trunk::frame_issue<NTB>(obs + (idx ? idx[bb] : bb) * (C0 * H0 * H0), fr);
#pragma unroll
    for (int k = 0; k < B2_PER; k++) {
      const int v = min(int(threadIdx.x) + NTB * k, B2_N - 1);
      const int64_t o = (bb * NP1 + (v >> 1)) * C1 + 8 * (v & 1);
      vh[k] = *reinterpret_cast<const u16x8*>(&dpre1.hi[o]);
      vl[k] = *reinterpret_cast<const u16x8*>(&dpre1.lo[o]);
    }
  };
  x3_ts(ts, TS_C1W, 0);
  if (int64_t(blockIdx.x) < B) issue(blockIdx.x);
  trunk::zero_lds(st, trunk::ST_ELEMS * 2);
  trunk::zero_lds(dp, 4 * DB_B * 2);
  Acc aw[2];
  aw[0] = aw[1] = acc0();
  __syncthreads();

  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    trunk::frame_store_s2d<NTB>(fr, st);
#pragma unroll
    for (int k = 0; k < B2_PER; k++) {
      const int v = threadIdx.x + NTB * k;
      if (v < B2_N) {
        const int p = v >> 1, c0 = 8 * (v & 1), y = p / H1, x = p - y * H1;
        const int o = (y + 1) * ST_W + x;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int e = (c0 + j) * DB_CP + o;
          dp[e] = vh[k][j];
          dp[DB_B + e + 1] = vh[k][j];
          dp[2 * DB_B + e] = vl[k][j];
          dp[3 * DB_B + e + 1] = vl[k][j];
        }
      }
    }
    __syncthreads();
    const int fi = int((b - blockIdx.x) / gridDim.x);
    x3_ts(ts, TS_C1W, 1 + 2 * fi);
    if (b + gridDim.x < B) issue(b + gridDim.x);
    {
      const int cb = wave & 3, a = wave >> 2;
      const unsigned short* sa = st + trunk::st_chan(16 * cb + r) + 8 * g;
      const unsigned short* d0 = dp + r * DB_CP + (1 - a) * ST_W + 8 * g;
#pragma unroll
      for (int s = 0; s < KSTEPS1; s++) {
        const bf16x8 av = ld8(sa + 32 * s);
        mma2a(aw[0], av, ld8(d0 + 32 * s), ld8(d0 + 2 * DB_B + 32 * s));
        mma2a(aw[1], av, ld8(d0 + DB_B + 32 * s), ld8(d0 + 3 * DB_B + 32 * s));
      }
    }
    __syncthreads();
    x3_ts(ts, TS_C1W, 2 + 2 * fi);
  }
  // tile b holds D[m = 4g+e][co = r], channel c = 16cb + m -> ry = cb, rx = g, ci = e; ky = 4a+ry, kx = 4b+rx
  float* out = partial + int64_t(blockIdx.x) * PART1;
#pragma unroll
  for (int bb = 0; bb < 2; bb++) {
    const f32x4 t = total(aw[bb]);
    const int ky = 4 * (wave >> 2) + (wave & 3), kx = 4 * bb + g;
#pragma unroll
    for (int e = 0; e < 4; e++) out[r * 256 + ky * 32 + kx * 4 + e] = t[e] * (1.0f / 255.0f);
  }
  x3_ts(ts, TS_C1W, 15);
}

// ================================================================ K10x reduce
// Sum the two backward launches' per-workgroup partials in a fixed order into fp32 gradients in the
// parameters' memory order (deterministic). Output index e as conv_kernels.hip: [dW1 4096][dW2 8192][db1 16][db2 32].
constexpr int PARTX = C1 * 256 + C2 * 256 + C1 + C2;
// the step counters advance once every workgroup of the launch has read them
__device__ __forceinline__ void x3_tail_bump(const X3Adam& xa) {
  if (xa.bump_next) {  // parity counters: the next step reads the other copy
    if (blockIdx.x == 0 && threadIdx.x == 0)
      for (int k = 0; k < xa.nbump; k++) xa.bump_next[k] = xa.bump[k] + 1;
    return;
  }
  last_block_bump(xa.bump, xa.nbump, xa.done);
}
constexpr int RED_SLICES = 8, RED_BATCH = 16;
__device__ __forceinline__ float* trunk_grad_dst_f32(int e, float* dW1, WStrides w1, float* db1, float* dW2,
                                                     WStrides w2, float* db2) {
  if (e < C1 * 256) {
    const int co = e >> 8, k = e & 255, ky = k >> 5, kx = (k >> 2) & 7, ci = k & 3;
    return &dW1[co * w1.s0 + ci * w1.s1 + ky * w1.s2 + kx * w1.s3];
  }
  if (e < C1 * 256 + C2 * 256) {
    const int f = e - C1 * 256, co = f >> 8, k = f & 255, ky = k >> 6, kx = (k >> 4) & 3, ci = k & 15;
    return &dW2[co * w2.s0 + ci * w2.s1 + ky * w2.s2 + kx * w2.s3];
  }
  if (e < C1 * 256 + C2 * 256 + C1) return &db1[e - C1 * 256 - C2 * 256];
  return &db2[e - C1 * 256 - C2 * 256 - C1];
}
__global__ __launch_bounds__(512) void k_trunk_reduce_x3(const float* __restrict__ part1, int G1,
                                                         const float* __restrict__ part2, int G2, float* dW1,
                                                         WStrides w1, float* db1, float* dW2, WStrides w2, float* db2,
                                                         const X3Adam xa, int nred, uint64_t* __restrict__ ts) {
  __shared__ float red[RED_SLICES][64];
  x3_ts(ts, TS_RED, 0);
  if (int(blockIdx.x) >= nred) {  // Adam workgroups: K6's vector pass over the dense + heads range
    const AdamCoef ac = adam_coef(xa.hp, xa.step_ctr);
    const int64_t o = xa.n_trunk;
    const int64_t tid = int64_t(blockIdx.x - nred) * blockDim.x + threadIdx.x;
    const int64_t nthr = int64_t(gridDim.x - nred) * blockDim.x;
    adam_span<float, true, 2>(xa.master + o, xa.m1 + o, xa.m2 + o, xa.grad + o,
                              static_cast<__hip_bfloat16*>(xa.whi) + o, xa.grad_scale, ac, tid, nthr, xa.n - o,
                              static_cast<__hip_bfloat16*>(xa.wlo) + o, xa.grad2);
    x3_ts(ts, TS_RED, 15);
    x3_tail_bump(xa);
    return;
  }
  const int c = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + c;
  // source: dW1 from the conv1 launch (stride PART1), the rest from the conv2 launch: its layout is
  // [dW2][db2][db1], the output order [dW2][db1][db2]
  const float* src = nullptr;
  int G = 0, stride = 0;
  if (e < C1 * 256) {
    src = part1 + e, G = G1, stride = PART1;
  } else if (e < PARTX) {
    const int f = e - C1 * 256;
    const int o = f < C2 * 256 ? f : (f < C2 * 256 + C1 ? C2 * 256 + C2 + (f - C2 * 256) : C2 * 256 + (f - C2 * 256 - C1));
    src = part2 + o, G = G2, stride = PART2;
  }
  float s = 0.f;
  if (src) {
    for (int g0 = slice; g0 < G; g0 += RED_SLICES * RED_BATCH) {
      float v[RED_BATCH];
#pragma unroll
      for (int j = 0; j < RED_BATCH; j++) v[j] = src[int64_t(min(g0 + RED_SLICES * j, G - 1)) * stride];
#pragma unroll
      for (int j = 0; j < RED_BATCH; j++)
        if (g0 + RED_SLICES * j < G) s += v[j];
    }
  }
  red[slice][c] = s;
  __syncthreads();
  if (slice == 0 && e < PARTX) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < RED_SLICES; k++) t += red[k][c];
    float* dst = trunk_grad_dst_f32(e, dW1, w1, db1, dW2, w2, db2);
    *dst = t;
    if (xa.master) {  // the trunk gradient is final: Adam on it (same math as K6's scalar pass)
      const AdamCoef ac = adam_coef(xa.hp, xa.step_ctr);
      const int64_t i = dst - xa.grad;
      float a = xa.m1[i], b = xa.m2[i];
      const float w = adam_one(xa.master[i], t * xa.grad_scale, a, b, ac);
      xa.m1[i] = a;
      xa.m2[i] = b;
      xa.master[i] = w;
      unsigned short hi, lo;
      split(w, hi, lo);
      static_cast<unsigned short*>(xa.whi)[i] = hi;
      static_cast<unsigned short*>(xa.wlo)[i] = lo;
    }
  }
  x3_ts(ts, TS_RED, 15);
  if (xa.master) x3_tail_bump(xa);
}

// The dense + heads range's Adam as its own launch (no counter advance: the trunk-reduce launch of the same
// step advances the parity counters). The learner forks it onto a side stream right after K12x, so it
// runs beside the trunk backward (conv2 bwd + conv1 wgrad, one workgroup per CU) instead of after it.
__global__ __launch_bounds__(512) void k_dense_adam_x3(const X3Adam xa) {
  const AdamCoef ac = adam_coef(xa.hp, xa.step_ctr);
  const int64_t o = xa.n_trunk;
  const int64_t tid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nthr = int64_t(gridDim.x) * blockDim.x;
  adam_span<float, true, 2>(xa.master + o, xa.m1 + o, xa.m2 + o, xa.grad + o, static_cast<__hip_bfloat16*>(xa.whi) + o,
                            xa.grad_scale, ac, tid, nthr, xa.n - o, static_cast<__hip_bfloat16*>(xa.wlo) + o, xa.grad2);
}

}  // namespace x3

// ---------------------------------------------------------------- host launchers (K10x)
static trunk::WStrides wsx(const int64_t* s) { return trunk::WStrides{s[0], s[1], s[2], s[3]}; }
static x3::CPair cp(const X3In& p) {
  return x3::CPair{static_cast<const unsigned short*>(p.hi), static_cast<const unsigned short*>(p.lo)};
}
static x3::Pair pp(const X3Out& p) { return x3::Pair{static_cast<unsigned short*>(p.hi), static_cast<unsigned short*>(p.lo)}; }

static void check_pair(const X3In& p, const char* what) {
  if ((p.hi == nullptr) != (p.lo == nullptr)) throw std::invalid_argument(std::string(what) + ": hi and lo planes");
}

void x3_probe_set(uint64_t* ts) { x3::g_x3_probe = ts; }

int x3_trunk_fwd_groups(int64_t B) { return int(std::max<int64_t>(1, std::min<int64_t>(B, 256))); }

void x3_trunk_fwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B, X3In W1,
                  const int64_t* w1s, X3In b1, X3In W2, const int64_t* w2s, X3In b2, X3Out h1, X3Out h2,
                  hipStream_t stream, const float* cols, float* cols_out, int ncols) {
  if (B <= 0) return;
  if (period <= 0) period = 1;
  for (const X3In* p : {&W1, &b1, &W2, &b2})
    if (!p->hi || !p->lo) throw std::invalid_argument("x3_trunk_fwd: weights need hi and lo planes");
  if (!h2.hi || !h2.lo || (h1.hi == nullptr) != (h1.lo == nullptr))
    throw std::invalid_argument("x3_trunk_fwd: h2 (and h1) need hi and lo planes");
  if ((cols == nullptr) != (cols_out == nullptr) || (cols_out && (ncols < 1 || ncols > x3::NTF)))
    throw std::invalid_argument("x3_trunk_fwd: cols and cols_out together, 1 <= ncols <= 512");
  hipLaunchKernelGGL(x3::k_trunk_fwd_x3, dim3(uint32_t(x3_trunk_fwd_groups(B))), dim3(x3::NTF), 0, stream, obs, idx,
                     ctr, period, B, cp(W1), wsx(w1s), cp(b1), cp(W2), wsx(w2s), cp(b2), pp(h1), pp(h2), nullptr,
                     nullptr, nullptr, nullptr, nullptr, int64_t(0), nullptr, 1, 0, cols, cols_out, ncols, x3::g_x3_probe);
  RMM_HIP_CHECK(hipGetLastError());
}

void x3_trunk_fwd_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* rows, const int64_t* t_ptr, int64_t B,
                       X3In W1, const int64_t* w1s, X3In b1, X3In W2, const int64_t* w2s, X3In b2, X3Out h2,
                       hipStream_t stream, const int64_t* gate, int64_t gate_want, int* gate_err, int gate_parts,
                       int gate_timeout_ms) {
  if (B <= 0) return;
  if (stack == nullptr || new_frames == nullptr) throw std::invalid_argument("x3_trunk_fwd_push: stack and new frames");
  if (gate_parts < 1 || gate_parts > B) throw std::invalid_argument("x3_trunk_fwd_push: 1 <= gate_parts <= B");
  if (rows != nullptr && t_ptr == nullptr) throw std::invalid_argument("x3_trunk_fwd_push: rows need the row counter");
  if ((reinterpret_cast<uintptr_t>(stack) | reinterpret_cast<uintptr_t>(new_frames) | reinterpret_cast<uintptr_t>(rows)) & 3)
    throw std::invalid_argument("x3_trunk_fwd_push: buffers must be 4-byte aligned");
  for (const X3In* p : {&W1, &b1, &W2, &b2})
    if (!p->hi || !p->lo) throw std::invalid_argument("x3_trunk_fwd_push: weights need hi and lo planes");
  if (!h2.hi || !h2.lo) throw std::invalid_argument("x3_trunk_fwd_push: h2 needs hi and lo planes");
  // push mode: one frame per workgroup (each workgroup shifts its own env's stack)
  hipLaunchKernelGGL(x3::k_trunk_fwd_x3, dim3(uint32_t(B)), dim3(x3::NTF), 0, stream, nullptr, nullptr, nullptr,
                     int64_t(1), B, cp(W1), wsx(w1s), cp(b1), cp(W2), wsx(w2s), cp(b2), x3::Pair{}, pp(h2), stack,
                     new_frames, rows, t_ptr, gate, gate_want, gate_err, gate_parts, gate_timeout_ms, nullptr,
                     nullptr, 0, nullptr);
  RMM_HIP_CHECK(hipGetLastError());
}

// conv2 backward: at most one workgroup per CU, frames spread evenly (B = 500: 250 workgroups x 2 frames,
// the second frame's loads in flight during the first). One frame per workgroup (two per CU) measured 29.9 us
// vs 22.9 us, and it doubles the partials the reduce reads (11.4 vs 10.1 us); 3 frames each: 28.1 us
// (profiles/x3_kernels_r5.txt). conv1's weight gradient: 256 (14.8 us; 128: 22.9, 500: 17.7).
int x3_conv2_bwd_groups(int64_t B) {
  const int64_t per = std::max<int64_t>(1, (B + 255) / 256);
  return int(std::max<int64_t>(1, (B + per - 1) / per));
}
int x3_conv1_wgrad_groups(int64_t B) { return int(std::max<int64_t>(1, std::min<int64_t>(B, 256))); }
int64_t x3_trunk_partial_floats(int64_t B) {
  return int64_t(x3_conv2_bwd_groups(B)) * x3::PART2 + int64_t(x3_conv1_wgrad_groups(B)) * x3::PART1;
}

int x3_dense_adam_groups(const X3Adam& xa) {
  return int(std::max<int64_t>(1, ((xa.n - xa.n_trunk + 3) / 4 + 1023) / 1024));
}

void x3_dense_adam(const X3Adam& xa, hipStream_t stream) {
  if (!xa.master || !xa.m1 || !xa.m2 || !xa.grad || !xa.whi || !xa.wlo || !xa.hp || !xa.step_ctr || xa.n <= xa.n_trunk ||
      xa.n_trunk % 4 != 0)
    throw std::invalid_argument("x3_dense_adam: flat buffers, both weight planes, hp and the step counter");
  hipLaunchKernelGGL(x3::k_dense_adam_x3, dim3(uint32_t(x3_dense_adam_groups(xa))), dim3(512), 0, stream, xa);
  RMM_HIP_CHECK(hipGetLastError());
}

void x3_trunk_bwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B, X3In W2,
                  const int64_t* w2s, X3In h1, const void* h2hi, X3In dh2, X3Out dpre1, float* partial, float* dW1,
                  const int64_t* w1s, float* db1, float* dW2, float* db2, hipStream_t stream, const X3Adam& xa,
                  bool dense_separate) {
  if (B <= 0) return;
  if (dense_separate && (!xa.master || !xa.bump_next))
    throw std::invalid_argument("x3_trunk_bwd: a separate dense Adam needs the tail Adam with parity counters");
  if (xa.master) {
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool ok = al(xa.master) && al(xa.m1) && al(xa.m2) && al(xa.grad) && xa.whi && xa.wlo &&
                    (reinterpret_cast<uintptr_t>(xa.whi) & 7) == 0 && (reinterpret_cast<uintptr_t>(xa.wlo) & 7) == 0 &&
                    xa.n_trunk % 4 == 0 && xa.n_trunk >= x3::PARTX && xa.n > xa.n_trunk && xa.hp && xa.step_ctr &&
                    xa.bump && xa.nbump > 0 && (xa.bump_next || xa.done) && dW1 >= xa.grad &&
                    db2 < xa.grad + xa.n_trunk;
    if (!ok)
      throw std::invalid_argument("x3_trunk_bwd: Adam tail needs aligned flat buffers (trunk range first, "
                                  "n_trunk % 4 == 0), both weight planes, hp, the step counters and a bump target");
  }
  if (period <= 0) period = 1;
  for (const X3In* p : {&W2, &h1, &dh2})
    if (!p->hi || !p->lo) throw std::invalid_argument("x3_trunk_bwd: W2 / h1 / dh2 need hi and lo planes");
  if (!dpre1.hi || !dpre1.lo || !h2hi || !partial) throw std::invalid_argument("x3_trunk_bwd: dpre1 / h2 / partial");
  const int G2 = x3_conv2_bwd_groups(B), G1 = x3_conv1_wgrad_groups(B);
  float* p2 = partial;                              // conv2 launch partials [G2][PART2]
  float* p1 = partial + int64_t(G2) * x3::PART2;    // conv1 launch partials [G1][PART1]
  hipLaunchKernelGGL(x3::k_conv2_bwd_x3, dim3(uint32_t(G2)), dim3(x3::NTB), 0, stream, B, cp(W2), wsx(w2s), cp(h1),
                     static_cast<const unsigned short*>(h2hi), cp(dh2), pp(dpre1), p2, 0, x3::g_x3_probe);
  RMM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(x3::k_conv1_wgrad_x3, dim3(uint32_t(G1)), dim3(x3::NTB), 0, stream, obs, idx, ctr, period, B,
                     x3::CPair{static_cast<const unsigned short*>(dpre1.hi), static_cast<const unsigned short*>(dpre1.lo)},
                     p1, x3::g_x3_probe);
  RMM_HIP_CHECK(hipGetLastError());
  const int nred = (x3::PARTX + 63) / 64;
  // Adam workgroups: two groups of 4 elements per lane (K6's default unroll)
  const int nadam = xa.master && !dense_separate ? x3_dense_adam_groups(xa) : 0;
  hipLaunchKernelGGL(x3::k_trunk_reduce_x3, dim3(nred + nadam), dim3(512), 0, stream, p1, G1, p2, G2, dW1, wsx(w1s),
                     db1, dW2, wsx(w2s), db2, xa, nred, x3::g_x3_probe);
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm

// ================================================================ dense tail (K13x, K15x, K12x, K16x)
namespace rmm {
namespace hip {
namespace x3 {

constexpr int H = dense::H;

// ---- K13x: split-K dense layer hidden_pre = x Wᵀ over split pairs -> fp32 partials part[S][M][N]
// (no bias / ReLU: the consumer K15x / K16x sums the S slices, adds the bias, applies ReLU in fp32).
// Unit = FM x FN 16x16 fragments per wave, the workgroup's 4 waves split the slice's k-steps and
// combine through LDS in a fixed order (deterministic). Each wave has only ~8 k-steps at ~2 waves per
// SIMD, so a step's loads are issued D steps ahead (a register ring of D stages): the MFMAs of step i
// overlap the global latency of steps i+1..i+D-1 instead of waiting for it.
template <int FM, int FN, int D>
__device__ __forceinline__ void dense_part_tile_x3(CPair x, CPair w, int64_t M, int64_t K, int N, int S,
                                                   float* __restrict__ part, f32x4 (&red)[3][FM * FN][64],
                                                   int64_t* tm_out) {
  // the wave index is wave-uniform: in an SGPR the k-step guards below are scalar branches
  const int lane = threadIdx.x & 63, kw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 15,
            g = lane >> 4;
  const int nt = N / (16 * FN);
  const int64_t mt = (M + 16 * FM - 1) / (16 * FM);
  const int64_t tiles = mt * nt, total_ = gridDim.x;
  int64_t id = blockIdx.x;
  if ((total_ & 7) == 0) id = (id & 7) * (total_ >> 3) + (id >> 3);  // XCD-contiguous runs
  const int64_t sl = id / tiles, rem = id % tiles, tm = rem / nt, tn = rem % nt;
  *tm_out = tm;
  const int64_t m0 = tm * 16 * FM, n0 = tn * 16 * FN;
  const int64_t steps = K / 32, lo = steps * sl / S, hi = steps * (sl + 1) / S;
  const unsigned short *xh[FM], *xl[FM], *wh[FN], *wl[FN];
#pragma unroll
  for (int i = 0; i < FM; i++) {
    const int64_t o = min(m0 + 16 * i + r, M - 1) * K + 8 * g + (lo + kw) * 32;
    xh[i] = x.hi + o, xl[i] = x.lo + o;
  }
#pragma unroll
  for (int j = 0; j < FN; j++) {
    const int64_t o = (n0 + 16 * j + r) * K + 8 * g + (lo + kw) * 32;
    wh[j] = w.hi + o, wl[j] = w.lo + o;
  }
  // this wave's k-steps: lo + kw + 4 t, t < n (step t is 128 t elements past the pointers above)
  const int n = lo + kw < hi ? int((hi - lo - kw + 3) / 4) : 0;
  Acc acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++) acc[i][j] = acc0();
  bf16x8 ah[D][FM], al[D][FM], bh[D][FN], bl[D][FN];
#define K13X_LOAD(slot, t)                                                                      \
  {                                                                                             \
    const int64_t e_ = int64_t(t) * 128;                                                        \
    _Pragma("unroll") for (int i = 0; i < FM; i++) ah[slot][i] = ld8(xh[i] + e_), al[slot][i] = ld8(xl[i] + e_); \
    _Pragma("unroll") for (int j = 0; j < FN; j++) bh[slot][j] = ld8(wh[j] + e_), bl[slot][j] = ld8(wl[j] + e_); \
  }
#define K13X_MMA(slot)                                                                          \
  _Pragma("unroll") for (int i = 0; i < FM; i++) _Pragma("unroll") for (int j = 0; j < FN; j++)  \
      mma3(acc[i][j], ah[slot][i], al[slot][i], bh[slot][j], bl[slot][j]);
  if (n > 0) {
    // prologue: steps 0..D-1 (clamped: a repeated last step is loaded but never multiplied)
#pragma unroll
    for (int d = 0; d < D; d++) K13X_LOAD(d, min(d, n - 1));
    int t0 = 0;
    // steady state, no guards: every slot is multiplied and refilled D steps ahead
    for (; t0 + 2 * D <= n; t0 += D) {
#pragma unroll
      for (int d = 0; d < D; d++) {
        K13X_MMA(d);
        K13X_LOAD(d, t0 + d + D);
      }
    }
    // tail: steps t0 .. n-1 (fewer than 2D)
#pragma unroll
    for (int d = 0; d < D; d++) {
      if (t0 + d < n) {
        K13X_MMA(d);
        if (t0 + d + D < n) K13X_LOAD(d, t0 + d + D);
      }
    }
#pragma unroll
    for (int d = 0; d < D; d++)
      if (t0 + D + d < n) K13X_MMA(d);
  }
#undef K13X_MMA
#undef K13X_LOAD
  if (kw > 0) {
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
      for (int j = 0; j < FN; j++) red[kw - 1][i * FN + j][lane] = total(acc[i][j]);
  }
  __syncthreads();
  if (kw != 0) return;
  float* out = part + (sl * M) * N + n0 + r;
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++) {
      const f32x4 t = ((total(acc[i][j]) + red[0][i * FN + j][lane]) + red[1][i * FN + j][lane]) + red[2][i * FN + j][lane];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int64_t row = m0 + 16 * i + 4 * g + e;
        if (row < M) out[row * N + 16 * j] = t[e];
      }
    }
}
template <int FM, int FN, int D>
__global__ __launch_bounds__(256) void k_dense_fwd_part_x3(CPair x, CPair w, int64_t M, int64_t K, int N, int S,
                                                           float* __restrict__ part) {
  __shared__ f32x4 red[3][FM * FN][64];
  int64_t tm;
  dense_part_tile_x3<FM, FN, D>(x, w, M, K, N, S, part, red, &tm);
}

// ---- K13x-L: the same product for the SGD step's M = 500 rows, staged through LDS. The register-direct
// K13x above is L1-bound there (each 16-B fragment load touches 16 rows x 64 B, and no two waves share an
// operand: TA stalled by TCP ~45% of the time, profiles/x3_kernels_r5.txt). Here a workgroup owns a
// 64 x 64 output tile of one K slice; per stage (2 k-steps = 128 B of every row) it loads the A and B
// tiles of both planes with full-line coalesced 16-B loads (registers for stage s+1 in flight while
// stage s multiplies), stores them into padded LDS rows (144-B pitch: the 16-row fragment reads are
// bank-conflict free) and its 4 waves (2 x 2, 32 x 32 each) read their fragments from there: 4x less
// L1 traffic per MFMA and no half-line requests.
constexpr int KL_T = 64, KL_PITCH = 72, KL_PLANE = KL_T * KL_PITCH;  // elements
constexpr int KL_STAGE = 4 * KL_PLANE;  // A hi, A lo, B hi, B lo
constexpr int KL_D = 4;                 // register-ring depth (stages of global loads in flight)
__global__ __launch_bounds__(256) void k_dense_fwd_lds_x3(CPair x, CPair w, int64_t M, int64_t K, int N, int S,
                                                          float* __restrict__ part, uint64_t* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) unsigned short t[2 * KL_STAGE];
  x3_ts(ts, TS_K13L, 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4, wm = wave >> 1, wn = wave & 1;
  const int nt = N / KL_T;
  const int64_t mt = (M + KL_T - 1) / KL_T, tiles = mt * nt, total_ = gridDim.x;
  int64_t id = blockIdx.x;
  if ((total_ & 7) == 0) id = (id & 7) * (total_ >> 3) + (id >> 3);  // XCD-contiguous runs
  const int64_t sl = id / tiles, rem = id % tiles, tm = rem / nt, tn = rem % nt;
  const int64_t m0 = tm * KL_T, n0 = tn * KL_T;
  const int64_t steps = K / 32, lo = steps * sl / S, hi = steps * (sl + 1) / S;
  const int nst = int((hi - lo + 1) / 2);  // stages of 2 k-steps (the last may hold one)
  // loader: 8 x 16 B per thread per stage = {A, B} x {hi, lo} x 2 row halves; thread -> (row, 16-B segment)
  const int lrow = tid >> 3, lseg = tid & 7;  // rows lrow and lrow + 32
  const unsigned short* src[8];
  int64_t kend = hi * 32;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int64_t ar = min(m0 + lrow + 32 * h, M - 1), br = n0 + lrow + 32 * h;
    src[0 + h] = x.hi + ar * K + lo * 32 + lseg * 8;
    src[2 + h] = x.lo + ar * K + lo * 32 + lseg * 8;
    src[4 + h] = w.hi + br * K + lo * 32 + lseg * 8;
    src[6 + h] = w.lo + br * K + lo * 32 + lseg * 8;
  }
  const int64_t kseg = lo * 32 + lseg * 8;  // this thread's k within the stage (+ 64 per stage)
  // register ring: stage st lives in slot st % KL_D from its issue until it is stashed into LDS one stage
  // ahead of its use, so KL_D - 1 stages of global loads are in flight behind the MFMAs
  u16x8 v[KL_D][8];
  bool okv[KL_D];
  // loads are unconditional, from an address clamped into the slice (never past a row / the buffer); a
  // segment past the slice end (the odd last step's second half) is zeroed when it is stashed, so no
  // load result is consumed before its stash and the loads stay in flight
#define KL_ISSUE(slot, st_)                                                                             \
  {                                                                                                     \
    const int64_t k_ = kseg + int64_t(st_) * 64;                                                        \
    okv[slot] = k_ < kend;                                                                              \
    const int64_t o_ = (okv[slot] ? k_ : kend - 8) - kseg;                                              \
    _Pragma("unroll") for (int q = 0; q < 8; q++) v[slot][q] = *reinterpret_cast<const u16x8*>(src[q] + o_); \
  }
#define KL_STASH(slot, buf_)                                                                            \
  {                                                                                                     \
    unsigned short* b_ = t + (buf_) * KL_STAGE;                                                         \
    _Pragma("unroll") for (int q = 0; q < 8; q++)                                                       \
        *reinterpret_cast<u16x8*>(b_ + (q >> 1) * KL_PLANE + (lrow + 32 * (q & 1)) * KL_PITCH + lseg * 8) = \
            okv[slot] ? v[slot][q] : u16x8{0, 0, 0, 0, 0, 0, 0, 0};                                     \
  }
  Acc acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++) acc[i][0] = acc[i][1] = acc0();
#define KL_MMA(st_)                                                                                     \
  {                                                                                                     \
    const unsigned short* b = t + ((st_) & 1) * KL_STAGE;                                               \
    _Pragma("unroll") for (int kk = 0; kk < 2; kk++) {                                                  \
      bf16x8 ah[2], al[2], bh[2], bl[2];                                                                \
      _Pragma("unroll") for (int i = 0; i < 2; i++) {                                                   \
        const int ao = (wm * 32 + 16 * i + r) * KL_PITCH + kk * 32 + 8 * g;                             \
        ah[i] = ld8(b + ao), al[i] = ld8(b + KL_PLANE + ao);                                            \
        const int bo = (wn * 32 + 16 * i + r) * KL_PITCH + kk * 32 + 8 * g;                             \
        bh[i] = ld8(b + 2 * KL_PLANE + bo), bl[i] = ld8(b + 3 * KL_PLANE + bo);                         \
      }                                                                                                 \
      _Pragma("unroll") for (int i = 0; i < 2; i++) _Pragma("unroll") for (int j = 0; j < 2; j++)       \
          mma3(acc[i][j], ah[i], al[i], bh[j], bl[j]);                                                  \
    }                                                                                                   \
  }
  if (nst > 0) {
    // stage indices are clamped to the last stage: loads and stashes stay unconditional (a clamped
    // repeat is never multiplied), so the compiler can count the loads in flight instead of draining them
    const int last = nst - 1;
#pragma unroll
    for (int d = 0; d < KL_D; d++) KL_ISSUE(d, min(d, last));
    KL_STASH(0, 0);
    KL_ISSUE(0, min(KL_D, last));
    __syncthreads();
    int st0 = 0;
    for (; st0 + KL_D <= nst; st0 += KL_D) {  // steady state: KL_D stages, no guards
#pragma unroll
      for (int d = 0; d < KL_D; d++) {
        const int st = st0 + d;
        KL_MMA(st);
        KL_STASH((d + 1) % KL_D, (st + 1) & 1);              // stage st+1 (a clamped repeat past the end)
        KL_ISSUE((d + 1) % KL_D, min(st + 1 + KL_D, last));  // its slot takes stage st+1+KL_D
        __syncthreads();
      }
    }
#pragma unroll
    for (int d = 0; d < KL_D - 1; d++) {  // tail: fewer than KL_D stages, all already loaded
      const int st = st0 + d;
      if (st < nst) {
        KL_MMA(st);
        if (st + 1 < nst) KL_STASH((d + 1) % KL_D, (st + 1) & 1);
        __syncthreads();
      }
    }
  }
#undef KL_MMA
#undef KL_ISSUE
#undef KL_STASH
  float* out = part + (sl * M) * N + n0 + wn * 32 + r;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const f32x4 tt = total(acc[i][j]);
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int64_t row = m0 + wm * 32 + 16 * i + 4 * g + e;
        if (row < M) out[row * N + 16 * j] = tt[e];
      }
    }
  x3_ts(ts, TS_K13L, 15);
}

// consumer prologue: a lane's 4 hidden values of row rr = ReLU(Σ_s part[s] + b) in fp32 (slice order).
// The slices' loads are issued in batches of 8 before any is waited for: a runtime-bounded loop of
// load -> add compiled to one load and one `s_waitcnt vmcnt(0)` per slice, i.e. S serial round trips to
// the partials (written by another launch, so L2 misses) — most of K15x's / K16x's time.
constexpr int HID_BATCH = 8;
__device__ __forceinline__ void load_hidden4_x3(const float* __restrict__ hpart, int S, CPair hb, int64_t M,
                                                int64_t rr, int lane, float (&hv)[4]) {
  unsigned short bh4[4], bl4[4];  // bias pair first: in flight with the slices
#pragma unroll
  for (int k = 0; k < 4; k++) bh4[k] = hb.hi[4 * lane + k], bl4[k] = hb.lo[4 * lane + k];
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* p = hpart + rr * H + 4 * lane;
  for (int s0 = 0; s0 < S; s0 += HID_BATCH) {
    float4 v[HID_BATCH];
#pragma unroll
    for (int j = 0; j < HID_BATCH; j++)  // clamped: every load is valid, only the first S - s0 are summed
      v[j] = *reinterpret_cast<const float4*>(p + int64_t(min(s0 + j, S - 1)) * M * H);
#pragma unroll
    for (int j = 0; j < HID_BATCH; j++)
      if (s0 + j < S) a.x += v[j].x, a.y += v[j].y, a.z += v[j].z, a.w += v[j].w;
  }
  hv[0] = fmaxf(a.x + join(bh4[0], bl4[0]), 0.f);
  hv[1] = fmaxf(a.y + join(bh4[1], bl4[1]), 0.f);
  hv[2] = fmaxf(a.z + join(bh4[2], bl4[2]), 0.f);
  hv[3] = fmaxf(a.w + join(bh4[3], bl4[3]), 0.f);
}

// the heads' split weights joined into fp32 LDS images (whs [A1][H], bhs [A1]) by a workgroup of exactly NT
// threads, in two halves: issue() puts every global load in flight (the kernels issue it before their other
// loads), store() joins them into LDS. The strided loop it replaces waited for each pass in turn.
template <int A1, int NT>
struct HeadsStage {
  static constexpr int PER = (A1 * H + NT - 1) / NT;
  unsigned short vh[PER], vl[PER], bhh = 0, bhl = 0;
  __device__ __forceinline__ void issue(CPair wh, CPair bh) {
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int e = min(int(threadIdx.x) + NT * k, A1 * H - 1);
      vh[k] = wh.hi[e];
      vl[k] = wh.lo[e];
    }
    const int eb = min(int(threadIdx.x), A1 - 1);  // unconditional (clamped): a guarded load is waited for at once
    bhh = bh.hi[eb], bhl = bh.lo[eb];
  }
  __device__ __forceinline__ void store(float* whs, float* bhs) const {
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int e = int(threadIdx.x) + NT * k;
      if (e < A1 * H) whs[e] = join(vh[k], vl[k]);
    }
    if (threadIdx.x < A1) bhs[threadIdx.x] = join(bhh, bhl);
  }
};

// ---- K15x: heads + PPO loss statistics + dheads + dpre, one wave per row, all fp32 math
// (dense_kernels.hip K15 with fp32 heads / gradients). Outputs as split pairs: dz [M, A1], dpre [M, 256]
// and the hidden row hid [M, 256] (K12x reads them).
template <int A1>
__global__ __launch_bounds__(256) void k_heads_ppo_x3(const float* __restrict__ hpart, int S, CPair hb, CPair wh,
                                                      CPair bh, const float* __restrict__ cols,
                                                      const float* __restrict__ coef, float* __restrict__ acc,
                                                      const float* __restrict__ gout, int64_t M, Pair dz, Pair dpre,
                                                      Pair hid, const int64_t* __restrict__ cidx,
                                                      const int64_t* __restrict__ ctr, int64_t period, int acc_slab,
                                                      uint64_t* __restrict__ ts) {
  constexpr int A = A1 - 1;
  x3_ts(ts, TS_K15, 0);
  // slab mode: this workgroup's running sums, loaded now (in flight with everything else), rewritten at the end
  float* srow = acc + int64_t(blockIdx.x) * 8;
  const float sold = (acc && acc_slab && threadIdx.x < 6) ? srow[threadIdx.x] : 0.f;
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  __shared__ float red[6][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = int64_t(blockIdx.x) * (blockDim.x >> 6) + wave;
  const bool valid = row < M;
  const int64_t rr = valid ? row : M - 1;
  const int64_t crr = cidx ? (ctr ? cidx[(ctr[0] % period) * M + rr] : cidx[rr]) : rr;
  const float* crow = cols + crr * (A + 4);
  float cv[A + 4];
#pragma unroll
  for (int j = 0; j < A + 4; j++) cv[j] = crow[j];
  HeadsStage<A1, 256> hs;  // launched with 256 threads; its loads in flight with the row's
  hs.issue(wh, bh);
  float hv[4];
  load_hidden4_x3(hpart, S, hb, M, rr, lane, hv);
  hs.store(whs, bhs);
  __syncthreads();
  const float gs = gout[0] / float(M);
  if (valid) store4(hid, row * H + 4 * lane, hv);
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
  for (int a = 0; a < A1; a++) hd[a] += bhs[a];
  float s[6], g[A1];
  dense::ppo_loss_row<A1, false>(hd, cv, coef[0], coef[1], coef[2], coef[3], coef[4], gs, valid && lane == 0, s, g);
  if (valid) {
    if (lane < A1) {
      float gl = g[0];
#pragma unroll
      for (int j = 1; j < A1; j++)
        if (lane == j) gl = g[j];
      store1(dz, row * A1 + lane, gl);
    }
    float dp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < A1; a++) {
      const float4 w = *reinterpret_cast<const float4*>(&whs[a * H + 4 * lane]);
      dp[0] += g[a] * w.x, dp[1] += g[a] * w.y, dp[2] += g[a] * w.z, dp[3] += g[a] * w.w;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) dp[k] = hv[k] > 0.f ? dp[k] : 0.f;
    store4(dpre, row * H + 4 * lane, dp);
  }
  if (lane == 0)
    for (int k = 0; k < 6; k++) red[k][wave] = s[k];
  __syncthreads();
  if (acc && threadIdx.x < 6) {
    float t = 0.f;
    for (int k = 0; k < int(blockDim.x >> 6); k++) t += red[threadIdx.x][k];
    // 125 workgroups' atomics on the same 6 words serialise at the device-coherent atomic unit (~1.3 us of
    // the launch at M = 500); the slab gives each workgroup its own row
    if (acc_slab)
      srow[threadIdx.x] = sold + t;
    else
      atomicAdd(&acc[threadIdx.x], t);
  }
  x3_ts(ts, TS_K15, 15);
}

// ---- K16x: heads + Gumbel-max sampling + rollout-row stores (+ step advance), fp32 head row
template <int A1>
__global__ __launch_bounds__(256) void k_heads_sample_x3(const float* __restrict__ hpart, int S, CPair hb, CPair wh,
                                                         CPair bh, const int64_t* t_ptr, const int64_t* ctr,
                                                         uint32_t seed, int64_t* __restrict__ act,
                                                         float* __restrict__ logp, float* __restrict__ vf,
                                                         float* __restrict__ lout, int64_t* __restrict__ act_now,
                                                         int64_t B, unsigned int* __restrict__ done, int64_t* host_seq) {
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  const int lane = threadIdx.x & 63;
  const int64_t b = int64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  HeadsStage<A1, 256> hs;  // launched with 256 threads
  hs.issue(wh, bh);
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  float hv[4] = {0.f, 0.f, 0.f, 0.f};
  if (b < B) load_hidden4_x3(hpart, S, hb, B, b, lane, hv);
  hs.store(whs, bhs);
  __syncthreads();
  if (b < B) dense::heads_sample_row_pre<A1, false>(hv, whs, bhs, t, c, seed, act, logp, vf, lout, act_now, B, b, lane);
  if (done) {
    __shared__ unsigned int last;
    if (host_seq) __threadfence_system();
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
      if (host_seq) __hip_atomic_store(host_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
// ---- K13x + K16x in ONE launch (rollout step, M <= 16 * 63 rows): every workgroup computes its split-K
// partial tile exactly as K13x (FM = FN = 1, D = 4) and takes a ticket on its 16-row tile; the workgroup
// that completes a row tile (the last of its N/16 x S contributors) sums the partials, adds bias + ReLU
// and runs K16x's heads + Gumbel-max sampling for those 16 rows (one wave per 4 rows); the last row tile's
// finisher advances the step counters and publishes the host word. The kernel boundary between K13x and
// K16x (their launch gap and K16x's fill) is gone; the sums and the sampling are bit-identical.
// tickets: done[0] = row tiles finished this step, done[1 + tm] = contributors of row tile tm (reset by
// the tile's finisher, so every counter is 0 again when the launch ends).
template <int A1>
__global__ __launch_bounds__(256) void k_dense_heads_sample_x3(CPair x, CPair w, int64_t M, int64_t K, int S,
                                                               float* __restrict__ part, CPair hb, CPair wh, CPair bh,
                                                               const int64_t* t_ptr, const int64_t* ctr, uint32_t seed,
                                                               int64_t* __restrict__ act, float* __restrict__ logp,
                                                               float* __restrict__ vf, float* __restrict__ lout,
                                                               int64_t* __restrict__ act_now,
                                                               unsigned int* __restrict__ done, int64_t* host_seq) {
  __shared__ f32x4 red[3][1][64];
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  __shared__ unsigned int s_last;
  int64_t tm;
  dense_part_tile_x3<1, 1, 4>(x, w, M, K, H, S, part, red, &tm);
  const unsigned int contributors = unsigned(H / 16) * unsigned(S);
  __threadfence();  // this workgroup's partial tile before its ticket
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&done[1 + tm], 1u) == contributors - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();  // every contributor's partial tile of row tile tm
  {
    HeadsStage<A1, 256> hs;
    hs.issue(wh, bh);
    hs.store(whs, bhs);
  }
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int64_t b = 16 * tm + wv + 4 * q;
    if (b < M) {
      float hv[4];
      load_hidden4_x3(part, S, hb, M, b, lane, hv);
      dense::heads_sample_row_pre<A1, false>(hv, whs, bhs, t, c, seed, act, logp, vf, lout, act_now, M, b, lane);
    }
  }
  if (host_seq) __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    done[1 + tm] = 0u;
    __threadfence();
    const unsigned int ntm = unsigned((M + 15) / 16);
    if (atomicAdd(done, 1u) == ntm - 1) {
      int64_t* tw = const_cast<int64_t*>(t_ptr);
      int64_t* cw = const_cast<int64_t*>(ctr);
      *tw += 1;
      if (cw != tw) *cw += 1;
      atomicExch(done, 0u);
      if (host_seq) __hip_atomic_store(host_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
// single-workgroup K16x (B <= 16 R rows) with the step advance after a workgroup barrier (as k_heads_sample1)
template <int A1, int R>
__global__ __launch_bounds__(1024) void k_heads_sample1_x3(const float* __restrict__ hpart, int S, CPair hb, CPair wh,
                                                           CPair bh, int64_t* t_ptr, int64_t* ctr, uint32_t seed,
                                                           int64_t* __restrict__ act, float* __restrict__ logp,
                                                           float* __restrict__ vf, float* __restrict__ lout,
                                                           int64_t* __restrict__ act_now, int64_t B, int64_t* host_seq) {
  __shared__ __attribute__((aligned(16))) float whs[A1 * H];
  __shared__ float bhs[A1];
  constexpr int kWaves = 16;
  const int lane = threadIdx.x & 63;
  const int64_t b0 = threadIdx.x >> 6;
  HeadsStage<A1, 1024> hs;  // launched with 1024 threads
  hs.issue(wh, bh);
  const int64_t t = *t_ptr;
  const uint32_t c = uint32_t(*ctr);
  float hv[R][4];
#pragma unroll
  for (int q = 0; q < R; q++)
    if (b0 + q * kWaves < B) load_hidden4_x3(hpart, S, hb, B, b0 + q * kWaves, lane, hv[q]);
  hs.store(whs, bhs);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < R; q++)
    if (b0 + q * kWaves < B)
      dense::heads_sample_row_pre<A1, false>(hv[q], whs, bhs, t, c, seed, act, logp, vf, lout, act_now, B,
                                             b0 + q * kWaves, lane);
  if (host_seq) __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    *t_ptr = t + 1;
    if (ctr != t_ptr) *ctr = int64_t(c) + 1;
    if (host_seq) __hip_atomic_store(host_seq, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- K12x: backward of hidden = ReLU(x Wᵀ + b), heads = hidden Whᵀ + bh over split pairs.
// Column-block role (workgroup j < K/32): dx[:, J] (split pair, for the trunk backward) and
// dW[:, J] (fp32) for J = [32j, 32j+32); head role (workgroup K/32): dWh, db, dbh (fp32).
// 64-row chunks, each staged once into LDS (hi and lo planes); the next chunk's global loads are in
// registers while the current chunk's MFMAs run; two barriers per chunk.
constexpr int MC = 64, JB = 32, NT = 512;
constexpr int DMP = H + 16;  // row pitch of the [m][h] images (transposed reads conflict-free)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__device__ __forceinline__ bf16x8 tr8(const unsigned short* p0, const unsigned short* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}
constexpr int IMG = MC * DMP;                      // one plane of a 64-row [m][h] chunk image
constexpr int K12X_COLS = 2 * IMG + 2 * 2 * MC * 16 + 2 * 2 * H * 16;
constexpr int HQ = 64, HQP = HQ + 16;              // head role: h-columns per workgroup, image pitch
constexpr int K12X_HEAD = 4 * MC * HQP + 2 * MC * 16;
constexpr int K12X_LDS = K12X_COLS > K12X_HEAD ? K12X_COLS : K12X_HEAD;
static_assert(K12X_LDS * 2 <= 160 * 1024, "K12x LDS");

__device__ __forceinline__ void k12x_cols(CPair x, CPair w, CPair dpre, int64_t M, int64_t K, int64_t J0, Pair dx,
                                          float* __restrict__ dw, unsigned short* lds, int c0, int c1) {
  unsigned short* dm = lds;                       // [plane][m][DMP]
  unsigned short* xs = lds + 2 * IMG;             // [plane][jt][m][16]
  unsigned short* ws = xs + 2 * 2 * MC * 16;      // [plane][jt][h][16]  (setup)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int q = r >> 2, p = r & 3;
  const int64_t Mend = min(M, int64_t(c1) * MC);  // rows [c0 MC, Mend): this workgroup's row part
  // two register stages: chunk c + 2's loads are issued while chunk c computes. Loads are unconditional
  // from clamped rows, masked at the LDS store, so the compiler's vmcnt counting never drains a stage
  uint4 sdh[2][4], sdl[2][4], sxh[2], sxl[2];
  auto load = [&](int st, int c) {
    const int64_t m0 = int64_t(c) * MC;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      const int64_t o = min(m0 + row, M - 1) * H + 8 * pc;
      sdh[st][k] = *reinterpret_cast<const uint4*>(&dpre.hi[o]);
      sdl[st][k] = *reinterpret_cast<const uint4*>(&dpre.lo[o]);
    }
    const int row = (tid >> 2) & (MC - 1), pc = tid & 3;
    const int64_t o = min(m0 + row, M - 1) * K + J0 + 8 * pc;
    sxh[st] = *reinterpret_cast<const uint4*>(&x.hi[o]);
    sxl[st] = *reinterpret_cast<const uint4*>(&x.lo[o]);
  };
  auto store = [&](int st, int c) {
    const int64_t m0 = int64_t(c) * MC;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int v = tid + NT * k, row = v >> 5, pc = v & 31;
      const bool ok = m0 + row < Mend;
      *reinterpret_cast<uint4*>(&dm[row * DMP + 8 * pc]) = keep_if(ok, sdh[st][k]);
      *reinterpret_cast<uint4*>(&dm[IMG + row * DMP + 8 * pc]) = keep_if(ok, sdl[st][k]);
    }
    if (tid < MC * 4) {
      const int row = tid >> 2, pc = tid & 3;
      const bool ok = m0 + row < Mend;
      const int o = ((pc >> 1) * MC + row) * 16 + 8 * (pc & 1);
      *reinterpret_cast<uint4*>(&xs[o]) = keep_if(ok, sxh[st]);
      *reinterpret_cast<uint4*>(&xs[2 * MC * 16 + o]) = keep_if(ok, sxl[st]);
    }
  };
  {  // W[:, J] -> ws planes, then the Wᵀ fragments into registers
    uint4 wvh[2], wvl[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int v = tid + NT * k, h = v >> 2, pc = v & 3;
      wvh[k] = *reinterpret_cast<const uint4*>(&w.hi[int64_t(h) * K + J0 + 8 * pc]);
      wvl[k] = *reinterpret_cast<const uint4*>(&w.lo[int64_t(h) * K + J0 + 8 * pc]);
    }
    load(0, c0);
    load(1, min(c0 + 1, c1 - 1));
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int v = tid + NT * k, h = v >> 2, pc = v & 3;
      const int o = ((pc >> 1) * H + h) * 16 + 8 * (pc & 1);
      *reinterpret_cast<uint4*>(&ws[o]) = wvh[k];
      *reinterpret_cast<uint4*>(&ws[2 * H * 16 + o]) = wvl[k];
    }
  }
  __syncthreads();
  const int mt = wave >> 1, nt = wave & 1;
  // Wᵀ fragments are re-read from the resident ws planes per chunk: holding them in registers (64 VGPRs)
  // with two load stages in flight spilled
  Acc adw[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++) adw[i][0] = adw[i][1] = acc0();

  auto chunk = [&](int st, int c) {
    store(st, c);
    __syncthreads();
    load(st, min(c + 2, c1 - 1));  // in flight during this and the next chunk's MFMAs
    {  // dxᵀ tile: D[j][m] = Σ_h Wᵀ[j][h] dpre[m][h]
      Acc a = acc0();
      const int ro = (16 * mt + r) * DMP + 8 * g;
#pragma unroll
      for (int s = 0; s < H / 32; s++) {
        const unsigned short* p0 = &ws[(nt * H + 32 * s + 8 * g + q) * 16 + 4 * p];
        mma3(a, tr8(p0, p0 + 4 * 16), tr8(p0 + 2 * H * 16, p0 + 2 * H * 16 + 4 * 16), ld8(&dm[ro + 32 * s]),
             ld8(&dm[IMG + ro + 32 * s]));
      }
      const int64_t row = int64_t(c) * MC + 16 * mt + r;
      if (row < Mend) {
        const f32x4 t = total(a);
        const float v[4] = {t[0], t[1], t[2], t[3]};
        store4(dx, row * K + J0 + 16 * nt + 4 * g, v);
      }
    }
    // dW[h][j] += Σ_m dpre[m][h] x[m][j] (both operands by transposed reads)
#pragma unroll
    for (int ks = 0; ks < MC / 32; ks++) {
      bf16x8 bxh[2], bxl[2];
#pragma unroll
      for (int jt = 0; jt < 2; jt++) {
        const unsigned short* p0 = &xs[(jt * MC + 32 * ks + 4 * g + q) * 16 + 4 * p];
        bxh[jt] = tr8(p0, p0 + 16 * 16);
        bxl[jt] = tr8(p0 + 2 * MC * 16, p0 + 2 * MC * 16 + 16 * 16);
      }
#pragma unroll
      for (int hi = 0; hi < 2; hi++) {
        const unsigned short* p0 = &dm[(32 * ks + 4 * g + q) * DMP + 16 * (wave + 8 * hi) + 4 * p];
        const bf16x8 adh = tr8(p0, p0 + 16 * DMP), adl = tr8(p0 + IMG, p0 + IMG + 16 * DMP);
        mma3(adw[hi][0], adh, adl, bxh[0], bxl[0]);
        mma3(adw[hi][1], adh, adl, bxh[1], bxl[1]);
      }
    }
    __syncthreads();  // chunk images free
  };
  for (int c = c0; c < c1; c += 2) {  // pairs of chunks; an odd count runs one all-zero chunk past the end
    chunk(0, c);
    chunk(1, c + 1);
  }
#pragma unroll
  for (int hi = 0; hi < 2; hi++)
#pragma unroll
    for (int jt = 0; jt < 2; jt++) {
      const f32x4 t = total(adw[hi][jt]);
#pragma unroll
      for (int i = 0; i < 4; i++) dw[int64_t(16 * (wave + 8 * hi) + 4 * g + i) * K + J0 + 16 * jt + r] = t[i];
    }
}

// Head role, one workgroup per 64 h-columns (H / HQ of them; one workgroup for all 256 streamed 1 MB
// through one CU, ~21 us): dWh[:, Hq], db[Hq] and (hq = 0) dbh over all rows. Wave w takes h-tile w & 3
// of the 64-row chunk's 32-row half w >> 2; the halves are summed through LDS at the end.
template <int A1>
__device__ __forceinline__ void k12x_head(CPair dz, CPair y, CPair dpre, int64_t M, float* __restrict__ db,
                                          float* __restrict__ dwh, float* __restrict__ dbh, unsigned short* lds,
                                          int hq, int c0, int c1) {
  unsigned short* dm = lds;                  // [plane][m][HQP]
  unsigned short* ys = lds + 2 * MC * HQP;   // [plane][m][HQP]
  unsigned short* zs = lds + 4 * MC * HQP;   // [plane][m][16] (a >= A1 and rows >= M zero)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int q = r >> 2, p = r & 3, ht = wave & 3, ks = wave >> 2;
  const int64_t Mend = min(M, int64_t(c1) * MC);
  const int64_t h0 = int64_t(hq) * HQ;
  // 64 rows x 64 h x 4 planes = 32 KB per chunk: one uint4 per plane per thread; two stages
  uint4 sd[2][2], sy[2][2];
  unsigned short zh[2][2], zl[2][2];
  const int lrow = tid >> 3, lpc = tid & 7;
  auto load = [&](int st, int c) {
    const int64_t o = min(int64_t(c) * MC + lrow, M - 1) * H + h0 + 8 * lpc;
    sd[st][0] = *reinterpret_cast<const uint4*>(&dpre.hi[o]);
    sd[st][1] = *reinterpret_cast<const uint4*>(&dpre.lo[o]);
    sy[st][0] = *reinterpret_cast<const uint4*>(&y.hi[o]);
    sy[st][1] = *reinterpret_cast<const uint4*>(&y.lo[o]);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int e = tid + NT * k, m = e >> 4, a = e & 15;
      const int64_t oz = min(int64_t(c) * MC + m, M - 1) * A1 + min(a, A1 - 1);
      zh[st][k] = dz.hi[oz];
      zl[st][k] = dz.lo[oz];
    }
  };
  auto store = [&](int st, int c) {
    const int64_t m0 = int64_t(c) * MC;
    const bool ok = m0 + lrow < Mend;
    const int o = lrow * HQP + 8 * lpc;
    *reinterpret_cast<uint4*>(&dm[o]) = keep_if(ok, sd[st][0]);
    *reinterpret_cast<uint4*>(&dm[MC * HQP + o]) = keep_if(ok, sd[st][1]);
    *reinterpret_cast<uint4*>(&ys[o]) = keep_if(ok, sy[st][0]);
    *reinterpret_cast<uint4*>(&ys[MC * HQP + o]) = keep_if(ok, sy[st][1]);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int e = tid + NT * k, m = e >> 4, a = e & 15;
      const bool okz = m0 + m < Mend && a < A1;
      zs[e] = okz ? zh[st][k] : static_cast<unsigned short>(0);
      zs[MC * 16 + e] = okz ? zl[st][k] : static_cast<unsigned short>(0);
    }
  };
  u16x8 onev;
#pragma unroll
  for (int j = 0; j < 8; j++) onev[j] = (r == 0) ? static_cast<unsigned short>(0x3f80) : static_cast<unsigned short>(0);
  const bf16x8 ones = as_bf(onev);  // as A: row 0 all ones; as B: column 0 all ones
  const bool want_bh = hq == 0 && ht == 0;
  Acc awh = acc0(), adb = acc0(), abh = acc0();
  load(0, c0);
  load(1, min(c0 + 1, c1 - 1));
  auto chunk = [&](int st, int c) {
    store(st, c);
    __syncthreads();
    load(st, min(c + 2, c1 - 1));
    const unsigned short* pz = &zs[(32 * ks + 4 * g + q) * 16 + 4 * p];
    const bf16x8 azh = tr8(pz, pz + 16 * 16), azl = tr8(pz + MC * 16, pz + MC * 16 + 16 * 16);
    const int off = (32 * ks + 4 * g + q) * HQP + 16 * ht + 4 * p;
    const bf16x8 byh = tr8(&ys[off], &ys[off + 16 * HQP]), byl = tr8(&ys[MC * HQP + off], &ys[MC * HQP + off + 16 * HQP]);
    const bf16x8 bdh = tr8(&dm[off], &dm[off + 16 * HQP]), bdl = tr8(&dm[MC * HQP + off], &dm[MC * HQP + off + 16 * HQP]);
    mma3(awh, azh, azl, byh, byl);
    mma2a(adb, ones, bdh, bdl);
    if (want_bh) {  // dbh: dzᵀ times a ones column (B exact)
      abh.x = mfma(azl, ones, abh.x);
      abh.hh = mfma(azh, ones, abh.hh);
    }
    __syncthreads();
  };
  for (int c = c0; c < c1; c += 2) {  // an odd count runs one all-zero chunk past the end
    chunk(0, c);
    chunk(1, c + 1);
  }
  // sum the two row halves: waves 4..7 park their totals in LDS (the images are free after the last barrier)
  float* red = reinterpret_cast<float*>(lds);
  f32x4 tw = total(awh), tb = total(adb), tbh = total(abh);
  if (ks == 1) {
    float* o = red + (ht * 64 + lane) * 12;
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = tw[i], o[4 + i] = tb[i], o[8 + i] = tbh[i];
  }
  __syncthreads();
  if (ks == 0) {
    const float* o = red + (ht * 64 + lane) * 12;
#pragma unroll
    for (int i = 0; i < 4; i++) tw[i] += o[i], tb[i] += o[4 + i], tbh[i] += o[8 + i];
    const int64_t h = h0 + 16 * ht + r;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * g + i < A1) dwh[(4 * g + i) * H + h] = tw[i];
    if (g == 0) db[h] = tb[0];
    if (want_bh && r == 0) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (4 * g + i < A1) dbh[4 * g + i] = tbh[i];
    }
  }
}

// Row parts: with rs = 2 every column / head workgroup exists twice, each over half of the 64-row chunks;
// part 0 writes dW / db / dWh / dbh in place, part 1 into the second slab (same layout), and the next
// launch's Adam workgroups add the two (x3 trunk reduce, X3Adam::grad2) — no merge inside this launch (an
// in-launch merge measured slower: its agent-scope release / acquire writes back and invalidates the XCD's
// L2 under the workgroups still streaming dpre, 21.8 -> 34.7 us at M = 500, profiles/x3_kernels_r5.txt).
template <int A1>
__global__ __launch_bounds__(NT) void k_dense_heads_bwd_x3(CPair dz, CPair y, CPair x, CPair w, CPair dpre, int64_t M,
                                                           int64_t K, Pair dx, float* __restrict__ dw,
                                                           float* __restrict__ db, float* __restrict__ dwh,
                                                           float* __restrict__ dbh, int rs, float* __restrict__ dw2,
                                                           float* __restrict__ db2, float* __restrict__ dwh2,
                                                           float* __restrict__ dbh2, uint64_t* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[K12X_LDS];
  // grid: rs x K / JB column workgroups, then rs x H / HQ head workgroups
  const int NJ = int(K / JB), b = blockIdx.x, NC = int((M + MC - 1) / MC);
  const bool head = b >= NJ * rs;
  const int i = head ? b - NJ * rs : b, per = head ? H / HQ : NJ, part = i / per, j = i - part * per;
  const int c0 = NC * part / rs, c1 = NC * (part + 1) / rs;
  x3_ts(ts, TS_K12, 0);
  if (head)
    k12x_head<A1>(dz, y, dpre, M, part ? db2 : db, part ? dwh2 : dwh, part ? dbh2 : dbh, lds, j, c0, c1);
  else
    k12x_cols(x, w, dpre, M, K, int64_t(j) * JB, dx, part ? dw2 : dw, lds, c0, c1);
  x3_ts(ts, TS_K12, 15);
}

}  // namespace x3

// ---------------------------------------------------------------- host launchers (dense tail)
// K13x configurations: M <= 64: 16x16 per wave (FM = FN = 1); larger M: 32x32 (FM = FN = 2)
static void x3_part_cfg(int64_t M, int64_t K, int N, int* fm, int* S) {
  if (M > 64 && N % 64 == 0) {  // K13x-L: 64 x 64 tiles, slices for >= 256 workgroups, >= 4 k-steps each
    const int64_t tiles = ((M + 63) / 64) * (N / 64), steps = K / 32;
    // 256 workgroups (one per CU): 512 / 1024 measured slower for both K13x-L and its consumer, which sums
    // the S slices (11.2 / 13.2 / 16.1 us at M = 500, profiles/x3_kernels_r5.txt)
    int64_t s = (256 + tiles - 1) / tiles;
    s = std::max<int64_t>(1, std::min<int64_t>({s, 32, std::max<int64_t>(1, steps / 4)}));
    *fm = 0;
    *S = int(s);
    return;
  }
  const int f = M <= 64 ? 1 : 2;
  const int64_t tiles = ((M + 16 * f - 1) / (16 * f)) * (N / (16 * f));
  const int64_t steps = K / 32;
  int64_t s = M <= 64 ? 8 : (512 + tiles - 1) / tiles;  // ~512+ workgroups
  s = std::min<int64_t>(s, std::max<int64_t>(1, steps / 8));
  s = std::max<int64_t>(1, std::min<int64_t>(s, 16));
  *fm = f;
  *S = int(s);
}
int x3_dense_fwd_part_slices(int64_t M, int64_t K, int N) {
  int f, S;
  x3_part_cfg(M, K, N, &f, &S);
  return S;
}
void x3_dense_fwd_part(X3In x, X3In w, int64_t M, int64_t K, int N, float* part, int S, hipStream_t stream) {
  if (M <= 0) return;
  if (K % 32 != 0 || N % 32 != 0) throw std::invalid_argument("x3_dense_fwd_part: K % 32 == 0 and N % 32 == 0");
  check_pair(x, "x3_dense_fwd_part x");
  check_pair(w, "x3_dense_fwd_part w");
  int f, s_cfg;
  x3_part_cfg(M, K, N, &f, &s_cfg);
  if (S != s_cfg) throw std::invalid_argument("x3_dense_fwd_part: S must be x3_dense_fwd_part_slices(M, K, N)");
  if (f == 0) {
    const int64_t tiles = ((M + 63) / 64) * (N / 64);
    hipLaunchKernelGGL(x3::k_dense_fwd_lds_x3, dim3(uint32_t(tiles * S)), dim3(256), 0, stream, cp(x), cp(w), M, K, N,
                       S, part, x3::g_x3_probe);
    RMM_HIP_CHECK(hipGetLastError());
    return;
  }
  const int64_t tiles = ((M + 16 * f - 1) / (16 * f)) * (N / (16 * f));
  const dim3 grid(uint32_t(tiles * S)), block(256);
  if (f == 1)
    hipLaunchKernelGGL((x3::k_dense_fwd_part_x3<1, 1, 4>), grid, block, 0, stream, cp(x), cp(w), M, K, N, S, part);
  else
    hipLaunchKernelGGL((x3::k_dense_fwd_part_x3<2, 2, 4>), grid, block, 0, stream, cp(x), cp(w), M, K, N, S, part);
  RMM_HIP_CHECK(hipGetLastError());
}

int x3_heads_ppo_groups(int64_t M) { return int((M + 3) / 4); }
void x3_heads_ppo(const float* hpart, int S, X3In hb, X3In wh, X3In bh, const float* cols, const float* coef, float* acc,
                  const float* gout, int64_t M, int A1, X3Out dz, X3Out dpre, X3Out hid, hipStream_t stream,
                  const int64_t* cidx, const int64_t* ctr, int64_t period, bool acc_slab) {
  if (M <= 0) return;
  if (period < 1) period = 1;
  if (A1 < 3 || A1 > dense::AMAX) throw std::invalid_argument("x3_heads_ppo: 2 <= A <= 15 actions");
  if (!hpart || S < 1 || !hb.hi || !hb.lo || !wh.hi || !wh.lo || !bh.hi || !bh.lo || !dz.hi || !dz.lo || !dpre.hi ||
      !dpre.lo || !hid.hi || !hid.lo)
    throw std::invalid_argument("x3_heads_ppo: partials, split weights and split outputs required");
  const dim3 grid(uint32_t(x3_heads_ppo_groups(M))), block(256);
#define RMM_K15X(N)                                                                                               \
  case N:                                                                                                         \
    hipLaunchKernelGGL(x3::k_heads_ppo_x3<N>, grid, block, 0, stream, hpart, S, cp(hb), cp(wh), cp(bh), cols, coef, \
                       acc, gout, M, pp(dz), pp(dpre), pp(hid), cidx, ctr, period, int(acc_slab), x3::g_x3_probe); \
    break;
  switch (A1) {
    RMM_K15X(3) RMM_K15X(4) RMM_K15X(5) RMM_K15X(6) RMM_K15X(7) RMM_K15X(8) RMM_K15X(9)
    RMM_K15X(10) RMM_K15X(11) RMM_K15X(12) RMM_K15X(13) RMM_K15X(14) RMM_K15X(15) RMM_K15X(16)
  }
#undef RMM_K15X
  RMM_HIP_CHECK(hipGetLastError());
}

void x3_heads_sample(const float* hpart, int S, X3In hb, X3In wh, X3In bh, const int64_t* t_ptr, const int64_t* ctr,
                     uint32_t seed, int64_t* act, float* logp, float* vf, float* lout, int64_t* act_now, int64_t B, int A1,
                     hipStream_t stream, unsigned int* done, int64_t* host_seq) {
  if (B <= 0) return;
  if (host_seq != nullptr && done == nullptr) throw std::invalid_argument("x3_heads_sample: host_seq needs done");
  if (A1 < 3 || A1 > dense::AMAX) throw std::invalid_argument("x3_heads_sample: 2 <= A <= 15 actions");
  if (!hpart || S < 1 || !hb.hi || !hb.lo || !wh.hi || !wh.lo || !bh.hi || !bh.lo)
    throw std::invalid_argument("x3_heads_sample: partials and split weights required");
  if (done != nullptr && B <= 32) {  // one workgroup, thread 0 advances the step after a barrier
    auto* tw = const_cast<int64_t*>(t_ptr);
    auto* cw = const_cast<int64_t*>(ctr);
#define RMM_K16X1(N)                                                                                               \
  case N:                                                                                                          \
    hipLaunchKernelGGL((x3::k_heads_sample1_x3<N, 2>), dim3(1), dim3(1024), 0, stream, hpart, S, cp(hb), cp(wh),    \
                       cp(bh), tw, cw, seed, act, logp, vf, lout, act_now, B, host_seq);                           \
    break;
    switch (A1) {
      RMM_K16X1(3) RMM_K16X1(4) RMM_K16X1(5) RMM_K16X1(6) RMM_K16X1(7) RMM_K16X1(8) RMM_K16X1(9)
      RMM_K16X1(10) RMM_K16X1(11) RMM_K16X1(12) RMM_K16X1(13) RMM_K16X1(14) RMM_K16X1(15) RMM_K16X1(16)
    }
#undef RMM_K16X1
    RMM_HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid(uint32_t((B + 3) / 4)), block(256);
#define RMM_K16X(N)                                                                                                \
  case N:                                                                                                          \
    hipLaunchKernelGGL(x3::k_heads_sample_x3<N>, grid, block, 0, stream, hpart, S, cp(hb), cp(wh), cp(bh), t_ptr,   \
                       ctr, seed, act, logp, vf, lout, act_now, B, done, host_seq);                                \
    break;
  switch (A1) {
    RMM_K16X(3) RMM_K16X(4) RMM_K16X(5) RMM_K16X(6) RMM_K16X(7) RMM_K16X(8) RMM_K16X(9)
    RMM_K16X(10) RMM_K16X(11) RMM_K16X(12) RMM_K16X(13) RMM_K16X(14) RMM_K16X(15) RMM_K16X(16)
  }
#undef RMM_K16X
  RMM_HIP_CHECK(hipGetLastError());
}

void x3_dense_heads_sample(X3In x, X3In w, int64_t M, int64_t K, float* part, int S, X3In hb, X3In wh, X3In bh,
                           const int64_t* t_ptr, const int64_t* ctr, uint32_t seed, int64_t* act, float* logp, float* vf,
                           float* lout, int64_t* act_now, int A1, hipStream_t stream, unsigned int* done,
                           int64_t* host_seq) {
  if (M <= 0) return;
  int f, s_cfg;
  x3_part_cfg(M, K, dense::H, &f, &s_cfg);
  if (f != 1 || S != s_cfg) throw std::invalid_argument("x3_dense_heads_sample: M <= 64 and S = x3_dense_fwd_part_slices");
  if (K % 32 != 0) throw std::invalid_argument("x3_dense_heads_sample: K % 32 == 0");
  if (!done || !part) throw std::invalid_argument("x3_dense_heads_sample: ticket words (1 + ceil(M / 16)) and partials");
  if (A1 < 3 || A1 > dense::AMAX) throw std::invalid_argument("x3_dense_heads_sample: 2 <= A <= 15 actions");
  check_pair(x, "x3_dense_heads_sample x");
  check_pair(w, "x3_dense_heads_sample w");
  if (!hb.hi || !hb.lo || !wh.hi || !wh.lo || !bh.hi || !bh.lo)
    throw std::invalid_argument("x3_dense_heads_sample: split head weights required");
  const int64_t tiles = ((M + 15) / 16) * (dense::H / 16);
  const dim3 grid(uint32_t(tiles * S)), block(256);
#define RMM_K1316X(N)                                                                                              \
  case N:                                                                                                          \
    hipLaunchKernelGGL(x3::k_dense_heads_sample_x3<N>, grid, block, 0, stream, cp(x), cp(w), M, K, S, part, cp(hb), \
                       cp(wh), cp(bh), t_ptr, ctr, seed, act, logp, vf, lout, act_now, done, host_seq);           \
    break;
  switch (A1) {
    RMM_K1316X(3) RMM_K1316X(4) RMM_K1316X(5) RMM_K1316X(6) RMM_K1316X(7) RMM_K1316X(8) RMM_K1316X(9)
    RMM_K1316X(10) RMM_K1316X(11) RMM_K1316X(12) RMM_K1316X(13) RMM_K1316X(14) RMM_K1316X(15) RMM_K1316X(16)
  }
#undef RMM_K1316X
  RMM_HIP_CHECK(hipGetLastError());
}

void x3_dense_heads_bwd(X3In dz, int A1, X3In y, X3In x, X3In w, X3In dpre, int64_t M, int64_t K, X3Out dx, float* dw,
                        float* db, float* dwh, float* dbh, hipStream_t stream, int rs, float* dw2, float* db2,
                        float* dwh2, float* dbh2) {
  if (M <= 0) return;
  if (K % x3::JB != 0) throw std::invalid_argument("x3_dense_heads_bwd: K must be a multiple of 32");
  if (A1 < 1 || A1 > dense::AMAX) throw std::invalid_argument("x3_dense_heads_bwd: 1 <= A+1 <= 16");
  for (const X3In* p : {&dz, &y, &x, &w, &dpre})
    if (!p->hi || !p->lo) throw std::invalid_argument("x3_dense_heads_bwd: inputs need hi and lo planes");
  if (!dx.hi || !dx.lo || !dw || !db || !dwh || !dbh) throw std::invalid_argument("x3_dense_heads_bwd: outputs");
  if (rs != 1 && rs != 2) throw std::invalid_argument("x3_dense_heads_bwd: rs (row parts) is 1 or 2");
  if (rs == 2 && (!dw2 || !db2 || !dwh2 || !dbh2 || (M + x3::MC - 1) / x3::MC < 2))
    throw std::invalid_argument("x3_dense_heads_bwd: rs = 2 needs the second slab's outputs and >= 2 row chunks");
  const dim3 grid(uint32_t(rs * (K / x3::JB + x3::H / x3::HQ))), block(x3::NT);
#define RMM_K12X(N)                                                                                                 \
  case N:                                                                                                           \
    hipLaunchKernelGGL(x3::k_dense_heads_bwd_x3<N>, grid, block, 0, stream, cp(dz), cp(y), cp(x), cp(w), cp(dpre), M, \
                       K, pp(dx), dw, db, dwh, dbh, rs, dw2, db2, dwh2, dbh2, x3::g_x3_probe);                       \
    break;
  switch (A1) {
    RMM_K12X(1) RMM_K12X(2) RMM_K12X(3) RMM_K12X(4) RMM_K12X(5) RMM_K12X(6) RMM_K12X(7) RMM_K12X(8)
    RMM_K12X(9) RMM_K12X(10) RMM_K12X(11) RMM_K12X(12) RMM_K12X(13) RMM_K12X(14) RMM_K12X(15) RMM_K12X(16)
  }
#undef RMM_K12X
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm

namespace rmm {
namespace hip {
namespace x3 {
__global__ __launch_bounds__(256) void k_split(const float* __restrict__ src, unsigned short* __restrict__ hi,
                                               unsigned short* __restrict__ lo, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    unsigned short h, l;
    split(src[i], h, l);
    hi[i] = h;
    lo[i] = l;
  }
}
}  // namespace x3
void x3_split(const float* src, void* hi, void* lo, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(x3::k_split, dim3(uint32_t(blocks)), dim3(256), 0, stream, src, static_cast<unsigned short*>(hi),
                     static_cast<unsigned short*>(lo), n);
  RMM_HIP_CHECK(hipGetLastError());
}
}  // namespace hip
}  // namespace rmm
