// K10 — fused Nature-CNN trunk (RLlib's default 84x84 Atari vision net) on MFMA.
//
// Geometry (rllib/models/utils.py:get_filter_config for 84x84, SAME padding as RLlib SlimConv2d):
//   frames u8 [B,4,84,84] --conv1 8x8/4 pad 2, 4->16, +b, ReLU--> h1 [B,21,21,16]
//                          --conv2 4x4/2 pad 2, 16->32, +b, ReLU--> h2 [B,11,11,32] (= NHWC flatten 3872)
// The 11x11 "valid" third conv is a dense layer (3872 -> 256): the hand-written K13s / K12 kernels in
// dense_kernels.hip (bf16) and K13x / K12x in x3_kernels.hip (fp32-level) run it, not hipBLASLt.
//
// Why fused: per SGD minibatch (500 frames) these two layers are ~3.6+2.0 MFLOP/frame — nothing
// for MFMA — but MIOpen runs them as 10+ launches (gather/convert, implicit-GEMM fwd, bias/ReLU,
// bwd-data, two weight-grad kernels with zero-fills, bias-grad reductions) of 5-35 us each. Here
// one workgroup owns one frame at a time entirely in LDS:
//   fwd:  gather u8 frame by minibatch index (device counter window, HIP-graph friendly) → LDS,
//         conv1 as im2col-on-the-fly GEMM  M=441 pos x N=16 x K=256 (k = ky,kx,ci over an HWC LDS frame) (v_mfma_f32_16x16x32_bf16),
//         bias+ReLU epilogue into an LDS NHWC tile (and h1 out for backward), conv2 the same way
//         M=121 x N=32 x K=256 from LDS, bias+ReLU → h2.  1 launch.
//   bwd:  dpre2 = dh2·[h2>0] (+db2), dW2 += dpre2ᵀ·im2col(h1) (K = positions), dh1 = conv2ᵀ by
//         stride-parity class (each class is a dense K=4 taps x 32 GEMM), dpre1 = dh1·[h1>0]
//         (+db1), dW1 += dpre1ᵀ·im2col(frame) computed in space-to-depth form (a 2x2 stride-1
//         correlation over a 64-channel 22x22 grid: contiguous operands). Weight-grad accumulators stay in registers across
//         the frames a workgroup owns; one deterministic reduce launch sums the per-workgroup
//         partials and writes bf16 grads in the parameters' memory order.  2 launches.
// The 1/255 frame scale is applied to the fp32 conv1 accumulator (exact integer pixels in bf16).
//
// MFMA 16x16x32 bf16 fragment maps (gfx950): lane l holds A[row l&15][k 8(l>>4)+j],
// B[k 8(l>>4)+j][col l&15], j = 0..7; C/D: col l&15, row 4(l>>4)+i, i = 0..3.
#include <hip/hip_bf16.h>

#include "adam_device.h"
#include "common.h"
#include "dense_device.h"
#include "kernels.h"
#include "trunk_device.h"

namespace rmm {
namespace hip {
namespace trunk {


// ================================================================ forward
// grid = B workgroups (one frame each), NTF threads.
constexpr int NTF = 512;  // forward: 8 waves per frame halve each wave's serial MFMA/LDS chain
__global__ __launch_bounds__(NTF) void k_trunk_fwd(
    const uint8_t* __restrict__ obs, const int64_t* __restrict__ idx0, const int64_t* __restrict__ ctr, int64_t period,
    int64_t B, const unsigned short* __restrict__ W1, WStrides w1, const unsigned short* __restrict__ b1,
    const unsigned short* __restrict__ W2, WStrides w2, const unsigned short* __restrict__ b2,
    unsigned short* __restrict__ h1_out, unsigned short* __restrict__ h2_out, int dbg, uint8_t* push_stack,
    const uint8_t* __restrict__ push_new, uint8_t* push_rows, const int64_t* __restrict__ push_t) {
  __shared__ __attribute__((aligned(16))) unsigned short fh[HF_ELEMS];  // bf16 half image (two passes)
  __shared__ __attribute__((aligned(16))) unsigned short h1p[H1P_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short w1s[C1 * W1_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w2s[C2 * W2_PITCH];
  const int64_t b = blockIdx.x;
  const int64_t* idx = window(idx0, ctr, period, B);
  const int64_t src = idx ? idx[b] : b;

  // the frame's HBM loads go out first and stay in flight through the weight staging (L2) and the
  // LDS zeroing; one barrier then covers weights, zeros and the frame interior
  if (dbg & 128) return;  // profiling: launch + dispatch floor
  // weight loads first (L2-resident, shorter round trip): their LDS stores below then wait for them
  // alone while the frame's loads stay in flight
  WeightRegs<NTF, C1, C0, 8> wr1;
  WeightRegs<NTF, C2, C1, 4> wr2;
  if (!(dbg & 8)) {
    weight_issue(W1, w1, wr1);
    weight_issue(W2, w2, wr2);
  }
  FrameRegs<NTF> fr;
  constexpr int64_t FB = C0 * H0 * H0;
  if (push_stack)
    frame_issue_push<NTF>(push_stack + b * FB, push_new + b * (H0 * H0), fr);
  else if (!(dbg & 32))
    frame_issue<NTF>(obs + src * FB, fr);
  const TrunkBias tb = trunk_bias(b1, b2);
  zero_half_frame_border(fh);
  zero_lds(h1p, H1P_ELEMS * 2);
  if (!(dbg & 8)) {
    weight_store(wr1, W1, w1, w1s, W1_PITCH);
    weight_store(wr2, W2, w2, w2s, W2_PITCH);
  }
  if (push_stack) frame_push_store<NTF>(fr, push_stack + b * FB, push_rows ? push_rows + (push_t[0] * B + b) * FB : nullptr);
  // trunk_convs' first barrier covers the border / h1p zeros, the weights and pass 0's frame rows
  trunk_convs<NTF>(fr, fh, h1p, w1s, w2s, tb, h1_out ? h1_out + b * NP1 * C1 : nullptr, h2_out + b * NP2 * C2, dbg);
}


// ================================================================ forward, rollout band mode
// Rollout step at small B (one env per frame, B ~ 12-50): one workgroup per frame leaves most CUs
// idle and the launch is a single frame's latency chain (~12 µs at any B <= 256). Here each frame
// is split into NBAND workgroups by bands of conv2 output rows; a band computes the conv1 rows its
// conv2 rows need (a 1-2 row halo, ~25% extra conv1 work) from the frame rows those need.
// The frame stack is the previous rollout row: rows[(t-1) mod T] planes 1..3 + the env's newest
// frame (may be device-mapped pinned host memory); each band writes its own disjoint 21 frame rows
// of all 4 planes into rollout row t, and reads only row t-1 — so no band reads what another band
// writes in the same launch, and no separate frame-stack buffer exists.
constexpr int NBAND = 4, NTFB = 512;
constexpr int BAND_FR = 36;              // padded frame rows per band tile (band 1: input rows 14..49)
constexpr int BAND_H1R = 8;              // padded h1 rows per band tile
__device__ __forceinline__ void band_geom(int s, int& o0, int& o1, int& ya, int& yb) {
  o0 = 3 * s;                            // conv2 rows [o0, o1)
  o1 = min(H2, o0 + 3);
  ya = max(0, 2 * o0 - 2);               // conv1 (h1) rows [ya, yb] they read
  yb = min(H1 - 1, 2 * o1 - 1);
}
__global__ __launch_bounds__(NTFB) void k_trunk_fwd_band(
    const unsigned short* __restrict__ W1, WStrides w1, const unsigned short* __restrict__ b1,
    const unsigned short* __restrict__ W2, WStrides w2, const unsigned short* __restrict__ b2,
    unsigned short* __restrict__ h2_out, int64_t B, uint8_t* rows, int64_t T, const uint8_t* __restrict__ nf,
    const int64_t* __restrict__ t_ptr) {
  __shared__ __attribute__((aligned(16))) uint8_t frame[BAND_FR * P0 * 4];
  __shared__ __attribute__((aligned(16))) unsigned short h1p[BAND_H1R * P1 * C1];
  __shared__ __attribute__((aligned(16))) unsigned short w1s[C1 * W1_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short w2s[C2 * W2_PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t b = blockIdx.x / NBAND;
  const int s = blockIdx.x % NBAND;
  int o0, o1, ya, yb;
  band_geom(s, o0, o1, ya, yb);
  const int fr0 = max(0, 4 * ya - 2), fr1 = min(H0 - 1, 4 * yb + 5);  // frame rows read
  const int pr0 = 4 * ya;                                              // padded row of tile row 0
  constexpr int64_t FB = C0 * H0 * H0;
  constexpr int NWP = H0 * H0 / 4;                                     // u32 words per plane
  const int64_t t = t_ptr[0];
  const uint8_t* prev = rows + (((t == 0 ? T : t) - 1) * B + b) * FB;
  uint32_t* cur32 = reinterpret_cast<uint32_t*>(rows + (t * B + b) * FB);
  const uint32_t* p32 = reinterpret_cast<const uint32_t*>(prev);
  const uint32_t* n32 = reinterpret_cast<const uint32_t*>(nf + b * (H0 * H0));
  constexpr int PER = (BAND_FR * 21 + NTFB - 1) / NTFB;
  const int w0 = fr0 * 21, nw = (fr1 - fr0 + 1) * 21;
  WeightRegs<NTFB, C1, C0, 8> wr1;
  WeightRegs<NTFB, C2, C1, 4> wr2;
  weight_issue(W1, w1, wr1);
  weight_issue(W2, w2, wr2);
  uint32_t v[PER][C0];
#pragma unroll
  for (int k = 0; k < PER; k++) {  // all loads first (unconditional, clamped): one round trip
    const int o = w0 + min(tid + NTFB * k, nw - 1);
#pragma unroll
    for (int c = 0; c < C0 - 1; c++) v[k][c] = p32[(c + 1) * NWP + o];
    v[k][C0 - 1] = n32[o];
  }
  zero_lds(frame, BAND_FR * P0 * 4);
  zero_lds(h1p, BAND_H1R * P1 * C1 * 2);
  weight_store(wr1, W1, w1, w1s, W1_PITCH);
  weight_store(wr2, W2, w2, w2s, W2_PITCH);
  __syncthreads();
  const int own0 = 21 * s, own1 = own0 + 21;  // the frame rows this band stores into rollout row t
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int i = tid + NTFB * k;
    if (i < nw) {
      const int o = w0 + i, y = o / 21, xw = o - y * 21;
      uint32_t px[4];
#pragma unroll
      for (int q = 0; q < 4; q++)
        px[q] = ((v[k][0] >> (8 * q)) & 0xffu) | (((v[k][1] >> (8 * q)) & 0xffu) << 8) |
                (((v[k][2] >> (8 * q)) & 0xffu) << 16) | (((v[k][3] >> (8 * q)) & 0xffu) << 24);
      uint2* d = reinterpret_cast<uint2*>(frame + ((y + 2 - pr0) * P0 + 4 * xw + 2) * 4);
      d[0] = make_uint2(px[0], px[1]);
      d[1] = make_uint2(px[2], px[3]);
      if (y >= own0 && y < own1) {
#pragma unroll
        for (int c = 0; c < C0; c++) cur32[c * NWP + o] = v[k][c];
      }
    }
  }
  __syncthreads();

  bf16x8 wf1[8];
#pragma unroll
  for (int k = 0; k < 8; k++) wf1[k] = as_bf(*reinterpret_cast<const u16x8*>(&w1s[r * W1_PITCH + (k * 8 + 2 * g) * 4]));
  const float bias1 = bf2f(b1[r]);
  // ---- conv1 over h1 rows [ya, yb]: position p -> (y = ya + p / 21, x = p % 21)
  const int np1 = (yb - ya + 1) * H1;
  for (int mt = wave; mt * 16 < np1; mt += NTFB / 64) {
    const int p = min(mt * 16 + r, np1 - 1);
    const int oy = ya + p / H1, ox = p - (p / H1) * H1;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; k++) acc = mfma(frame8(frame, ((4 * (oy - ya) + k) * P0 + 4 * ox + 2 * g) * 4), wf1[k], acc);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int q = mt * 16 + 4 * g + i;
      if (q < np1) {
        const int y = ya + q / H1, x = q - (q / H1) * H1;
        h1p[((y + 2 - 2 * o0) * P1 + (x + 2)) * C1 + r] = f2bf(fmaxf(acc[i] * (1.0f / 255.0f) + bias1, 0.f));
      }
    }
  }
  bf16x8 wf2[2][8];
#pragma unroll
  for (int nt = 0; nt < 2; nt++)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int pp = 2 * k + (g >> 1), co = nt * 16 + r;
      wf2[nt][k] = as_bf(*reinterpret_cast<const u16x8*>(&w2s[co * W2_PITCH + pp * 16 + 8 * (g & 1)]));
    }
  const float bias2[2] = {bf2f(b2[r]), bf2f(b2[16 + r])};
  __syncthreads();
  // ---- conv2 over rows [o0, o1): position q -> (oy = o0 + q / 11, ox = q % 11)
  const int np2 = (o1 - o0) * H2;
  for (int mt = wave; mt * 16 < np2; mt += NTFB / 64) {
    const int q = min(mt * 16 + r, np2 - 1);
    const int oy = o0 + q / H2, ox = q - (q / H2) * H2;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int pp = 2 * k + (g >> 1), ky = pp >> 2, kx = pp & 3;
      const bf16x8 a = as_bf(*reinterpret_cast<const u16x8*>(
          &h1p[((2 * (oy - o0) + ky) * P1 + (2 * ox + kx)) * C1 + 8 * (g & 1)]));
      acc0 = mfma(a, wf2[0][k], acc0);
      acc1 = mfma(a, wf2[1][k], acc1);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int qq = mt * 16 + 4 * g + i;
      if (qq < np2) {
        const int64_t pos = int64_t(o0) * H2 + qq;  // = oy * 11 + ox
        h2_out[(b * NP2 + pos) * C2 + r] = f2bf(fmaxf(acc0[i] + bias2[0], 0.f));
        h2_out[(b * NP2 + pos) * C2 + 16 + r] = f2bf(fmaxf(acc1[i] + bias2[1], 0.f));
      }
    }
  }
}

// ================================================================ backward
constexpr int PART = C1 * 256 + C2 * 256 + C1 + C2;  // per-workgroup fp32 partial: dW1, dW2, db1, db2
// row pitches of the transposed dpre tiles: +8 elements so the 16 rows written by one lane
// group land 4 dwords apart (2-way instead of 16-way bank conflicts) while keeping 16-B reads
constexpr int DP2_PITCH = NP2P + 8;
// dpre2 in a 12x12 grid (row/column 11 zero) so the dh1 taps read it without bounds branches
constexpr int D2W = 12;
// dpre1 for the dW1 GEMM: two copies (b = 0, 1) [co][Yrow*24 + X] = dpre1[Yrow-1][X-b], zero
// elsewhere, so input-grid position t = Y*24+X pairs with copy b at t + (1-a)*24 (a, b = the
// space-to-depth tap offsets). 24 rows; co pitch 584 el = 292 dwords (conflict-free 16-B reads).
constexpr int DB_CP = 24 * ST_W + 8, DB_B = 16 * DB_CP;
constexpr int KSTEPS1 = (22 * ST_W + 31) / 32;  // 17 K-steps of 32 grid positions
static_assert(KSTEPS1 * 32 + 8 <= ST_CP, "st K padding");
static_assert(KSTEPS1 * 32 + ST_W <= 24 * ST_W, "dpre1 copy K padding");

// grid = G workgroups of 8 waves (2 per SIMD hide the LDS/MFMA latency chains of one frame),
// each loops over frames b = blockIdx.x, +G, ...
constexpr int NTB = 512;
constexpr int BWD_NH1 = NP1 * 2, BWD_PH1 = (BWD_NH1 + NTB - 1) / NTB;  // 882 x 16 B
constexpr int BWD_NH2 = NP2 * 4, BWD_PH2 = (BWD_NH2 + NTB - 1) / NTB;  // 484 x 16 B
__device__ __forceinline__ void h1_issue(int64_t bb, const unsigned short* __restrict__ h1, u16x8 (&hv1)[BWD_PH1]) {
#pragma unroll
  for (int k = 0; k < BWD_PH1; k++) {
    const int v = min(int(threadIdx.x) + NTB * k, BWD_NH1 - 1);
    hv1[k] = *reinterpret_cast<const u16x8*>(&h1[(bb * NP1 + (v >> 1)) * C1 + 8 * (v & 1)]);
  }
}
// P0 global loads of frame bb (clamped and unconditional, see load_frame)
__device__ __forceinline__ void bwd_issue(int64_t bb, const int64_t* __restrict__ idx, const uint8_t* __restrict__ obs,
                                          const unsigned short* __restrict__ h1, const unsigned short* __restrict__ h2,
                                          const unsigned short* __restrict__ dh2, FrameRegs<NTB>& fr,
                                          u16x8 (&hv1)[BWD_PH1], u16x8 (&hv2)[BWD_PH2], u16x8 (&gv2)[BWD_PH2]) {
  const int64_t src = idx ? idx[bb] : bb;
  frame_issue<NTB>(obs + src * (C0 * H0 * H0), fr);
#pragma unroll
  for (int k = 0; k < BWD_PH2; k++) {
    const int v = min(int(threadIdx.x) + NTB * k, BWD_NH2 - 1);
    hv2[k] = *reinterpret_cast<const u16x8*>(&h2[(bb * NP2 + (v >> 2)) * C2 + 8 * (v & 3)]);
    gv2[k] = *reinterpret_cast<const u16x8*>(&dh2[(bb * NP2 + (v >> 2)) * C2 + 8 * (v & 3)]);
  }
}
__global__ __launch_bounds__(NTB) void k_trunk_bwd(
    const uint8_t* __restrict__ obs, const int64_t* __restrict__ idx0, const int64_t* __restrict__ ctr, int64_t period,
    int64_t B, const unsigned short* __restrict__ W2, WStrides w2, const unsigned short* __restrict__ h1,
    const unsigned short* __restrict__ h2, const unsigned short* __restrict__ dh2, float* __restrict__ partial,
    int dbg) {
  __shared__ __attribute__((aligned(16))) unsigned short st[ST_ELEMS];  // space-to-depth frame
  __shared__ __attribute__((aligned(16))) unsigned short h1p[H1P_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short dp2[D2W * D2W * C2];  // [oy*12+ox][co2]
  __shared__ __attribute__((aligned(16))) unsigned short dp2t[C2 * DP2_PITCH];   // [co2][kperm(q)]
  __shared__ __attribute__((aligned(16))) unsigned short dp1s[2 * DB_B];       // dpre1 copies b = 0, 1
  __shared__ float red[8 * 64];
  static_assert(C2 * W2_PITCH <= 2 * DB_B, "w2s aliases the dpre1 copies");
  unsigned short* w2s = dp1s;  // only read before the frame loop (into wt registers)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t* idx = window(idx0, ctr, period, B);
  if (dbg & 64) return;

  // prologue: the W2 loads (L2), then the first frame's HBM loads (frame, h1, h2, dh2) go out
  // before the LDS zeroing, so the weight round trip and the frame's hide behind it
  constexpr int NH1 = BWD_NH1, PH1 = BWD_PH1, NH2 = BWD_NH2, PH2 = BWD_PH2;
  WeightRegs<NTB, C2, C1, 4> wr;
  if (!(dbg & 512)) weight_issue(W2, w2, wr);
  FrameRegs<NTB> fr;
  u16x8 hv1[PH1];
  u16x8 hv2[PH2], gv2[PH2];
  if (!(dbg & 8) && int64_t(blockIdx.x) < B) {
    bwd_issue(blockIdx.x, idx, obs, h1, h2, dh2, fr, hv1, hv2, gv2);
    h1_issue(blockIdx.x, h1, hv1);
  }
  if (!(dbg & (32 | 256))) zero_lds(st, ST_ELEMS * 2);
  if (!(dbg & 256)) {
    zero_lds(h1p, H1P_ELEMS * 2);
    zero_lds(dp2, D2W * D2W * C2 * 2);
    zero_lds(dp2t, C2 * DP2_PITCH * 2);
  }
  if (!(dbg & 512)) weight_store(wr, W2, w2, w2s, W2_PITCH);

  // dh1 = conv2ᵀ(dpre2): waves 2c, 2c+1 own stride-parity class c = (py, px). In a class,
  // input pixel (y, x) = (2a+py, 2c+px) receives taps ky ∈ {py, py+2}, kx ∈ {px, px+2} from
  // output pixel (a+1-ty, c+1-tx); k = tap*32 + co2, tap = 2ty+tx → one k-step per tap.
  const int cls = wave >> 1, half = wave & 1;
  const int py = cls >> 1, px = cls & 1;
  const int nrow = py ? 10 : 11, ncol = px ? 10 : 11, ncls = nrow * ncol;
  // m / ncol for m < 200 as a multiply-shift (ncol is wave-uniform but not compile-time: a real
  // division is ~30 VALU ops, and the dh1 loop does five per tile)
  const uint32_t cdiv = px ? 6554u : 5958u;
  __syncthreads();  // w2s staged
  bf16x8 wt[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int ky = py + 2 * (t >> 1), kx = px + 2 * (t & 1);
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = w2s[(8 * g + j) * W2_PITCH + (ky * 4 + kx) * 16 + r];
    wt[t] = as_bf(v);
  }
  f32x4 aw2[2][2], aw1[2];  // dW2 tiles (mt 0/1 x nt w+8i), dW1 tiles (b = 0, 1; see P2)
#pragma unroll
  for (int i = 0; i < 2; i++) {
    aw1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    aw2[0][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    aw2[1][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float db1 = 0.f;                       // this lane's ci = r
  float db2[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // co2 = 8(tid&3) + j
  __syncthreads();  // wt read from w2s
  if (!(dbg & 256)) zero_lds(dp1s, 2 * DB_B * 2);
  __syncthreads();

  // P0 is software-pipelined across this workgroup's frames: the global loads of frame b + G are
  // issued right after frame b's LDS tiles are written and stay in flight (registers) through
  // frame b's P1 / P2 MFMA phases, so only the first frame pays the HBM latency in the open.
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    // ---- P0: frame (space-to-depth), h1 → padded tile, h2 / dh2 → dpre2 (both layouts) + db2
    if (!(dbg & 8)) {
      frame_store_s2d<NTB>(fr, st);
#pragma unroll
      for (int k = 0; k < PH1; k++) {
        const int v = threadIdx.x + NTB * k;
        if (v < NH1) {
          const int p = v >> 1, y = p / H1, x = p - y * H1;
          *reinterpret_cast<u16x8*>(&h1p[((y + 2) * P1 + (x + 2)) * C1 + 8 * (v & 1)]) = hv1[k];
        }
      }
#pragma unroll
      for (int k = 0; k < PH2; k++) {
        const int v = threadIdx.x + NTB * k;
        if (v < NH2) {
          const int q = v >> 2, c0 = 8 * (v & 3), oy = q / H2, ox = q - oy * H2;
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; j++) {
            const unsigned short hj = hv2[k][j];
            const unsigned short d = (hj != 0 && !(hj & 0x8000)) ? gv2[k][j] : static_cast<unsigned short>(0);
            o[j] = d;
            db2[j] += bf2f(d);
            dp2t[(c0 + j) * DP2_PITCH + kperm(q)] = d;
          }
          *reinterpret_cast<u16x8*>(&dp2[(oy * D2W + ox) * C2 + c0]) = o;
        }
      }
    }
    __syncthreads();
    if (!(dbg & 8) && b + gridDim.x < B) {  // next frame: in flight through P1 / P2
      bwd_issue(b + gridDim.x, idx, obs, h1, h2, dh2, fr, hv1, hv2, gv2);
      h1_issue(b + gridDim.x, h1, hv1);
    }

    // ---- P1a: dW2[co2][k=(ky,kx,ci)] += Σ_q dpre2[q][co2] · h1p[2oy+ky][2ox+kx][ci]
#pragma unroll
    for (int s = 0; s < ((dbg & 1) ? 0 : NP2P / 32); s++) {
      const bf16x8 a0 = as_bf(*reinterpret_cast<const u16x8*>(&dp2t[r * DP2_PITCH + 32 * s + 8 * g]));
      const bf16x8 a1 = as_bf(*reinterpret_cast<const u16x8*>(&dp2t[(16 + r) * DP2_PITCH + 32 * s + 8 * g]));
      int qoff[8];  // positions q = 32s + g + 4j → element offset of (2oy, 2ox) in h1p
      {
        const int q0 = 32 * s + g;
        int oy = q0 / H2, ox = q0 - oy * H2;
#pragma unroll
        for (int j = 0; j < 8; j++) {
          qoff[j] = (q0 + 4 * j < NP2) ? (oy * 2 * P1 + ox * 2) * C1 : 0;  // dpre2 is 0 there
          ox += 4;
          if (ox >= H2) { ox -= H2; oy++; }
        }
      }
#pragma unroll
      for (int i = 0; i < 2; i++) {
        const int k = (wave + 8 * i) * 16 + r;
        const int ky = k >> 6, kx = (k >> 4) & 3, ci = k & 15;
        const unsigned short* base = h1p + (ky * P1 + kx) * C1 + ci;
        u16x8 bv;
#pragma unroll
        for (int j = 0; j < 8; j++) bv[j] = base[qoff[j]];
        const bf16x8 bb = as_bf(bv);
        aw2[0][i] = mfma(a0, bb, aw2[0][i]);
        aw2[1][i] = mfma(a1, bb, aw2[1][i]);
      }
    }
    // ---- P1b: dh1 for this wave's parity class, masked by h1 > 0 → dp1t, db1
    for (int mt = half; mt * 16 < ((dbg & 2) ? 0 : ncls); mt += 2) {
      const int m = min(mt * 16 + r, ncls - 1);  // rows >= ncls are computed but not stored
      const int a = int((uint32_t(m) * cdiv) >> 16), c = m - a * ncol;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; t++) {  // oy = a+1-ty, ox = c+1-tx ∈ [0, 11]; row/col 11 of dp2 is zero
        const int oy = a + 1 - (t >> 1), ox = c + 1 - (t & 1);
        const u16x8 av = *reinterpret_cast<const u16x8*>(&dp2[(oy * D2W + ox) * C2 + 8 * g]);
        acc = mfma(as_bf(av), wt[t], acc);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int mm = mt * 16 + 4 * g + i;
        if (mm < ncls) {
          const int aa = int((uint32_t(mm) * cdiv) >> 16), cc = mm - aa * ncol;
          const int y = 2 * aa + py, x = 2 * cc + px;
          const unsigned short hv = h1p[((y + 2) * P1 + (x + 2)) * C1 + r];
          const float d = (hv != 0 && !(hv & 0x8000)) ? acc[i] : 0.f;
          const unsigned short db = f2bf(d);
          db1 += bf2f(db);
          dp1s[r * DB_CP + (y + 1) * ST_W + x] = db;
          dp1s[DB_B + r * DB_CP + (y + 1) * ST_W + x + 1] = db;
        }
      }
    }
    __syncthreads();

    // ---- P2: dW1 in space-to-depth form: D[(a, b, c)][co] = Σ_t st[c][t] · dpre1_b[co][t + (1-a)*24]
    // over grid positions t (K). Wave w: channel block cb = w&3 (16 channels), a = w>>2, b = 0, 1
    // share the st operand.
    {
      const int cb = wave & 3, a = wave >> 2;
      const unsigned short* sa = st + st_chan(16 * cb + r) + 8 * g;
      const unsigned short* d0 = dp1s + r * DB_CP + (1 - a) * ST_W + 8 * g;
#pragma unroll
      for (int s = 0; s < ((dbg & 4) ? 0 : KSTEPS1); s++) {
        const bf16x8 av = as_bf(*reinterpret_cast<const u16x8*>(sa + 32 * s));
        const bf16x8 b0 = as_bf(*reinterpret_cast<const u16x8*>(d0 + 32 * s));
        const bf16x8 b1 = as_bf(*reinterpret_cast<const u16x8*>(d0 + DB_B + 32 * s));
        aw1[0] = mfma(av, b0, aw1[0]);
        aw1[1] = mfma(av, b1, aw1[1]);
      }
    }
    __syncthreads();
  }

  // ---- write this workgroup's partials (fp32): [dW1 16x256][dW2 32x256][db1 16][db2 32]
  // (row-major: 16 consecutive columns per lane group; measured faster than 16-B fragment-order
  // stores here, 54 vs 65 us per backward at B=500)
  float* out = partial + int64_t(blockIdx.x) * PART;
#pragma unroll
  for (int i = 0; i < ((dbg & 16) ? 0 : 2); i++) {
    const int col = (wave + 8 * i) * 16 + r;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int row = 4 * g + e;
      out[C1 * 256 + row * 256 + col] = aw2[0][i][e];
      out[C1 * 256 + (16 + row) * 256 + col] = aw2[1][i][e];
    }
  }
  // dW1: tile b holds D[m = 4g+e][co = r], channel c = 16cb + m → ry = cb, rx = g, ci = e;
  // ky = 4a + ry, kx = 4b + rx, k = 32ky + 4kx + ci
#pragma unroll
  for (int bb = 0; bb < ((dbg & 16) ? 0 : 2); bb++) {
    const int ky = 4 * (wave >> 2) + (wave & 3), kx = 4 * bb + g;
#pragma unroll
    for (int e = 0; e < 4; e++) out[r * 256 + ky * 32 + kx * 4 + e] = aw1[bb][e] * (1.0f / 255.0f);
  }
  if (dbg & 1024) return;  // profiling: no bias-gradient epilogue
  // db1: lanes r, r+16, r+32, r+48 of every wave share ci = r
  db1 += __shfl_xor(db1, 16);
  db1 += __shfl_xor(db1, 32);
  if (lane < 16) red[wave * 16 + lane] = db1;
  __syncthreads();
  if (threadIdx.x < 16) {
    const int t = threadIdx.x;
    float s1 = 0.f;
    for (int w = 0; w < 8; w++) s1 += red[w * 16 + t];
    out[C1 * 256 + C2 * 256 + t] = s1;
  }
  __syncthreads();
  // db2: thread t holds co2 = 8(t&3)+j; 64 threads share each (t&3)
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
    const int co = threadIdx.x;  // = 8*(lane&3) + j
    const int q4 = co >> 3, j = co & 7;
    float s = 0.f;
    for (int w = 0; w < 8; w++) s += red[w * 64 + q4 * 8 + j];
    out[C1 * 256 + C2 * 256 + C1 + co] = s;
  }
}

// Sum the G partials in a fixed order and write bf16 grads in each parameter's memory order.
// Workgroup = 64 consecutive outputs x 8 slices of G; a slice's loads (G / 8 = 32 at G = 256) are
// ALL issued before the first add: the partials were just written and sit in the MALL / L2, so the
// cost is round trips, not bytes (a 4-load loop paid ~8 of them; float4 columns over 49 workgroups
// measured slower: 6.3 vs 4.9 µs). The 8 slice sums are combined in LDS in a fixed order →
// deterministic.
constexpr int RED_SLICES = 8, RED_BATCH = 32;
__device__ __forceinline__ unsigned short* trunk_grad_dst(int e, unsigned short* dW1, WStrides w1, unsigned short* db1,
                                                          unsigned short* dW2, WStrides w2, unsigned short* db2) {
  if (e < C1 * 256) {  // k = (ky, kx, ci)
    const int co = e >> 8, k = e & 255, ky = k >> 5, kx = (k >> 2) & 7, ci = k & 3;
    return &dW1[co * w1.s0 + ci * w1.s1 + ky * w1.s2 + kx * w1.s3];
  }
  if (e < C1 * 256 + C2 * 256) {  // k = (ky, kx, ci)
    const int f = e - C1 * 256, co = f >> 8, k = f & 255, ky = k >> 6, kx = (k >> 4) & 3, ci = k & 15;
    return &dW2[co * w2.s0 + ci * w2.s1 + ky * w2.s2 + kx * w2.s3];
  }
  if (e < C1 * 256 + C2 * 256 + C1) return &db1[e - C1 * 256 - C2 * 256];
  return &db2[e - C1 * 256 - C2 * 256 - C1];
}
// one partial-sum workgroup of k_trunk_reduce: 64 consecutive outputs x RED_SLICES slices of G
__device__ __forceinline__ void trunk_reduce_block(const float* __restrict__ partial, int G, unsigned short* dW1,
                                                   WStrides w1, unsigned short* db1, unsigned short* dW2, WStrides w2,
                                                   unsigned short* db2, const FusedAdam& fa,
                                                   float (&red)[RED_SLICES][64]) {
  const int c = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + c;
  const bool owner = slice == 0 && e < PART;  // the thread that finishes output e
  unsigned short* dst = nullptr;
  AdamState st{0.f, 0.f, 0.f};
  if (owner) {
    dst = trunk_grad_dst(e, dW1, w1, db1, dW2, w2, db2);
    st = adam_prefetch(fa, dst);  // fused Adam: state loads fly during the partial sums
  }
  float s = 0.f;
  if (e < PART) {
    for (int g0 = slice; g0 < G; g0 += RED_SLICES * RED_BATCH) {
      float v[RED_BATCH];
#pragma unroll
      for (int j = 0; j < RED_BATCH; j++)  // clamped, unconditional: every load of the batch in flight
        v[j] = partial[int64_t(min(g0 + RED_SLICES * j, G - 1)) * PART + e];
#pragma unroll
      for (int j = 0; j < RED_BATCH; j++)
        if (g0 + RED_SLICES * j < G) s += v[j];
    }
  }
  red[slice][c] = s;
  __syncthreads();
  if (owner) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < RED_SLICES; k++) t += red[k][c];
    // the trunk gradients are final here: store them, or (FusedAdam) apply Adam to them
    const AdamCoef ac = fa.grad_base ? adam_coef(fa.hp, fa.step_ctr) : AdamCoef{};
    grad_store_pf(fa, ac, dst, t, st);
  }
}
__global__ __launch_bounds__(512) void k_trunk_reduce(const float* __restrict__ partial, int G,
                                                      unsigned short* __restrict__ dW1, WStrides w1,
                                                      unsigned short* __restrict__ db1,
                                                      unsigned short* __restrict__ dW2, WStrides w2,
                                                      unsigned short* __restrict__ db2, const FusedAdam fa,
                                                      const AdamTail at, int nred, const DenseFinalize df, int nfin) {
  __shared__ float red[RED_SLICES][64];
  if (int(blockIdx.x) >= nred + nfin) {  // Adam workgroups (AdamTail): K6's pass over the dense + heads range
    const AdamCoef ac = adam_coef(at.hp, at.step_ctr);
    const int64_t tid = int64_t(blockIdx.x - nred - nfin) * blockDim.x + threadIdx.x;
    const int64_t nthr = int64_t(gridDim.x - nred - nfin) * blockDim.x;
    if (at.part)  // deferred K12 finalize: gradients summed from the row-split partials
      adam_span_split<2>(at.master, at.m1, at.m2, at.part, at.rs, at.K, static_cast<__hip_bfloat16*>(at.wbf16),
                         at.grad_scale, ac, tid, nthr, at.n);
    else
      adam_span<__hip_bfloat16, true, 2>(at.master, at.m1, at.m2, static_cast<const __hip_bfloat16*>(at.grad),
                                         static_cast<__hip_bfloat16*>(at.wbf16), at.grad_scale, ac, tid, nthr, at.n);
  } else if (int(blockIdx.x) >= nred) {  // the deferred K12 row-split finalize, each element through FusedAdam
    const int j = int(blockIdx.x) - nred;
    const AdamCoef ac = adam_coef(fa.hp, fa.step_ctr);
    dense::split_finalize_elem(df.part, df.rs, df.K, df.A1, static_cast<unsigned short*>(df.dw),
                               static_cast<unsigned short*>(df.db), static_cast<unsigned short*>(df.dwh),
                               static_cast<unsigned short*>(df.dbh), df.group0 + j / dense::kK12PSlots,
                               j % dense::kK12PSlots, fa, ac);
  } else {
    trunk_reduce_block(partial, G, dW1, w1, db1, dW2, w2, db2, fa, red);
  }
  if (at.bump_next) {  // parity counters (see k_adam_flat): the next step reads the other copy
    if (blockIdx.x == 0 && threadIdx.x == 0)
      for (int k = 0; k < at.nbump; k++) at.bump_next[k] = at.bump[k] + 1;
    return;
  }
  // fused Adam: this launch is the last reader of the step counters in the SGD step
  last_block_bump(fa.bump, fa.nbump, fa.done);
}

}  // namespace trunk

static trunk::WStrides ws(const int64_t* s) { return trunk::WStrides{s[0], s[1], s[2], s[3]}; }

void nature_trunk_fwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B,
                      const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                      const void* b2, void* h1, void* h2, hipStream_t stream, int dbg) {
  if (B <= 0) return;
  if (period <= 0) period = 1;
  hipLaunchKernelGGL(trunk::k_trunk_fwd, dim3(uint32_t(B)), dim3(trunk::NTF), 0, stream, obs, idx, ctr, period, B,
                     static_cast<const unsigned short*>(W1), ws(w1s), static_cast<const unsigned short*>(b1),
                     static_cast<const unsigned short*>(W2), ws(w2s), static_cast<const unsigned short*>(b2),
                     static_cast<unsigned short*>(h1), static_cast<unsigned short*>(h2), dbg, nullptr, nullptr,
                     nullptr, nullptr);
  RMM_HIP_CHECK(hipGetLastError());
}

void nature_trunk_fwd_push_rows(uint8_t* rows, int64_t T, const uint8_t* new_frames, const int64_t* t_ptr, int64_t B,
                                const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                                const void* b2, void* h2, hipStream_t stream) {
  if (B <= 0) return;
  if (rows == nullptr || new_frames == nullptr || t_ptr == nullptr || T < 1)
    throw std::invalid_argument("nature_trunk_fwd_push_rows: rollout rows, T, new frames and the row counter");
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(new_frames)) & 3)
    throw std::invalid_argument("nature_trunk_fwd_push_rows: buffers must be 4-byte aligned");
  hipLaunchKernelGGL(trunk::k_trunk_fwd_band, dim3(uint32_t(B * trunk::NBAND)), dim3(trunk::NTFB), 0, stream,
                     static_cast<const unsigned short*>(W1), ws(w1s), static_cast<const unsigned short*>(b1),
                     static_cast<const unsigned short*>(W2), ws(w2s), static_cast<const unsigned short*>(b2),
                     static_cast<unsigned short*>(h2), B, rows, T, new_frames, t_ptr);
  RMM_HIP_CHECK(hipGetLastError());
}

void nature_trunk_fwd_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* rows, const int64_t* t_ptr, int64_t B,
                           const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                           const void* b2, void* h2, hipStream_t stream) {
  if (B <= 0) return;
  if (stack == nullptr || new_frames == nullptr) throw std::invalid_argument("nature_trunk_fwd_push: stack and new frames");
  if (rows != nullptr && t_ptr == nullptr) throw std::invalid_argument("nature_trunk_fwd_push: rows need the row counter");
  if ((reinterpret_cast<uintptr_t>(stack) | reinterpret_cast<uintptr_t>(new_frames) |
       reinterpret_cast<uintptr_t>(rows)) & 3)
    throw std::invalid_argument("nature_trunk_fwd_push: buffers must be 4-byte aligned");
  hipLaunchKernelGGL(trunk::k_trunk_fwd, dim3(uint32_t(B)), dim3(trunk::NTF), 0, stream, nullptr, nullptr, nullptr,
                     int64_t(1), B, static_cast<const unsigned short*>(W1), ws(w1s),
                     static_cast<const unsigned short*>(b1), static_cast<const unsigned short*>(W2), ws(w2s),
                     static_cast<const unsigned short*>(b2), nullptr, static_cast<unsigned short*>(h2), 0, stack,
                     new_frames, rows, t_ptr);
  RMM_HIP_CHECK(hipGetLastError());
}

int nature_trunk_bwd_groups(int64_t B) { return int(std::max<int64_t>(1, std::min<int64_t>(B, 256))); }
int64_t nature_trunk_partial_floats(int64_t B) { return int64_t(nature_trunk_bwd_groups(B)) * trunk::PART; }

void nature_trunk_bwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B,
                      const void* W2, const int64_t* w2s, const void* h1, const void* h2, const void* dh2,
                      float* partial, void* dW1, const int64_t* w1s, void* db1, void* dW2, void* db2,
                      hipStream_t stream, int dbg, const FusedAdam& fa, const AdamTail& at,
                      const DenseFinalize& df) {
  if (B <= 0) return;
  if (period <= 0) period = 1;
  if (at.master) {
    auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
    if (!(al(at.master, 16) && al(at.m1, 16) && al(at.m2, 16) && (at.part || al(at.grad, 8)) && al(at.wbf16, 8)) ||
        at.n <= 0 || (at.part && (at.rs < 1 || at.K % 32 != 0 || at.n != 256 * at.K || !al(at.part, 16))) ||
        !fa.grad_base || !at.hp || !at.step_ctr || (at.bump_next && (!at.bump || at.nbump <= 0)))
      throw std::invalid_argument("nature_trunk_bwd: Adam tail needs aligned buffers, the trunk FusedAdam and counters");
  }
  if (at.bump_next && (!at.bump || at.nbump <= 0))
    throw std::invalid_argument("nature_trunk_bwd: parity counters need bump / nbump");
  const int G = nature_trunk_bwd_groups(B);
  hipLaunchKernelGGL(trunk::k_trunk_bwd, dim3(uint32_t(G)), dim3(trunk::NTB), 0, stream, obs, idx, ctr, period, B,
                     static_cast<const unsigned short*>(W2), ws(w2s), static_cast<const unsigned short*>(h1),
                     static_cast<const unsigned short*>(h2), static_cast<const unsigned short*>(dh2), partial, dbg);
  RMM_HIP_CHECK(hipGetLastError());
  if (dbg & 128) return;  // profiling: the backward kernel alone
  if (df.part && (!fa.grad_base || df.rs < 1 || df.groups < 1 || !df.dw || !df.db || !df.dwh || !df.dbh))
    throw std::invalid_argument("nature_trunk_bwd: the deferred K12 finalize needs FusedAdam and all four gradients");
  const int nred = (trunk::PART + 63) / 64, NTR = 64 * trunk::RED_SLICES;
  static_assert(64 * trunk::RED_SLICES == dense::kK12NT, "finalize workgroups are K12-sized");
  const int nfin = df.part ? (df.groups - df.group0) * dense::kK12PSlots : 0;
  // Adam workgroups: two groups of 4 elements per lane (K6's default unroll)
  const int nadam = at.master ? int(std::max<int64_t>(1, ((at.n + 3) / 4 + 2 * NTR - 1) / (2 * NTR))) : 0;
  hipLaunchKernelGGL(trunk::k_trunk_reduce, dim3(nred + nfin + nadam), dim3(NTR), 0, stream, partial, G,
                     static_cast<unsigned short*>(dW1), ws(w1s), static_cast<unsigned short*>(db1),
                     static_cast<unsigned short*>(dW2), ws(w2s), static_cast<unsigned short*>(db2), fa, at, nred, df,
                     nfin);
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
