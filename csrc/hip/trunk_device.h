// Device helpers of the K10 Nature-CNN trunk kernels (conv_kernels.hip), shared with the persistent
// rollout-server kernel (rollout_server.hip): geometry, frame staging (u8 NCHW -> padded HWC LDS
// image), weight staging, and the conv1 -> conv2 MFMA body of one frame held in LDS.
#pragma once
#include <hip/hip_bf16.h>

#include "common.h"

namespace rmm {
namespace hip {
namespace trunk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C0 = 4, H0 = 84, P0 = 88;            // frame, padded by 2 each side
constexpr int H1 = 21, C1 = 16, NP1 = 441, NP1P = 448;
constexpr int P1 = 25;                              // h1 padded by 2 each side
constexpr int H2 = 11, C2 = 32, NP2 = 121, NP2P = 128;
constexpr int FRAME_BYTES = C0 * P0 * P0;          // 30976
constexpr int H1P_ELEMS = P1 * P1 * C1;            // 10000 bf16

__device__ __forceinline__ unsigned short f2bf(float f) {  // round-to-nearest-even
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<unsigned short>(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ __forceinline__ unsigned short u8bf(uint32_t b) { return static_cast<unsigned short>(__float_as_uint(float(b)) >> 16); }

__device__ __forceinline__ bf16x8 as_bf(u16x8 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct WStrides { int64_t s0, s1, s2, s3; };  // [co][ci][ky][kx] element strides

__device__ __forceinline__ const int64_t* window(const int64_t* idx, const int64_t* ctr, int64_t period, int64_t rows) {
  return (ctr && idx) ? idx + (ctr[0] % period) * rows : idx;
}

// Copy one u8 frame [4][84][84] (NCHW) into the padded HWC LDS image: pixel (y, x) channel c at
// byte ((y+2)*88 + x+2)*4 + c. A thread takes the same 4-pixel word from the 4 channel planes
// (4 coalesced u32 loads), transposes the 4x4 bytes in registers and writes 16 B of HWC pixels.
// All of a thread's loads are issued before any LDS write (28 in flight): a load→store per
// iteration would serialise ~28 HBM round trips per frame. NT = blockDim.
template <int NT>
__device__ __forceinline__ void load_frame(const uint8_t* __restrict__ src, uint8_t* frame) {
  constexpr int NW = H0 * H0 / 4, PER = (NW + NT - 1) / NT;  // 1764 words per plane
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
  uint32_t v[PER][C0];
  // unconditional loads at a clamped index: a guarded load inside an unrolled batch makes hipcc
  // branch around each one and wait vmcnt(0) per load (an HBM round trip each)
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = min(int(threadIdx.x) + NT * k, NW - 1);
#pragma unroll
    for (int c = 0; c < C0; c++) v[k][c] = s32[c * NW + o];
  }
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
      const int y = o / 21, x = 4 * (o - y * 21);
      uint32_t px[4];
#pragma unroll
      for (int q = 0; q < 4; q++)  // pixel q: bytes (c0, c1, c2, c3) = byte q of each plane word
        px[q] = ((v[k][0] >> (8 * q)) & 0xffu) | (((v[k][1] >> (8 * q)) & 0xffu) << 8) |
                (((v[k][2] >> (8 * q)) & 0xffu) << 16) | (((v[k][3] >> (8 * q)) & 0xffu) << 24);
      uint2* d = reinterpret_cast<uint2*>(frame + ((y + 2) * P0 + x + 2) * 4);  // 8-B aligned
      d[0] = make_uint2(px[0], px[1]);
      d[1] = make_uint2(px[2], px[3]);
    }
  }
}

// load_frame split in two so the HBM frame loads can be issued before the weight staging and the
// LDS zeroing (they are independent): frame_issue starts the loads, frame_store transposes and writes
// the interior; only the 2-pixel border needs zeros (zero_frame_border), so no barrier separates
// zeroing from the interior stores.
template <int NT>
struct FrameRegs {
  static constexpr int NW = H0 * H0 / 4, PER = (NW + NT - 1) / NT;
  uint32_t v[PER][C0];
};
template <int NT>
__device__ __forceinline__ void frame_issue(const uint8_t* __restrict__ src, FrameRegs<NT>& f) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = min(int(threadIdx.x) + NT * k, NW - 1);
#pragma unroll
    for (int c = 0; c < C0; c++) f.v[k][c] = s32[c * NW + o];
  }
}
template <int NT>
__device__ __forceinline__ void frame_store(const FrameRegs<NT>& f, uint8_t* frame) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
      const int y = o / 21, x = 4 * (o - y * 21);
      uint32_t px[4];
#pragma unroll
      for (int q = 0; q < 4; q++)
        px[q] = ((f.v[k][0] >> (8 * q)) & 0xffu) | (((f.v[k][1] >> (8 * q)) & 0xffu) << 8) |
                (((f.v[k][2] >> (8 * q)) & 0xffu) << 16) | (((f.v[k][3] >> (8 * q)) & 0xffu) << 24);
      uint2* d = reinterpret_cast<uint2*>(frame + ((y + 2) * P0 + x + 2) * 4);
      d[0] = make_uint2(px[0], px[1]);
      d[1] = make_uint2(px[2], px[3]);
    }
  }
}
// Rollout push mode (K19 folded into the trunk): the frame to run is the env's device stack
// shifted by one with the newest frame appended. The thread that loads word o of planes 1..3 of
// the stack and of the new frame also writes word o of the 4 shifted planes back (stack, in place:
// no other thread touches word o of this env) and into rollout row t — so the rollout step needs
// no separate frame-push launch. `nf` may be device-mapped pinned host memory (zero-copy upload).
template <int NT>
__device__ __forceinline__ void frame_issue_push(const uint8_t* stack, const uint8_t* __restrict__ nf,
                                                 FrameRegs<NT>& f) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(stack);
  const uint32_t* n32 = reinterpret_cast<const uint32_t*>(nf);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = min(int(threadIdx.x) + NT * k, NW - 1);
#pragma unroll
    for (int c = 0; c < C0 - 1; c++) f.v[k][c] = s32[(c + 1) * NW + o];
    f.v[k][C0 - 1] = n32[o];
  }
}
template <int NT>
__device__ __forceinline__ void frame_push_store(const FrameRegs<NT>& f, uint8_t* stack, uint8_t* row) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
  uint32_t* s32 = reinterpret_cast<uint32_t*>(stack);
  uint32_t* r32 = reinterpret_cast<uint32_t*>(row);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
#pragma unroll
      for (int c = 0; c < C0; c++) {
        s32[c * NW + o] = f.v[k][c];
        if (row) r32[c * NW + o] = f.v[k][c];
      }
    }
  }
}

// zero rows 0, 1, 86, 87 and columns 0, 1, 86, 87 of the padded HWC frame (one u32 = one pixel)
__device__ __forceinline__ void zero_frame_border(uint8_t* frame) {
  uint32_t* f32 = reinterpret_cast<uint32_t*>(frame);
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
    f32[y * P0 + x] = 0u;
  }
}

// Backward variant: the padded frame in space-to-depth form, transposed, bf16 (exact for 0..255):
// padded pixel (yp, xp) = (y+2, x+2) = (4Y+ry, 4X+rx), channel ci → st[c][Y*ST_W + X] with
// c = 16ry + 4rx + ci. conv1 (8x8/4) is then a 2x2 stride-1 correlation over a 64-channel 22x22
// grid: ky = 4a+ry, kx = 4b+rx, input (Y, X) = (oy+a, ox+b). Its weight gradient reduces over
// grid positions, which are CONTIGUOUS per channel here (one 16-B LDS read per MFMA operand
// instead of 8 strided 2-B gathers). Row pitch ST_W = 24 (3 chunks of 8), 23 rows (row 22 and
// columns 22, 23 stay zero: K padding), channel pitch 552 el = 276 dwords (8 lanes reading 8
// channels hit distinct 4-bank groups). The four 16-channel blocks (ry = yp & 3) are ST_BP = 32 el
// apart beyond that: a wave's staging stores span ~3 frame rows, i.e. 3 blocks, whose stride 16 x 276
// dwords is 0 mod 64 banks — without the pad those rows' stores met on the same banks.
constexpr int ST_W = 24, ST_CP = 23 * ST_W, ST_C = 64, ST_BP = 32;
constexpr int ST_ELEMS = ST_C * ST_CP + (ST_C / 16) * ST_BP;
__device__ __forceinline__ int st_chan(int c) { return c * ST_CP + (c >> 4) * ST_BP; }  // channel c's base
template <int NT>
__device__ __forceinline__ void frame_store_s2d(const FrameRegs<NT>& f, unsigned short* st) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
      const int y = o / 21, xw = o - y * 21;  // pixels x = 4xw .. 4xw+3 → xp = 4xw+2 .. 4xw+5
      const int yp = y + 2;
      unsigned short* row = st + st_chan(16 * (yp & 3)) + (yp >> 2) * ST_W + xw;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int rx = (q + 2) & 3, dX = (q + 2) >> 2;
#pragma unroll
        for (int c = 0; c < C0; c++) row[(4 * rx + c) * ST_CP + dX] = u8bf((f.v[k][c] >> (8 * q)) & 0xffu);
      }
    }
  }
}
template <int NT>
__device__ __forceinline__ void load_frame_s2d(const uint8_t* __restrict__ src, unsigned short* st) {
  constexpr int NW = H0 * H0 / 4, PER = (NW + NT - 1) / NT;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
  uint32_t v[PER][C0];
  // unconditional loads at a clamped index: a guarded load inside an unrolled batch makes hipcc
  // branch around each one and wait vmcnt(0) per load (an HBM round trip each)
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = min(int(threadIdx.x) + NT * k, NW - 1);
#pragma unroll
    for (int c = 0; c < C0; c++) v[k][c] = s32[c * NW + o];
  }
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    if (o < NW) {
      const int y = o / 21, xw = o - y * 21;  // pixels x = 4xw .. 4xw+3 → xp = 4xw+2 .. 4xw+5
      const int yp = y + 2;
      unsigned short* row = st + st_chan(16 * (yp & 3)) + (yp >> 2) * ST_W + xw;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int rx = (q + 2) & 3, dX = (q + 2) >> 2;  // compile-time after unrolling
#pragma unroll
        for (int c = 0; c < C0; c++) row[(4 * rx + c) * ST_CP + dX] = u8bf((v[k][c] >> (8 * q)) & 0xffu);
      }
    }
  }
}

// Stage a conv weight into LDS as canonical [co][ky][kx][ci] rows of `pitch` elements (row = co).
// Every workgroup needs the whole (tiny) weight: per-lane fragment loads straight from global make
// all workgroups hammer the same few L2 lines (measured: skeleton cost grew 7→20-30 µs from 1 to
// 256 workgroups). Here each element is read once per workgroup, 16 B at a time when the weight
// is channels-last contiguous ([co][ky][kx][ci] in memory).
// Split in issue / store: all of a lane's 16-B loads go out at once (a load→store loop waits one L2
// round trip per trip: the bwd kernel's prologue paid 2, the fwd's 3, ~1 µs each) and the kernels
// issue them FIRST, so the round trip hides behind the frame issue and the LDS zeroing.
template <int NT, int CO, int CI, int KH>
struct WeightRegs {
  static constexpr int ROW = KH * KH * CI, N = CO * ROW / 8, PER = (N + NT - 1) / NT;
  u16x8 v[PER];
  bool fast;  // channels-last contiguous: 16-B copies; otherwise weight_store gathers elements
};
template <int NT, int CO, int CI, int KH>
__device__ __forceinline__ void weight_issue(const unsigned short* __restrict__ W, WStrides ws_,
                                             WeightRegs<NT, CO, CI, KH>& r) {
  using R = WeightRegs<NT, CO, CI, KH>;
  r.fast = ws_.s1 == 1 && ws_.s3 == CI && ws_.s2 == KH * CI && ws_.s0 == R::ROW;
  if (!r.fast) return;
#pragma unroll
  for (int k = 0; k < R::PER; k++)
    r.v[k] = *reinterpret_cast<const u16x8*>(&W[8 * min(int(threadIdx.x) + NT * k, R::N - 1)]);
}
template <int NT, int CO, int CI, int KH>
__device__ __forceinline__ void weight_store(const WeightRegs<NT, CO, CI, KH>& r, const unsigned short* __restrict__ W,
                                             WStrides ws_, unsigned short* dst, int pitch) {
  using R = WeightRegs<NT, CO, CI, KH>;
  constexpr int ROW = R::ROW;
  if (r.fast) {
#pragma unroll
    for (int k = 0; k < R::PER; k++) {
      const int v = threadIdx.x + NT * k;
      if (v < R::N) {
        const int co = (8 * v) / ROW, e = 8 * v - co * ROW;
        *reinterpret_cast<u16x8*>(&dst[co * pitch + e]) = r.v[k];
      }
    }
  } else {
    for (int v = threadIdx.x; v < CO * ROW; v += NT) {
      const int co = v / ROW, e = v - co * ROW, ky = e / (KH * CI), kx = (e / CI) % KH, ci = e % CI;
      dst[co * pitch + e] = W[co * ws_.s0 + ci * ws_.s1 + ky * ws_.s2 + kx * ws_.s3];
    }
  }
}
template <int NT, int CO, int CI, int KH>
__device__ __forceinline__ void stage_weight(const unsigned short* __restrict__ W, WStrides ws_, unsigned short* dst,
                                             int pitch) {
  WeightRegs<NT, CO, CI, KH> r;
  weight_issue(W, ws_, r);
  weight_store(r, W, ws_, dst, pitch);
}
constexpr int W1_PITCH = 256 + 8, W2_PITCH = 256 + 8;  // +16 B: 16 lanes x 16-B reads hit distinct banks

__device__ __forceinline__ void zero_lds(void* p, int bytes) {
  uint4* q = reinterpret_cast<uint4*>(p);
  for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) q[i] = make_uint4(0, 0, 0, 0);
}

// 8 consecutive bytes of the HWC frame (8-byte aligned: 2 pixels x 4 channels) → bf16x8
__device__ __forceinline__ bf16x8 frame8(const uint8_t* frame, int off) {
  const uint2 w = *reinterpret_cast<const uint2*>(frame + off);
  const uint32_t a = w.x, b = w.y;
  u16x8 v;
  v[0] = u8bf(a & 0xff); v[1] = u8bf((a >> 8) & 0xff); v[2] = u8bf((a >> 16) & 0xff); v[3] = u8bf(a >> 24);
  v[4] = u8bf(b & 0xff); v[5] = u8bf((b >> 8) & 0xff); v[6] = u8bf((b >> 16) & 0xff); v[7] = u8bf(b >> 24);
  return as_bf(v);
}


// Weight-grad GEMMs reduce over positions (MFMA K). Lane group g's 8 K values are taken as
// positions 32s + g + 4j (j = 0..7) so the four lane groups gather NEIGHBOURING pixels (distinct
// LDS banks; with 8g + j they sit 8 positions apart, on the same bank: 4-way conflicts). The
// transposed dpre tiles are stored in that permuted order so the A operand stays one 16-B read.
__device__ __forceinline__ int kperm(int p) { return (p & ~31) + 8 * (p & 3) + ((p & 31) >> 2); }

// ---- forward staging: the frame as bf16 in LDS, one HALF at a time
// conv1's im2col A operand is 8 consecutive bf16 (2 pixels x 4 channels) of the padded HWC image.
// Converting u8 → bf16 inside the conv1 loop redid every pixel ~4 times (the 8x8/4 windows overlap)
// and made conv1 VALU-bound; converting once needs a 62 KB bf16 image, which would leave ONE
// workgroup per CU. So the frame (already in registers, FrameRegs) is converted in two passes of
// 48 padded rows each: pass 0 holds padded rows 0..47 for conv1 positions 0..223 (M-tiles 0..13,
// output rows 0..10), pass 1 rows 40..87 for positions 224..440 (tiles 14..27). 33.8 KB of LDS
// (the u8 image was 31 KB): still two workgroups per CU. Identical bf16 inputs and MFMA order →
// bit-identical conv1 results.
constexpr int HF_ROWS = 48, HF_ELEMS = HF_ROWS * P0 * C0, HF_BASE1 = 40, HF_TILES = 14;
static_assert(HF_TILES * 16 == 224 && 4 * (224 / H1) >= HF_BASE1, "pass split at an M-tile boundary");

// zero the padding of the half image that no pass overwrites: columns 0, 1, 86, 87 of every row
// and rows 0, 1 (pass 0's top padding); pass 1 zeroes rows 46, 47 itself (its bottom padding)
__device__ __forceinline__ void zero_half_frame_border(unsigned short* fh) {
  uint2* f = reinterpret_cast<uint2*>(fh);  // one uint2 = one pixel (4 bf16)
  constexpr int NCOL = HF_ROWS * 4, NROW = 2 * P0;
  for (int i = threadIdx.x; i < NCOL + NROW; i += blockDim.x) {
    int y, x;
    if (i < NCOL) {
      const int c = i & 3;
      y = i >> 2;
      x = c < 2 ? c : c + (P0 - 4);
    } else {
      const int j = i - NCOL;
      y = j / P0;
      x = j - y * P0;
    }
    f[y * P0 + x] = make_uint2(0u, 0u);
  }
}

__device__ __forceinline__ uint32_t bf16pair(uint32_t lo_f32, uint32_t hi_f32) {
  return __builtin_amdgcn_perm(hi_f32, lo_f32, 0x07060302u);  // {hi[31:16], lo[31:16]}
}

// store the frame words of padded rows [base, base + 48) from registers as bf16 HWC
template <int NT>
__device__ __forceinline__ void half_frame_store(const FrameRegs<NT>& f, unsigned short* fh, int base) {
  constexpr int NW = FrameRegs<NT>::NW, PER = FrameRegs<NT>::PER;
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int o = threadIdx.x + NT * k;
    const int y = o / 21, xw = o - y * 21, yr = y + 2 - base;
    if (o < NW && yr >= 0 && yr < HF_ROWS) {
      uint32_t w[8];
#pragma unroll
      for (int q = 0; q < 4; q++) {  // pixel q: channel c = byte q of plane word c
        const uint32_t c0 = __float_as_uint(float((f.v[k][0] >> (8 * q)) & 0xffu));
        const uint32_t c1 = __float_as_uint(float((f.v[k][1] >> (8 * q)) & 0xffu));
        const uint32_t c2 = __float_as_uint(float((f.v[k][2] >> (8 * q)) & 0xffu));
        const uint32_t c3 = __float_as_uint(float((f.v[k][3] >> (8 * q)) & 0xffu));
        w[2 * q] = bf16pair(c0, c1);
        w[2 * q + 1] = bf16pair(c2, c3);
      }
      uint4* d = reinterpret_cast<uint4*>(fh + (yr * P0 + 4 * xw + 2) * C0);  // 16-B aligned
      d[0] = make_uint4(w[0], w[1], w[2], w[3]);
      d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
  }
}

// conv1 -> conv2 of ONE frame (`fr`: its words in registers; `fh`: the bf16 half-image LDS region,
// border zeroed by zero_half_frame_border; `h1p`: zeroed padded h1 tile; w1s / w2s: staged
// weights; the caller's barrier has made the border, h1p and the weights visible), NT threads.
// Writes h1 (for backward, when h1_out != nullptr) and h2 (NHWC flatten, 3872 bf16) of this
// frame. Ends after the h2 stores (no trailing barrier); `fh` is reused as the h2 staging tile.
// dbg bits: 1 / 2 skip the conv1 / conv2 MFMAs, 16 the h1 store, 32 the frame conversion, 64 the
// h2 store (profiling masks).
// The biases come in as registers (TrunkBias, loaded by the caller at kernel start with the frame:
// a bias load issued here would expose an L2 round trip right before the first epilogue).
struct TrunkBias {
  float b1, b2a, b2b;  // b1[r], b2[r], b2[16 + r] for this lane's r = lane & 15
};
__device__ __forceinline__ TrunkBias trunk_bias(const unsigned short* __restrict__ b1,
                                                const unsigned short* __restrict__ b2) {
  const int r = threadIdx.x & 15;
  return TrunkBias{bf2f(b1[r]), bf2f(b2[r]), bf2f(b2[16 + r])};
}

template <int NT>
__device__ __forceinline__ void trunk_convs(const FrameRegs<NT>& fr, unsigned short* fh, unsigned short* h1p,
                                            const unsigned short* w1s, const unsigned short* w2s, TrunkBias tb,
                                            unsigned short* __restrict__ h1_out, unsigned short* __restrict__ h2_out,
                                            int dbg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  bf16x8 wf1[8];
  const float bias1 = tb.b1;

  // ---- conv1 in two half-image passes of 14 M-tiles (16 positions each) over the waves
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    const int base = pass ? HF_BASE1 : 0;
    if (pass) {
      __syncthreads();  // pass 0's conv1 reads of the half image are done
      uint2* f = reinterpret_cast<uint2*>(fh);
      for (int i = threadIdx.x; i < 2 * P0; i += NT) f[(HF_ROWS - 2) * P0 + i] = make_uint2(0u, 0u);  // rows 86, 87
    }
    if (!(dbg & 32)) half_frame_store<NT>(fr, fh, base);
    __syncthreads();
    if (pass == 0) {
      // conv1 weight fragments, k = (ky, kx, ci): k-step s = ky, lane group g → kx ∈ {2g, 2g+1},
      // j → (kx = 2g + (j>>2), ci = j&3); col = co = r: one 16-B LDS read each. Read AFTER the
      // barrier: w1s is staged by every thread of the workgroup (a read before it raced with
      // slower waves' stores — wrong conv1 weights for a frame, seen with two workgroups per CU)
#pragma unroll
      for (int s = 0; s < 8; s++)
        wf1[s] = as_bf(*reinterpret_cast<const u16x8*>(&w1s[r * W1_PITCH + (s * 8 + 2 * g) * 4]));
    }
    for (int mt = pass * HF_TILES + wave; mt < (pass + 1) * HF_TILES; mt += NT / 64) {
      const int p = min(mt * 16 + r, NP1 - 1);
      const int oy = p / H1, ox = p - oy * H1;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (!(dbg & 1)) {
#pragma unroll
        for (int s = 0; s < 8; s++)
          acc = mfma(as_bf(*reinterpret_cast<const u16x8*>(&fh[((4 * oy + s - base) * P0 + 4 * ox + 2 * g) * C0])),
                     wf1[s], acc);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int q = mt * 16 + 4 * g + i;
        if (q < NP1) {
          const float v = fmaxf(acc[i] * (1.0f / 255.0f) + bias1, 0.f);
          const int y = q / H1, x = q - y * H1;
          h1p[((y + 2) * P1 + (x + 2)) * C1 + r] = f2bf(v);
        }
      }
    }
  }
  // conv2 weight fragments (two 16-wide N tiles): k = 32s + 8g + j → pixel pp = 2s + (g>>1)
  // (ky = pp>>2, kx = pp&3), ci = 8(g&1) + j
  bf16x8 wf2[2][8];
#pragma unroll
  for (int nt = 0; nt < 2; nt++)
#pragma unroll
    for (int s = 0; s < 8; s++) {  // pixel pp = (ky, kx) → canonical offset pp*16 + ci
      const int pp = 2 * s + (g >> 1), co = nt * 16 + r;
      wf2[nt][s] = as_bf(*reinterpret_cast<const u16x8*>(&w2s[co * W2_PITCH + pp * 16 + 8 * (g & 1)]));
    }
  const float bias2[2] = {tb.b2a, tb.b2b};
  __syncthreads();
  // h1 out for backward: coalesced 16-B rows from the LDS tile
  if (h1_out && !(dbg & 16)) {
    for (int v = threadIdx.x; v < NP1 * 2; v += NT) {
      const int p = v >> 1, y = p / H1, x = p - y * H1;
      *reinterpret_cast<uint4*>(&h1_out[p * C1 + 8 * (v & 1)]) =
          *reinterpret_cast<const uint4*>(&h1p[((y + 2) * P1 + (x + 2)) * C1 + 8 * (v & 1)]);
    }
  }
  unsigned short* h2s = fh;  // the half image is dead after conv1

  // ---- conv2: 8 M-tiles x 2 N-tiles
  for (int mt = wave; mt < NP2P / 16; mt += NT / 64) {
    const int q = min(mt * 16 + r, NP2 - 1);
    const int oy = q / H2, ox = q - oy * H2;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (!(dbg & 2)) {
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int pp = 2 * s + (g >> 1), ky = pp >> 2, kx = pp & 3;
        const u16x8 av =
            *reinterpret_cast<const u16x8*>(&h1p[((2 * oy + ky) * P1 + (2 * ox + kx)) * C1 + 8 * (g & 1)]);
        const bf16x8 a = as_bf(av);
        acc0 = mfma(a, wf2[0][s], acc0);
        acc1 = mfma(a, wf2[1][s], acc1);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int qq = mt * 16 + 4 * g + i;
      if (qq < NP2) {
        h2s[qq * C2 + r] = f2bf(fmaxf(acc0[i] + bias2[0], 0.f));
        h2s[qq * C2 + 16 + r] = f2bf(fmaxf(acc1[i] + bias2[1], 0.f));
      }
    }
  }
  __syncthreads();
  if (dbg & 64) return;
  for (int v = threadIdx.x; v < NP2 * C2 / 8; v += NT)
    *reinterpret_cast<uint4*>(&h2_out[8 * v]) = *reinterpret_cast<const uint4*>(&h2s[8 * v]);
}

}  // namespace trunk
}  // namespace hip
}  // namespace rmm
