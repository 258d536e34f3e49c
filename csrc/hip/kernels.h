// Host launchers for the CDNA4 kernels (all asynchronous on the given stream unless noted).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

namespace rmm {
namespace hip {

struct CopySeg {
  uint64_t src;
  uint64_t dst;
  uint64_t nbytes;
};

// K1/K2: one launch copies many (src,dst,n) segments — tensor pack/unpack for
// serialization, sample-batch concat. Any alignment; 16 B/lane vector path when possible.
void multi_copy(const std::vector<CopySeg>& segs, hipStream_t stream);

// K2: out[i,:] = in[idx[i],:] for `rows` rows of `row_bytes` bytes (minibatch gather).
void gather_rows(const void* in, const int64_t* idx, void* out, int64_t rows, int64_t row_bytes,
                 hipStream_t stream, const int64_t* ctr = nullptr, int64_t period = 1);

// K2b: uint8 NCHW frames (optionally gathered by idx) -> scaled bf16 NHWC (conv input).
void frames_to_nhwc_bf16(const uint8_t* src, const int64_t* idx, void* dst, int64_t B, int64_t C, int64_t H,
                         int64_t W, float scale, hipStream_t stream, const int64_t* ctr = nullptr,
                         int64_t period = 1);
// fp32 output twin of K2b (precision-matched learner)
void frames_to_nhwc_f32(const uint8_t* src, const int64_t* idx, float* dst, int64_t B, int64_t C, int64_t H,
                        int64_t W, float scale, hipStream_t stream, const int64_t* ctr = nullptr, int64_t period = 1);

// K3: GAE over time-major [T,B] fp32 tensors. dones is fp32 0/1 (1 = episode ended after t).
// adv[t] = delta[t] + gamma*lam*(1-d[t])*adv[t+1];  ret = adv + values.
void gae(const float* rewards, const float* values, const float* dones, const float* last_values,
         float* adv, float* ret, int64_t T, int64_t B, float gamma, float lam, hipStream_t stream);

// K4: lossless block compression for the spill path.
// elem_bits = 16 (bf16/fp16) or 32 (fp32). Returns the upper bound of the compressed stream.
uint64_t compress_bound(uint64_t n_elems, int elem_bits);
// Workspace bytes needed by compress/decompress.
uint64_t compress_workspace(uint64_t n_elems);
// Compress `n_elems` elements at `src` into `dst` (device, >= compress_bound bytes).
// Synchronises the stream once to read back the total; returns compressed byte count. readback = false:
// no synchronisation, returns 0 (the size stays in the stream's header on the device).
uint64_t compress(const void* src, uint64_t n_elems, int elem_bits, void* dst, void* workspace,
                  hipStream_t stream, bool readback = true);
// Device-placed spill chunk: a copy kernel writes chunk bytes into the host arena's device mapping at
// host_dev + *base_dev (compressed from `scratch` when try_compressed and it saves >= len / 16, else `raw`),
// then *csize_dev = compressed bytes or 0 and *base_dev advances by the bytes rounded up to 64.
void spill_commit(const void* scratch, const void* raw, uint64_t len, bool try_compressed, void* host_dev,
                  uint64_t* base_dev, uint64_t* csize_dev, hipStream_t stream);
// Inverse of compress(); `src` is the device copy of the compressed stream.
void decompress(const void* src, void* dst, uint64_t n_elems, int elem_bits, void* workspace,
                hipStream_t stream);

// Exclusive scan of u16 -> u64 with total written to out[n] (device); helper exposed for tests.
void scan_u16(const uint16_t* in, uint64_t* out, uint64_t n, void* workspace, hipStream_t stream);

// K5: fused PPO surrogate loss pieces (ratio/clip/value/entropy reductions) — see kernels.hip.
void ppo_loss_fwd(const float* logp_new, const float* logp_old, const float* adv,
                  const float* v_new, const float* v_old, const float* v_tgt, const float* ent,
                  float* grad_logp, float* grad_v, float* grad_ent, float* stats, int64_t n,
                  float clip, float vf_clip, float vf_coeff, float ent_coeff, hipStream_t stream);

// K5b: whole categorical PPO loss head (fwd: stats; bwd: d/dlogits, d/dvalues scaled by *gout).
void ppo_cat_loss(bool fwd, const void* logits, bool logits_bf16, const float* old_logits, const int64_t* actions,
                  const float* old_logp, const float* adv, const void* values, bool values_bf16, const float* vtgt,
                  const float* coef, float* stats, const float* gout, void* g_logits, void* g_values, int64_t N,
                  int A, hipStream_t stream);

// K6: flat Adam/AdamW with fp32 master weights, bf16 or fp32 grads, optional bf16 weight output.
void adam_flat(float* master, float* m1, float* m2, const void* grad, bool grad_bf16, void* wbf16, const float* hp,
               float grad_scale, int64_t n, hipStream_t stream, const int64_t* step_ctr = nullptr,
               int64_t* bump = nullptr, int nbump = 0, uint32_t* done = nullptr, const float* scale_ptr = nullptr, int max_blocks = 0,
               int64_t* bump_next = nullptr, void* wlo = nullptr);  // wlo: split-pair lo plane (wbf16 = hi)
// K6b: out[0] = min(1, max_norm / ||grad*grad_scale||), out[1] = the norm (device; feeds K6 scale_ptr).
// workspace: grad_clip_workspace_floats() floats, zero-initialised once (its ticket resets itself).
int64_t grad_clip_workspace_floats();
void grad_clip_coef(const void* grad, bool grad_bf16, int64_t n, float grad_scale, float max_norm, float* workspace,
                    float* out, hipStream_t stream);

// K5c: merged policy/value head PPO loss reading packed columns (see rl_kernels.hip).
void ppo_heads_loss(bool bwd, const void* heads, const float* cols, const float* coef, float* acc, const float* gout,
                    void* g_heads, int64_t N, int A, hipStream_t stream);

// K7: Gumbel-max categorical sampling + rollout buffer writes at device-side row *t_ptr.
void sample_store(const void* logits, bool logits_bf16, const void* values, bool values_bf16, const int64_t* t_ptr,
                  const int64_t* ctr, uint32_t seed, int64_t* act, float* logp, float* vf, float* lout,
                  int64_t* act_now, int64_t B, int A, hipStream_t stream, int64_t ldl = 0, int64_t ldv = 0);

// K9: synthetic 84x84x4 Atari vector-env step fused with the rollout-buffer writes.
// ctr_t = device int64[2] {rng counter, rollout row}.
// K19: shift a device frame stack [B,4,hw] by one frame, append new_frames [B,hw], store row *t_ptr of buf_obs
// rollout step gate: wait (bounded) until *host_release >= *dev_seq + 1, then *dev_seq += 1
void step_gate(const int64_t* host_release, int64_t* dev_seq, int64_t max_polls, int* err, hipStream_t stream);
void frame_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* buf_obs, const int64_t* t_ptr, int64_t B,
                int64_t hw, hipStream_t stream);
void synth_env_step(uint8_t* frames, const uint8_t* pool, const int64_t* actions, int32_t* tenv, const int64_t* ctr_t,
                    uint8_t* buf_obs, float* buf_rew, float* buf_done, uint32_t seed, int episode_len, int64_t B,
                    hipStream_t stream, int64_t* bump = nullptr, uint32_t* done = nullptr);
// bump/done (optional, K6 and K9): the kernel's last workgroup adds 1 to bump[0..n) after every
// workgroup has read its counters (replaces a separate counter-increment launch per step).
// done: a zero-initialised device buffer of bump_done_words() u32 per call site.
int bump_done_words();

// K8: conv epilogue for NHWC bf16 maps [M, C]: y = relu(y + b) in place; backward dpre = dy*(y>0)
// and db = column sums of dpre (two-pass, deterministic; `partial` holds bias_relu_bwd_partials(M)*C f32).
void bias_relu_fwd(void* y, const void* bias, int64_t M, int C, bool relu, hipStream_t stream);
int64_t bias_relu_bwd_partials(int64_t M);
void bias_relu_bwd(const void* dy, const void* y, void* dpre, void* dbias_bf16, float* partial, int64_t M, int C,
                   bool relu, hipStream_t stream);

// K8b: dpre = dy*[y>0] (relu) or dy, and bf16 column sums db, one launch (dense layers, small M).
// dpre may be null (bias grad only). y is read only when relu.
void mask_colsum(const void* dy, const void* y, void* dpre, void* db, int64_t M, int C, bool relu,
                 hipStream_t stream);

// K12: fused backward of hidden = ReLU(x Wᵀ + b) [M,256] -> heads = hidden Whᵀ + bh [M,A1] given
// dheads: dx [M,K], dW [256,K], db [256], dWh [A1,256], dbh [A1] (all bf16, row-major), one launch.
// K % 32 == 0, A1 <= 16, M <= 640 (a PPO minibatch; larger batches take the hipBLASLt path).
void dense_heads_bwd(const void* dz, int A1, const void* wh, const void* y, const void* x, const void* w, int64_t M,
                     int64_t K, void* dx, void* dw, void* db, void* dwh, void* dbh, void* dpre_scratch,
                     hipStream_t stream, bool dpre_ready = false,
                     const FusedAdam& fa = FusedAdam{}, bool defer_finalize = false, int split = -1);  // dpre_scratch: M*256 bf16; fa: Adam epilogue
// K12 row split (RMM_K12_SPLIT=rs): the partial workspace [groups][rs][20][512] fp32 of a deferred finalize
struct DenseSplitPlan {
  float* part = nullptr;
  int rs = 1, groups = 0;
};
DenseSplitPlan dense_split_plan(int64_t M, int64_t K, int split, hipStream_t stream);
// The deferred K12 finalize run by the K10 trunk-reduce launch (with its FusedAdam): destinations are the
// dense / heads gradient views inside the flat bucket (so FusedAdam applies Adam to them)
struct DenseFinalize {
  const float* part = nullptr;  // null: none
  int rs = 0, groups = 0, A1 = 0;
  int group0 = 0;  // first K12 group finalized here (the head group K/32 when the dense weight goes through
                   // the split-reading Adam tail)
  int64_t K = 0;
  void *dw = nullptr, *db = nullptr, *dwh = nullptr, *dbh = nullptr;
};

// K11: shuffle partitioning. dest = splitmix64(key) % R (mode 0) or key mod R (mode 1), R <= 1024.
// partition_hist writes counts[G][R] (G = partition_groups(n)); the caller turns them into
// exclusive offsets (destination-major: all of destination 0's rows first) and partition_scatter
// moves keys + row_bytes payloads to out_keys / out_vals.
int64_t partition_groups(int64_t n);
void partition_hist(const int64_t* keys, int64_t n, int R, int mode, int64_t* counts, hipStream_t stream);
void partition_scatter(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, int R, int mode,
                       const int64_t* offsets, int64_t* out_keys, void* out_vals, hipStream_t stream);

// K13: y = ReLU(x Wᵀ + b), x [M,K], W [N,K] row-major bf16, K % 32 == 0, N % 16 == 0 (small-M GEMM).
// K16: K14 + Gumbel-max sampling and rollout-row stores (as sample_store)
// hpart/S/hb: read hidden as bf16(ReLU(Σ_s hpart[s] + hb)) from K13s partials instead of `hidden`
void dense_heads_sample(const void* hidden, const void* wh, const void* bh, const int64_t* t_ptr, const int64_t* ctr,
                        uint32_t seed, int64_t* act, float* logp, float* vf, float* lout, int64_t* act_now, int64_t B,
                        int A1, hipStream_t stream, unsigned int* done = nullptr, const float* hpart = nullptr,
                        int S = 0, const void* hb = nullptr, int64_t* host_seq = nullptr);
// K15: K14 + fused PPO loss stats + dheads + dpre (for dense_heads_bwd(dpre_ready=true))
void dense_heads_ppo(const void* hidden, const void* wh, const void* bh, const float* cols, const float* coef,
                     float* acc, const float* gout, int64_t M, int A1, void* dz, void* dpre, hipStream_t stream,
                     const int64_t* cidx = nullptr, const int64_t* ctr = nullptr, int64_t period = 1,
                     const float* hpart = nullptr, int S = 0, const void* hb = nullptr, void* hid_out = nullptr);
// K13s: split-K dense layer, fp32 partials part[S][M][N] (no bias / ReLU: K15 / K16 finish them)
int dense_fwd_part_slices(int64_t M, int64_t K, int N);
void dense_fwd_part(const void* x, const void* w, int64_t M, int64_t K, int N, float* part, int S,
                    hipStream_t stream);
// K14: heads[M, A1] = hidden[M, 256] Whᵀ + bh (bf16), one wave per row
void dense_heads_fwd(const void* hidden, const void* wh, const void* bh, int64_t M, int A1, void* heads,
                     hipStream_t stream);
void dense_relu_fwd(const void* x, const void* w, const void* b, int64_t M, int64_t K, int N, void* y,
                    hipStream_t stream);

// K10: fused Nature-CNN trunk (conv 8x8/4 4->16 + conv 4x4/2 16->32, bias+ReLU) on MFMA, one
// workgroup per frame in LDS. Frames u8 [.,4,84,84] gathered by idx (device-counter window like
// gather_rows); weights bf16 with element strides w*s = [co, ci, ky, kx]. h1 [B,441,16] (may be
// null: inference) and h2 [B,121,32] bf16 outputs. Backward writes bf16 dW1/db1/dW2/db2 (param
// memory order) through `partial` (nature_trunk_partial_floats(B) fp32).
void nature_trunk_fwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B,
                      const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                      const void* b2, void* h1, void* h2, hipStream_t stream, int dbg = 0);
// K10 forward in rollout push mode (K19 folded in): frames = stack[b] shifted by one + new_frames[b]
// (may be device-mapped pinned host memory); writes the shifted stack back and, with rows, rollout
// row *t_ptr ([T, B, 4, 84, 84] u8). h2 as nature_trunk_fwd.
void nature_trunk_fwd_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* rows, const int64_t* t_ptr, int64_t B,
                           const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                           const void* b2, void* h2, hipStream_t stream);
// K10 rollout band mode: each frame split over 4 workgroups (conv2 row bands); the frame stack is
// rollout row (t-1) mod T planes 1..3 + new_frames[b]; writes rollout row t ([T, B, 4, 84, 84] u8) and h2.
void nature_trunk_fwd_push_rows(uint8_t* rows, int64_t T, const uint8_t* new_frames, const int64_t* t_ptr, int64_t B,
                                const void* W1, const int64_t* w1s, const void* b1, const void* W2, const int64_t* w2s,
                                const void* b2, void* h2, hipStream_t stream);
int nature_trunk_bwd_groups(int64_t B);
int64_t nature_trunk_partial_floats(int64_t B);
void nature_trunk_bwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B,
                      const void* W2, const int64_t* w2s, const void* h1, const void* h2, const void* dh2,
                      float* partial, void* dW1, const int64_t* w1s, void* db1, void* dW2, void* db2,
                      hipStream_t stream, int dbg = 0, const FusedAdam& fa = FusedAdam{},
                      const AdamTail& at = AdamTail{}, const DenseFinalize& df = DenseFinalize{});
// dbg (profiling only, 0 in production): fwd bit0/1 skip conv1/conv2 MFMA, bit2 skip the frame
// load; bwd bit0/1/2 skip the dW2 / dh1 / dW1 phases, bit3 the staging loads, bit4 the partial stores,
// bit5 the st zeroing, bit6 return at once, bit7 the reduce launch, bit8 all LDS zeroing, bit9 the W2
// staging, bit10 the bias-gradient epilogue.

// ---- precision-matched (fp32-level) kernels over split-bf16 pairs (x3_kernels.hip, x3_device.h):
// a split tensor is two bf16 planes hi / lo of the same shape with x = hi + lo; products are
// hi*hi + hi*lo + lo*hi on the bf16 MFMA with fp32 accumulation; gradients are fp32.
struct X3In {
  const void* hi = nullptr;
  const void* lo = nullptr;
};
struct X3Out {
  void* hi = nullptr;
  void* lo = nullptr;
};
// K10x: trunk forward (h1 may be {null, null}: inference); grid min(B, 256) workgroups loop over frames
int x3_trunk_fwd_groups(int64_t B);
void x3_trunk_fwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B, X3In W1,
                  const int64_t* w1s, X3In b1, X3In W2, const int64_t* w2s, X3In b2, X3Out h1, X3Out h2,
                  hipStream_t stream, const float* cols = nullptr, float* cols_out = nullptr, int ncols = 0);
void x3_trunk_fwd_push(uint8_t* stack, const uint8_t* new_frames, uint8_t* rows, const int64_t* t_ptr, int64_t B,
                       X3In W1, const int64_t* w1s, X3In b1, X3In W2, const int64_t* w2s, X3In b2, X3Out h2,
                       hipStream_t stream,
                       const int64_t* gate = nullptr, int64_t gate_want = 0, int* gate_err = nullptr,
                       int gate_parts = 1, int gate_timeout_ms = 2000);
// K10x backward: conv2 launch (dW2, db2, dpre1 -> dpre1 pair, db1) + conv1 weight-grad launch + reduce;
// fp32 gradients in the parameters' memory order. partial: x3_trunk_partial_floats(B) floats.
int x3_conv2_bwd_groups(int64_t B);
int x3_conv1_wgrad_groups(int64_t B);
int64_t x3_trunk_partial_floats(int64_t B);
void x3_trunk_bwd(const uint8_t* obs, const int64_t* idx, const int64_t* ctr, int64_t period, int64_t B, X3In W2,
                  const int64_t* w2s, X3In h1, const void* h2hi, X3In dh2, X3Out dpre1, float* partial, float* dW1,
                  const int64_t* w1s, float* db1, float* dW2, float* db2, hipStream_t stream,
                  const X3Adam& xa = X3Adam{}, bool dense_separate = false);
// the tail Adam's dense + heads range as its own launch (dense_separate above): forked beside the trunk
// backward; the trunk-reduce launch of the same step still advances the (parity) counters
int x3_dense_adam_groups(const X3Adam& xa);
void x3_dense_adam(const X3Adam& xa, hipStream_t stream);
// K13x: split-K dense layer -> fp32 partials part[S][M][N]
int x3_dense_fwd_part_slices(int64_t M, int64_t K, int N);
void x3_dense_fwd_part(X3In x, X3In w, int64_t M, int64_t K, int N, float* part, int S, hipStream_t stream);
// K15x: hidden = ReLU(Σ partials + hb) (fp32), heads, PPO loss stats into acc, dz / dpre / hid split pairs.
// acc_slab: acc is a per-workgroup slab [x3_heads_ppo_groups(M)][8] (each workgroup adds its 6 sums into its
// own row, no atomics; the caller sums the rows) instead of 6 floats every workgroup adds to atomically
int x3_heads_ppo_groups(int64_t M);
void x3_heads_ppo(const float* hpart, int S, X3In hb, X3In wh, X3In bh, const float* cols, const float* coef, float* acc,
                  const float* gout, int64_t M, int A1, X3Out dz, X3Out dpre, X3Out hid, hipStream_t stream,
                  const int64_t* cidx = nullptr, const int64_t* ctr = nullptr, int64_t period = 1,
                  bool acc_slab = false);
// K16x: fp32 head row + Gumbel-max sampling + rollout-row stores (+ the step advance with `done`)
void x3_heads_sample(const float* hpart, int S, X3In hb, X3In wh, X3In bh, const int64_t* t_ptr, const int64_t* ctr,
                     uint32_t seed, int64_t* act, float* logp, float* vf, float* lout, int64_t* act_now, int64_t B, int A1,
                     hipStream_t stream, unsigned int* done = nullptr, int64_t* host_seq = nullptr);
// K13x + K16x in one launch (rollout, M <= 64): split-K partials, per-row-tile tickets, the finisher of a
// row tile runs the heads + sampling of its 16 rows, the last one advances the step. done: 1 + ceil(M/16)
// zero-initialised words (zero again when the launch ends)
void x3_dense_heads_sample(X3In x, X3In w, int64_t M, int64_t K, float* part, int S, X3In hb, X3In wh, X3In bh,
                           const int64_t* t_ptr, const int64_t* ctr, uint32_t seed, int64_t* act, float* logp, float* vf,
                           float* lout, int64_t* act_now, int A1, hipStream_t stream, unsigned int* done,
                           int64_t* host_seq = nullptr);
// K12x: dx (split pair) and fp32 dW, db, dWh, dbh. rs = 2: two row parts, the second one's dW / db / dWh / dbh
// into dw2 / db2 / dwh2 / dbh2 (summed by the tail Adam, X3Adam::grad2)
void x3_dense_heads_bwd(X3In dz, int A1, X3In y, X3In x, X3In w, X3In dpre, int64_t M, int64_t K, X3Out dx, float* dw,
                        float* db, float* dwh, float* dbh, hipStream_t stream, int rs = 1, float* dw2 = nullptr,
                        float* db2 = nullptr, float* dwh2 = nullptr, float* dbh2 = nullptr);
// fp32 -> split pair (weights after a host-side update, tests)
void x3_split(const float* src, void* hi, void* lo, int64_t n, hipStream_t stream);
// phase probe of the x3 SGD-step kernels: a device buffer of 7 x 1024 x 16 uint64 (nullptr: off)
void x3_probe_set(uint64_t* ts);

// K17: learner-side sample-batch ingest (see ingest_kernels.hip). raw [rows, A+5] fp32 =
// [logits(A) | logp | vf | reward | done | action], blocks = one entry per rollout fragment
// (time-major rows t*n+env starting at row0; bootstrap values at boot[boot0 .. boot0+n)).
// cols [rows, A+4] = [logits | logp | adv | value target | action]; stats (2 doubles, zeroed by
// the caller) accumulate sum(adv), sum(adv^2) for standardize_col (K17b).
struct IngestBlock {
  int64_t row0;
  int32_t T;
  int32_t n;
  int32_t boot0;
  int32_t pad;
};
void ingest_gae(const float* raw, const float* boot, const IngestBlock* blocks_dev, int nblocks, int A, float gamma,
                float lam, float* cols, double* stats, hipStream_t stream);
void standardize_col(float* cols, int64_t N, int C, int col, const double* stats, hipStream_t stream);
// K18: V-trace targets over time-major [T, B] columns (vtrace_kernels.hip). clip_rho /
// clip_pg_rho = +inf disables the clip.
void vtrace(const float* blogp, const float* tlogp, const float* rew, const float* val, const float* done,
            const float* boot, int64_t T, int64_t B, float gamma, float clip_rho, float clip_pg_rho, float lam,
            float* vs, float* pg, hipStream_t stream);
// Page-locked DMA out of a shared-memory object-store segment: chunks of the registered segment
// are hipHostRegister'ed on first use. Returns the bytes newly registered by this call.
// K21 persistent rollout server (rollout_server.hip): one launch runs a hybrid worker's T policy
// steps, synchronising with the host through mapped words (go / done_seq). Returns the grid size.
struct RolloutServerArgs {
  const void *W1 = nullptr, *b1 = nullptr, *W2 = nullptr, *b2 = nullptr;
  int64_t w1s[4] = {0, 0, 0, 0}, w2s[4] = {0, 0, 0, 0};
  const void *Wd = nullptr, *bd = nullptr, *Wh = nullptr, *bh = nullptr;
  int64_t B = 0, T = 0;
  int S = 0, A1 = 0;
  uint32_t seed = 0;
  uint8_t* stack = nullptr;
  const uint8_t* nf = nullptr;
  uint8_t* rows = nullptr;
  void* h2 = nullptr;
  float* hpart = nullptr;
  int64_t* act = nullptr;
  float *logp = nullptr, *vf = nullptr, *lout = nullptr;
  int64_t* act_now = nullptr;
  int64_t* ctr_t = nullptr;
  const int64_t* go = nullptr;   // device view of the host word
  int64_t* done_seq = nullptr;   // device view of the host word
  unsigned int* bar = nullptr;   // 10 device words (global / phase-C / 8 per-XCD counters)
  int64_t* err_dev = nullptr;
  int64_t* err_host = nullptr;   // device view of the host word
  double go_timeout_s = 20.0, barrier_timeout_s = 5.0;
  int workgroups = 0;            // 0: one per CU
  uint64_t* prof = nullptr;      // optional device [T][5] phase timestamps (s_memrealtime)
  // fp32 policy (direct launches only): the weights above are the hi planes of split-bf16 pairs and these
  // the lo planes; h2 / h2lo the trunk output pair (K10x push -> K13x -> K16x, x3_kernels.hip)
  bool x3 = false;
  const void *W1lo = nullptr, *b1lo = nullptr, *W2lo = nullptr, *b2lo = nullptr;
  const void *Wdlo = nullptr, *bdlo = nullptr, *Whlo = nullptr, *bhlo = nullptr;
  void* h2lo = nullptr;
  // in-kernel step gate (fp32 direct launches): K10x waits until *gate (device view of the host release
  // counter) reaches the step's number before it reads the newest frames; bounded, *gate_err set on timeout
  const int64_t* gate = nullptr;
  int* gate_err = nullptr;
  int gate_timeout_ms = 2000;  // wall-clock bound of one gate wait (s_memrealtime)
  // fp32 direct launches: K13x + K16x as ONE launch (x3_dense_heads_sample; k16_done then holds
  // 1 + ceil(B / 16) ticket words)
  bool fused_heads = false;
};
int rollout_server_launch(const RolloutServerArgs& a, hipStream_t stream);

void host_register_segment(uintptr_t base, uint64_t size);
// Page-lock the registered-segment chunks covering [p, p+n); true if all of them are pinned
// (then DMA straight from/to the range is safe). newly (optional) accumulates bytes pinned now.
bool host_pin_range(const void* p, uint64_t n, uint64_t* newly = nullptr);
uint64_t h2d_from_segment(void* dst, const void* src, uint64_t n, hipStream_t stream);
// Host<->device copy of a range of a registered segment, split at registration-chunk boundaries:
// page-locked chunks are async DMA on `stream`, chunks that could not be pinned go through the
// bounce buffers (synchronously). One copy never straddles pinned and pageable memory.
void dma_host_segment(void* host, void* dev, uint64_t n, bool to_device, hipStream_t stream);
std::string host_register_last_error();
// {bytes DMA'd straight from registered chunks, bytes staged via bounce buffers, chunks pinned,
//  chunks that could not be pinned}
std::vector<uint64_t> h2d_stats();
void host_unregister_all();
// Unpin every chunk of a segment and forget it: MUST run before the segment is unmapped (a stale
// registration would alias whatever is mapped at that address next).
void host_unregister_segment(uintptr_t base);
// page-lock [base, base + bytes) of a registered segment chunk by chunk (stops early once *stop is set)
void host_prepin(uintptr_t base, uint64_t bytes, const std::atomic<bool>* stop,
                 std::atomic<uint64_t>* done_bytes = nullptr);

}  // namespace hip
}  // namespace rmm
