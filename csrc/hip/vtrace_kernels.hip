// K18: V-trace off-policy targets (IMPALA / APPO learner).
//
// Time-major [T, B] columns in, vs and policy-gradient advantages out:
//   rho_t   = exp(target_logp_t - behaviour_logp_t)
//   delta_t = min(rho_bar, rho_t) * (r_t + disc_t V_{t+1} - V_t)
//   vs_t    = V_t + delta_t + disc_t * lam * min(1, rho_t) * (vs_{t+1} - V_{t+1})
//   pg_t    = min(pg_rho_bar, rho_t) * (r_t + disc_t vs_{t+1} - V_t)
// with disc_t = gamma (1 - done_t), V_T = vs_T = bootstrap. Parity: reference
// rllib/algorithms/impala/vtrace_torch.py:from_importance_weights (which runs the backward
// recursion as T sequential torch ops on [B] slices).
//
// One lane per trajectory column, all T steps in registers: the loads of an 8-step chunk are
// issued together (they do not depend on the recursion), so the sequential part is FMA latency
// only. 64-lane workgroups so small B still spreads over several CUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace rmm {
namespace hip {

namespace {
constexpr int kVtU = 8;

__global__ __launch_bounds__(kWave) void k_vtrace(const float* __restrict__ blogp, const float* __restrict__ tlogp,
                                                  const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ done, const float* __restrict__ boot,
                                                  int64_t T, int64_t B, float gamma, float clip_rho, float clip_pg_rho,
                                                  float lam, float* __restrict__ vs, float* __restrict__ pg) {
  const int64_t b = int64_t(blockIdx.x) * kWave + threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;          // vs_{t+1} - V_{t+1}
  float v_tp1 = boot[b];    // V_{t+1}
  float vs_tp1 = v_tp1;     // vs_{t+1}
  for (int64_t t = T - 1; t >= 0; t -= kVtU) {
    const int n = int(t + 1 < kVtU ? t + 1 : kVtU);
    float lb[kVtU], lt[kVtU], r[kVtU], v[kVtU], d[kVtU];
#pragma unroll
    for (int i = 0; i < kVtU; i++) {
      if (i < n) {
        const int64_t k = (t - i) * B + b;
        lb[i] = blogp[k];
        lt[i] = tlogp[k];
        r[i] = rew[k];
        v[i] = val[k];
        d[i] = done[k];
      }
    }
#pragma unroll
    for (int i = 0; i < kVtU; i++) {
      if (i < n) {
        const int64_t k = (t - i) * B + b;
        const float rho = __expf(lt[i] - lb[i]);
        const float disc = gamma * (1.f - d[i]);
        const float delta = fminf(clip_rho, rho) * (r[i] + disc * v_tp1 - v[i]);
        acc = delta + disc * lam * fminf(1.f, rho) * acc;
        const float vs_t = acc + v[i];
        pg[k] = fminf(clip_pg_rho, rho) * (r[i] + disc * vs_tp1 - v[i]);
        vs[k] = vs_t;
        vs_tp1 = vs_t;
        v_tp1 = v[i];
      }
    }
  }
}
}  // namespace

void vtrace(const float* blogp, const float* tlogp, const float* rew, const float* val, const float* done,
            const float* boot, int64_t T, int64_t B, float gamma, float clip_rho, float clip_pg_rho, float lam,
            float* vs, float* pg, hipStream_t stream) {
  if (T <= 0 || B <= 0) return;
  const int64_t blocks = (B + kWave - 1) / kWave;
  if (blocks > (int64_t(1) << 31) - 1) throw std::invalid_argument("vtrace: B too large");
  hipLaunchKernelGGL(k_vtrace, dim3(uint32_t(blocks)), dim3(kWave), 0, stream, blogp, tlogp, rew, val, done, boot, T,
                     B, gamma, clip_rho, clip_pg_rho, lam, vs, pg);
  RMM_HIP_CHECK(hipGetLastError());
}

}  // namespace hip
}  // namespace rmm
