"""Phase timestamps inside the fp32 (x3) SGD-step kernels on one MI355X.

Runs the fused fp32 learner on synthetic frames (no rollout: the rollout's trunk launch shares K10x's probe
rows), sets the x3 phase probe (csrc/hip/x3_kernels.hip `x3_probe_set`) for one update, and reports from the
LAST SGD step: each kernel's span (first workgroup start -> last workgroup end), the gap to the previous
kernel, the workgroup start skew, and the mean time from a workgroup's start to each probed phase boundary.
Timestamps are the 100 MHz real-time counter (10 ns).

The probe sites compile to nothing in the default build (their cost showed up in the kernels): build the
extension with them first, and rebuild without them afterwards:
    RMM_X3_PROBE=1 python build_native.py --force --only _hip

usage: python benchmarks/x3_phase_probe.py [--mbs 500]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KERNELS = ["K10x fwd", "conv2 bwd", "conv1 wgrad", "K12x", "reduce+Adam", "K13x-L", "K15x"]
ORDER = [0, 5, 6, 3, 1, 2, 4]  # launch order inside one SGD step
PHASES = {
    0: {1: "weights staged", 2: "f0 image", 3: "f0 conv1", 4: "f0 conv2", 5: "f1 image", 6: "f1 conv1",
        7: "f1 conv2"},
    1: {1: "prologue", 2: "f0 P0 staged", 3: "f0 P1a dW2", 4: "f0 P1b dh1", 5: "f0 dpre1 out", 6: "f1 P0 staged",
        7: "f1 P1a dW2", 8: "f1 P1b dh1", 9: "f1 dpre1 out"},
    2: {1: "f0 staged", 2: "f0 MFMA", 3: "f1 staged", 4: "f1 MFMA"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbs", type=int, default=500)
    a = ap.parse_args()
    import torch

    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    h = require_hip()
    dev = torch.device("cuda", 0)
    # the probe buffer is a kernel argument: set it before the learner captures its SGD graphs
    ts = torch.zeros(7 * 1024 * 16, dtype=torch.int64, device=dev)
    h.x3_probe_set(ts.data_ptr())
    torch.manual_seed(0)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": a.mbs, "num_sgd_iter": 10, "train_batch_size": 5000,
                                      "compute_dtype": "fp32"}, device=dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    N, A = 5000, 4
    obs = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    cols = torch.cat([torch.randn(N, A, generator=g), torch.randn(N, 1, generator=g) - 1.4,
                      torch.randn(N, 2, generator=g), torch.randint(0, A, (N, 1), generator=g).float()], 1).to(dev)
    try:
        for _ in range(3):  # every update rewrites the rows: the last one's last SGD step is read
            L._update_tables(obs, cols, A)
        torch.cuda.synchronize()
    finally:
        h.x3_probe_set(0)
    t = ts.view(7, 1024, 16).cpu()
    out = {}
    prev_end = None
    for k in ORDER:
        rows = t[k][t[k][:, 0] > 0]
        if rows.shape[0] == 0:
            continue
        st, en = rows[:, 0], rows[:, 15]
        d = {"workgroups": int(rows.shape[0]), "span_us": float(en.max() - st.min()) / 100,
             "start_skew_us": float(st.max() - st.min()) / 100,
             "wg_mean_us": float((en - st).float().mean()) / 100, "wg_max_us": float((en - st).max()) / 100}
        if prev_end is not None:
            d["gap_from_prev_us"] = float(st.min() - prev_end) / 100
        prev_end = int(en.max())
        ph = {}
        for slot, name in PHASES.get(k, {}).items():
            m = rows[:, slot] > 0
            if m.any():
                ph[name] = round(float((rows[m, slot] - rows[m, 0]).float().mean()) / 100, 2)
        if ph:
            d["phase_mean_us_from_wg_start"] = ph
        out[KERNELS[k]] = d
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
