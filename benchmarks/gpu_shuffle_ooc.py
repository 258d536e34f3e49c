"""Out-of-core GPU Exoshuffle (BASELINE.json config #5, reference python/ray/experimental/shuffle.py:231
run): more data than the GPU actors' HBM object-store quota, streamed through `--rounds` map/merge
rounds; partition blocks live in the HBM object store, spill to host memory (K4-compressed) under the
quota and are restored for the reduce (sort by key on the GPU). Prints one JSON line: end-to-end GB/s,
map / reduce seconds, spilled / restored bytes, correctness (rows, key checksums, payload bytes).

    python benchmarks/gpu_shuffle_ooc.py --quota-gb 8 --factor 4 --rounds 16 --partitions 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--quota-gb", type=float, default=8.0, help="HBM object-store quota per GPU process")
    ap.add_argument("--factor", type=float, default=4.0, help="total data = factor x quota x workers")
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--partitions", type=int, default=8, help="output partitions per worker")
    ap.add_argument("--row-bytes", type=int, default=248)
    ap.add_argument("--no-compress", action="store_true")
    ap.add_argument("--no-prealloc", action="store_true",
                    help="do not MAP_POPULATE the host store / pre-pin the spill arena")
    ap.add_argument("--spill-threshold", type=float, default=0.7,
                    help="HBM store occupancy above which its background thread spills (0 = only on demand)")
    a = ap.parse_args()

    import ray_memory_management_amd as ray
    from ray_memory_management_amd.experimental.gpu_shuffle import run_out_of_core_gpu_shuffle

    quota = int(a.quota_gb * (1 << 30))
    total = int(a.factor * quota * a.workers)
    ray.init(num_cpus=max(4, 2 * a.workers + 2), num_gpus=a.workers,
             object_store_memory=int(total * 1.25) + (2 << 30),
             _system_config={"gpu_object_store_memory": quota, "prestart_workers": 0,
                             "gpu_spill_compression": not a.no_compress,
                             "gpu_object_spilling_threshold": a.spill_threshold,
                             # the host arena the HBM blocks spill into: faulted in at init (reference
                             # preallocate_plasma_memory) and page-locked by the GPU store in the background
                             "preallocate_plasma_memory": not a.no_prealloc,
                             "gpu_spill_prepin_bytes": 0 if a.no_prealloc else int(total * 1.1)})
    try:
        r = run_out_of_core_gpu_shuffle(num_workers=a.workers, total_bytes=total, rounds=a.rounds,
                                        partitions_per_worker=a.partitions, row_bytes=a.row_bytes)
    finally:
        ray.shutdown()
    # the arena pre-pin (setup_prepin_seconds) is a one-time actor setup cost, like plasma's preallocation;
    # the rate with it counted in the timed region is reported next to the shuffle rate
    if r.get("setup_prepin_seconds") is not None and r.get("seconds"):
        r["GBps_including_prepin"] = r["bytes"] / 1e9 / (r["seconds"] + r["setup_prepin_seconds"])
    r.update(metric="out-of-core GPU shuffle throughput", unit="GB/s", quota_bytes=quota,
             data_over_quota=round(r["bytes"] / (quota * a.workers), 2),
             data="synthetic random int64 keys + key-derived uint8 payload")
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
