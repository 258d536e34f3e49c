"""Per-kernel stats (calls, total / mean / median us, grid, workgroup, LDS, VGPRs) from a rocprofv3 rocpd
SQLite database (ROCm 7.2's default --kernel-trace output). Usage: python tools/rocpd_stats.py DB [N]"""
import sqlite3
import statistics
import sys


def main(db: str, top: int = 30) -> None:
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    q = f"select {name}, start, end, grid_x, workgroup_x, lds_size, vgpr_count from kernels"
    per = {}
    for n, s, e, grid, wg, lds, vg in c.execute(q):
        d = per.setdefault(n, {"t": [], "grid": grid, "wg": wg, "lds": lds, "vgpr": vg})
        d["t"].append((e - s) / 1e3)
    rows = sorted(per.items(), key=lambda kv: -sum(kv[1]["t"]))
    tot = sum(sum(d["t"]) for _, d in rows)
    print(f"{'tot ms':>8} {'%':>5} {'calls':>6} {'mean us':>8} {'med us':>7} {'grid':>8} {'wg':>4} {'lds':>7} {'vgpr':>4}  kernel")
    for n, d in rows[:top]:
        t = d["t"]
        print(f"{sum(t) / 1e3:8.2f} {100 * sum(t) / tot:5.1f} {len(t):6d} {statistics.mean(t):8.1f} "
              f"{statistics.median(t):7.1f} {d['grid']:8d} {d['wg']:4d} {d['lds']:7d} {d['vgpr']:4d}  {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
