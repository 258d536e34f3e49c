"""Summarise a rocprofv3 profile: top kernels by total time.

Accepts either `<prefix>_kernel_stats.csv` (``--output-format csv``) or the default
`<prefix>_results.db` (rocpd sqlite). Usage: python summarize_prof.py FILE [TOP_N]"""
import csv
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        q = "select name, total_calls, total_duration, average from top_kernels order by total_duration desc"
        # the rocpd views report microseconds; normalise to ns like the csv
        return [(n, int(c), float(t) * 1e3, float(a) * 1e3) for n, c, t, a in db.execute(q)]
    rows = list(csv.DictReader(open(path)))
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"])) for r in rows]


def main():
    rows = load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} launches")
    print(f"{'total':>9}    {'pct':>6} {'calls':>7} {'avg':>9}")
    for name, calls, t, avg in rows[:n]:
        print(f"{t / 1e6:9.2f} ms {100 * t / tot:6.2f}% {calls:7d} {avg / 1e3:9.1f} us  {name[:100]}")


if __name__ == "__main__":
    main()
