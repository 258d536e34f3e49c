"""Summarise rocprofv3 PMC results (SQLite `*_results.db` or CSV) per kernel: mean counter value
per dispatch for kernels whose name contains a substring.
Usage: python benchmarks/pmc_summary.py <dir-or-file> [kernel-substring]"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def rows(path):
    files = [path] if os.path.isfile(path) else (glob.glob(os.path.join(path, "**", "*.db"), recursive=True) +
                                                glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                          recursive=True))
    for f in files:
        if f.endswith(".db"):
            con = sqlite3.connect(f)
            cols = [c[1] for c in con.execute("pragma table_info(counters_collection)")]
            kcol = "kernel_name" if "kernel_name" in cols else "name"
            q = f"select dispatch_id, {kcol}, counter_name, value from counters_collection"
            for d, k, c, v in con.execute(q):
                yield d, k, c, v
        else:
            for r in csv.DictReader(open(f)):
                yield r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])


def main():
    path, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d, k, c, v in rows(path):
        if sub in k:
            short = k.split("(")[0][-60:]
            acc[short][c] += v
            disp[short].add(d)
    for k, cs in acc.items():
        n = len(disp[k])
        print(f"{k}  dispatches={n}")
        for c, v in sorted(cs.items()):
            print(f"  {c:28s} {v / n:16.1f}")


if __name__ == "__main__":
    main()
