"""Condensed memory-op trace of one kernel in a gfx950 assembly file (hipcc --cuda-device-only -S):
global / buffer loads and stores, vmcnt / lgkmcnt waits, barriers, branches and loop headers, runs of the
same op collapsed. To audit where a kernel waits out a memory round trip before its next loads are issued.
usage: python tools/asm_trace.py FILE.s SYMBOL_SUBSTRING [max_lines]"""
import re
import sys


def main(path, sub, n=400):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sub in l)
    out, prev, cnt = [], None, 0
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip()
        key = None
        if "Loop Header" in t or (t.startswith(".LBB") and t.endswith(":")):
            key = t.split(";")[0] + ("  <loop>" if "Loop Header" in t else "")
        else:
            op = t.split()[0] if t else ""
            if op.startswith(("global_load", "global_store", "buffer_load", "buffer_store", "global_atomic")) or \
                    op in ("s_barrier", "s_waitcnt") or op.startswith(("s_cbranch", "s_branch")):
                key = op if op != "s_waitcnt" else t
        if key is None:
            continue
        if key == prev:
            cnt += 1
            continue
        if prev is not None:
            out.append(f"{prev}{'  x' + str(cnt) if cnt > 1 else ''}")
        prev, cnt = key, 1
    out.append(f"{prev}{'  x' + str(cnt) if cnt > 1 else ''}")
    print("\n".join(out[:n]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 400)
