"""Distributed sort benchmark (Exoshuffle / CloudSort style) on the runtime.

Parity: reference python/ray/experimental/raysort/main.py — generate gensort-format input parts,
map (partition by key range), two-stage merge (per round of mappers, then per reducer), write the
output parts, validate. Differences, by design:

* input generation and validation are built in (numpy), not the external gensort / valsort
  binaries: every record carries its global index in bytes 10..17, and validation checks global
  order, per-part key ranges, the record count and an order-independent checksum of all bytes;
* ``--gpu``: mappers partition on the GPU with K11's "range" mode (one histogram + one scatter
  launch; the payload moves as 16-byte vectors), the first-stage merge sorts; host mappers sort and
  split like the reference (both produce the same key ranges);
* map outputs are store objects consumed by the merge tasks (zero-copy reads of the shared-memory
  store, spilled under pressure by the store's IO workers), with at most ``--max_rounds_in_flight``
  mapper rounds outstanding (the reference's round-based backpressure).

Usage: ``python -m ray_memory_management_amd.experimental.raysort.main --total_data_size 1e9``.
"""
from __future__ import annotations

import argparse
import csv
import os
import tempfile
import time
from typing import Dict, List

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.experimental.raysort import constants, sortlib
from ray_memory_management_amd.experimental.raysort.types import PartInfo

Args = argparse.Namespace


def get_args(*args, **kwargs) -> Args:
    p = argparse.ArgumentParser()
    p.add_argument("--ray_address", default=None, type=str, help="None: start a local cluster")
    p.add_argument("--total_data_size", default=int(1e9), type=lambda s: int(float(s)), help="bytes")
    p.add_argument("--num_mappers", default=16, type=int)
    p.add_argument("--num_mappers_per_round", default=4, type=int)
    p.add_argument("--num_reducers", default=8, type=int)
    p.add_argument("--max_rounds_in_flight", default=2, type=int)
    p.add_argument("--data_dir", default=None, type=str)
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--gpu", action="store_true", help="partition map inputs on the GPU (K11 range mode)")
    p.add_argument("--skip_input", action="store_true")
    p.add_argument("--skip_sorting", action="store_true")
    p.add_argument("--skip_output", action="store_true")
    a = p.parse_args(*args, **kwargs)
    if a.data_dir is None:
        a.data_dir = os.path.join(tempfile.gettempdir(), constants.DATA_DIR_NAME)
    constants.bytes_to_records(a.total_data_size)
    if a.total_data_size // constants.RECORD_SIZE < a.num_mappers:
        raise ValueError("fewer records than mappers")
    return a


def _path(args: Args, part_id: int, kind: str) -> str:
    return os.path.join(args.data_dir, f"{kind}-{part_id:08d}")


# ------------------------------------------------------------------------------ input
@ray.remote
def generate_part(args: Args, part_id: int, num_records: int, offset: int):
    rng = np.random.default_rng([args.seed, part_id])
    recs = rng.integers(0, 256, (num_records, constants.RECORD_SIZE), dtype=np.uint8)
    recs[:, constants.KEY_SIZE:constants.KEY_SIZE + 8] = \
        np.arange(offset, offset + num_records, dtype="<u8").view(np.uint8).reshape(-1, 8)
    path = _path(args, part_id, "input")
    recs.tofile(path)
    return PartInfo(part_id, "local", path, num_records), sortlib.checksum(recs)


def generate_input(args: Args) -> Dict:
    os.makedirs(args.data_dir, exist_ok=True)
    total = constants.bytes_to_records(args.total_data_size)
    size = -(-total // args.num_mappers)
    refs, off = [], 0
    for m in range(args.num_mappers):
        n = min(size, total - off)
        refs.append(generate_part.remote(args, m, n, off))
        off += n
    res = ray.get(refs)
    with open(os.path.join(args.data_dir, constants.INPUT_MANIFEST_FILE), "w", newline="") as f:
        w = csv.writer(f)
        for info, cs in res:
            w.writerow([info.part_id, info.node, info.path, info.num_records, cs])
    return {"records": total, "checksum": sum(cs for _, cs in res) % (1 << 64)}


def _load_manifest(path: str) -> List[List[str]]:
    with open(path) as f:
        return [row for row in csv.reader(f)]


def _load_part(path: str) -> np.ndarray:
    return np.fromfile(path, dtype=np.uint8).reshape(-1, constants.RECORD_SIZE)


# ------------------------------------------------------------------------------ sort
def _gpu_partition(part: np.ndarray, R: int) -> List[np.ndarray]:
    """K11 range partition on the GPU: keys = big-endian prefixes (as int64 bits), payload = the
    whole 100-byte record (rows move as 16-B vectors after padding to 112 bytes)."""
    import torch

    from ray_memory_management_amd.experimental.gpu_shuffle import partition

    dev = torch.device("cuda", torch.cuda.current_device())
    keys = torch.from_numpy(sortlib.key_prefix(part).view(np.int64)).to(dev)
    rows = torch.zeros((len(part), 112), dtype=torch.uint8)
    rows[:, :constants.RECORD_SIZE] = torch.from_numpy(part)
    _, vals, counts = partition(keys, rows.to(dev), R, mode="range")
    host = vals[:, :constants.RECORD_SIZE].cpu().numpy()
    bounds = np.concatenate([[0], np.cumsum(counts.cpu().numpy())])
    return [host[bounds[r]:bounds[r + 1]] for r in range(R)]


@ray.remote
def mapper(args: Args, mapper_id: int, path: str):
    part = _load_part(path).copy()
    R = args.num_reducers
    if args.gpu:
        blocks = _gpu_partition(part, R)
    else:
        bounds = sortlib.sort_and_partition(part, R)
        blocks = [part[b.offset:b.offset + b.size] for b in bounds]
    return blocks if R > 1 else blocks[0]


@ray.remote
def merge_mapper_blocks(args: Args, reducer_id: int, mapper_round: int, *blocks):
    return sortlib.merge_partitions(blocks)


@ray.remote
def final_merge(args: Args, reducer_id: int, *merged):
    out = sortlib.merge_partitions(merged)
    path = _path(args, reducer_id, "output")
    if not args.skip_output:
        out.tofile(path)
    return PartInfo(reducer_id, "local", path, len(out))


def sort_main(args: Args) -> List[PartInfo]:
    parts = _load_manifest(os.path.join(args.data_dir, constants.INPUT_MANIFEST_FILE))
    M, R, per = len(parts), args.num_reducers, args.num_mappers_per_round
    rounds = -(-M // per)
    merged: List[List] = [[] for _ in range(R)]
    in_flight: List[List] = []
    for rnd in range(rounds):
        ids = range(rnd * per, min(M, (rnd + 1) * per))
        maps = [mapper.options(num_returns=R).remote(args, m, parts[m][2]) for m in ids]
        if R == 1:
            maps = [[m] for m in maps]
        round_refs = []
        for r in range(R):
            ref = merge_mapper_blocks.remote(args, r, rnd, *[mr[r] for mr in maps])
            merged[r].append(ref)
            round_refs.append(ref)
        del maps  # the merge tasks hold the map outputs now
        in_flight.append(round_refs)
        if len(in_flight) >= args.max_rounds_in_flight:  # round-based backpressure
            ray.wait(in_flight.pop(0), num_returns=R)
    outs = ray.get([final_merge.remote(args, r, *merged[r]) for r in range(R)])
    with open(os.path.join(args.data_dir, constants.OUTPUT_MANIFEST_FILE), "w", newline="") as f:
        w = csv.writer(f)
        for o in outs:
            w.writerow([o.part_id, o.node, o.path, o.num_records])
    return outs


# ------------------------------------------------------------------------------ validate
def validate_output(args: Args) -> Dict:
    """Global order, key ranges per output part, record count and checksum vs the input."""
    inp = _load_manifest(os.path.join(args.data_dir, constants.INPUT_MANIFEST_FILE))
    out = _load_manifest(os.path.join(args.data_dir, constants.OUTPUT_MANIFEST_FILE))
    want_n = sum(int(r[3]) for r in inp)
    want_cs = sum(int(r[4]) for r in inp) % (1 << 64)
    n, cs, last = 0, 0, None
    R = len(out)
    for r, row in enumerate(out):
        recs = _load_part(row[2])
        if len(recs):
            pre, suf = sortlib.key_prefix(recs), sortlib.key_suffix(recs)
            if not ((pre[1:] > pre[:-1]) | ((pre[1:] == pre[:-1]) & (suf[1:] >= suf[:-1]))).all():
                raise AssertionError(f"output part {r} is not sorted")
            if (sortlib.range_of(pre, R) != r).any():
                raise AssertionError(f"output part {r} holds keys of another range")
            first = (int(pre[0]), int(suf[0]))
            if last is not None and first < last:
                raise AssertionError(f"output part {r} starts below the end of part {r - 1}")
            last = (int(pre[-1]), int(suf[-1]))
        n += len(recs)
        cs = (cs + sortlib.checksum(recs)) % (1 << 64)
    if n != want_n:
        raise AssertionError(f"{n} output records, {want_n} input records")
    if cs != want_cs:
        raise AssertionError("checksum mismatch between input and output")
    return {"records": n, "checksum": cs}


def main(args: Args) -> Dict:
    started = False
    if not ray.is_initialized():
        ray.init(address=args.ray_address) if args.ray_address else ray.init()
        started = True
    try:
        res: Dict = {}
        if not args.skip_input:
            t0 = time.perf_counter()
            res["input"] = generate_input(args)
            res["generate_s"] = time.perf_counter() - t0
        if not args.skip_sorting:
            t0 = time.perf_counter()
            sort_main(args)
            dt = time.perf_counter() - t0
            res["sort_s"] = dt
            res["sort_GBps"] = args.total_data_size / dt / 1e9
        if not args.skip_output and not args.skip_sorting:
            res["validated"] = validate_output(args)
        return res
    finally:
        if started:
            ray.shutdown()


if __name__ == "__main__":
    print(main(get_args()))
