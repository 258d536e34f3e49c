"""GPU-resident all-to-all shuffle of keyed tensor blocks (the Exoshuffle data path on MI355X).

Parity: the reference shuffles through the object store only (python/ray/experimental/shuffle.py,
python/ray/data/_internal/push_based_shuffle.py): map tasks partition host blocks, reduce tasks
fetch partitions through plasma. On a node of MI355X GPUs the blocks already live in HBM and the
GPUs are directly connected by xGMI, so here a shuffle round is:

  1. partition on the GPU (K11, ``csrc/hip/shuffle_kernels.hip``): histogram + scatter so every
     destination's rows are contiguous (two launches, no host round trip except the [R] counts);
  2. exchange the per-destination row counts with one tiny all-to-all;
  3. ONE ``all_to_all`` of keys and ONE of payload bytes over RCCL (xGMI point-to-point links:
     each pair of GPUs exchanges its block directly, no host staging);
  4. optionally ``ray.put`` the received block: the HBM object store keeps it resident and spills
     it to host memory (compressed, K4) under HBM pressure.

CPU tensors take the same path with torch ops and a gloo group (tests, rehearsal).

Entry points: :func:`partition` (local), :func:`shuffle` (collective, inside a process group),
:class:`ShuffleWorker` + :func:`run_gpu_shuffle` (driver API: one actor per GPU, a collective
group between them, synthetic blocks, throughput + an order-independent checksum).
"""
from __future__ import annotations

import time
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

MODES = {"hash": 0, "mod": 1, "range": 2}


def _splitmix64(keys: torch.Tensor) -> np.ndarray:
    """The K11 hash on the host (numpy uint64 arithmetic wraps like the device's)."""
    x = keys.detach().cpu().numpy().astype(np.uint64)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xbf58476d1ce4e5b9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94d049bb133111eb)
        x ^= x >> np.uint64(31)
    return x


def destinations(keys: torch.Tensor, num_partitions: int, mode: str = "hash") -> torch.Tensor:
    """dest(key) exactly as K11 computes it (CPU reference / CPU path)."""
    k = keys.detach().cpu().to(torch.int64)
    if mode == "mod":
        return torch.remainder(k, num_partitions)
    if mode == "range":  # floor(u64(key) * R / 2^64) without 128-bit arithmetic (R <= 1024)
        u = k.numpy().view(np.uint64)
        hi, lo = u >> np.uint64(32), u & np.uint64(0xFFFFFFFF)
        R = np.uint64(num_partitions)
        return torch.from_numpy(((hi * R + ((lo * R) >> np.uint64(32))) >> np.uint64(32)).astype(np.int64))
    return torch.from_numpy((_splitmix64(k) % np.uint64(num_partitions)).astype(np.int64))


def partition(keys: torch.Tensor, values: Optional[torch.Tensor], num_partitions: int,
              mode: str = "hash") -> Tuple[torch.Tensor, Optional[torch.Tensor], torch.Tensor]:
    """Reorder rows so destination 0's rows come first, then destination 1's, ...

    keys: int64 [n]; values: any dtype [n, ...] (rows travel as raw bytes) or None.
    Returns (keys_out, values_out, counts[num_partitions] int64 on the keys' device)."""
    if keys.dtype != torch.int64 or keys.dim() != 1:
        raise ValueError("partition: keys must be a 1-D int64 tensor")
    n = keys.shape[0]
    if values is not None and values.shape[0] != n:
        raise ValueError("partition: values must have one row per key")
    if not 1 <= num_partitions <= 1024:
        raise ValueError("partition: 1 <= num_partitions <= 1024")
    if keys.is_cuda:
        return _partition_hip(keys.contiguous(), None if values is None else values.contiguous(), num_partitions,
                              MODES[mode])
    dest = destinations(keys, num_partitions, mode)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=num_partitions).to(torch.int64)
    return keys[order], (None if values is None else values[order]), counts


def _partition_hip(keys, values, R, mode):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    dev = keys.device
    n = keys.shape[0]
    stream = torch.cuda.current_stream(dev).cuda_stream
    G = h.partition_groups(n)
    counts_wg = torch.zeros((G, R), dtype=torch.int64, device=dev)
    h.partition_hist(keys.data_ptr(), n, R, mode, counts_wg.data_ptr(), stream)
    counts = counts_wg.sum(0)
    # destination-major exclusive offsets: base[r] + rows of destination r in earlier workgroups
    base = torch.cumsum(counts, 0) - counts
    offsets = (torch.cumsum(counts_wg, 0) - counts_wg + base.unsqueeze(0)).contiguous()
    out_keys = torch.empty_like(keys)
    out_vals = None
    row_bytes = 0
    if values is not None:
        out_vals = torch.empty_like(values)
        row_bytes = values[0].numel() * values.element_size() if n else 0
    h.partition_scatter(keys.data_ptr(), values.data_ptr() if values is not None else 0, n, row_bytes, R, mode,
                        offsets.data_ptr(), out_keys.data_ptr(), out_vals.data_ptr() if out_vals is not None else 0,
                        stream)
    return out_keys, out_vals, counts


def _alltoall(pg, out, inp, out_splits, in_splits):
    if pg is None:
        dist.all_to_all_single(out, inp, out_splits, in_splits)
    else:
        pg.alltoall_base(out, inp, out_splits, in_splits, dist.AllToAllOptions()).wait()


def shuffle(keys: torch.Tensor, values: Optional[torch.Tensor] = None, group=None, mode: str = "hash",
            world_size: Optional[int] = None, rank: Optional[int] = None):
    """Collective: every rank calls it with its block; returns the rows whose dest == this rank.

    group: a ``torch.distributed`` ProcessGroup object (e.g. from util.collective) or None for the
    default group. Keys and payload bytes each go in ONE all_to_all with split sizes."""
    world = world_size if world_size is not None else (group.size() if group is not None else dist.get_world_size())
    k, v, counts = partition(keys, values, world, mode)
    send_counts = counts.to(keys.device)
    recv_counts = torch.empty_like(send_counts)
    _alltoall(group, recv_counts, send_counts, [1] * world, [1] * world)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    out_k = torch.empty(sum(rc), dtype=torch.int64, device=keys.device)
    _alltoall(group, out_k, k, rc, sc)
    out_v = None
    if v is not None:
        row = values.element_size()
        for d in values.shape[1:]:
            row *= int(d)
        vb = v.contiguous().view(torch.uint8).reshape(-1) if v.numel() else \
            torch.empty(0, dtype=torch.uint8, device=keys.device)
        out_b = torch.empty(sum(rc) * row, dtype=torch.uint8, device=keys.device)
        _alltoall(group, out_b, vb.contiguous(), [c * row for c in rc], [c * row for c in sc])
        out_v = out_b.view(values.dtype).reshape(sum(rc), *values.shape[1:])
    return out_k, out_v


class ShuffleWorker:
    """Actor body (wrap with ray.remote): owns one device and one block of synthetic rows."""

    def __init__(self, rank: int, world: int, device: str = "cuda"):
        self.rank, self.world = rank, world
        self.device = torch.device(device if device != "cuda" else f"cuda:{torch.cuda.current_device()}") \
            if device.startswith("cuda") else torch.device("cpu")
        self.group_name = None

    def _collective_init(self, world_size, rank, backend, group_name):
        from ray_memory_management_amd.util import collective as col

        col.init_collective_group(world_size, rank, backend, group_name)
        self.group_name = group_name
        return True

    def generate(self, rows: int, row_bytes: int, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(1000 + self.rank + seed)
        self.keys = torch.randint(0, 2 ** 62, (rows,), generator=g, dtype=torch.int64).to(self.device)
        self.vals = torch.randint(0, 256, (rows, row_bytes), generator=g, dtype=torch.uint8).to(self.device)
        return int(self.keys.sum().item() % (1 << 61))

    def shuffle(self, mode: str = "hash"):
        from ray_memory_management_amd.util.collective.collective import get_group_handle

        pg = get_group_handle(self.group_name).pg
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        k, v = shuffle(self.keys, self.vals, group=pg, mode=mode, world_size=self.world, rank=self.rank)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        dest = destinations(k, self.world, mode)
        ok = bool((dest == self.rank).all().item())
        bytes_moved = self.keys.numel() * 8 + self.vals.numel()
        return {"rows_in": int(self.keys.numel()), "rows_out": int(k.numel()), "seconds": dt, "ok": ok,
                "bytes": bytes_moved, "key_sum": int(k.sum().item() % (1 << 61)) if k.numel() else 0}


def run_gpu_shuffle(num_workers: int = 2, rows_per_worker: int = 1 << 20, row_bytes: int = 256,
                    backend: str = "nccl", mode: str = "hash") -> dict:
    """Driver API: one ShuffleWorker actor per GPU (or CPU worker with backend='gloo'), one
    collective group, one shuffle round. Returns throughput and correctness checks."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.util import collective as col

    gpu = backend == "nccl"
    Actor = ray.remote(num_gpus=1 if gpu else 0, num_cpus=1)(ShuffleWorker)
    workers = [Actor.remote(r, num_workers, "cuda" if gpu else "cpu") for r in range(num_workers)]
    name = f"shuffle-{time.time_ns()}"
    col.create_collective_group(workers, num_workers, list(range(num_workers)), backend=backend, group_name=name)
    sums_in = ray.get([w.generate.remote(rows_per_worker, row_bytes) for w in workers])
    res = ray.get([w.shuffle.remote(mode) for w in workers])
    total_bytes = sum(r["bytes"] for r in res)
    secs = max(r["seconds"] for r in res)
    for w in workers:
        ray.kill(w)
    return {"ok": all(r["ok"] for r in res) and sum(r["rows_out"] for r in res) == rows_per_worker * num_workers
            and sum(sums_in) % (1 << 61) == sum(r["key_sum"] for r in res) % (1 << 61),
            "GBps": total_bytes / secs / 1e9, "seconds": secs, "bytes": total_bytes, "workers": num_workers}


# ================================================================== out-of-core (multi-round) shuffle
def _payload(keys: torch.Tensor, row_bytes: int) -> torch.Tensor:
    """Row payload derived from its key (so the reduce side can verify every byte after the block
    was spilled, compressed, restored and moved): byte j of row i = low byte of (key_i * 0x9E3779B1 + j).
    Only the key's low byte matters for that, so it is computed in uint8 (no [n, row_bytes] int64
    temporary): ((key & 0xFF) * 0xB1 + j) mod 256."""
    base = ((keys & 0xFF) * 0xB1 & 0xFF).to(torch.uint8)
    j = torch.arange(row_bytes, device=keys.device, dtype=torch.int64).to(torch.uint8)
    return base.unsqueeze(1) + j.unsqueeze(0)  # uint8 addition wraps mod 256


def _count_at(keys: torch.Tensor, num_partitions: int, mode: str, gid: int) -> int:
    """How many keys the partition function sends to partition `gid` (on the GPU: the K11 histogram)."""
    if keys.numel() == 0:
        return 0
    if keys.is_cuda:
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        n = keys.shape[0]
        cw = torch.zeros((h.partition_groups(n), num_partitions), dtype=torch.int64, device=keys.device)
        h.partition_hist(keys.data_ptr(), n, num_partitions, MODES[mode], cw.data_ptr(),
                         torch.cuda.current_stream(keys.device).cuda_stream)
        return int(cw[:, gid].sum().item())
    return int((destinations(keys, num_partitions, mode) == gid).sum().item())


class OutOfCoreShuffleWorker(ShuffleWorker):
    """One rank of the multi-round Exoshuffle (reference python/ray/experimental/shuffle.py:152
    simple_shuffle / :231 run, map → merge → reduce). Per round the rank generates its next input
    block in HBM, and in ONE collective round K11 partitions it by destination rank, the all-to-all
    exchanges the pieces over xGMI, and K11 partitions what arrived into this rank's P output
    partitions — the merged map output of every mapper for this round. Each (round, partition)
    block is ``ray.put`` into the HBM object store; the store's background spiller moves the least
    recently used blocks to host memory (K4-compressed, pinned DMA) while later rounds are partitioned.
    The reduce of partition p gathers its blocks (restoring spilled ones) and sorts them by key on
    the GPU; destinations, sort order and every payload byte are verified on the GPU.

    Nothing in a map round waits for the host except the [P] partition counts: the input block is
    generated on the device, its checksum accumulates on the device, puts are asynchronous."""

    def setup(self, partitions: int, row_bytes: int, rows_per_round: int, mode: str = "range"):
        self.P, self.row_bytes, self.rows = int(partitions), int(row_bytes), int(rows_per_round)
        self.mode = mode
        self.blocks = [[] for _ in range(self.P)]
        self.in_rows = 0
        self._in_sum = torch.zeros((), dtype=torch.int64, device=self.device)  # wraps mod 2^64
        prepin_s = 0.0
        if self.device.type == "cuda":
            # start-up, like the reference's plasma preallocation: create this process's HBM store now
            # and let it page-lock its spill arena (gpu_spill_prepin_bytes) before the first round
            from ray_memory_management_amd._private import gpu_object_store as gos
            from ray_memory_management_amd._private.worker import global_worker

            g = gos.process_store(global_worker, self.device.index or 0)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 300:
                done, total = g.prepin_progress()
                if done >= total:
                    break
                time.sleep(0.01)
            prepin_s = time.perf_counter() - t0
        return {"prepin_seconds": prepin_s}

    def map_round(self, r: int):
        import ray_memory_management_amd as ray

        dev = self.device
        t0 = time.perf_counter()
        g = torch.Generator(device=dev).manual_seed(7919 * (r + 1) + self.rank)
        # keys over the whole u64 range: "range" partitioning splits the UNSIGNED key space evenly
        keys = torch.randint(-(2 ** 63), 2 ** 63 - 1, (self.rows,), generator=g, dtype=torch.int64, device=dev)
        vals = _payload(keys, self.row_bytes)
        self.in_rows += int(keys.numel())
        self._in_sum += keys.sum()
        if self.world > 1:
            from ray_memory_management_amd.util.collective.collective import get_group_handle

            pg = get_group_handle(self.group_name).pg
            keys, vals = shuffle(keys, vals, group=pg, mode=self.mode, world_size=self.world, rank=self.rank)
        # merge: this rank's P partitions of everything that arrived (global partition ids
        # rank*P .. rank*P + P - 1 under the same range function)
        k, v, counts = partition(keys, vals, self.world * self.P, self.mode)
        cs = counts.tolist()[self.rank * self.P:(self.rank + 1) * self.P]
        off = 0
        for p, c in enumerate(cs):  # put copies the slice into the store (asynchronously)
            self.blocks[p].append(ray.put((k[off:off + c], v[off:off + c])))
            off += c
        return {"round": r, "seconds": time.perf_counter() - t0, "rows": int(k.numel())}

    def finish_map(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return True

    def reduce_partition(self, p: int):
        import ray_memory_management_amd as ray

        t0 = time.perf_counter()
        parts = ray.get(self.blocks[p])
        if parts:
            keys = torch.cat([x[0] for x in parts]).to(self.device)
            vals = torch.cat([x[1] for x in parts]).to(self.device)
        else:
            keys = torch.empty(0, dtype=torch.int64, device=self.device)
            vals = torch.empty((0, self.row_bytes), dtype=torch.uint8, device=self.device)
        del parts
        keys, order = torch.sort(keys)
        vals = vals[order]
        del order
        gid = self.rank * self.P + p
        n = int(keys.numel())
        dest_ok = _count_at(keys, self.world * self.P, self.mode, gid) == n
        payload_ok, step = True, 1 << 20  # row chunks bound the reference payload's size
        for i in range(0, n, step):
            payload_ok = payload_ok and bool(torch.equal(vals[i:i + step], _payload(keys[i:i + step], self.row_bytes)))
        sorted_ok = bool((keys[1:] >= keys[:-1]).all().item()) if n > 1 else True
        out = {"partition": gid, "rows": n, "key_sum": int(keys.sum().item()) % (1 << 61) if n else 0,
               "ok": dest_ok and payload_ok and sorted_ok, "payload_ok": payload_ok,
               "seconds": time.perf_counter() - t0}
        self.blocks[p] = []  # the partition's blocks are freed with their last reference
        return out

    def inputs(self):
        return {"rows": self.in_rows, "key_sum": int(self._in_sum.item()) % (1 << 61)}

    def gpu_store_stats(self):
        from ray_memory_management_amd._private import gpu_object_store as gos
        from ray_memory_management_amd._private.worker import global_worker

        st = {int(k): dict(v) for k, v in gos.stats(global_worker).items()}
        hs = global_worker.store.stats()  # the host shm store (spill target of HBM blocks / CPU blocks)
        st[-1] = {"host_spilled_bytes_total": int(hs.get("bytes_spilled_total", 0)),
                  "host_restored_bytes_total": int(hs.get("bytes_restored_total", 0))}
        return st


def run_out_of_core_gpu_shuffle(num_workers: int = 1, total_bytes: int = 16 << 30, rounds: int = 16,
                                partitions_per_worker: int = 8, row_bytes: int = 248, backend: str = "nccl",
                                mode: str = "range") -> dict:
    """Driver API (BASELINE config #5): shuffle `total_bytes` of synthetic keyed rows through
    `num_workers` GPU actors in `rounds` rounds, more data than their HBM object-store quota
    (``gpu_object_store_memory``) holds, so partition blocks spill to host memory and are restored
    for the reduce. Returns end-to-end GB/s, per-phase times, spilled / restored bytes and the
    correctness checks (every row once, at its partition, payload intact, partitions sorted)."""
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.util import collective as col

    gpu = backend == "nccl"
    row = 8 + int(row_bytes)
    rows_per_round = max(1, int(total_bytes) // (num_workers * rounds * row))
    Actor = ray.remote(num_gpus=1 if gpu else 0, num_cpus=1)(OutOfCoreShuffleWorker)
    workers = [Actor.remote(r, num_workers, "cuda" if gpu else "cpu") for r in range(num_workers)]
    try:
        if num_workers > 1:
            col.create_collective_group(workers, num_workers, list(range(num_workers)), backend=backend,
                                        group_name=f"oocshuffle-{time.time_ns()}")
        setup = ray.get([w.setup.remote(partitions_per_worker, row_bytes, rows_per_round, mode) for w in workers])
        t0 = time.perf_counter()
        # every round is submitted at once: each actor runs them in order (the collective rounds of
        # several ranks line up), so the driver is off the per-round critical path
        refs = [w.map_round.remote(r) for r in range(rounds) for w in workers]
        ray.get(refs)
        ray.get([w.finish_map.remote() for w in workers])
        t_map = time.perf_counter() - t0
        st_map = ray.get([w.gpu_store_stats.remote() for w in workers])
        red = []
        for p in range(partitions_per_worker):
            red.extend(ray.get([w.reduce_partition.remote(p) for w in workers]))
        elapsed = time.perf_counter() - t0
        st_end = ray.get([w.gpu_store_stats.remote() for w in workers])
        ins = ray.get([w.inputs.remote() for w in workers])
    finally:
        for w in workers:
            ray.kill(w)
    in_rows = sum(x["rows"] for x in ins)
    in_sum = sum(x["key_sum"] for x in ins) % (1 << 61)
    out_rows = sum(x["rows"] for x in red)
    out_sum = sum(x["key_sum"] for x in red) % (1 << 61)

    def tot(stats, key):
        return sum(int(v.get(key, 0)) for s in stats for v in s.values())

    data = in_rows * row
    return {"ok": all(x["ok"] for x in red) and in_rows == out_rows and in_sum == out_sum,
            "rows": in_rows, "bytes": data, "GBps": data / elapsed / 1e9, "seconds": elapsed,
            "map_seconds": t_map, "reduce_seconds": elapsed - t_map, "rounds": rounds,
            "partitions": partitions_per_worker * num_workers, "workers": num_workers,
            "setup_prepin_seconds": max(s["prepin_seconds"] for s in setup),
            "payload_ok": all(x["payload_ok"] for x in red),
            "partition_rows_min": min((x["rows"] for x in red), default=0),
            "partition_rows_max": max((x["rows"] for x in red), default=0),
            "spilled_bytes": tot(st_end, "spilled_bytes_total"), "spilled_host_bytes": tot(st_end, "spilled_host_bytes_total"),
            "restored_bytes": tot(st_end, "restored_bytes_total"), "spilled_after_map": tot(st_map, "spilled_bytes_total"),
            "gpu_store_capacity": tot(st_end, "capacity"),
            # one host store per node: every worker reports the same counters
            "host_store_spilled_bytes": max(int(s.get(-1, {}).get("host_spilled_bytes_total", 0)) for s in st_end),
            "host_store_restored_bytes": max(int(s.get(-1, {}).get("host_restored_bytes_total", 0)) for s in st_end)}
