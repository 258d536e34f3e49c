"""A minimal communicator handle for learners: all-reduce / broadcast on either the default
``torch.distributed`` group (torchrun ranks) or a ``util.collective`` group (learner actors whose
RCCL group was rendezvoused through the runtime).

Parity: the reference's multi-GPU learner averages tower gradients in-process
(rllib/execution/multi_gpu_learner_thread.py) and DD-PPO all-reduces with torch.distributed
(rllib/algorithms/ddppo/ddppo.py:_sample_and_train_torch_distributed). Here one object hides which
process group carries the collective so the fused PPO learner code is the same in both cases.

``allreduce(t, stream=...)`` can run the collective on a dedicated comm stream: the caller records
an event on its compute stream, the comm stream waits for it, and RCCL launches there — compute
that does not depend on the reduced buffer keeps running (the overlap the PPO learner uses to hide
the dense-bucket all-reduce behind the trunk backward).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist


class _Done:
    def wait(self):
        return True


class Comm:
    world: int = 1
    rank: int = 0

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> None:
        raise NotImplementedError

    def allreduce_async(self, t: torch.Tensor, op: str = "sum"):
        """Start an all-reduce; returns a handle whose wait() orders the caller's current stream
        (RCCL) or host (gloo) after it. Compute issued before wait() overlaps the collective."""
        self.allreduce(t, op)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        pass


class LocalComm(Comm):
    """World of one: every collective is the identity."""

    def allreduce(self, t, op="sum"):
        return None

    def broadcast(self, t, src=0):
        return None


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchDistComm(Comm):
    """The default (or a registered) torch.distributed group."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def allreduce(self, t, op="sum"):
        dist.all_reduce(t, op=_OPS[op], group=self.group)

    def allreduce_async(self, t, op="sum"):
        return dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=True)

    def broadcast(self, t, src=0):
        g = dist.get_global_rank(self.group, src) if self.group is not None else src
        dist.broadcast(t, src=g, group=self.group)

    def barrier(self):
        dist.barrier(group=self.group)


class GroupComm(Comm):
    """A util.collective group (a bare ProcessGroup object: RCCL for GPU tensors, its gloo side
    channel for CPU tensors). Works identically in actors and plain processes."""

    def __init__(self, group_name: str):
        from ray_memory_management_amd.util.collective import collective as col

        self.name = group_name
        self._g = col.get_group_handle(group_name)
        self.world = self._g.world_size
        self.rank = self._g.rank

    def allreduce(self, t, op="sum"):
        from ray_memory_management_amd.util.collective import collective as col

        col.allreduce(t, self.name, {"sum": col.ReduceOp.SUM, "max": col.ReduceOp.MAX,
                                     "min": col.ReduceOp.MIN}[op])

    def allreduce_async(self, t, op="sum"):
        from ray_memory_management_amd.util.collective import collective as col

        return col.allreduce_async(t, self.name, {"sum": col.ReduceOp.SUM, "max": col.ReduceOp.MAX,
                                                  "min": col.ReduceOp.MIN}[op])

    def broadcast(self, t, src=0):
        from ray_memory_management_amd.util.collective import collective as col

        col.broadcast(t, src, self.name)

    def barrier(self):
        from ray_memory_management_amd.util.collective import collective as col

        col.barrier(self.name)


_RCCL_DT = None


def _rccl_dtypes(h):
    global _RCCL_DT
    if _RCCL_DT is None:
        _RCCL_DT = {torch.float32: h.NCCL_FLOAT32, torch.bfloat16: h.NCCL_BFLOAT16, torch.float16: h.NCCL_FLOAT16,
                    torch.int32: h.NCCL_INT32, torch.int64: h.NCCL_INT64, torch.uint8: h.NCCL_UINT8,
                    torch.float64: h.NCCL_FLOAT64}
    return _RCCL_DT


def rehearsal_host_id(tag: str, rank: int) -> None:
    """1-GPU rehearsal of a multi-GPU RCCL group (``RMM_RCCL_SAME_DEVICE=1``): RCCL refuses two
    ranks on one device of one host, so each rank claims its own host id and the ranks talk over
    the socket transport on loopback. Functional only (the xGMI path needs one GPU per rank).
    Must run before the process's first RCCL call."""
    if os.environ.get("RMM_RCCL_SAME_DEVICE") == "1":
        os.environ["NCCL_HOSTID"] = f"rmm-{tag}-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")


class _StreamJoin:
    def __init__(self, cs):
        self.cs = cs

    def wait(self):
        torch.cuda.current_stream(self.cs.device).wait_stream(self.cs)
        return True


class RcclComm(Comm):
    """A communicator the framework owns (csrc/hip/rccl_comm.cc), not torch.distributed's:

    * collectives are enqueued on the stream the caller names, so they can be CAPTURED in a HIP
      graph (``graph_capturable``) — the PPO learner forks its bucket all-reduces onto
      ``self.stream`` inside the per-minibatch graph, next to the trunk backward;
    * rendezvous: rank 0 makes the 128-byte unique id and publishes it in `store` (any
      torch.distributed Store, e.g. the util.collective FileStore in the session directory).

    Reference parity: the role of rllib/execution/multi_gpu_learner_thread.py's tower averaging and
    util/collective/collective_group/nccl_collective_group.py's communicator cache."""

    graph_capturable = True

    def __init__(self, store, rank: int, world: int, key: str = "rmm-rccl-uid", device=None):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        h.rccl_load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
        rehearsal_host_id(key, rank)
        if rank == 0:
            uid = h.rccl_unique_id()
            store.set(key, uid)
        else:
            uid = store.get(key)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._h = h
        self._c = h.RcclComm(bytes(uid), int(world), int(rank), self.device.index)
        self.world, self.rank = int(world), int(rank)
        self.stream = torch.cuda.Stream(self.device)  # comm stream (forked to inside graphs)
        self._ops = {"sum": h.NCCL_SUM, "max": h.NCCL_MAX, "min": h.NCCL_MIN, "prod": h.NCCL_PROD}

    def _args(self, t):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm collectives need contiguous device tensors")
        return t.data_ptr(), t.numel(), _rccl_dtypes(self._h)[t.dtype]

    def allreduce_on(self, t, stream, op="sum"):
        p, n, dt = self._args(t)
        self._c.all_reduce(p, p, n, dt, self._ops[op], stream.cuda_stream)

    def allreduce(self, t, op="sum"):
        self.allreduce_on(t, torch.cuda.current_stream(self.device), op)

    def allreduce_async(self, t, op="sum"):
        """Fork onto the comm stream; wait() joins the caller's current stream back."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        self.allreduce_on(t, self.stream, op)
        t.record_stream(self.stream)
        return _StreamJoin(self.stream)

    def broadcast(self, t, src=0):
        p, n, dt = self._args(t)
        self._c.broadcast(p, p, n, dt, int(src), torch.cuda.current_stream(self.device).cuda_stream)

    def barrier(self):
        x = torch.zeros(1, device=self.device)
        self.allreduce(x)
        torch.cuda.current_stream(self.device).synchronize()

    def check(self):
        """Raise if the communicator hit an asynchronous error (e.g. a peer died)."""
        e = self._c.async_error()
        if e:
            raise RuntimeError(f"RCCL communicator error: {e}")

    def close(self):
        try:
            self._c.destroy()
        except Exception:
            self._c.abort()


_PEER_DT = {torch.bfloat16: 0, torch.float32: 1}


class PeerUnavailable(RuntimeError):
    """Some rank could not export or map the peer regions (e.g. no IPC / peer access)."""


def _store_barrier(store, key: str, world: int, timeout_s: float = 300.0) -> None:
    store.add(key, 1)
    t0 = time.monotonic()
    while int(store.add(key, 0)) < world:
        if time.monotonic() - t0 > timeout_s:
            raise TimeoutError(f"store barrier {key}: {int(store.add(key, 0))}/{world} ranks arrived")
        time.sleep(0.002)


class _FlatView:
    """(pointer, element count) of an fp32 device range handed to the native communicator."""

    def __init__(self, ptr: int, count: int, device):
        if ptr % 16:
            raise ValueError("PeerComm: 16-B aligned fp32 ranges only")
        self.ptr, self.count, self.device = ptr, count, device


def zero1_blocks_for(h, device: int, ranks_on_device: int = 1, cap: int = 256, concurrent_per_cu: int = 1) -> int:
    """Workgroups of the ZeRO-1 launch, from the kernel's occupancy instead of a constant.

    Every workgroup of `k_peer_zero1` waits (bounded) on its peers' same-index workgroups, so ALL the
    workgroups of every rank driving the GPU must be resident at once, next to the kernels the learner
    runs concurrently on its compute stream (fork mode: the trunk backward, one 512-thread workgroup per
    CU): per rank ((zero1 workgroups per CU - concurrent_per_cu) x CUs) / ranks on the device, capped at
    `cap` (256 measured best for the fp32 PPO bucket on one GPU per rank: the Adam pass over 1/W of the
    bucket is latency-bound at 64), rounded down to a multiple of 8, at least 8."""
    try:
        occ = h.peer_occupancy(int(device))
        slots = max(0, int(occ["zero1_per_cu"]) - int(concurrent_per_cu)) * int(occ["cus"])
    except Exception:  # noqa: BLE001 - no query: the conservative all-reduce count
        return 64
    n = min(int(cap), slots // max(1, int(ranks_on_device)))
    if int(ranks_on_device) >= 8:
        # 8 ranks on one device (1-GPU rehearsals): 32 spinning workgroups per rank kept a slot busy on every
        # CU and a lagging rank's trunk kernels (one ~150 KB-LDS workgroup per CU) could not run; 8 completes
        # (profiles/multirank_r6.txt)
        n = 8
    return max(8, n - n % 8)


class PeerComm(Comm):
    """MI355X-native intra-node all-reduce (csrc/hip/peer_allreduce.hip): every rank exports a
    staging region once through hipIPC and maps every peer's; one kernel per all-reduce reads the
    peers' slices over xGMI, sums them in fp32 in rank order and rounds once, with per-workgroup
    flag barriers (bounded spins that report a dead peer instead of hanging). No host involvement
    per call, so the collective lives INSIDE the learner's chained SGD graph (``in_graph``).

    bf16 / fp32 sums natively, plus the ZeRO-1 optimizer step (`allreduce_adam_on`); `broadcast` of
    a device tensor is an all-reduce against zeros from the other ranks, bit-exact for every dtype
    (bf16 / fp32 directly, anything else as its raw bytes); host tensors and other ops go to
    `fallback` (an RcclComm or a torch group) when one is given. Reference parity: rllib/execution/multi_gpu_learner_thread.py:20 (tower gradient
    averaging), rllib/execution/train_ops.py:98."""

    graph_capturable = True
    in_graph = True

    def __init__(self, store, rank: int, world: int, key: str = "rmm-peer", device=None,
                 cap_bytes: int = 8 << 20, nblocks: int = 0, timeout_s: float = 0.0, fallback: Optional[Comm] = None,
                 zero1_blocks: Optional[int] = None):
        from ray_memory_management_amd._native import require_hip

        h = require_hip()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.world, self.rank = int(world), int(rank)
        timeout_s = timeout_s or float(os.environ.get("RMM_PEER_TIMEOUT_S", "60"))
        try:  # which physical GPU each rank drives: ranks sharing one only contend when they overlap
            bus = h.pci_bus_id(self.device.index).encode()
        except Exception:  # noqa: BLE001
            bus = f"?{self.rank}".encode()
        store.set(f"{key}/bus{self.rank}", bus)
        buses = [store.get(f"{key}/bus{r}") for r in range(self.world)]
        #: True when some ranks share a physical GPU (1-GPU rehearsals, several learners per GPU)
        self.shared_device = len(set(buses)) < self.world
        #: ranks driving this rank's physical GPU (1 = one process per GPU)
        self.ranks_on_device = max(1, buses.count(buses[self.rank]))
        # one workgroup per CU would saturate the links long before the payload does; 64 keeps the
        # barrier fan-in small (64 x W flags) and still leaves most of the chip to the trunk kernels
        # (8 when 8 ranks share the device: see zero1_blocks_for)
        nblocks = nblocks or int(os.environ.get("RMM_PEER_BLOCKS", "64" if self.ranks_on_device < 8 else "8"))
        # every rank reaches every store key even when its own setup fails, so the ranks agree on
        # the outcome (all PeerComm, or all raise PeerUnavailable and fall back) instead of hanging
        err, blob, self._c = None, b"", None
        try:
            self._c = h.PeerAllReduce(self.rank, self.world, self.device.index, int(cap_bytes), int(nblocks),
                                      float(timeout_s))
            blob = self._c.handles()
        except Exception as e:  # noqa: BLE001
            err = e
        store.set(f"{key}/h{self.rank}", blob)
        hs = [store.get(f"{key}/h{r}") for r in range(self.world)]
        ok = err is None and all(len(b) > 0 for b in hs)
        if ok:
            try:
                self._c.open(hs)
            except Exception as e:  # noqa: BLE001
                err, ok = e, False
        store.set(f"{key}/ok{self.rank}", b"1" if ok else b"0")
        bad = [r for r in range(self.world) if store.get(f"{key}/ok{r}") != b"1"]
        if bad:
            if self._c is not None:
                self._c.close()
            raise PeerUnavailable(f"peer all-reduce unavailable (ranks {bad} failed; here: {err!r})")
        # nobody launches before every rank mapped every region
        _store_barrier(store, f"{key}/ready", self.world)
        self.fallback = fallback
        self.stream = torch.cuda.Stream(self.device)
        self.algo = int(os.environ.get("RMM_PEER_ALGO", "0"))
        # self-test before anyone relies on it: one small all-reduce under a short flag timeout,
        # checked on every rank; the ranks agree through the store, and any failure (a peer mapping
        # the kernel cannot reach, a timeout, a wrong sum) makes ALL of them fall back together
        ok = True
        try:
            self._c.set_timeout(5.0)
            x = torch.full((1024,), float(self.rank + 1), dtype=torch.float32, device=self.device)
            self.allreduce(x)
            torch.cuda.synchronize(self.device)
            want = self.world * (self.world + 1) / 2.0
            ok = int(self._c.error()) == 0 and bool((x == want).all().item())
        except Exception:  # noqa: BLE001
            ok = False
        finally:
            try:
                self._c.set_timeout(float(timeout_s))
            except Exception:  # noqa: BLE001
                pass
        store.set(f"{key}/test{self.rank}", b"1" if ok else b"0")
        bad = [r for r in range(self.world) if store.get(f"{key}/test{r}") != b"1"]
        if bad:
            self._c.close()
            raise PeerUnavailable(f"peer all-reduce self-test failed on ranks {bad}")
        # the ZeRO-1 optimizer launch (allreduce_adam_on) runs on its OWN communicator: its Adam pass
        # over 1/W of the bucket wants many more workgroups than the plain all-reduce's barrier fan-in
        # does (64 -> 256: the fp32 PPO bucket's step on 64 workgroups was latency-bound), and one
        # communicator must keep one workgroup count (its staging reuse is argued per workgroup slice)
        if zero1_blocks is None:
            env = os.environ.get("RMM_PEER_ZERO1_BLOCKS")
            zero1_blocks = int(env) if env else zero1_blocks_for(h, self.device.index, self.ranks_on_device)
        self.zero1_blocks = int(zero1_blocks)
        self._cz = None
        if zero1_blocks > 0:
            zerr, zblob = None, b""
            try:
                self._cz = h.PeerAllReduce(self.rank, self.world, self.device.index, int(cap_bytes),
                                           int(zero1_blocks), float(timeout_s))
                zblob = self._cz.handles()
            except Exception as e:  # noqa: BLE001
                zerr = e
            store.set(f"{key}/zh{self.rank}", zblob)
            zhs = [store.get(f"{key}/zh{r}") for r in range(self.world)]
            zok = zerr is None and all(len(b) > 0 for b in zhs)
            if zok:
                try:
                    self._cz.open(zhs)
                except Exception:  # noqa: BLE001
                    zok = False
            store.set(f"{key}/zok{self.rank}", b"1" if zok else b"0")
            if any(store.get(f"{key}/zok{r}") != b"1" for r in range(self.world)):
                if self._cz is not None:
                    self._cz.close()
                self._cz = None  # every rank agrees: plain all-reduce -> Adam
            _store_barrier(store, f"{key}/zready", self.world)
            if self._cz is not None:
                self._zero1_selftest(store, key, timeout_s)

    def _zero1_selftest(self, store, key: str, timeout_s: float) -> None:
        """One small ZeRO-1 launch before the learner relies on it (as the all-reduce self-test above): every
        rank's gradient is rank + 1, so after the first Adam step every master element is -lr (Adam's first
        step is lr x sign), on every rank, bit for bit. Any failure (a flag timeout, a wrong or diverging
        master) closes the ZeRO-1 communicator on ALL ranks together; the learner then runs all-reduce -> K6."""
        import hashlib

        n = 8192 * self.world
        ok = True
        digest = b""
        try:
            self._cz.set_timeout(5.0)
            d = self.device
            g = torch.full((n,), float(self.rank + 1), dtype=torch.float32, device=d)
            master, m1, m2 = (torch.zeros(n, dtype=torch.float32, device=d) for _ in range(3))
            whi, wlo = torch.zeros(n, dtype=torch.bfloat16, device=d), torch.zeros(n, dtype=torch.bfloat16, device=d)
            hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0], dtype=torch.float32, device=d)
            st = torch.cuda.current_stream(d)
            self.allreduce_adam_on(g, st, master=master.data_ptr(), m1=m1.data_ptr(), m2=m2.data_ptr(),
                                   whi=whi.data_ptr(), wlo=wlo.data_ptr(), hp=hp.data_ptr(), grad_scale=1.0 / self.world)
            st.synchronize()
            ok = int(self._cz.error()) == 0 and bool((master - (-1e-3)).abs().max().item() < 1e-6)
            digest = hashlib.sha256(master.cpu().numpy().tobytes()).hexdigest().encode()
        except Exception:  # noqa: BLE001
            ok = False
        finally:
            try:
                self._cz.set_timeout(float(timeout_s))
            except Exception:  # noqa: BLE001
                pass
        store.set(f"{key}/ztest{self.rank}", digest if ok else b"bad")
        got = [store.get(f"{key}/ztest{r}") for r in range(self.world)]
        if any(x == b"bad" for x in got) or len(set(got)) != 1:
            self._cz.close()
            self._cz = None
            self.zero1_selftest_failed = True

    @property
    def zero1_ready(self) -> bool:
        """allreduce_adam_on is available (its communicator opened on every rank)."""
        return self._cz is not None

    @property
    def launches(self) -> int:
        return int(self._c.launches) + (int(self._cz.launches) if self._cz is not None else 0)

    def allreduce_on(self, t, stream, op="sum"):
        if op != "sum" or t.dtype not in _PEER_DT or not t.is_cuda or not t.is_contiguous() or t.data_ptr() % 16:
            if self.fallback is None:
                raise ValueError(f"PeerComm: sum of contiguous 16-B aligned bf16/fp32 device tensors only "
                                 f"(got op={op}, dtype={t.dtype})")
            return self.fallback.allreduce(t, op)
        self._c.all_reduce(t.data_ptr(), t.numel(), _PEER_DT[t.dtype], stream.cuda_stream, self.algo)

    def allreduce_adam_on(self, grad, stream, *, master: int, m1: int, m2: int, whi: int, wlo: int = 0, hp: int,
                          grad_scale: float = 1.0, step_ctr: int = 0, bump: int = 0, nbump: int = 0, done: int = 0,
                          bump_next: int = 0) -> None:
        """ZeRO-1 optimizer step in one launch (per `cap / 4` elements): reduce-scatter `grad` (bf16 / fp32,
        summed in fp32 in rank order), K6's Adam on this rank's chunk of the fp32 master / moments (device
        pointers to `grad.numel()` elements) writing the bf16 weight plane `whi` (+ split lo plane `wlo`),
        all-gather of the updated masters. Masters and weights end bit-identical on every rank and equal
        to all-reduce -> K6; m1 / m2 are current on their owner only (`replicate_moments`). Counters as
        K6: Adam step from `step_ctr`, `bump` advanced by the last launch (`done` ticket words or parity
        `bump_next`). Reference: rllib/execution/train_ops.py:98 (the tower-averaged gradient step)."""
        if grad.dtype not in _PEER_DT or not grad.is_cuda or not grad.is_contiguous():
            raise ValueError(f"PeerComm.allreduce_adam_on: contiguous bf16/fp32 device gradient (got {grad.dtype})")
        if self._cz is None:
            raise RuntimeError("PeerComm: the ZeRO-1 communicator is not open (zero1_blocks=0 or setup failed)")
        self._cz.all_reduce_adam(grad.data_ptr(), grad.numel(), _PEER_DT[grad.dtype], stream.cuda_stream,
                                int(master), int(m1), int(m2), int(whi), int(wlo), int(hp), float(grad_scale),
                                int(step_ctr), int(bump), int(nbump), int(done), int(bump_next))

    def replicate_moments(self, grad_dtype, count: int, *bufs, stream=None) -> None:
        """Make fp32 buffers (moment pointers) that `allreduce_adam_on(count elements of grad_dtype)` only
        keeps current on each element's owner identical on every rank: zero the unowned elements, then
        sum (exact: one non-zero term per element)."""
        if self._cz is None:
            raise RuntimeError("PeerComm: the ZeRO-1 communicator is not open (zero1_blocks=0 or setup failed)")
        st = stream or torch.cuda.current_stream(self.device)
        for ptr in bufs:
            t = _FlatView(int(ptr), int(count), self.device)
            self._cz.mask_unowned(int(ptr), int(count), _PEER_DT[grad_dtype], st.cuda_stream)
            self._c.all_reduce(t.ptr, t.count, _PEER_DT[torch.float32], st.cuda_stream, self.algo)

    def allreduce(self, t, op="sum"):
        if t.data_ptr() % 16 and op == "sum" and t.dtype in _PEER_DT and t.is_cuda:
            tmp = t.contiguous().clone()
            self.allreduce_on(tmp, torch.cuda.current_stream(self.device), op)
            t.copy_(tmp)
            return
        self.allreduce_on(t, torch.cuda.current_stream(self.device), op)

    def allreduce_async(self, t, op="sum"):
        """Fork onto the comm stream; wait() joins the caller's current stream back."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        self.allreduce_on(t, self.stream, op)
        t.record_stream(self.stream)
        return _StreamJoin(self.stream)

    def broadcast(self, t, src=0):
        if t.dtype in _PEER_DT and t.is_cuda:
            buf = t if (t.is_contiguous() and t.data_ptr() % 16 == 0) else t.contiguous().clone()
            if self.rank != src:
                buf.zero_()
            self.allreduce(buf)
            if buf is not t:
                t.copy_(buf)
            return
        if t.is_cuda:
            # any other dtype (float64, integers, bool): its raw bytes, one fp32 per byte (0..255 are
            # exact in fp32 and so is x + 0), so the result is bit-exact whatever the dtype
            src_t = t.contiguous().reshape(-1)  # 1-d first: a 0-dim tensor of a wide dtype cannot view as bytes
            f = src_t.view(torch.uint8).float() if src_t.numel() else torch.zeros(0, device=t.device)
            self.broadcast(f, src)
            t.copy_(f.to(torch.uint8).view(t.dtype).view(t.shape))
            return
        if self.fallback is None:
            raise ValueError(f"PeerComm.broadcast: unsupported tensor {t.dtype} on {t.device}")
        self.fallback.broadcast(t, src)

    def barrier(self):
        x = torch.zeros(4, device=self.device)
        self.allreduce(x)
        torch.cuda.current_stream(self.device).synchronize()
        self.check()

    def check(self):
        """Raise if a flag wait timed out (a peer died or never launched its side)."""
        e = int(self._c.error()) or (int(self._cz.error()) if self._cz is not None else 0)
        if e:
            raise RuntimeError(f"PeerComm rank {self.rank}: all-reduce flag wait timed out "
                               f"(peer {(e - 1) & 0xff}, workgroup {((e - 1) >> 8) & 0xffff}, phase {(e - 1) >> 24})")

    def close(self):
        if self._cz is not None:
            self._cz.close()
        self._c.close()


def default_comm(process_group=None) -> Comm:
    """torch.distributed when it is initialised (torchrun ranks), else a world of one."""
    if dist.is_available() and dist.is_initialized():
        c = TorchDistComm(process_group)
        if c.world > 1:
            return c
    return LocalComm()


def as_comm(x: Optional[object]) -> Comm:
    if x is None:
        return default_comm()
    if isinstance(x, Comm):
        return x
    if isinstance(x, str):
        return GroupComm(x)
    return default_comm(x)  # a torch.distributed ProcessGroup
