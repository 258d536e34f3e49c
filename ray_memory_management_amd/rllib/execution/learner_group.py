"""GPU learner actors: N data-parallel PPO learners, one per MI355X, averaging gradients over RCCL.

Parity: reference rllib/execution/multi_gpu_learner_thread.py (MultiGPULearnerThread: towers on
several GPUs, per-minibatch gradient averaging), rllib/execution/train_ops.py:98
(multi_gpu_train_one_step: load the train batch into the per-device buffers, num_sgd_iter x
minibatch SGD) and rllib/algorithms/ddppo/ddppo.py (torch.distributed all-reduce between learner
processes). The reference keeps its towers in the driver process; on an 8-GPU xGMI node a learner
per *process* avoids one Python thread driving eight devices, and the all-reduce of ~2 MB of bf16
gradients per minibatch is one RCCL ring over the point-to-point links.

Data path per training iteration (see PPO.training_step):

* rollout-worker actors return fragments → shared-memory object store (zero-copy pickle5 buffers);
* ``LearnerActor.update(*fragment_refs)`` receives its shard (refs resolved from the store as
  zero-copy numpy views), DMAs it onto its GPU and runs GAE + standardisation there (K17), then the
  fused SGD epochs with one all-reduce of the whole gradient bucket per minibatch step;
* each learner publishes its bf16 weights as ONE flat HBM object (``get_weights_device``) that the
  GPU rollout workers of its bundle map zero-copy (hipIPC); CPU rollout workers read learner 0's
  fp32 weights (``get_weights``) from the shared-memory store in place.
"""
from __future__ import annotations

import os
import time
import uuid
from typing import Dict, List, Optional

import ray_memory_management_amd as ray


class LearnerActor:
    """One PPO learner replica (runs as an actor with one GPU, or on CPU for tests)."""

    def __init__(self, obs_space, action_space, model_config: dict, learner_cfg: dict, rank: int, world: int,
                 group_name: Optional[str], backend: str, seed: int = 0, use_gpu: bool = True):
        import torch

        from ray_memory_management_amd.parallel.comm import GroupComm, LocalComm
        from ray_memory_management_amd.rllib.models import build_model
        from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

        self.rank, self.world = rank, world
        idx = 0
        if use_gpu and world > 1 and backend == "nccl":
            from ray_memory_management_amd._private.gpu_visibility import share_node_devices

            idx = share_node_devices()  # RCCL peers on this node see each other's GPUs
        self.device = f"cuda:{idx}" if use_gpu and torch.cuda.is_available() else "cpu"
        if self.device != "cpu":
            from ray_memory_management_amd._native import require_hip

            require_hip()  # the fused learner needs the HIP kernels: fail loudly if they are missing
            torch.cuda.set_device(idx)
            from ray_memory_management_amd._private.numa import pin_to_gpu

            self.cpu_affinity = pin_to_gpu(idx)  # CPUs local to this GPU (before any buffer is allocated)
        if world > 1 and backend == "nccl" and self.device != "cpu" and not os.environ.get("RMM_TORCH_PG_COMM"):
            # framework-owned RCCL communicator (parallel/comm.py:RcclComm): collectives enqueued on
            # the learner's own stream, capturable in graphs (torch's ProcessGroupNCCL watchdog
            # aborts on captured collectives on ROCm)
            import torch.distributed as dist

            from ray_memory_management_amd.parallel.comm import PeerComm, PeerUnavailable, RcclComm
            from ray_memory_management_amd.util.collective.collective import _store_path

            store = dist.FileStore(_store_path(group_name), world)
            comm = None
            if os.environ.get("RMM_PEER_COMM", "1") != "0":
                # MI355X-native peer-memory all-reduce over xGMI (hipIPC), captured inside the chained
                # SGD graph; RCCL only when some rank cannot map its peers
                try:
                    comm = PeerComm(store, rank, world, key=f"{group_name}-peer", device=idx)
                except PeerUnavailable as e:
                    print(f"[LearnerActor {rank}] {e}; using RCCL", flush=True)
            if comm is None:
                comm = RcclComm(store, rank, world, key=f"{group_name}-rccl")
        elif world > 1:
            from ray_memory_management_amd.util.collective import collective as col

            col.init_collective_group(world, rank, backend, group_name)
            comm = GroupComm(group_name)
        else:
            comm = LocalComm()
        torch.manual_seed(seed)  # every rank builds the same init; rank 0's is broadcast anyway
        model = build_model(obs_space, action_space, model_config)
        self.learner = PPOLearner(model, learner_cfg, device=self.device, action_space=action_space, comm=comm)
        self.update_time = 0.0
        self.updates = 0

    def update(self, *fragments) -> Dict:
        t0 = time.perf_counter()
        stamps = getattr(self, "_stamps", None)
        if stamps is not None:
            stamps.append(("update_start", time.time()))
        st = self.learner.update_fragments(list(fragments))  # ends with a device sync (stats to host)
        dt = time.perf_counter() - t0
        if stamps is not None:
            stamps.append(("update_end", time.time()))
        self.update_time += dt
        self.updates += 1
        st = dict(st)
        st["learner_update_s"] = dt
        st["rank"] = self.rank
        if self.learner._ingest is not None:
            st["ingest_bytes"] = self.learner._ingest.bytes_ingested
            if self.device != "cpu":
                from ray_memory_management_amd._native import require_hip

                d, sg, ok, bad = require_hip().h2d_stats()
                st.update(ingest_direct_bytes=d, ingest_staged_bytes=sg, ingest_chunks_pinned=ok,
                          ingest_chunks_unpinnable=bad)
        return st

    def update_batch(self, batch) -> Dict:
        """Train on an already-postprocessed SampleBatch (rollout workers ran GAE)."""
        import torch

        from ray_memory_management_amd.rllib.sample_batch import SampleBatch

        b = SampleBatch({k: torch.as_tensor(v) for k, v in batch.items()})
        if self.device != "cpu":
            b = b.to_device(self.device)
        return dict(self.learner.update(b))

    def get_weights(self):
        return self.learner.get_weights(numpy=True)

    def get_weights_device(self):
        """The bf16 compute weights as ONE flat HBM tensor (+ per-parameter layout). Returned
        through the HBM object store: a GPU rollout worker on the same device maps it zero-copy
        (hipIPC) and copies each parameter device-to-device — no D2H / pickle / H2D round trip of
        the fp32 masters per iteration."""
        L = self.learner
        if self.device == "cpu" or not getattr(L, "fast", False):
            return self.get_weights()
        names = {id(p): n for n, p in L.model.named_parameters()}
        layout, off = [], 0
        for p in L.params:
            layout.append((names[id(p)], off, tuple(p.shape), tuple(p.stride())))
            off += p.numel()
        # bf16 compute weights, or the fp32 master for a precision-matched (compute_dtype fp32) learner
        flat = L.w_bf16 if L.w_bf16 is not None else L.master
        return {"__rmm_flat_bf16__": flat.detach().clone(), "__rmm_layout__": layout}

    def shared_weights_kind(self):
        """Which live weights this learner can share zero-copy: "bf16" (the bf16 compute weights), "x3"
        (the fp32 learner's split-bf16 pair) or None (CPU / autograd learners: publish copies instead)."""
        L = self.learner
        if self.device == "cpu" or not getattr(L, "fast", False):
            return None
        if L.w_bf16 is not None:
            return "bf16"
        return "x3" if getattr(L, "w_x3", None) is not None else None

    def _layout(self):
        L = self.learner
        names = {id(p): n for n, p in L.model.named_parameters()}
        layout, off = [], 0
        for p in L.params:
            layout.append((names[id(p)], off, tuple(p.shape), tuple(p.stride())))
            off += p.numel()
        return layout

    def shared_weights_device(self):
        """Zero-copy weight sharing with co-located rollout workers (default on): the live compute
        weights (bf16, or the fp32 learner's split pair) move ONCE into HBM objects of this process's GPU
        object store and the learner keeps updating them in place there; a rollout worker on the same
        GPU maps the objects (hipIPC) and points its parameters at them, so no weights move per
        iteration. Safe because the training loop orders every update (ends with a host sync) before
        the next sample, and every sample (ends with a stream sync) before the next update. The owner's
        views pin the objects (never spilled). Learners without live weights to share raise: the
        driver checks shared_weights_kind() first and publishes copies for them."""
        L = self.learner
        kind = self.shared_weights_kind()
        if kind is None:
            raise RuntimeError("this learner has no live device weights to share; publish get_weights_device()")
        if kind == "x3":
            if getattr(self, "_shared", None) is None:
                import ray_memory_management_amd as rt

                # three objects: the fp32 master (the parameters) and its split pair (what the kernels read)
                refs = [rt.put(L.master.detach().clone()), rt.put(L.w_x3.hi.detach().clone()),
                        rt.put(L.w_x3.lo.detach().clone())]
                views = [rt.get(r) for r in refs]  # owner-side zero-copy views (pin the objects)
                L.rebind_master(views[0])
                L.rebind_x3(views[1], views[2])
                self._shared = (refs, views, self._layout())
            refs, _, layout = self._shared
            return {"__rmm_shared_x3__": list(refs), "__rmm_layout__": layout}
        if getattr(self, "_shared", None) is None:
            import os
            import sys

            import ray_memory_management_amd as rt

            ref = rt.put(L.w_bf16.detach().clone())
            view = rt.get(ref)  # owner-side zero-copy view of the HBM object (pins it)
            old = L.w_bf16.data_ptr()
            L.rebind_bf16(view)
            if os.environ.get("RMM_SHARED_WEIGHTS_DEBUG"):
                print(f"[shared-weights] learner pid {os.getpid()}: w_bf16 {old:#x} -> store view "
                      f"{view.data_ptr():#x} .. {view.data_ptr() + view.numel() * 2:#x}", file=sys.stderr, flush=True)
            names = {id(p): n for n, p in L.model.named_parameters()}
            layout, off = [], 0
            for p in L.params:
                layout.append((names[id(p)], off, tuple(p.shape), tuple(p.stride())))
                off += p.numel()
            self._shared = (ref, view, layout)
        ref, _, layout = self._shared
        return {"__rmm_shared_bf16__": [ref], "__rmm_layout__": layout}

    def set_weights(self, w):
        self.learner.set_weights(w)

    def get_state(self):
        return {"weights": self.learner.get_weights(numpy=True), "kl_coeff": self.learner.kl_coeff,
                "timesteps": self.learner.timesteps}

    def set_state(self, s):
        self.learner.set_weights(s["weights"])
        self.learner.kl_coeff = s.get("kl_coeff", self.learner.kl_coeff)
        self.learner.timesteps = s.get("timesteps", self.learner.timesteps)

    def weights_digest(self) -> str:
        """Hash of the fp32 weights: replicas must agree bit-for-bit."""
        import hashlib

        h = hashlib.sha256()
        for k, v in sorted(self.learner.get_weights(numpy=True).items()):
            h.update(k.encode())
            h.update(v.tobytes())
        return h.hexdigest()

    def phase_stamps(self, on: bool = True):
        """Wall-clock (start, end) stamps of every update from now on (hand-off latency probes); returns
        and clears the stamps recorded so far."""
        from ray_memory_management_amd._private import worker as _w

        cw = _w.global_worker
        out = (getattr(self, "_stamps", None) or []) + [("task",) + t for t in (getattr(cw, "task_stamps", None) or [])]
        self._stamps = [] if on else None
        if cw is not None:
            cw.task_stamps = [] if on else None
        return out

    def comm_info(self):
        """Which communicator carries the gradients and whether the SGD-step graph contains them."""
        L = self.learner
        return {"comm": type(L.comm).__name__, "graph_has_comm": bool(L._graph_has_comm),
                "split_graphs": L._graphs_split is not None, "graphs": bool(L.graphs),
                "chain": int(getattr(L, "_chain", 1)), "launches": int(getattr(L.comm, "launches", 0)),
                "zero1": bool(getattr(L, "_zero1", lambda: False)()),
                "zero1_blocks": getattr(L.comm, "zero1_blocks", None),
                "ranks_on_device": getattr(L.comm, "ranks_on_device", None),
                "peer_mode": L._peer_mode() if hasattr(L, "_peer_mode") and L.world > 1 else None}

    def device_info(self):
        import torch

        info = {"rank": self.rank, "device": self.device, "pid": os.getpid(),
                "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
                "comm": type(self.learner.comm).__name__}
        if self.device != "cpu":
            info["pci_bus_id"] = getattr(torch.cuda.get_device_properties(self.device), "pci_bus_id", None)
            info["visible_devices"] = torch.cuda.device_count()
            aff = getattr(self, "cpu_affinity", None)  # NUMA-local pin (None: left to the OS)
            info["cpus"] = f"{len(aff)} GPU-local" if aff else "os"
        return info


class LearnerGroup:
    """Driver-side handle on N LearnerActors (one per GPU; gloo on CPU for tests)."""

    def __init__(self, num_learners: int, obs_space, action_space, model_config: dict, learner_cfg: dict,
                 num_gpus_per_learner: float = 1.0, num_cpus_per_learner: float = 1.0, backend: str = "auto",
                 seed: int = 0, strategy=None):
        """`strategy(rank)` (optional): the learner's scheduling strategy (e.g. its GPU's bundle)."""
        self.n = int(num_learners)
        use_gpu = num_gpus_per_learner > 0
        if backend == "auto":
            backend = "nccl" if use_gpu else "gloo"
        self.backend = backend
        self.group_name = f"learners-{uuid.uuid4().hex[:8]}" if self.n > 1 else None
        cls = ray.remote(LearnerActor).options(num_gpus=num_gpus_per_learner, num_cpus=num_cpus_per_learner)
        # all ranks must be alive together: their constructors rendezvous in the collective group
        self.learners = [(cls.options(scheduling_strategy=strategy(r)) if strategy is not None else cls).remote(
            obs_space, action_space, model_config, learner_cfg, r, self.n, self.group_name, backend, seed, use_gpu)
            for r in range(self.n)]
        ray.get([l.__ray_ready__.remote() for l in self.learners])

    def update(self, shards: List[List]) -> List[Dict]:
        if len(shards) != self.n:
            raise ValueError(f"need one shard per learner ({self.n}), got {len(shards)}")
        return ray.get([l.update.remote(*s) for l, s in zip(self.learners, shards)])

    def update_async(self, shards: List[List]):
        return [l.update.remote(*s) for l, s in zip(self.learners, shards)]

    def weights_ref(self):
        """ObjectRef of learner 0's weights (fp32 numpy dict): pass it straight to the rollout
        workers' set_weights — they read it from the store, the driver never materialises it."""
        return self.learners[0].get_weights.remote()

    def get_weights(self):
        return ray.get(self.weights_ref())

    def shared_kind(self):
        """Learner 0's shareable live-weight kind ("bf16", "x3" or None), asked once."""
        if not hasattr(self, "_shared_kind"):
            self._shared_kind = ray.get(self.learners[0].shared_weights_kind.remote()) if self.learners else None
        return self._shared_kind

    def shared_weights_refs(self) -> List:
        """One shared-weights descriptor per learner (LearnerActor.shared_weights_device)."""
        return [l.shared_weights_device.remote() for l in self.learners]

    def device_weights_refs(self) -> List:
        """One device-weights object per learner (identical replicas): rollout worker i reads
        learner i % n's, which sits on its own GPU (same placement-group bundle)."""
        return [l.get_weights_device.remote() for l in self.learners]

    def set_weights(self, w):
        ray.get([l.set_weights.remote(w) for l in self.learners])

    def get_state(self):
        return ray.get(self.learners[0].get_state.remote())

    def set_state(self, s):
        ray.get([l.set_state.remote(s) for l in self.learners])

    def weights_digests(self) -> List[str]:
        return ray.get([l.weights_digest.remote() for l in self.learners])

    def device_info(self):
        return ray.get([l.device_info.remote() for l in self.learners])

    def stop(self):
        for l in self.learners:
            try:
                ray.kill(l)
            except Exception:
                pass
        self.learners = []
