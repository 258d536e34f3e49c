"""GPU objects through the public API on a real MI355X: ray.put/get of HIP tensors, cross-process
zero-copy (hipIPC/dmabuf) reads, copy-on-put semantics, LRU spill to host under HBM pressure, and
lineage reconstruction when the process owning a GPU object dies.
North-star component M8 (the reference has no GPU object store; its closest behaviour is
test_object_spilling.py / test_reconstruction.py on host objects)."""
import os
import signal
import time

import pytest

import ray_memory_management_amd as ray

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu_ray():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ray.init(num_cpus=2, num_gpus=1, object_store_memory=1 << 30,
             _system_config={"gpu_object_store_memory": 2 << 30, "gpu_object_store_slab_bytes": 512 << 20})
    yield ray
    ray.shutdown()


def test_put_get_same_process_copy_semantics(gpu_ray):
    import torch

    t = torch.randn(1 << 20, device="cuda", dtype=torch.bfloat16)
    ref = ray.put(t)
    expect = t.clone()
    t.add_(1.0)  # mutating the source after put must not change the stored object
    got = ray.get(ref)
    assert got.device.type == "cuda" and got.dtype == torch.bfloat16
    assert torch.equal(got, expect)


def test_cross_process_zero_copy_read(gpu_ray):
    import torch

    t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    ref = ray.put(t)

    @ray.remote(num_gpus=1)
    def consume(x):
        assert x.is_cuda
        return float(x.double().sum().item()), os.getpid()

    s, pid = ray.get(consume.remote(ref))
    assert pid != os.getpid()
    assert s == float(t.double().sum().item())


def test_task_returns_gpu_tensor(gpu_ray):
    import torch

    @ray.remote(num_gpus=1)
    def make(n):
        return torch.full((n,), 3.0, device="cuda", dtype=torch.float16)

    out = ray.get(make.remote(4096))
    assert out.is_cuda and out.shape == (4096,)
    assert torch.all(out == 3.0)


def test_spill_and_restore_under_hbm_pressure(gpu_ray):
    import torch

    # 2 GiB GPU store cap: 6 x 512 MiB objects force LRU spill of the oldest to host memory
    refs, sums = [], []
    for i in range(6):
        t = torch.full((256 << 20,), float(i), device="cuda", dtype=torch.bfloat16)
        refs.append(ray.put(t))
        sums.append(float(i))
        del t
    torch.cuda.synchronize()
    for r, v in zip(refs, sums):
        x = ray.get(r)
        assert x.shape == (256 << 20,)
        assert float(x[0].float()) == v and float(x[-1].float()) == v
        del x


def test_gpu_object_reconstructed_when_owner_dies(gpu_ray, tmp_path):
    import torch

    counter = tmp_path / "count"

    @ray.remote(num_gpus=1, num_returns=2, max_retries=2)
    def make(path):
        with open(path, "a") as f:
            f.write("x")
        return os.getpid(), torch.full((1 << 16,), 5.0, device="cuda")

    pid_ref, t_ref = make.remote(str(counter))
    pid = ray.get(pid_ref)
    v = ray.get(t_ref)
    assert float(v[0]) == 5.0
    del v
    os.kill(pid, signal.SIGKILL)
    deadline = time.time() + 60
    while time.time() < deadline and counter.read_text() != "xx":
        time.sleep(0.1)
    again = ray.get(t_ref, timeout=60)
    assert float(again.sum()) == 5.0 * (1 << 16)
    assert counter.read_text() == "xx"


def test_freed_object_not_recycled_while_reader_holds_view(gpu_ray):
    """The owner must not recycle HBM whose descriptor a reader in another process still pins
    (a temporary ref dropped right after get): the free is deferred until the view dies."""
    import torch

    @ray.remote(num_gpus=1)
    class Owner:
        def make(self, v, n):
            return torch.full((n,), float(v), device="cuda")

        def gpu_objects(self):
            from ray_memory_management_amd._private import gpu_object_store as gos
            from ray_memory_management_amd._private.worker import global_worker

            return sum(s["num_objects"] for s in gos.stats(global_worker).values())

    o = Owner.remote()
    x = ray.get(o.make.remote(1.0, 1 << 20))  # the ref is a temporary: refcount drops to 0 now
    time.sleep(0.5)  # FREE_GPU reaches the owner, which must defer (the view pins the descriptor)
    ys = [ray.get(o.make.remote(2.0 + i, 1 << 20)) for i in range(4)]  # would reuse the region
    torch.cuda.synchronize()
    assert float(x.min()) == 1.0 and float(x.max()) == 1.0
    for i, y in enumerate(ys):
        assert float(y.min()) == 2.0 + i
    del x, ys, y  # (y: the loop variable still references the last view)
    deadline = time.time() + 20
    while time.time() < deadline and ray.get(o.gpu_objects.remote()) > 0:
        time.sleep(0.1)
    assert ray.get(o.gpu_objects.remote()) == 0  # deferred frees completed once the views died


def test_killed_cross_process_reader_releases_hbm(gpu_ray):
    """A reader in another process maps an HBM object zero-copy (its view pins the descriptor in the
    shm store) and is SIGKILLed while holding it: the head releases the dead client's store pins
    (Store::ReleaseClient), the descriptor goes, and the owner's deferred free recycles the HBM."""
    import torch

    from ray_memory_management_amd._private import gpu_object_store as gos
    from ray_memory_management_amd._private.worker import global_worker

    def n_objects():
        return sum(s["num_objects"] for s in gos.stats(global_worker).values())

    @ray.remote(num_gpus=0.5)
    class Reader:
        def hold(self, refs):
            self.x = ray.get(refs[0])  # zero-copy hipIPC view: pins the descriptor
            return float(self.x.sum())

    base = n_objects()
    ref = ray.put(torch.ones(1 << 22, device="cuda"))
    assert n_objects() == base + 1
    r = Reader.remote()
    assert ray.get(r.hold.remote([ref])) == float(1 << 22)
    oid = ref.binary()
    ray.kill(r)
    del ref
    deadline = time.time() + 20
    while time.time() < deadline and n_objects() > base:
        time.sleep(0.1)
    st = global_worker.store
    assert n_objects() == base, (gos.stats(global_worker), "descriptor state", st.state(oid),
                                 "deferred", len(getattr(global_worker, "_gpu_deferred_free", ())),
                                 "pin overflows", st.pin_overflows())


def test_nested_cuda_tensors_stay_in_hbm(gpu_ray):
    import torch

    @ray.remote(num_gpus=1)
    def make():
        return {"a": torch.arange(1000, device="cuda", dtype=torch.float32),
                "b": [torch.ones(7, device="cuda", dtype=torch.bfloat16), 3]}

    d = ray.get(make.remote())
    assert d["a"].is_cuda and d["b"][0].is_cuda and d["b"][1] == 3
    assert float(d["a"].sum()) == sum(range(1000)) and float(d["b"][0].sum()) == 7.0
    # and a dict put from the driver round-trips through a task on the same GPU
    r = ray.put({"x": torch.full((64,), 4.0, device="cuda")})

    @ray.remote(num_gpus=1)
    def total(dd):
        return float(dd["x"].sum())

    assert ray.get(total.remote(r)) == 256.0


def test_object_created_in_place_is_returned_without_copy(gpu_ray):
    """create_object / publish_created: an actor writes a GPU-store object in place (a producer kernel's
    output buffer), returns its handle nested in a value, the driver reads it zero-copy (descriptor sealed
    at once after a sync, or by the host callback), and dropping the reference frees the HBM."""
    import torch

    @ray.remote(num_gpus=1)
    class Producer:
        def make(self, k):
            from ray_memory_management_amd._native import require_hip
            from ray_memory_management_amd._private import gpu_object_store as gos
            from ray_memory_management_amd._private import ids
            from ray_memory_management_amd._private.worker import global_worker as w

            src = torch.arange(3 * 1000, device="cuda", dtype=torch.int32).reshape(3, 1000) + k
            oid = ids.new_put_id()
            ptr = gos.create_object(w, oid, (3, 1000), torch.int32, 0)
            s = torch.cuda.current_stream()
            require_hip().memcpy_async(ptr, src.data_ptr(), src.numel() * 4, s.cuda_stream)
            if k == 1:  # the descriptor sealed at once (the copy is done) ...
                s.synchronize()
            puts = gos.stats(w)
            # ... or by the host callback after the copy on `s`
            h = gos.publish_created(w, oid, (3, 1000), torch.int32, 0, s.cuda_stream, synced=k == 1)
            return {"x": h, "k": k, "puts": sum(v["puts"] for v in puts.values())}

        def n_objects(self):
            from ray_memory_management_amd._private import gpu_object_store as gos
            from ray_memory_management_amd._private.worker import global_worker as w

            return sum(v["num_objects"] for v in gos.stats(w).values())

    p = Producer.remote()
    for k in range(3):
        d = ray.get(p.make.remote(k))
        assert d["k"] == k and d["x"].is_cuda and d["x"].dtype == torch.int32 and d["x"].shape == (3, 1000)
        assert torch.equal(d["x"].cpu(), torch.arange(3000, dtype=torch.int32).reshape(3, 1000) + k)
        assert d["puts"] == k + 1  # one store allocation per call: the handle was not copied again
        del d
    deadline = time.time() + 20
    while time.time() < deadline and ray.get(p.n_objects.remote()) > 0:
        time.sleep(0.1)
    assert ray.get(p.n_objects.remote()) == 0


def test_cross_gpu_pull_path_with_quota(gpu_ray):
    """Forced peer path (RMM_TEST_FORCE_PEER_COPY): the consumer imports the owner's slab and DMAs
    the object into its own memory under the pull quota instead of aliasing it."""
    import torch

    t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    ref = ray.put(t)

    @ray.remote(num_gpus=1, runtime_env={"env_vars": {"RMM_TEST_FORCE_PEER_COPY": "1"}})
    def consume(x):
        from ray_memory_management_amd._private import gpu_object_store as gos

        x.add_(1.0)  # a private replica: mutating it must not touch the owner's object
        return float(x.double().sum()), gos.pull_stats()

    s, st = ray.get(consume.remote(ref))
    assert s == float(t.double().sum()) + (1 << 20)
    assert st["pulls"] == 1 and st["bytes_pulled"] == t.numel() * 4
    assert torch.equal(ray.get(ref), t)


def test_async_put_then_cross_process_read(gpu_ray):
    """put() returns before the device copy finishes; a reader in another process waits for the
    descriptor seal (host callback after the copy) and sees complete data."""
    import torch

    big = torch.randn(64 << 20, device="cuda", dtype=torch.bfloat16)  # 128 MiB copy
    refs = [ray.put(big) for _ in range(3)]

    @ray.remote(num_gpus=1)
    def checksum(x):
        return float(x.float().sum())

    want = float(big.float().sum())
    assert all(abs(v - want) <= 1e-3 * abs(want) + 1e-3 for v in ray.get([checksum.remote(r) for r in refs]))


def test_owner_frees_unescaped_object_immediately(gpu_ray):
    """A put whose ref never left the owner is freed by the owner the moment the last ref dies
    (no head round trip); a ref handed to a task is not, and the owner-local view keeps its HBM."""
    import torch

    from ray_memory_management_amd._private import gpu_object_store as gos
    from ray_memory_management_amd._private.worker import global_worker

    def n_objs():
        return sum(s["num_objects"] for s in gos.stats(global_worker).values())

    base = n_objs()
    t = torch.ones(1 << 20, device="cuda")
    r = ray.put(t)
    torch.cuda.synchronize()
    deadline = time.time() + 5
    while global_worker.store.state(r.binary()) != 2 and time.time() < deadline:
        time.sleep(0.001)  # async put: descriptor sealed by the HIP host callback
    assert n_objs() == base + 1
    del r
    assert n_objs() == base  # freed synchronously inside `del`
    # a view obtained by get pins the HBM until the tensor dies
    r = ray.put(t * 3)
    torch.cuda.synchronize()
    while global_worker.store.state(r.binary()) != 2 and time.time() < deadline:
        time.sleep(0.001)
    v = ray.get(r)
    del r
    r2 = ray.put(t * 5)  # must not reuse v's region
    torch.cuda.synchronize()
    assert float(v.min()) == 3.0 and float(v.max()) == 3.0
    del v, r2

    @ray.remote(num_gpus=1)
    def total(x):
        return float(x.sum())

    r = ray.put(t)
    out = total.remote(r)
    assert r.binary() not in global_worker._gpu_unescaped  # escaped into a task
    assert ray.get(out) == float(1 << 20)


def test_large_arg_with_nested_cuda_tensor_does_not_leak(gpu_ray):
    """A task arg holding a CUDA tensor AND enough host data to travel by reference is serialized
    once: its nested GPU object is contained in the by-ref object and freed with it."""
    import numpy as np
    import torch

    from ray_memory_management_amd._private import gpu_object_store as gos
    from ray_memory_management_amd._private.worker import global_worker

    def n_objs():
        return sum(s["num_objects"] for s in gos.stats(global_worker).values())

    @ray.remote(num_gpus=1)
    def use(d):
        return float(d["t"].sum()) + float(d["x"].sum())

    base = n_objs()
    for _ in range(3):
        assert ray.get(use.remote({"x": np.ones(1 << 16), "t": torch.ones(1024, device="cuda")})) == 1024.0 + (1 << 16)
    deadline = time.time() + 20
    while time.time() < deadline and n_objs() > base:
        time.sleep(0.1)
    assert n_objs() == base


def test_share_node_devices_plan(monkeypatch):
    """Visible-device sharing for collective groups (reference backend_executor
    _share_cuda_visible_devices): own GPU 3 of an 8-GPU node -> sees 0..7, selects local index 3."""
    from ray_memory_management_amd._private import gpu_visibility as gv

    assert gv.plan("3", "0,1,2,3,4,5,6,7") == ("0,1,2,3,4,5,6,7", 3)
    assert gv.plan("0", "0") is None            # single-GPU node: nothing to share
    assert gv.plan("", "0,1") is None           # no GPU of its own
    assert gv.plan("9", "0,1") is None          # inconsistent: stay isolated
    monkeypatch.setenv("RMM_GPU_IDS", "5")
    monkeypatch.setenv("RMM_NODE_GPU_IDS", "0,1,2,3,4,5,6,7")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    monkeypatch.delenv("RMM_SHARED_VISIBLE_DEVICES", raising=False)
    monkeypatch.setattr(gv, "_hip_initialized", lambda: False)
    assert gv.share_node_devices() == 5
    import os

    assert os.environ["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7"
    assert gv.current_own_index() == 5
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    monkeypatch.delenv("RMM_SHARED_VISIBLE_DEVICES")
    monkeypatch.setattr(gv, "_hip_initialized", lambda: True)  # too late: stays isolated
    assert gv.share_node_devices() == 0 and os.environ["HIP_VISIBLE_DEVICES"] == "5"
    monkeypatch.setattr(gv, "_hip_initialized", lambda: False)
    monkeypatch.setenv("RMM_SHARE_VISIBLE_DEVICES", "0")
    assert gv.share_node_devices() == 0 and os.environ["HIP_VISIBLE_DEVICES"] == "5"
