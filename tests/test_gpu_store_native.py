"""Native HBM GPU object store: put/get zero-copy, LRU spill (with compression) and restore."""
import os
import tempfile
import uuid

import pytest
import torch

pytestmark = pytest.mark.gpu


def _oid():
    return os.urandom(20)


@pytest.fixture
def stores(cuda):
    from ray_memory_management_amd._native import require_hip, store_ext

    h = require_hip()
    name = "/rmm-test-" + uuid.uuid4().hex[:8]
    d = tempfile.mkdtemp()
    host = store_ext().ObjectStore.create_segment(name, 512 << 20, d, 0.8, 1 << 20, True)
    g = h.GpuStore(0, 96 << 20, 32 << 20, name, True)
    yield h, g, host
    del g
    del host


def test_put_get_zero_copy(stores, cuda):
    h, g, _ = stores
    x = torch.randn(1000, 1000, device=cuda).to(torch.bfloat16)
    oid = _oid()
    s = torch.cuda.current_stream().cuda_stream
    g.put_segments(oid, [(x.data_ptr(), x.numel() * 2)], 16, s)
    t = torch.from_dlpack(h.store_dlpack(g, oid, [1000, 1000], 4, 16, s))
    assert t.dtype == torch.bfloat16 and t.device.type == "cuda"
    assert torch.equal(t, x)
    assert g.stats()["num_objects"] == 1
    # pinned while the view is alive: spilling must skip it
    assert g.spill_object(oid) == 0
    del t
    assert g.spill_object(oid) > 0
    assert g.is_spilled(oid)
    t2 = torch.from_dlpack(h.store_dlpack(g, oid, [1000, 1000], 4, 16, s))
    assert torch.equal(t2, x)
    del t2
    assert g.delete(oid)


def test_lru_spill_under_pressure(stores, cuda):
    h, g, host = stores
    s = torch.cuda.current_stream().cuda_stream
    xs, ids = [], []
    for i in range(8):  # 8 x 16 MiB into a 96 MiB store
        x = (torch.randn(8 << 20, device=cuda) * (i + 1)).to(torch.bfloat16)
        oid = _oid()
        g.put_segments(oid, [(x.data_ptr(), x.numel() * 2)], 16, s)
        xs.append(x)
        ids.append(oid)
    st = g.stats()
    assert st["spilled_objects"] >= 2
    assert st["spilled_host_bytes_total"] < st["spilled_bytes_total"]  # compression paid off
    for x, oid in zip(xs, ids):
        t = torch.from_dlpack(h.store_dlpack(g, oid, [x.numel()], 4, 16, s))
        assert torch.equal(t, x)
        del t
    for oid in ids:
        g.delete(oid)
    assert host.stats()["num_objects"] == 0


def test_ipc_handle_roundtrip(stores, cuda):
    h, g, _ = stores
    x = torch.arange(4096, device=cuda, dtype=torch.float32)
    oid = _oid()
    s = torch.cuda.current_stream().cuda_stream
    g.put_segments(oid, [(x.data_ptr(), x.numel() * 4)], 32, s)
    slab, off, n = g.locate(oid)
    assert slab >= 0 and n == 4096 * 4
    assert len(g.slab_ipc_handle(slab)) == 64


def test_delete_deferred_while_local_view_alive(stores, cuda):
    h, g, _ = stores
    x = torch.full((1 << 20,), 7.0, device=cuda)
    oid = _oid()
    s = torch.cuda.current_stream().cuda_stream
    g.put_segments(oid, [(x.data_ptr(), x.numel() * 4)], 32, s)
    t = torch.from_dlpack(h.store_dlpack(g, oid, [1 << 20], 2, 32, s))
    assert g.delete(oid)
    assert not g.contains(oid) and g.stats()["deferred_deletes"] == 1
    # the memory is still ours: a new object must not overwrite the live view
    y = torch.full((1 << 20,), 9.0, device=cuda)
    oid2 = _oid()
    g.put_segments(oid2, [(y.data_ptr(), y.numel() * 4)], 32, s)
    torch.cuda.synchronize()
    assert float(t.min()) == 7.0 and float(t.max()) == 7.0
    del t
    assert g.stats()["num_objects"] == 1
    g.delete(oid2)


def test_spill_single_pass_restore_foreign_and_threshold(stores, cuda):
    h, g, host = stores
    s = torch.cuda.current_stream().cuda_stream
    x = (torch.randn(8 << 20, device=cuda) * 3).to(torch.bfloat16)  # 16 MiB bf16
    oid = _oid()
    g.put_segments(oid, [(x.data_ptr(), x.numel() * 2)], 16, s)
    assert g.spill_object(oid) > 0
    st = g.stats()
    assert st["spill_s_total"] > 0 and st["spilled_host_bytes_total"] < st["spilled_bytes_total"]
    # another process's view of the spill copy: restore into caller-owned memory
    out = torch.empty_like(x)
    assert g.restore_foreign(h.GpuStore.host_id(oid), out.data_ptr(), x.numel() * 2) == x.numel() * 2
    assert torch.equal(out, x)
    g.delete(oid)
    assert host.stats()["num_objects"] == 0  # the host copy went with the object
    # proactive spilling above 50 % of the 96 MiB capacity, by the background thread
    g.set_spill_threshold(0.5)
    keep = []
    for i in range(4):  # 4 x 16 MiB = 64 MiB > 48 MiB
        y = torch.full((8 << 20,), float(i), device=cuda, dtype=torch.bfloat16)
        o2 = _oid()
        g.put_segments(o2, [(y.data_ptr(), y.numel() * 2)], 16, s)
        keep.append((o2, y))
    import time

    deadline = time.time() + 10
    while time.time() < deadline and g.stats()["proactive_spills"] == 0:
        time.sleep(0.05)
    assert g.stats()["proactive_spills"] >= 1
    assert g.stats()["bytes_in_use"] <= 0.5 * (96 << 20)
    for o2, y in keep:
        v = torch.from_dlpack(h.store_dlpack(g, o2, [8 << 20], 4, 16, s))
        assert torch.equal(v, y)
        del v
        g.delete(o2)
