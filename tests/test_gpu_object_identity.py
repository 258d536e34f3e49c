"""GPU-object device identity without a GPU: a descriptor names its physical GPU by PCI address and
every consumer resolves that to ITS OWN local device index (workers run with per-GPU
HIP_VISIBLE_DEVICES, so local indices differ between processes). Mocked device tables."""
import pytest


@pytest.fixture
def mocked(monkeypatch):
    import torch

    from ray_memory_management_amd._private import gpu_object_store as gos

    table = {}
    monkeypatch.setattr(gos, "_pci_cache", {})
    monkeypatch.setattr(gos, "pci_bus_id", lambda d: table[d])
    monkeypatch.setattr(torch.cuda, "device_count", lambda: len(table))
    monkeypatch.delenv("RMM_TEST_FORCE_PEER_COPY", raising=False)
    return gos, table


def test_same_physical_gpu_under_different_visible_sets(mocked):
    gos, table = mocked
    # driver sees all GPUs; worker A runs with HIP_VISIBLE_DEVICES=3 (its cuda:0 is physical GPU 3)
    driver = {i: f"0000:{0x10 + i:02x}:00.0" for i in range(8)}
    table.update({0: driver[3]})  # consumer = worker A
    assert gos.local_device_for_pci(driver[3]) == 0   # zero-copy IPC view on ITS device 0
    assert gos.local_device_for_pci(driver[5]) == -1  # another GPU: pull over xGMI
    table.clear()
    table.update(driver)  # consumer = the driver
    assert gos.local_device_for_pci(driver[3]) == 3
    assert gos.local_device_for_pci("0000:ff:00.0") == -1


def test_force_peer_hook(mocked, monkeypatch):
    gos, table = mocked
    table.update({0: "0000:10:00.0"})
    monkeypatch.setenv("RMM_TEST_FORCE_PEER_COPY", "1")
    assert gos.local_device_for_pci("0000:10:00.0") == -1


def test_pull_quota_admission():
    import threading
    import time

    from ray_memory_management_amd._private.gpu_object_store import _PullQuota

    q = _PullQuota()
    q.acquire(60, 100)
    got = []
    t = threading.Thread(target=lambda: (q.acquire(50, 100), got.append(1)))
    t.start()
    time.sleep(0.2)
    assert not got  # 60 + 50 > 100: waits for the first replica to be released
    q.release(60)
    t.join(5)
    assert got == [1] and q.in_use == 50
    q.release(50)
    q.acquire(500, 100)  # an oversized pull is admitted when nothing else is in flight
    assert q.in_use == 500
