"""NUMA-local placement of GPU-driving processes (_private/numa.py): sysfs parsing on a fake tree."""
import os

from ray_memory_management_amd._private import numa


def _fake_sysfs(tmp_path, bus, local=None, node=None, node_cpus=None):
    dev = tmp_path / "bus" / "pci" / "devices" / bus
    dev.mkdir(parents=True)
    if local is not None:
        (dev / "local_cpulist").write_text(local + "\n")
    if node is not None:
        (dev / "numa_node").write_text(f"{node}\n")
        nd = tmp_path / "devices" / "system" / "node" / f"node{node}"
        nd.mkdir(parents=True)
        (nd / "cpulist").write_text(node_cpus + "\n")
    return str(tmp_path)


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.parse_cpulist("") == set()


def test_pci_local_cpus_prefers_local_cpulist(tmp_path):
    root = _fake_sysfs(tmp_path, "0000:75:00.0", local="0-23,96-119", node=1, node_cpus="24-47")
    assert numa.pci_local_cpus("0000:75:00.0", root) == set(range(24)) | set(range(96, 120))


def test_pci_local_cpus_falls_back_to_numa_node(tmp_path):
    root = _fake_sysfs(tmp_path, "0000:0d:00.0", node=1, node_cpus="4-7")
    assert numa.pci_local_cpus("0000:0D:00.0", root) == {4, 5, 6, 7}
    root2 = _fake_sysfs(tmp_path / "b", "0000:0e:00.0", node=-1, node_cpus="")
    assert numa.pci_local_cpus("0000:0e:00.0", root2) is None
    assert numa.pci_local_cpus("0000:ff:00.0", root) is None


def test_pin_to_gpu_is_a_no_op_without_a_gpu(monkeypatch):
    before = os.sched_getaffinity(0)
    monkeypatch.delenv("RMM_NUMA_PIN", raising=False)
    assert numa.pin_to_gpu(0) is None  # no HIP device here: nothing changes
    assert os.sched_getaffinity(0) == before
    monkeypatch.setenv("RMM_NUMA_PIN", "0")
    assert numa.pin_to_gpu(0) is None
