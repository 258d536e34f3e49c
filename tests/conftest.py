import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def ray_start():
    """A fresh local cluster per test (mirrors the reference's ray_start_regular fixture)."""
    import ray_memory_management_amd as ray

    ray.init(num_cpus=4, object_store_memory=256 << 20, ignore_reinit_error=True)
    yield ray
    ray.shutdown()


@pytest.fixture(scope="module")
def ray_shared():
    """One cluster shared by every test of a module (for tests that do not disturb cluster state)."""
    import ray_memory_management_amd as ray

    ray.init(num_cpus=4, object_store_memory=256 << 20, ignore_reinit_error=True)
    yield ray
    ray.shutdown()
