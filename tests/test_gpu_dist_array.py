"""DistArray with CUDA blocks on the MI355X: blocks live in the HBM object store, blocked GEMMs run
in GPU tasks and the result matches numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_cuda_blocked_matmul_matches_numpy():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ray_memory_management_amd as ray
    from ray_memory_management_amd.experimental.array import distributed as da
    from ray_memory_management_amd.experimental.locations import get_object_locations

    ray.init(num_cpus=4, num_gpus=1, object_store_memory=256 << 20)
    try:
        g = np.random.default_rng(0)
        A, B = g.standard_normal((300, 200)).astype(np.float32), g.standard_normal((200, 260)).astype(np.float32)
        x = da.numpy_to_dist(torch.as_tensor(A, device="cuda"), block_size=128, device="cuda")
        y = da.numpy_to_dist(torch.as_tensor(B, device="cuda"), block_size=128, device="cuda")
        c = da.dot(x, y).assemble()
        assert c.is_cuda and tuple(c.shape) == (300, 260)
        np.testing.assert_allclose(c.cpu().numpy(), A @ B, rtol=2e-3, atol=2e-2)
        loc = get_object_locations([x.object_refs[0, 0]])[x.object_refs[0, 0]]
        assert loc["object_size"] == 128 * 128 * 4 and loc.get("gpu")
    finally:
        ray.shutdown()
