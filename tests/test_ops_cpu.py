"""CPU semantics of the ops wrappers (the HIP kernels are checked against these in the GPU tests)."""
import torch

from ray_memory_management_amd import ops


def test_counter_window_gather_cpu():
    x = torch.arange(50).float().reshape(25, 2)
    idx = torch.randperm(25)[:20]
    ctr = torch.tensor([7, 0])
    out = ops.gather_rows(x, idx, rows=5, ctr=ctr, period=4)   # 7 % 4 = 3 → idx[15:20]
    assert torch.equal(out, x[idx[15:20]])


def test_frames_to_nhwc_counter_cpu():
    f = torch.randint(0, 255, (10, 4, 6, 6), dtype=torch.uint8)
    idx = torch.tensor([3, 1, 4, 1, 5, 9])
    y = ops.frames_to_nhwc(f, idx, rows=3, ctr=torch.tensor([1]), period=2)
    assert y.shape == (3, 4, 6, 6) and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), (f[idx[3:]].float() / 255).to(torch.bfloat16).float())


def test_vision_network_merged_heads():
    from ray_memory_management_amd.rllib.models import VisionNetwork

    m = VisionNetwork(6)
    obs = torch.randint(0, 255, (3, 4, 84, 84), dtype=torch.uint8)
    logits, v = m(obs)
    h = m.forward_heads(obs)
    assert logits.shape == (3, 6) and v.shape == (3,) and h.shape == (3, 7)
    torch.testing.assert_close(logits, h[:, :6])
    torch.testing.assert_close(v, h[:, 6])
    # policy rows are initialised small (orthogonal * 0.01) as in RLlib
    assert float(m.heads.weight[:6].abs().max()) < 0.05
