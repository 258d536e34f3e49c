"""Numerics of the CDNA4 kernels against plain PyTorch fp32 references (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu(cuda):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    assert "gfx950" in h.arch(0)
    return h


def test_multi_copy_any_alignment(cuda):
    from ray_memory_management_amd import ops

    torch.manual_seed(0)
    srcs = [torch.randint(0, 255, (n,), dtype=torch.uint8, device=cuda) for n in (1, 15, 16, 1000, 1 << 20, 3 << 20 | 7)]
    # misaligned views
    srcs.append(torch.randint(0, 255, (5000,), dtype=torch.uint8, device=cuda)[3:])
    dsts = [torch.empty(s.numel() + 13, dtype=torch.uint8, device=cuda)[5:5 + s.numel()] for s in srcs]
    ops.multi_copy(list(zip(srcs, dsts)))
    torch.cuda.synchronize()
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)


def test_many_segments_split_launches(cuda):
    from ray_memory_management_amd import ops

    srcs = [torch.full((100 + i,), i % 251, dtype=torch.uint8, device=cuda) for i in range(200)]
    dsts = [torch.empty_like(s) for s in srcs]
    ops.multi_copy(list(zip(srcs, dsts)))
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)


def test_pack_unpack_roundtrip(cuda):
    from ray_memory_management_amd import ops

    ts = [torch.randn(37, 5, device=cuda, dtype=torch.bfloat16), torch.arange(11, device=cuda),
          torch.randn(3, 4, 5, device=cuda), torch.empty(0, device=cuda)]
    buf, layout = ops.pack_tensors(ts)
    outs = ops.unpack_tensors(buf, layout, copy=True)
    for a, b in zip(ts, outs):
        assert torch.equal(a, b)


def test_concat_matches_torch_cat(cuda):
    from ray_memory_management_amd import ops

    ts = [torch.randn(n, 84, 84, device=cuda).to(torch.bfloat16) for n in (3, 0, 17, 64)]
    assert torch.equal(ops.concat(ts), torch.cat(ts))


def test_gather_rows(cuda):
    from ray_memory_management_amd import ops

    x = torch.randn(1000, 4, 84, 84, device=cuda).to(torch.bfloat16)
    idx = torch.randperm(1000, device=cuda)[:333]
    assert torch.equal(ops.gather_rows(x, idx), x[idx])
    y = torch.arange(999 * 3, dtype=torch.uint8, device=cuda).view(999, 3)  # odd row bytes
    idx2 = torch.randint(0, 999, (77,), device=cuda)
    assert torch.equal(ops.gather_rows(y, idx2), y[idx2])


@pytest.mark.parametrize("T,B", [(1, 1), (7, 3), (128, 64), (200, 1000), (1000, 17)])
def test_gae_matches_fp32_reference(cuda, T, B):
    from ray_memory_management_amd import ops

    g = torch.Generator(device="cpu").manual_seed(T * 1000 + B)
    r = torch.randn(T, B, generator=g).to(cuda)
    v = torch.randn(T, B, generator=g).to(cuda)
    d = (torch.rand(T, B, generator=g) < 0.05).float().to(cuda)
    lv = torch.randn(B, generator=g).to(cuda)
    adv, ret = ops.gae(r, v, d, lv, 0.99, 0.95)
    ra, rr = ops.gae_reference(r.cpu().double(), v.cpu().double(), d.cpu().double(), lv.cpu().double(), 0.99, 0.95)
    torch.testing.assert_close(adv.cpu().double(), ra, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ret.cpu().double(), rr, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("n", [1, 255, 256, 257, 100_003, 1 << 20])
def test_compress_lossless(cuda, dtype, n):
    from ray_memory_management_amd import ops

    x = (torch.randn(n, device=cuda) * 0.02).to(dtype)
    x[: n // 3] = 0  # zero blocks
    c = ops.compress(x)
    y = ops.decompress(c, n, dtype)
    assert torch.equal(x.view(torch.int16 if dtype != torch.float32 else torch.int32),
                       y.view(torch.int16 if dtype != torch.float32 else torch.int32))
    if n >= 100_000:
        assert c.numel() < x.numel() * x.element_size() * 0.85


def test_compress_special_values(cuda):
    from ray_memory_management_amd import ops

    x = torch.tensor([float("inf"), -float("inf"), float("nan"), -0.0, 0.0, 1e-40, -3.5] * 100, device=cuda)
    for dt in (torch.float32, torch.bfloat16):
        xx = x.to(dt)
        y = ops.decompress(ops.compress(xx), xx.numel(), dt)
        assert torch.equal(xx.view(torch.int32 if dt == torch.float32 else torch.int16),
                           y.view(torch.int32 if dt == torch.float32 else torch.int16))


def test_ppo_loss_matches_reference(cuda):
    from ray_memory_management_amd import ops

    torch.manual_seed(1)
    n = 4097
    ln = (torch.randn(n, device=cuda) * 0.3).requires_grad_()
    lo = torch.randn(n, device=cuda) * 0.3
    adv = torch.randn(n, device=cuda)
    vn = torch.randn(n, device=cuda).requires_grad_()
    vt = torch.randn(n, device=cuda) * 3
    ent = torch.rand(n, device=cuda).requires_grad_()
    tot, means = ops.ppo_loss(ln, lo, adv, vn, vt, ent, 0.2, 4.0, 0.5, 0.01)
    tot.backward()
    g1 = (ln.grad.clone(), vn.grad.clone(), ent.grad.clone())
    ln.grad = vn.grad = ent.grad = None
    rt, rmeans = ops.ppo_loss_reference(ln, lo, adv, vn, vt, ent, 0.2, 4.0, 0.5, 0.01)
    rt.backward()
    torch.testing.assert_close(tot, rt, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(means, rmeans, rtol=1e-4, atol=1e-5)
    for a, b in zip(g1, (ln.grad, vn.grad, ent.grad)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("C", [1, 3, 4])
def test_frames_to_nhwc(cuda, C):
    from ray_memory_management_amd import ops

    x = torch.randint(0, 256, (37, C, 84, 84), dtype=torch.uint8, device=cuda)
    ref = (x.float() / 255.0).to(torch.bfloat16)
    y = ops.frames_to_nhwc(x)
    assert y.is_contiguous(memory_format=torch.channels_last) or C == 1
    assert torch.equal(y.contiguous(), ref)
    idx = torch.randint(0, 37, (11,), device=cuda)
    y2 = ops.frames_to_nhwc(x, idx)
    assert torch.equal(y2.contiguous(), ref[idx])


def _trunk_reference(frames_u8, w1, b1, w2, b2):
    x = frames_u8.float() / 255.0
    h1 = torch.relu(torch.nn.functional.conv2d(x, w1.float(), b1.float(), stride=4, padding=2))
    # the kernel keeps h1 in bf16 (LDS tile / saved activation): round it the same way, with a
    # straight-through gradient, so ReLU masks of h2 agree and the test isolates the kernel math
    h1 = h1 + (h1.to(torch.bfloat16).float() - h1).detach()
    h2 = torch.relu(torch.nn.functional.conv2d(h1, w2.float(), b2.float(), stride=2, padding=2))
    return h2.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten


@pytest.mark.parametrize("rows", [23, 300])
@pytest.mark.parametrize("use_ctr", [False, True])
@pytest.mark.parametrize("channels_last", [False, True])
def test_nature_trunk_fwd_bwd_match_fp32(cuda, use_ctr, channels_last, rows):
    """K10 fused trunk (MFMA) vs fp32 torch conv2d with the same bf16 weights: forward values and
    all four weight/bias gradients for a random upstream gradient, with minibatch gathering.
    rows=300 > 256 backward workgroups: workgroups loop over two frames (the prefetch path).
    The backward also runs twice and must give bit-identical gradients."""
    from ray_memory_management_amd.rllib.models import nature_trunk

    torch.manual_seed(0)
    obs = torch.randint(0, 256, (57, 4, 84, 84), dtype=torch.uint8, device=cuda)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    w1 = (torch.randn(16, 4, 8, 8, device=cuda) * 0.05).to(torch.bfloat16).contiguous(memory_format=fmt)
    b1 = (torch.randn(16, device=cuda) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(32, 16, 4, 4, device=cuda) * 0.1).to(torch.bfloat16).contiguous(memory_format=fmt)
    b2 = (torch.randn(32, device=cuda) * 0.1).to(torch.bfloat16)
    period = 3
    idx = torch.randint(0, 57, (rows * period,), device=cuda)
    ctr = torch.tensor([4, 0], dtype=torch.int64, device=cuda) if use_ctr else None
    sel = idx[(4 % period) * rows:(4 % period + 1) * rows] if use_ctr else idx[:rows]
    params = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]
    out = nature_trunk(obs, *params, idx=idx, ctr=ctr, period=period, rows=rows)
    ref_params = [t.detach().float().requires_grad_(True) for t in (w1, b1, w2, b2)]
    ref = _trunk_reference(obs[sel], *ref_params)
    assert out.shape == ref.shape == (rows, 3872)
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, f"forward rel err {err}"
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16), retain_graph=True)
    first = [p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    out.backward(g.to(torch.bfloat16))
    for a, p in zip(first, params):
        assert torch.equal(a, p.grad), "K10 backward is not deterministic"
    ref.backward(g)
    errs = {}
    for name, p, rp in zip(("dW1", "db1", "dW2", "db2"), params, ref_params):
        assert p.grad.stride() == p.stride()
        errs[name] = float((p.grad.float() - rp.grad).abs().max() / rp.grad.abs().max())
    assert max(errs.values()) < 2e-2, errs


def test_vision_network_fused_matches_unfused(cuda, monkeypatch):
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(1)
    m = VisionNetwork(6).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    obs = torch.randint(0, 256, (40, 4, 84, 84), dtype=torch.uint8, device=cuda)
    assert m.nature and m.fused_trunk_ok(obs)
    with torch.no_grad():
        fused = m.forward_heads(obs).float()
        monkeypatch.setenv("RMM_NO_FUSED_TRUNK", "1")
        plain = m.forward_heads(obs).float()
    err = (fused - plain).abs().max() / plain.abs().max().clamp_min(1e-3)
    assert err < 3e-2, err


@pytest.mark.parametrize("C,relu", [(256, True), (5, False), (40, True)])
def test_mask_colsum(cuda, C, relu):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    M = 517
    dy = torch.randn(M, C, device=cuda).to(torch.bfloat16)
    y = torch.relu(torch.randn(M, C, device=cuda)).to(torch.bfloat16)
    dpre = torch.empty_like(dy)
    db = torch.empty(C, dtype=torch.bfloat16, device=cuda)
    h.mask_colsum(dy.data_ptr(), y.data_ptr(), dpre.data_ptr(), db.data_ptr(), M, C, relu,
                  torch.cuda.current_stream().cuda_stream)
    ref = dy.float() * (y.float() > 0) if relu else dy.float()
    assert torch.equal(dpre.float(), ref)
    torch.testing.assert_close(db.float(), ref.sum(0), rtol=1e-2, atol=1e-2)


def test_dense_fn_matches_linear(cuda):
    from ray_memory_management_amd.rllib.models import dense

    torch.manual_seed(0)
    lin = torch.nn.Linear(96, 64).to(cuda).to(torch.bfloat16)
    x = torch.randn(33, 96, device=cuda).to(torch.bfloat16).requires_grad_(True)
    gout = torch.empty_like(lin.weight)
    lin.weight._rmm_grad_out = gout
    y = dense(x, lin, True)
    ref_lin = torch.nn.Linear(96, 64).to(cuda)
    ref_lin.load_state_dict({k: v.float() for k, v in lin.state_dict().items()})
    xr = x.detach().float().requires_grad_(True)
    yr = torch.relu(ref_lin(xr))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(yr)
    gw, gb, gx = torch.autograd.grad(y, (lin.weight, lin.bias, x), g.to(torch.bfloat16))
    yr.backward(g)
    assert gw.data_ptr() == gout.data_ptr()  # written in place into the bucket view (learner path)
    for a, b in ((gw, ref_lin.weight.grad), (gb, ref_lin.bias.grad), (gx, xr.grad)):
        assert float((a.float() - b).abs().max() / b.abs().max()) < 2e-2


@pytest.mark.parametrize("M,K,A1", [(500, 3872, 5), (37, 96, 7), (64, 64, 1), (130, 64, 16), (640, 96, 3)])
def test_dense_heads_bwd_matches_fp32(cuda, M, K, A1):
    """K12 fused dense+heads backward vs fp32 autograd of ReLU(x Wᵀ+b) Whᵀ+bh (same bf16 inputs)."""
    from ray_memory_management_amd.rllib.models import dense_heads

    torch.manual_seed(0)
    layer = torch.nn.Linear(K, 256).to(cuda).to(torch.bfloat16)
    heads = torch.nn.Linear(256, A1).to(cuda).to(torch.bfloat16)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16).requires_grad_(True)
    out = dense_heads(x, layer, heads)
    g = torch.randn(M, A1, device=cuda).to(torch.bfloat16)
    got = torch.autograd.grad(out, (x, layer.weight, layer.bias, heads.weight, heads.bias), g)
    xr = x.detach().float().requires_grad_(True)
    ps = [t.detach().float().requires_grad_(True) for t in (layer.weight, layer.bias, heads.weight, heads.bias)]
    hidden = torch.relu(xr @ ps[0].t() + ps[1])
    ref_out = hidden @ ps[2].t() + ps[3]
    assert float((out.float() - ref_out).abs().max() / ref_out.abs().max()) < 2e-2
    ref = torch.autograd.grad(ref_out, [xr] + ps, g.float())
    errs = {n: float((a.float() - b).abs().max() / b.abs().max().clamp_min(1e-6))
            for n, a, b in zip(("dx", "dW", "db", "dWh", "dbh"), got, ref)}
    assert max(errs.values()) < 2e-2, errs


@pytest.mark.parametrize("M", [1, 12, 13, 25, 33, 50, 64, 100, 500, 777])
def test_dense_relu_fwd_matches_fp32(cuda, M):
    """K13 vs an fp32 torch reference over tile-tail shapes; repeated calls and a HIP-graph replay."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(M)
    K, N = 3872, 256
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    ref = torch.relu(x.float() @ w.float().t() + b.float())
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        y.zero_()
        h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, y.data_ptr(), st)
        torch.cuda.synchronize()
        torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    # graph capture + replay (the workspace for this shape already exists)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    y2 = torch.empty_like(y)
    with torch.cuda.graph(g, stream=s):
        h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, y2.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        y2.zero_()
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(y2.float(), ref, atol=2e-2, rtol=2e-2)
