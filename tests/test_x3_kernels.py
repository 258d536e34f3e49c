"""Numerics of the precision-matched split-bf16 (x3) kernels against float64 PyTorch references (GPU).

The x3 kernels carry fp32 operands as hi + lo bf16 pairs and multiply with three bf16 MFMAs
(csrc/hip/x3_device.h): their error budget is ~1e-5 relative, three orders of magnitude below the
bf16 kernels' 2e-2 tolerances in test_hip_kernels.py. ReLU masks are taken from the kernels' own
outputs (a pre-activation within ~1e-6 of zero may land on either side at fp32-level precision), so
the comparison isolates the arithmetic."""
import pytest
import torch

pytestmark = pytest.mark.gpu

FWD_TOL = 2e-5   # max |err| / max |ref| of activations
GRAD_TOL = 1e-4  # max |err| / max |ref| of gradients (sums over hundreds of rows)


@pytest.fixture(autouse=True)
def _need_gpu(cuda):
    from ray_memory_management_amd._native import require_hip

    assert "gfx950" in require_hip().arch(0)


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def test_split_roundtrip(cuda):
    from ray_memory_management_amd.ops import x3

    torch.manual_seed(0)
    x = torch.randn(100_003, device=cuda) * torch.logspace(-3, 3, 100_003, device=cuda)
    p = x3.split(x)
    rel = ((p.float() - x).abs() / x.abs().clamp_min(1e-30)).max()
    assert rel <= 2.0 ** -16, float(rel)
    assert torch.equal(p.hi, x.to(torch.bfloat16))  # hi is the round-to-nearest bf16 of x
    cpu = x3.split(x.cpu())
    assert torch.equal(cpu.hi, p.hi.cpu()) and torch.equal(cpu.lo, p.lo.cpu())


def _trunk_ref(frames, w1, b1, w2, b2, m1, m2):
    x = frames.double() / 255.0
    h1 = (torch.nn.functional.conv2d(x, w1, b1, stride=4, padding=2)) * m1
    h2 = (torch.nn.functional.conv2d(h1, w2, b2, stride=2, padding=2)) * m2
    return h1, h2


@pytest.mark.parametrize("rows", [23, 600])
@pytest.mark.parametrize("channels_last", [False, True])
def test_x3_trunk_fwd_bwd_match_fp64(cuda, rows, channels_last):
    """K10x forward (h1, h2) and backward (dW1, db1, dW2, db2) vs float64 autograd; rows=600 makes
    every launch loop over several frames per workgroup (fwd 256, conv2-bwd 512, conv1-wgrad 256
    workgroups). Deterministic: a second backward gives bit-identical gradients."""
    from ray_memory_management_amd.ops import x3

    torch.manual_seed(0)
    n = 97
    obs = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=cuda)
    fmt = torch.channels_last if channels_last else torch.contiguous_format
    w1 = (torch.randn(16, 4, 8, 8, device=cuda) * 0.05).contiguous(memory_format=fmt)
    b1 = torch.randn(16, device=cuda) * 0.1
    w2 = (torch.randn(32, 16, 4, 4, device=cuda) * 0.1).contiguous(memory_format=fmt)
    b2 = torch.randn(32, device=cuda) * 0.1
    period = 2
    idx = torch.randint(0, n, (rows * period,), device=cuda)
    ctr = torch.tensor([3, 0], dtype=torch.int64, device=cuda)
    sel = idx[(3 % period) * rows:(3 % period + 1) * rows]
    P = [x3.split_like(t) for t in (w1, b1, w2, b2)]
    h1 = x3.Pair.empty((rows, 441, 16), cuda)
    h1, h2 = x3.trunk_fwd(obs, *P, idx=idx, ctr=ctr, period=period, rows=rows, h1=h1)
    torch.cuda.synchronize()
    # reference with the kernel's ReLU masks and the kernel's (split-exact) weights
    wr = [p.float().double().requires_grad_(True) for p in P]
    m1 = (h1.float() > 0).view(rows, 21, 21, 16).permute(0, 3, 1, 2).double()
    m2 = (h2.float() > 0).view(rows, 11, 11, 32).permute(0, 3, 1, 2).double()
    r1, r2 = _trunk_ref(obs[sel], *wr, m1, m2)
    r1f = r1.permute(0, 2, 3, 1).reshape(rows, 441, 16)
    r2f = r2.permute(0, 2, 3, 1).reshape(rows, 3872)
    assert _rel(h1.float(), r1f) < FWD_TOL
    assert _rel(h2.float(), r2f) < FWD_TOL
    # backward for a random upstream gradient (itself a split pair: the K12x dx)
    g = x3.split(torch.randn(rows, 3872, device=cuda))
    dpre1 = x3.Pair.empty((rows, 441, 16), cuda)
    part = torch.empty(x3.trunk_partial_floats(rows), dtype=torch.float32, device=cuda)
    grads = []
    for _ in range(2):
        dw1 = torch.empty_strided(w1.size(), w1.stride(), device=cuda)
        dw2 = torch.empty_strided(w2.size(), w2.stride(), device=cuda)
        db1, db2 = torch.empty(16, device=cuda), torch.empty(32, device=cuda)
        x3.trunk_bwd(obs, P[2], h1, h2, g, dpre1, part, dw1, db1, dw2, db2, w1.stride(), idx=idx, ctr=ctr,
                     period=period, rows=rows)
        torch.cuda.synchronize()
        grads.append((dw1, db1, dw2, db2))
    for a, b in zip(*grads):
        assert torch.equal(a, b), "K10x backward is not deterministic"
    r2f.backward(g.float().double())
    errs = {nm: _rel(a, rp.grad) for nm, a, rp in zip(("dW1", "db1", "dW2", "db2"), grads[0], wr)}
    assert max(errs.values()) < GRAD_TOL, errs


@pytest.mark.parametrize("M,K", [(12, 3872), (50, 3872), (500, 3872), (777, 3872), (200, 320), (130, 96)])
def test_x3_dense_fwd_part_matches_fp64(cuda, M, K):
    """M <= 64: register-direct K13x; larger M: the LDS-staged K13x-L (odd slice lengths: a half stage)."""
    from ray_memory_management_amd.ops import x3

    torch.manual_seed(M)
    N = 256
    x = x3.split(torch.relu(torch.randn(M, K, device=cuda)))
    w = x3.split(torch.randn(N, K, device=cuda) * 0.02)
    part, S = x3.dense_fwd_part(x, w)
    torch.cuda.synchronize()
    got = part.view(S, M, N).double().sum(0)
    ref = x.float().double() @ w.float().double().t()
    assert _rel(got, ref) < FWD_TOL


def _ppo_ref(heads, cols, coef, A):
    clip, vf_clip, vf_coeff, ent_coeff, kl_coeff = [float(c) for c in coef.tolist()]
    lp = torch.log_softmax(heads[:, :A], -1)
    lpo = torch.log_softmax(cols[:, :A].double(), -1)
    act = cols[:, A + 3].long()
    r = torch.exp(lp.gather(1, act[:, None])[:, 0] - cols[:, A].double())
    adv = cols[:, A + 1].double()
    surr = torch.minimum(r * adv, r.clamp(1 - clip, 1 + clip) * adv)
    vf = torch.clamp((heads[:, A] - cols[:, A + 2].double()) ** 2, max=vf_clip)
    ent = -(lp.exp() * lp).sum(-1)
    kl = (lpo.exp() * (lpo - lp)).sum(-1)
    per = -surr + vf_coeff * vf - ent_coeff * ent + kl_coeff * kl
    stats = torch.stack([-surr.sum(), vf.sum(), ent.sum(), kl.sum()])
    return per.mean(), stats


@pytest.mark.parametrize("M,K,A", [(500, 3872, 4), (37, 96, 6), (130, 64, 15), (640, 3872, 2), (200, 96, 5)])
def test_x3_dense_heads_ppo_chain_matches_fp64(cuda, M, K, A):
    """K13x -> K15x (hidden, heads, PPO loss stats, dheads, dpre) -> K12x (dx, dW, db, dWh, dbh) vs
    float64 autograd of the same PPO loss of heads(ReLU(x Wᵀ + b)); K12x launched twice, bit-identical."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.ops import x3

    h = require_hip()
    torch.manual_seed(K + A)
    A1 = A + 1
    x = x3.split(torch.relu(torch.randn(M, K, device=cuda)))
    W = x3.split(torch.randn(256, K, device=cuda) * (1.0 / K ** 0.5))
    b = x3.split(torch.randn(256, device=cuda) * 0.1)
    Wh = x3.split(torch.randn(A1, 256, device=cuda) * 0.1)
    bh = x3.split(torch.randn(A1, device=cuda) * 0.1)
    cols = torch.zeros(M, A + 4, device=cuda)
    cols[:, :A] = torch.randn(M, A, device=cuda) * 0.3
    cols[:, A] = torch.log_softmax(cols[:, :A], -1)[:, 0] + 0.05 * torch.randn(M, device=cuda)
    cols[:, A + 1] = torch.randn(M, device=cuda)
    cols[:, A + 2] = torch.randn(M, device=cuda)
    cols[:, A + 3] = torch.randint(0, A, (M,), device=cuda).float()
    coef = torch.tensor([0.2, 10.0, 0.5, 0.01, 0.2], device=cuda)
    one = torch.ones((), device=cuda)
    acc = torch.zeros(6, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    part, S = x3.dense_fwd_part(x, W)
    dz, dpre, hid = x3.Pair.empty((M, A1), cuda), x3.Pair.empty((M, 256), cuda), x3.Pair.empty((M, 256), cuda)
    h.x3_heads_ppo(part.data_ptr(), S, b.ptrs(), Wh.ptrs(), bh.ptrs(), cols.data_ptr(), coef.data_ptr(),
                   acc.data_ptr(), one.data_ptr(), M, A1, dz.ptrs(), dpre.ptrs(), hid.ptrs(), s)
    dx = x3.Pair.empty((M, K), cuda)
    dW, db = torch.empty(256, K, device=cuda), torch.empty(256, device=cuda)
    dWh, dbh = torch.empty(A1, 256, device=cuda), torch.empty(A1, device=cuda)
    outs = []
    for _ in range(2):
        h.x3_dense_heads_bwd(dz.ptrs(), A1, hid.ptrs(), x.ptrs(), W.ptrs(), dpre.ptrs(), M, K, dx.ptrs(),
                             dW.data_ptr(), db.data_ptr(), dWh.data_ptr(), dbh.data_ptr(), s)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (dx.hi, dx.lo, dW, db, dWh, dbh)])
    for first, second in zip(*outs):
        assert torch.equal(first, second)
    xr = x.float().double().requires_grad_(True)
    ps = [t.float().double().requires_grad_(True) for t in (W, b, Wh, bh)]
    mask = (hid.float() > 0).double()
    hidden = (xr @ ps[0].t() + ps[1]) * mask
    heads = hidden @ ps[2].t() + ps[3]
    heads.retain_grad()
    loss, stats = _ppo_ref(heads, cols, coef, A)
    loss.backward()
    assert _rel(hid.float(), hidden) < FWD_TOL
    torch.testing.assert_close(acc[:4].double(), stats.detach(), rtol=1e-4, atol=1e-4)
    assert _rel(dz.float(), heads.grad) < FWD_TOL
    errs = {n: _rel(a, r.grad) for n, a, r in zip(("dx", "dW", "db", "dWh", "dbh"),
                                                   (dx.float(), dW, db, dWh, dbh), [xr] + ps)}
    assert max(errs.values()) < GRAD_TOL, errs
    # slab mode (the learner's): each workgroup adds its sums into its own row, no atomics; two launches
    # accumulate, the rows sum to twice the atomic total; outputs unchanged
    slab = torch.zeros(h.x3_heads_ppo_groups(M), 8, device=cuda)
    dz0 = dz.hi.clone()
    for _ in range(2):
        h.x3_heads_ppo(part.data_ptr(), S, b.ptrs(), Wh.ptrs(), bh.ptrs(), cols.data_ptr(), coef.data_ptr(),
                       slab.data_ptr(), one.data_ptr(), M, A1, dz.ptrs(), dpre.ptrs(), hid.ptrs(), s, acc_slab=True)
    torch.cuda.synchronize()
    assert torch.equal(dz.hi, dz0)
    torch.testing.assert_close(slab[:, :6].sum(0), 2 * acc, rtol=1e-5, atol=1e-5)
    assert not slab[:, 6:].any()


@pytest.mark.parametrize("M,K,A", [(500, 3872, 4), (130, 64, 15), (257, 96, 5)])
def test_x3_dense_heads_bwd_row_parts(cuda, M, K, A):
    """K12x with two row parts (rs = 2): the second part's dW / db / dWh / dbh land in their own slab;
    part 0 + part 1 match one part to fp32 rounding and float64 autograd, dx is bit-identical (per row)."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.ops import x3

    h = require_hip()
    torch.manual_seed(M + K + A)
    A1 = A + 1
    x = x3.split(torch.relu(torch.randn(M, K, device=cuda)))
    W = x3.split(torch.randn(256, K, device=cuda) * (1.0 / K ** 0.5))
    dz = x3.split(torch.randn(M, A1, device=cuda) * 0.1)
    hid = x3.split(torch.relu(torch.randn(M, 256, device=cuda)))
    dpre = x3.split(torch.randn(M, 256, device=cuda) * 0.1 * (hid.float() > 0))
    s = torch.cuda.current_stream().cuda_stream

    def run(rs):
        dx = x3.Pair.empty((M, K), cuda)
        o = [torch.full((256, K), 7.0, device=cuda), torch.full((256,), 7.0, device=cuda),
             torch.full((A1, 256), 7.0, device=cuda), torch.full((A1,), 7.0, device=cuda)]
        o2 = [torch.full_like(t, 7.0) for t in o]
        side = dict(dw2=o2[0].data_ptr(), db2=o2[1].data_ptr(), dwh2=o2[2].data_ptr(), dbh2=o2[3].data_ptr()) \
            if rs == 2 else {}
        h.x3_dense_heads_bwd(dz.ptrs(), A1, hid.ptrs(), x.ptrs(), W.ptrs(), dpre.ptrs(), M, K, dx.ptrs(),
                             *[t.data_ptr() for t in o], s, rs=rs, **side)
        torch.cuda.synchronize()
        return dx, o, o2

    dx1, one, _ = run(1)
    dx2, p0, p1 = run(2)
    assert torch.equal(dx1.hi, dx2.hi) and torch.equal(dx1.lo, dx2.lo)
    xd, dpd, dzd, hd = x.float().double(), dpre.float().double(), dz.float().double(), hid.float().double()
    ref = [dpd.t() @ xd, dpd.sum(0), dzd.t() @ hd, dzd.sum(0)]
    for a, b_, u, r in zip(p0, p1, one, ref):
        assert _rel(a + b_, r) < GRAD_TOL and _rel(u, r) < GRAD_TOL
        assert _rel(a + b_, u) < 1e-5
    with pytest.raises(ValueError):  # rs = 2 without the second slab
        h.x3_dense_heads_bwd(dz.ptrs(), A1, hid.ptrs(), x.ptrs(), W.ptrs(), dpre.ptrs(), M, K, dx1.ptrs(),
                             *[t.data_ptr() for t in one], s, rs=2)


@pytest.mark.parametrize("B", [12, 50, 77])
def test_x3_heads_sample_fp32_rows(cuda, B):
    """K16x: fp32 head rows (logits / value) vs float64, logp consistent with the logits and the
    sampled action, the step counters advanced once per launch."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.ops import x3

    h = require_hip()
    torch.manual_seed(B)
    A, T, K = 6, 3, 96
    A1 = A + 1
    x = x3.split(torch.relu(torch.randn(B, K, device=cuda)))
    W = x3.split(torch.randn(256, K, device=cuda) * 0.1)
    b = x3.split(torch.randn(256, device=cuda) * 0.1)
    Wh = x3.split(torch.randn(A1, 256, device=cuda) * 0.5)
    bh = x3.split(torch.randn(A1, device=cuda) * 0.1)
    part, S = x3.dense_fwd_part(x, W)
    t = torch.tensor([1], device=cuda)
    ctr = torch.tensor([12345], device=cuda)
    done = torch.zeros(1, dtype=torch.int32, device=cuda)
    act = torch.zeros(T, B, dtype=torch.int64, device=cuda)
    logp, vf = torch.zeros(T, B, device=cuda), torch.zeros(T, B, device=cuda)
    lout, now = torch.zeros(T, B, A, device=cuda), torch.zeros(B, dtype=torch.int64, device=cuda)
    h.x3_heads_sample(part.data_ptr(), S, b.ptrs(), Wh.ptrs(), bh.ptrs(), t.data_ptr(), ctr.data_ptr(), 7,
                      act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(), now.data_ptr(), B, A1,
                      torch.cuda.current_stream().cuda_stream, done=done.data_ptr())
    torch.cuda.synchronize()
    assert int(t) == 2 and int(ctr) == 12346 and int(done) == 0
    hidden = torch.relu(x.float().double() @ W.float().double().t() + b.float().double())
    heads = hidden @ Wh.float().double().t() + bh.float().double()
    assert _rel(lout[1], heads[:, :A]) < FWD_TOL
    assert _rel(vf[1], heads[:, A]) < FWD_TOL
    ref_lp = torch.log_softmax(lout[1].double(), -1).gather(1, act[1][:, None])[:, 0]
    torch.testing.assert_close(logp[1].double(), ref_lp, rtol=1e-5, atol=1e-5)
    assert torch.equal(now, act[1]) and int(act[0].abs().sum()) == 0


@pytest.mark.parametrize("B", [12, 50, 64])
def test_x3_dense_heads_sample_fused_matches_two_launches(cuda, B):
    """K13x + K16x in one launch (per-row-tile tickets, the tile finisher samples its rows) vs the K13x and
    K16x launches: identical actions, log-probs, values and logits (same partial sums, same row math), the
    step counters advanced once per launch, every ticket word back at 0 (three launches in a row)."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.ops import x3

    h = require_hip()
    torch.manual_seed(B)
    A, T, K = 4, 3, 3872
    A1 = A + 1
    x = x3.split(torch.relu(torch.randn(B, K, device=cuda)))
    W = x3.split(torch.randn(256, K, device=cuda) * 0.02)
    b = x3.split(torch.randn(256, device=cuda) * 0.1)
    Wh = x3.split(torch.randn(A1, 256, device=cuda) * 0.5)
    bh = x3.split(torch.randn(A1, device=cuda) * 0.1)
    S = h.x3_dense_fwd_part_slices(B, K, 256)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for fused in (False, True):
        part = torch.zeros(S, B, 256, device=cuda)
        t = torch.tensor([0], device=cuda)
        ctr = torch.tensor([777], device=cuda)
        done = torch.zeros(64, dtype=torch.int32, device=cuda)
        act = torch.zeros(T, B, dtype=torch.int64, device=cuda)
        logp, vf = torch.zeros(T, B, device=cuda), torch.zeros(T, B, device=cuda)
        lout, now = torch.zeros(T, B, A, device=cuda), torch.zeros(B, dtype=torch.int64, device=cuda)
        for _ in range(T):
            if fused:
                h.x3_dense_heads_sample(x.ptrs(), W.ptrs(), B, K, part.data_ptr(), S, b.ptrs(), Wh.ptrs(), bh.ptrs(),
                                        t.data_ptr(), ctr.data_ptr(), 7, act.data_ptr(), logp.data_ptr(), vf.data_ptr(),
                                        lout.data_ptr(), now.data_ptr(), A1, st, done.data_ptr())
            else:
                h.x3_dense_fwd_part(x.ptrs(), W.ptrs(), B, K, 256, part.data_ptr(), S, st)
                h.x3_heads_sample(part.data_ptr(), S, b.ptrs(), Wh.ptrs(), bh.ptrs(), t.data_ptr(), ctr.data_ptr(), 7,
                                  act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(), now.data_ptr(), B,
                                  A1, st, done=done.data_ptr())
        torch.cuda.synchronize()
        assert int(t) == T and int(ctr) == 777 + T and int(done.abs().sum()) == 0
        outs.append((act.clone(), logp.clone(), vf.clone(), lout.clone(), now.clone()))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_forward_value_matches_plain_forward(cuda, dtype):
    """VisionNetwork.forward_value (the rollout's bootstrap value: one fused sampling step into scratch
    rows) equals the value column of the plain forward, on the x3 (fp32) and bf16 fused paths."""
    from ray_memory_management_amd.rllib.models import VisionNetwork

    torch.manual_seed(3)
    m = VisionNetwork(4).to(cuda).to(memory_format=torch.channels_last)
    with torch.no_grad():
        m.heads.weight.normal_(0, 0.05)  # a value column that is not ~0
    if dtype == "bf16":
        m = m.to(torch.bfloat16)
    else:
        m.refresh_x3()
    obs = torch.randint(0, 256, (50, 4, 84, 84), dtype=torch.uint8, device=cuda)
    assert (m.fused_x3_ok(obs) if dtype == "fp32" else m.fused_trunk_ok(obs))
    v = m.forward_value(obs)
    with torch.no_grad():
        ref = m.float()(obs)[1].double() if dtype == "fp32" else m(obs)[1].double()
    tol = 2e-4 if dtype == "fp32" else 3e-2
    assert v.shape == (50,) and v.dtype == torch.float32
    assert _rel(v, ref) < tol, _rel(v, ref)
