"""GPU PPO learner: fused-kernel numerics vs PyTorch reference, HIP-graph path == eager path,
sampler produces sane batches."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, graphs, seed=0):
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner

    torch.manual_seed(seed)
    env = GPUSyntheticAtariVectorEnv(16, cuda, num_actions=4, seed=seed)
    model = VisionNetwork(4)
    learner = PPOLearner(model, {"sgd_minibatch_size": 64, "num_sgd_iter": 2, "use_graphs": graphs}, device=cuda,
                         action_space=env.action_space)
    return env, learner


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_cat_loss_matches_reference(cuda, dt):
    from ray_memory_management_amd.rllib.ppo_learner import (ppo_categorical_loss,
                                                             ppo_categorical_loss_reference)

    torch.manual_seed(3)
    N, A = 513, 6
    logits = (torch.randn(N, A, device=cuda) * 2).to(dt).requires_grad_()
    values = (torch.randn(N, device=cuda)).to(dt).requires_grad_()
    old_logits = torch.randn(N, A, device=cuda)
    act = torch.randint(0, A, (N,), device=cuda)
    old_logp = torch.log_softmax(old_logits, -1).gather(1, act[:, None]).squeeze(1)
    adv = torch.randn(N, device=cuda)
    vt = torch.randn(N, device=cuda) * 3
    coef = torch.tensor([0.2, 4.0, 0.5, 0.01, 0.3], device=cuda)
    tot, stats = ppo_categorical_loss(logits, values, old_logits, act, old_logp, adv, vt, coef)
    (2.0 * tot).backward()
    g1 = (logits.grad.clone(), values.grad.clone())
    logits.grad = values.grad = None
    lf, vf = logits.detach().float().requires_grad_(), values.detach().float().requires_grad_()
    rt, rstats = ppo_categorical_loss_reference(lf, vf, old_logits, act, old_logp, adv, vt, coef)
    (2.0 * rt).backward()
    torch.testing.assert_close(tot.float(), rt, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(stats, rstats, rtol=1e-4, atol=1e-3)
    tol = dict(rtol=2e-2, atol=1e-5) if dt == torch.bfloat16 else dict(rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(g1[0].float(), lf.grad, **tol)
    torch.testing.assert_close(g1[1].float(), vf.grad, **tol)


def test_adam_flat_matches_torch(cuda):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(0)
    n = 10007
    w = torch.randn(n, device=cuda)
    p = w.clone().requires_grad_()
    opt = torch.optim.Adam([p], lr=1e-3)
    master, m1, m2 = w.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    wb = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0, 0.0], device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        g = torch.randn(n, device=cuda)
        p.grad = g.clone()
        opt.step()
        hp[5] += 1
        h.adam_flat(master.data_ptr(), m1.data_ptr(), m2.data_ptr(), g.data_ptr(), False, wb.data_ptr(),
                    hp.data_ptr(), 1.0, n, s)
    torch.testing.assert_close(master, p.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(wb.float(), p.detach(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("offset", [0, 1])
def test_adam_flat_bf16_grad_vector_and_scalar_paths(cuda, offset):
    """bf16 gradients; offset 0 takes the 4-wide vector path (plus a 3-element tail), offset 1
    misaligns every pointer and takes the scalar path. Reference: fp32 torch.optim.Adam."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(1)
    n = 4099
    w = torch.randn(n + offset, device=cuda)[offset:]
    p = w.clone().requires_grad_()
    opt = torch.optim.Adam([p], lr=1e-3)
    master = w.clone() if offset == 0 else torch.cat([w.new_zeros(1), w])[1:]
    m1 = torch.zeros(n + offset, device=cuda)[offset:]
    m2 = torch.zeros(n + offset, device=cuda)[offset:]
    wb = torch.empty(n + offset, dtype=torch.bfloat16, device=cuda)[offset:]
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0, 0.0], device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(4):
        gb = torch.randn(n + offset, device=cuda).to(torch.bfloat16)[offset:]
        p.grad = gb.float()
        opt.step()
        hp[5] += 1
        h.adam_flat(master.data_ptr(), m1.data_ptr(), m2.data_ptr(), gb.data_ptr(), True, wb.data_ptr(),
                    hp.data_ptr(), 1.0, n, s)
    torch.testing.assert_close(master, p.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(wb.float(), p.detach(), rtol=1e-2, atol=1e-2)


def test_graph_matches_eager(cuda):
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler

    env, le = _setup(cuda, False)
    sampler = GPURolloutSampler(env, le.model, fragment=16, use_graphs=False)
    batch = sampler.sample()
    frozen = {k: v.clone() for k, v in batch.items()}
    _, lg = _setup(cuda, True)
    lg.set_weights(le.get_weights())
    torch.manual_seed(123)
    s1 = le.update(type(batch)({k: v.clone() for k, v in frozen.items()}))
    torch.manual_seed(123)
    s2 = lg.update(type(batch)({k: v.clone() for k, v in frozen.items()}))
    assert lg.graphs, "graph capture should succeed on MI355X"
    torch.testing.assert_close(le.master, lg.master, rtol=1e-3, atol=1e-4)
    assert abs(s1["total_loss"] - s2["total_loss"]) < 1e-2 * max(1.0, abs(s1["total_loss"]))


def test_graph_sampler_fills_buffers(cuda):
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler

    env, lg = _setup(cuda, True)
    sampler = GPURolloutSampler(env, lg.model, fragment=12, use_graphs=True)
    sampler.sample()
    b2 = sampler.sample()
    assert sampler._graph is not None
    assert b2.count == 12 * 16
    a = b2["actions"]
    assert int(a.min()) >= 0 and int(a.max()) < 4
    # actions are not constant (the sampler RNG advances per step)
    assert len(torch.unique(a)) > 1
    obs = b2["obs"].view(12, 16, 4, 84, 84)
    assert torch.equal(obs[1, :, 0], obs[0, :, 1])  # frame stack shifts between steps
    assert torch.isfinite(b2["advantages"]).all()
    lp = torch.log_softmax(b2["action_dist_inputs"], -1).gather(1, a[:, None]).squeeze(1)
    torch.testing.assert_close(lp, b2["action_logp"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("C,k,s", [(16, 8, 4), (32, 4, 2)])
def test_conv_bias_relu_fused_matches_torch(cuda, C, k, s):
    from ray_memory_management_amd.rllib.models import ConvReLU

    torch.manual_seed(0)
    cin = 4 if C == 16 else 16
    hw = 84 if C == 16 else 21
    m = ConvReLU(cin, C, k, s, padding=2).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(37, cin, hw, hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = m(x)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    xr = x.detach().float()
    wr = m.weight.detach().float()
    yr = torch.relu(torch.nn.functional.conv2d(xr, wr, m.bias.detach().float(), s, 2))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    # fp32 reference backward through the SAME activation mask (bf16 vs fp32 forward differ in the
    # sign of near-zero pre-activations, which is not what this test is about)
    dpre = gy.float() * (y.float() > 0).float()
    db_ref = dpre.sum((0, 2, 3))
    dw_ref = torch.nn.grad.conv2d_weight(xr, wr.shape, dpre, s, 2)
    dx_ref = torch.nn.grad.conv2d_input(xr.shape, wr, dpre, s, 2)

    def rel(a, b):
        return float((a.float() - b).norm() / b.norm().clamp_min(1e-6))

    assert rel(m.bias.grad, db_ref) < 2e-2
    assert rel(m.weight.grad, dw_ref) < 2e-2
    assert rel(x.grad, dx_ref) < 2e-2


def test_many_graph_replays_stay_finite(cuda):
    """Regression: 1000+ back-to-back SGD-step replays at bench scale must stay finite."""
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner

    torch.manual_seed(1234)
    env = GPUSyntheticAtariVectorEnv(50, cuda, num_actions=4)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 500, "num_sgd_iter": 10}, device=cuda,
                   action_space=env.action_space)
    S = GPURolloutSampler(env, L.model, fragment=100)
    for _ in range(12):
        st = L.update(S.sample())
        assert all(v == v for v in st.values()), st  # no NaN
    assert torch.isfinite(L.master).all()


def test_fused_env_step_semantics(cuda):
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv

    env = GPUSyntheticAtariVectorEnv(7, cuda, num_actions=4, episode_len=3, seed=1)
    env.t.zero_()
    T, B = 5, 7
    buf_obs = torch.zeros((T, B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    rew = torch.full((T, B), -1.0, device=cuda)
    done = torch.full((T, B), -1.0, device=cuda)
    ctr_t = torch.zeros(2, dtype=torch.int64, device=cuda)
    for t in range(T):
        before = env.frames.clone()
        a = torch.randint(0, 4, (B,), device=cuda)
        env.fused_step(a, ctr_t, buf_obs, rew, done, seed=9)
        ctr_t += 1
        assert torch.equal(buf_obs[t], before)                      # current obs stored at row t
        assert torch.equal(env.frames[:, :3], before[:, 1:])        # stack shifted
        # new frame = some pool frame shifted right by 3*(a%4) columns
        nf = env.frames[:, 3]
        for b in range(B):
            sh = int(a[b] % 4) * 3
            unshift = torch.roll(nf[b], -sh, dims=1)
            assert any(torch.equal(unshift, env.pool[k]) for k in range(64))
    assert set(rew.unique().tolist()) <= {0.0, 1.0}
    assert done[2].eq(1).all() and done[0].eq(0).all()              # episode_len = 3


def test_learning_reduces_value_loss(cuda):
    """A few PPO iterations on the synthetic env must reduce the value loss (sanity of training)."""
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler

    env, lg = _setup(cuda, True)
    lg.cfg["lr"] = 1e-3
    lg.hp[0] = 1e-3
    sampler = GPURolloutSampler(env, lg.model, fragment=32)
    first = lg.update(sampler.sample())["vf_loss"]
    for _ in range(6):
        last = lg.update(sampler.sample())["vf_loss"]
    assert last < first


def test_fused_heads_loss_matches_reference(cuda):
    """K5c (merged [N, A+1] head, packed columns, stats accumulated in place) vs fp32 torch."""
    from ray_memory_management_amd.rllib.ppo_learner import ppo_categorical_loss_reference, ppo_heads_loss

    torch.manual_seed(5)
    N, A = 777, 6
    heads = (torch.randn(N, A + 1, device=cuda) * 2).to(torch.bfloat16).requires_grad_()
    old_logits = torch.randn(N, A, device=cuda)
    act = torch.randint(0, A, (N,), device=cuda)
    old_logp = torch.log_softmax(old_logits, -1).gather(1, act[:, None]).squeeze(1)
    adv, vt = torch.randn(N, device=cuda), torch.randn(N, device=cuda) * 3
    cols = torch.cat([old_logits, old_logp[:, None], adv[:, None], vt[:, None], act[:, None].float()], 1).contiguous()
    coef = torch.tensor([0.2, 4.0, 0.5, 0.01, 0.3], device=cuda)
    acc = torch.full((6,), 1.0, device=cuda)  # accumulates on top of what is there
    h = ppo_heads_loss(heads, cols, coef, acc)
    (g,) = torch.autograd.grad(h, heads, grad_outputs=torch.tensor(2.0, device=cuda))
    hf = heads.detach().float().requires_grad_()
    rt, rstats = ppo_categorical_loss_reference(hf[:, :A], hf[:, A], old_logits, act, old_logp, adv, vt, coef)
    (2.0 * rt).backward()
    torch.testing.assert_close(acc - 1.0, rstats, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(g.float(), hf.grad, rtol=2e-2, atol=1e-5)


def test_counter_gathers_walk_index_table(cuda):
    from ray_memory_management_amd import ops

    torch.manual_seed(0)
    n, rows, period = 300, 40, 5
    frames = torch.randint(0, 255, (n, 4, 84, 84), dtype=torch.uint8, device=cuda)
    cols = torch.randn(n, 10, device=cuda)
    idx = torch.randperm(n, device=cuda)[:rows * period].contiguous()
    ctr = torch.zeros(2, dtype=torch.int64, device=cuda)
    for k in range(period + 2):  # wraps modulo period
        sel = idx[(k % period) * rows:(k % period + 1) * rows]
        torch.testing.assert_close(ops.gather_rows(cols, idx, rows=rows, ctr=ctr, period=period), cols[sel])
        x = ops.frames_to_nhwc(frames, idx, rows=rows, ctr=ctr, period=period)
        torch.testing.assert_close(x.float(), (frames[sel].float() / 255.0).to(torch.bfloat16).float())
        ctr.add_(1)


def test_adam_step_counter_matches_host_step(cuda):
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(0)
    n = 4099
    s = torch.cuda.current_stream().cuda_stream
    st = [torch.randn(n, device=cuda) for _ in range(1)] * 2
    ma, mb = st[0].clone(), st[1].clone()
    z = [torch.zeros(n, device=cuda) for _ in range(4)]
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.0, 0.0], device=cuda)
    ctr = torch.zeros(2, dtype=torch.int64, device=cuda)
    for _ in range(4):
        g = torch.randn(n, device=cuda)
        hp[5] += 1
        h.adam_flat(ma.data_ptr(), z[0].data_ptr(), z[1].data_ptr(), g.data_ptr(), False, 0, hp.data_ptr(), 1.0, n, s)
        h.adam_flat(mb.data_ptr(), z[2].data_ptr(), z[3].data_ptr(), g.data_ptr(), False, 0, hp.data_ptr(), 1.0, n, s,
                    step_ctr=ctr.data_ptr() + 8)
        ctr.add_(1)
    torch.testing.assert_close(ma, mb, rtol=0, atol=0)


@pytest.mark.parametrize("M,A", [(500, 4), (37, 6), (130, 15)])
def test_dense_heads_ppo_matches_unfused(cuda, M, A):
    """K15 (heads GEMM + PPO loss stats + dheads + dpre in one launch, K12 without its dpre
    pre-kernel) vs the unfused K14 + K5c + K12 path, and the loss statistics vs fp32."""
    from ray_memory_management_amd.rllib.models import dense_heads, dense_heads_ppo
    from ray_memory_management_amd.rllib.ppo_learner import ppo_heads_loss

    torch.manual_seed(0)
    K = 96
    layer = torch.nn.Linear(K, 256).to(cuda).to(torch.bfloat16)
    heads = torch.nn.Linear(256, A + 1).to(cuda).to(torch.bfloat16)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16).requires_grad_(True)
    cols = torch.zeros(M, A + 4, device=cuda)
    cols[:, :A] = torch.randn(M, A, device=cuda) * 0.1
    cols[:, A] = torch.log_softmax(cols[:, :A], -1)[:, 0] + 0.05 * torch.randn(M, device=cuda)
    cols[:, A + 1] = torch.randn(M, device=cuda)
    cols[:, A + 2] = torch.randn(M, device=cuda)
    cols[:, A + 3] = torch.randint(0, A, (M,), device=cuda).float()
    coef = torch.tensor([0.2, 10.0, 0.5, 0.01, 0.2], device=cuda)
    one = torch.ones((), device=cuda)
    ps = [x, layer.weight, layer.bias, heads.weight, heads.bias]

    acc1 = torch.zeros(6, device=cuda)
    t1 = dense_heads_ppo(x, layer, heads, cols, coef, acc1, one)
    g1 = torch.autograd.grad(t1, ps, grad_outputs=one)
    acc2 = torch.zeros(6, device=cuda)
    h2 = dense_heads(x, layer, heads)
    t2 = ppo_heads_loss(h2, cols, coef, acc2, gout=one)
    g2 = torch.autograd.grad(t2, ps, grad_outputs=one)
    torch.testing.assert_close(acc1, acc2, rtol=1e-3, atol=1e-3)
    for n, a, b in zip(("dx", "dW", "db", "dWh", "dbh"), g1, g2):
        err = float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))
        assert err < 2e-2, (n, err)
    # statistics vs an fp32 evaluation of the same loss on the same (bf16) head outputs
    hf = h2.float()
    lp = torch.log_softmax(hf[:, :A], -1)
    lpo = torch.log_softmax(cols[:, :A], -1)
    act = cols[:, A + 3].long()
    r = torch.exp(lp.gather(1, act[:, None])[:, 0] - cols[:, A])
    adv = cols[:, A + 1]
    surr = torch.minimum(r * adv, r.clamp(0.8, 1.2) * adv)
    vf = torch.clamp((hf[:, A] - cols[:, A + 2]) ** 2, max=10.0)
    ent = -(lp.exp() * lp).sum(-1)
    kl = (lpo.exp() * (lpo - lp)).sum(-1)
    ref = torch.stack([-surr.sum(), vf.sum(), ent.sum(), kl.sum()])
    torch.testing.assert_close(acc1[:4], ref, rtol=2e-3, atol=2e-3)


def test_heads_sample_matches_unfused(cuda):
    """K16 (heads + Gumbel-max sampling + row stores) vs K14 heads + K7 sample_store: same hash
    stream, so actions match exactly; logp / vf / logits to bf16 rounding."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.rllib.models import dense_heads

    h = require_hip()
    torch.manual_seed(0)
    B, A, T, K = 37, 6, 3, 96
    layer = torch.nn.Linear(K, 256).to(cuda).to(torch.bfloat16)
    heads = torch.nn.Linear(256, A + 1).to(cuda).to(torch.bfloat16)
    heads.weight.data *= 8  # spread the logits so sampling is not uniform
    x = torch.randn(B, K, device=cuda).to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    hidden = torch.empty(B, 256, dtype=torch.bfloat16, device=cuda)
    h.dense_relu_fwd(x.data_ptr(), layer.weight.data_ptr(), layer.bias.data_ptr(), B, K, 256, hidden.data_ptr(), s)
    t = torch.tensor([1], device=cuda)
    ctr = torch.tensor([12345], device=cuda)
    outs = []
    for fused in (True, False):
        act = torch.zeros(T, B, dtype=torch.int64, device=cuda)
        logp, vf = torch.zeros(T, B, device=cuda), torch.zeros(T, B, device=cuda)
        lout, now = torch.zeros(T, B, A, device=cuda), torch.zeros(B, dtype=torch.int64, device=cuda)
        if fused:
            h.dense_heads_sample(hidden.data_ptr(), heads.weight.data_ptr(), heads.bias.data_ptr(), t.data_ptr(),
                                 ctr.data_ptr(), 7, act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(),
                                 now.data_ptr(), B, A + 1, s)
        else:
            hd = dense_heads(x, layer, heads).contiguous()
            h.sample_store(hd.data_ptr(), True, hd.data_ptr() + 2 * A, True, t.data_ptr(), ctr.data_ptr(), 7,
                           act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(), now.data_ptr(), B, A, s,
                           ldl=A + 1, ldv=A + 1)
        outs.append((act, logp, vf, lout, now))
    (a1, l1, v1, o1, n1), (a2, l2, v2, o2, n2) = outs
    assert torch.equal(n1, n2) and torch.equal(a1, a2) and int(a1[0].abs().sum()) == 0
    for u, w in ((l1, l2), (v1, v2), (o1, o2)):
        torch.testing.assert_close(u, w, rtol=2e-2, atol=2e-2)
    assert len(set(n1.tolist())) > 1


def test_dense_heads_ppo_gathers_cols_through_index_window(cuda):
    """K15 reading cols[idx[(ctr % period) * M + row]] in place == K15 on pre-gathered cols."""
    from ray_memory_management_amd.rllib.models import dense_heads_ppo

    torch.manual_seed(2)
    M, A, K, period = 50, 4, 64, 3
    layer = torch.nn.Linear(K, 256).to(cuda).to(torch.bfloat16)
    heads = torch.nn.Linear(256, A + 1).to(cuda).to(torch.bfloat16)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    full = torch.randn(M * period, A + 4, device=cuda)
    full[:, A + 3] = torch.randint(0, A, (M * period,), device=cuda).float()
    full[:, A] = -1.5
    idx = torch.randperm(M * period, device=cuda)
    ctr = torch.tensor([4], device=cuda)  # window 4 % 3 = 1
    coef = torch.tensor([0.2, 10.0, 0.5, 0.01, 0.2], device=cuda)
    one = torch.ones((), device=cuda)
    res = []
    for gathered in (False, True):
        xx = x.clone().requires_grad_(True)
        acc = torch.zeros(6, device=cuda)
        if gathered:
            t = dense_heads_ppo(xx, layer, heads, full[idx[M:2 * M]].contiguous(), coef, acc, one)
        else:
            t = dense_heads_ppo(xx, layer, heads, full, coef, acc, one, idx=idx, ctr=ctr, period=period)
        g = torch.autograd.grad(t, [xx, layer.weight, heads.weight], grad_outputs=one)
        res.append((acc, g))
    torch.testing.assert_close(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_heads_sample_advances_step_counters(cuda):
    """K16 with a completion counter: same outputs as without, and the last workgroup bumps the
    row / RNG counters by one and re-arms the counter (many workgroups, repeated launches)."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(1)
    B, A, T = 203, 6, 4
    hidden = torch.randn(B, 256, device=cuda).to(torch.bfloat16)
    heads = torch.nn.Linear(256, A + 1).to(cuda).to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    res = []
    for adv in (False, True):
        ctr_t = torch.tensor([777, 0], dtype=torch.int64, device=cuda)
        done = torch.zeros(1, dtype=torch.int32, device=cuda)
        act = torch.zeros(T, B, dtype=torch.int64, device=cuda)
        logp, vf = torch.zeros(T, B, device=cuda), torch.zeros(T, B, device=cuda)
        lout, now = torch.zeros(T, B, A, device=cuda), torch.zeros(B, dtype=torch.int64, device=cuda)
        for _ in range(T):
            h.dense_heads_sample(hidden.data_ptr(), heads.weight.data_ptr(), heads.bias.data_ptr(),
                                 ctr_t[1:2].data_ptr(), ctr_t[0:1].data_ptr(), 3, act.data_ptr(), logp.data_ptr(),
                                 vf.data_ptr(), lout.data_ptr(), now.data_ptr(), B, A + 1, s,
                                 done.data_ptr() if adv else 0)
            if not adv:
                ctr_t.add_(1)
        torch.cuda.synchronize()
        assert ctr_t.tolist() == [777 + T, T] and int(done) == 0
        res.append((act, logp, vf, lout))
    for u, w in zip(*res):
        assert torch.equal(u, w)


@pytest.mark.parametrize("M", [12, 25, 500])
def test_dense_split_k_partials_feed_k15_k16(cuda, M):
    """K13s (split-K dense layer → fp32 partials) with the reduction in the consumer: the hidden
    K15 rebuilds (Σ partials + b, ReLU, bf16) matches the fp32 reference and K13's bf16 hidden to
    rounding, and K15 / K16 fed from partials match K15 / K16 fed from K13's hidden."""
    from ray_memory_management_amd._native import require_hip

    h = require_hip()
    torch.manual_seed(M)
    K, N, A = 3872, 256, 4
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.02).to(torch.bfloat16)
    b = (torch.randn(N, device=cuda) * 0.1).to(torch.bfloat16)
    wh = (torch.randn(A + 1, N, device=cuda) * 0.1).to(torch.bfloat16)
    bh = (torch.randn(A + 1, device=cuda) * 0.1).to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    S = h.dense_fwd_part_slices(M, K, N)
    assert 1 <= S <= 16
    part = torch.full((S * M * N,), float("nan"), device=cuda)
    h.dense_fwd_part(x.data_ptr(), w.data_ptr(), M, K, N, part.data_ptr(), S, s)
    ref = torch.relu(x.float() @ w.float().t() + b.float())
    pre = part.view(S, M, N).sum(0)
    torch.testing.assert_close(pre + b.float(), x.float() @ w.float().t() + b.float(), rtol=1e-4, atol=1e-4)
    hid = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    h.dense_relu_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, K, N, hid.data_ptr(), s)
    # K15 both ways
    cols = torch.randn(M, A + 4, device=cuda)
    cols[:, A + 3] = torch.randint(0, A, (M,), device=cuda).float()
    coef = torch.tensor([0.2, 10.0, 1.0, 0.01, 0.2], device=cuda)
    one = torch.ones(1, device=cuda)
    res = []
    for use_part in (False, True):
        acc = torch.zeros(6, device=cuda)
        dz = torch.empty(M, A + 1, dtype=torch.bfloat16, device=cuda)
        dpre = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
        hid_out = torch.zeros(M, N, dtype=torch.bfloat16, device=cuda)
        kw = dict(hpart=part.data_ptr(), S=S, hb=b.data_ptr(), hid_out=hid_out.data_ptr()) if use_part else {}
        h.dense_heads_ppo(0 if use_part else hid.data_ptr(), wh.data_ptr(), bh.data_ptr(), cols.data_ptr(),
                          coef.data_ptr(), acc.data_ptr(), one.data_ptr(), M, A + 1, dz.data_ptr(), dpre.data_ptr(), s,
                          **kw)
        res.append((acc, dz, dpre, hid_out))
    (a0, z0, p0, _), (a1, z1, p1, ho) = res
    torch.testing.assert_close(ho.float(), ref, rtol=1e-2, atol=1e-2)
    assert (ho.float() - hid.float()).abs().max() <= 2 ** -6 * max(1.0, float(hid.float().abs().max()))
    torch.testing.assert_close(a1, a0, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(z1.float(), z0.float(), rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(p1.float(), p0.float(), rtol=2e-2, atol=2e-3)
    # K16 both ways: actions agree (same hash stream; hidden differs at most by bf16 rounding)
    t = torch.tensor([0], device=cuda)
    ctr = torch.tensor([99], device=cuda)
    acts = []
    for use_part in (False, True):
        act = torch.zeros(1, M, dtype=torch.int64, device=cuda)
        logp, vf = torch.zeros(1, M, device=cuda), torch.zeros(1, M, device=cuda)
        lout, now = torch.zeros(1, M, A, device=cuda), torch.zeros(M, dtype=torch.int64, device=cuda)
        kw = dict(hpart=part.data_ptr(), S=S, hb=b.data_ptr()) if use_part else {}
        h.dense_heads_sample(0 if use_part else hid.data_ptr(), wh.data_ptr(), bh.data_ptr(), t.data_ptr(),
                             ctr.data_ptr(), 7, act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(),
                             now.data_ptr(), M, A + 1, s, **kw)
        acts.append((act, lout))
    assert float((acts[0][0] == acts[1][0]).float().mean()) >= 0.95
    torch.testing.assert_close(acts[1][1], acts[0][1], rtol=2e-2, atol=2e-2)


def test_trunk_push_mode_matches_frame_push_then_trunk(cuda):
    """K10 push mode (K19 folded in): shifting the device frame stack, appending the new frames and
    storing rollout row t inside the trunk launch gives the same stack, row and h2 as K19 followed
    by the plain K10 forward."""
    from ray_memory_management_amd._native import require_hip
    from ray_memory_management_amd.rllib.models import nature_trunk

    h = require_hip()
    torch.manual_seed(3)
    B, T = 13, 4
    c1 = torch.nn.Conv2d(4, 16, 8, 4, padding=2).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    c2 = torch.nn.Conv2d(16, 32, 4, 2, padding=2).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    stack0 = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    nf = torch.randint(0, 256, (B, 84, 84), dtype=torch.uint8, device=cuda)
    t = torch.tensor([2], device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    # reference: K19 then K10
    st_a, rows_a = stack0.clone(), torch.zeros((T, B, 4, 84, 84), dtype=torch.uint8, device=cuda)
    h.frame_push(st_a.data_ptr(), nf.data_ptr(), rows_a.data_ptr(), t.data_ptr(), B, 84 * 84, s)
    h2_a = nature_trunk(st_a, c1.weight, c1.bias, c2.weight, c2.bias)
    # push mode
    st_b, rows_b = stack0.clone(), torch.zeros_like(rows_a)
    h2_b = torch.empty_like(h2_a)
    h.nature_trunk_fwd_push(st_b.data_ptr(), nf.data_ptr(), rows_b.data_ptr(), t.data_ptr(), B, c1.weight.data_ptr(),
                            list(c1.weight.stride()), c1.bias.data_ptr(), c2.weight.data_ptr(),
                            list(c2.weight.stride()), c2.bias.data_ptr(), h2_b.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(st_a, st_b) and torch.equal(rows_a, rows_b)
    assert torch.equal(st_b[:, :3], stack0[:, 1:]) and torch.equal(st_b[:, 3], nf)
    assert torch.equal(h2_a, h2_b)


@pytest.mark.parametrize("B", [12, 25, 33, 50, 64])  # 33-64: four rows per wave, all preloaded
def test_heads_sample_single_workgroup_advance(cuda, B):
    """K16 with the step advance for small batches runs as ONE workgroup (no device-scope fence):
    same rows as the multi-workgroup launch and the counters advance by exactly one."""
    import subprocess
    import sys

    code = f"""
import torch, json
from ray_memory_management_amd._native import require_hip
h = require_hip(); torch.manual_seed(1); B, A = {B}, 6
wh = (torch.randn(A + 1, 256, device='cuda') * 0.3).to(torch.bfloat16)
bh = torch.zeros(A + 1, device='cuda', dtype=torch.bfloat16)
hid = torch.relu(torch.randn(B, 256, device='cuda')).to(torch.bfloat16)
ct = torch.tensor([5, 1], device='cuda'); done = torch.zeros(1, dtype=torch.int32, device='cuda')
act = torch.zeros(3, B, dtype=torch.int64, device='cuda'); logp = torch.zeros(3, B, device='cuda')
vf = torch.zeros(3, B, device='cuda'); lout = torch.zeros(3, B, A, device='cuda'); now = torch.zeros(B, dtype=torch.int64, device='cuda')
for _ in range(2):
    h.dense_heads_sample(hid.data_ptr(), wh.data_ptr(), bh.data_ptr(), ct[1:].data_ptr(), ct[:1].data_ptr(), 7,
                         act.data_ptr(), logp.data_ptr(), vf.data_ptr(), lout.data_ptr(), now.data_ptr(), B, A + 1,
                         torch.cuda.current_stream().cuda_stream, done.data_ptr())
torch.cuda.synchronize()
print(json.dumps({{"ct": ct.tolist(), "act": act.tolist(), "logp": logp.tolist(), "done": int(done)}}))
"""
    outs = []
    for multi, wpw in (("0", "4"), ("1", "4"), ("1", "1")):  # one workgroup / 4 rows per WG / 1 row per WG
        env = dict(os.environ, RMM_K16_MULTI=multi, RMM_K16_WPW=wpw)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    a, b, c = outs
    assert a["ct"] == [7, 3] and b["ct"] == [7, 3] and c["ct"] == [7, 3]  # rng counter 5 -> 7, row 1 -> 3
    assert a["act"] == b["act"] == c["act"] and a["logp"] == b["logp"] == c["logp"] and c["done"] == 0
    assert a["act"][0] == [0] * B and any(a["act"][1]) and any(a["act"][2])
    assert a["done"] == 0 and b["done"] == 0



@pytest.mark.parametrize("chain_cap", [3, 4])
def test_parity_counters_match_ticket_bump(cuda, monkeypatch, chain_cap):
    """Chained SGD graphs with parity step counters (K6 writes the advanced counters into the other
    copy) vs the last-workgroup ticket bump in place: bit-identical weights and counters over two
    updates, for an odd chain (3: the last step bumps in place) and an even one (4)."""
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork

    monkeypatch.setenv("RMM_SGD_CHAIN", str(chain_cap))
    env = GPUSyntheticAtariVectorEnv(16, cuda, num_actions=4, seed=0)
    torch.manual_seed(0)
    base = VisionNetwork(4)
    cfg = {"sgd_minibatch_size": 64, "num_sgd_iter": 3, "use_graphs": True}  # 12 SGD steps per update
    learners = {}
    for parity in ("0", "1"):
        monkeypatch.setenv("RMM_CTR_PARITY", parity)
        m = VisionNetwork(4)
        m.load_state_dict(base.state_dict())
        learners[parity] = PPOLearner(m, dict(cfg), device=cuda, action_space=env.action_space)
    sampler = GPURolloutSampler(env, learners["0"].model, fragment=16, use_graphs=False)
    first = sampler.sample()
    Batch = type(first)
    batches = [{k: v.clone() for k, v in first.items()}, {k: v.clone() for k, v in sampler.sample().items()}]
    for parity, ln in learners.items():
        monkeypatch.setenv("RMM_CTR_PARITY", parity)
        for i, b in enumerate(batches):
            torch.manual_seed(100 + i)
            ln.update(Batch({k: v.clone() for k, v in b.items()}))
        assert ln.graphs and ln._chain == chain_cap
    a, b = learners["0"], learners["1"]
    assert torch.equal(a.master, b.master)
    assert torch.equal(a.w_bf16, b.w_bf16)
    assert torch.equal(a.ctr, b.ctr)
    assert int(b.ctr[1]) == 24  # Adam steps: 2 updates x 12


@pytest.mark.parametrize("split", ["1", "2"])
@pytest.mark.parametrize("chain_cap,graphs", [(3, True), (4, True), (4, False)])
def test_tail_adam_matches_k6(cuda, monkeypatch, chain_cap, graphs, split):
    """K6 folded into the K10 trunk-reduce launch (RMM_TAIL_ADAM=1: FusedAdam on the trunk range in
    the reduce epilogue + extra Adam workgroups over the dense + heads range) vs the separate K6:
    bit-identical master / moments / bf16 weights / step counters over two updates — chained graphs
    with parity counters (odd chain: the last step bumps in place) and the eager path."""
    from ray_memory_management_amd.rllib.ppo_learner import GPURolloutSampler, PPOLearner
    from ray_memory_management_amd.rllib.env import GPUSyntheticAtariVectorEnv
    from ray_memory_management_amd.rllib.models import VisionNetwork

    monkeypatch.setenv("RMM_SGD_CHAIN", str(chain_cap))
    # split "2": K12 row split; with tail Adam its finalize (+ Adam) is deferred into the reduce launch,
    # the reference side runs split K12 -> finalize kernel -> K6 (the same bf16-rounded sums)
    monkeypatch.setenv("RMM_K12_SPLIT", split)
    env = GPUSyntheticAtariVectorEnv(16, cuda, num_actions=4, seed=0)
    torch.manual_seed(0)
    base = VisionNetwork(4)
    cfg = {"sgd_minibatch_size": 128 if split == "2" else 64, "num_sgd_iter": 3, "use_graphs": graphs}
    learners = {}
    for tail in ("0", "1"):
        monkeypatch.setenv("RMM_TAIL_ADAM", tail)
        m = VisionNetwork(4)
        m.load_state_dict(base.state_dict())
        learners[tail] = PPOLearner(m, dict(cfg), device=cuda, action_space=env.action_space)
    sampler = GPURolloutSampler(env, learners["0"].model, fragment=16, use_graphs=False)
    first = sampler.sample()
    Batch = type(first)
    batches = [{k: v.clone() for k, v in first.items()}, {k: v.clone() for k, v in sampler.sample().items()}]
    for tail, ln in learners.items():
        monkeypatch.setenv("RMM_TAIL_ADAM", tail)
        for i, b in enumerate(batches):
            torch.manual_seed(100 + i)
            ln.update(Batch({k: v.clone() for k, v in b.items()}))
        assert ln.graphs == graphs and ln._tail_adam() == (tail == "1")
    a, b = learners["0"], learners["1"]
    for name in ("master", "m1", "m2", "w_bf16", "ctr"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert int(b.ctr[1]) == (12 if split == "2" else 24)  # Adam steps: 2 updates x (256 / mbs) x 3
