"""Legacy Train API + train.torch helpers. Mirrors reference python/ray/train/tests/test_trainer.py
(Trainer.start / run / run_iterator, callbacks, report / world_rank / save_checkpoint /
load_checkpoint) and test_torch_utils (accelerate / prepare_optimizer / enable_reproducibility)."""
import torch

import ray_memory_management_amd as ray
from ray_memory_management_amd import train


def _loop(config):
    import torch.distributed as dist

    from ray_memory_management_amd import train as T

    ck = T.load_checkpoint()
    start = ck["epoch"] + 1 if ck else 0
    for e in range(start, start + config["epochs"]):
        t = torch.tensor([float(T.world_rank() + 1)])
        dist.all_reduce(t)
        T.report(epoch=e, total=float(t), rank=T.world_rank())
        T.save_checkpoint(epoch=e)
    return T.world_size() * 10 + T.world_rank()


class Collect(train.TrainingCallback):
    def __init__(self):
        self.results, self.finished = [], None

    def handle_result(self, results, **info):
        self.results.append(results)

    def finish_training(self, error=False, **info):
        self.finished = error


def test_legacy_trainer_run_iterator_checkpoint(ray_start):
    t = train.Trainer("torch", num_workers=2)
    t.start()
    cb = Collect()
    out = t.run(_loop, config={"epochs": 2}, callbacks=[cb])
    assert sorted(out) == [20, 21] and cb.finished is False
    assert len(cb.results) == 2 and all(len(r) == 1 for r in cb.results)
    assert {r["total"] for rs in cb.results for r in rs} == {3.0}
    assert t.latest_checkpoint["epoch"] == 1
    it = t.run_iterator(_loop, config={"epochs": 1}, checkpoint=t.latest_checkpoint)
    rounds = list(it)
    assert rounds[0][0]["epoch"] == 2 and sorted(it.get_final_results()) == [20, 21]
    t.shutdown()


def test_torch_accelerate_and_reproducibility():
    from ray_memory_management_amd.train import torch as tt

    tt.enable_reproducibility(3)
    a = torch.rand(3)
    tt.enable_reproducibility(3)
    assert torch.equal(a, torch.rand(3))
    torch.use_deterministic_algorithms(False)
    tt.accelerate(amp=True)
    try:
        m = tt.prepare_model(torch.nn.Linear(4, 2))
        opt = tt.prepare_optimizer(torch.optim.SGD(m.parameters(), lr=0.1))
        y = m(torch.randn(5, 4))
        assert y.dtype == torch.float32
        y.sum().backward()
        opt.step()
        opt.zero_grad()
        assert "state" in opt.state_dict()
    finally:
        tt.accelerate(amp=False)
    prof = tt.TorchWorkerProfiler()
    with torch.profiler.profile(on_trace_ready=prof.trace_handler, schedule=torch.profiler.schedule(
            wait=0, warmup=0, active=1)) as p:
        torch.ones(8).sum()
        p.step()
    traces = prof.get_and_clear_profile_traces()["_train_torch_profiler_traces"]
    assert len(traces) >= 1 and "traceEvents" in next(iter(traces.values()))
