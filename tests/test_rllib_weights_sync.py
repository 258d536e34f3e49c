"""Learner → rollout-worker weight sync rules (CPU, stubs):

* HBM weight publication (flat bf16 + layout) is used only when the remote rollout workers are the
  GPU classes that understand it; a plain RolloutWorker also unpacks it if it ever gets one;
* PPO.set_weights (and so checkpoint restore into a live trainer) refreshes the device weight
  refs, so the next iteration does not push pre-restore weights to the rollout workers."""
import types

import numpy as np
import torch

from ray_memory_management_amd.rllib.algorithms.ppo import PPO
from ray_memory_management_amd.rllib.evaluation.rollout_worker import unpack_flat_weights


def _flat_publication(sd):
    flat, layout, off = [], [], 0
    for k, v in sd.items():
        flat.append(v.reshape(-1).to(torch.bfloat16))
        layout.append((k, off, tuple(v.shape), tuple(v.stride())))
        off += v.numel()
    return {"__rmm_flat_bf16__": torch.cat(flat), "__rmm_layout__": layout}


def test_unpack_flat_weights_round_trip():
    sd = {"a.weight": torch.randn(4, 3), "a.bias": torch.randn(4), "b.weight": torch.randn(2, 4)}
    out = unpack_flat_weights(_flat_publication(sd))
    assert set(out) == set(sd)
    for k in sd:
        assert out[k].shape == sd[k].shape and out[k].dtype == torch.float32
        assert torch.equal(out[k], sd[k].to(torch.bfloat16).float())


def test_plain_rollout_worker_loads_flat_publication():
    from ray_memory_management_amd.rllib.evaluation.rollout_worker import RolloutWorker

    w = RolloutWorker.__new__(RolloutWorker)
    model = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.BatchNorm1d(4))
    loaded = {}

    class _Pol:
        pass

    pol = _Pol()
    pol.model = model
    pol.set_weights = lambda ws: (loaded.update(ws), model.load_state_dict(ws))
    w.policy = pol
    new = {k: torch.randn_like(v) for k, v in model.state_dict().items() if v.is_floating_point() and v.dim() > 0}
    params = {k: new[k] for k in ("0.weight", "0.bias")}
    w.set_weights(_flat_publication(params))
    assert torch.equal(model[0].weight.detach(), params["0.weight"].to(torch.bfloat16).float())
    assert "1.running_mean" in loaded  # buffers kept (not in the learner's parameter layout)


def _stub_ppo(remote_cls_name, gpu_worker=0.5):
    algo = PPO.__new__(PPO)
    algo.algo_config = types.SimpleNamespace(num_gpus_per_learner_worker=1, num_gpus_per_worker=gpu_worker,
                                             gpu_rollouts=False)
    algo.workers = types.SimpleNamespace(remote_worker_class=type(remote_cls_name, (), {}))
    return algo


def test_device_weights_only_for_gpu_rollout_classes():
    assert _stub_ppo("HybridRolloutWorker")._device_weights_ok()
    assert _stub_ppo("GPURolloutWorker")._device_weights_ok()
    assert not _stub_ppo("RolloutWorker")._device_weights_ok()  # non-registry env / env_creator
    assert not _stub_ppo("HybridRolloutWorker", gpu_worker=0)._device_weights_ok()


def test_set_weights_refreshes_device_refs():
    calls = []

    class _LG:
        def set_weights(self, w):
            calls.append("set")

        def weights_ref(self):
            return "host-ref"

        def device_weights_refs(self):
            calls.append("dev")
            return ["fresh-dev-ref"]

    class _Local:
        def set_weights(self, w):
            pass

    algo = PPO.__new__(PPO)
    algo.learner_group = _LG()
    algo._dev_refs = ["stale-dev-ref"]
    algo.workers = types.SimpleNamespace(local_worker=lambda: _Local(), sync_weights=lambda ref=None: None)
    algo.set_weights({"w": np.zeros(3)})
    assert algo._dev_refs == ["fresh-dev-ref"] and calls == ["set", "dev"]
