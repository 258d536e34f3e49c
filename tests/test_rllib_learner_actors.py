"""PPO through the runtime with learner ACTORS (CPU, gloo): N data-parallel learners fed by
rollout-worker actors through the object store. Mirrors the reference's
rllib/execution/tests/test_multi_gpu_learner_thread.py and rllib/algorithms/ddppo/tests/test_ddppo.py
(replicas stay in sync, learning runs end to end), plus the learner-side ingest path."""
import numpy as np
import pytest
import torch


def _cfg(n_learners=2, workers=2, postprocess_on_learner=True):
    from ray_memory_management_amd.rllib.algorithms.ppo import PPOConfig

    return (PPOConfig().environment("SyntheticAtariVec-v0", env_config={"episode_len": 12})
            .rollouts(num_rollout_workers=workers, num_envs_per_worker=2, rollout_fragment_length=8,
                      postprocess_on_learner=postprocess_on_learner)
            .training(train_batch_size=32, sgd_minibatch_size=8, num_sgd_iter=2, lr=1e-3)
            .resources(num_learner_workers=n_learners, num_gpus_per_learner_worker=0)
            .debugging(seed=3))


def test_two_learner_actors_stay_identical(ray_start):
    algo = _cfg().build()
    try:
        for _ in range(2):
            r = algo.train()
        st = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert st["num_learners"] == 2 and np.isfinite(st["total_loss"])
        assert r["num_env_steps_trained"] == 64
        d = algo.learner_group.weights_digests()
        assert len(d) == 2 and d[0] == d[1]  # data-parallel replicas agree bit-for-bit
        # the rollout workers received the learners' weights (published as one store object)
        lw = algo.get_weights()
        pw = algo.get_policy().get_weights()
        for k, v in lw.items():
            np.testing.assert_array_equal(np.asarray(v), pw[k].numpy())
    finally:
        algo.stop()


def test_four_learner_actors_stay_identical():
    """A wider data-parallel group (the 1-node bench runs one learner per GPU, up to 8): four gloo
    learners, one rollout worker each, stay bit-identical and train on every worker's samples."""
    import ray_memory_management_amd as ray

    ray.init(num_cpus=8, object_store_memory=256 << 20)
    try:
        algo = _cfg(n_learners=4, workers=4).build()
        try:
            for _ in range(2):
                r = algo.train()
            st = r["info"]["learner"]["default_policy"]["learner_stats"]
            assert st["num_learners"] == 4 and np.isfinite(st["total_loss"])
            assert r["num_env_steps_trained"] >= 64
            d = algo.learner_group.weights_digests()
            assert len(d) == 4 and len(set(d)) == 1
        finally:
            algo.stop()
    finally:
        ray.shutdown()


def test_learner_actor_checkpoint_roundtrip(ray_start, tmp_path):
    algo = _cfg(n_learners=1, workers=1).build()
    try:
        algo.train()
        path = algo.save(str(tmp_path))
        w0 = algo.get_weights()
        algo.train()
        algo.restore(path)
        w1 = algo.get_weights()
        for k in w0:
            np.testing.assert_array_equal(np.asarray(w0[k]), np.asarray(w1[k]))
    finally:
        algo.stop()


def test_fragment_ingest_matches_worker_postprocessing():
    """GAE on the learner (fragment ingest) == GAE in the rollout worker (reference placement)."""
    from ray_memory_management_amd.rllib.evaluation.rollout_worker import RolloutWorker
    from ray_memory_management_amd.rllib.execution.sample_ingest import fragments_to_batch_cpu
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch

    base = {"env": "SyntheticAtariVec-v0", "num_envs_per_worker": 3, "rollout_fragment_length": 16,
            "env_config": {"episode_len": 7}, "gamma": 0.97, "lambda": 0.9, "lambda_": 0.9, "model": {}}
    torch.manual_seed(0)
    w1 = RolloutWorker(None, {**base, "postprocess_on_learner": True}, 1, 1, seed=5)
    torch.manual_seed(0)
    w2 = RolloutWorker(None, {**base, "postprocess_on_learner": False}, 1, 1, seed=5)
    w2.set_weights(w1.get_weights())
    torch.manual_seed(11)
    f = w1.sample()
    torch.manual_seed(11)
    b = w2.sample()
    obs, cols = fragments_to_batch_cpu([f], 0.97, 0.9, standardize=False)
    np.testing.assert_array_equal(obs.numpy(), b[SampleBatch.OBS])
    A = 4
    np.testing.assert_allclose(cols[:, A + 1].numpy(), b[SampleBatch.ADVANTAGES], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(cols[:, A + 2].numpy(), b[SampleBatch.VALUE_TARGETS], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(cols[:, A + 3].numpy().astype(np.int64), b[SampleBatch.ACTIONS])
    # dones came from truncations at episode_len: GAE must not bootstrap across them
    assert f["_raw"][:, A + 3].sum() > 0


def test_schedules_and_grad_clip_cpu():
    from ray_memory_management_amd.rllib.models import VisionNetwork
    from ray_memory_management_amd.rllib.ppo_learner import PPOLearner
    from ray_memory_management_amd.rllib.sample_batch import SampleBatch
    from ray_memory_management_amd.rllib.utils.schedules import PiecewiseSchedule

    s = PiecewiseSchedule([[0, 1.0], [100, 0.0]])
    assert s(0) == 1.0 and abs(s(50) - 0.5) < 1e-9 and s(1000) == 0.0
    torch.manual_seed(0)
    L = PPOLearner(VisionNetwork(4), {"sgd_minibatch_size": 8, "num_sgd_iter": 1, "grad_clip": 0.5,
                                      "lr_schedule": [[0, 1e-3], [16, 0.0]],
                                      "entropy_coeff_schedule": [[0, 0.02], [16, 0.0]]}, device="cpu")
    n = 16
    batch = lambda: SampleBatch({SampleBatch.OBS: torch.randint(0, 255, (n, 4, 84, 84), dtype=torch.uint8),  # noqa
                                 SampleBatch.ACTIONS: torch.randint(0, 4, (n,)),
                                 SampleBatch.ACTION_LOGP: torch.full((n,), -1.386),
                                 SampleBatch.ACTION_DIST_INPUTS: torch.zeros(n, 4),
                                 SampleBatch.ADVANTAGES: torch.randn(n), SampleBatch.VALUE_TARGETS: torch.randn(n)})
    st = L.update(batch())
    assert st["cur_lr"] == 1e-3 and st["entropy_coeff"] == 0.02
    st = L.update(batch())
    assert st["cur_lr"] == 0.0 and st["entropy_coeff"] == 0.0  # schedules advanced by trained timesteps
