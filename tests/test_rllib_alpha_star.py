"""AlphaStar-style league on rock-paper-scissors: learners train through the multi-agent
machinery, matchmaking follows the league builder, win rates are tracked and a snapshot joins the
league once a learner beats it. Mirrors reference rllib/algorithms/alpha_star/tests/test_alpha_star.py
(compilation on a 2-player game) plus the league mechanics."""
import numpy as np


def test_matchmaker_pairs_learner_with_weighted_opponent():
    from ray_memory_management_amd.rllib.algorithms.alpha_star import _Matchmaker

    mm = _Matchmaker(["main_0", "main_exploiter_0"], {"main_0": [("random_0", 1.0), ("main_0", 0.0)],
                                                      "main_exploiter_0": [("main_0", 1.0)]})
    assert mm(0, episode=0) == "main_0" and mm(1, episode=0) == "random_0"
    assert mm(0, episode=1) == "main_exploiter_0" and mm(1, episode=1) == "main_0"


def test_league_learns_and_snapshots(ray_shared):
    from ray_memory_management_amd.rllib.algorithms import get_algorithm_class

    cfg = (get_algorithm_class("AlphaStar").get_default_config().environment("RockPaperScissors-v0")
           .rollouts(num_rollout_workers=1, rollout_fragment_length=100)
           .training(train_batch_size=400, lr=1e-2, entropy_coeff=0.0)
           .debugging(seed=0))
    cfg.league_random_policy_probs = [0.7, 0.15, 0.15]  # the seed opponent over-plays rock
    cfg.league_builder_config = {**cfg.league_builder_config, "win_rate_threshold_for_new_snapshot": 0.6,
                                 "min_matches_for_snapshot": 10, "num_league_exploiters": 0}
    a = cfg.build()
    assert set(a.learners) == {"main_0", "main_exploiter_0"} and a.league == ["random_0"]
    added = []
    for _ in range(25):
        r = a.train()
        lg = r["info"]["learner"]["league"]["learner_stats"]
        added += lg["snapshots_added"]
        if added:
            break
    assert a._p_win("main_0", "random_0") > 0.6 or any(x.startswith("main_0") for x in added), a.win
    assert added and len(a.league) >= 2 and "main_0" in r["info"]["learner"]
    a.stop()
