"""reference python/ray/tune/analysis: ExperimentAnalysis (from a run or an experiment directory)."""
from ray_memory_management_amd.tune.result_grid import ExperimentAnalysis  # noqa: F401
