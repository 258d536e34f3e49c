"""Hyperparameter tuning. Parity: reference python/ray/tune/__init__.py."""
from ray_memory_management_amd.tune import schedulers, search, stopper  # noqa: F401
from ray_memory_management_amd.tune.callback import Callback  # noqa: F401
from ray_memory_management_amd.tune.error import TuneError  # noqa: F401
from ray_memory_management_amd.tune.execution import Trial  # noqa: F401
from ray_memory_management_amd.tune.progress_reporter import (  # noqa: F401
    CLIReporter, JupyterNotebookReporter, ProgressReporter)
from ray_memory_management_amd.tune.registry import register_env, register_trainable  # noqa: F401
from ray_memory_management_amd.tune.result_grid import ExperimentAnalysis, ResultGrid  # noqa: F401
from ray_memory_management_amd.tune.search.sample import (  # noqa: F401
    choice, grid_search, lograndint, loguniform, qlograndint, qloguniform, qrandint, qrandn, quniform, randint, randn,
    sample_from, uniform)
from ray_memory_management_amd.tune.stopper import Stopper  # noqa: F401
from ray_memory_management_amd.tune.syncer import SyncConfig  # noqa: F401
from ray_memory_management_amd.tune.trainable import (  # noqa: F401
    PlacementGroupFactory, Trainable, checkpoint_dir, report, with_parameters, with_resources)
from ray_memory_management_amd.tune.tune_config import TuneConfig  # noqa: F401
from ray_memory_management_amd.tune.tuner import Tuner, run, run_experiments  # noqa: F401
from ray_memory_management_amd.tune.experiment import (  # noqa: F401
    Experiment, convert_to_experiment_list, create_scheduler, create_searcher)
from ray_memory_management_amd.air.session import (  # noqa: F401
    get_trial_dir, get_trial_id, get_trial_name, get_trial_resources)


def is_session_enabled() -> bool:
    """True inside a Tune trial / Train worker (reference tune.is_session_enabled)."""
    from ray_memory_management_amd.air import session as _s

    return _s._get_session(warn=False) is not None

__all__ = ["SyncConfig", "CLIReporter", "JupyterNotebookReporter", "ProgressReporter", "Trainable", "TuneError", "Tuner", "TuneConfig", "ResultGrid", "ExperimentAnalysis", "run",
           "run_experiments", "report", "checkpoint_dir", "with_parameters", "with_resources", "Callback", "Stopper",
           "PlacementGroupFactory", "grid_search", "choice", "uniform", "quniform", "loguniform", "qloguniform",
           "randn", "qrandn", "randint", "qrandint", "lograndint", "qlograndint", "sample_from", "register_env",
           "register_trainable", "schedulers", "search", "stopper", "Trial"]
