"""``tune`` command line (reference python/ray/tune/cli/{scripts,commands}.py): list the trials of an
experiment directory (``ls``) or the experiments of a project directory (``lsx``), as a table or
CSV, with column selection, filtering, sorting and a row limit.

Usage: ``python -m ray_memory_management_amd.tune.cli ls ~/ray_results/my_exp --sort score --desc``."""
from ray_memory_management_amd.tune.cli.commands import list_experiments, list_trials  # noqa: F401
