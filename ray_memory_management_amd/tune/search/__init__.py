"""Search algorithms. Parity: reference python/ray/tune/search/__init__.py."""
from ray_memory_management_amd.tune.search.sample import (  # noqa: F401
    Categorical, Domain, Float, Function, Integer, choice, grid_search, loguniform, randint, sample_from, uniform)
from ray_memory_management_amd.tune.search.variant_generator import (  # noqa: F401
    BasicVariantGenerator, ConcurrencyLimiter, Repeater, Searcher, generate_variants)

from ray_memory_management_amd.tune.search.bayesopt import BayesOptSearch  # noqa: F401

# reference search/__init__.py constants + the SearchAlgorithm / SearchGenerator names (in this
# framework every searcher is driven through the Searcher interface directly)
UNRESOLVED_SEARCH_SPACE = "Trial config contains unresolved search-space values ({par}); the searcher {cls} " \
                          "cannot handle them — pass the space to the searcher or use BasicVariantGenerator."
UNDEFINED_SEARCH_SPACE = "Trying to sample a configuration from {cls}, but no search space has been defined " \
                         "(pass `space` to the searcher, or `param_space`/`config` to Tune)."
UNDEFINED_METRIC_MODE = "Trying to sample a configuration from {cls}, but the `metric` ({metric}) or `mode` " \
                        "({mode}) parameters have not been set."
SearchAlgorithm = Searcher
SearchGenerator = Searcher

__all__ = ["BayesOptSearch", "BasicVariantGenerator", "ConcurrencyLimiter", "Repeater", "Searcher", "generate_variants"]
