"""Search algorithms. Parity: reference python/ray/tune/search/__init__.py."""
from ray_memory_management_amd.tune.search.sample import (  # noqa: F401
    Categorical, Domain, Float, Function, Integer, choice, grid_search, loguniform, randint, sample_from, uniform)
from ray_memory_management_amd.tune.search.variant_generator import (  # noqa: F401
    BasicVariantGenerator, ConcurrencyLimiter, Repeater, Searcher, generate_variants)

from ray_memory_management_amd.tune.search.bayesopt import BayesOptSearch  # noqa: F401

__all__ = ["BayesOptSearch", "BasicVariantGenerator", "ConcurrencyLimiter", "Repeater", "Searcher", "generate_variants"]
