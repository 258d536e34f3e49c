"""Distributed tracing (reference python/ray/util/tracing): see tracing_helper.py."""
from ray_memory_management_amd.util.tracing.tracing_helper import (  # noqa: F401
    _is_tracing_enabled, _setup_tracing, execution_span, inject, set_exporter)
