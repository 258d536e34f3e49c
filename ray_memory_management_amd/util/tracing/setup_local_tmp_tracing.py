"""Tracing startup hook writing spans to /tmp/spans/<pid>.json, one JSON object per line
(reference python/ray/util/tracing/setup_local_tmp_tracing.py). Use as
``ray.init(_tracing_startup_hook="ray_memory_management_amd.util.tracing.setup_local_tmp_tracing:setup_tracing")``."""
import json
import os

from ray_memory_management_amd.util.tracing.tracing_helper import set_exporter

SPAN_DIR = os.environ.get("RMM_SPAN_DIR", "/tmp/spans")


def setup_tracing() -> None:
    os.makedirs(SPAN_DIR, exist_ok=True)
    path = os.path.join(SPAN_DIR, f"{os.getpid()}.json")

    def export(span):
        with open(path, "a") as f:
            f.write(json.dumps(span) + "\n")

    set_exporter(export)
