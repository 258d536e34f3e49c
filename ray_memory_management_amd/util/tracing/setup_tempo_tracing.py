"""reference python/ray/util/tracing/setup_tempo_tracing.py exports over OTLP/gRPC to Grafana
Tempo; that needs the opentelemetry OTLP exporter, which is not installed in this stack."""


def setup_tracing() -> None:
    raise ImportError("setup_tempo_tracing needs opentelemetry-exporter-otlp, which is not installed; "
                      "use ray_memory_management_amd.util.tracing.setup_local_tmp_tracing:setup_tracing")
