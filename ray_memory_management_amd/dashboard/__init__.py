"""Dashboard (JSON + Prometheus HTTP API). Parity: reference dashboard/ (head + modules)."""
from ray_memory_management_amd.dashboard.head import DashboardHead  # noqa: F401
