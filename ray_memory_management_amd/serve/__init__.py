"""Model serving. Parity: reference python/ray/serve/__init__.py."""
from ray_memory_management_amd.serve.api import (  # noqa: F401
    Application, Deployment, delete, deployment, get_deployment, get_deployment_handle, http_port, ingress,
    list_deployments, run, shutdown, start, status)
from ray_memory_management_amd.serve.batching import batch  # noqa: F401
from ray_memory_management_amd.serve.config import AutoscalingConfig, DeploymentConfig, HTTPOptions  # noqa: F401
from ray_memory_management_amd.serve.context import get_replica_context  # noqa: F401
from ray_memory_management_amd.serve.handle import RayServeHandle, RayServeSyncHandle  # noqa: F401

__all__ = ["batch", "deployment", "delete", "get_deployment", "get_replica_context", "ingress", "list_deployments",
           "run", "shutdown", "start", "status", "Deployment", "Application", "RayServeHandle", "RayServeSyncHandle",
           "AutoscalingConfig", "DeploymentConfig", "HTTPOptions", "http_port", "get_deployment_handle"]


def __getattr__(name):
    import importlib

    if name in ("drivers", "http_adapters", "air_integrations"):
        return importlib.import_module(f"ray_memory_management_amd.serve.{name}")
    if name == "DAGDriver":
        return importlib.import_module("ray_memory_management_amd.serve.drivers").DAGDriver
    if name == "PredictorDeployment":
        return importlib.import_module("ray_memory_management_amd.serve.air_integrations").PredictorDeployment
    raise AttributeError(name)
