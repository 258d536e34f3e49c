"""Autoscaler. Parity: reference python/ray/autoscaler/ (NodeProvider interface, StandardAutoscaler,
resource-demand bin packing, idle-node termination, ``sdk.request_resources``).

Cloud node providers (AWS/GCP/Azure/...) need network access this framework's targets do not have;
the shipped provider is the head-backed virtual-node provider (reference
``autoscaler/_private/fake_multi_node``), and ``NodeProvider`` is the extension point for real ones.
"""
from ray_memory_management_amd.autoscaler import sdk  # noqa: F401
from ray_memory_management_amd.autoscaler.node_provider import NodeProvider  # noqa: F401
