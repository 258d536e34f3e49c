"""Parity: reference python/ray/experimental/dynamic_resources.py — dynamic custom resources are
deprecated there too; placement groups or start-time `resources` replace them."""


def set_resource(resource_name, capacity, node_id=None):
    raise DeprecationWarning(
        "Dynamic custom resources are deprecated. Use placement groups instead, or declare custom "
        "resources when the node starts (ray.init(resources=...), `rmm start --resources`).")
