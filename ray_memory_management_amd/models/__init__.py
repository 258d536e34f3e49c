"""Model zoo used by the libraries and benchmarks.

* ``resnet18/34/50/101/152`` — Train / AIR benchmark models (``models/resnet.py``)
* ``VisionNetwork`` / ``FullyConnectedNetwork`` — RLlib policy models (``rllib/models.py``:
  Nature-CNN Atari filters with the fused HIP bias/ReLU epilogues, and the FC net)
"""
from ray_memory_management_amd.models.resnet import (ResNet, resnet18, resnet34, resnet50, resnet101,  # noqa: F401
                                                     resnet152)


def __getattr__(name):
    if name in ("VisionNetwork", "FullyConnectedNetwork"):
        from ray_memory_management_amd.rllib import models as _m

        return getattr(_m, name)
    raise AttributeError(name)
