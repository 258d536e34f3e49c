"""Data-parallel building blocks over ``torch.distributed`` (RCCL over xGMI on MI355X, gloo on CPU):
bucketed gradient all-reduce overlapped with backward and coalesced all-reduce. Used by
``train.torch.prepare_model(parallel_strategy="bucketed")`` and available to custom learners."""
from ray_memory_management_amd.parallel.ddp import (BucketedAllReduce, all_reduce_coalesced,  # noqa: F401
                                                    default_bucket_cap_mb)
