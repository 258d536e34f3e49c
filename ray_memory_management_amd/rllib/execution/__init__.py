"""Execution building blocks: rollout sampling, learner groups, sample-batch GPU ingest.
Parity: reference rllib/execution/{rollout_ops,train_ops,multi_gpu_learner_thread}.py."""
from ray_memory_management_amd.rllib.execution.learner_group import LearnerActor, LearnerGroup  # noqa: F401
from ray_memory_management_amd.rllib.execution.sample_ingest import (SampleIngest, pack_fragment,  # noqa: F401
                                                                      split_for_learners)
from ray_memory_management_amd.rllib.execution.ops import (  # noqa: F401,E402
    ApplyGradients, AsyncGradients, AverageGradients, CollectMetrics, ComputeGradients, ConcatBatches, Concurrently,
    Dequeue, Enqueue, LearnerThread, MinibatchBuffer, MixInReplay, MultiGPULearnerThread, MultiGPUTrainOneStep,
    OncePerTimeInterval, OncePerTimestepsElapsed, ParallelRollouts, Replay, SelectExperiences, SimpleReplayBuffer,
    StandardizeFields, StandardMetricsReporting, StoreToReplayBuffer, TrainOneStep, UpdateTargetNetwork,
    synchronous_parallel_sample, train_one_step)
