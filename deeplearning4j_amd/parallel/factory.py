"""Trainer factories for ParallelWrapper (reference deeplearning4j-scaleout-parallelwrapper
``parallelism/factory/TrainerContext.java:14-54``, ``DefaultTrainerContext.java``, ``SymmetricTrainerContext.java`` and
deeplearning4j-scaleout-parallelwrapper-parameter-server ``ParameterServerTrainerContext.java:20-84`` /
``ParameterServerTrainer.java:32-67``).

In the reference a TrainerContext creates one Trainer thread per device inside one JVM. Here each ``torch.distributed``
rank (one process per GPU) is one trainer. The context decides what happens around every local fit:

* ``DefaultTrainerContext``: local fits. Every ``averagingFrequency`` rounds the parameters (and optionally the updater
  state) are averaged with one RCCL all-reduce each (AVERAGING mode).
* ``SymmetricTrainerContext``: symmetric gradient sharing. Every step's gradient is all-reduced (bucketed, overlapped with
  backward) before the local update, so replicas never diverge (SHARED_GRADIENTS mode).
* ``ParameterServerTrainerContext``: after each fit every trainer pushes its parameters to the server (rank 0), which
  averages them and publishes the result back. This is the Aeron parameter server's push/pull done as an RCCL reduce
  to rank 0 plus a broadcast. It is kept for API parity; on one node the symmetric context moves fewer bytes.
"""
import uuid as _uuid

import torch
import torch.distributed as dist

from .accumulation import AllReduceGradientsAccumulator, average_params_and_state
from .distributed import is_dist, rank, world_size


class Trainer:
    """One replica's training loop step (reference ``parallelism/trainer/Trainer.java``)."""

    def __init__(self, model, threadId=0, uuid=None, context=None):
        self.model, self.threadId, self.uuid, self.context = model, threadId, uuid or str(_uuid.uuid4()), context
        self.iterations = 0

    def feedDataSet(self, ds, etl_ms=0):
        from ..datasets.dataset import MultiDataSet
        m = self.model
        if isinstance(ds, MultiDataSet):
            m._fit_batch(ds.features, ds.labels, ds.featuresMasks, ds.labelsMasks)
        elif type(m).__name__ == "ComputationGraph":
            m._fit_batch([ds.features], [ds.labels], None if ds.featuresMask is None else [ds.featuresMask],
                         None if ds.labelsMask is None else [ds.labelsMask])
        else:
            m._fit_batch(ds.features, ds.labels, ds.featuresMask, ds.labelsMask)
        self.iterations += 1

    feedMultiDataSet = feedDataSet

    def getModel(self):
        return self.model

    def updateModel(self, model):
        with torch.no_grad():
            self.model.flattenedParams.copy_(model.flattenedParams)
        self.model.sync_shadow()


class TrainerContext:
    """Interface: init / create / finalizeRound / finalizeTraining."""

    def init(self, model, *args):
        pass

    def create(self, uuid, threadId, model, rootDevice=0, useMDS=False, wrapper=None, mode=None,
               averagingFrequency=1):
        return Trainer(model, threadId, uuid, self)

    def finalizeRound(self, originalModel, *models):
        pass

    def finalizeTraining(self, originalModel, *models):
        pass


class DefaultTrainerContext(TrainerContext):
    def __init__(self, averageUpdaters=True):
        self.averageUpdaters = averageUpdaters

    def finalizeRound(self, originalModel, *models):
        average_params_and_state(originalModel, self.averageUpdaters)

    def finalizeTraining(self, originalModel, *models):
        self.finalizeRound(originalModel, *models)


class SymmetricTrainerContext(TrainerContext):
    def __init__(self, bucket_mb=None):
        self.bucket_mb = bucket_mb

    def init(self, model, *args):
        if is_dist() and getattr(model, "gradientsAccumulator", None) is None:
            model.setGradientsAccumulator(AllReduceGradientsAccumulator(self.bucket_mb))


class ParameterServerTrainerContext(TrainerContext):
    """Parameter server on rank 0: every trainer pushes its parameters after each fit; the server averages them and
    every trainer pulls the average (reference ParameterServerTrainer.java:36-67 push after fit)."""

    def __init__(self, server_rank=0):
        self.server_rank = server_rank
        self.pushes = 0

    def create(self, uuid, threadId, model, rootDevice=0, useMDS=False, wrapper=None, mode=None,
               averagingFrequency=1):
        return _PSTrainer(model, threadId, uuid, self)

    def push_pull(self, model):
        self.pushes += 1
        if not is_dist():
            return
        p = model.flattenedParams
        dist.reduce(p, dst=self.server_rank, op=dist.ReduceOp.SUM)          # push
        if rank() == self.server_rank:
            p.div_(world_size())                                             # server-side average
        dist.broadcast(p, src=self.server_rank)                              # pull
        model.sync_shadow()

    def finalizeTraining(self, originalModel, *models):
        if is_dist():
            dist.broadcast(originalModel.flattenedParams, src=self.server_rank)
            originalModel.sync_shadow()


class _PSTrainer(Trainer):
    def feedDataSet(self, ds, etl_ms=0):
        super().feedDataSet(ds, etl_ms)
        self.context.push_pull(self.model)

    feedMultiDataSet = feedDataSet
