"""Data parallelism over torch.distributed (RCCL over xGMI on MI355X; gloo for CPU tests) and parallel
inference. See SURVEY §2.6 for the mapping from the reference's ParallelWrapper / gradient sharing."""
from .accumulation import AllReduceGradientsAccumulator, average_params_and_state
from .distributed import barrier, destroy, init_distributed, is_dist, rank, world_size
from .encoded import EncodedGradientsAccumulator, EncodingHandler
from .factory import (DefaultTrainerContext, ParameterServerTrainerContext, SymmetricTrainerContext,  # noqa: F401
                      Trainer, TrainerContext)
from .inference import InferenceMode, ParallelInference
from .wrapper import ParallelWrapper, TrainingMode
from .cluster import (ParameterAveragingTrainingMaster, SharedTrainingMaster, SparkComputationGraph,  # noqa: F401
                      SparkDl4jMultiLayer, StatsUtils, TrainingMaster, TrainingStats)
from .basic import BasicGradientsAccumulator, FancyBlockingQueue, LocalHandler  # noqa: E402,F401

from .concurrency import AsyncIterator, MultiBoolean  # noqa: F401,E402
