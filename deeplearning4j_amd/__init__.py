"""deeplearning4j_amd — an MI355X-native deep-learning framework with Deeplearning4j's capabilities.

Compute path: PyTorch-ROCm tensors as storage + hand-written HIP/CDNA4 kernels (gfx950) for the hot
ops + RCCL over xGMI for data parallelism. See SURVEY.md for the component map.
"""
__version__ = "0.1.0"

from .datasets import *  # noqa: F401,F403
from .exceptions import (DL4JException, DL4JInvalidConfigException, DL4JInvalidInputException,  # noqa: F401
                         InvalidInputTypeException)
from .nn.conf import *  # noqa: F401,F403
from .nn.graph import ComputationGraph
from .nn.multilayer import MultiLayerNetwork
from .nn.transferlearning import FineTuneConfiguration, TransferLearning, TransferLearningHelper  # noqa: F401
from .nn.simple import RankClassificationResult  # noqa: F401
from .utils.misc_util import FeatureUtil, SerializationUtils  # noqa: F401
from .eval import (Evaluation, EvaluationBinary, EvaluationCalibration, RegressionEvaluation,  # noqa: F401
                   ROC, ROCBinary, ROCMultiClass)
