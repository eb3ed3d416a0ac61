"""Configuration layer (reference nn/conf): builders, layer/vertex/preprocessor configs, JSON serde."""
from .activations import Activation, IActivation
from .base import Config
from .enums import (AlgoMode, BackpropType, CacheMode, ConvolutionMode, DataType, GradientNormalization,
                    OptimizationAlgorithm, PoolingType, Updater, WorkspaceMode)
from .graph import *  # noqa: F401,F403
from .inputs import InputType
from .layers import *  # noqa: F401,F403
from .losses import ILossFunction, LossFunction, LossFunctions
from .network import ComputationGraphConfiguration, MultiLayerConfiguration, NeuralNetConfiguration
from .preprocessors import *  # noqa: F401,F403
from .regularization import *  # noqa: F401,F403
from .updaters import *  # noqa: F401,F403
from .variational import *  # noqa: F401,F403
from .weights import *  # noqa: F401,F403
