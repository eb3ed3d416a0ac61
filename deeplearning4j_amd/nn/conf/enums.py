"""Configuration enums mirroring the reference's `nn/conf` enums.

Reference: deeplearning4j-nn/src/main/java/org/deeplearning4j/nn/conf/
  ConvolutionMode.java:61-63, GradientNormalization.java, WorkspaceMode.java,
  CacheMode.java, BackpropType.java, Updater.java, layers/PoolingType.java,
  api/OptimizationAlgorithm.java.
"""
from enum import Enum


class _StrEnum(str, Enum):
    def __str__(self):
        return self.value

    @classmethod
    def of(cls, v):
        if isinstance(v, cls) or v is None:
            return v
        if isinstance(v, str):
            for m in cls:
                if m.value.lower() == v.lower() or m.name.lower() == v.lower():
                    return m
        raise ValueError(f"{v!r} is not a valid {cls.__name__}")


class ConvolutionMode(_StrEnum):
    """Strict: (in - k + 2p) must divide stride exactly; Truncate: floor; Same: ceil(in/stride) with
    top/left padding computed automatically (reference ConvolutionMode.java:4-63)."""
    Strict = "Strict"
    Truncate = "Truncate"
    Same = "Same"


class GradientNormalization(_StrEnum):
    None_ = "None"
    RenormalizeL2PerLayer = "RenormalizeL2PerLayer"
    RenormalizeL2PerParamType = "RenormalizeL2PerParamType"
    ClipElementWiseAbsoluteValue = "ClipElementWiseAbsoluteValue"
    ClipL2PerLayer = "ClipL2PerLayer"
    ClipL2PerParamType = "ClipL2PerParamType"


class WorkspaceMode(_StrEnum):
    NONE = "NONE"
    SINGLE = "SINGLE"
    SEPARATE = "SEPARATE"
    ENABLED = "ENABLED"


class CacheMode(_StrEnum):
    NONE = "NONE"
    HOST = "HOST"
    DEVICE = "DEVICE"


class BackpropType(_StrEnum):
    Standard = "Standard"
    TruncatedBPTT = "TruncatedBPTT"


class OptimizationAlgorithm(_StrEnum):
    STOCHASTIC_GRADIENT_DESCENT = "STOCHASTIC_GRADIENT_DESCENT"
    LINE_GRADIENT_DESCENT = "LINE_GRADIENT_DESCENT"
    CONJUGATE_GRADIENT = "CONJUGATE_GRADIENT"
    HESSIAN_FREE = "HESSIAN_FREE"          # deprecated in the reference; configurable, refused at fit time
    LBFGS = "LBFGS"


class PoolingType(_StrEnum):
    MAX = "MAX"
    AVG = "AVG"
    SUM = "SUM"
    PNORM = "PNORM"


class AlgoMode(_StrEnum):
    """cuDNN algo-mode knob kept for config compatibility; the HIP helpers pick their own tiles."""
    NO_WORKSPACE = "NO_WORKSPACE"
    PREFER_FASTEST = "PREFER_FASTEST"
    USER_SPECIFIED = "USER_SPECIFIED"


class DataType(_StrEnum):
    """Compute dtype policy. Parameters / updater state are always kept in fp32 (fp64 for DOUBLE);
    BFLOAT16/HALF run activations and matmuls in reduced precision with fp32 accumulation."""
    DOUBLE = "DOUBLE"
    FLOAT = "FLOAT"
    HALF = "HALF"
    BFLOAT16 = "BFLOAT16"

    def torch_dtype(self):
        import torch
        return {DataType.DOUBLE: torch.float64, DataType.FLOAT: torch.float32,
                DataType.HALF: torch.float16, DataType.BFLOAT16: torch.bfloat16}[self]

    def master_dtype(self):
        import torch
        return torch.float64 if self is DataType.DOUBLE else torch.float32


class Updater(_StrEnum):
    """Legacy updater enum (reference nn/conf/Updater.java) → IUpdater with default hyperparameters."""
    SGD = "SGD"
    ADAM = "ADAM"
    ADAMAX = "ADAMAX"
    ADADELTA = "ADADELTA"
    NESTEROVS = "NESTEROVS"
    NADAM = "NADAM"
    ADAGRAD = "ADAGRAD"
    RMSPROP = "RMSPROP"
    NONE = "NONE"
    CUSTOM = "CUSTOM"

    def getIUpdaterWithDefaultConfig(self):
        from . import updaters as u
        return {Updater.SGD: u.Sgd, Updater.ADAM: u.Adam, Updater.ADAMAX: u.AdaMax,
                Updater.ADADELTA: u.AdaDelta, Updater.NESTEROVS: u.Nesterovs, Updater.NADAM: u.Nadam,
                Updater.ADAGRAD: u.AdaGrad, Updater.RMSPROP: u.RmsProp, Updater.NONE: u.NoOp}[self]()


def _register_all():
    from .base import register_enum
    for e in (ConvolutionMode, GradientNormalization, WorkspaceMode, CacheMode, BackpropType,
              OptimizationAlgorithm, PoolingType, AlgoMode, DataType, Updater):
        register_enum(e)


_register_all()
