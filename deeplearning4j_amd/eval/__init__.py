"""Evaluation metrics (reference deeplearning4j-nn/src/main/java/org/deeplearning4j/eval/*).

All accumulators reduce each minibatch ON the device that produced the predictions (argmax, bincount, sums)
and only pull small count tables to the host, so evaluating on the GPU costs one small D2H copy per batch.
"""
from .base import BaseEvaluation, EvaluationAveraging, EvaluationUtils
from .binary import EvaluationBinary
from .calibration import EvaluationCalibration
from .confusion import ConfusionMatrix
from .curves import Histogram, PrecisionRecallCurve, ReliabilityDiagram, RocCurve
from .evaluation import Evaluation, Prediction
from .regression import RegressionEvaluation
from .roc import ROC, ROCBinary, ROCMultiClass

__all__ = ["BaseEvaluation", "EvaluationAveraging", "EvaluationUtils", "Evaluation", "EvaluationBinary",
           "EvaluationCalibration", "ConfusionMatrix", "RegressionEvaluation", "ROC", "ROCBinary", "ROCMultiClass",
           "RocCurve", "PrecisionRecallCurve", "Histogram", "ReliabilityDiagram", "Prediction"]
from .tools import EvaluationTools  # noqa: F401
