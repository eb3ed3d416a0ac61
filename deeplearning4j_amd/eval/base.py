"""Shared evaluation plumbing: time-series/mask flattening (reference eval/BaseEvaluation.java evalTimeSeries),
JSON serde, merge, and EvaluationUtils (eval/EvaluationUtils.java)."""
import enum
import json
import math

import numpy as np
import torch


class EvaluationAveraging(enum.Enum):
    Macro = "Macro"
    Micro = "Micro"


class EvaluationUtils:
    @staticmethod
    def precision(tp, fp, edge=0.0):
        return edge if tp == 0 and fp == 0 else tp / float(tp + fp)

    @staticmethod
    def recall(tp, fn, edge=0.0):
        return edge if tp == 0 and fn == 0 else tp / float(tp + fn)

    @staticmethod
    def falsePositiveRate(fp, tn, edge=0.0):
        return edge if fp == 0 and tn == 0 else fp / float(fp + tn)

    @staticmethod
    def falseNegativeRate(fn, tp, edge=0.0):
        return edge if fn == 0 and tp == 0 else fn / float(fn + tp)

    @staticmethod
    def fBeta(beta, a, b, c=None):
        """fBeta(beta, precision, recall) or fBeta(beta, tp, fp, fn)."""
        if c is not None:
            tp, fp, fn = a, b, c
            p = EvaluationUtils.precision(tp, fp, -1)
            r = EvaluationUtils.recall(tp, fn, -1)
            if p == -1 or r == -1:
                return 0.0
            a, b = p, r
        p, r = a, b
        if p == 0.0 or r == 0.0:
            return 0.0
        nb = beta * beta
        return (1 + nb) * p * r / (nb * p + r)

    @staticmethod
    def gMeasure(p, r):
        return math.sqrt(p * r)

    @staticmethod
    def matthewsCorrelation(tp, fp, fn, tn):
        num = float(tp) * tn - float(fp) * fn
        den = math.sqrt(float(tp + fp) * (tp + fn) * (tn + fp) * (tn + fn))
        return num / den if den != 0 else 0.0


def to_2d(labels, preds, mask=None):
    """Flatten [mb, n, T] time series (reference BaseEvaluation.evalTimeSeries: permute to [mb*T, n], drop
    masked-out steps) and per-output masks [mb, n] (kept as a 2d mask)."""
    labels = torch.as_tensor(labels)
    preds = torch.as_tensor(preds)
    if labels.dim() == 3:
        n = labels.shape[1]
        l2 = labels.permute(0, 2, 1).reshape(-1, n)
        p2 = preds.permute(0, 2, 1).reshape(-1, n)
        if mask is not None:
            mk = torch.as_tensor(mask).to(l2.device)
            if mk.dim() == 3:                         # per-output time-series mask [mb, n, T]: a 2d per-output mask
                return l2, p2, mk.permute(0, 2, 1).reshape(-1, n)
            m = mk.reshape(-1) != 0
            l2, p2 = l2[m], p2[m]
        return l2, p2, None
    if labels.dim() == 4:   # CNN segmentation-style output: [mb, c, h, w] -> [mb*h*w, c]
        c = labels.shape[1]
        return (labels.permute(0, 2, 3, 1).reshape(-1, c), preds.permute(0, 2, 3, 1).reshape(-1, c), None)
    if mask is not None:
        mask = torch.as_tensor(mask).to(labels.device)
        if mask.dim() == 2 and mask.shape[1] == 1 and labels.shape[1] != 1:
            keep = mask.reshape(-1) != 0
            return labels[keep], preds[keep], None
        if mask.dim() == 1:
            keep = mask != 0
            return labels[keep], preds[keep], None
    return labels, preds, mask


def _enc(v):
    if hasattr(v, "to_state") and hasattr(type(v), "from_state"):      # per-label ROC accumulators
        return {"@roc": v.to_state()}
    if isinstance(v, np.ndarray):
        return {"@nd": v.tolist(), "dtype": str(v.dtype)}
    if torch.is_tensor(v):
        return {"@nd": v.cpu().numpy().tolist(), "dtype": str(v.cpu().numpy().dtype)}
    if isinstance(v, enum.Enum):
        return {"@enum": v.value}
    if isinstance(v, dict):
        return {"@map": [[_enc(k), _enc(x)] for k, x in v.items()]}
    if isinstance(v, (list, tuple)):
        return [_enc(x) for x in v]
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return {"@float": repr(v)}
    return v


def _dec(v):
    if isinstance(v, dict):
        if "@roc" in v:
            from .roc import _BinaryROCState
            return _BinaryROCState.from_state(v["@roc"])
        if "@nd" in v:
            return np.asarray(v["@nd"], dtype=v["dtype"])
        if "@map" in v:
            return {_dec(k) if not isinstance(k, list) else tuple(k): _dec(x) for k, x in v["@map"]}
        if "@float" in v:
            return float(v["@float"])
        if "@enum" in v:
            return v["@enum"]
    if isinstance(v, list):
        return [_dec(x) for x in v]
    return v


class BaseEvaluation:
    _REG = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        BaseEvaluation._REG[cls.__name__] = cls

    _TRANSIENT = ()

    def evalTimeSeries(self, labels, preds, mask=None):
        self.eval(labels, preds, mask)

    def eval(self, labels, predictions, mask=None):
        raise NotImplementedError

    def merge(self, other):
        raise NotImplementedError

    def reset(self):
        raise NotImplementedError

    def stats(self):
        raise NotImplementedError

    def __str__(self):
        return self.stats()

    # -------------------------------------------------------------------- serde (reference eval/serde)
    def toJson(self):
        d = {k: _enc(v) for k, v in self.__dict__.items() if k not in self._TRANSIENT and not k.startswith("_c")}
        return json.dumps({"@class": type(self).__name__, "fields": d})

    toYaml = toJson

    @classmethod
    def fromJson(cls, s):
        obj = json.loads(s)
        k = BaseEvaluation._REG[obj["@class"]]
        if "fields" not in obj and k.fromJson.__func__ is not BaseEvaluation.fromJson.__func__:
            return k.fromJson(s)                  # a class with its own JSON layout (ROC)
        inst = k.__new__(k)
        for f, v in obj["fields"].items():
            setattr(inst, f, _dec(v))
        if hasattr(inst, "_after_load"):
            inst._after_load()
        return inst

    def __eq__(self, other):
        return type(self) is type(other) and self.toJson() == other.toJson()
