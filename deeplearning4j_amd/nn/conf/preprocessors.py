"""Input preprocessors (reference nn/conf/preprocessor/*): config + runtime in one object.

RNN <-> FF reshapes use the reference's time-major row order: row ``t*mb + m`` holds example m at
time t (RnnToFeedForwardPreProcessor permutes to [mb,T,size] and reshapes in 'f' order).
"""
import torch

from .base import Config
from .inputs import InputType, InputTypeConvolutional, InputTypeFeedForward, InputTypeRecurrent


class InputPreProcessor(Config):
    def __init__(self, *args, **kw):
        # the reference's positional constructors, e.g. CnnToFeedForwardPreProcessor(inputHeight, inputWidth,
        # numChannels): positional arguments fill the fields in declaration order
        names = tuple(type(self)._all_fields())
        if len(args) > len(names):
            raise TypeError(f"{type(self).__name__} takes at most {len(names)} positional arguments")
        for n, a in zip(names, args):
            if n in kw:
                raise TypeError(f"{type(self).__name__}: {n} given twice")
            kw[n] = a
        super().__init__(**kw)

    def preProcess(self, x, miniBatchSize, training=False):
        raise NotImplementedError

    def backprop(self, eps, miniBatchSize):
        raise NotImplementedError

    def getOutputType(self, inputType):
        return inputType

    def feedForwardMaskArray(self, mask, currentMaskState, miniBatchSize):
        return mask, currentMaskState


class CnnToFeedForwardPreProcessor(InputPreProcessor):
    FIELDS = {"inputHeight": 0, "inputWidth": 0, "numChannels": 0}

    def preProcess(self, x, miniBatchSize, training=False):
        if x.dim() == 2:
            return x
        exp = (self.numChannels, self.inputHeight, self.inputWidth)
        if x.dim() == 4 and all(v > 0 for v in exp) and tuple(x.shape[1:]) != tuple(exp):
            # the flattened size can agree while the layout does not (reference CnnToFeedForwardPreProcessor:84-89)
            from ...exceptions import IllegalStateException
            raise IllegalStateException(
                f"Invalid input array: expected shape [minibatch, channels, height, width] = [minibatch, {exp[0]}, "
                f"{exp[1]}, {exp[2]}] - got {list(x.shape)}")
        self._shape = x.shape
        if x.is_cuda and not x.is_contiguous():
            # NCHW flatten order (the reference's c-order reshape) of a channels-last activation: one in-tree copy
            from ...ops import nd4j_kernels as NK
            y = NK.materialize(x)
            if y is not None:
                return y.reshape(x.shape[0], -1)
        return x.reshape(x.shape[0], -1)

    def backprop(self, eps, miniBatchSize):
        if eps.dim() == 4:
            return eps
        shp = getattr(self, "_shape", None)
        if shp is None:
            shp = (eps.shape[0], self.numChannels, self.inputHeight, self.inputWidth)
        return eps.reshape(shp)

    def getOutputType(self, inputType):
        if isinstance(inputType, InputTypeConvolutional):
            return InputType.feedForward(inputType.channels * inputType.height * inputType.width)
        return inputType


class FeedForwardToCnnPreProcessor(InputPreProcessor):
    FIELDS = {"inputHeight": 0, "inputWidth": 0, "numChannels": 1}

    def preProcess(self, x, miniBatchSize, training=False):
        if x.dim() == 4:
            return x
        return x.reshape(x.shape[0], self.numChannels, self.inputHeight, self.inputWidth)

    def backprop(self, eps, miniBatchSize):
        return eps.reshape(eps.shape[0], -1)

    def getOutputType(self, inputType):
        return InputType.convolutional(self.inputHeight, self.inputWidth, self.numChannels)


class RnnToFeedForwardPreProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        if x.dim() == 2:
            return x
        mb, size, T = x.shape
        self._shape = (mb, size, T)
        return x.permute(2, 0, 1).reshape(T * mb, size)

    def backprop(self, eps, miniBatchSize):
        if eps.dim() == 3:
            return eps
        mb, size, T = self._shape if hasattr(self, "_shape") else (miniBatchSize, eps.shape[1],
                                                                     eps.shape[0] // miniBatchSize)
        return eps.reshape(T, mb, eps.shape[1]).permute(1, 2, 0)

    def getOutputType(self, inputType):
        return InputType.feedForward(inputType.size) if isinstance(inputType, InputTypeRecurrent) else inputType

    def feedForwardMaskArray(self, mask, currentMaskState, miniBatchSize):
        if mask is None or mask.dim() != 2:
            return mask, currentMaskState
        return mask.t().reshape(-1, 1), currentMaskState


class FeedForwardToRnnPreProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        if x.dim() == 3:
            return x
        n, size = x.shape
        T = n // miniBatchSize
        return x.reshape(T, miniBatchSize, size).permute(1, 2, 0)

    def backprop(self, eps, miniBatchSize):
        mb, size, T = eps.shape
        return eps.permute(2, 0, 1).reshape(T * mb, size)

    def feedForwardMaskArray(self, mask, currentMaskState, miniBatchSize):
        """[T*mb, 1] per-row mask (time-major, as RnnToFeedForward produced it) back to [mb, T]."""
        if mask is None or mask.dim() != 2 or mask.shape[1] != 1 or mask.shape[0] == miniBatchSize:
            return mask, currentMaskState
        return mask.reshape(-1, miniBatchSize).t(), currentMaskState

    def getOutputType(self, inputType):
        if isinstance(inputType, InputTypeFeedForward):
            return InputType.recurrent(inputType.size)
        return inputType


class CnnToRnnPreProcessor(InputPreProcessor):
    """[mb*T, c, h, w] -> [mb, c*h*w, T] (time-major rows)."""
    FIELDS = {"inputHeight": 0, "inputWidth": 0, "numChannels": 0}

    def preProcess(self, x, miniBatchSize, training=False):
        n = x.shape[0]
        T = n // miniBatchSize
        f = x.reshape(n, -1)
        return f.reshape(T, miniBatchSize, -1).permute(1, 2, 0)

    def backprop(self, eps, miniBatchSize):
        mb, size, T = eps.shape
        return eps.permute(2, 0, 1).reshape(T * mb, self.numChannels, self.inputHeight, self.inputWidth)

    def getOutputType(self, inputType):
        return InputType.recurrent(self.numChannels * self.inputHeight * self.inputWidth)


class RnnToCnnPreProcessor(InputPreProcessor):
    FIELDS = {"inputHeight": 0, "inputWidth": 0, "numChannels": 0}

    def preProcess(self, x, miniBatchSize, training=False):
        mb, size, T = x.shape
        return x.permute(2, 0, 1).reshape(T * mb, self.numChannels, self.inputHeight, self.inputWidth)

    def backprop(self, eps, miniBatchSize):
        n = eps.shape[0]
        T = n // miniBatchSize
        return eps.reshape(T, miniBatchSize, -1).permute(1, 2, 0)

    def getOutputType(self, inputType):
        return InputType.convolutional(self.inputHeight, self.inputWidth, self.numChannels)


class ComposableInputPreProcessor(InputPreProcessor):
    FIELDS = {"inputPreProcessors": []}

    def __init__(self, *pps, **kw):
        if pps:
            kw["inputPreProcessors"] = list(pps)
        super().__init__(**kw)

    def preProcess(self, x, miniBatchSize, training=False):
        for p in self.inputPreProcessors:
            x = p.preProcess(x, miniBatchSize, training)
        return x

    def backprop(self, eps, miniBatchSize):
        for p in reversed(self.inputPreProcessors):
            eps = p.backprop(eps, miniBatchSize)
        return eps

    def getOutputType(self, inputType):
        for p in self.inputPreProcessors:
            inputType = p.getOutputType(inputType)
        return inputType


class ZeroMeanPrePreProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        return x - x.mean(dim=0, keepdim=True)

    def backprop(self, eps, miniBatchSize):
        return eps


class UnitVarianceProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        self._std = x.std(dim=0, keepdim=True) + 1e-8
        return x / self._std

    def backprop(self, eps, miniBatchSize):
        return eps / self._std


class ZeroMeanAndUnitVariancePreProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        self._std = x.std(dim=0, keepdim=True) + 1e-8
        return (x - x.mean(dim=0, keepdim=True)) / self._std

    def backprop(self, eps, miniBatchSize):
        return eps / self._std


class BinomialSamplingPreProcessor(InputPreProcessor):
    def preProcess(self, x, miniBatchSize, training=False):
        return torch.bernoulli(torch.clamp(x.float(), 0, 1)).to(x.dtype)

    def backprop(self, eps, miniBatchSize):
        return eps
