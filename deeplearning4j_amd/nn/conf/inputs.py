"""InputType: shape inference across layers (reference nn/conf/inputs/InputType.java:43).

Activations are NCHW (CNN), [mb, size, T] (RNN, DL4J's NCW) and [mb, size] (FF), as in the reference.
"""
from .base import Config


class InputType(Config):
    def arrayElementsPerExample(self):
        raise NotImplementedError

    def getShape(self, mb=-1):
        raise NotImplementedError

    # factories ---------------------------------------------------------------------------------
    @staticmethod
    def feedForward(size):
        return InputTypeFeedForward(size=int(size))

    @staticmethod
    def recurrent(size, timeSeriesLength=-1):
        return InputTypeRecurrent(size=int(size), timeSeriesLength=int(timeSeriesLength))

    @staticmethod
    def convolutional(height, width, depth):
        return InputTypeConvolutional(height=int(height), width=int(width), channels=int(depth))

    @staticmethod
    def convolutionalFlat(height, width, depth):
        return InputTypeConvolutionalFlat(height=int(height), width=int(width), depth=int(depth))

    @staticmethod
    def convolutional3D(depth, height, width, channels):
        return InputTypeConvolutional3D(depth=int(depth), height=int(height), width=int(width),
                                        channels=int(channels))


class InputTypeFeedForward(InputType):
    FIELDS = {"size": 0}

    def arrayElementsPerExample(self):
        return self.size

    def getShape(self, mb=-1):
        return [mb, self.size]


class InputTypeRecurrent(InputType):
    FIELDS = {"size": 0, "timeSeriesLength": -1}

    def arrayElementsPerExample(self):
        return self.size * max(self.timeSeriesLength, 1)

    def getShape(self, mb=-1):
        return [mb, self.size, self.timeSeriesLength]


class InputTypeConvolutional(InputType):
    FIELDS = {"height": 0, "width": 0, "channels": 0}

    @property
    def depth(self):
        return self.channels

    def arrayElementsPerExample(self):
        return self.height * self.width * self.channels

    def getShape(self, mb=-1):
        return [mb, self.channels, self.height, self.width]


class InputTypeConvolutionalFlat(InputType):
    FIELDS = {"height": 0, "width": 0, "depth": 0}

    def getFlattenedSize(self):
        return self.height * self.width * self.depth

    def arrayElementsPerExample(self):
        return self.getFlattenedSize()

    def getUnflattenedType(self):
        return InputType.convolutional(self.height, self.width, self.depth)

    def getShape(self, mb=-1):
        return [mb, self.getFlattenedSize()]


class InputTypeConvolutional3D(InputType):
    FIELDS = {"depth": 0, "height": 0, "width": 0, "channels": 0}

    def arrayElementsPerExample(self):
        return self.depth * self.height * self.width * self.channels

    def getShape(self, mb=-1):
        return [mb, self.channels, self.depth, self.height, self.width]
