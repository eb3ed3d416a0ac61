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
    def inferInputType(arr):
        """The InputType of one activation array (reference InputType.inferInputType): [mb, n] feed-forward,
        [mb, n, T] recurrent, [mb, c, h, w] convolutional."""
        shp = tuple(arr.shape)
        if len(shp) == 2:
            return InputType.feedForward(shp[1])
        if len(shp) == 3:
            return InputType.recurrent(shp[1], shp[2])
        if len(shp) == 4:
            return InputType.convolutional(shp[2], shp[3], shp[1])
        if len(shp) == 5:
            return InputType.convolutional3D(shp[2], shp[3], shp[4], shp[1])
        raise ValueError(f"cannot infer an InputType for an array of rank {len(shp)}")

    @staticmethod
    def inferInputTypes(arrays):
        return [InputType.inferInputType(a) for a in arrays]

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
