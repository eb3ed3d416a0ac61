"""ArrayUtil: the shape / stride helpers the reference uses from ND4J (org.nd4j.linalg.util.ArrayUtil, exercised by
deeplearning4j-core/src/test/java/org/deeplearning4j/util/ArrayUtilTest.java)."""
import math


class ArrayUtil:
    @staticmethod
    def range(begin, end):
        """[begin, end) as a list of ints."""
        return list(range(int(begin), int(end)))

    @staticmethod
    def calcStrides(shape, startValue=1):
        """C-order (row-major) strides, in elements."""
        out, acc = [0] * len(shape), startValue
        for i in range(len(shape) - 1, -1, -1):
            out[i] = acc
            acc *= int(shape[i])
        return out

    @staticmethod
    def calcStridesFortran(shape, startValue=1):
        """Fortran-order (column-major) strides, in elements."""
        out, acc = [0] * len(shape), startValue
        for i in range(len(shape)):
            out[i] = acc
            acc *= int(shape[i])
        return out

    @staticmethod
    def prod(shape):
        return int(math.prod(int(s) for s in shape))
