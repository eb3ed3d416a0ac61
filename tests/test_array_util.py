"""ArrayUtil, after the reference's ArrayUtilTest (deeplearning4j-core/src/test/java/org/deeplearning4j/util/
ArrayUtilTest.java): ranges and C / Fortran strides. CPU."""
import torch

from deeplearning4j_amd.nd4j.array_util import ArrayUtil


def test_range():
    assert ArrayUtil.range(0, 2) == [0, 1]
    assert ArrayUtil.range(-1, 1) == [-1, 0]


def test_strides():
    assert ArrayUtil.calcStrides([5, 4, 3]) == [12, 3, 1]
    assert ArrayUtil.calcStridesFortran([5, 4, 3]) == [1, 5, 20]
    assert ArrayUtil.calcStrides([2, 2]) == [2, 1]
    assert ArrayUtil.calcStridesFortran([2, 2]) == [1, 2]
    assert ArrayUtil.calcStrides([5, 4, 3]) == list(torch.empty(5, 4, 3).stride())
    assert ArrayUtil.prod([5, 4, 3]) == 60
