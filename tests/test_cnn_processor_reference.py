"""FeedForwardToCnnPreProcessor / CnnToFeedForwardPreProcessor, after the reference's CNNProcessorTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/preprocessor/CNNProcessorTest.java:32-287): 2-D <-> 4-D
reshapes keep already-shaped inputs, the flattened vector is depth 0's rows then depth 1's (c order) for 'c' and
'f' ordered inputs alike, backprop inverts the forward exactly, and a strict-mode CNN built for 20 x 10 inputs rejects
a 10 x 20 input (IllegalStateException from the preprocessor: both flatten to 96 values). CPU."""
import itertools

import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.exceptions import IllegalStateException

ROWS, COLS = 28, 28


def _f_order(t):
    """Same values as ``t`` in a column-major ('f') layout."""
    return t.permute(*reversed(range(t.dim()))).contiguous().permute(*reversed(range(t.dim())))


def test_feed_forward_to_cnn_preprocessor():
    p = D.FeedForwardToCnnPreProcessor(ROWS, COLS, 1)
    out = p.preProcess(torch.zeros(1, 784), -1)
    assert out.dim() == 4 and torch.equal(out, torch.zeros(1, 1, 28, 28))
    out = p.preProcess(torch.zeros(20, 1, 28, 28), -1)
    assert out.dim() == 4 and torch.equal(out, torch.zeros(20, 1, 28, 28))


@pytest.mark.parametrize("rows,cols,d", list(itertools.product([1, 5, 20], [1, 5, 20], [1, 3])))
def test_feed_forward_to_cnn_preprocessor_values(rows, cols, d):
    p = D.FeedForwardToCnnPreProcessor(rows, cols, d)
    for mb in (1, 5):
        rand = torch.rand(mb, rows * cols * d, dtype=torch.float64)
        ff_c, ff_f = rand.clone(), _f_order(rand)
        act_c, act_f = p.preProcess(ff_c, -1), p.preProcess(ff_f, -1)
        assert tuple(act_c.shape) == (mb, d, rows, cols) == tuple(act_f.shape)
        assert torch.equal(act_c, act_f)
        # vector position depth * rows * cols + r * cols + c
        assert torch.equal(act_c, ff_c.reshape(mb, d, rows, cols))
        eps_c, eps_f = act_c.clone(), _f_order(act_f)
        assert torch.equal(p.backprop(eps_c, -1), ff_c)
        assert torch.equal(p.backprop(eps_f, -1), ff_c)


def test_feed_forward_to_cnn_preprocessor_backprop_keeps_2d():
    p = D.FeedForwardToCnnPreProcessor(ROWS, COLS, 1)
    p.preProcess(torch.zeros(1, 784), -1)
    out = p.backprop(torch.zeros(1, 784), -1)
    assert out.dim() == 2 and torch.equal(out, torch.zeros(1, 784))


def test_cnn_to_feed_forward_processor_backprop_shapes():
    p = D.CnnToFeedForwardPreProcessor(ROWS, COLS, 1)
    out = p.backprop(torch.zeros(1, 784), -1)
    assert out.dim() == 4 and torch.equal(out, torch.zeros(1, 1, 28, 28))
    out = p.backprop(torch.zeros(20, 1, 28, 28), -1)
    assert out.dim() == 4 and torch.equal(out, torch.zeros(20, 1, 28, 28))


def test_cnn_to_feed_forward_preprocessor_keeps_2d():
    p = D.CnnToFeedForwardPreProcessor(ROWS, COLS, 1)
    p.preProcess(torch.zeros(20, 1, 28, 28), -1)
    out = p.preProcess(torch.zeros(1, 784), -1)
    assert out.dim() == 2 and torch.equal(out, torch.zeros(1, 784))
    out = p.preProcess(torch.zeros(20, 1, 28, 28), -1)
    assert out.dim() == 2 and torch.equal(out, torch.zeros(20, 784))


@pytest.mark.parametrize("rows,cols,d", list(itertools.product([1, 5, 20], [1, 5, 20], [1, 3])))
def test_cnn_to_feed_forward_preprocessor_values(rows, cols, d):
    p = D.CnnToFeedForwardPreProcessor(rows, cols, d)
    for mb in (1, 5):
        rand = torch.rand(mb, d, rows, cols, dtype=torch.float64)
        conv_c, conv_f = rand.clone(), _f_order(rand)
        ff_c, ff_f = p.preProcess(conv_c, -1), p.preProcess(conv_f, -1)
        assert tuple(ff_c.shape) == (mb, d * rows * cols) == tuple(ff_f.shape)
        assert torch.equal(ff_c, ff_f)
        assert torch.equal(ff_c, conv_c.reshape(mb, -1))
        eps_c, eps_f = ff_c.clone(), _f_order(ff_c)
        assert torch.equal(p.backprop(eps_c, -1), conv_c)
        assert torch.equal(p.backprop(eps_f, -1), conv_c)


def test_invalid_input_shape():
    b = (D.NeuralNetConfiguration.Builder().seed(123).miniBatch(True).cacheMode(D.CacheMode.DEVICE)
         .updater(D.Nesterovs(0.9)).gradientNormalization(D.GradientNormalization.RenormalizeL2PerLayer)
         .optimizationAlgo(D.OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT))
    lb = b.list()
    for i in range(4):
        cb = D.ConvolutionLayer.Builder([3, 3], [1, 1], [0, 0]).name(f"cnn{i + 1}") \
            .convolutionMode(D.ConvolutionMode.Strict).nOut(4).weightInit(D.WeightInit.XAVIER_UNIFORM) \
            .activation(D.Activation.RELU)
        if i == 0:
            cb = cb.nIn(2)
        if i < 2:
            cb = cb.biasInit(1e-2)
        lb = lb.layer(i, cb.build())
    lb = lb.layer(4, D.OutputLayer.Builder(D.LossFunction.MSE).name("output").nOut(1)
                  .activation(D.Activation.TANH).build())
    conf = lb.setInputType(D.InputType.convolutional(20, 10, 2)).build()
    net = D.MultiLayerNetwork(conf)
    net.init()
    net.output(torch.zeros(1, 2, 20, 10))                               # valid
    with pytest.raises(IllegalStateException):
        net.output(torch.zeros(1, 2, 10, 20))
