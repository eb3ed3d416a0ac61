"""Convolutional ComputationGraphs, after the reference's TestCompGraphCNN
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/graph/TestCompGraphCNN.java:40-290): two convolutions of one
input merged (by the automatically inserted MergeVertex) into a max pool, topological order as vertex indices,
parameter count and setParams round trip, forward activations per vertex, gradient and score; a kernel larger than its
input fails at build time with InvalidInputTypeException; a single-feature-map convolution and an LRN + BN stack
build and train. CPU."""
import pytest
import torch

import deeplearning4j_amd as D


def _multi_input_conf():
    return (D.NeuralNetConfiguration.Builder().graphBuilder().addInputs("input")
            .setInputTypes(D.InputType.convolutional(32, 32, 3))
            .addLayer("cnn1", D.ConvolutionLayer.Builder(4, 4).stride(2, 2).nIn(3).nOut(3).build(), "input")
            .addLayer("cnn2", D.ConvolutionLayer.Builder(4, 4).stride(2, 2).nIn(3).nOut(3).build(), "input")
            .addLayer("max1", D.SubsamplingLayer.Builder(D.PoolingType.MAX).stride(1, 1).kernelSize(2, 2).build(),
                      "cnn1", "cnn2")
            .addLayer("dnn1", D.DenseLayer.Builder().nOut(7).build(), "max1")
            .addLayer("output", D.OutputLayer.Builder().nIn(7).nOut(10).build(), "dnn1")
            .setOutputs("output").build())


N_PARAMS = 2 * (3 * 1 * 4 * 4 * 3 + 3) + (7 * 14 * 14 * 6 + 7) + (7 * 10 + 10)


@pytest.fixture
def graph():
    g = D.ComputationGraph(_multi_input_conf())
    g.init()
    return g


def _ds():
    f = torch.zeros(5, 3, 32, 32)
    lab = torch.eye(10)[:5]
    return f, lab


def test_config_basic(graph):
    # input 0, cnn1 1, cnn2 2, max1 3, max1-merge 4 (added right after max1), dnn1 5, output 6
    assert graph.topologicalSortOrder() in ([0, 1, 2, 4, 3, 5, 6], [0, 2, 1, 4, 3, 5, 6])
    p = graph.params()
    assert p.numel() == N_PARAMS
    arr = torch.linspace(0, N_PARAMS, N_PARAMS, dtype=p.dtype)
    graph.setParams(arr)
    assert torch.equal(graph.params().reshape(-1), arr)
    assert graph.getNumInputArrays() == 1 and graph.getNumOutputArrays() == 1


def test_forward_basic(graph):
    f, _ = _ds()
    graph.setInput(0, f)
    acts = graph.feedForward(True)
    for k in ("input", "cnn1", "cnn2", "max1", "dnn1", "output"):
        assert k in acts, k
    assert tuple(acts["cnn1"].shape) == (5, 3, 15, 15)
    assert tuple(acts["max1"].shape) == (5, 6, 14, 14)
    assert tuple(acts["output"].shape) == (5, 10)


def test_backward_basic(graph):
    f, lab = _ds()
    graph.setInput(0, f.clone())
    graph.setLabel(0, lab.clone())
    graph.computeGradientAndScore()
    g, score = graph.gradientAndScore()
    assert torch.isfinite(torch.tensor(float(score)))
    gv = g.gradientForVariable()
    assert sum(v.numel() for v in gv.values()) == N_PARAMS
    assert tuple(gv["cnn1_W"].shape) == (3, 3, 4, 4)


def _small_cnn(input_type, kh, kw, n_out, pool_kh):
    return (D.NeuralNetConfiguration.Builder().seed(123).graphBuilder().addInputs("input")
            .setInputTypes(input_type)
            .addLayer("conv1", D.ConvolutionLayer.Builder().kernelSize(kh, kw).stride(1, 1).nIn(1).nOut(n_out)
                      .weightInit(D.WeightInit.XAVIER).activation(D.Activation.RELU).build(), "input")
            .addLayer("pool1", D.SubsamplingLayer.Builder().poolingType(D.PoolingType.MAX).kernelSize(pool_kh, 1)
                      .stride(1, 1).build(), "conv1")
            .addLayer("output", D.OutputLayer.Builder().nOut(2).build(), "pool1")
            .setOutputs("output").build())


def test_kernel_too_large_is_an_invalid_input_type():
    # InputType.convolutional(height=1, width=23, channels=19): a 3 x 23 kernel does not fit a height-1 input
    with pytest.raises(D.InvalidInputTypeException):
        _small_cnn(D.InputType.convolutional(1, 23, 19), 3, 23, 2, 17)


def test_single_output_feature_map_trains():
    conf = _small_cnn(D.InputType.convolutional(23, 23, 1), 3, 3, 1, 20)
    g = D.ComputationGraph(conf)
    g.init()
    x = torch.zeros(200, 1, 23, 23)
    y = torch.zeros(200, 2)
    g.fit(D.DataSet(x, y))
    assert tuple(g.output(x[:4])[0].shape) == (4, 2)


def test_cnn_lrn_bn_builds():
    conf = (D.NeuralNetConfiguration.Builder().seed(123).graphBuilder().addInputs("input")
            .setInputTypes(D.InputType.convolutional(40, 40, 1))
            .addLayer("cnn1", D.ConvolutionLayer.Builder([2, 2], [1, 1], [0, 0]).nIn(1).nOut(64).biasInit(0.2)
                      .build(), "input")
            .addLayer("max1", D.SubsamplingLayer.Builder(D.PoolingType.MAX, [2, 2], [1, 1]).build(), "cnn1")
            .addLayer("lrn1", D.LocalResponseNormalization.Builder(5, 1e-4, 0.75).build(), "max1")
            .addLayer("batchnorm", D.BatchNormalization.Builder().nOut(64).build(), "lrn1")
            .addLayer("out", D.OutputLayer.Builder().nOut(10).build(), "batchnorm")
            .setOutputs("out").build())
    g = D.ComputationGraph(conf)
    g.init()
    assert float(g.getLayer("cnn1").paramTable()["b"].mean()) == pytest.approx(0.2)
    out = g.output(torch.rand(2, 1, 40, 40))[0]
    assert tuple(out.shape) == (2, 10)
