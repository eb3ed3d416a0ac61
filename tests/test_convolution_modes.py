"""Convolution modes (Strict / Truncate / Same), after the reference's TestConvolutionModes
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/convolution/TestConvolutionModes.java:34-442):
Truncate ignores edge data the kernel never covers and Strict refuses sizes the stride does not tile; the global
mode is inherited by layers that set none while a per-layer mode wins; output-size arithmetic per mode; Same-mode
activation shapes for convolution and subsampling."""
import pytest
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.exceptions import DL4JException
from deeplearning4j_amd.nn.conf.enums import ConvolutionMode as CM
from deeplearning4j_amd.nn.conf.layers import conv_out_size


def _net(layer, cm, size, depth):
    conf = (D.NeuralNetConfiguration.Builder().seed(12345).weightInit(D.WeightInit.XAVIER).convolutionMode(cm).list()
            .layer(0, layer)
            .layer(1, D.OutputLayer.Builder(D.LossFunction.MCXENT).nOut(3).activation(D.Activation.SOFTMAX).build())
            .setInputType(D.InputType.convolutional(size, size, depth)).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


@pytest.mark.parametrize("subsampling", [False, True])
@pytest.mark.parametrize("mb,depth", [(1, 1), (3, 3)])
def test_strict_truncate_edge_data_does_not_matter(subsampling, mb, depth):
    """9x9 data embedded in 9/10/11-square inputs, kernel 3 stride 3 padding 0: Truncate gives the output of the 9x9
    data whatever sits in the uncovered edge; Strict builds only for 9 (10 and 11 do not tile)."""
    g = torch.Generator().manual_seed(12345)
    orig = torch.rand(mb, depth, 9, 9, generator=g)
    for size in (9, 10, 11):
        for cm in (CM.Strict, CM.Truncate):
            data = torch.rand(mb, depth, size, size, generator=g)
            data[:, :, :9, :9] = orig
            layer = (D.SubsamplingLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0]).build()
                     if subsampling else
                     D.ConvolutionLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0]).nOut(3).build())
            if size > 9 and cm == CM.Strict:
                with pytest.raises(DL4JException):
                    _net(layer, cm, size, depth)
                continue
            torch.manual_seed(7)
            net = _net(layer, cm, size, depth)
            if size > 9:
                ref_layer = (D.SubsamplingLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0]).build()
                             if subsampling else
                             D.ConvolutionLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0]).nOut(3)
                             .build())
                ref = _net(ref_layer, cm, 9, depth)
                ref.setParams(net.params())
                a = ref.output(orig)
            else:
                a = net.output(orig)
            b = net.output(data)
            assert torch.allclose(a, b, atol=1e-6), (subsampling, size, cm)


@pytest.mark.parametrize("cm", [CM.Strict, CM.Truncate])
def test_global_and_local_modes(cm):
    """The global mode fills layers that set none; a layer's own mode wins (conv and subsampling)."""
    def conv(mode=None):
        b = D.ConvolutionLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0]).nIn(3).nOut(3)
        return (b.convolutionMode(mode) if mode else b).build()

    def pool(mode=None):
        b = D.SubsamplingLayer.Builder().kernelSize([3, 3]).stride([3, 3]).padding([0, 0])
        return (b.convolutionMode(mode) if mode else b).build()
    layers = [conv(), conv(CM.Strict), conv(CM.Truncate), conv(CM.Same), pool(), pool(CM.Strict), pool(CM.Truncate),
              pool(CM.Same)]
    b = D.NeuralNetConfiguration.Builder().weightInit(D.WeightInit.XAVIER).convolutionMode(cm).list()
    for i, l in enumerate(layers):
        b = b.layer(i, l)
    conf = b.layer(len(layers), D.OutputLayer.Builder(D.LossFunction.MCXENT).nOut(3).build()).build()
    want = [cm, CM.Strict, CM.Truncate, CM.Same, cm, CM.Strict, CM.Truncate, CM.Same]
    got = [conf.getConf(i).getLayer().convolutionMode for i in range(len(layers))]
    assert got == want


def test_output_size_arithmetic_per_mode():
    """Input 3x3, kernel 2, stride 1: Strict = Truncate = 2, Same = ceil(3/1) = 3. Input 3x4, kernel 3, stride 2:
    Strict raises ((4-3)/2 is not an integer), Truncate = 1x1, Same = ceil(3/2) x ceil(4/2) = 2x2 — through the
    size helper and through the layer's InputType inference."""
    assert conv_out_size(3, 2, 1, 0, 1, CM.Strict) == 2
    assert conv_out_size(3, 2, 1, 0, 1, CM.Truncate) == 2
    assert conv_out_size(3, 2, 1, 0, 1, CM.Same) == 3
    with pytest.raises(DL4JException):
        conv_out_size(4, 3, 2, 0, 1, CM.Strict)
    assert (conv_out_size(3, 3, 2, 0, 1, CM.Truncate), conv_out_size(4, 3, 2, 0, 1, CM.Truncate)) == (1, 1)
    assert (conv_out_size(3, 3, 2, 0, 1, CM.Same), conv_out_size(4, 3, 2, 0, 1, CM.Same)) == (2, 2)
    it = D.InputType.convolutional(3, 4, 5)
    for cm, hw in ((CM.Truncate, (1, 1)), (CM.Same, (2, 2))):
        layer = D.ConvolutionLayer.Builder().kernelSize([3, 3]).stride([2, 2]).nIn(5).nOut(7).convolutionMode(cm) \
            .build()
        out = layer.getOutputType(0, it)
        assert (out.height, out.width, out.channels) == (*hw, 7)
    strict = D.ConvolutionLayer.Builder().kernelSize([3, 3]).stride([2, 2]).nIn(5).nOut(7) \
        .convolutionMode(CM.Strict).build()
    with pytest.raises(DL4JException):
        strict.getOutputType(0, it)


@pytest.mark.parametrize("subsampling", [False, True])
def test_same_mode_activation_sizes(subsampling):
    """Same mode, 3x4 input, kernel 3 stride 2: activations [mb, C, ceil(3/2), ceil(4/2)] for conv and pooling."""
    layer = (D.SubsamplingLayer.Builder().kernelSize([3, 3]).stride([2, 2]).build() if subsampling else
             D.ConvolutionLayer.Builder().nOut(4).kernelSize([3, 3]).stride([2, 2]).build())
    conf = (D.NeuralNetConfiguration.Builder().convolutionMode(CM.Same).list().layer(0, layer)
            .layer(1, D.OutputLayer.Builder(D.LossFunction.MCXENT).nOut(3).activation(D.Activation.SOFTMAX).build())
            .setInputType(D.InputType.convolutional(3, 4, 3)).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    acts = net.feedForward(torch.zeros(5, 3, 3, 4))
    assert tuple(acts[1].shape) == (5, 3 if subsampling else 4, 2, 2)
