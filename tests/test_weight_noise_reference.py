"""Weight noise, after the reference's TestWeightNoise
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/weightnoise/TestWeightNoise.java:37-245): a global
weightNoise (DropConnect with a fixed or scheduled retain probability, or additive Gaussian WeightNoise) is inherited
by every layer unless a layer sets its own, in MultiLayerNetwork and ComputationGraph, and survives ModelSerializer;
DropConnect leaves the parameter untouched at inference and, in training, keeps each weight (value 1 with ONES init) or
drops it to 0, about half of each at p = 0.5. CPU."""
import io

import pytest
import torch

import deeplearning4j_amd as D


def _noises():
    return [D.DropConnect(0.5),
            D.DropConnect(D.SigmoidSchedule(D.ScheduleType.ITERATION, 0.5, 0.5, 100)),
            D.WeightNoise(D.NormalDistribution(0, 0.1))]


def _layers():
    return [D.DenseLayer.Builder().nIn(10).nOut(10).build(),
            D.DenseLayer.Builder().nIn(10).nOut(10).weightNoise(D.DropConnect(0.25)).build(),
            D.OutputLayer.Builder().nIn(10).nOut(10).build()]


def _same(a, b):
    return a.toJson() == b.toJson()


@pytest.mark.parametrize("i", range(3))
def test_weight_noise_config_inherited_and_serialized(i):
    wn = _noises()[i]
    lb = D.NeuralNetConfiguration.Builder().weightNoise(wn).list()
    for l in _layers():
        lb = lb.layer(l)
    net = D.MultiLayerNetwork(lb.build())
    net.init()
    assert _same(net.getLayer(0).conf.weightNoise, wn)
    assert _same(net.getLayer(1).conf.weightNoise, D.DropConnect(0.25))
    assert _same(net.getLayer(2).conf.weightNoise, wn)
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    buf = io.BytesIO()
    ModelSerializer.writeModel(net, buf, True)
    buf.seek(0)
    back = ModelSerializer.restoreMultiLayerNetwork(buf, True)
    assert _same(back.getLayer(0).conf.weightNoise, wn)
    assert torch.equal(back.params(), net.params())

    gb = D.NeuralNetConfiguration.Builder().weightNoise(wn).graphBuilder().addInputs("in")
    prev = "in"
    for j, l in enumerate(_layers()):
        gb = gb.addLayer(str(j), l, prev)
        prev = str(j)
    g = D.ComputationGraph(gb.setOutputs("2").build())
    g.init()
    assert _same(g.getLayer("0").conf.weightNoise, wn)
    assert _same(g.getLayer("1").conf.weightNoise, D.DropConnect(0.25))
    assert _same(g.getLayer("2").conf.weightNoise, wn)


def test_drop_connect_values():
    torch.manual_seed(12345)
    net = D.MultiLayerNetwork(D.NeuralNetConfiguration.Builder().weightInit(D.WeightInit.ONES).list()
                              .layer(D.OutputLayer.Builder().nIn(10).nOut(10).build()).build())
    net.init()
    layer = net.getLayer(0)
    w = layer.getParam("W")
    d = D.DropConnect(0.5)
    assert d.getParameter(layer, "W", w, 0, 0, False) is w          # inference: the parameter itself
    out = d.getParameter(layer, "W", w, 0, 0, True)
    assert torch.equal(w, torch.ones(10, 10, dtype=w.dtype))       # the parameter is not modified
    zeros, ones = int((out == 0).sum()), int((out == 1).sum())
    assert zeros + ones == 100
    assert 25 <= zeros <= 75 and 25 <= ones <= 75


def test_schedules_take_reference_constructor_order():
    """ISchedule implementations take the reference's (ScheduleType, values...) constructor arguments."""
    it = D.ScheduleType.ITERATION
    assert D.SigmoidSchedule(it, 0.5, 0.5, 100).valueAt(100, 0) == pytest.approx(0.25)
    assert D.StepSchedule(it, 1.0, 0.5, 10).valueAt(25, 0) == pytest.approx(0.25)
    assert D.ExponentialSchedule(it, 2.0, 0.5).valueAt(3, 0) == pytest.approx(0.25)
    assert D.InverseSchedule(it, 1.0, 1.0, 2.0).valueAt(1, 0) == pytest.approx(0.25)
    assert D.PolySchedule(it, 1.0, 2.0, 10).valueAt(0, 0) == pytest.approx(1.0)
    assert D.MapSchedule(D.ScheduleType.EPOCH, {0: 1.0, 5: 0.5}).valueAt(0, 7) == pytest.approx(0.5)
    assert D.FixedSchedule(0.3).valueAt(99, 9) == pytest.approx(0.3)
    s = D.SigmoidSchedule(it, 0.5, 0.5, 100)
    assert type(s).fromJson(s.toJson()).toJson() == s.toJson()
