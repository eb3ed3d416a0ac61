"""GravesLSTM sequence output, after the reference's GravesLSTMOutputTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/multilayer/GravesLSTMOutputTest.java:30-137): a GravesLSTM
(20 -> 15, N(0, 0.01) weights, AdaGrad 0.1, l2 2.5e-3, NegativeDefaultStepFunction) feeding a softmax output layer
through an RnnToFeedForwardPreProcessor learns to echo a 300-step one-hot sequence given 2d [300, 20] labels (F1 >
0.9 after 40 fits), and the same network trains with truncated BPTT (window 100) over 3d labels. The reference draws
the sequence with java.util.Random(1); a seeded torch draw of the same shape stands in. CPU."""
import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.optimize.listeners import ScoreIterationListener
from deeplearning4j_amd.optimize.solvers import NegativeDefaultStepFunction

N_IN, LAYER, WINDOW = 20, 15, 300


def _data():
    g = torch.Generator().manual_seed(1)
    return D.FeatureUtil.toOutcomeMatrix(torch.randint(N_IN, (WINDOW,), generator=g).tolist(), N_IN)


def _reshape(inp):
    # [T, nIn] -> [1, nIn, T] (reference reshapeInput: reshape to [1, T, nIn], permute(0, 2, 1))
    return inp.reshape(1, inp.shape[0], inp.shape[1]).permute(0, 2, 1).contiguous()


def _conf(tbptt):
    b = (D.NeuralNetConfiguration.Builder().updater(D.AdaGrad(0.1)).l2(0.0025).seed(12345)
         .stepFunction(NegativeDefaultStepFunction()).list()
         .layer(0, D.GravesLSTM.Builder().weightInit(D.WeightInit.DISTRIBUTION).dist(D.NormalDistribution(0.0, 0.01))
                .nIn(N_IN).nOut(LAYER).activation(D.Activation.TANH).build())
         .layer(1, D.OutputLayer.Builder(D.LossFunction.NEGATIVELOGLIKELIHOOD).nIn(LAYER).nOut(N_IN)
                .activation(D.Activation.SOFTMAX).build())
         .inputPreProcessor(1, D.RnnToFeedForwardPreProcessor()).backprop(True).pretrain(False))
    if tbptt:
        b = b.backpropType(D.BackpropType.TruncatedBPTT).tBPTTBackwardLength(WINDOW // 3) \
            .tBPTTForwardLength(WINDOW // 3)
    return b.build()


def _eval(net, data):
    ev = D.Evaluation(N_IN)
    ev.eval(data, net.output(_reshape(data)))
    return ev


def test_same_labels_output():
    data = _data()
    net = D.MultiLayerNetwork(_conf(False))
    net.init()
    net.setListeners([ScoreIterationListener(100)])
    for _ in range(40):
        net.fit(_reshape(data.clone()), data.clone())
    assert _eval(net, data).f1() > 0.90


def test_same_labels_output_with_tbptt():
    data = _data()
    net = D.MultiLayerNetwork(_conf(True))
    net.init()
    for i in range(WINDOW // 100):
        d = data[100 * i:100 * (i + 1)]
        for _ in range(40):
            net.fit(_reshape(d.clone()), _reshape(d.clone()))
    out = net.output(_reshape(data))
    assert out.shape == (WINDOW, N_IN) and torch.isfinite(out).all()
    _eval(net, data)
