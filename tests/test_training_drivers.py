"""Listeners, checkpointing, line-search optimizers, normalizers and model serialization round trips
(reference CORET: optimize/solver/TestOptimizers.java, optimizer/listener/TestListeners.java,
optimizer/listener/TestCheckpointListener.java, util/ModelSerializerTest.java,
datasets/iterator/NormalizerTests)."""
import io
import os

import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.datasets.normalizers import (DataNormalization, ImagePreProcessingScaler,
                                                     NormalizerMinMaxScaler, NormalizerStandardize)
from deeplearning4j_amd.optimize import (CheckpointListener, CollectScoresIterationListener,
                                         ComposableIterationListener, EvaluativeListener, InvocationType,
                                         ParamAndGradientIterationListener, PerformanceListener,
                                         ScoreIterationListener, SleepyTrainingListener, TrainingListener)
from deeplearning4j_amd.utils.model_serializer import ModelSerializer

DEV = torch.device("cpu")


def _data(n=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 4, generator=g)
    cls = (x[:, 0] + x[:, 1] > 0).long() + (x[:, 2] > 0.5).long()
    y = torch.zeros(n, 3)
    y[torch.arange(n), cls] = 1
    return x, y


def _net(updater=None, algo=None, dtype=DataType.FLOAT):
    b = NeuralNetConfiguration.Builder().seed(42).dataType(dtype).updater(updater or Adam(0.05))
    if algo is not None:
        b.optimizationAlgo(algo)
    conf = (b.list()
            .layer(0, DenseLayer.Builder().nIn(4).nOut(16).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(16).nOut(3).activation(Activation.SOFTMAX)
                   .build()).build())
    net = MultiLayerNetwork(conf)
    net.init(device=DEV)
    return net


def test_listeners_receive_all_hooks():
    calls = []

    class Rec(TrainingListener):
        def iterationDone(self, m, it, ep):
            calls.append(("it", it, ep))

        def onEpochStart(self, m):
            calls.append(("es",))

        def onEpochEnd(self, m):
            calls.append(("ee",))

        def onForwardPass(self, m, a):
            calls.append(("ff", len(a)))

        def onGradientCalculation(self, m):
            calls.append(("gc",))

        def onBackwardPass(self, m):
            calls.append(("bp",))

    x, y = _data()
    net = _net()
    col = CollectScoresIterationListener(1)
    perf = PerformanceListener(1, reportScore=True)
    net.setListeners(ComposableIterationListener(Rec(), col), ScoreIterationListener(2), perf,
                     SleepyTrainingListener(timerIteration=1))
    it = ListDataSetIterator(DataSet(x, y).asList(), 16)
    net.fit(it, 2)
    names = [c[0] for c in calls]
    assert names.count("es") == 2 and names.count("ee") == 2 and names.count("it") == 8
    assert names.count("ff") == 8 and names.count("bp") == 8 and names.count("gc") == 8
    assert [c[1] for c in calls if c[0] == "it"] == list(range(1, 9))
    assert len(col.getScoreVsIter()) == 8
    s = [v for _, v in col.getScoreVsIter()]
    assert s[-1] < s[0]
    assert len(perf.records) == 7 and perf.records[-1]["samples_per_sec"] > 0
    buf = io.StringIO()
    col.exportScores(buf)
    assert buf.getvalue().startswith("Iteration,Score")


def test_param_and_evaluative_listeners(tmp_path):
    x, y = _data()
    net = _net()
    out = tmp_path / "pg.tsv"
    pg = ParamAndGradientIterationListener(iterations=2, outputToConsole=False, outputToLogger=False,
                                           outputToFile=True, file=str(out))
    seen = []
    ev = EvaluativeListener(DataSet(x, y), 1, InvocationType.EPOCH_END,
                            callback=lambda l, m, n, evals: seen.append(evals[0].accuracy()))
    net.setListeners(pg, ev)
    net.fit(ListDataSetIterator(DataSet(x, y).asList(), 32), 3)
    assert len(seen) == 3 and seen[-1] >= seen[0]
    assert out.exists() and len(out.read_text().splitlines()) == 1 + 3


def test_checkpoint_listener_keep_last(tmp_path):
    x, y = _data()
    net = _net()
    cl = CheckpointListener.Builder(str(tmp_path)).keepLast(2).saveEveryNIterations(2).logSaving(False).build()
    net.setListeners(cl)
    net.fit(ListDataSetIterator(DataSet(x, y).asList(), 8), 1)   # 8 iterations
    cps = cl.availableCheckpoints()
    assert len(cps) == 2
    assert [c.checkpointNum for c in cps] == [cl.lastCheckpointNum - 1, cl.lastCheckpointNum]
    zips = sorted(f for f in os.listdir(tmp_path) if f.endswith(".zip"))
    assert len(zips) == 2 and all("MultiLayerNetwork" in z for z in zips)
    restored = CheckpointListener.loadLastCheckpointMLN(str(tmp_path))
    assert restored.getIterationCount() == cps[-1].iteration
    # resume numbering in a fresh listener
    cl2 = CheckpointListener(str(tmp_path))
    assert cl2.lastCheckpointNum == cl.lastCheckpointNum


def test_checkpoint_keep_last_and_every(tmp_path):
    x, y = _data()
    net = _net()
    cl = CheckpointListener.Builder(str(tmp_path)).keepLastAndEvery(1, 3).saveEveryNIterations(1) \
        .logSaving(False).build()
    net.setListeners(cl)
    net.fit(ListDataSetIterator(DataSet(x, y).asList(), 8), 1)
    nums = [c.checkpointNum for c in cl.availableCheckpoints()]
    assert nums[-1] == cl.lastCheckpointNum
    assert all((n + 1) % 3 == 0 or n == cl.lastCheckpointNum for n in nums)


@pytest.mark.parametrize("algo", [OptimizationAlgorithm.LINE_GRADIENT_DESCENT, OptimizationAlgorithm.CONJUGATE_GRADIENT,
                                  OptimizationAlgorithm.LBFGS, OptimizationAlgorithm.STOCHASTIC_GRADIENT_DESCENT])
def test_optimizers_decrease_score(algo):
    """TestOptimizers: every optimization algorithm reduces the score on a fixed batch."""
    x, y = _data(128, seed=3)
    net = _net(updater=Sgd(0.5), algo=algo, dtype=DataType.DOUBLE)
    ds = DataSet(x.double(), y.double())
    s0 = net.score(ds)
    for _ in range(8):
        net.fit(ds)
    s1 = net.score(ds)
    assert s1 < s0 * 0.9, (algo, s0, s1)
    assert net.getIterationCount() == 8


def test_model_serializer_round_trip_mln_and_normalizer(tmp_path):
    x, y = _data()
    net = _net()
    net.fit(DataSet(x, y))
    norm = NormalizerStandardize().fit(DataSet(x, y))
    p = tmp_path / "m.zip"
    ModelSerializer.writeModel(net, str(p), True, norm)
    net2, norm2 = ModelSerializer.restoreMultiLayerNetworkAndNormalizer(str(p))
    assert torch.equal(net2.params(), net.params())
    assert torch.equal(net2.updater.getStateViewArray(), net.updater.getStateViewArray())
    assert torch.allclose(net2.output(x), net.output(x))
    assert norm2 == norm
    # both continue training identically
    net.fit(DataSet(x, y))
    net2.fit(DataSet(x, y))
    assert torch.allclose(net2.params(), net.params(), atol=1e-6)
    assert ModelSerializer.restoreNormalizerFromFile(str(p)) == norm


def test_model_serializer_graph(tmp_path):
    conf = (NeuralNetConfiguration.Builder().seed(1).updater(Nesterovs(0.1, 0.9)).graphBuilder()
            .addInputs("in")
            .addLayer("d", DenseLayer.Builder().nIn(4).nOut(8).activation(Activation.RELU).build(), "in")
            .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nIn(8).nOut(3)
                      .activation(Activation.SOFTMAX).build(), "d")
            .setOutputs("out").build())
    g = ComputationGraph(conf)
    g.init(device=DEV)
    x, y = _data()
    g.fit(DataSet(x, y))
    p = tmp_path / "g.zip"
    ModelSerializer.writeModel(g, str(p), True)
    g2 = ModelSerializer.restoreComputationGraph(str(p))
    assert torch.equal(g2.params(), g.params())
    assert torch.allclose(g2.outputSingle(x), g.outputSingle(x))
    assert type(ModelSerializer.restoreModel(str(p))).__name__ == "ComputationGraph"


def test_normalizers():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(100, 5, generator=g) * torch.tensor([1., 2., 3., 4., 5.]) + torch.arange(5.)
    ds = DataSet(x.clone(), torch.randn(100, 2, generator=g))
    n = NormalizerStandardize().fit(ListDataSetIterator(ds.asList(), 10))
    assert torch.allclose(n.getMean().float(), x.mean(0), atol=1e-5)
    assert torch.allclose(n.getStd().float(), x.std(0, unbiased=False), atol=1e-4)
    d2 = ds.copy()
    n.preProcess(d2)
    assert torch.allclose(d2.features.mean(0), torch.zeros(5), atol=1e-5)
    n.revert(d2)
    assert torch.allclose(d2.features, x, atol=1e-4)
    mm = NormalizerMinMaxScaler(-1, 1).fitLabel(True).fit(ds)
    t = mm.transform(x)
    assert torch.allclose(t.min(0).values, -torch.ones(5)) and torch.allclose(t.max(0).values, torch.ones(5))
    assert torch.allclose(mm.revertFeatures(t), x, atol=1e-5)
    img = ImagePreProcessingScaler(0, 1)
    assert torch.allclose(img.transform(torch.tensor([[0., 255.]])), torch.tensor([[0., 1.]]))
    for obj in (n, mm, img):
        assert DataNormalization.from_bytes(obj.to_bytes()) == obj
    # 3d time series: stats over (examples, time)
    ts = torch.randn(4, 3, 7, generator=g) * 3 + 1
    nt = NormalizerStandardize().fit(DataSet(ts, torch.zeros(4, 2, 7)))
    assert torch.allclose(nt.getMean().float(), ts.permute(0, 2, 1).reshape(-1, 3).mean(0), atol=1e-5)


def test_memory_report():
    """NetworkMemoryReport semantics (reference CORET: nn/conf/memory/MemoryReportTest.java)."""
    from deeplearning4j_amd.nn.conf.memory import MemoryType, MemoryUseMode
    conf = (NeuralNetConfiguration.Builder().updater(Adam(1e-3)).list()
            .layer(0, DenseLayer.Builder().nIn(10).nOut(20).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(20).nOut(5).activation(Activation.SOFTMAX).build())
            .setInputType(InputType.feedForward(10)).build())
    r = conf.getMemoryReport()
    P = 10 * 20 + 20 + 20 * 5 + 5
    assert r.getMemoryBytes(MemoryType.PARAMETERS, 1, MemoryUseMode.INFERENCE) == 4 * P
    assert r.getMemoryBytes(MemoryType.UPDATER_STATE, 1, MemoryUseMode.TRAINING) == 4 * 2 * P   # Adam m+v
    assert r.getMemoryBytes(MemoryType.UPDATER_STATE, 1, MemoryUseMode.INFERENCE) == 0
    assert r.getMemoryBytes(MemoryType.ACTIVATIONS, 7, MemoryUseMode.INFERENCE) == 4 * 7 * (20 + 5)
    tr = r.getTotalMemoryBytes(8, MemoryUseMode.TRAINING)
    inf = r.getTotalMemoryBytes(8, MemoryUseMode.INFERENCE)
    assert tr > inf > 0
    assert r.getMemoryBytes(MemoryType.PARAMETERS, 1, MemoryUseMode.INFERENCE, None, "DOUBLE") == 8 * P
    assert "Network Memory Report" in r.toString()
    assert r.maxMinibatchFor(1 << 20) > 0
