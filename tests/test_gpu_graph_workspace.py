"""The training workspace on the HIP-graph path (memory/arena.py graph_workspace, nn/hipgraph.py): the captured
step carves its activations (conv / BatchNorm / pooling outputs, BN masks and statistics, gradients in flight) from
its own frozen LOOP_FF_BP arena, sized from what the eager warmup iteration learned, and trains exactly like eager
steps. Reference: NN:nn/multilayer/MultiLayerNetwork.java:126-144, NN:nn/graph/ComputationGraph.java:107-136."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403

pytestmark = pytest.mark.gpu


def _net():
    from deeplearning4j_amd.nn.conf.layers import (BatchNormalization, ConvolutionLayer, GlobalPoolingLayer,
                                                   OutputLayer, SubsamplingLayer)
    b = (NeuralNetConfiguration.Builder().seed(5).dataType(DataType.BFLOAT16).updater(Adam(0.01)).graphBuilder()
         .addInputs("in")
         .addLayer("c1", ConvolutionLayer.Builder(3, 3).nIn(8).nOut(64).padding(1, 1)
                   .activation(Activation.IDENTITY).build(), "in")
         .addLayer("bn1", BatchNormalization.Builder().nOut(64).activation(Activation.RELU).build(), "c1")
         .addLayer("p1", SubsamplingLayer.Builder(PoolingType.MAX).kernelSize(2, 2).stride(2, 2).build(), "bn1")
         .addLayer("c2", ConvolutionLayer.Builder(3, 3).nIn(64).nOut(64).padding(1, 1)
                   .activation(Activation.IDENTITY).build(), "p1")
         .addLayer("bn2", BatchNormalization.Builder().nOut(64).activation(Activation.RELU).build(), "c2")
         .addLayer("gap", GlobalPoolingLayer.Builder().build(), "bn2")
         .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nIn(64).nOut(10)
                   .activation(Activation.SOFTMAX).build(), "gap")
         .setOutputs("out").setInputTypes(InputType.convolutional(16, 16, 8)).build())
    net = ComputationGraph(b)
    net.init(device=torch.device("cuda", 0))
    return net


def _batches(n=5, mb=32):
    g = torch.Generator().manual_seed(1)
    out = []
    for _ in range(n):
        x = torch.randn(mb, 8, 16, 16, generator=g).cuda().contiguous(memory_format=torch.channels_last)
        y = torch.zeros(mb, 10, device="cuda")
        y[torch.arange(mb), torch.randint(0, 10, (mb,), generator=g).cuda()] = 1
        out.append((x.to(torch.bfloat16), y))
    return out


def test_captured_step_lives_in_its_workspace(monkeypatch):
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    from deeplearning4j_amd.memory import arena
    batches = _batches()
    net = _net()
    ref2 = _net()
    net.enableHipGraphs(True, warmup=1)
    for x, y in batches:
        net.fit([x], [y])
        ref2.fit([x], [y])
    torch.cuda.synchronize()
    cs = net._hipgraph
    assert cs is not None and cs.ok, "step was not captured"
    assert cs.ws is not None and cs.ws._buf is not None and cs.ws.frozen
    assert cs.ws.estimate_bytes > 0
    # every layer's input after the first is an activation of the captured iteration: inside the arena buffer
    for name in ("bn1", "p1", "c2", "bn2", "gap"):
        t = net.layers_by_name[name].input
        assert arena._owned(cs.ws, t), f"{name} input not carved from the graph workspace"
    assert cs.ws.external_bytes == 0, "captured iteration spilled outside its arena"
    # the eager warmup arena was released for the graph's
    eager = getattr(net, "_loop_ws", None)
    assert eager is None or eager._buf is None
    # graph training == eager training (deterministic weight gradients)
    assert torch.allclose(net.params(), ref2.params(), atol=1e-6, rtol=0), (net.params() - ref2.params()).abs().max()


def test_workspace_too_large_degrades_to_graph_pool(monkeypatch, caplog):
    """an arena larger than the free HBM is not made (None: the capture uses the graph's private pool),
    with a warning naming the numbers, instead of raising out of fit()."""
    from deeplearning4j_amd.memory import arena
    net = _net()
    x, y = _batches(1)[0]
    net.fit([x], [y])
    net._loop_ws = None                     # no learned size: the memory report's estimate sizes the arena
    assert arena._activation_estimate(net, 4096) > (1 << 20)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (1 << 20, 288 << 30))
    with caplog.at_level("WARNING", logger="deeplearning4j_amd"):
        assert arena.graph_workspace(net, 4096, ("k",)) is None
    assert "capturing without a frozen arena" in caplog.text


def test_workspace_sized_per_key_minibatch():
    """A tail-batch capture key gets an arena scaled by its minibatch over the learned one."""
    from deeplearning4j_amd.memory import arena
    net = _net()
    x, y = _batches(1)[0]
    net.fit([x], [y])
    learned_mb = net._ws_learned_mb
    assert learned_mb == x.shape[0]
    full = arena.graph_workspace(net, learned_mb, ("full",))
    half = arena.graph_workspace(net, max(1, learned_mb // 2), ("half",))
    if full is None or half is None:
        pytest.skip("network below the arena threshold")
    assert half.conf.initialSize < full.conf.initialSize
