"""Training iterations run inside the per-iteration LOOP_FF_BP workspace (memory/arena.py; reference
MultiLayerNetwork.java:126-144): identical results to WorkspaceMode.NONE, activations carved from the arena after the
learning cycle (no spills), stable addresses across iterations, and SCOPE_PANIC on an activation leaked out of an
iteration."""
import pytest
import torch

from deeplearning4j_amd import DenseLayer, MultiLayerNetwork, NeuralNetConfiguration, OutputLayer, Sgd
from deeplearning4j_amd.memory.workspace import ND4JWorkspaceException, check_scope
from deeplearning4j_amd.nn.conf import WorkspaceMode


def _net(mode):
    conf = (NeuralNetConfiguration.Builder().seed(11).updater(Sgd(0.1)).trainingWorkspaceMode(mode).list()
            .layer(DenseLayer.Builder().nIn(12).nOut(16).activation("TANH").build())
            .layer(DenseLayer.Builder().nIn(16).nOut(16).activation("RELU").build())
            .layer(OutputLayer.Builder("MCXENT").nIn(16).nOut(4).activation("SOFTMAX").build()).build())
    net = MultiLayerNetwork(conf)
    net.init()
    return net


def _data():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(32, 12, generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 4, (32,), generator=g), 4).float()
    return x, y


def test_workspace_training_matches_no_workspace_and_reuses_arena():
    x, y = _data()
    a, b = _net(WorkspaceMode.ENABLED), _net(WorkspaceMode.NONE)
    ptrs = []
    for i in range(5):
        a.fit(x, y)
        b.fit(x, y)
        ws = a._loop_ws
        st = ws.stats()
        if i >= 1:
            assert st["spilled"] == 0 and st["learned"] == 1, st     # after the learning cycle: all carved
        ptrs.append(a._layer_offsets[0][2]._z.data_ptr() if hasattr(a._layer_offsets[0][2], "_z") else None)
    assert torch.equal(a.params(), b.params())
    assert a.score() == pytest.approx(b.score())
    assert getattr(b, "_loop_ws", None) is None                         # NONE: no arena
    assert ptrs[2] == ptrs[3] == ptrs[4]                                # same address every iteration


def test_scope_panic_on_leaked_activation():
    x, y = _data()
    net = _net(WorkspaceMode.ENABLED)
    net.fit(x, y)
    net.fit(x, y)
    z = net._layer_offsets[0][2]._z                                     # carved inside the last iteration
    with pytest.raises(ND4JWorkspaceException):
        check_scope(z, "leaked activation")
    out = net.output(x)                                                 # outside any iteration: plain allocation
    check_scope(out, "output")
