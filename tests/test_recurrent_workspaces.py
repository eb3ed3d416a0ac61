"""Training workspaces for recurrent networks (reference MultiLayerNetwork.java:126-144 LOOP_FF_BP and :1556-1583
LOOP_TBPTT): LSTM / GravesLSTM / SimpleRnn networks train inside the arenas (memory/arena.py), every TBPTT window
gets its own LOOP_TBPTT cycle, the carried state is leveraged out of the arena, and the result equals training
with workspaces disabled (trainingWorkspaceMode NONE)."""
import pytest
import torch

from deeplearning4j_amd import Adam, LossFunction, MultiLayerNetwork, NeuralNetConfiguration
from deeplearning4j_amd.memory import arena
from deeplearning4j_amd.nn.conf.enums import WorkspaceMode


def _net(kind, mode, tbptt=None):
    from deeplearning4j_amd.nn.conf.layers import LSTM, GravesLSTM, RnnOutputLayer, SimpleRnn
    L = {"lstm": LSTM, "graves": GravesLSTM, "simple": SimpleRnn}[kind]
    b = (NeuralNetConfiguration.Builder().seed(5).updater(Adam(0.01)).trainingWorkspaceMode(mode).list()
         .layer(0, L.Builder().nIn(4).nOut(8).build())
         .layer(1, RnnOutputLayer.Builder(LossFunction.MCXENT).nIn(8).nOut(3).build()))
    if tbptt:
        b = b.backpropType("TruncatedBPTT").tBPTTForwardLength(tbptt).tBPTTBackwardLength(tbptt)
    n = MultiLayerNetwork(b.build())
    n.init()
    return n


def _data(seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(5, 4, 13, generator=g)
    y = torch.nn.functional.one_hot(torch.randint(0, 3, (5, 13), generator=g), 3).permute(0, 2, 1).float()
    return x, y


@pytest.mark.parametrize("kind", ["lstm", "graves", "simple"])
@pytest.mark.parametrize("tbptt", [None, 5])
def test_recurrent_training_in_workspaces_equals_no_workspace(kind, tbptt):
    a = _net(kind, WorkspaceMode.ENABLED, tbptt)
    b = _net(kind, WorkspaceMode.NONE, tbptt)
    b.setParams(a.params().clone())
    for i in range(3):
        x, y = _data(i)
        a.fit(x, y)
        b.fit(x, y)
    assert a._ws_ok and not b._ws_ok
    assert torch.equal(a.params(), b.params())
    ws = a._loop_ws
    assert ws.stats()["cycles"] >= 3
    if tbptt:
        st = a._tbptt_ws.stats()
        assert st["cycles"] >= 3 * 3                       # ceil(13 / 5) windows per fit
        assert st["maxPeak"] > 0                          # the windows' arrays were carved from LOOP_TBPTT


def test_state_carried_out_of_the_arena():
    """rnnTimeStep state and TBPTT state never point into a closed arena (no leaked workspace pointers)."""
    n = _net("simple", WorkspaceMode.ENABLED, 5)
    x, y = _data(7)
    n.fit(x, y)
    impl = n.layers[0]
    for m in (impl.stateMap, impl.tBpttStateMap):
        for v in m.values():
            for ws in (n._loop_ws, n._tbptt_ws):
                assert not arena._owned(ws, v)
    out = n.rnnTimeStep(x[:, :, :3])
    assert out.shape == (5, 3, 3)
    for v in impl.stateMap.values():
        assert not arena._owned(n._loop_ws, v)
