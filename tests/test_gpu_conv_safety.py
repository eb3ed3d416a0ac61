"""Correctness guards around the conv kernels' in-place and overlap-stream paths (run on MI355X):

* x + conv(x) with an identity activation: the graph must not hand the conv's own dY to its bwd-data kernel as the
  in-place accumulation target (computation_graph.py fan-out).
* the first eager step of a 1x1-conv network times GEMM vs implicit-GEMM weight-gradient candidates on scratch
  buffers: with the overlap stream on, the candidates must still run inline (ops/side_stream.suspended) and the
  resulting gradients must equal an overlap-off run.
* DL4J_AMD_DETERMINISTIC=1 weight gradients: equal to the fp32 torch reference and bitwise reproducible.
"""
import pytest
import torch
import torch.nn.functional as F

from deeplearning4j_amd.ops import conv_native

pytestmark = pytest.mark.gpu


def _graph(C, dtype, seed=3):
    from deeplearning4j_amd import Activation, LossFunction, NeuralNetConfiguration, Sgd
    from deeplearning4j_amd.nn.conf.graph import ElementWiseVertex
    from deeplearning4j_amd.nn.conf.inputs import InputType
    from deeplearning4j_amd.nn.conf.layers import ConvolutionLayer, GlobalPoolingLayer, OutputLayer
    from deeplearning4j_amd.nn.graph.computation_graph import ComputationGraph
    conf = (NeuralNetConfiguration.Builder().seed(seed).updater(Sgd(0.1)).dataType(dtype).graphBuilder()
            .addInputs("in")
            .addLayer("c1", ConvolutionLayer.Builder(3, 3).nIn(8).nOut(C).padding(1, 1)
                      .activation(Activation.RELU).build(), "in")
            .addLayer("c2", ConvolutionLayer.Builder(3, 3).nIn(C).nOut(C).padding(1, 1)
                      .activation(Activation.IDENTITY).build(), "c1")
            .addVertex("add", ElementWiseVertex(ElementWiseVertex.Op.Add), "c1", "c2")
            .addLayer("c3", ConvolutionLayer.Builder(1, 1).nIn(C).nOut(C)
                      .activation(Activation.IDENTITY).build(), "add")
            .addVertex("add2", ElementWiseVertex(ElementWiseVertex.Op.Add), "add", "c3")
            .addLayer("gap", GlobalPoolingLayer.Builder().build(), "add2")
            .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nIn(C).nOut(4)
                      .activation(Activation.SOFTMAX).build(), "gap")
            .setOutputs("out").setInputTypes(InputType.convolutional(10, 10, 8)).build())
    net = ComputationGraph(conf)
    net.init(device=torch.device("cuda", 0))
    return net


def _data(bs=6):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(bs, 8, 10, 10, generator=g).cuda()
    y = torch.zeros(bs, 4)
    y[torch.arange(bs), torch.randint(0, 4, (bs,), generator=g)] = 1
    return x, y.cuda()


def _grad(net, x, y):
    net.computeGradientAndScore([x], [y])
    torch.cuda.synchronize()
    return net.getGradientsViewArray().float().clone()


@pytest.mark.parametrize("C", [8, 64])
def test_x_plus_conv_x_gradient_matches_out_of_place(C, monkeypatch):
    """In-place fan-out accumulation on vs off (every gradient summed out of place): the same bf16 gradients up to
    the rounding of one extra bf16 add. A kernel overwriting the dY it reads would differ by O(1). The fp32 network
    is only a gross sanity bound here: global pooling makes the weight gradients differences of nearly equal
    pixel sums, so bf16 activation rounding alone moves them by several percent."""
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.nn.graph import computation_graph as cgm
    x, y = _data()
    ref = _graph(C, DataType.FLOAT)
    net = _graph(C, DataType.BFLOAT16)
    net.setParams(ref.params().clone())
    g32 = _grad(ref, x, y)
    g16 = _grad(net, x, y)
    monkeypatch.setattr(cgm, "_shares_storage", lambda a, b: True)
    g16b = _grad(net, x, y)
    rel = ((g16 - g16b).norm() / g16b.norm()).item()
    assert rel <= 1e-2, rel
    assert ((g16 - g32).norm() / g32.norm()).item() <= 0.2


def test_first_eager_1x1_step_same_with_and_without_overlap_stream(monkeypatch):
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.ops import side_stream
    x, y = _data(8)
    grads = {}
    for on in ("0", "1"):
        monkeypatch.setenv("DL4J_AMD_WRW_STREAM", on)
        monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
        conv_native._CHOICE.clear()              # force the first-call timing of the 1x1 candidates
        net = _graph(64, DataType.BFLOAT16, seed=9)
        n0 = side_stream.LAUNCHES[0]
        grads[on] = _grad(net, x, y)
        if on == "1":
            assert side_stream.LAUNCHES[0] > n0
    assert torch.equal(grads["0"], grads["1"])


@pytest.mark.parametrize("case", [(4, 64, 14, 14, 128, 3, 3, (1, 1), (1, 1, 1, 1)),
                                  (8, 256, 7, 7, 64, 1, 1, (2, 2), (0, 0, 0, 0)),
                                  (2, 32, 9, 9, 136, 3, 3, (2, 2), (1, 1, 1, 1))])
def test_deterministic_weight_gradient(monkeypatch, case):
    monkeypatch.setenv("DL4J_AMD_DETERMINISTIC", "1")
    N, C, H, W, K, R, S, stride, pad4 = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, S, generator=g) * 0.1).cuda().bfloat16()
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    br = torch.zeros(K, device="cuda", requires_grad=True)
    yr = F.conv2d(F.pad(xr, (pad4[2], pad4[3], pad4[0], pad4[1])), wr, br, stride)
    dy = torch.randn(yr.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    outs = []
    for _ in range(2):
        gW = torch.full((K, C, R, S), 7.0, device="cuda")     # overwritten, not accumulated
        gb = torch.full((K,), 7.0, device="cuda")
        conv_native._conv2d_wrw(x, dy, N, H, W, C, K, R, S, dy.shape[2], dy.shape[3], stride, pad4, (1, 1), True,
                                gW, gb, False, False)
        torch.cuda.synchronize()
        outs.append((gW.clone(), gb.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    scale = wr.grad.abs().max().item()
    assert (outs[0][0] - wr.grad).abs().max().item() <= 1e-2 * scale
    assert (outs[0][1] - br.grad).abs().max().item() <= 1e-2 * br.grad.abs().max().item()
