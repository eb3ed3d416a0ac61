"""SameDiff's own reverse-mode autodiff: every registered op's explicit backward against fp64 central finite
differences (the reference's GradCheckUtil-style check, NN:gradientcheck/GradientCheckUtil.java and the SameDiff op
validation of ND4J's OpValidation), whole-graph gradient checks through ``execBackwards``, training without
torch.autograd, and graph save / load."""
import pathlib

import pytest
import torch

from deeplearning4j_amd.samediff import SameDiff, TrainingConfig
from deeplearning4j_amd.samediff.autodiff import REGISTRY

D = torch.float64


def _fd_check(op, ins, attrs, wrt, eps=1e-6, rtol=1e-5, atol=1e-7, seed=0):
    gen = torch.Generator().manual_seed(seed)
    y, ctx = REGISTRY[op].fwd(ins, attrs)
    g = torch.randn(y.shape, generator=gen, dtype=D)
    grads = REGISTRY[op].bwd(ctx, g, ins, attrs)
    for i in wrt:
        x = ins[i]
        num = torch.zeros_like(x)
        flat = x.reshape(-1)
        for j in range(flat.numel()):
            old = flat[j].item()
            flat[j] = old + eps
            fp = (REGISTRY[op].fwd(ins, attrs)[0] * g).sum().item()
            flat[j] = old - eps
            fm = (REGISTRY[op].fwd(ins, attrs)[0] * g).sum().item()
            flat[j] = old
            num.reshape(-1)[j] = (fp - fm) / (2 * eps)
        assert grads[i] is not None, (op, i)
        torch.testing.assert_close(grads[i].to(D), num, rtol=rtol, atol=atol, msg=lambda m: f"{op} input {i}: {m}")


def _r(*shape, seed=1, lo=None):
    t = torch.randn(*shape, generator=torch.Generator().manual_seed(seed), dtype=D)
    return t.abs() + lo if lo is not None else t


BINARY = ["add", "sub", "mul", "div", "rsub", "rdiv"]


@pytest.mark.parametrize("op", BINARY)
def test_binary_broadcast_grad(op):
    a, b = _r(3, 4, seed=1, lo=0.5), _r(1, 4, seed=2, lo=0.5)
    _fd_check(op, [a, b], {}, [0, 1])


@pytest.mark.parametrize("op,lo", [("neg", None), ("identity", None), ("exp", None), ("log", 0.3), ("sqrt", 0.3),
                                   ("square", None), ("abs", 0.1), ("relu", None), ("sigmoid", None),
                                   ("tanh", None), ("softplus", None), ("elu", None), ("gelu", None),
                                   ("softmax", None)])
def test_unary_grad(op, lo):
    x = _r(3, 5, seed=3, lo=lo)
    if op in ("relu", "elu"):
        x = torch.where(x.abs() < 1e-3, x + 0.01, x)     # keep away from the kink
    _fd_check(op, [x], {}, [0])


def test_param_unary_grads():
    _fd_check("pow", [_r(3, 4, lo=0.2)], {"p": 2.5}, [0])
    _fd_check("leakyRelu", [_r(3, 4, seed=5)], {"alpha": 0.2}, [0])
    _fd_check("activation", [_r(3, 4, seed=6)], {"act": "SWISH"}, [0])
    _fd_check("activation", [_r(3, 4, seed=7)], {"act": "SOFTSIGN"}, [0])


def test_linear_algebra_grads():
    _fd_check("mmul", [_r(3, 4, seed=1), _r(4, 5, seed=2)], {}, [0, 1])
    _fd_check("mmul", [_r(2, 3, 4, seed=1), _r(2, 4, 5, seed=2)], {}, [0, 1])
    _fd_check("linear", [_r(3, 4, seed=1), _r(4, 5, seed=2), _r(5, seed=3)], {}, [0, 1, 2])
    _fd_check("linear", [_r(2, 3, 4, seed=1), _r(4, 5, seed=2), _r(1, 5, seed=3)], {}, [0, 1, 2])


def test_shape_and_reduction_grads():
    x = _r(2, 3, 4)
    _fd_check("sum", [x], {"dims": [1]}, [0])
    _fd_check("sum", [x], {"dims": []}, [0])
    _fd_check("mean", [x], {"dims": [0, 2]}, [0])
    _fd_check("reshape", [x], {"shape": [6, 4]}, [0])
    _fd_check("permute", [x], {"dims": [2, 0, 1]}, [0])
    _fd_check("transpose", [x], {}, [0])
    _fd_check("get", [x], {"idx": [{"slice": [None, None, None]}, 0]}, [0])
    _fd_check("get", [x], {"idx": [1, {"slice": [0, 2, None]}]}, [0])
    _fd_check("concat", [_r(2, 3, seed=1), _r(2, 2, seed=2)], {"dim": 1}, [0, 1])
    idx = torch.tensor([[0, 2], [2, 1]])
    _fd_check("gather", [_r(4, 3), idx], {"axis": 0}, [0])


def test_nn_block_grads():
    x = _r(4, 6, seed=1)
    _fd_check("layerNorm", [x, _r(6, seed=2), _r(6, seed=3)], {"eps": 1e-5}, [0, 1, 2])
    qkv = _r(2, 5, 12, seed=4)
    _fd_check("fusedSelfAttention", [qkv, None], {"nHeads": 2}, [0])
    _fd_check("fusedSelfAttention", [qkv, None], {"nHeads": 2, "causal": True}, [0])
    mask = torch.tensor([[1, 1, 1, 0, 0], [1, 1, 1, 1, 1]], dtype=D)
    _fd_check("fusedSelfAttention", [qkv, mask], {"nHeads": 4}, [0])


def test_conv_pool_grads():
    x = _r(2, 3, 6, 6, seed=1)
    w = _r(4, 3, 3, 3, seed=2)
    b = _r(4, seed=3)
    _fd_check("conv2d", [x, w, b], {"stride": [1, 1], "padding": [1, 1]}, [0, 1, 2])
    _fd_check("conv2d", [x, w, None], {"stride": [2, 2], "padding": [0, 0]}, [0, 1])
    _fd_check("maxPooling2d", [x], {"kernel": [2, 2], "stride": [2, 2]}, [0])
    _fd_check("avgPooling2d", [x], {"kernel": [3, 3], "stride": [1, 1], "padding": [1, 1]}, [0])


@pytest.mark.parametrize("peephole", [False, True])
def test_lstm_grads(peephole):
    mb, nIn, T, H = 2, 3, 4, 3
    x = _r(mb, nIn, T, seed=1)
    W = _r(nIn, 4 * H, seed=2) * 0.5
    RW = _r(H, 4 * H + (3 if peephole else 0), seed=3) * 0.5
    b = _r(1, 4 * H, seed=4) * 0.1
    h0, c0 = _r(mb, H, seed=5) * 0.3, _r(mb, H, seed=6) * 0.3
    _fd_check("lstmLayer", [x, W, RW, b, h0, c0], {"peephole": peephole}, [0, 1, 2, 3, 4, 5])
    _fd_check("lstmLayer", [x, W, RW, b, None, None], {"peephole": peephole}, [0, 2])
    # two stacked layers as one fused op (the planner's lstmLayer -> lstmLayer fusion; CPU: the paired path)
    W2 = _r(H, 4 * H, seed=7) * 0.5
    RW2 = _r(H, 4 * H + (3 if peephole else 0), seed=8) * 0.5
    b2 = _r(1, 4 * H, seed=9) * 0.1
    _fd_check("lstmStack2", [x, W, RW, b, W2, RW2, b2], {"peephole": peephole}, [0, 1, 2, 3, 4, 5, 6])


def test_lstm_stack_fusion_planned_and_equal():
    """sd.rnn().lstmLayer twice in a row is planned as one lstmStack2 record with the same loss and gradients."""
    from deeplearning4j_amd.samediff import SameDiff
    mb, nIn, T, H = 2, 3, 5, 4
    vals = {"W0": _r(nIn, 4 * H, seed=2) * 0.5, "RW0": _r(H, 4 * H + 3, seed=3) * 0.5, "b0": _r(4 * H, seed=4) * 0.1,
            "W1": _r(H, 4 * H, seed=5) * 0.5, "RW1": _r(H, 4 * H + 3, seed=6) * 0.5, "b1": _r(4 * H, seed=7) * 0.1}
    res = []
    for fusion in (True, False):
        sd = SameDiff.create()
        sd.fusion = fusion
        h = sd.placeHolder("x", _r(mb, nIn, T, seed=1))
        for i in range(2):
            h = sd.rnn().lstmLayer(f"l{i}", h, sd.var(f"W{i}", vals[f"W{i}"].clone()),
                                   sd.var(f"RW{i}", vals[f"RW{i}"].clone()), sd.var(f"b{i}", vals[f"b{i}"].clone()),
                                   peephole=True)
        loss = h.mul(h).sum()
        ops = [r[1] for r in sd._plan([loss.name])]
        assert ("lstmStack2" in ops) == fusion and (ops.count("lstmLayer") == (0 if fusion else 2))
        res.append(sd.execBackwards(loss))
    for k in vals:
        torch.testing.assert_close(res[0][k], res[1][k], rtol=1e-10, atol=1e-12)


def test_loss_grads():
    logits = _r(4, 5, seed=1)
    lab = torch.nn.functional.one_hot(torch.tensor([0, 3, 1, 4]), 5).to(D)
    _fd_check("softmaxCrossEntropy", [lab, logits], {}, [1])
    _fd_check("softmaxCrossEntropy", [lab, logits], {"labelSmoothing": 0.1}, [1])
    _fd_check("meanSquaredError", [_r(3, 4, seed=2), _r(3, 4, seed=3)], {}, [1])
    p = torch.sigmoid(_r(3, 4, seed=4))
    _fd_check("logLoss", [(torch.rand(3, 4, generator=torch.Generator().manual_seed(1)) > 0.5).to(D), p], {}, [1])


def test_every_registered_op_is_gradient_checked():
    src = pathlib.Path(__file__).read_text()
    missing = [n for n in REGISTRY if f'"{n}"' not in src]
    assert not missing, missing


def test_samediff_package_never_uses_torch_autograd():
    pkg = pathlib.Path(__file__).resolve().parents[1] / "deeplearning4j_amd" / "samediff"
    for f in pkg.glob("*.py"):
        text = f.read_text()
        assert "torch.autograd." not in text and "requires_grad" not in text and ".backward(" not in text, f.name


def _mlp(seed=0):
    g = torch.Generator().manual_seed(seed)
    sd = SameDiff.create()
    x = sd.placeHolder("x", torch.randn(5, 4, generator=g, dtype=D))
    y = sd.placeHolder("y", torch.nn.functional.one_hot(torch.tensor([0, 1, 2, 1, 0]), 3).to(D))
    w0 = sd.var("w0", torch.randn(4, 6, generator=g, dtype=D) * 0.5)
    b0 = sd.var("b0", torch.zeros(1, 6, dtype=D))
    w1 = sd.var("w1", torch.randn(6, 3, generator=g, dtype=D) * 0.5)
    gam = sd.var("gam", torch.ones(6, dtype=D) + 0.1 * torch.randn(6, generator=g, dtype=D))
    bet = sd.var("bet", torch.zeros(6, dtype=D))
    h = sd.nn().tanh(sd.nn().linear(x, w0, b0))
    h = sd.nn().layerNorm(h, gam, bet)
    h = h * 0.5 + h.pow(2.0).mul(0.1)
    logits = h.mmul(w1)
    loss = sd.loss().softmaxCrossEntropy("loss", y, logits)
    return sd, loss


def test_graph_gradient_check_fp64():
    sd, loss = _mlp()
    grads = sd.execBackwards(loss)
    eps = 1e-6
    for v in sd.trainableVariables():
        arr = v.value.reshape(-1)
        for j in range(arr.numel()):
            old = arr[j].item()
            arr[j] = old + eps
            fp = float(sd.output({}, "loss")["loss"])
            arr[j] = old - eps
            fm = float(sd.output({}, "loss")["loss"])
            arr[j] = old
            assert abs(grads[v.name].reshape(-1)[j].item() - (fp - fm) / (2 * eps)) < 1e-7, (v.name, j)
        assert torch.equal(v.gradient(), grads[v.name])


def test_shared_variable_gradients_accumulate():
    sd = SameDiff.create()
    w = sd.var("w", torch.tensor([1.5, -2.0], dtype=D))
    out = (w * w).add(w).sum()                       # d/dw = 2w + 1 (w used three times)
    g = sd.execBackwards(out)["w"]
    torch.testing.assert_close(g, 2 * w.value + 1)


def test_fit_trains_and_save_load_roundtrip(tmp_path):
    from deeplearning4j_amd.datasets.dataset import DataSet
    from deeplearning4j_amd.nn.conf.updaters import Adam
    sd, loss = _mlp(seed=3)
    x = sd.getVariable("x").value.clone()
    y = sd.getVariable("y").value.clone()
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(0.05)).dataSetFeatureMapping("x")
                         .dataSetLabelMapping("y").build())
    ds = DataSet(x, y)
    first = sd.fit(ds)
    for _ in range(40):
        last = sd.fit(ds)
    assert last < first * 0.5
    p = tmp_path / "g.sdz"
    sd.save(str(p))
    sd2 = SameDiff.load(str(p))
    assert [r[:2] for r in sd2.ops()] == [r[:2] for r in sd.ops()]
    o1 = sd.output({"x": x, "y": y}, "loss")["loss"]
    o2 = sd2.output({"x": x, "y": y}, "loss")["loss"]
    torch.testing.assert_close(o1, o2)
    g1, g2 = sd.execBackwards(loss), sd2.execBackwards(sd2.getVariable("loss"))
    for k in g1:
        torch.testing.assert_close(g1[k], g2[k])


def test_fused_forms_grads():
    """The fused records the planner emits: linear with the GELU epilogue, LayerNorm with a residual input."""
    _fd_check("linear", [_r(2, 3, 4, seed=1), _r(4, 5, seed=2), _r(5, seed=3)], {"act": "gelu"}, [0, 1, 2])
    _fd_check("layerNorm", [_r(4, 6, seed=1), _r(6, seed=2), _r(6, seed=3), _r(4, 6, seed=4)], {"eps": 1e-5},
              [0, 1, 2, 3])


def _block(fusion):
    g = torch.Generator().manual_seed(7)
    sd = SameDiff.create()
    sd.fusion = fusion
    x = sd.placeHolder("x", torch.randn(3, 5, 8, generator=g, dtype=D))
    w1 = sd.var("w1", torch.randn(8, 16, generator=g, dtype=D) * 0.3)
    b1 = sd.var("b1", torch.randn(16, generator=g, dtype=D) * 0.1)
    w2 = sd.var("w2", torch.randn(16, 8, generator=g, dtype=D) * 0.3)
    gam = sd.var("g", torch.ones(8, dtype=D))
    bet = sd.var("b", torch.zeros(8, dtype=D))
    h = sd.nn().gelu(sd.nn().linear(x, w1, b1))
    y = sd.nn().layerNorm(h.mmul(w2).add(x), gam, bet)
    loss = y.mul(y).sum()
    return sd, loss


def test_fusion_pass_is_exact_and_fuses():
    sd0, l0 = _block(False)
    sd1, l1 = _block(True)
    g0, g1 = sd0.execBackwards(l0), sd1.execBackwards(l1)
    ops = [r[1] for r in sd1._plan([l1.name])]
    assert "gelu" not in ops and "add" not in ops, ops
    for k in g0:
        torch.testing.assert_close(g0[k], g1[k])
    x = torch.randn(3, 5, 8, dtype=D)
    torch.testing.assert_close(sd0.output({"x": x}, l0)[l0.name], sd1.output({"x": x}, l1)[l1.name])
