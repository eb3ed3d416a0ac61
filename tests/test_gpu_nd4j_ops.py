"""ND4J op-surface kernels (csrc/nd4j_ops.hip, ops/nd4j_kernels.py) against plain fp32 torch references, and the
framework paths wired to them (activations, INDArray arithmetic / reductions / Transforms, shape-only layers,
ElementWiseVertex Max). Runs on MI355X."""
import pytest
import torch

from deeplearning4j_amd.ops import nd4j_kernels as K

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16, torch.float16]
TOL = {torch.float32: 1e-5, torch.bfloat16: 2e-2, torch.float16: 2e-3}


def _close(got, want, dt, scale_floor=1.0):
    err = (got.float() - want.float()).abs().max().item()
    scale = max(want.float().abs().max().item(), scale_floor)
    assert err <= TOL[dt] * scale * 4, (err, scale)


UNARY_REF = {
    "identity": lambda x: x, "relu": torch.relu, "relu6": lambda x: x.clamp(0, 6),
    "leakyrelu": lambda x: torch.nn.functional.leaky_relu(x, 0.1), "elu": lambda x: torch.nn.functional.elu(x, 0.7),
    "selu": torch.selu, "sigmoid": torch.sigmoid, "hardsigmoid": lambda x: (0.2 * x + 0.5).clamp(0, 1),
    "tanh": torch.tanh, "hardtanh": lambda x: x.clamp(-1, 1), "rectifiedtanh": lambda x: torch.tanh(x).clamp(min=0),
    "softplus": torch.nn.functional.softplus, "softsign": lambda x: x / (1 + x.abs()), "cube": lambda x: x ** 3,
    "swish": lambda x: x * torch.sigmoid(x), "gelu_tanh": lambda x: torch.nn.functional.gelu(x, approximate="tanh"),
    "gelu": torch.nn.functional.gelu, "exp": torch.exp, "abs": torch.abs, "neg": torch.neg,
    "square": lambda x: x * x, "sign": torch.sign, "floor": torch.floor, "ceil": torch.ceil, "sin": torch.sin,
    "cos": torch.cos, "clip": lambda x: x.clamp(-0.5, 0.25), "step": lambda x: (x > 0.1).float(),
    "add_s": lambda x: x + 0.1, "mul_s": lambda x: x * 0.1, "rsub_s": lambda x: 0.1 - x, "max_s": lambda x: x.clamp(min=0.1),
    "min_s": lambda x: x.clamp(max=0.1), "atan": torch.atan, "sinh": torch.sinh, "erf": torch.erf,
    "expm1": torch.expm1, "sub_s": lambda x: x - 0.1,
}
A0 = {"leakyrelu": 0.1, "elu": 0.7, "clip": -0.5, "step": 0.1, "add_s": 0.1, "mul_s": 0.1, "rsub_s": 0.1,
      "max_s": 0.1, "min_s": 0.1, "sub_s": 0.1}


@pytest.mark.parametrize("dt", DTYPES)
def test_transforms_match_torch(cuda, dt):
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(3, 5, 7, 9, generator=g) * 2).to(cuda).to(dt)
    for op, ref in UNARY_REF.items():
        y = K.transform(x, op, A0.get(op, 0.0), 0.25 if op == "clip" else 0.0)
        _close(y, ref(x.float()), dt)
    pos = x.float().abs().to(dt) + 0.5
    for op, ref in {"log": torch.log, "sqrt": torch.sqrt, "reciprocal": torch.reciprocal, "rsqrt": torch.rsqrt,
                    "log1p": torch.log1p}.items():
        _close(K.transform(pos, op), ref(pos.float()), dt)
    # channels-last input keeps its layout
    xc = x.contiguous(memory_format=torch.channels_last)
    yc = K.transform(xc, "tanh")
    assert yc.is_contiguous(memory_format=torch.channels_last)
    _close(yc, torch.tanh(x.float()), dt)


@pytest.mark.parametrize("dt", DTYPES)
def test_activation_derivatives_match_autograd(cuda, dt):
    g = torch.Generator().manual_seed(1)
    z = (torch.randn(4, 33, generator=g) * 2).to(cuda).to(dt)
    e = torch.randn(4, 33, generator=g).to(cuda).to(dt)
    for op in ["identity", "relu", "relu6", "leakyrelu", "elu", "selu", "sigmoid", "tanh", "softplus", "softsign",
               "cube", "swish", "gelu_tanh", "gelu", "rectifiedtanh"]:
        zr = z.float().clone().requires_grad_(True)
        (gref,) = torch.autograd.grad(UNARY_REF[op](zr), zr, e.float())
        _close(K.transform_bp(z, e, op, A0.get(op, 0.0)), gref, dt)


@pytest.mark.parametrize("dt", DTYPES)
def test_broadcast_binary(cuda, dt):
    g = torch.Generator().manual_seed(2)
    shapes = [((4, 5, 6), (4, 5, 6)), ((4, 5, 6), (1, 5, 1)), ((4, 1, 6), (5, 1)), ((2, 3, 4, 5), (5,)),
              ((7, 1), (1, 9)), ((3, 8), ())]
    refs = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div, "rsub": lambda a, b: b - a,
            "rdiv": lambda a, b: b / a, "max": torch.maximum, "min": torch.minimum, "sqdiff": lambda a, b: (a - b) ** 2,
            "gt": lambda a, b: (a > b).float(), "eq": lambda a, b: (a == b).float(), "atan2": torch.atan2}
    for sa, sb in shapes:
        a = torch.randn(sa, generator=g).to(cuda).to(dt)
        b = (torch.randn(sb, generator=g).abs() + 0.5).to(cuda).to(dt)
        for op, ref in refs.items():
            _close(K.binary(a, b, op), ref(a.float(), b.float()), dt)
    a = torch.randn(6, 7, generator=g).to(cuda).to(dt)
    _close(K.binary(a, 2.5, "mul"), a.float() * 2.5, dt)
    # transposed (non-contiguous) operand through the strided path
    bt = torch.randn(7, 6, generator=g).to(cuda).to(dt).t()
    _close(K.binary(a, bt, "add"), a.float() + bt.float(), dt)


@pytest.mark.parametrize("dt", DTYPES)
def test_reductions(cuda, dt):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(6, 70, 9, 5, generator=g).to(cuda).to(dt)
    xf = x.float()
    cases = [None, [0], [1], [3], [1, 2], [0, 3], [0, 2, 3]]
    for dims in cases:
        d = tuple(range(4)) if dims is None else tuple(dims)
        for op, ref in {"sum": lambda t: t.sum(d), "mean": lambda t: t.mean(d), "max": lambda t: t.amax(d),
                        "min": lambda t: t.amin(d), "norm1": lambda t: t.abs().sum(d),
                        "norm2": lambda t: t.pow(2).sum(d).sqrt(), "amax": lambda t: t.abs().amax(d),
                        "var": lambda t: t.var(d, correction=1), "std": lambda t: t.std(d, correction=0),
                        "logsumexp": lambda t: torch.logsumexp(t, d)}.items():
            r = K.reduce(x, op, dims, bias_corrected=(op != "std"))
            _close(r, ref(xf), dt)
    # large reduction (segmented path) is bitwise reproducible
    big = torch.randn(1 << 22, generator=g).to(cuda).to(dt)
    r1, r2 = K.reduce(big, "sum"), K.reduce(big, "sum")
    assert torch.equal(r1, r2)
    _close(r1, big.float().sum(), dt, scale_floor=big.float().abs().sum().item() ** 0.5)
    # argmax / argmin with the first index on ties (ND4J IndexReduce semantics)
    t = torch.zeros(3, 40, device=cuda, dtype=dt)
    t[:, 5] = 2
    t[:, 17] = 2
    assert K.reduce(t, "argmax", [1]).tolist() == [5, 5, 5]
    assert K.reduce(-t, "argmin", [1]).tolist() == [5, 5, 5]
    m = torch.randn(50, 33, generator=g).to(cuda).to(dt)
    assert torch.equal(K.reduce(m, "argmax", [0]).cpu(), m.float().argmax(0).cpu())


@pytest.mark.parametrize("dt", DTYPES)
def test_data_movement(cuda, dt):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 3, 8, 12, generator=g).to(cuda).to(dt)
    assert torch.equal(K.reverse(x, [1, 3]), torch.flip(x, [1, 3]))
    assert torch.equal(K.materialize(x.permute(0, 2, 3, 1)), x.permute(0, 2, 3, 1).contiguous())
    s2d = K.space_to_depth(x, 2)
    ref = x.reshape(2, 3, 4, 2, 6, 2).permute(0, 3, 5, 1, 2, 4).reshape(2, 12, 4, 6)
    assert torch.equal(s2d, ref)
    assert torch.equal(K.depth_to_space(s2d, 2), x)
    up = K.upsample_nearest2d(x, 2, 3)
    assert torch.equal(up, x.repeat_interleave(2, 2).repeat_interleave(3, 3))
    e = torch.randn(up.shape, generator=g).to(cuda).to(dt)
    _close(K.upsample_nearest2d_bp(e, 2, 3), e.float().reshape(2, 3, 8, 2, 12, 3).sum((3, 5)), dt)
    p = K.pad2d(x, (1, 2, 0, 3))
    assert torch.equal(p, torch.nn.functional.pad(x, (0, 3, 1, 2)))
    sb = K.space_to_batch(x, (2, 2), ((1, 1), (0, 2)))
    xp = torch.nn.functional.pad(x, (0, 2, 1, 1))
    refb = xp.reshape(2, 3, 5, 2, 7, 2).permute(3, 5, 0, 1, 2, 4).reshape(8, 3, 5, 7)
    assert torch.equal(sb, refb)
    assert torch.equal(K.batch_to_space(sb, (2, 2), ((1, 1), (0, 2))), x)


def test_mergemax(cuda):
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(4, 9, generator=g).to(cuda) for _ in range(3)]
    y, am = K.mergemax(xs)
    st = torch.stack(xs)
    assert torch.equal(y, st.max(0).values)
    e = torch.randn(4, 9, generator=g).to(cuda)
    gs = K.mergemax_bp(e, am, 3)
    for i in range(3):
        assert torch.equal(gs[i], e * (st.argmax(0) == i).float())


def test_framework_paths_use_the_kernels(cuda):
    from deeplearning4j_amd import Activation
    from deeplearning4j_amd.nd4j.ndarray import INDArray, Transforms
    K.CALLS.clear()
    g = torch.Generator().manual_seed(6)
    xc = torch.randn(5, 7, generator=g)
    ga, ca = INDArray(xc.to(cuda)), INDArray(xc.clone())
    v = torch.randn(7, generator=g)
    assert torch.allclose(ga.addRowVector(INDArray(v.to(cuda))).toTensor().cpu(), ca.addRowVector(INDArray(v)).toTensor())
    assert torch.allclose(ga.sum(1).toTensor().cpu(), ca.sum(1).toTensor(), atol=1e-5)
    assert torch.allclose(ga.std(0).toTensor().cpu(), ca.std(0).toTensor(), atol=1e-5)
    assert ga.argMax(1).toTensor().cpu().tolist() == ca.argMax(1).toTensor().tolist()
    assert torch.allclose(Transforms.sigmoid(ga).toTensor().cpu(), Transforms.sigmoid(ca).toTensor(), atol=1e-6)
    for act in [Activation.RELU, Activation.TANH, Activation.ELU, Activation.SWISH, Activation.SOFTSIGN]:
        f = act.getActivationFunction()
        assert torch.allclose(f.getActivation(xc.to(cuda)).cpu(), f.getActivation(xc), atol=1e-6)
        e = torch.randn(5, 7, generator=g)
        assert torch.allclose(f.backprop(xc.to(cuda), e.to(cuda)).cpu(), f.backprop(xc, e), atol=1e-6)
    assert K.CALLS["binary"] >= 1 and K.CALLS["reduce"] >= 3 and K.CALLS["transform"] >= 6
    assert K.CALLS["transform_bp"] >= 5


def test_inplace_ops_with_overlapping_operands(cuda):
    """In-place ops whose operand is another view of the same array: the result equals the CPU one
    (the operand is read from a copy), not an order-dependent race inside the kernel."""
    from deeplearning4j_amd.nd4j.ndarray import INDArray
    g = torch.Generator().manual_seed(8)
    xc = torch.randn(64, 64, generator=g)
    ga, ca = INDArray(xc.to(cuda)), INDArray(xc.clone())
    ga.subiRowVector(ga.getRow(0))
    ca.subiRowVector(ca.getRow(0))
    assert torch.equal(ga.toTensor().cpu(), ca.toTensor())
    gb, cb = INDArray(xc.to(cuda)), INDArray(xc.clone())
    gb.addi(gb.transpose())
    cb.addi(cb.transpose())
    assert torch.allclose(gb.toTensor().cpu(), cb.toTensor(), atol=0, rtol=0)


def test_shape_layers_and_max_vertex_on_gpu(cuda):
    from deeplearning4j_amd.nn.conf import layers as L
    from deeplearning4j_amd.nn.conf.graph import ElementWiseVertex
    from deeplearning4j_amd.nn.layers.convolution import SpaceToBatchImpl, SpaceToDepthImpl, Upsampling2DImpl
    K.CALLS.clear()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 4, 6, 8, generator=g)
    for impl in (Upsampling2DImpl(L.Upsampling2D(size=[2, 3])), SpaceToDepthImpl(L.SpaceToDepthLayer(blockSize=2)),
                 SpaceToBatchImpl(L.SpaceToBatchLayer(blocks=[2, 2], padding=[[1, 1], [0, 2]]))):
        yc = impl.activate(x)
        yg = impl.activate(x.to(cuda))
        assert torch.equal(yg.cpu(), yc)
        e = torch.randn(yc.shape, generator=g)
        _, gc = impl.backpropGradient(e)
        impl.activate(x.to(cuda))
        _, gg = impl.backpropGradient(e.to(cuda))
        assert torch.allclose(gg.cpu(), gc, atol=1e-5)
    v = ElementWiseVertex(op="Max")
    xs = [torch.randn(3, 5, generator=g) for _ in range(3)]
    out, ctx = v.forward([t.to(cuda) for t in xs], True) if hasattr(v, "forward") else (None, None)
    if out is not None:
        assert torch.equal(out.cpu(), torch.stack(xs).max(0).values)
        grads = v.backward(torch.ones(3, 5, device=cuda), ctx)
        assert torch.equal(sum(gr.cpu() for gr in grads), torch.ones(3, 5))
    assert K.CALLS["strided_copy"] >= 4


@pytest.mark.parametrize("case", [((2, 3, 9, 11), (4, 3, 3, 3), (1, 1), (1, 1, 1, 1), (1, 1)),
                                  ((2, 5, 12, 10), (6, 5, 5, 3), (2, 1), (2, 1, 0, 2), (1, 2)),
                                  ((1, 4, 8, 8), (3, 4, 1, 1), (2, 2), (0, 0, 0, 0), (1, 1)),
                                  ((64, 20, 12, 12), (50, 20, 5, 5), (1, 1), (0, 0, 0, 0), (1, 1))])
@pytest.mark.parametrize("channels_last", [False, True])
def test_fp32_conv_im2col_col2im_kernels(cuda, case, channels_last):
    """fp32 conv forward / backward on the in-tree row-per-pixel im2col (padding in the same launch) and gather
    col2im kernels + one fp32 MFMA GEMM per product, against torch's fp32 conv, with the kernels' launch counters
    advancing (no ATen unfold / fold). The last case is LeNet's second conv at batch 64."""
    from deeplearning4j_amd.ops import conv as C
    xs, ws, st, pad4, dil = case
    g = torch.Generator().manual_seed(9)
    x = torch.randn(xs, generator=g).to(cuda)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn(ws, generator=g).to(cuda) * 0.2
    b = torch.randn(ws[0], generator=g).to(cuda)
    K.CALLS.clear()
    y = C._fp32_conv_fwd(x, w, b, st, pad4, dil)
    # fp64 reference on the CPU (no library conv on the GPU in this test)
    xr = torch.nn.functional.pad(x.cpu().double(), (pad4[2], pad4[3], pad4[0], pad4[1])).requires_grad_(True)
    wr = w.cpu().double().requires_grad_(True)
    br = b.cpu().double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, br, st, 0, dil)
    assert torch.allclose(y.cpu().double(), yr.detach(), atol=1e-4, rtol=1e-4)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    dy = dy.to(cuda)
    if channels_last:
        dy = dy.contiguous(memory_format=torch.channels_last)
    dx, dw, db = C._fp32_conv_bwd(x, w, dy, st, pad4, dil, True, True, True)
    H, W = xs[2], xs[3]
    assert torch.allclose(dx.cpu().double(), xr.grad[:, :, pad4[0]:pad4[0] + H, pad4[2]:pad4[2] + W], atol=1e-4,
                          rtol=1e-4)
    assert torch.allclose(dw.cpu().double(), wr.grad, atol=1e-3, rtol=1e-4)
    assert torch.allclose(db.cpu().double(), br.grad, atol=1e-4, rtol=1e-4)
    assert K.CALLS["im2col_rows"] == 2 and K.CALLS["col2im_rows"] == 1
