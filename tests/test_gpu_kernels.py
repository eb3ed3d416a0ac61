"""HIP kernel numerics vs the plain-torch fp32 reference of the same op (run on a real MI355X).

Reference-vs-helper parity is the reference's own strategy for its cuDNN helpers
(CUDAT:convolution/TestConvolution.java:72-147, CUDAT:lstm/ValidateCudnnLSTM.java:32-246)."""
import pytest
import torch

from deeplearning4j_amd import ops
from deeplearning4j_amd.ops import native

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"max abs err {err} (scale {scale})"


def test_native_library_loaded(cuda):
    assert ops.native_lib() is not None
    assert ops.use_native(torch.zeros(1, device=cuda), "bn")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("shape", [(4, 64, 9, 7), (2, 256, 5, 5), (3, 2048, 2, 2), (16, 24),
                                   # grid-capped sizes: several grid-stride steps (register-resident factors,
                                   # two vectors per step + tail) and an odd channel-group count (factors reloaded)
                                   (200, 64, 32, 32), (500000, 24),
                                   # several channel columns x several folded partial rows: ticketed fold
                                   (64, 256, 16, 16)])
def test_batchnorm_fwd_bwd(cuda, dtype, relu, shape):
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(*shape, generator=g) * 3 + 1.5)
    C = shape[1]
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    dy = torch.randn(*shape, generator=g)
    rm_c, rv_c = torch.zeros(C), torch.ones(C)
    xr = x.to(dtype)
    y_ref, ctx_ref = ops.bn_forward(xr.float(), gamma, beta, rm_c, rv_c, True, 0.9, 1e-5, relu)
    dx_ref, dg_ref, db_ref, _ = ops.bn_backward(dy.to(dtype).float(), ctx_ref)
    xd = xr.to(cuda)
    if xd.dim() == 4:
        xd = xd.contiguous(memory_format=torch.channels_last)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, ctx = ops.bn_forward(xd, gamma.to(cuda), beta.to(cuda), rm, rv, True, 0.9, 1e-5, relu)
    assert ctx[0] == "NATIVE"
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, y_ref, tol)
    _close(rm, rm_c, 1e-4)
    _close(rv, rv_c, 1e-4)
    dyd = dy.to(dtype).to(cuda)
    if dyd.dim() == 4:
        dyd = dyd.contiguous(memory_format=torch.channels_last)
    dx, dgm, dbt, _ = ops.bn_backward(dyd, ctx)
    _close(dx, dx_ref, tol * 2)
    _close(dgm, dg_ref, 1e-3 if dtype == torch.float32 else 3e-2)
    _close(dbt, db_ref, 1e-3 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ptype", ["MAX", "AVG"])
@pytest.mark.parametrize("geom", [((3, 3), (2, 2), (0, 0, 0, 0)), ((2, 2), (2, 2), (0, 0, 0, 0)),
                                  ((3, 3), (1, 1), (1, 1, 1, 1)), ((3, 3), (2, 2), (0, 1, 0, 1))])
def test_pool(cuda, dtype, ptype, geom):
    k, s, p = geom
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 16, 11, 9, generator=g).to(dtype)
    y_ref, ctx_ref = ops.pool2d_forward(x.float(), ptype, k, s, p)
    xd = x.to(cuda).contiguous(memory_format=torch.channels_last)
    y, ctx = ops.pool2d_forward(xd, ptype, k, s, p)
    assert ctx[0] == "NATIVE"
    _close(y, y_ref, 1e-6 if dtype == torch.float32 else 1e-2)
    dy = torch.randn(y_ref.shape, generator=g).to(dtype)
    dx_ref = ops.pool2d_backward(dy.float(), ctx_ref)
    dx = ops.pool2d_backward(dy.to(cuda).contiguous(memory_format=torch.channels_last), ctx)
    _close(dx, dx_ref, 1e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_softmax_xent(cuda, dtype):
    g = torch.Generator().manual_seed(2)
    z = (torch.randn(37, 1000, generator=g) * 4).to(dtype)
    y = torch.zeros(37, 1000)
    y[torch.arange(37), torch.randint(0, 1000, (37,), generator=g)] = 1
    s_ref, g_ref, _ = ops.softmax_xent(z.float(), y, None, 1e-10)
    s, gr, _ = ops.softmax_xent(z.to(cuda), y.to(cuda), None, 1e-10)
    _close(s, s_ref, 1e-4)
    _close(gr, g_ref, 1e-5 if dtype == torch.float32 else 1e-2)
    # per-row mask (RNN output time steps) on the kernel: no fallback, rows scaled
    from deeplearning4j_amd.ops import fallback
    m = (torch.rand(37, 1, generator=g) > 0.3).float()
    s_ref, g_ref, _ = ops.softmax_xent(z.float(), y, m, 1e-10)
    n0 = fallback.count()
    s, gr, _ = ops.softmax_xent(z.to(cuda), y.to(cuda), m.to(cuda), 1e-10)
    assert fallback.count() == n0
    _close(s, s_ref, 1e-4)
    _close(gr, g_ref, 1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("upd", ["Sgd", "Nesterovs", "Adam", "AdaMax", "Nadam", "AdaGrad", "AdaDelta", "RmsProp",
                                 "NoOp"])
def test_fused_updater_matches_reference(cuda, upd):
    from deeplearning4j_amd.nn.conf import updaters as U
    from deeplearning4j_amd.ops.update import Segment, UpdatePlan, fused_update
    u = getattr(U, upd)()
    n1, n2 = 1000, 3001
    nb = n1 + n2
    segs = [Segment(0, n1, 0, 0, nb, u, 0.01, 0.0, 0), Segment(n1, n2, 0, n1, nb, u, 0.0, 0.02, 0)]
    plan = UpdatePlan(segs, [(0, nb, 0, u)])
    g = torch.Generator().manual_seed(3)
    p = torch.randn(nb, generator=g)
    st = torch.rand(u.stateSize(nb), generator=g)
    for it in range(3):
        gr = torch.randn(nb, generator=g)
        pc, gc, sc = p.clone(), gr.clone(), st.clone()
        fused_update(plan, pc, gc, sc, it, 0, 8)
        pd, gd, sd = p.to(cuda), gr.to(cuda), st.to(cuda)
        shadow = torch.empty(nb, dtype=torch.bfloat16, device=cuda)
        fused_update(plan, pd, gd, sd, it, 0, 8, shadow=shadow)
        _close(pd, pc, 1e-5)
        _close(gd, gc, 1e-5)
        if sc.numel():
            _close(sd, sc, 1e-5)
        _close(shadow, pc, 1e-2)
        p, st = pc, sc


def test_resnet50_step_bf16(cuda):
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    net = ResNet50(numLabels=10, dataType=DataType.BFLOAT16).init(device=cuda)
    x = torch.rand(4, 3, 224, 224, device=cuda)
    y = torch.zeros(4, 10, device=cuda)
    y[torch.arange(4), torch.tensor([1, 2, 3, 4])] = 1
    s = []
    for _ in range(3):
        net.fit([x], [y])
        s.append(net.score())
    assert all(v == v for v in s)
    assert net.shadow is not None and net.shadow.dtype == torch.bfloat16
    p = net.flattenedParams
    assert ((net.shadow.float() - p).abs() <= 1e-2 * p.abs() + 1e-3).all()


def test_lenet_gpu_matches_cpu(cuda):
    """Same LeNet, same data: fp32 GPU (native BN-free path: pool + softmax-xent + fused updater) vs CPU."""
    from deeplearning4j_amd.models import LeNet
    g = torch.Generator().manual_seed(5)
    x = torch.rand(16, 1, 28, 28, generator=g)
    y = torch.zeros(16, 10)
    y[torch.arange(16), torch.randint(0, 10, (16,), generator=g)] = 1
    a = LeNet().init(device=torch.device("cpu"))
    b = LeNet().init(device=cuda)
    _close(b.params(), a.params(), 0)
    for _ in range(3):
        a.fit(x.reshape(16, -1), y)
        b.fit(x.reshape(16, -1), y)
    _close(b.params(), a.params(), 2e-3)
    assert abs(a.score() - b.score()) < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 64, 6, 5), (200, 64, 32, 32)])
def test_batchnorm_residual_relu_fused(cuda, dtype, shape):
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(*shape, generator=g) * 2 + 0.5).to(dtype)
    r = torch.randn(*shape, generator=g).to(dtype)
    dy = torch.randn(*shape, generator=g).to(dtype)
    gamma, beta = torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g)
    y_ref, c_ref = ops.bn_forward(x.float(), gamma, beta, torch.zeros(64), torch.ones(64), True, 0.9, 1e-5,
                                  residual=r.float())
    dx_ref, dg_ref, db_ref, dr_ref = ops.bn_backward(dy.float(), c_ref)
    cl = lambda t: t.to(cuda).contiguous(memory_format=torch.channels_last)  # noqa: E731
    y, c = ops.bn_forward(cl(x), gamma.to(cuda), beta.to(cuda), torch.zeros(64, device=cuda),
                          torch.ones(64, device=cuda), True, 0.9, 1e-5, residual=cl(r))
    assert c[0] == "NATIVE"
    dx, dgm, dbt, dr = ops.bn_backward(cl(dy), c)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, y_ref, tol)
    # the kernel recomputes the ReLU pre-activation x*scale+shift+res; among millions of elements a few sit within
    # rounding of 0 and may take the other side of the mask than the reference, so those are left out of dx / dres
    _, xc, mu, istd, gm, bt = c_ref[:6]
    pre = (xc.float() - mu.reshape(1, -1, 1, 1)) * istd.reshape(1, -1, 1, 1) * gm.reshape(1, -1, 1, 1) \
        + bt.reshape(1, -1, 1, 1) + r.float()
    keep = (pre.abs() > 1e-3).float()
    _close(dx.float().cpu() * keep, dx_ref.float() * keep, 2 * tol)
    _close(dr.float().cpu() * keep, dr_ref.float() * keep, tol)
    _close(dgm, dg_ref, 3e-2 if dtype == torch.bfloat16 else 1e-3)
    _close(dbt, db_ref, 3e-2 if dtype == torch.bfloat16 else 1e-3)


@pytest.mark.parametrize("n", [1000, 2048 * 37 + 5, 300000])
def test_threshold_codec_gpu_matches_cpu(cuda, n):
    from deeplearning4j_amd.ops import compression as C
    g = torch.Generator().manual_seed(11)
    r = torch.randn(n, generator=g) * 1e-3
    thr = 1.2e-3
    rc, rg = r.clone(), r.to(cuda)
    assert C.threshold_count(rg, thr) == C.threshold_count(rc, thr)
    mc = C.threshold_encode(rc, thr, capacity=n)
    mg = C.threshold_encode(rg, thr, capacity=n)
    assert torch.equal(mg.cpu(), mc)                    # deterministic, in-order compaction
    assert torch.equal(rg.cpu(), rc)
    dc = C.decode(mc, torch.zeros(n))
    dg = C.decode(mg, torch.zeros(n, device=cuda))
    assert torch.equal(dg.cpu(), dc)
    r2c, r2g = r.clone(), r.to(cuda)
    bc, bg = C.bitmap_encode(r2c, thr), C.bitmap_encode(r2g, thr)
    assert torch.equal(bg.cpu(), bc) and torch.equal(r2g.cpu(), r2c)
    assert torch.equal(C.decode(bg, torch.zeros(n, device=cuda)).cpu(), C.decode(bc, torch.zeros(n)))
    r3 = r.to(cuda)
    m3 = C.threshold_encode(r3, thr, capacity=17)       # capacity clamp keeps the rest in the residual
    assert int(m3[0]) == 17
    assert torch.allclose((C.decode(m3, torch.zeros(n, device=cuda)) + r3).cpu(), r, atol=1e-7)


def test_hip_graph_training_matches_eager(cuda):
    """Captured (HIP graph) training iterations == eager iterations, incl. Adam bias correction per step."""
    from deeplearning4j_amd import (Activation, Adam, BatchNormalization, ConvolutionLayer, DataType, InputType,
                                    LossFunction, MultiLayerNetwork, NeuralNetConfiguration, OutputLayer,
                                    SubsamplingLayer)

    def make():
        conf = (NeuralNetConfiguration.Builder().seed(3).dataType(DataType.BFLOAT16).updater(Adam(1e-2)).l2(1e-4)
                .list()
                .layer(0, ConvolutionLayer.Builder([3, 3]).nOut(16).activation(Activation.IDENTITY).build())
                .layer(1, BatchNormalization.Builder().build())
                .layer(2, SubsamplingLayer.Builder([2, 2], [2, 2]).build())
                .layer(3, OutputLayer.Builder(LossFunction.MCXENT).nOut(10).activation(Activation.SOFTMAX).build())
                .setInputType(InputType.convolutional(12, 12, 8)).build())
        n = MultiLayerNetwork(conf)
        n.init(device=cuda)
        return n
    g = torch.Generator().manual_seed(0)
    xs = [torch.rand(16, 8, 12, 12, generator=g).to(cuda) for _ in range(6)]
    ys = []
    for _ in range(6):
        y = torch.zeros(16, 10)
        y[torch.arange(16), torch.randint(0, 10, (16,), generator=g)] = 1
        ys.append(y.to(cuda))
    eager, graphed = make(), make()
    graphed.enableHipGraphs(True, warmup=1)
    for x, y in zip(xs, ys):
        eager.fit(x, y)
        graphed.fit(x, y)
    assert graphed._hipgraph is not None and graphed._hipgraph.k == 5
    assert graphed.getIterationCount() == eager.getIterationCount() == 6
    assert torch.allclose(graphed.params(), eager.params(), atol=2e-3, rtol=1e-2)
    assert abs(graphed.score() - eager.score()) < 1e-2


@pytest.mark.parametrize("M,C", [(4096, 768), (1000, 3072), (77, 2304), (513, 16)])
def test_channel_sum_wide(cuda, M, C):
    x = torch.randn(M, C, device=cuda).bfloat16()
    out = torch.empty(C, device=cuda)
    r = native.channel_sum(x, out=out)
    assert r is not None and r.data_ptr() == out.data_ptr()
    _close(out, x.float().sum(0), 1e-3)


def test_wrw_overlap_stream_matches_inline(cuda, monkeypatch):
    """Conv weight gradients computed on the overlap stream (ops/side_stream.py) equal the inline (single-stream)
    backward's. Gradients, not a trajectory, are compared: the zoo RmsProp(0.1) step amplifies the fp32 atomic-order
    noise of near-zero gradients into O(lr) parameter differences. (The HIP-graph capture of the overlapped step is
    covered by test_hip_graph_training_matches_eager.)"""
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    from deeplearning4j_amd.ops import side_stream
    g = torch.Generator().manual_seed(3)
    x = torch.rand(8, 3, 224, 224, generator=g).to(cuda)
    y = torch.zeros(8, 10, device=cuda)
    y[torch.arange(8), torch.arange(8) % 10] = 1
    net = ResNet50(numLabels=10, dataType=DataType.BFLOAT16).init(device=cuda)
    grads = {}
    for mode in ("0", "1", "1"):
        monkeypatch.setenv("DL4J_AMD_WRW_STREAM", mode)
        net.computeGradientAndScore([x], [y])
        torch.cuda.synchronize()
        assert not side_stream.active()
        grads.setdefault(mode, []).append(net.flattenedGradients.clone())
    g0 = grads["0"][0]
    scale = g0.abs().max().item()
    for g1 in grads["1"]:
        d = (g0 - g1).abs().max().item()
        assert d <= 2e-3 * scale + 1e-5, (d, scale)


def test_batchnorm_fold_ticket_reuse(cuda):
    """The fused fold+finalize draws its ticket counters round-robin from a fixed device array and the reducing block
    resets them: 600 launches (slots reused twice) must give bitwise the same statistics and gradients."""
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(64, 256, 16, 16, generator=g) + 0.3).to(torch.bfloat16).to(cuda)
    x = x.contiguous(memory_format=torch.channels_last)
    r = torch.randn(64, 256, 16, 16, generator=g).to(torch.bfloat16).to(cuda).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(64, 256, 16, 16, generator=g).to(torch.bfloat16).to(cuda).contiguous(memory_format=torch.channels_last)
    gamma, beta = torch.rand(256, device=cuda) + 0.5, torch.randn(256, device=cuda)
    first = None
    for _ in range(300):
        y, c = ops.bn_forward(x, gamma, beta, torch.zeros(256, device=cuda), torch.ones(256, device=cuda), True, 0.9,
                              1e-5, residual=r)
        dx, dgm, dbt, dr = ops.bn_backward(dy, c)
        cur = (y, dx, dgm, dbt, dr)
        if first is None:
            first = [t.clone() for t in cur]
        else:
            for a, b in zip(first, cur):
                assert torch.equal(a, b)
