"""Which kernels one training step launches (a torch-compute-free step). torch.profiler records
the device kernels of one steady-state ResNet-50 (zoo graph, bf16) training step; every compute kernel must be an
in-tree HIP kernel of libdl4j_amd_kernels.so — no at::native elementwise / reduce / fill / softmax / copy kernels.
Also checks the in-tree fill kernel (nd4j_kernels.fill_) that replaced torch's fills on the step's path."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step_kernels(net, x, y, steps=1, step=None):
    from torch.profiler import ProfilerActivity, profile
    step = step or (lambda: net.fit([x], [y]))
    step()                                 # warm-up: autotuners / kernel-choice database, arena sizing
    step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    out = []
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            out.append((e.name, e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total))
    return out


def _is_torch_kernel(name):
    return "at::native" in name or "at6native" in name or name.startswith("void at::") or "elementwise_kernel" in name


def test_fill_kernel():
    from deeplearning4j_amd.ops import nd4j_kernels as NK
    for dt, v in [(torch.float32, 0.0), (torch.float32, -2.5), (torch.bfloat16, 0.0), (torch.bfloat16, 1.5),
                  (torch.float16, -3.0)]:
        for n in (1, 7, 8, 1000, 12345, 1 << 20):
            base = torch.full((n + 3,), 9.0, device="cuda", dtype=dt)
            t = base[1:n + 1]                                  # unaligned start, ragged tail
            NK.fill_(t, v)
            torch.cuda.synchronize()
            assert torch.all(t == v) and base[0] == 9 and torch.all(base[n + 1:] == 9), (dt, v, n)
    x = torch.ones(4, 8, 5, 5, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    NK.zero_(x)
    assert torch.count_nonzero(x) == 0


def _audit(ks, what):
    assert len(ks) > 20, what
    torch_ks = sorted({n for n, _ in ks if _is_torch_kernel(n)})
    t_all = sum(t for _, t in ks)
    t_torch = sum(t for n, t in ks if _is_torch_kernel(n))
    print(f"{what}: {len(ks)} kernels, {len(torch_ks)} distinct torch kernels, {100 * t_torch / max(t_all, 1):.2f} % "
          f"of time")
    for n in torch_ks:
        print("  torch:", n[:140])
    assert not torch_ks, f"torch compute kernels in the {what} step: {torch_ks[:6]}"


def test_bert_step_launches_no_torch_compute_kernels():
    """BertBase fine-tuning step (tools/bench_bert.py's model; 2 encoder layers, seq 128, bf16)."""
    from deeplearning4j_amd.models import BertBase
    from deeplearning4j_amd.nn.conf import DataType
    net = BertBase(numLabels=2, inputShape=[128], layers=2, dataType=DataType.BFLOAT16).init(device=torch.device("cuda", 0))
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randint(0, 30522, (8, 128), generator=g).cuda()
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (8,), generator=g), 2).float().cuda()
    _audit(_step_kernels(net, x, y), "BERT")


def test_lstm_char_lm_step_launches_no_torch_compute_kernels():
    """TextGenerationLSTM (tools/bench_lstm.py's model, 2x GravesLSTM-256, TBPTT 50, bf16), eager so the profiler sees
    every launch: one fit over two TBPTT windows."""
    from deeplearning4j_amd.models import TextGenerationLSTM
    from deeplearning4j_amd.nn.conf import DataType
    net = TextGenerationLSTM(numLabels=77, inputShape=[1, 77], hidden=256,
                             dataType=DataType.BFLOAT16).init(device=torch.device("cuda", 0))
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, 77, (8, 101), generator=g)
    x = torch.nn.functional.one_hot(idx[:, :-1], 77).permute(0, 2, 1).float().cuda()
    y = torch.nn.functional.one_hot(idx[:, 1:], 77).permute(0, 2, 1).float().cuda()
    _audit(_step_kernels(net, x, y, step=lambda: net.fit(x, y)), "LSTM char-LM")


def test_lenet_fp32_step_launches_no_torch_compute_kernels():
    """The exact-fp32 LeNet step (tools/bench_lenet.py's model: BASELINE config 1): convs as row-im2col + one fp32 GEMM
    per product, channel-padded pooling, NCHW flatten — all on in-tree kernels."""
    from deeplearning4j_amd.models import LeNet
    net = LeNet(numLabels=10).init(device=torch.device("cuda", 0))
    g = torch.Generator().manual_seed(7)
    x = torch.rand(64, 784, generator=g).cuda()
    y = torch.nn.functional.one_hot(torch.randint(0, 10, (64,), generator=g), 10).float().cuda()
    _audit(_step_kernels(net, x, y, step=lambda: net.fit(x, y)), "LeNet fp32")


def test_resnet50_step_launches_no_torch_compute_kernels():
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    net = ResNet50(numLabels=100, dataType=DataType.BFLOAT16, inputShape=[3, 224, 224]).init(torch.device("cuda", 0))
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.rand(16, 3, 224, 224, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.zeros(16, 100, device="cuda")
    y[torch.arange(16), torch.randint(0, 100, (16,), generator=g).cuda()] = 1.0
    ks = _step_kernels(net, x, y)
    assert len(ks) > 100
    torch_ks = sorted({n for n, _ in ks if _is_torch_kernel(n)})
    t_all = sum(t for _, t in ks)
    t_torch = sum(t for n, t in ks if _is_torch_kernel(n))
    print(f"{len(ks)} kernels, {len(torch_ks)} distinct torch kernels, {100 * t_torch / max(t_all, 1):.2f} % of time")
    for n in torch_ks:
        print("  torch:", n[:140])
    assert not torch_ks, f"torch compute kernels in the ResNet-50 step: {torch_ks[:6]}"


@pytest.mark.parametrize("view", ["contiguous", "f_order"])
def test_stem_weight_packing_kernel(view):
    from deeplearning4j_amd.ops import conv_native, conv_stem
    torch.manual_seed(2)
    w = torch.randn(64, 3, 7, 7, device="cuda").to(torch.bfloat16)
    if view == "f_order":
        w = w.permute(3, 2, 1, 0).contiguous().permute(3, 2, 1, 0)      # same values, reversed strides
    conv_native.bump_version()
    pk = conv_stem.pack_weights(w)
    torch.cuda.synchronize()
    assert torch.equal(pk, conv_stem.pack_weights_reference(w))
