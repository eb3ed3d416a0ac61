"""Where do torch compute kernels come from in one training step? Profiles one steady-state step of BERT (2 layers),
the LSTM char-LM or ResNet-50 with Python stacks and prints every aten op that launched a device kernel, with the
framework frames that called it. Diagnostic companion to tests/test_gpu_step_kernels.py.

Usage: python tools/step_torch_ops.py [bert|lstm|resnet|lenet]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(which):
    from deeplearning4j_amd.nn.conf import DataType
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    if which == "bert":
        from deeplearning4j_amd.models import BertBase
        net = BertBase(numLabels=2, inputShape=[128], layers=2, dataType=DataType.BFLOAT16).init(device=dev)
        x = torch.randint(0, 30522, (8, 128), generator=g).to(dev)
        y = torch.nn.functional.one_hot(torch.randint(0, 2, (8,), generator=g), 2).float().to(dev)
        return lambda: net.fit([x], [y])
    if which == "lstm":
        from deeplearning4j_amd.models import TextGenerationLSTM
        net = TextGenerationLSTM(numLabels=77, inputShape=[1, 77], hidden=256, dataType=DataType.BFLOAT16).init(device=dev)
        idx = torch.randint(0, 77, (8, 101), generator=g)
        x = torch.nn.functional.one_hot(idx[:, :-1], 77).permute(0, 2, 1).float().to(dev)
        y = torch.nn.functional.one_hot(idx[:, 1:], 77).permute(0, 2, 1).float().to(dev)
        return lambda: net.fit(x, y)
    if which == "lenet":
        from deeplearning4j_amd.models import LeNet
        net = LeNet(numLabels=10).init(device=dev)                  # tools/bench_lenet.py's model and input
        x = torch.rand(64, 784, generator=g).to(dev)
        y = torch.nn.functional.one_hot(torch.randint(0, 10, (64,), generator=g), 10).float().to(dev)
        return lambda: net.fit(x, y)
    from deeplearning4j_amd.models import ResNet50
    net = ResNet50(numLabels=100, dataType=DataType.BFLOAT16, inputShape=[3, 224, 224]).init(dev)
    x = torch.rand(16, 3, 224, 224, generator=g).to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.zeros(16, 100, device=dev)
    y[torch.arange(16), torch.randint(0, 100, (16,), generator=g).to(dev)] = 1.0
    return lambda: net.fit([x], [y])


def main():
    import collections
    import traceback
    from torch.profiler import ProfilerActivity, profile, record_function
    from torch.utils._python_dispatch import TorchDispatchMode
    which = sys.argv[1] if len(sys.argv) > 1 else "bert"
    step = build(which)
    step()
    step()
    torch.cuda.synchronize()

    class Spy(TorchDispatchMode):
        """Labels every aten call with the framework frames that issued it, so the profiler's kernel -> op links
        name the call site."""
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            fr = [f"{os.path.relpath(f.filename)}:{f.lineno} {f.name}" for f in traceback.extract_stack()[:-1]
                  if "deeplearning4j_amd" in f.filename]
            with record_function("SITE|" + str(func) + "|" + " <- ".join(reversed(fr[-3:]))):
                return func(*args, **(kwargs or {}))

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        with Spy():
            step()
        torch.cuda.synchronize()

    def kernels_under(e):
        out = [k.name for k in getattr(e, "kernels", [])]
        for c in e.cpu_children:
            out += kernels_under(c)
        return out

    hits = collections.Counter()
    for e in prof.events():
        if e.name.startswith("SITE|"):
            ks = [k for k in kernels_under(e) if "at::native" in k or "at6native" in k or k.startswith("void at::")]
            if ks and not any(c.name.startswith("SITE|") for c in e.cpu_children):
                hits[(e.name, ks[0][:90])] += 1
    for (site, k), n in sorted(hits.items(), key=lambda kv: kv[0]):
        _, op, fr = site.split("|", 2)
        print(f"{n:3d}x {op}  ->  {k}")
        print(f"       {fr}")


if __name__ == "__main__":
    main()
