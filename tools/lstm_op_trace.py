#!/usr/bin/env python3
"""Which framework lines issue torch (library) tensor ops during one TextGenerationLSTM training step on the GPU:
torch.Tensor / torch functions that launch copy / fill / elementwise kernels are wrapped and counted per innermost
deeplearning4j_amd source line. Usage: python tools/lstm_op_trace.py [--length 100]"""
import argparse
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COUNTS = collections.Counter()
ACTIVE = [False]


def _where():
    for f in reversed(traceback.extract_stack()[:-2]):
        if "deeplearning4j_amd" in f.filename:
            return f"{f.filename.split('deeplearning4j_amd/')[-1]}:{f.lineno}"
    return "?"


def _wrap(owner, name):
    orig = getattr(owner, name)

    def w(*a, **k):
        if ACTIVE[0]:
            t = a[0] if a and torch.is_tensor(a[0]) else None
            if t is None or t.is_cuda:
                COUNTS[(name, _where())] += 1
        return orig(*a, **k)
    setattr(owner, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=100)
    a = ap.parse_args()
    from deeplearning4j_amd.models import TextGenerationLSTM
    from deeplearning4j_amd.nn.conf import DataType
    dev = torch.device("cuda", 0)
    net = TextGenerationLSTM(numLabels=77, inputShape=[1, 77], hidden=256, dataType=DataType.BFLOAT16).init(device=dev)
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, 77, (32, a.length + 1), generator=g)
    x = torch.nn.functional.one_hot(idx[:, :-1], 77).permute(0, 2, 1).float().to(dev)
    y = torch.nn.functional.one_hot(idx[:, 1:], 77).permute(0, 2, 1).float().to(dev)
    net.fit(x, y)
    torch.cuda.synchronize()
    for n in ("to", "contiguous", "clone", "zero_", "fill_", "copy_", "float", "sum", "add", "add_", "mul", "div",
              "__add__", "__mul__", "__truediv__", "__sub__", "reshape", "bfloat16", "masked_fill", "sub", "neg",
              "softmax", "log_softmax", "cat", "stack", "expand_as", "abs", "pow", "sqrt", "where", "clamp", "max"):
        if hasattr(torch.Tensor, n):
            _wrap(torch.Tensor, n)
    for n in ("zeros", "ones", "full", "zeros_like", "ones_like", "full_like", "cat", "stack", "where", "softmax"):
        _wrap(torch, n)
    ACTIVE[0] = True
    net.fit(x, y)
    torch.cuda.synchronize()
    ACTIVE[0] = False
    for (n, w), c in COUNTS.most_common(70):
        print(f"{c:5d}  {n:14s} {w}")


if __name__ == "__main__":
    main()
