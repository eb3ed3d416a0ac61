"""Per-parameter gradient error of a bf16 graph against the same graph in fp32 (diagnostic for the conv paths).
Usage: python tools/grad_diag.py [C]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_conv_safety import _data, _graph, _grad  # noqa: E402

from deeplearning4j_amd.nn.conf import DataType  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
x, y = _data()
ref = _graph(C, DataType.FLOAT)
net = _graph(C, DataType.BFLOAT16)
net.setParams(ref.params().clone())
g32 = _grad(ref, x, y)
g16 = _grad(net, x, y)
for name, view in ref.paramTable().items():
    off = view.data_ptr() - ref.params().data_ptr()
    n = view.numel()
    o = off // 4
    a, b = g16[0, o:o + n], g32[0, o:o + n]
    print(f"{name:10s} n={n:7d} max|g32|={b.abs().max().item():9.4f} maxerr={(a - b).abs().max().item():9.4f} "
          f"relnorm={((a - b).norm() / (b.norm() + 1e-12)).item():.4f}")
