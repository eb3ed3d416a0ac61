#!/usr/bin/env python3
"""Large-batch numerics check for the ResNet-50 bench path: a batch made of the same B images repeated R times has
the same per-example mean loss, the same batch-norm statistics and hence the same gradients as the B-image batch,
so two nets with identical init trained on x and on cat([x] * R) must follow the same score trajectory (up to bf16
rounding and kernel choices). The score itself is (loss sum + L1 + L2) / minibatch as in the reference's
BaseOutputLayer.computeScore, so its regularization share halves with the batch; the check therefore compares the
loss-only part the gradients and the parameters after the steps. Caveat measured on the CPU in fp32: the randomly initialised
zoo ResNet-50 saturates its softmax (loss ~ 23 = the 1e-10 clip), and a 1e-7 relative input perturbation already
moves its gradient by 1.5 %, so with bf16 rounding and the GPU's atomics-based reductions the gradient comparison is
O(1) even between two passes on the same batch; the parameter difference after one step (RmsProp's first update is
sign-like) is the usable number. Catches index-width overflows that only appear at large per-GPU batches.
Usage on a GPU box: python tools/batch_dup_check.py [--batch 512 --repeat 2 --steps 8]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(xb, yb, steps, seed):
    from deeplearning4j_amd.models import ResNet50
    from deeplearning4j_amd.nn.conf import DataType
    torch.manual_seed(seed)
    dt = DataType.BFLOAT16 if xb.device.type == "cuda" else DataType.FLOAT
    net = ResNet50(numLabels=1000, dataType=dt).init(device=xb.device)
    net.computeGradientAndScore([xb], [yb])
    g0 = net.getFlattenedGradients().detach().float().cpu().clone()
    net.computeGradientAndScore([xb], [yb])          # second pass: every kernel shape already tuned
    grad = net.getFlattenedGradients().detach().float().cpu().clone()
    print(json.dumps({"batch": xb.shape[0], "grad_rel_first_vs_second_pass": ((g0 - grad).norm() / grad.norm()).item(),
                      "grad_norm": grad.norm().item()}), flush=True)
    scores = []
    for _ in range(steps):
        reg = net.calcL1() + net.calcL2()            # the score of fit() is taken before its update
        net.fit([xb], [yb])
        scores.append(round(float(net.score()) - float(reg) / xb.shape[0], 4))
    return scores, net.params().detach().float().cpu(), grad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0) if args.device == "cuda" else torch.device("cpu")
    B = args.batch
    g = torch.Generator().manual_seed(42)
    x = torch.rand(B, 3, 224, 224, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    x = x.to(torch.bfloat16 if dev.type == "cuda" else torch.float32)
    y = torch.zeros(B, 1000, device=dev)
    y[torch.arange(B), torch.randint(0, 1000, (B,), generator=g).to(dev)] = 1.0
    small, p1, g1 = run(x, y, args.steps, 1234)
    xr = torch.cat([x] * args.repeat).contiguous(memory_format=torch.channels_last)
    big, p2, g2 = run(xr, torch.cat([y] * args.repeat), args.steps, 1234)
    rel = max(abs(a - b) / max(abs(a), 1e-3) for a, b in zip(small, big))
    prel = ((p1 - p2).norm() / p1.norm()).item()
    g2 = g2 / args.repeat                       # gradients are example sums here; the updater divides by the batch
    grel = ((g1 - g2).norm() / g1.norm()).item()
    print(json.dumps({"batch": B, "repeat": args.repeat, "loss_small": small, "loss_repeated": big,
                      "max_rel_loss_diff": round(rel, 5), "grad_rel_diff": grel, "param_rel_diff": prel}), flush=True)


if __name__ == "__main__":
    main()
