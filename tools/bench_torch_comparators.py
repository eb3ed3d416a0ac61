#!/usr/bin/env python3
"""Same-GPU PyTorch-ROCm comparators for the headline and LSTM configurations: plain ``torch.nn``
models trained the idiomatic PyTorch way on the same MI355X, so the framework's numbers can be placed.

  --model resnet50   canonical ResNet-50 (v1.5 bottlenecks, torchvision-equivalent topology written out here since
                     torchvision is not installed), channels_last, bf16 autocast with fp32 weights, RMSprop
                     (foreach) - the bench.py config: batch 512, 224x224, 1000 classes.
  --model lstm       char-LM: 2-layer torch.nn.LSTM(77 -> 256) + Linear(77), bf16 autocast, RMSprop, truncated BPTT
                     windows of 50 over a [32, 1000] sequence batch per step (the tools/bench_lstm.py config; torch's
                     LSTM has no peepholes, so it does slightly less work than GravesLSTM).

Synthetic data, random-init weights. Prints one JSON line. Usage:
  python tools/bench_torch_comparators.py --model resnet50 --steps 10 --warmup 3
  python tools/bench_torch_comparators.py --model lstm --steps 5 --warmup 2
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride, down):
        super().__init__()
        cout = width * 4
        self.c1 = nn.Conv2d(cin, width, 1, bias=False)
        self.b1 = nn.BatchNorm2d(width)
        self.c2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(width)
        self.c3 = nn.Conv2d(width, cout, 1, bias=False)
        self.b3 = nn.BatchNorm2d(cout)
        self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout)) if down else None

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + (self.down(x) if self.down is not None else x))


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for width, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            for i in range(n):
                layers.append(Bottleneck(cin, width, stride if i == 0 else 1, i == 0))
                cin = width * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, classes)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def bench_resnet(args, dev):
    mf = torch.contiguous_format if args.nchw else torch.channels_last
    model = ResNet50().to(dev).to(memory_format=mf)
    opt = torch.optim.RMSprop(model.parameters(), lr=0.1, alpha=0.96, eps=1e-3, weight_decay=5e-5, foreach=True)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(args.batch, 3, 224, 224, generator=g).to(dev).contiguous(memory_format=mf)
    y = torch.randint(0, 1000, (args.batch,), generator=g).to(dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss
    return step, args.batch, "images/sec", \
        f"ResNet-50 (canonical, torch.nn, {'NCHW' if args.nchw else 'channels_last'}, bf16 autocast)"


class CharLSTM(nn.Module):
    def __init__(self, V, H):
        super().__init__()
        self.lstm = nn.LSTM(V, H, num_layers=2, batch_first=True)
        self.out = nn.Linear(H, V)

    def forward(self, x, state):
        h, state = self.lstm(x, state)
        return self.out(h), state


def bench_lstm(args, dev):
    V, H, B, L, W = 77, 256, 32, 1000, 50
    model = CharLSTM(V, H).to(dev)
    opt = torch.optim.RMSprop(model.parameters(), lr=0.01, weight_decay=1e-3, foreach=True)
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, V, (B, L + 1), generator=g).to(dev)
    x = F.one_hot(idx[:, :-1], V).float()
    y = idx[:, 1:]

    def step():
        state = None
        loss = None
        for t0 in range(0, L, W):                      # truncated BPTT, state carried (detached) across windows
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, state = model(x[:, t0:t0 + W], state)
                loss = F.cross_entropy(logits.reshape(-1, V), y[:, t0:t0 + W].reshape(-1))
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            state = tuple(s.detach() for s in state)
        return loss
    return step, B * L, "characters/sec", "2x torch.nn.LSTM(256) char-LM, bf16 autocast, TBPTT 50"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", choices=["resnet50", "lstm"], default="resnet50")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--nchw", type=int, default=0, help="ResNet: NCHW activations instead of channels_last")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    import sys
    import threading
    t_start = time.time()

    def heartbeat():                                   # MIOpen's first-call kernel search can be silent for minutes
        while True:
            time.sleep(30)
            print(f"[cmp] still running, {time.time() - t_start:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    step, per_step, unit, name = (bench_resnet if args.model == "resnet50" else bench_lstm)(args, dev)
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        print(f"[cmp] warmup step {i} done {time.time() - t_start:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": f"PyTorch-ROCm comparator: {name}", "value": round(per_step * args.steps / dt, 1),
                      "unit": unit, "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
                      "ms_per_step": round(dt / args.steps * 1e3, 2), "impl": "torch", "torch": torch.__version__,
                      "loss": float(loss), "data": "synthetic; random-init weights"}))


if __name__ == "__main__":
    main()
