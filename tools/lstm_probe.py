#!/usr/bin/env python3
"""Time the whole-sequence LSTM kernels (csrc/lstm.hip) in isolation over minibatch / hidden sizes.

Prints us per timestep for forward (with / without the training caches) and backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deeplearning4j_amd.ops import rnn_native  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    dev = torch.device("cuda", 0)
    T = 50
    for H in (128, 256, 512):
        for mb in (16, 32, 128, 1024):
            for peep in (True,):
                zx = torch.randn(T, mb, 4 * H, device=dev).to(torch.bfloat16)
                RW = (torch.randn(H, 4 * H + 3, device=dev) * 0.05).to(torch.bfloat16)
                us_nc = timeit(lambda: rnn_native.lstm_seq_fwd(zx, RW, H, peep, need_cache=False))
                us_c = timeit(lambda: rnn_native.lstm_seq_fwd(zx, RW, H, peep, need_cache=True))
                out, hT, cT, gates, call = rnn_native.lstm_seq_fwd(zx, RW, H, peep, need_cache=True)[:5]
                eps = torch.randn(T, mb, H, device=dev)
                us_b = timeit(lambda: rnn_native.lstm_seq_bwd(eps, gates, call, None, RW, H, peep))
                print(f"H={H:4d} mb={mb:5d} fwd(nocache) {us_nc / T:7.2f} us/step  fwd(cache) {us_c / T:7.2f}  "
                      f"bwd {us_b / T:7.2f}", flush=True)


if __name__ == "__main__":
    main()
