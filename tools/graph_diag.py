"""Diagnose graph-vs-eager TBPTT differences window by window (GPU). Usage: python tools/graph_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_lstm_graph import _char_data, _textgen  # noqa: E402


def main():
    # 1) eager determinism
    a, b = _textgen(64, 10), _textgen(64, 10)
    b.setParams(a.params().clone())
    for i in range(3):
        x, y = _char_data(8, 35, 24, i)
        a.fit(x, y)
        b.fit(x, y)
    print("eager-vs-eager max diff", (a.params() - b.params()).abs().max().item())
    # 2) per window: patch _apply_update_kernels to snapshot params after every window
    e, g = _textgen(64, 10), _textgen(64, 10)
    g.setParams(e.params().clone())
    g.enableHipGraphs(True, warmup=1)
    snaps = {"e": [], "g": []}
    for name, net in (("e", e), ("g", g)):
        orig = net._iteration_done

        def hook(orig=orig, net=net, name=name):
            torch.cuda.synchronize()
            snaps[name].append((net.params().clone(), net.score(),
                                {k: v.clone() for l in [net.layers[0], net.layers[1]]
                                 for k, v in l.tBpttStateMap.items()}))
            orig()
        net._iteration_done = hook
    for i in range(3):
        x, y = _char_data(8, 35, 24, i)
        e.fit(x, y)
        g.fit(x, y)
    for w, ((pe, se, ste), (pg, sg, stg)) in enumerate(zip(snaps["e"], snaps["g"])):
        sd = max(((ste[k] - stg[k]).abs().max().item() if k in stg else -1) for k in ste) if ste else 0
        print(f"window {w}: param diff {(pe - pg).abs().max().item():.3e} score {se:.6f} vs {sg:.6f} "
              f"state diff {sd:.3e} keys {sorted(ste)} / {sorted(stg)}")
    print("graphs:", {k[-1]: (cs.ok, len(cs.state)) for k, cs in g._hipgraphs.items()})


if __name__ == "__main__":
    main()
