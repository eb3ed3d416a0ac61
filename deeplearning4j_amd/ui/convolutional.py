"""ConvolutionalIterationListener: renders convolution-layer activations as image grids.

Reference: deeplearning4j-ui/.../weights/ConvolutionalIterationListener.java (every ``freq`` iterations, take the
first example's activations of each convolution / subsampling layer, normalise each channel map, tile them into a
grid and publish the image to the UI). Here the tiled grid is written as a grayscale PNG (stdlib zlib encoder) into
``outputDir`` and, when a stats router is given, referenced from a "ConvolutionalListener" update record.
"""
import os
import struct
import zlib

import torch

from ..optimize.listeners import TrainingListener
from .storage import Persistable


def write_png_gray(path, img):
    """8-bit grayscale PNG from a 2-D uint8 tensor / array."""
    a = img.detach().cpu().to(torch.uint8).numpy() if torch.is_tensor(img) else img
    h, w = a.shape
    raw = b"".join(b"\x00" + a[r].tobytes() for r in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)) + \
        chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(png)


def tile_activations(act, pad=1, max_channels=64):
    """[C, H, W] activations -> [rows*(H+pad), cols*(W+pad)] uint8 grid, each channel min-max normalised."""
    a = act.detach().float()[:max_channels]
    C, H, W = a.shape
    mn = a.reshape(C, -1).min(1).values.reshape(C, 1, 1)
    mx = a.reshape(C, -1).max(1).values.reshape(C, 1, 1)
    a = (a - mn) / (mx - mn).clamp_min(1e-12) * 255.0
    cols = int(max(1, round(C ** 0.5)))
    rows = (C + cols - 1) // cols
    grid = torch.zeros(rows * (H + pad), cols * (W + pad), device=a.device)
    for c in range(C):
        r, k = divmod(c, cols)
        grid[r * (H + pad):r * (H + pad) + H, k * (W + pad):k * (W + pad) + W] = a[c]
    return grid.round().clamp(0, 255).to(torch.uint8)


class ConvolutionalIterationListener(TrainingListener):
    def __init__(self, freq=10, outputDir="conv_activations", router=None, sessionID="conv", workerID="0"):
        self.freq = max(1, int(freq))
        self.outputDir = outputDir
        self.router = router
        self.sessionID, self.workerID = sessionID, workerID
        self._pending = None
        self.written = []

    def onForwardPass(self, model, activations):
        if (model.conf.iterationCount + 1) % self.freq != 0:
            return
        if isinstance(activations, dict):      # ComputationGraph: skip the network inputs
            skip = set(getattr(model.conf, "networkInputs", []) or [])
            acts = {k: a for k, a in activations.items() if k not in skip}
        else:                                   # MultiLayerNetwork: entry 0 is the input, entry i+1 is layer i
            acts = {str(i - 1): a for i, a in enumerate(activations) if i > 0}
        self._pending = {k: a[0].detach() for k, a in acts.items() if torch.is_tensor(a) and a.dim() == 4}

    def iterationDone(self, model, iteration, epoch):
        if not self._pending:
            return
        os.makedirs(self.outputDir, exist_ok=True)
        files = {}
        for k, a in self._pending.items():
            p = os.path.join(self.outputDir, f"iter{iteration}_layer{k}.png")
            write_png_gray(p, tile_activations(a))
            files[k] = p
            self.written.append(p)
        self._pending = None
        if self.router is not None:
            self.router.putUpdate(Persistable(self.sessionID, "ConvolutionalListener", self.workerID,
                                              data={"iteration": iteration, "images": files}))
