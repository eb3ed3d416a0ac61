"""Weight-gradient overlap stream for the training backward pass.

In a conv layer's backward the weight gradient (dW = dY^T . im2col(X)) and the data gradient (dX) are independent;
the reference computes them back to back (ConvolutionLayer.java:215-257 — im2col GEMM for dW, then col2im for
epsilon). On MI355X the small late-stage ResNet convs fill only part of the 256 CUs (e.g. 392 output tiles for a
7x7x256 3x3 conv at batch 512), so running dW on a second HIP stream lets it fill the CUs the next layer's
bwd-data / BatchNorm-backward kernels leave idle.

Contract (``nn/network_base.py`` drives it):
  * ``begin(ref)`` at the start of a backward pass (active only for CUDA networks, ``DL4J_AMD_WRW_STREAM`` != 0);
  * ``run(fn, *keep)`` launches ``fn`` on the side stream after the main stream's pending work (its inputs) and keeps
    ``keep`` (the X / dY operands) referenced until the next join, so the caching allocator cannot hand their memory
    to later main-stream kernels while the side stream still reads it. ``fn`` must write only into persistent
    buffers (the flat fp32 gradient views) — nothing it allocates is returned to the main stream;
  * ``join()`` makes the main stream wait for every side launch (before a data-parallel bucket reads gradients) and
    ``end()`` joins and closes the pass. Under HIP-graph capture the fork/join become graph edges (the side stream
    joins the capture through the event wait), so the replayed graph runs dW and dX as parallel branches.
"""
import os
import threading

import torch

_tl = threading.local()
LAUNCHES = [0]   # side-stream launches so far (tests check the overlap path really ran)


def enabled():
    return os.environ.get("DL4J_AMD_WRW_STREAM", "1") == "1"


def side_cus():
    """CUs the weight-gradient stream may use (``DL4J_AMD_WRW_CUS``; 0 = all). A CU-masked side stream leaves the
    rest of the chip to the main chain, whose short BatchNorm / elementwise kernels would otherwise wait for the
    long-running weight-gradient blocks to retire before they get a CU."""
    try:
        return int(os.environ.get("DL4J_AMD_WRW_CUS", "0"))
    except ValueError:
        return 0


def _side(dev):
    # one side stream per (host thread, device): a stream shared by two threads would join one thread's HIP-graph
    # capture and pull the other thread's weight-gradient launches into it (in-process ParallelWrapper workers)
    streams = _tl.__dict__.setdefault("streams", {})
    s = streams.get(dev.index)
    if s is None:
        cus = side_cus()
        if cus > 0:
            from .. import runtime as rt
            native = rt.Stream(dev.index, cus=cus)
            s = native.torch_stream()
            s._dl4j_native = native          # keeps the HIP stream alive as long as the torch wrapper
        else:
            s = torch.cuda.Stream(dev)
        streams[dev.index] = s
    return s


def begin(ref):
    _tl.st = None
    if enabled() and ref is not None and getattr(ref, "is_cuda", False):
        _tl.st = {"dev": ref.device, "main": None, "refs": [], "pending": False}


def active():
    return getattr(_tl, "st", None) is not None


def run(fn, *keep):
    st = getattr(_tl, "st", None)
    if st is None:
        return fn()
    main = torch.cuda.current_stream(st["dev"])
    if st["main"] is None:
        st["main"] = main
    elif st["main"] != main:          # the caller switched streams mid-pass: stay on its stream
        return fn()
    side = _side(st["dev"])
    side.wait_stream(main)
    with torch.cuda.stream(side):
        r = fn()
    st["refs"].extend(keep)
    st["pending"] = True
    LAUNCHES[0] += 1
    return r


class suspended:
    """Run a block with the overlap stream off (every ``run`` executes inline on the caller's stream). Used while
    the conv layer times candidate kernels on scratch buffers: a candidate sent to the side stream would outlive
    its scratch outputs and escape the main-stream timing events."""

    def __enter__(self):
        self._st = getattr(_tl, "st", None)
        _tl.st = None
        return self

    def __exit__(self, *exc):
        _tl.st = self._st
        return False


def join():
    st = getattr(_tl, "st", None)
    if st is not None and st["pending"]:
        st["main"].wait_stream(_side(st["dev"]))
        st["pending"] = False
        st["refs"].clear()


def end():
    join()
    _tl.st = None
