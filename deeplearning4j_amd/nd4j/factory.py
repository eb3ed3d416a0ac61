"""``Nd4j`` factory namespace and ``AffinityManager``: array creation on the current
device, ``gemm``, stacking, ``averageAndPropagate``, the binary ``write``/``read`` codec and the executioner /
workspace / memory managers.

Arrays are created on the default device: the current MI355X when one is visible (``Nd4j.setDefaultDevice`` or
``DL4J_AMD_ND4J_DEVICE`` override it), the CPU otherwise; the default floating-point type is fp32
(``Nd4j.setDataType``)."""
import os

import numpy as np
import torch

from .ndarray import INDArray, _unwrap

_STATE = {"dtype": torch.float32, "device": None, "seed": None}

_DTYPES = {"FLOAT": torch.float32, "DOUBLE": torch.float64, "HALF": torch.float16, "BFLOAT16": torch.bfloat16,
           "INT": torch.int32, "LONG": torch.int64, "BOOL": torch.bool, "float": torch.float32,
           "double": torch.float64, "half": torch.float16}


def _dtype(d):
    if d is None:
        return _STATE["dtype"]
    if isinstance(d, torch.dtype):
        return d
    return _DTYPES[str(getattr(d, "name", d))]


def _device():
    if _STATE["device"] is not None:
        return _STATE["device"]
    env = os.environ.get("DL4J_AMD_ND4J_DEVICE")
    if env:
        return torch.device(env)
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _shape_args(shape):
    if len(shape) == 1 and isinstance(shape[0], (list, tuple)):
        return tuple(int(s) for s in shape[0])
    return tuple(int(s) for s in shape)


def _split_order(args):
    """Accept ND4J's (order, shape...) / (shape..., order) call forms."""
    order = "c"
    args = list(args)
    if args and isinstance(args[0], str):
        order = args.pop(0)
    if args and isinstance(args[-1], str):
        order = args.pop()
    return order, args


def _make(t, order="c"):
    t = t.to(_device())
    if order == "f" and t.dim() >= 2:
        t = t.permute(*reversed(range(t.dim()))).contiguous().permute(*reversed(range(t.dim())))
    return INDArray(t)


class AffinityManager:
    """``Nd4j.getAffinityManager()``: one process per GPU, so the thread's device is the process's device."""

    @staticmethod
    def getNumberOfDevices():
        return torch.cuda.device_count() if torch.cuda.is_available() else 1

    @staticmethod
    def getDeviceForCurrentThread():
        return torch.cuda.current_device() if torch.cuda.is_available() else 0

    @staticmethod
    def attachThreadToDevice(thread=None, device=0):
        if torch.cuda.is_available():
            torch.cuda.set_device(int(device))

    @staticmethod
    def getDeviceForArray(arr):
        d = _unwrap(arr).device
        return d.index if d.type == "cuda" else -1

    @staticmethod
    def replicateToDevice(device, arr):
        t = _unwrap(arr)
        return INDArray(t.to(torch.device("cuda", int(device)) if torch.cuda.is_available() else t.device))

    @staticmethod
    def ensureLocation(arr, location=None):
        return arr

    @staticmethod
    def tagLocation(arr, location=None):
        return arr


class Nd4j:
    """Factory namespace mirroring ``org.nd4j.linalg.factory.Nd4j``."""

    # ------------------------------------------------------------------ configuration
    @staticmethod
    def setDataType(dtype):
        _STATE["dtype"] = _dtype(dtype)

    setDefaultDataTypes = setDataType

    @staticmethod
    def dataType():
        return INDArray(torch.zeros(0, dtype=_STATE["dtype"])).dataType()

    @staticmethod
    def setDefaultDevice(device):
        _STATE["device"] = None if device is None else torch.device(device)

    @staticmethod
    def getAffinityManager():
        return AffinityManager()

    @staticmethod
    def getRandom():
        return _Random()

    # ------------------------------------------------------------------ creation
    @staticmethod
    def create(*args, dtype=None):
        """create(double[] / nested lists / ndarray [, shape] [, order]) or create(shape... [, order]) (zeros)."""
        order, args = _split_order(args)
        dt = _dtype(dtype)
        if args and isinstance(args[0], (list, np.ndarray, torch.Tensor, INDArray)):
            data = args[0]
            if isinstance(data, INDArray):
                data = data.toTensor()
            t = torch.as_tensor(np.asarray(data) if not torch.is_tensor(data) else data).to(dt)
            if len(args) > 1:                                      # create(data, shape): data in `order`
                shape = _shape_args(args[1:])
                flat = t.reshape(-1)
                if order == "f":
                    return _make_f_view(flat.reshape(tuple(reversed(shape))).permute(*reversed(range(len(shape)))))
                t = flat.reshape(shape)
            elif t.dim() == 1:
                t = t.reshape(1, -1)                                # ND4J row vector
            return _make(t, order)
        return _make(torch.zeros(_shape_args(args), dtype=dt), order)

    @staticmethod
    def createUninitialized(*shape, dtype=None):
        order, shape = _split_order(shape)
        return _make(torch.empty(_shape_args(shape), dtype=_dtype(dtype)), order)

    @staticmethod
    def zeros(*shape, dtype=None):
        order, shape = _split_order(shape)
        return _make(torch.zeros(_shape_args(shape), dtype=_dtype(dtype)), order)

    @staticmethod
    def ones(*shape, dtype=None):
        order, shape = _split_order(shape)
        return _make(torch.ones(_shape_args(shape), dtype=_dtype(dtype)), order)

    @staticmethod
    def valueArrayOf(shape, value, dtype=None):
        shape = tuple(shape) if isinstance(shape, (list, tuple)) else (int(shape),)
        return _make(torch.full(shape, float(value), dtype=_dtype(dtype)))

    @staticmethod
    def scalar(value, dtype=None):
        return _make(torch.tensor(value, dtype=_dtype(dtype)).reshape(1, 1))

    @staticmethod
    def zerosLike(a):
        return INDArray(torch.zeros_like(_unwrap(a)))

    @staticmethod
    def onesLike(a):
        return INDArray(torch.ones_like(_unwrap(a)))

    @staticmethod
    def rand(*shape, seed=None):
        g = torch.Generator().manual_seed(int(seed)) if seed is not None else _Random.gen()
        return _make(torch.rand(_shape_args(shape), generator=g, dtype=_STATE["dtype"]))

    @staticmethod
    def randn(*shape, seed=None):
        g = torch.Generator().manual_seed(int(seed)) if seed is not None else _Random.gen()
        return _make(torch.randn(_shape_args(shape), generator=g, dtype=_STATE["dtype"]))

    @staticmethod
    def linspace(a, b, n):
        return _make(torch.linspace(float(a), float(b), int(n), dtype=_STATE["dtype"]).reshape(1, -1))

    @staticmethod
    def arange(a, b=None):
        lo, hi = (0, a) if b is None else (a, b)
        return _make(torch.arange(lo, hi, dtype=_STATE["dtype"]).reshape(1, -1))

    @staticmethod
    def eye(n):
        return _make(torch.eye(int(n), dtype=_STATE["dtype"]))

    @staticmethod
    def diag(x):
        t = _unwrap(x)
        if t.dim() == 2 and 1 in t.shape:
            return INDArray(torch.diag(t.reshape(-1)))
        return INDArray(torch.diagonal(t).reshape(-1, 1).clone())

    # ------------------------------------------------------------------ combination
    @staticmethod
    def hstack(*xs):
        xs = xs[0] if len(xs) == 1 and isinstance(xs[0], (list, tuple)) else xs
        return INDArray(torch.cat([_unwrap(x) for x in xs], dim=1))

    @staticmethod
    def vstack(*xs):
        xs = xs[0] if len(xs) == 1 and isinstance(xs[0], (list, tuple)) else xs
        return INDArray(torch.cat([_unwrap(x) for x in xs], dim=0))

    @staticmethod
    def concat(dim, *xs):
        xs = xs[0] if len(xs) == 1 and isinstance(xs[0], (list, tuple)) else xs
        return INDArray(torch.cat([_unwrap(x) for x in xs], dim=dim))

    @staticmethod
    def stack(dim, *xs):
        xs = xs[0] if len(xs) == 1 and isinstance(xs[0], (list, tuple)) else xs
        return INDArray(torch.stack([_unwrap(x) for x in xs], dim=dim))

    @staticmethod
    def pile(*xs):
        return Nd4j.stack(0, *xs)

    @staticmethod
    def tile(x, *reps):
        reps = reps[0] if len(reps) == 1 and isinstance(reps[0], (list, tuple)) else reps
        return INDArray(_unwrap(x).repeat(*reps))

    @staticmethod
    def toFlattened(*xs, order="c"):
        xs = xs[0] if len(xs) == 1 and isinstance(xs[0], (list, tuple)) else xs
        parts = []
        for x in xs:
            t = _unwrap(x)
            parts.append(t.reshape(-1) if order == "c" else t.permute(*reversed(range(t.dim()))).reshape(-1))
        return INDArray(torch.cat(parts).reshape(1, -1))

    # ------------------------------------------------------------------ linear algebra / misc ops
    @staticmethod
    def gemm(a, b, transposeA=False, transposeB=False, c=None, alpha=1.0, beta=0.0):
        A, B = _unwrap(a), _unwrap(b)
        A = A.t() if transposeA else A
        B = B.t() if transposeB else B
        from ..ops.gemm import mmul as _mm
        if c is not None:
            ct = _unwrap(c)
            with torch.no_grad():
                _mm(A, B.to(A.dtype), out=ct, alpha=alpha, beta=beta)
            return c
        r = _mm(A, B.to(A.dtype), alpha=alpha)
        return INDArray(r)

    @staticmethod
    def argMax(x, *dims):
        return INDArray(_unwrap(x)).argMax(*dims)

    @staticmethod
    def sort(x, dim, ascending=True):
        return INDArray(torch.sort(_unwrap(x), dim=dim, descending=not ascending).values)

    @staticmethod
    def sortWithIndices(x, dim, ascending=True):
        r = torch.sort(_unwrap(x), dim=dim, descending=not ascending)
        return INDArray(r.indices.to(_unwrap(x).dtype)), INDArray(r.values)

    @staticmethod
    def cumsum(x, dim=1):
        return INDArray(_unwrap(x).cumsum(dim))

    @staticmethod
    def reverse(x):
        t = _unwrap(x)
        return INDArray(t.reshape(-1).flip(0).reshape(t.shape))

    @staticmethod
    def averageAndPropagate(target, arrays):
        """Mean of same-shape arrays written back to all of them (and to ``target`` when given). Across processes
        the equivalent is the RCCL all-reduce in ``parallel.distributed``."""
        ts = [_unwrap(a) for a in arrays]
        with torch.no_grad():
            m = torch.stack([t.to(ts[0].device) for t in ts]).mean(0)
            for t in ts:
                t.copy_(m.to(t.device))
            if target is not None:
                _unwrap(target).copy_(m.to(_unwrap(target).device))
        return target if target is not None else INDArray(m)

    # ------------------------------------------------------------------ serialization
    @staticmethod
    def write(arr, out, order="c"):
        from ..utils import nd4j_io
        nd4j_io.write(_unwrap(arr), out, order)

    @staticmethod
    def read(inp):
        from ..utils import nd4j_io
        return nd4j_io.read(inp)

    @staticmethod
    def readArray(inp):
        """Read into an INDArray on the default device."""
        return _make(Nd4j.read(inp))

    @staticmethod
    def saveBinary(arr, path):
        with open(path, "wb") as f:
            Nd4j.write(arr, f)

    @staticmethod
    def readBinary(path):
        with open(path, "rb") as f:
            return Nd4j.readArray(f)

    @staticmethod
    def writeTxt(arr, path):
        np.savetxt(path, np.atleast_2d(np.asarray(arr)), delimiter=",")

    @staticmethod
    def readTxt(path):
        return _make(torch.from_numpy(np.atleast_2d(np.loadtxt(path, delimiter=","))).to(_STATE["dtype"]))

    # ------------------------------------------------------------------ executioner / memory
    @staticmethod
    def getExecutioner():
        from ..profiling import getExecutioner
        return getExecutioner()

    @staticmethod
    def getWorkspaceManager():
        from ..memory import getWorkspaceManager
        return getWorkspaceManager()

    @staticmethod
    def getMemoryManager():
        return _MemoryManager()


def _make_f_view(t_f):
    """``t_f`` already has column-major strides over its values; move it to the device keeping them."""
    dev = _device()
    if t_f.device == dev:
        return INDArray(t_f)
    rev = tuple(reversed(range(t_f.dim())))
    return INDArray(t_f.permute(*rev).contiguous().to(dev).permute(*rev))


class _Random:
    """``Nd4j.getRandom()``: process-wide seedable generator."""
    _g = None

    @classmethod
    def gen(cls):
        if cls._g is None:
            cls._g = torch.Generator()
            cls._g.seed()
        return cls._g

    def setSeed(self, seed):
        _Random.gen().manual_seed(int(seed))
        torch.manual_seed(int(seed))

    def nextDouble(self):
        return float(torch.rand(1, generator=_Random.gen()))

    def nextGaussian(self):
        return float(torch.randn(1, generator=_Random.gen()))

    def nextInt(self, n=2 ** 31 - 1):
        return int(torch.randint(0, int(n), (1,), generator=_Random.gen()))


class _MemoryManager:
    """Nd4j.getMemoryManager(): memset / current workspace / device memory info."""

    @staticmethod
    def memset(t):
        with torch.no_grad():
            _unwrap(t).zero_()

    @staticmethod
    def getCurrentWorkspace():
        from ..memory import getWorkspaceManager
        return getWorkspaceManager().getCurrentWorkspace()

    @staticmethod
    def invokeGc():
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.empty_cache()

    @staticmethod
    def getDeviceMemoryInfo(device=0):
        """(free, total) bytes of the device (hipMemGetInfo)."""
        if not torch.cuda.is_available():
            return (0, 0)
        return torch.cuda.mem_get_info(device)
