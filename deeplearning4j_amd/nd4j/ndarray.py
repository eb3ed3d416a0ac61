"""ND4J-compatible array API: ``INDArray``, ``NDArrayIndex``, ``Transforms``.

The reference's user code talks to ND4J (``org.nd4j.linalg.api.ndarray.INDArray``, imported 638 times across the
reference). This is the same surface over a device tensor: an INDArray owns a strided torch tensor
that lives on the current device (the MI355X when present), so every op runs as a device kernel and arrays pass
into ``MultiLayerNetwork.fit/output``, ``DataSet`` etc. without copies.

Semantics kept from ND4J:
* ``c``/``f`` ordering: ``Nd4j.create(..., order='f')`` and ``dup('f')`` produce column-major strides, and
  ``reshape('f', ...)`` / ``ravel('f')`` walk elements in column-major order. ``ordering()`` reports the layout.
* Vectors are rank 2: ``Nd4j.create(double[])`` is a ``[1, n]`` row vector, ``getRow``/``getColumn`` return
  ``[1, n]`` / ``[n, 1]``.
* Views: ``get(NDArrayIndex...)``, ``getRow``, ``getColumn``, ``transpose``, ``permute``, ``slice`` and
  ``tensorAlongDimension`` return views that share storage; the ``*i`` ops write in place (through views too).
* Reductions along dimensions (``sum(0)``, ``mean(1)``, ``norm2(...)``) drop the reduced dimensions but keep
  results at least rank 2 (a row vector), and the ``*Number()`` forms return Python scalars.
"""
import math

import numpy as np
import torch


def _unwrap(x):
    return x._t if isinstance(x, INDArray) else x


def _partial_overlap(a, b):
    """True when ``b`` shares memory with ``a`` other than as the very same element-for-element view (in-place ops
    write ``a`` while reading ``b``; identical views are safe elementwise, anything else races)."""
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return False
    same = (a.shape == b.shape and a.stride() == b.stride() and a.storage_offset() == b.storage_offset())
    return not same


def _wrap(t):
    return INDArray(t)


def _as_2d(t):
    """ND4J keeps vectors rank 2: 0-d -> [1,1], 1-d -> [1, n]."""
    if t.dim() == 0:
        return t.reshape(1, 1)
    if t.dim() == 1:
        return t.reshape(1, -1)
    return t


def _f_strided(t):
    """Same values, column-major storage."""
    if t.dim() < 2:
        return t.clone()
    return t.permute(*reversed(range(t.dim()))).contiguous().permute(*reversed(range(t.dim())))


def _norm_dims(dims, rank):
    out = []
    for d in dims:
        if isinstance(d, (list, tuple)):
            out.extend(d)
        else:
            out.append(d)
    return [d % rank for d in out]


class NDArrayIndex:
    """``NDArrayIndex.all() / point(i) / interval(a, b[, inclusive]) / interval(a, stride, b) / indices(...)``."""

    def __init__(self, kind, a=None, b=None, step=1):
        self.kind, self.a, self.b, self.step = kind, a, b, step

    @staticmethod
    def all():
        return NDArrayIndex("all")

    @staticmethod
    def point(i):
        return NDArrayIndex("point", int(i))

    @staticmethod
    def newAxis():
        return NDArrayIndex("newaxis")

    @staticmethod
    def interval(a, b, c=None, inclusive=False):
        if isinstance(c, bool):
            return NDArrayIndex("interval", int(a), int(b) + (1 if c else 0))
        if c is not None:                                        # interval(begin, stride, end)
            return NDArrayIndex("interval", int(a), int(c), int(b))
        return NDArrayIndex("interval", int(a), int(b) + (1 if inclusive else 0))

    @staticmethod
    def indices(*idx):
        return NDArrayIndex("indices", [int(i) for i in (idx[0] if len(idx) == 1 and
                                                         isinstance(idx[0], (list, tuple)) else idx)])

    def to_py(self):
        if self.kind == "all":
            return slice(None)
        if self.kind == "point":
            return self.a
        if self.kind == "newaxis":
            return None
        if self.kind == "interval":
            return slice(self.a, self.b, self.step)
        return list(self.a)


class INDArray:
    __slots__ = ("_t", "__weakref__")

    def __init__(self, t):
        self._t = t if torch.is_tensor(t) else torch.as_tensor(np.asarray(t))

    # ------------------------------------------------------------------ interop
    def toTensor(self):
        return self._t

    def __array__(self, dtype=None, copy=None):
        a = self._t.detach().float().cpu().numpy() if self._t.dtype in (torch.bfloat16,) else \
            self._t.detach().cpu().numpy()
        return a if dtype is None else a.astype(dtype)

    def toNumpy(self):
        return self.__array__()

    def toDoubleVector(self):
        return self._t.detach().double().reshape(-1).cpu().tolist()

    def toFloatVector(self):
        return self._t.detach().float().reshape(-1).cpu().tolist()

    def toIntVector(self):
        return self._t.detach().long().reshape(-1).cpu().tolist()

    def toDoubleMatrix(self):
        return self._t.detach().double().cpu().tolist()

    def __repr__(self):
        return "INDArray" + repr(self.__array__()).replace("array", "", 1)

    toString = __repr__

    # ------------------------------------------------------------------ shape information
    def shape(self):
        return list(self._t.shape)

    def stride(self, dim=None):
        return list(self._t.stride()) if dim is None else self._t.stride(dim)

    def rank(self):
        return self._t.dim()

    def length(self):
        return self._t.numel()

    def size(self, dim):
        return self._t.shape[dim]

    def rows(self):
        return self._t.shape[0] if self._t.dim() >= 1 else 1

    def columns(self):
        return self._t.shape[1] if self._t.dim() >= 2 else self._t.numel()

    def ordering(self):
        t = self._t
        if t.dim() >= 2 and not t.is_contiguous() and t.permute(*reversed(range(t.dim()))).is_contiguous():
            return "f"
        return "c"

    def dataType(self):
        return {torch.float32: "FLOAT", torch.float64: "DOUBLE", torch.float16: "HALF", torch.bfloat16: "BFLOAT16",
                torch.int32: "INT", torch.int64: "LONG", torch.bool: "BOOL"}.get(self._t.dtype, str(self._t.dtype))

    def isVector(self):
        return self._t.dim() <= 2 and (self._t.dim() == 1 or 1 in self._t.shape) and self._t.numel() >= 1

    def isRowVector(self):
        return self._t.dim() == 1 or (self._t.dim() == 2 and self._t.shape[0] == 1)

    def isColumnVector(self):
        return self._t.dim() == 2 and self._t.shape[1] == 1

    def isMatrix(self):
        return self._t.dim() == 2

    def isScalar(self):
        return self._t.numel() == 1

    def isSquare(self):
        return self._t.dim() == 2 and self._t.shape[0] == self._t.shape[1]

    def isEmpty(self):
        return self._t.numel() == 0

    def isView(self):
        return self._t._base is not None

    def device(self):
        return self._t.device

    def __len__(self):
        return self._t.shape[0]

    # ------------------------------------------------------------------ copies, casts, reshapes
    def dup(self, order=None):
        if (order or self.ordering()) == "f":
            return _wrap(_f_strided(self._t))
        return _wrap(self._t.clone(memory_format=torch.contiguous_format))

    def castTo(self, dtype):
        from .factory import _dtype
        return _wrap(self._t.to(_dtype(dtype)))

    def reshape(self, *shape):
        order = "c"
        if shape and isinstance(shape[0], str):
            order, shape = shape[0], shape[1:]
        if len(shape) == 1 and isinstance(shape[0], (list, tuple)):
            shape = tuple(shape[0])
        shape = tuple(int(s) for s in shape)
        if order == "f":
            r = tuple(reversed(range(self._t.dim())))
            t = self._t.permute(*r).reshape(tuple(reversed(shape)))
            return _wrap(t.permute(*reversed(range(len(shape)))))
        return _wrap(self._t.reshape(shape))

    def ravel(self, order="c"):
        return self.reshape(order, 1, self.length())

    def flatten(self, order="c"):
        return self.ravel(order)

    def transpose(self):
        if self._t.dim() < 2:
            return _wrap(self._t.reshape(-1, 1))
        return _wrap(self._t.permute(*reversed(range(self._t.dim()))))

    def transposei(self):
        self._t = self.transpose()._t
        return self

    def permute(self, *dims):
        dims = dims[0] if len(dims) == 1 and isinstance(dims[0], (list, tuple)) else dims
        return _wrap(self._t.permute(*dims))

    def permutei(self, *dims):
        self._t = self.permute(*dims)._t
        return self

    def swapAxes(self, a, b):
        return _wrap(self._t.transpose(a, b))

    def broadcast(self, *shape):
        shape = shape[0] if len(shape) == 1 and isinstance(shape[0], (list, tuple)) else shape
        return _wrap(self._t.expand(*shape).clone())

    def repmat(self, *reps):
        reps = reps[0] if len(reps) == 1 and isinstance(reps[0], (list, tuple)) else reps
        return _wrap(self._t.repeat(*reps))

    def repeat(self, dim, n):
        return _wrap(torch.repeat_interleave(self._t, int(n), dim=dim))

    def like(self):
        return _wrap(torch.zeros_like(self._t))

    ulike = like

    def detach(self):
        return _wrap(self._t.detach().clone())

    def leverageTo(self, workspaceId=None):
        return self

    def migrate(self):
        return self

    # ------------------------------------------------------------------ element access and views
    def _index(self, idx):
        out = []
        for i in idx:
            out.append(i.to_py() if isinstance(i, NDArrayIndex) else i)
        return tuple(out)

    def get(self, *idx):
        if len(idx) == 1 and isinstance(idx[0], INDArray):          # get(indices array) along rows
            return _wrap(self._t[idx[0]._t.long().reshape(-1)])
        py = self._index(idx)
        if any(isinstance(i, list) for i in py):                     # index lists copy (like ND4J's SpecifiedIndex)
            t = self._t
            for d, i in enumerate(py):
                if isinstance(i, list):
                    t = t.index_select(d, torch.tensor(i, device=t.device))
                elif isinstance(i, slice):
                    t = t[(slice(None),) * d + (i,)]
            return _wrap(t)
        t = self._t[py]
        # ND4J keeps matrices rank 2 when a point index drops a dimension of a matrix
        if self._t.dim() == 2 and t.dim() == 1:
            t = t.reshape(1, -1) if isinstance(py[0], int) else t.reshape(-1, 1)
        return _wrap(t)

    def __getitem__(self, idx):
        if not isinstance(idx, tuple):
            idx = (idx,)
        return _wrap(self._t[self._index(idx)])

    def __setitem__(self, idx, value):
        if not isinstance(idx, tuple):
            idx = (idx,)
        with torch.no_grad():
            self._t[self._index(idx)] = _unwrap(value)

    def put(self, idx, value):
        if isinstance(idx, (list, tuple)):
            py = self._index(idx)
        else:
            py = self._index((idx,))
        v = _unwrap(value)
        with torch.no_grad():
            tgt = self._t[py]
            self._t[py] = v.reshape(tgt.shape) if torch.is_tensor(v) and v.numel() == tgt.numel() else v
        return self

    def getRow(self, i):
        return _wrap(self._t[i:i + 1] if self._t.dim() == 2 else self._t[i])

    def getColumn(self, i):
        return _wrap(self._t[:, i:i + 1])

    def getRows(self, *rows):
        rows = rows[0] if len(rows) == 1 and isinstance(rows[0], (list, tuple)) else rows
        return _wrap(self._t[list(rows)])

    def getColumns(self, *cols):
        cols = cols[0] if len(cols) == 1 and isinstance(cols[0], (list, tuple)) else cols
        return _wrap(self._t[:, list(cols)])

    def putRow(self, i, row):
        with torch.no_grad():
            self._t[i] = _unwrap(row).reshape(self._t[i].shape)
        return self

    def putColumn(self, i, col):
        with torch.no_grad():
            self._t[:, i] = _unwrap(col).reshape(self._t[:, i].shape)
        return self

    def slice(self, i, dim=0):
        return _wrap(self._t.select(dim, i))

    def slices(self):
        return self._t.shape[0]

    def tensorAlongDimension(self, index, *dims):
        """The index-th sub-tensor spanning ``dims`` (a view), iterating the other dims in c order."""
        dims = _norm_dims(dims, self._t.dim())
        other = [d for d in range(self._t.dim()) if d not in dims]
        t = self._t.permute(*other, *dims)
        lead = t.shape[:len(other)]
        idx = np.unravel_index(index, lead) if lead else ()
        return _wrap(t[tuple(int(i) for i in idx)])

    def tensorsAlongDimension(self, *dims):
        dims = _norm_dims(dims, self._t.dim())
        n = 1
        for d in range(self._t.dim()):
            if d not in dims:
                n *= self._t.shape[d]
        return n

    def vectorAlongDimension(self, index, dim):
        return self.tensorAlongDimension(index, dim)

    def getDouble(self, *idx):
        return float(self._scalar_at(idx))

    def getFloat(self, *idx):
        return float(self._scalar_at(idx))

    def getInt(self, *idx):
        return int(self._scalar_at(idx))

    def getLong(self, *idx):
        return int(self._scalar_at(idx))

    def getScalar(self, *idx):
        return _wrap(self._scalar_at(idx).reshape(1, 1))

    def _scalar_at(self, idx):
        if len(idx) == 1 and isinstance(idx[0], (list, tuple)):
            idx = tuple(idx[0])
        if len(idx) == 1 and self._t.dim() > 1:                      # linear index, c order
            return self._t.reshape(-1)[idx[0]] if self._t.is_contiguous() else self._t.flatten()[idx[0]]
        return self._t[tuple(idx)]

    def putScalar(self, *args):
        *idx, value = args
        if len(idx) == 1 and isinstance(idx[0], (list, tuple)):
            idx = list(idx[0])
        with torch.no_grad():
            if len(idx) == 1 and self._t.dim() > 1:
                pos = np.unravel_index(int(idx[0]), tuple(self._t.shape))
                self._t[tuple(int(p) for p in pos)] = value
            else:
                self._t[tuple(idx)] = value
        return self

    def assign(self, value):
        with torch.no_grad():
            v = _unwrap(value)
            if torch.is_tensor(v):
                self._t.copy_(v.reshape(self._t.shape) if v.numel() == self._t.numel() else v)
            else:
                self._t.fill_(v)
        return self

    # ------------------------------------------------------------------ arithmetic (copy and in-place forms)
    def _bin(self, other, fn, inplace, kop=None):
        """GPU operands go through the ND4J broadcast / scalar kernels (csrc/nd4j_ops.hip, ``kop``); the result of
        an in-place op is written straight into this array when the broadcast shape is its own."""
        o = _unwrap(other)
        if kop is not None and self._t.is_cuda:
            from ..ops import nd4j_kernels as K
            ob = o if torch.is_tensor(o) or isinstance(o, (int, float)) else None
            if ob is not None and not (torch.is_tensor(ob) and ob.dtype != self._t.dtype):
                if inplace:
                    if torch.is_tensor(ob) and _partial_overlap(self._t, ob):
                        # the operand is another view of this array's memory (x.subiRowVector(x.getRow(0)),
                        # x.addi(x.T)): the kernel would read elements it already overwrote, so read a copy
                        ob = ob.clone()
                    with torch.no_grad():
                        r = K.binary(self._t, ob, kop, out=self._t if self._t.is_contiguous() else None)
                        if r is not None:
                            if r is not self._t:
                                self._t.copy_(r)
                            return self
                else:
                    r = K.binary(self._t, ob, kop)
                    if r is not None:
                        return _wrap(r)
        if inplace:
            with torch.no_grad():
                r = fn(self._t, o)
                self._t.copy_(r)
            return self
        return _wrap(fn(self._t, o))

    def add(self, o):
        return self._bin(o, torch.add, False, "add")

    def addi(self, o):
        return self._bin(o, torch.add, True, "add")

    def sub(self, o):
        return self._bin(o, torch.sub, False, "sub")

    def subi(self, o):
        return self._bin(o, torch.sub, True, "sub")

    def mul(self, o):
        return self._bin(o, torch.mul, False, "mul")

    def muli(self, o):
        return self._bin(o, torch.mul, True, "mul")

    def div(self, o):
        return self._bin(o, torch.div, False, "div")

    def divi(self, o):
        return self._bin(o, torch.div, True, "div")

    def rsub(self, o):
        return self._bin(o, lambda a, b: b - a, False, "rsub")

    def rsubi(self, o):
        return self._bin(o, lambda a, b: b - a, True, "rsub")

    def rdiv(self, o):
        return self._bin(o, lambda a, b: b / a, False, "rdiv")

    def rdivi(self, o):
        return self._bin(o, lambda a, b: b / a, True, "rdiv")

    def neg(self):
        return _wrap(-self._t)

    def negi(self):
        with torch.no_grad():
            self._t.neg_()
        return self

    def fmod(self, o):
        return self._bin(o, torch.fmod, False)

    def remainder(self, o):
        return self._bin(o, torch.remainder, False)

    # row / column vector broadcasts (GPU: the ND4J broadcast kernel)
    def _vec(self, v, row):
        t = _unwrap(v)
        return t.reshape(1, -1) if row else t.reshape(-1, 1)

    def addRowVector(self, v):
        return self._bin(self._vec(v, True), torch.add, False, "add")

    def addiRowVector(self, v):
        return self._bin(self._vec(v, True), torch.add, True, "add")

    def subRowVector(self, v):
        return self._bin(self._vec(v, True), torch.sub, False, "sub")

    def subiRowVector(self, v):
        return self._bin(self._vec(v, True), torch.sub, True, "sub")

    def mulRowVector(self, v):
        return self._bin(self._vec(v, True), torch.mul, False, "mul")

    def muliRowVector(self, v):
        return self._bin(self._vec(v, True), torch.mul, True, "mul")

    def divRowVector(self, v):
        return self._bin(self._vec(v, True), torch.div, False, "div")

    def diviRowVector(self, v):
        return self._bin(self._vec(v, True), torch.div, True, "div")

    def rsubRowVector(self, v):
        return self._bin(self._vec(v, True), lambda a, b: b - a, False, "rsub")

    def rdivRowVector(self, v):
        return self._bin(self._vec(v, True), lambda a, b: b / a, False, "rdiv")

    def addColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.add, False, "add")

    def addiColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.add, True, "add")

    def subColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.sub, False, "sub")

    def subiColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.sub, True, "sub")

    def mulColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.mul, False, "mul")

    def muliColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.mul, True, "mul")

    def divColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.div, False, "div")

    def diviColumnVector(self, v):
        return self._bin(self._vec(v, False), torch.div, True, "div")

    def rsubColumnVector(self, v):
        return self._bin(self._vec(v, False), lambda a, b: b - a, False, "rsub")

    def rdivColumnVector(self, v):
        return self._bin(self._vec(v, False), lambda a, b: b / a, False, "rdiv")

    # matrix products
    def mmul(self, other, result=None):
        from ..ops.gemm import mmul as _mm
        o = _unwrap(other)
        r = _mm(self._t, o) if self._t.dim() == 2 and o.dim() == 2 else torch.matmul(self._t, o)
        if result is not None:
            result.assign(r)
            return result
        return _wrap(r)

    def mmuli(self, other, result=None):
        return self.mmul(other, result if result is not None else self)

    def dot(self, other):
        return float((self._t.reshape(-1).double() * _unwrap(other).reshape(-1).double()).sum())

    # comparisons (0/1 arrays of the same dtype, like ND4J's scalar/pairwise conditions)
    def _cmp(self, o, fn):
        return _wrap(fn(self._t, _unwrap(o)).to(self._t.dtype if self._t.is_floating_point() else torch.float32))

    def gt(self, o):
        return self._cmp(o, torch.gt)

    def gte(self, o):
        return self._cmp(o, torch.ge)

    def lt(self, o):
        return self._cmp(o, torch.lt)

    def lte(self, o):
        return self._cmp(o, torch.le)

    def eq(self, o):
        return self._cmp(o, torch.eq)

    def neq(self, o):
        return self._cmp(o, torch.ne)

    def equalsWithEps(self, other, eps):
        o = _unwrap(other)
        if not torch.is_tensor(o) or tuple(o.shape) != tuple(self._t.shape):
            return False
        return bool(((self._t.double() - o.to(self._t.device).double()).abs() <= eps).all())

    def equals(self, other):
        return self.equalsWithEps(other, 1e-5)

    __eq__ = equals

    def __hash__(self):
        return id(self)

    # python operators
    def __add__(self, o):
        return self.add(o)

    __radd__ = __add__

    def __sub__(self, o):
        return self.sub(o)

    def __rsub__(self, o):
        return self.rsub(o)

    def __mul__(self, o):
        return self.mul(o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self.div(o)

    def __rtruediv__(self, o):
        return self.rdiv(o)

    def __matmul__(self, o):
        return self.mmul(o)

    def __neg__(self):
        return self.neg()

    def __iadd__(self, o):
        return self.addi(o)

    def __isub__(self, o):
        return self.subi(o)

    def __imul__(self, o):
        return self.muli(o)

    def __itruediv__(self, o):
        return self.divi(o)

    # ------------------------------------------------------------------ reductions
    def _red(self, fn, dims, keep2d=True, kop=None, bias_corrected=True):
        t = self._t
        if kop is not None and t.is_cuda and t.is_floating_point():
            from ..ops import nd4j_kernels as K
            whole = not dims or (len(dims) == 1 and dims[0] == 2147483647)
            r = K.reduce(t, kop, None if whole else _norm_dims(dims, t.dim()), bias_corrected=bias_corrected)
            if r is not None:
                return _wrap(r.reshape(1, 1) if whole else (_as_2d(r) if keep2d else r))
        if not t.is_floating_point():
            t = t.double()
        if not dims or (len(dims) == 1 and dims[0] == 2147483647):       # Integer.MAX_VALUE = whole array
            return _wrap(fn(t, None).reshape(1, 1))
        dims = _norm_dims(dims, t.dim())
        r = fn(t, dims)
        return _wrap(_as_2d(r) if keep2d else r)

    def sum(self, *dims):
        return self._red(lambda t, d: t.sum() if d is None else t.sum(d), dims, kop="sum")

    def mean(self, *dims):
        return self._red(lambda t, d: t.mean() if d is None else t.mean(d), dims, kop="mean")

    def prod(self, *dims):
        return self._red(lambda t, d: t.prod() if d is None else _multi(torch.prod, t, d), dims, kop="prod")

    def max(self, *dims):
        return self._red(lambda t, d: t.max() if d is None else t.amax(d), dims, kop="max")

    def min(self, *dims):
        return self._red(lambda t, d: t.min() if d is None else t.amin(d), dims, kop="min")

    def amax(self, *dims):
        return self._red(lambda t, d: t.abs().max() if d is None else t.abs().amax(d), dims, kop="amax")

    def amin(self, *dims):
        return self._red(lambda t, d: t.abs().min() if d is None else t.abs().amin(d), dims, kop="amin")

    def std(self, *dims, biasCorrected=True):
        if dims and isinstance(dims[0], bool):
            biasCorrected, dims = dims[0], dims[1:]
        c = 1 if biasCorrected else 0
        return self._red(lambda t, d: t.std(correction=c) if d is None else t.std(d, correction=c), dims,
                         kop="std", bias_corrected=biasCorrected)

    def var(self, *dims, biasCorrected=True):
        if dims and isinstance(dims[0], bool):
            biasCorrected, dims = dims[0], dims[1:]
        c = 1 if biasCorrected else 0
        return self._red(lambda t, d: t.var(correction=c) if d is None else t.var(d, correction=c), dims,
                         kop="var", bias_corrected=biasCorrected)

    def norm1(self, *dims):
        return self._red(lambda t, d: t.abs().sum() if d is None else t.abs().sum(d), dims, kop="norm1")

    def norm2(self, *dims):
        return self._red(lambda t, d: t.pow(2).sum().sqrt() if d is None else t.pow(2).sum(d).sqrt(), dims,
                         kop="norm2")

    def normmax(self, *dims):
        return self.amax(*dims)

    def argMax(self, *dims):
        if self._t.is_cuda and self._t.is_floating_point():
            from ..ops import nd4j_kernels as K
            r = K.reduce(self._t, "argmax", [dims[0]] if dims else None)
            if r is not None:
                return _wrap(r.reshape(1, 1) if not dims else _as_2d(r))
        if not dims:
            return _wrap(self._t.reshape(-1).argmax().reshape(1, 1))
        return _wrap(_as_2d(self._t.argmax(dims[0])))

    def argMin(self, *dims):
        if self._t.is_cuda and self._t.is_floating_point():
            from ..ops import nd4j_kernels as K
            r = K.reduce(self._t, "argmin", [dims[0]] if dims else None)
            if r is not None:
                return _wrap(r.reshape(1, 1) if not dims else _as_2d(r))
        if not dims:
            return _wrap(self._t.reshape(-1).argmin().reshape(1, 1))
        return _wrap(_as_2d(self._t.argmin(dims[0])))

    def cumsum(self, dim):
        return _wrap(self._t.cumsum(dim))

    def cumsumi(self, dim):
        with torch.no_grad():
            self._t.copy_(self._t.cumsum(dim))
        return self

    def sumNumber(self):
        return float(self._t.double().sum())

    def meanNumber(self):
        return float(self._t.double().mean())

    def maxNumber(self):
        return float(self._t.max())

    def minNumber(self):
        return float(self._t.min())

    def prodNumber(self):
        return float(self._t.double().prod())

    def stdNumber(self):
        return float(self._t.double().std())

    def varNumber(self):
        return float(self._t.double().var())

    def norm1Number(self):
        return float(self._t.double().abs().sum())

    def norm2Number(self):
        return float(self._t.double().pow(2).sum().sqrt())

    def normmaxNumber(self):
        return float(self._t.double().abs().max())

    def amaxNumber(self):
        return self.normmaxNumber()

    def scan(self, condition):
        return int(condition(self._t).sum())

    # distances
    def distance1(self, o):
        return float((self._t.double() - _unwrap(o).double()).abs().sum())

    def distance2(self, o):
        return math.sqrt(self.squaredDistance(o))

    def squaredDistance(self, o):
        return float((self._t.double() - _unwrap(o).double()).pow(2).sum())


def _multi(fn, t, dims):
    for d in sorted(dims, reverse=True):
        t = fn(t, d)
    return t


class Transforms:
    """``org.nd4j.linalg.ops.transforms.Transforms``: elementwise transforms (``dup`` flag = copy or in place) and
    vector similarity helpers."""

    @staticmethod
    def _apply(x, fn, dup=True, kop=None, a0=0.0, a1=0.0):
        """GPU arrays run the ND4J transform kernel ``kop`` (csrc/nd4j_ops.hip), in place when ``dup`` is False."""
        t = _unwrap(x)
        if kop is not None and torch.is_tensor(t) and t.is_cuda:
            from ..ops import nd4j_kernels as K
            with torch.no_grad():
                r = K.transform(t, kop, a0, a1, out=None if dup or not t.is_contiguous() else t)
            if r is not None:
                if dup:
                    return _wrap(r)
                if r is not t:
                    with torch.no_grad():
                        x._t.copy_(r)
                return x
        if dup:
            return _wrap(fn(t))
        with torch.no_grad():
            x._t.copy_(fn(x._t))
        return x

    sigmoid = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.sigmoid, dup, "sigmoid"))
    tanh = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.tanh, dup, "tanh"))
    relu = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.relu, dup, "relu"))
    exp = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.exp, dup, "exp"))
    log = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.log, dup, "log"))
    abs = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.abs, dup, "abs"))
    sqrt = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.sqrt, dup, "sqrt"))
    sign = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.sign, dup, "sign"))
    floor = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.floor, dup, "floor"))
    ceil = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.ceil, dup, "ceil"))
    round = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.round, dup, "round"))
    sin = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.sin, dup, "sin"))
    cos = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.cos, dup, "cos"))
    acos = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.acos, dup, "acos"))
    asin = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.asin, dup, "asin"))
    atan = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.atan, dup, "atan"))
    softplus = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.nn.functional.softplus, dup, "softplus"))
    softsign = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.nn.functional.softsign, dup, "softsign"))
    elu = staticmethod(lambda x, dup=True: Transforms._apply(x, torch.nn.functional.elu, dup, "elu", 1.0))
    hardTanh = staticmethod(lambda x, dup=True: Transforms._apply(x, lambda t: t.clamp(-1, 1), dup, "hardtanh"))
    identity = staticmethod(lambda x, dup=True: Transforms._apply(x, lambda t: t, dup))
    stabilize = staticmethod(lambda x, k=1.0, dup=True: Transforms._apply(
        x, lambda t: t.clamp(-1e4 / k, 1e4 / k), dup))

    @staticmethod
    def leakyRelu(x, alpha=0.01, dup=True):
        return Transforms._apply(x, lambda t: torch.nn.functional.leaky_relu(t, alpha), dup, "leakyrelu", alpha)

    @staticmethod
    def pow(x, p, dup=True):
        return Transforms._apply(x, lambda t: torch.pow(t, _unwrap(p)), dup)

    @staticmethod
    def max(x, v, dup=True):
        return Transforms._apply(x, lambda t: torch.clamp(t, min=v) if not isinstance(v, INDArray)
                                 else torch.maximum(t, v._t), dup)

    @staticmethod
    def min(x, v, dup=True):
        return Transforms._apply(x, lambda t: torch.clamp(t, max=v) if not isinstance(v, INDArray)
                                 else torch.minimum(t, v._t), dup)

    @staticmethod
    def softmax(x, dup=True):
        """Row-wise softmax (ND4J's SoftMax over the last dimension of a matrix)."""
        return Transforms._apply(x, lambda t: torch.softmax(t, dim=-1), dup)

    @staticmethod
    def exp_(x):
        return Transforms.exp(x, False)

    @staticmethod
    def not_(x):
        return _wrap((_unwrap(x) == 0).to(_unwrap(x).dtype))

    @staticmethod
    def unitVec(x):
        t = _unwrap(x)
        n = t.double().pow(2).sum().sqrt()
        return _wrap(t if float(n) == 0 else t / n.to(t.dtype))

    @staticmethod
    def normalizeZeroMeanAndUnitVariance(x):
        t = _unwrap(x)
        return _wrap((t - t.mean(0, keepdim=True)) / (t.std(0, keepdim=True) + 1e-12))

    @staticmethod
    def dot(a, b):
        return _unwrap(a).reshape(-1).double().dot(_unwrap(b).reshape(-1).double()).item()

    @staticmethod
    def cosineSim(a, b):
        x, y = _unwrap(a).reshape(-1).double(), _unwrap(b).reshape(-1).double()
        return float(x.dot(y) / (x.norm() * y.norm()))

    @staticmethod
    def cosineDistance(a, b):
        return 1.0 - Transforms.cosineSim(a, b)

    @staticmethod
    def euclideanDistance(a, b):
        return float((_unwrap(a).double() - _unwrap(b).double()).pow(2).sum().sqrt())

    @staticmethod
    def manhattanDistance(a, b):
        return float((_unwrap(a).double() - _unwrap(b).double()).abs().sum())

    @staticmethod
    def allCosineSimilarities(a, b):
        """Pairwise cosine similarity of the rows of a and b: [rows(a), rows(b)]."""
        x, y = _unwrap(a).double(), _unwrap(b).double()
        x = x / x.norm(dim=1, keepdim=True).clamp_min(1e-300)
        y = y / y.norm(dim=1, keepdim=True).clamp_min(1e-300)
        return _wrap(x @ y.t())

    @staticmethod
    def allEuclideanDistances(a, b):
        return _wrap(torch.cdist(_unwrap(a).double(), _unwrap(b).double()))
