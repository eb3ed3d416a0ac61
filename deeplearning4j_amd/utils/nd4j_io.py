"""ND4J binary array codec (``Nd4j.write`` / ``Nd4j.read``) used by ModelSerializer's coefficients.bin and
updaterState.bin entries (reference NN:util/ModelSerializer.java:109-170; the format itself lives in ND4J).

Layout (Java DataOutputStream, big-endian):
  shape-info buffer:  writeUTF(allocMode) | int length | writeUTF("INT") | length x int
                      values = [rank, shape..., stride..., offset, elementWiseStride, order('c'=99/'f'=102)]
  data buffer:        writeUTF(allocMode) | int length | writeUTF(dtype) | length x value
                      dtype in {"FLOAT","DOUBLE","INT","HALF","LONG"}
"""
import io
import struct

import numpy as np
import torch


def _write_utf(out, s):
    b = s.encode("utf-8")
    out.write(struct.pack(">H", len(b)))
    out.write(b)


def _read_utf(inp):
    (n,) = struct.unpack(">H", inp.read(2))
    return inp.read(n).decode("utf-8")


_DT_NP = {"FLOAT": ">f4", "DOUBLE": ">f8", "INT": ">i4", "LONG": ">i8", "HALF": ">f2"}


def _write_buffer(out, values, dtype_name):
    _write_utf(out, "HEAP")
    out.write(struct.pack(">i", int(values.size)))
    _write_utf(out, dtype_name)
    out.write(np.ascontiguousarray(values, dtype=_DT_NP[dtype_name]).tobytes())


def _read_buffer(inp):
    _read_utf(inp)                       # allocation mode (HEAP/DIRECT/JAVACPP) - irrelevant here
    (n,) = struct.unpack(">i", inp.read(4))
    dt = _read_utf(inp)
    if dt == "COMPRESSED":
        raise ValueError("Compressed ND4J buffers are not supported")
    np_dt = np.dtype(_DT_NP[dt])
    arr = np.frombuffer(inp.read(n * np_dt.itemsize), dtype=np_dt)
    return arr, dt


def write(arr, out, order="c"):
    """Write a tensor/ndarray/INDArray in ND4J's binary format to a binary stream ``out``."""
    if hasattr(arr, "toTensor"):
        arr = arr.toTensor()
    if torch.is_tensor(arr):
        t = arr.detach().cpu()
        if t.dtype == torch.bfloat16:
            t = t.float()
        a = t.numpy()
    else:
        a = np.asarray(arr)
    if a.ndim == 1:
        a = a.reshape(1, -1)
    rank = a.ndim
    shape = list(a.shape)
    if order == "f":
        strides, acc = [], 1
        for s in shape:
            strides.append(acc)
            acc *= s
        flat = np.asfortranarray(a).reshape(-1, order="F")
    else:
        strides, acc = [], 1
        for s in reversed(shape):
            strides.insert(0, acc)
            acc *= s
        flat = a.reshape(-1)
    info = np.array([rank] + shape + strides + [0, 1, ord(order)], dtype=np.int64)
    _write_buffer(out, info, "INT")
    dt = {np.float32: "FLOAT", np.float64: "DOUBLE", np.int32: "INT", np.int64: "LONG", np.float16: "HALF"}.get(
        a.dtype.type, "FLOAT")
    _write_buffer(out, flat, dt)


def read(inp):
    """Read one ND4J array from a binary stream; returns a torch tensor (fp32/fp64/int)."""
    info, _ = _read_buffer(inp)
    info = info.astype(np.int64)
    rank = int(info[0])
    shape = [int(s) for s in info[1:1 + rank]]
    order = chr(int(info[-1])) if int(info[-1]) in (99, 102) else "c"
    data, dt = _read_buffer(inp)
    data = data.astype(data.dtype.newbyteorder("="))
    a = data.reshape(shape, order="F" if order == "f" else "C")
    return torch.from_numpy(np.ascontiguousarray(a))


def to_bytes(arr, order="c"):
    b = io.BytesIO()
    write(arr, b, order)
    return b.getvalue()


def from_bytes(b):
    return read(io.BytesIO(b))


# The Nd4j factory namespace lives in deeplearning4j_amd.nd4j (INDArray API); re-exported for existing imports.
from ..nd4j.factory import Nd4j  # noqa: E402,F401
