"""A self-contained, read-only HDF5 reader — enough of the format for Keras model files.

The reference reads Keras HDF5 through the JavaCPP hdf5 preset (KER:Hdf5Archive.java:48-120). No HDF5 binding
is importable here, so this module parses the file format directly (HDF5 File Format Specification v3):
  * superblock versions 0, 1, 2, 3
  * object headers v1 and v2 (with continuation blocks)
  * groups: symbol-table ("old style": v1 B-tree + local heap) and link-message ("compact new style")
  * attributes (message 0x000C v1-v3), fixed-length and variable-length strings (global heap), numerics
  * datasets: compact / contiguous / chunked (v1 B-tree index) layouts, deflate + shuffle (+ fletcher32 strip)
  * datatypes: fixed-point, IEEE float (little/big endian), fixed & variable-length strings
Dense (fractal-heap) link or attribute storage raises NotImplementedError with a clear message.

API: ``File(path)`` -> root ``Group``; ``group["a/b"]`` -> Group or Dataset; ``.attrs`` dict; ``Dataset.read()``
-> numpy array; ``keys()``, ``visit()``.
"""
import struct
import zlib

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"


class HDF5Error(Exception):
    pass


class _Reader:
    def __init__(self, data):
        self.d = data
        self.so = 8     # size of offsets
        self.sl = 8     # size of lengths

    def u(self, off, n):
        return int.from_bytes(self.d[off:off + n], "little")

    def addr(self, off):
        return self.u(off, self.so)

    def length(self, off):
        return self.u(off, self.sl)

    @staticmethod
    def undefined(a, n=8):
        return a == (1 << (8 * n)) - 1


# --------------------------------------------------------------------------------------------- datatypes
class DType:
    def __init__(self, cls, size, bits, props, base=None, little=True, signed=True, strpad=0, charset=0):
        self.cls, self.size, self.bits, self.props = cls, size, bits, props
        self.base, self.little, self.signed, self.strpad, self.charset = base, little, signed, strpad, charset

    def numpy(self):
        e = "<" if self.little else ">"
        if self.cls == 0:
            return np.dtype(f"{e}{'i' if self.signed else 'u'}{self.size}")
        if self.cls == 1:
            return np.dtype(f"{e}f{self.size}")
        if self.cls == 3:
            return np.dtype(f"S{self.size}")
        raise HDF5Error(f"unsupported datatype class {self.cls}")


def _parse_dtype(r, off):
    cv = r.d[off]
    cls, ver = cv & 0x0F, cv >> 4
    b0, b1, b2 = r.d[off + 1], r.d[off + 2], r.d[off + 3]
    bits = b0 | (b1 << 8) | (b2 << 16)
    size = r.u(off + 4, 4)
    p = off + 8
    if cls == 0:          # fixed point
        return DType(0, size, bits, None, little=not (bits & 1), signed=bool(bits & 0x8)), p + 4
    if cls == 1:          # floating point
        return DType(1, size, bits, None, little=not (bits & 1)), p + 12
    if cls == 3:          # string
        return DType(3, size, bits, None, strpad=bits & 0xF, charset=(bits >> 4) & 0xF), p
    if cls == 9:          # variable length
        base, q = _parse_dtype(r, p)
        return DType(9, size, bits, None, base=base, strpad=(bits >> 8) & 0xF), q
    if cls == 6:          # compound: not needed for Keras files
        return DType(6, size, bits, None), p
    if cls in (4, 5, 7, 8, 10):
        return DType(cls, size, bits, None), p
    raise HDF5Error(f"unknown datatype class {cls} (version {ver})")


def _parse_dataspace(r, off):
    ver = r.d[off]
    rank = r.d[off + 1]
    flags = r.d[off + 2]
    if ver == 1:
        p = off + 8
    elif ver == 2:
        if r.d[off + 3] == 2:        # null dataspace
            return None
        p = off + 4
    else:
        raise HDF5Error(f"dataspace version {ver}")
    dims = tuple(r.length(p + i * r.sl) for i in range(rank))
    _ = flags
    return dims


# --------------------------------------------------------------------------------------------- objects
class _Message:
    __slots__ = ("type", "off", "size")

    def __init__(self, t, off, size):
        self.type, self.off, self.size = t, off, size


def _object_messages(r, addr):
    d = r.d
    msgs = []
    if d[addr:addr + 4] == b"OHDR":
        ver = d[addr + 4]
        flags = d[addr + 5]
        p = addr + 6
        if flags & 0x20:
            p += 16
        if flags & 0x10:
            p += 4
        csz = 1 << (flags & 3)
        size0 = r.u(p, csz)
        p += csz
        blocks = [(p, size0)]
        _ = ver
        while blocks:
            start, size = blocks.pop(0)
            q, end = start, start + size
            while q + 4 <= end:
                t = d[q]
                sz = r.u(q + 1, 2)
                mflags = d[q + 3]
                q += 4
                if flags & 0x04:
                    q += 2
                if t == 0x10:
                    coff, clen = r.addr(q), r.length(q + r.so)
                    blocks.append((coff + 4, clen - 8))       # skip "OCHK" and trailing checksum
                elif t != 0:
                    msgs.append(_Message(t, q, sz))
                _ = mflags
                q += sz
        return msgs
    ver = d[addr]
    if ver != 1:
        raise HDF5Error(f"unsupported object header version {ver} at {addr}")
    nmsg = r.u(addr + 2, 2)
    hsize = r.u(addr + 8, 4)
    blocks = [(addr + 16, hsize)]
    count = 0
    while blocks and count < nmsg:
        start, size = blocks.pop(0)
        q, end = start, start + size
        while q + 8 <= end and count < nmsg:
            t = r.u(q, 2)
            sz = r.u(q + 2, 2)
            q += 8
            count += 1
            if t == 0x10:
                blocks.append((r.addr(q), r.length(q + r.so)))
            elif t != 0:
                msgs.append(_Message(t, q, sz))
            q += sz
    return msgs


class _Node:
    def __init__(self, f, addr, name):
        self._f, self.addr, self.name = f, addr, name
        self._msgs = _object_messages(f._r, addr)
        self._attrs = None

    @property
    def attrs(self):
        if self._attrs is None:
            self._attrs = {}
            for m in self._msgs:
                if m.type == 0x000C:
                    k, v = self._f._attribute(m.off)
                    self._attrs[k] = v
                elif m.type == 0x0015:
                    fh = self._f._r.addr(m.off + 2 + (2 if self._f._r.d[m.off + 1] & 1 else 0))
                    if not _Reader.undefined(fh):
                        raise NotImplementedError("dense (fractal heap) attribute storage is not supported")
        return self._attrs


class Dataset(_Node):
    def __init__(self, f, addr, name):
        super().__init__(f, addr, name)
        r = f._r
        self.shape, self.dtype, self.layout, self.filters = None, None, None, []
        for m in self._msgs:
            if m.type == 0x0001:
                self.shape = _parse_dataspace(r, m.off)
            elif m.type == 0x0003:
                self.dtype, _ = _parse_dtype(r, m.off)
            elif m.type == 0x0008:
                self.layout = m.off
            elif m.type == 0x000B:
                self.filters = _parse_filters(r, m.off)

    def read(self):
        f, r = self._f, self._f._r
        shape = self.shape or ()
        n = int(np.prod(shape)) if shape else 1
        dt = self.dtype
        esz = dt.size
        raw = _read_layout(f, self.layout, shape, esz, self.filters)
        if dt.cls == 9:
            return _read_vlen(f, raw, n, dt).reshape(shape)
        arr = np.frombuffer(raw[:n * esz], dtype=dt.numpy()).reshape(shape)
        return arr.astype(arr.dtype.newbyteorder("=")) if not dt.little else arr.copy()

    def __repr__(self):
        return f"<HDF5 dataset {self.name!r}: shape {self.shape}, type {self.dtype.numpy() if self.dtype.cls in (0, 1, 3) else self.dtype.cls}>"


class Group(_Node):
    def __init__(self, f, addr, name, stab=None):
        super().__init__(f, addr, name)
        self._links = None
        self._stab = stab

    def _load_links(self):
        if self._links is not None:
            return
        r = self._f._r
        links = {}
        stab = self._stab
        for m in self._msgs:
            if m.type == 0x0011:
                stab = (r.addr(m.off), r.addr(m.off + r.so))
            elif m.type == 0x0006:
                nm, a = _parse_link(r, m.off)
                if a is not None:
                    links[nm] = a
            elif m.type == 0x0002:
                ver_flags = r.d[m.off + 1]
                p = m.off + 2 + (8 if ver_flags & 1 else 0)
                if not _Reader.undefined(r.addr(p)):
                    raise NotImplementedError("dense (fractal heap) link storage is not supported")
        if stab is not None:
            links.update(self._f._symbol_table(*stab))
        self._links = links

    def keys(self):
        self._load_links()
        return list(self._links.keys())

    def __contains__(self, k):
        try:
            self[k]
            return True
        except KeyError:
            return False

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, Group):
                raise KeyError(path)
            node._load_links()
            if part not in node._links:
                raise KeyError(path)
            node = node._f._open(node._links[part], (node.name.rstrip("/") + "/" + part))
        return node

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def visit(self, fn, prefix=""):
        for k, v in self.items():
            p = prefix + k
            fn(p, v)
            if isinstance(v, Group):
                v.visit(fn, p + "/")

    def __repr__(self):
        return f"<HDF5 group {self.name!r} ({len(self.keys())} members)>"


def _parse_link(r, off):
    flags = r.d[off + 1]
    p = off + 2
    ltype = 0
    if flags & 0x08:
        ltype = r.d[p]
        p += 1
    if flags & 0x04:
        p += 8
    if flags & 0x10:
        p += 1
    ln = 1 << (flags & 3)
    nlen = r.u(p, ln)
    p += ln
    name = r.d[p:p + nlen].decode("utf-8")
    p += nlen
    if ltype == 0:
        return name, r.addr(p)
    return name, None       # soft / external links are ignored


def _parse_filters(r, off):
    ver = r.d[off]
    n = r.d[off + 1]
    p = off + (8 if ver == 1 else 2)
    out = []
    for _ in range(n):
        fid = r.u(p, 2)
        if ver == 1 or fid >= 256:
            nlen = r.u(p + 2, 2)
            flags, nvals = r.u(p + 4, 2), r.u(p + 6, 2)
            p += 8
            p += (nlen + 7) // 8 * 8 if ver == 1 else nlen
        else:
            flags, nvals = r.u(p + 2, 2), r.u(p + 4, 2)
            p += 6
        vals = [r.u(p + 4 * i, 4) for i in range(nvals)]
        p += 4 * nvals
        if ver == 1 and nvals % 2:
            p += 4
        out.append((fid, flags, vals))
    return out


def _unfilter(buf, filters, esz):
    for fid, flags, vals in reversed(filters):
        if fid == 1:
            buf = zlib.decompress(buf)
        elif fid == 2:          # shuffle
            size = vals[0] if vals else esz
            a = np.frombuffer(buf, dtype=np.uint8)
            n = len(a) // size
            body = a[:n * size].reshape(size, n).T.reshape(-1)
            buf = body.tobytes() + a[n * size:].tobytes()
        elif fid == 3:          # fletcher32: drop the trailing checksum
            buf = buf[:-4]
        else:
            raise NotImplementedError(f"HDF5 filter {fid} not supported")
    return buf


def _read_layout(f, off, shape, esz, filters):
    r = f._r
    d = r.d
    ver = d[off]
    n = int(np.prod(shape)) if shape else 1
    nbytes = n * esz
    if ver == 3:
        cls = d[off + 1]
        if cls == 0:
            sz = r.u(off + 2, 2)
            return bytes(d[off + 4:off + 4 + sz])
        if cls == 1:
            a = r.addr(off + 2)
            if _Reader.undefined(a):
                return bytes(nbytes)
            return bytes(d[a:a + nbytes])
        if cls == 2:
            rank = d[off + 2]
            bt = r.addr(off + 3)
            cdims = [r.u(off + 3 + r.so + 4 * i, 4) for i in range(rank)]
            return _read_chunked(f, bt, shape, cdims[:-1], esz, filters)
        raise HDF5Error(f"layout class {cls}")
    if ver in (1, 2):
        rank = d[off + 1]
        cls = d[off + 2]
        p = off + 8
        if cls != 0:
            a = r.addr(p)
            p += r.so
        dims = [r.u(p + 4 * i, 4) for i in range(rank)]
        p += 4 * rank
        if cls == 0:
            sz = r.u(p, 4)
            return bytes(d[p + 4:p + 4 + sz])
        if cls == 1:
            return bytes(d[a:a + nbytes])
        return _read_chunked(f, a, shape, dims[:-1] if len(dims) > len(shape) else dims, esz, filters)
    raise NotImplementedError(f"data layout message version {ver} (HDF5 1.10 chunk indexes) not supported")


def _read_chunked(f, btree, shape, cdims, esz, filters):
    r = f._r
    out = np.zeros(int(np.prod(shape)) * esz if shape else esz, dtype=np.uint8)
    rank = len(shape)
    full = np.frombuffer(out, dtype=np.uint8)
    arr = out.reshape(tuple(shape) + (esz,)) if shape else out.reshape((esz,))
    _ = full

    def walk(addr):
        d = r.d
        if d[addr:addr + 4] != b"TREE":
            raise HDF5Error("bad chunk B-tree node")
        level = d[addr + 5]
        used = r.u(addr + 6, 2)
        p = addr + 8 + 2 * r.so
        ksz = 8 + 8 * (rank + 1)
        for i in range(used):
            key = p + i * (ksz + r.so)
            csize = r.u(key, 4)
            fmask = r.u(key + 4, 4)
            offs = [r.u(key + 8 + 8 * j, 8) for j in range(rank)]
            child = r.addr(key + ksz)
            if level > 0:
                walk(child)
                continue
            raw = bytes(d[child:child + csize])
            active = [flt for k, flt in enumerate(filters) if not (fmask >> k) & 1]
            raw = _unfilter(raw, active, esz) if active else raw
            chunk = np.frombuffer(raw, dtype=np.uint8)[:int(np.prod(cdims)) * esz].reshape(tuple(cdims) + (esz,))
            sl_out = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
            sl_in = tuple(slice(0, s.stop - s.start) for s in sl_out)
            arr[sl_out] = chunk[sl_in]
    walk(btree)
    return out.tobytes()


def _read_vlen(f, raw, n, dt):
    r = f._r
    out = []
    step = 4 + r.so + 4
    for i in range(n):
        p = i * step
        ln = int.from_bytes(raw[p:p + 4], "little")
        coll = int.from_bytes(raw[p + 4:p + 4 + r.so], "little")
        idx = int.from_bytes(raw[p + 4 + r.so:p + step], "little")
        b = f._global_heap_object(coll, idx)[:ln * (dt.base.size if dt.base is not None else 1)]
        if dt.base is not None and dt.base.cls == 3 or (dt.bits & 0xF) == 1:
            out.append(b.decode("utf-8", "replace"))
        else:
            out.append(np.frombuffer(b, dtype=dt.base.numpy()))
    return np.array(out, dtype=object)


class File(Group):
    def __init__(self, path_or_bytes):
        if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
            data = bytes(path_or_bytes)
        else:
            with open(path_or_bytes, "rb") as fh:
                data = fh.read()
        base = data.find(SIG)
        if base < 0:
            raise HDF5Error("not an HDF5 file")
        if base:
            data = data[base:]
        r = self._r = _Reader(data)
        self._gheap = {}
        ver = data[8]
        if ver in (0, 1):
            r.so, r.sl = data[13], data[14]
            p = 24 + (4 if ver == 1 else 0)
            root_entry = p + 4 * r.so
            root_addr = r.addr(root_entry + r.so)
            ctype = r.u(root_entry + 2 * r.so, 4)
            stab = None
            if ctype == 1:
                sp = root_entry + 2 * r.so + 8
                stab = (r.addr(sp), r.addr(sp + r.so))
            Group.__init__(self, self, root_addr, "/", stab)
        elif ver in (2, 3):
            r.so, r.sl = data[9], data[10]
            p = 12
            root_addr = r.addr(p + 3 * r.so)
            Group.__init__(self, self, root_addr, "/")
        else:
            raise HDF5Error(f"superblock version {ver}")
        self.filename = None if isinstance(path_or_bytes, (bytes, bytearray, memoryview)) else str(path_or_bytes)

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    # ------------------------------------------------------------------ internals
    def _open(self, addr, name):
        msgs = _object_messages(self._r, addr)
        types = {m.type for m in msgs}
        if 0x0008 in types:
            return Dataset(self, addr, name)
        return Group(self, addr, name)

    def _symbol_table(self, btree, heap):
        r = self._r
        d = r.d
        if d[heap:heap + 4] != b"HEAP":
            raise HDF5Error("bad local heap")
        heap_data = r.addr(heap + 8 + 2 * r.sl)

        def name_at(off):
            s = heap_data + off
            e = d.index(b"\0", s)
            return d[s:e].decode("utf-8")
        links = {}

        def walk(addr):
            if d[addr:addr + 4] == b"TREE":
                level = d[addr + 5]
                used = r.u(addr + 6, 2)
                p = addr + 8 + 2 * r.so
                for i in range(used):
                    child = r.addr(p + r.sl + i * (r.sl + r.so))
                    walk(child) if level >= 0 else None
                return
            if d[addr:addr + 4] == b"SNOD":
                nsym = r.u(addr + 6, 2)
                p = addr + 8
                esz = 2 * r.so + 4 + 4 + 16
                for i in range(nsym):
                    e = p + i * esz
                    links[name_at(r.addr(e))] = r.addr(e + r.so)
                return
            raise HDF5Error(f"unexpected group node at {addr}")
        walk(btree)
        return links

    def _attribute(self, off):
        r = self._r
        d = r.d
        ver = d[off]
        nsz, tsz, ssz = r.u(off + 2, 2), r.u(off + 4, 2), r.u(off + 6, 2)
        if ver == 1:
            p = off + 8
            pad = lambda x: (x + 7) // 8 * 8  # noqa: E731
        else:
            p = off + 8 + (1 if ver == 3 else 0)
            pad = lambda x: x  # noqa: E731
        name = d[p:p + nsz].split(b"\0")[0].decode("utf-8")
        p += pad(nsz)
        dt, _ = _parse_dtype(r, p)
        p += pad(tsz)
        shape = _parse_dataspace(r, p)
        p += pad(ssz)
        n = int(np.prod(shape)) if shape else 1
        if dt.cls == 9:
            vals = _read_vlen(self, bytes(d[p:p + n * (8 + r.so)]), n, dt)
            return name, (vals[0] if not shape else vals.reshape(shape))
        raw = bytes(d[p:p + n * dt.size])
        arr = np.frombuffer(raw, dtype=dt.numpy())
        if not shape:
            v = arr[0]
            return name, (v.decode("utf-8") if isinstance(v, bytes) else v.item() if hasattr(v, "item") else v)
        arr = arr.reshape(shape)
        if dt.cls == 3:
            return name, np.array([x.decode("utf-8") for x in arr.reshape(-1)], dtype=object).reshape(shape)
        return name, arr.copy()

    def _global_heap_object(self, coll, idx):
        if coll not in self._gheap:
            r = self._r
            d = r.d
            if d[coll:coll + 4] != b"GCOL":
                raise HDF5Error("bad global heap collection")
            size = r.length(coll + 8)
            objs = {}
            p = coll + 8 + r.sl
            end = coll + size
            while p + 8 + r.sl <= end:
                oid = r.u(p, 2)
                if oid == 0:
                    break
                osz = r.length(p + 8)
                objs[oid] = bytes(d[p + 8 + r.sl:p + 8 + r.sl + osz])
                p += 8 + r.sl + (osz + 7) // 8 * 8
            self._gheap[coll] = objs
        return self._gheap[coll][idx]
