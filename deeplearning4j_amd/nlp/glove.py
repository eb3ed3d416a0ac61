"""GloVe: co-occurrence counting (native C++) + AdaGrad weighted least squares (gfx950 kernel / threaded C++).

Reference: NLP:models/glove/Glove.java (Builder: xMax 100, alpha 0.75, learningRate 0.05, symmetric, shuffle),
models/glove/AbstractCoOccurrences.java (windowed co-occurrences weighted 1/distance),
models/embeddings/learning/impl/elements/GloVe.java:182-225 (tied word/context matrix, per-row bias, AdaGrad on
both; loss f(x)(w_i.w_j + b_i + b_j - log x)^2 with f(x) = min(1, (x/xMax)^alpha)).
"""
import ctypes

import numpy as np
import torch

from ..ops import runtime as RT
from .embeddings import InMemoryLookupTable, _np_ptr, _t_ptr
from .word2vec import Word2Vec, _BaseBuilder

c_void_p, c_int, c_ll, c_float, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, \
    ctypes.c_double
RT.register("rt_glove_cooccur_new", [c_void_p, c_void_p, c_ll, c_int, c_int], c_void_p)
RT.register("rt_glove_cooccur_size", [c_void_p], c_ll)
RT.register("rt_glove_cooccur_fetch", [c_void_p, c_void_p, c_void_p, c_void_p, c_ll], c_ll)
RT.register("rt_glove_cooccur_free", [c_void_p], None)
RT.register("rt_glove_apply", [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                               c_float, c_float, c_float, c_int], c_double)


RT.register("rt_cooc_new", [ctypes.c_char_p, c_ll], c_void_p)
RT.register("rt_cooc_add", [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_int], c_int)
RT.register("rt_cooc_spills", [c_void_p], c_ll)
RT.register("rt_cooc_finish", [c_void_p, ctypes.c_char_p], c_ll)
RT.register("rt_cooc_free", [c_void_p], None)

# one merged co-occurrence record as the native counter writes it
COOC_DTYPE = np.dtype([("i", "<i4"), ("j", "<i4"), ("x", "<f4")])
_BYTES_PER_ENTRY = 64          # hash-map footprint per counted pair (key, value, bucket, node) for the memory cap


class RoundCount:
    """Cyclic counter 0..limit (reference models/glove/count/RoundCount.java): the shadow-copy thread of the
    co-occurrence counter alternates spill files by round; previous() is the round before the current one."""

    def __init__(self, limit):
        self.limit, self.current = int(limit), 0

    def previous(self):
        return self.limit if self.current == 0 else self.current - 1

    def get(self):
        return self.current

    def tick(self):
        self.current = 0 if self.current == self.limit else self.current + 1


class CoOccurrenceCounter:
    """Co-occurrence counting with bounded memory (reference NLP:models/glove/AbstractCoOccurrences.java:55-104,
    185-266, 387-520: its maxMemory-triggered shadow copies to temp files). Sequences are fed in chunks
    (``add``); the native counter (csrc/runtime/cooccur.cpp) keeps at most ``maxEntries`` pairs in its hash map and
    writes a sorted run file to ``workDir`` whenever it fills; ``finish`` merges every run into one sorted file of
    ``COOC_DTYPE`` records (equal pairs summed in a fixed order) and returns it memory-mapped."""

    def __init__(self, window, symmetric=True, maxEntries=None, maxMemoryBytes=None, workDir=None):
        import tempfile
        if maxEntries is None and maxMemoryBytes is not None:
            maxEntries = max(1024, int(maxMemoryBytes) // 2 // _BYTES_PER_ENTRY)   # the reference flushes at 1/2
        self.window, self.symmetric = int(window), bool(symmetric)
        self._tmp = None
        if workDir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="glove_cooc_")
            workDir = self._tmp.name
        self.workDir = workDir
        self._rt = RT.load()
        self._h = self._rt.rt_cooc_new(workDir.encode(), int(maxEntries or 0))

    def add(self, seqs):
        offs = np.zeros(len(seqs) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(s) for s in seqs])
        toks = np.concatenate(seqs).astype(np.int32) if offs[-1] else np.zeros(1, np.int32)
        if self._rt.rt_cooc_add(self._h, _np_ptr(toks), _np_ptr(offs), len(seqs), self.window,
                                int(self.symmetric)) != 0:
            raise OSError(f"co-occurrence spill to {self.workDir} failed")
        return self

    def spills(self):
        return int(self._rt.rt_cooc_spills(self._h))

    def finish(self, path=None):
        import os
        path = path or os.path.join(self.workDir, "cooccurrences.bin")
        n = self._rt.rt_cooc_finish(self._h, path.encode())
        if n < 0:
            raise OSError(f"co-occurrence merge into {path} failed")
        self.path, self.count = path, int(n)
        return np.memmap(path, dtype=COOC_DTYPE, mode="r", shape=(n,)) if n else np.zeros(0, COOC_DTYPE)

    def close(self):
        if self._h:
            self._rt.rt_cooc_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:       # noqa: BLE001 — interpreter shutdown
            pass


class BinaryCoOccurrenceWriter:
    """Reference count/BinaryCoOccurrenceWriter.java: per record big-endian int32 i, int32 j, float64 weight."""
    REC = np.dtype([("i", ">i4"), ("j", ">i4"), ("x", ">f8")])

    def __init__(self, path):
        self.fh = open(path, "wb")

    def writeObject(self, i, j, x):
        self.fh.write(np.array([(i, j, x)], dtype=self.REC).tobytes())

    def writeArrays(self, i, j, x):
        rec = np.empty(len(i), dtype=self.REC)
        rec["i"], rec["j"], rec["x"] = i, j, x
        self.fh.write(rec.tobytes())

    def finish(self):
        self.fh.close()


class BinaryCoOccurrenceReader:
    """Reads BinaryCoOccurrenceWriter files: ``hasMoreObjects`` / ``nextObject`` -> (i, j, weight), or ``arrays``."""

    def __init__(self, path):
        self.rec = np.memmap(path, dtype=BinaryCoOccurrenceWriter.REC, mode="r")
        self.pos = 0

    def hasMoreObjects(self):
        return self.pos < len(self.rec)

    def nextObject(self):
        r = self.rec[self.pos]
        self.pos += 1
        return int(r["i"]), int(r["j"]), float(r["x"])

    def arrays(self):
        return (self.rec["i"].astype(np.int32), self.rec["j"].astype(np.int32), self.rec["x"].astype(np.float32))


class ASCIICoOccurrenceWriter:
    """Reference count/ASCIICoOccurrenceWriter.java: one "i j weight" line per record."""

    def __init__(self, path):
        self.fh = open(path, "w")

    def writeObject(self, i, j, x):
        self.fh.write(f"{int(i)} {int(j)} {float(x)!r}\n")

    def finish(self):
        self.fh.close()


class ASCIICoOccurrenceReader:
    def __init__(self, path):
        self.fh = open(path)
        self._next = self.fh.readline()

    def hasMoreObjects(self):
        return bool(self._next.strip())

    def nextObject(self):
        a, b, x = self._next.split(" ")
        self._next = self.fh.readline()
        return int(a), int(b), float(x)

    def finish(self):
        self.fh.close()


def cooccurrences(seqs, window, symmetric=True):
    """Sorted (i, j, x) arrays of windowed co-occurrence weights over int32 index sequences."""
    rt = RT.load()
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    toks = np.concatenate(seqs).astype(np.int32) if offs[-1] else np.zeros(1, np.int32)
    h = rt.rt_glove_cooccur_new(_np_ptr(toks), _np_ptr(offs), len(seqs), int(window), int(bool(symmetric)))
    try:
        n = rt.rt_glove_cooccur_size(h)
        i = np.empty(n, np.int32)
        j = np.empty(n, np.int32)
        x = np.empty(n, np.float32)
        rt.rt_glove_cooccur_fetch(h, _np_ptr(i), _np_ptr(j), _np_ptr(x), n)
    finally:
        rt.rt_glove_cooccur_free(h)
    return i, j, x


class Glove(Word2Vec):
    class Builder(_BaseBuilder):
        def __init__(self):
            super().__init__()
            self.c.learningRate = 0.05
            self.c.window = 5
            self.c.layersSize = 100
            self._xmax, self._alpha, self._sym, self._shuffle = 100.0, 0.75, True, True
            self._maxmem = None

        def maxMemory(self, gbytes):
            """Cap the co-occurrence counting memory (reference AbstractCoOccurrences.Builder.maxMemory): past half
            of it the counter spills sorted runs to disk and training streams the merged file."""
            self._maxmem = float(gbytes) * (1 << 30)
            return self

        def xMax(self, v): self._xmax = float(v); return self  # noqa: E704
        def alpha(self, v): self._alpha = float(v); return self  # noqa: E704
        def symmetric(self, v): self._sym = bool(v); return self  # noqa: E704
        def shuffle(self, v): self._shuffle = bool(v); return self  # noqa: E704

        def build(self):
            from .text import DefaultTokenizerFactory
            m = Glove(self.c)
            m.sentenceIter = self._iter
            m.tokenizerFactory = self._tf or DefaultTokenizerFactory()
            m.xMax, m.alpha, m.symmetric, m.shuffle = self._xmax, self._alpha, self._sym, self._shuffle
            m.maxMemoryBytes = self._maxmem
            return self._finish(m)

    def __init__(self, conf=None):
        super().__init__(conf)
        self.xMax, self.alpha, self.symmetric, self.shuffle = 100.0, 0.75, True, True
        self.bias = None
        self.lossHistory = []
        self.maxMemoryBytes = None
        self.maxCoOccurrences = None      # direct cap on counted pairs held in memory (tests / tuning)
        self.streamBlock = 1 << 22        # records per training block when streaming the spilled table
        self.coOccurrenceSpills = 0

    def resetWeights(self):
        c = self.conf
        self._lookup = InMemoryLookupTable(self.vocabCache, c.layersSize, c.seed or 12345, False, 0.0,
                                           self._device())
        self._lookup.resetWeights()

    def fit(self):
        c = self.conf
        if self.vocabCache is None or self.vocabCache.numWords() == 0 or self.sequences is None:
            self.buildVocab()
        if self._lookup is None or self._lookup.syn0 is None:
            self.resetWeights()
        seqs, _ = self._index_sequences()
        if self.maxMemoryBytes is not None or self.maxCoOccurrences is not None:
            return self._fit_streamed(seqs)
        ei, ej, ex = cooccurrences(seqs, c.window, self.symmetric)
        dev = self._lookup.device
        W = self._lookup.syn0
        V, D = W.shape
        b = torch.zeros(V, device=dev)
        hW = torch.zeros(V, D, device=dev)
        hb = torch.zeros(V, device=dev)
        rng = np.random.RandomState(int(c.seed) & 0x7FFFFFFF)
        gpu = dev.type == "cuda"
        if gpu:
            from ..ops import native
            lib = native.load()
            native.register_sig("dl4j_glove", [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_int, c_float, c_float, c_float, c_void_p, c_int, c_void_p])
            cost = torch.zeros(1, device=dev)
            di, dj, dx = (torch.from_numpy(a).to(dev) for a in (ei, ej, ex))
        rt = RT.load()
        for _ in range(max(1, c.epochs) * max(1, c.iterations)):
            if gpu:
                if self.shuffle:
                    perm = torch.from_numpy(rng.permutation(len(ei))).to(dev)
                    a, bb, x = di[perm].contiguous(), dj[perm].contiguous(), dx[perm].contiguous()
                else:
                    a, bb, x = di, dj, dx
                cost.zero_()
                rc = lib.dl4j_glove(_t_ptr(a), _t_ptr(bb), _t_ptr(x), len(ei), _t_ptr(W), _t_ptr(b), _t_ptr(hW),
                                    _t_ptr(hb), D, c.learningRate, self.xMax, self.alpha, _t_ptr(cost),
                                    max(1, min(8192, V // 32)), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
                if rc != 0:
                    raise RuntimeError(f"dl4j_glove failed ({rc})")
                self.lossHistory.append(float(cost.item()))
            else:
                perm = rng.permutation(len(ei)) if self.shuffle else np.arange(len(ei))
                a, bb, x = (np.ascontiguousarray(v[perm]) for v in (ei, ej, ex))
                self.lossHistory.append(rt.rt_glove_apply(_np_ptr(a), _np_ptr(bb), _np_ptr(x), len(ei), _t_ptr(W),
                                                          _t_ptr(b), _t_ptr(hW), _t_ptr(hb), D, c.learningRate,
                                                          self.xMax, self.alpha, c.workers or 4))
        self.bias = b
        self.lastEpochLoss = self.lossHistory[-1] if self.lossHistory else 0.0
        self._lookup.invalidate()
        return self

    def _fit_streamed(self, seqs, chunk=4096):
        """Bounded-memory path: count in sequence chunks with spills, then train over the memory-mapped merged table
        in blocks (block order and the records inside each block shuffled per epoch; the reference's GloVe learner
        also consumes its co-occurrence file sequentially in shuffled batches)."""
        c = self.conf
        counter = CoOccurrenceCounter(c.window, self.symmetric, maxEntries=self.maxCoOccurrences,
                                      maxMemoryBytes=self.maxMemoryBytes)
        for a in range(0, len(seqs), chunk):
            counter.add(seqs[a:a + chunk])
        self.coOccurrenceSpills = counter.spills()
        table = counter.finish()
        dev = self._lookup.device
        W = self._lookup.syn0
        V, D = W.shape
        b = torch.zeros(V, device=dev)
        hW = torch.zeros(V, D, device=dev)
        hb = torch.zeros(V, device=dev)
        rng = np.random.RandomState(int(c.seed) & 0x7FFFFFFF)
        gpu = dev.type == "cuda"
        rt = RT.load()
        if gpu:
            from ..ops import native
            lib = native.load()
            native.register_sig("dl4j_glove", [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_int, c_float, c_float, c_float, c_void_p, c_int, c_void_p])
            cost = torch.zeros(1, device=dev)
        n, B = len(table), max(1, int(self.streamBlock))
        for _ in range(max(1, c.epochs) * max(1, c.iterations)):
            order = rng.permutation((n + B - 1) // B) if self.shuffle else np.arange((n + B - 1) // B)
            total = 0.0
            if gpu:
                cost.zero_()
            for blk in order:
                rec = np.asarray(table[blk * B:(blk + 1) * B])
                if self.shuffle:
                    rec = rec[rng.permutation(len(rec))]
                a = np.ascontiguousarray(rec["i"])
                bb = np.ascontiguousarray(rec["j"])
                x = np.ascontiguousarray(rec["x"])
                if gpu:
                    da, db_, dx = (torch.from_numpy(v).to(dev) for v in (a, bb, x))
                    rc = lib.dl4j_glove(_t_ptr(da), _t_ptr(db_), _t_ptr(dx), len(a), _t_ptr(W), _t_ptr(b),
                                        _t_ptr(hW), _t_ptr(hb), D, c.learningRate, self.xMax, self.alpha,
                                        _t_ptr(cost), max(1, min(8192, V // 32)),
                                        ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
                    if rc != 0:
                        raise RuntimeError(f"dl4j_glove failed ({rc})")
                else:
                    total += rt.rt_glove_apply(_np_ptr(a), _np_ptr(bb), _np_ptr(x), len(a), _t_ptr(W), _t_ptr(b),
                                               _t_ptr(hW), _t_ptr(hb), D, c.learningRate, self.xMax, self.alpha,
                                               c.workers or 4)
            self.lossHistory.append(float(cost.item()) if gpu else total)
        del table
        counter.close()
        self.bias = b
        self.lastEpochLoss = self.lossHistory[-1] if self.lossHistory else 0.0
        self._lookup.invalidate()
        return self
