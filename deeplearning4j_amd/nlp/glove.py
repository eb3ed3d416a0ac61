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
            return self._finish(m)

    def __init__(self, conf=None):
        super().__init__(conf)
        self.xMax, self.alpha, self.symmetric, self.shuffle = 100.0, 0.75, True, True
        self.bias = None
        self.lossHistory = []

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
