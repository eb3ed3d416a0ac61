"""Lookup table, the native training engine, and the WordVectors query API.

Reference: NLP:models/embeddings/inmemory/InMemoryLookupTable.java (syn0 uniform (r-0.5)/D init, syn1/syn1Neg
zeros, unigram^0.75 negative table), NLP:models/embeddings/wordvectors/WordVectorsImpl.java +
reader/impl/BasicModelUtils.java (similarity, wordsNearest with positive/negative sets, wordsNearestSum, accuracy).

Engine: sequences -> work items through the C++ batcher (``rt_w2v_batch``), then applied by the gfx950 kernels
(``dl4j_w2v_sg`` / ``dl4j_w2v_cbow`` in csrc/embeddings.hip) when the table lives on a GPU, or by the threaded C++
applier otherwise. Tables stay resident on the device for the whole fit; only int32 item arrays travel.
"""
import ctypes
import math
import os

import numpy as np
import torch

from ..ops import runtime as RT

c_void_p, c_int, c_ll, c_float, c_double, c_ull = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, \
    ctypes.c_float, ctypes.c_double, ctypes.c_ulonglong

RT.register("rt_w2v_batch", [c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                             c_float, c_float, c_ll, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ll,
                             c_ll, c_void_p], c_ll)
RT.register("rt_w2v_sg_apply", [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                c_void_p, c_void_p, c_int, c_void_p, c_ll, c_int, c_int, c_ull, c_ll, c_int],
            c_double)
RT.register("rt_w2v_cbow_apply", [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p,
                                  c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_int, c_int, c_ull,
                                  c_ll, c_int, c_void_p, c_int, c_void_p], c_double)

F_UPD_OUT, F_UPD_IN, F_HS, F_NS = 1, 2, 4, 8
M_SG, M_CBOW, M_DBOW, M_DM = 1, 2, 4, 8


def _np_ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _t_ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _native_kernels():
    from ..ops import native
    lib = native.load()
    native.register_sig("dl4j_w2v_sg", [c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p, c_void_p, c_int,
                                        c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_int, c_int, c_ull,
                                        c_ll, c_void_p, c_int, c_void_p])
    native.register_sig("dl4j_w2v_cbow", [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_void_p, c_void_p,
                                          c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_ll,
                                          c_int, c_int, c_ull, c_ll, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                          c_void_p])
    return lib


class InMemoryLookupTable:
    """syn0 (input vectors; rows for vocabulary words and, for ParagraphVectors, labels), syn1 (HS inner nodes),
    syn1Neg (negative-sampling output vectors), Huffman arrays and the negative table."""

    def __init__(self, vocab, vectorLength, seed=12345, useHierarchicSoftmax=True, negative=0.0, device=None,
                 tableSize=None):
        self.vocab = vocab
        self.vectorLength = int(vectorLength)
        self.seed = seed
        self.useHS = bool(useHierarchicSoftmax)
        self.negative = float(negative)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.tableSize = tableSize
        self.syn0 = self.syn1 = self.syn1Neg = None
        self.table = None
        self._norm = None

    # ------------------------------------------------------------------ init
    def resetWeights(self, reset=True):
        V, D = self.vocab.numWords(), self.vectorLength
        g = torch.Generator().manual_seed(int(self.seed))
        self.syn0 = ((torch.rand(V, D, generator=g) - 0.5) / D).to(self.device)
        self.syn1 = torch.zeros(max(V, 1), D, device=self.device) if self.useHS else None
        self.syn1Neg = None
        if self.negative > 0:
            self.initNegative()
        self._arrays()
        self._norm = None

    def initNegative(self):
        V, D = self.vocab.numWords(), self.vectorLength
        if self.syn1Neg is None:
            self.syn1Neg = torch.zeros(V, D, device=self.device)
        freqs = np.array([0.0 if e.special else e.elementFrequency for e in self.vocab.vocabWords()])
        p = freqs ** 0.75
        if p.sum() <= 0:
            p = np.ones_like(p)
        p /= p.sum()
        ts = int(self.tableSize or min(100_000_000, max(1_000_000, 1000 * V)))
        counts = np.floor(p * ts).astype(np.int64)
        # distribute the rounding remainder to the most probable words
        rem = ts - counts.sum()
        if rem > 0:
            counts[np.argsort(-p)[:rem]] += 1
        self.table_np = np.repeat(np.arange(V, dtype=np.int32), counts)
        self.table = torch.from_numpy(self.table_np).to(self.device)

    def _arrays(self):
        from .vocab import huffman_arrays
        c, p, l, m = huffman_arrays(self.vocab)
        self.codes_np, self.points_np, self.codelen_np, self.maxc = c, p, l, m
        self.codes = torch.from_numpy(c).to(self.device)
        self.points = torch.from_numpy(p).to(self.device)
        self.codelen = torch.from_numpy(l).to(self.device)
        if self.table is None:
            self.table_np = np.zeros(1, dtype=np.int32)
            self.table = torch.zeros(1, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------------ accessors
    def layerSize(self):
        return self.vectorLength

    def getSyn0(self):
        return self.syn0

    def setSyn0(self, s):
        self.syn0 = s.to(self.device)
        self._norm = None

    def getSyn1(self):
        return self.syn1

    def setSyn1(self, s):
        self.syn1 = s.to(self.device)

    def getSyn1Neg(self):
        return self.syn1Neg

    def setSyn1Neg(self, s):
        self.syn1Neg = s.to(self.device)

    def getVocabCache(self):
        return self.vocab

    def vector(self, word):
        i = self.vocab.indexOf(word)
        return None if i < 0 else self.syn0[i]

    def putVector(self, word, vec):
        i = self.vocab.indexOf(word)
        self.syn0[i] = torch.as_tensor(vec, dtype=self.syn0.dtype, device=self.device)
        self._norm = None

    def getWeights(self):
        return self.syn0

    def to(self, device):
        self.device = torch.device(device)
        for n in ("syn0", "syn1", "syn1Neg", "table", "codes", "points", "codelen"):
            t = getattr(self, n, None)
            if t is not None:
                setattr(self, n, t.to(self.device))
        self._norm = None
        return self

    def normalized(self):
        if self._norm is None:
            n = self.syn0.norm(dim=1, keepdim=True).clamp_min(1e-12)
            self._norm = self.syn0 / n
        return self._norm

    def invalidate(self):
        self._norm = None


class EmbeddingEngine:
    """Batches sequences natively and applies them to a lookup table on its device."""

    CHUNK_TOKENS = 1 << 20

    def __init__(self, table, nthreads=None):
        self.t = table
        self.nthreads = nthreads or max(1, min(8, os.cpu_count() or 1))
        self.rt = RT.load()
        if self.rt is None:
            raise RuntimeError("deeplearning4j_amd host runtime library is not available")
        self.gpu = table.device.type == "cuda"
        if self.gpu:
            self.lib = _native_kernels()
            self.loss_dev = torch.zeros(1, device=table.device)
        self.item_base = 0
        self.loss = 0.0

    @staticmethod
    def _max_blocks(rows):
        # ~1 resident wave per 8 table rows (4 waves per block): keeps the Hogwild collision rate low for small
        # vocabularies while large ones still fill all 256 CUs
        return max(1, min(8192, rows // 32))

    def flags(self, update_out=True, update_in=True):
        t = self.t
        f = 0
        if update_out:
            f |= F_UPD_OUT
        if update_in:
            f |= F_UPD_IN
        if t.useHS and t.syn1 is not None:
            f |= F_HS
        if t.negative > 0 and t.syn1Neg is not None:
            f |= F_NS
        return f

    def _batch(self, toks, offs, labs, loffs, keep, window, mode, seed_box, alpha0, amin, before, total):
        ntok = len(toks)
        nlab = 0 if labs is None else len(labs)
        maxlab = 0 if loffs is None else int(np.max(np.diff(loffs))) if len(loffs) > 1 else 0
        cap = max(16, ntok * (2 * window + maxlab + 1))
        while True:
            item_in = np.empty(cap, dtype=np.int32)
            item_tgt = np.empty(cap, dtype=np.int32)
            item_alpha = np.empty(cap, dtype=np.float32)
            cbow = bool(mode & (M_CBOW | M_DM))
            ctx_off = np.empty(cap + 1, dtype=np.int32) if cbow else None
            ctx = np.empty(cap, dtype=np.int32) if cbow else None
            words = ctypes.c_longlong(0)
            seed = ctypes.c_ulonglong(seed_box[0])
            n = self.rt.rt_w2v_batch(_np_ptr(toks), _np_ptr(offs), len(offs) - 1, _np_ptr(labs), _np_ptr(loffs),
                                     _np_ptr(keep), window, mode, ctypes.byref(seed), alpha0, amin, before, total,
                                     _np_ptr(item_in), _np_ptr(item_tgt), _np_ptr(item_alpha), _np_ptr(ctx_off),
                                     _np_ptr(ctx), cap, cap, ctypes.byref(words))
            if n >= 0:
                seed_box[0] = seed.value
                m = int(ctx_off[n]) if cbow else 0
                return (item_in[:n], item_tgt[:n], item_alpha[:n], None if not cbow else ctx_off[:n + 1],
                        None if not cbow else ctx[:m], int(words.value))
            cap *= 2
            _ = nlab

    def _apply(self, mode, items, flags, syn0=None, extra=None, extra_grad=None):
        t = self.t
        item_in, item_tgt, item_alpha, ctx_off, ctx, _ = items
        n = len(item_tgt)
        if n == 0:
            return
        syn0 = t.syn0 if syn0 is None else syn0
        D = t.vectorLength
        cbow = bool(mode & (M_CBOW | M_DM))
        seed = int(t.seed) & 0xFFFFFFFFFFFFFFFF
        if self.gpu:
            dev = t.device
            # host-side bounds check before a hand-written kernel dereferences these indices
            rows, V = syn0.shape[0], int(t.codelen.numel())
            if item_tgt.min() < 0 or item_tgt.max() >= V:
                raise IndexError("embedding target index out of range")
            if not cbow and (item_in.min() < 0 or item_in.max() >= rows):
                raise IndexError("embedding input row out of range")
            if cbow and (len(ctx) and (ctx.min() < 0 or ctx.max() >= rows) or ctx_off[0] != 0 or
                         ctx_off[-1] != len(ctx) or np.any(np.diff(ctx_off) < 0)):
                raise IndexError("CBOW context arrays inconsistent")
            if (t.syn1 is None and flags & F_HS) or (t.syn1Neg is None and flags & F_NS):
                raise ValueError("output table missing for the requested objective")
            if extra is not None and extra.shape[1] != D:
                raise ValueError("extra input width mismatch")

            # device copies are held in locals until after the launch: a temporary's block would go back to the
            # caching allocator and be reused by the next copy before the kernel reads it
            def up(a):
                return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(dev, non_blocking=True)
            s = torch.cuda.current_stream(dev).cuda_stream
            d_tgt, d_alpha = up(item_tgt), up(item_alpha)
            if cbow:
                d_off = up(ctx_off)
                d_ctx = up(ctx) if len(ctx) else torch.zeros(1, dtype=torch.int32, device=dev)
                rc = self.lib.dl4j_w2v_cbow(_t_ptr(d_tgt), _t_ptr(d_alpha), _t_ptr(d_off), _t_ptr(d_ctx),
                                            n, _t_ptr(syn0), _t_ptr(t.syn1), _t_ptr(t.syn1Neg), D, _t_ptr(t.codes),
                                            _t_ptr(t.points), _t_ptr(t.codelen), t.maxc, _t_ptr(t.table),
                                            t.table.numel(), int(t.negative), flags, seed, self.item_base,
                                            _t_ptr(extra), 0 if extra is None else extra.shape[0],
                                            _t_ptr(extra_grad), _t_ptr(self.loss_dev), self._max_blocks(rows), c_void_p(s))
                keep = (d_off, d_ctx)
            else:
                d_in = up(item_in)
                rc = self.lib.dl4j_w2v_sg(_t_ptr(d_in), _t_ptr(d_tgt), _t_ptr(d_alpha), n,
                                          _t_ptr(syn0), _t_ptr(t.syn1), _t_ptr(t.syn1Neg), D, _t_ptr(t.codes),
                                          _t_ptr(t.points), _t_ptr(t.codelen), t.maxc, _t_ptr(t.table),
                                          t.table.numel(), int(t.negative), flags, seed, self.item_base,
                                          _t_ptr(self.loss_dev), self._max_blocks(rows), c_void_p(s))
                keep = (d_in,)
            # the kernel is stream-ordered after these blocks; release them only once it has been enqueued
            del keep, d_tgt, d_alpha
            if rc != 0:
                raise RuntimeError(f"embedding kernel failed ({rc})")
        else:
            thr = 1 if extra is not None else self.nthreads
            if cbow:
                loss = self.rt.rt_w2v_cbow_apply(_np_ptr(item_tgt), _np_ptr(item_alpha), _np_ptr(ctx_off),
                                                 _np_ptr(ctx), n, _t_ptr(syn0), _t_ptr(t.syn1), _t_ptr(t.syn1Neg), D,
                                                 _np_ptr(t.codes_np), _np_ptr(t.points_np), _np_ptr(t.codelen_np),
                                                 t.maxc, _np_ptr(t.table_np), len(t.table_np), int(t.negative),
                                                 flags, seed, self.item_base, thr, _t_ptr(extra),
                                                 0 if extra is None else extra.shape[0], _t_ptr(extra_grad))
            else:
                loss = self.rt.rt_w2v_sg_apply(_np_ptr(item_in), _np_ptr(item_tgt), _np_ptr(item_alpha), n,
                                               _t_ptr(syn0), _t_ptr(t.syn1), _t_ptr(t.syn1Neg), D,
                                               _np_ptr(t.codes_np), _np_ptr(t.points_np), _np_ptr(t.codelen_np),
                                               t.maxc, _np_ptr(t.table_np), len(t.table_np), int(t.negative), flags,
                                               seed, self.item_base, thr)
            self.loss += loss
        self.item_base += n

    def train(self, sequences, labels=None, mode=M_SG, window=5, alpha0=0.025, alpha_min=1e-4, words_before=0,
              total_words=0, keep_prob=None, seed_box=None, flags=None):
        """sequences: list of int32 arrays (vocab indices, -1 = dropped); labels: list of int32 arrays (syn0 rows)
        or None. Returns the number of words processed."""
        if flags is None:
            flags = self.flags()
        seed_box = seed_box if seed_box is not None else [int(self.t.seed) or 1]
        done = 0
        i = 0
        N = len(sequences)
        if (mode & (M_SG | M_DBOW)) and (mode & (M_CBOW | M_DM)):
            raise ValueError("skip-gram and CBOW item kinds must be batched separately")
        while i < N:
            j, ntok = i, 0
            while j < N and (ntok == 0 or ntok + len(sequences[j]) <= self.CHUNK_TOKENS):
                ntok += len(sequences[j])
                j += 1
            chunk = sequences[i:j]
            offs = np.zeros(len(chunk) + 1, dtype=np.int64)
            offs[1:] = np.cumsum([len(s) for s in chunk])
            toks = np.concatenate(chunk).astype(np.int32) if ntok else np.zeros(0, np.int32)
            if labels is not None:
                lch = labels[i:j]
                loffs = np.zeros(len(lch) + 1, dtype=np.int64)
                loffs[1:] = np.cumsum([len(l) for l in lch])
                labs = np.concatenate(lch).astype(np.int32) if loffs[-1] else np.zeros(1, np.int32)
            else:
                labs = loffs = None
            items = self._batch(toks, offs, labs, loffs, keep_prob, window, mode, seed_box, alpha0, alpha_min,
                                words_before + done, total_words)
            self._apply(mode, items, flags)
            done += items[5]
            i = j
        self.t.invalidate()
        return done

    def take_loss(self):
        if self.gpu:
            v = float(self.loss_dev.item())
            self.loss_dev.zero_()
            return v
        v, self.loss = self.loss, 0.0
        return v


def keep_probabilities(vocab, sampling):
    """word2vec frequency subsampling keep probability per vocab index (SkipGram.applySubsampling)."""
    if not sampling or sampling <= 0:
        return None
    total = float(vocab.totalWordOccurrences()) or 1.0
    thr = sampling * total
    out = np.ones(vocab.numWords(), dtype=np.float32)
    for e in vocab.vocabWords():
        if e.special:
            continue
        f = max(e.elementFrequency, 1.0)
        out[e.index] = min(1.0, (math.sqrt(f / thr) + 1.0) * thr / f)
    return out


class WordVectorsImpl:
    """Query API shared by Word2Vec / ParagraphVectors / GloVe / static vectors."""

    UNK = "UNK"

    def __init__(self, lookup=None, vocab=None):
        self._lookup = lookup
        self._vocab = vocab
        self.useUnknown = False

    # --- plumbing
    def lookupTable(self):
        return self._lookup

    getLookupTable = lookupTable

    def setLookupTable(self, t):
        self._lookup = t

    def vocab(self):
        return self._vocab

    getVocab = vocab

    def setVocab(self, v):
        self._vocab = v

    def getLayerSize(self):
        return self._lookup.vectorLength

    def getUNK(self):
        return self.UNK

    def setUNK(self, u):
        self.UNK = u

    def outOfVocabularySupported(self):
        return self.useUnknown

    def hasWord(self, w):
        return self._vocab.containsWord(w)

    def indexOf(self, w):
        return self._vocab.indexOf(w)

    def _idx(self, w):
        i = self._vocab.indexOf(w)
        if i < 0 and self.useUnknown:
            i = self._vocab.indexOf(self.UNK)
        return i

    # --- vectors
    def getWordVector(self, w):
        i = self._idx(w)
        return None if i < 0 else self._lookup.syn0[i].detach().cpu().double().numpy()

    def getWordVectorMatrix(self, w):
        i = self._idx(w)
        return None if i < 0 else self._lookup.syn0[i].reshape(1, -1)

    def getWordVectorMatrixNormalized(self, w):
        i = self._idx(w)
        return None if i < 0 else self._lookup.normalized()[i].reshape(1, -1)

    def getWordVectors(self, words):
        """Rows of the words the vocabulary contains (UNK for the others when out-of-vocabulary words are
        supported), in order; the rest are dropped (reference WordVectorsImpl.getWordVectors)."""
        idx = []
        for w in words:
            if self._vocab.containsWord(w):
                idx.append(self._vocab.indexOf(w))
            elif self.useUnknown and self._vocab.containsWord(self.UNK):
                idx.append(self._vocab.indexOf(self.UNK))
        W = self._lookup.syn0 if getattr(self._lookup, "syn0", None) is not None else self._lookup.getWeights()
        return W[torch.as_tensor(idx, dtype=torch.long, device=W.device)]

    def getWordVectorsMean(self, words):
        return self.getWordVectors(words).mean(dim=0, keepdim=True)

    # --- similarity
    def similarity(self, a, b):
        ia, ib = self._idx(a), self._idx(b)
        if ia < 0 or ib < 0:
            return float("nan")
        if a == b:
            return 1.0
        n = self._lookup.normalized()
        return float((n[ia] * n[ib]).sum())

    def _nearest_to_vector(self, v, n, exclude=()):
        nrm = self._lookup.normalized()
        v = torch.as_tensor(v, dtype=nrm.dtype, device=nrm.device).reshape(-1)
        v = v / v.norm().clamp_min(1e-12)
        sims = nrm @ v
        V = sims.shape[0]
        for w in exclude:
            i = self._vocab.indexOf(w)
            if i >= 0:
                sims[i] = -float("inf")
        # labels (ParagraphVectors documents) are not words
        special = [e.index for e in self._vocab.vocabWords() if e.special]
        if special:
            sims[torch.as_tensor(special, device=sims.device)] = -float("inf")
        k = min(n, V)
        top = torch.topk(sims, k).indices.cpu().tolist()
        return [self._vocab.wordAtIndex(i) for i in top if sims[i] > -float("inf")]

    def wordsNearest(self, positive, negative=None, n=10):
        """wordsNearest(word, n) or wordsNearest(positive_list, negative_list, n) (BasicModelUtils.java)."""
        if isinstance(positive, str):
            if isinstance(negative, int):
                n, negative = negative, None
            positive = [positive]
        elif isinstance(positive, (np.ndarray, torch.Tensor)):
            return self._nearest_to_vector(positive, n if not isinstance(negative, int) else negative)
        negative = list(negative or [])
        nrm = self._lookup.normalized()
        acc = torch.zeros(nrm.shape[1], dtype=nrm.dtype, device=nrm.device)
        for w in positive:
            i = self._idx(w)
            if i >= 0:
                acc += nrm[i]
        for w in negative:
            i = self._idx(w)
            if i >= 0:
                acc -= nrm[i]
        return self._nearest_to_vector(acc, n, exclude=list(positive) + negative)

    def wordsNearestSum(self, positive, negative=None, n=10):
        if isinstance(positive, (np.ndarray, torch.Tensor)):
            k = n if not isinstance(negative, int) else negative
            syn0 = self._lookup.syn0
            v = torch.as_tensor(positive, dtype=syn0.dtype, device=syn0.device).reshape(-1)
            sims = syn0 @ v
            top = torch.topk(sims, min(k, sims.shape[0])).indices.cpu().tolist()
            return [self._vocab.wordAtIndex(i) for i in top]
        if isinstance(positive, str):
            if isinstance(negative, int):
                n, negative = negative, None
            positive = [positive]
        syn0 = self._lookup.syn0
        acc = torch.zeros(syn0.shape[1], dtype=syn0.dtype, device=syn0.device)
        for w in positive:
            acc += syn0[self._idx(w)]
        for w in negative or []:
            acc -= syn0[self._idx(w)]
        sims = syn0 @ acc
        for w in list(positive) + list(negative or []):
            sims[self._idx(w)] = -float("inf")
        top = torch.topk(sims, min(n, sims.shape[0])).indices.cpu().tolist()
        return [self._vocab.wordAtIndex(i) for i in top]

    def similarWordsInVocabTo(self, word, accuracy):
        """Vocabulary words whose string similarity (1 - normalised Levenshtein) to ``word`` is >= accuracy."""
        out = []
        for w in self._vocab.words():
            if _string_similarity(word, w) >= accuracy:
                out.append(w)
        return out

    def accuracy(self, questions):
        """Analogy accuracy over lines "a b c d" (a:b :: c:d), grouped by ": section" headers."""
        res = {}
        section, correct, total = "default", 0, 0
        for q in questions:
            if q.startswith(":"):
                if total:
                    res[section] = correct / total
                section, correct, total = q[1:].strip(), 0, 0
                continue
            ws = q.split()
            if len(ws) != 4 or not all(self.hasWord(w) for w in ws):
                continue
            total += 1
            pred = self.wordsNearest([ws[1], ws[2]], [ws[0]], 1)
            correct += int(bool(pred) and pred[0] == ws[3])
        if total:
            res[section] = correct / total
        return res


def _string_similarity(a, b):
    if a == b:
        return 1.0
    la, lb = len(a), len(b)
    if la == 0 or lb == 0:
        return 0.0
    prev = list(range(lb + 1))
    for i in range(1, la + 1):
        cur = [i] + [0] * lb
        for j in range(1, lb + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a[i - 1] != b[j - 1]))
        prev = cur
    return 1.0 - prev[lb] / max(la, lb)
