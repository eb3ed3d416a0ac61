"""SequenceVectors, Word2Vec and ParagraphVectors.

Reference: NLP:models/sequencevectors/SequenceVectors.java (vocab build, weight reset, epoch/iteration loop with
linear learning-rate decay ``alpha = max(minLR, LR * (1 - wordsSeen / (totalWords * epochs * iterations)))``),
models/word2vec/Word2Vec.java (Builder: iterate/tokenizerFactory/layerSize/windowSize/minWordFrequency/negativeSample/
useHierarchicSoftmax/sampling/elementsLearningAlgorithm ...), models/paragraphvectors/ParagraphVectors.java
(labels as extra syn0 rows, DBOW/DM, inferVector/predict/nearestLabels), embeddings/loader/VectorsConfiguration.java.
Training runs through EmbeddingEngine (native batcher + gfx950 kernels / threaded C++ applier).
"""
import json
import logging
import time
import zlib

import numpy as np

import torch

from .embeddings import (EmbeddingEngine, InMemoryLookupTable, M_CBOW, M_DBOW, M_DM, M_SG, WordVectorsImpl,
                         F_HS, F_NS, F_UPD_IN, keep_probabilities)
from .text import DefaultTokenizerFactory, LabelAwareIterator, LabelsSource, SentenceIterator
from .vocab import AbstractCache, VocabConstructor

log = logging.getLogger("deeplearning4j_amd")


class VectorsConfiguration:
    FIELDS = dict(minWordFrequency=5, learningRate=0.025, minLearningRate=0.0001, layersSize=200, useAdaGrad=False,
                  batchSize=512, iterations=1, epochs=1, window=5, seed=0, negative=0.0, useHierarchicSoftmax=True,
                  sampling=0.0, learningRateDecayWords=0, variableWindows=None, hugeModelExpected=False,
                  useUnknown=False, elementsLearningAlgorithm="SkipGram", sequenceLearningAlgorithm=None,
                  tokenizerFactory=None, tokenPreProcessor=None, UNK="UNK", STOP="STOP", stopList=[],
                  vocabSize=0, trainElementsVectors=True, trainSequenceVectors=True, workers=0)

    def __init__(self, **kw):
        for k, v in self.FIELDS.items():
            setattr(self, k, kw.get(k, v.copy() if isinstance(v, list) else v))

    def toJson(self):
        return json.dumps({k: getattr(self, k) for k in self.FIELDS}, sort_keys=True)

    @staticmethod
    def fromJson(s):
        d = json.loads(s)
        return VectorsConfiguration(**{k: v for k, v in d.items() if k in VectorsConfiguration.FIELDS})


class VectorsListener:
    """SequenceVectors listener (NLP:models/sequencevectors/interfaces/VectorsListener.java)."""

    def validateEvent(self, event, argument):
        return True

    def processEvent(self, event, model, argument):
        pass


class ScoreListener(VectorsListener):
    def __init__(self, frequency=1):
        self.frequency = frequency
        self.scores = []

    def validateEvent(self, event, argument):
        return event == "EPOCH" and argument % self.frequency == 0

    def processEvent(self, event, model, argument):
        self.scores.append(model.lastEpochLoss)
        log.info("epoch %d: loss %.4f", argument, model.lastEpochLoss)


class SerializingListener(VectorsListener):
    def __init__(self, path_template="vectors_%d.zip", frequency=1):
        self.tpl, self.frequency = path_template, frequency

    def validateEvent(self, event, argument):
        return event == "EPOCH" and argument % self.frequency == 0

    def processEvent(self, event, model, argument):
        from .serializer import WordVectorSerializer
        WordVectorSerializer.writeWord2VecModel(model, self.tpl % argument)


_ELEM = {"skipgram": M_SG, "cbow": M_CBOW}
_SEQ = {"dbow": M_DBOW, "dm": M_DM}


def _algo_name(a):
    if a is None:
        return None
    if not isinstance(a, str):
        a = type(a).__name__ if not isinstance(a, type) else a.__name__
    return a.split(".")[-1].lower().replace("pv-", "").replace("_", "")


class SkipGram:
    pass


class CBOW:
    pass


class DBOW:
    pass


class DM:
    pass


class SequenceVectors(WordVectorsImpl):
    """Generic embedding trainer over sequences of element labels (words, vertex ids, ...)."""

    def __init__(self, conf=None):
        super().__init__()
        self.conf = conf or VectorsConfiguration()
        self.sequences = None           # list of lists of labels
        self.seq_labels = None          # list of lists of sequence labels (ParagraphVectors)
        self.vocabCache = None
        self.listeners = []
        self.lastEpochLoss = 0.0
        self.device = None
        self._engine = None
        self.useUnknown = self.conf.useUnknown
        self.UNK = self.conf.UNK

    # ------------------------------------------------------------------ config accessors
    def getConfiguration(self):
        return self.conf

    def setVectorsListeners(self, ls):
        self.listeners = list(ls)

    def _device(self):
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

    # ------------------------------------------------------------------ data
    def _load_sequences(self):
        """Subclasses fill self.sequences / self.seq_labels (lists of label lists); the base class reads the
        Builder's source of ``Sequence`` objects (elements, optional sequence labels)."""
        src = getattr(self, "_source", None)
        if self.sequences is None and src is not None:
            seqs, labs, any_label = [], [], False
            for sq in src:
                els = sq.getElements() if hasattr(sq, "getElements") else list(sq)
                seqs.append([str(e) for e in els])
                ls = sq.getSequenceLabels() if hasattr(sq, "getSequenceLabels") else None
                labs.append([str(x) for x in (ls or [])])
                any_label |= bool(ls)
            self.sequences = seqs
            self.seq_labels = labs if (any_label and self.conf.sequenceLearningAlgorithm) else None
        if self.sequences is None:
            raise ValueError("no training sequences configured")

    def buildVocab(self):
        self._load_sequences()
        c = self.conf
        if self.vocabCache is None or self.vocabCache.numWords() == 0:
            vc = VocabConstructor(c.minWordFrequency, c.stopList, c.useUnknown, c.UNK)
            self.vocabCache = vc.buildJointVocabulary(self.sequences, self.seq_labels)
        self.setVocab(self.vocabCache)
        c.vocabSize = self.vocabCache.numWords()

    def _index_sequences(self):
        V = self.vocabCache
        unk = V.indexOf(self.conf.UNK) if self.conf.useUnknown else -1
        out = []
        for s in self.sequences:
            idx = np.fromiter((V.indexOf(t) for t in s), dtype=np.int32, count=len(s))
            if unk >= 0:
                idx[idx < 0] = unk
            out.append(idx)
        labs = None
        if self.seq_labels is not None:
            labs = [np.array([V.indexOf(l) for l in ls if V.indexOf(l) >= 0], dtype=np.int32)
                    for ls in self.seq_labels]
        return out, labs

    # ------------------------------------------------------------------ training
    def _modes(self):
        """List of (mode, flags-override) passes per epoch."""
        c = self.conf
        elem = _ELEM.get(_algo_name(c.elementsLearningAlgorithm) or "", 0) if c.trainElementsVectors else 0
        seq = _SEQ.get(_algo_name(c.sequenceLearningAlgorithm) or "", 0) if c.trainSequenceVectors else 0
        passes = []
        if seq == M_DBOW:
            passes.append(M_DBOW | (M_SG if elem == M_SG else 0))
            if elem == M_CBOW:
                passes.append(M_CBOW)
        elif seq == M_DM:
            passes.append(M_DM)
            if elem == M_SG:
                passes.append(M_SG)
        elif elem:
            passes.append(elem)
        return passes

    def resetWeights(self):
        c = self.conf
        self._lookup = InMemoryLookupTable(self.vocabCache, c.layersSize, c.seed or 12345, c.useHierarchicSoftmax,
                                           c.negative, self._device())
        self._lookup.resetWeights()

    def fit(self):
        c = self.conf
        if self.vocabCache is None or self.vocabCache.numWords() == 0 or self.sequences is None:
            self.buildVocab()
        if self._lookup is None or self._lookup.syn0 is None or self._lookup.vocab is not self.vocabCache:
            self.resetWeights()
        seqs, labs = self._index_sequences()
        engine = EmbeddingEngine(self._lookup, c.workers or None)
        self._engine = engine
        keep = keep_probabilities(self.vocabCache, c.sampling)
        passes = self._modes()
        total_words = sum(len(s) for s in seqs) * max(1, c.epochs) * max(1, c.iterations) * max(1, len(passes))
        seen = 0
        seed_box = [int(c.seed) or 1]
        rng = np.random.RandomState(int(c.seed) & 0x7FFFFFFF)
        t0 = time.time()
        for epoch in range(max(1, c.epochs)):
            order = rng.permutation(len(seqs))
            s_ep = [seqs[i] for i in order]
            l_ep = None if labs is None else [labs[i] for i in order]
            for _ in range(max(1, c.iterations)):
                for mode in passes:
                    need_labels = bool(mode & (M_DBOW | M_DM))
                    seen += engine.train(s_ep, l_ep if need_labels else None, mode, c.window, c.learningRate,
                                         c.minLearningRate, seen, total_words, keep, seed_box)
            self.lastEpochLoss = engine.take_loss()
            for l in self.listeners:
                if l.validateEvent("EPOCH", epoch):
                    l.processEvent("EPOCH", self, epoch)
        if self._lookup.device.type == "cuda":
            torch.cuda.synchronize(self._lookup.device)
        self.trainingTime = time.time() - t0
        self.wordsSeen = seen
        self._lookup.invalidate()
        return self


class _BaseBuilder:
    TARGET = None

    def __init__(self, conf=None):
        self.c = VectorsConfiguration() if conf is None else conf
        self._iter = None
        self._tf = None
        self._listeners = []
        self._vocab = None
        self._lookup = None
        self._device = None
        self._labels_source = None

    def minWordFrequency(self, v): self.c.minWordFrequency = int(v); return self  # noqa: E704
    def iterations(self, v): self.c.iterations = int(v); return self  # noqa: E704
    def epochs(self, v): self.c.epochs = int(v); return self  # noqa: E704
    def layerSize(self, v): self.c.layersSize = int(v); return self  # noqa: E704
    def learningRate(self, v): self.c.learningRate = float(v); return self  # noqa: E704
    def minLearningRate(self, v): self.c.minLearningRate = float(v); return self  # noqa: E704
    def windowSize(self, v): self.c.window = int(v); return self  # noqa: E704
    def seed(self, v): self.c.seed = int(v); return self  # noqa: E704
    def negativeSample(self, v): self.c.negative = float(v); return self  # noqa: E704
    def useHierarchicSoftmax(self, v): self.c.useHierarchicSoftmax = bool(v); return self  # noqa: E704
    def sampling(self, v): self.c.sampling = float(v); return self  # noqa: E704
    def batchSize(self, v): self.c.batchSize = int(v); return self  # noqa: E704
    def workers(self, v): self.c.workers = int(v); return self  # noqa: E704
    def useAdaGrad(self, v): self.c.useAdaGrad = bool(v); return self  # noqa: E704
    def useUnknown(self, v): self.c.useUnknown = bool(v); return self  # noqa: E704
    def unknownElement(self, e): self.c.UNK = getattr(e, "label", e); return self  # noqa: E704
    def stopWords(self, v): self.c.stopList = list(v); return self  # noqa: E704
    def trainElementsRepresentation(self, v): self.c.trainElementsVectors = bool(v); return self  # noqa: E704
    def trainSequencesRepresentation(self, v): self.c.trainSequenceVectors = bool(v); return self  # noqa: E704
    def vocabCache(self, v): self._vocab = v; return self  # noqa: E704
    def lookupTable(self, v): self._lookup = v; return self  # noqa: E704
    def setVectorsListeners(self, ls): self._listeners = list(ls); return self  # noqa: E704
    def device(self, d): self._device = d; return self  # noqa: E704
    def allowParallelTokenization(self, v): return self  # noqa: E704
    def enableScavenger(self, v): return self  # noqa: E704
    def limitVocabularySize(self, v): self.c.vocabSize = int(v); return self  # noqa: E704
    def modelUtils(self, v): return self  # noqa: E704

    def elementsLearningAlgorithm(self, a):
        self.c.elementsLearningAlgorithm = _algo_name(a) if not isinstance(a, str) else a
        return self

    def sequenceLearningAlgorithm(self, a):
        self.c.sequenceLearningAlgorithm = _algo_name(a) if not isinstance(a, str) else a
        return self

    def iterate(self, it):
        self._iter = it
        return self

    def tokenizerFactory(self, tf):
        self._tf = tf
        return self

    def _finish(self, m):
        m.listeners = self._listeners
        m.vocabCache = self._vocab
        if self._lookup is not None:
            m._lookup = self._lookup
        m.device = self._device
        m.useUnknown = self.c.useUnknown
        m.UNK = self.c.UNK
        return m


class _SequenceVectorsBuilder(_BaseBuilder):
    """SequenceVectors.Builder (NLP:models/sequencevectors/SequenceVectors.java Builder): trains on any iterable of
    ``Sequence`` objects (elements = labels, optional sequence labels) — e.g. a graph/walkers.GraphTransformer, the
    reference's route for graph embeddings (walkers -> GraphTransformer -> AbstractSequenceIterator ->
    SequenceVectors). Sequence labels are learned with ``sequenceLearningAlgorithm`` (DBOW / DM) when set."""

    def build(self):
        m = SequenceVectors(self.c)
        m._source = self._iter
        return self._finish(m)


SequenceVectors.Builder = _SequenceVectorsBuilder


class Word2Vec(SequenceVectors):
    """Word2Vec over a SentenceIterator (or any iterable of strings / token lists)."""

    class Builder(_BaseBuilder):
        def build(self):
            m = Word2Vec(self.c)
            m.sentenceIter = self._iter
            m.tokenizerFactory = self._tf or DefaultTokenizerFactory()
            return self._finish(m)

    def __init__(self, conf=None):
        super().__init__(conf)
        self.sentenceIter = None
        self.tokenizerFactory = DefaultTokenizerFactory()

    def setSentenceIterator(self, it):
        self.sentenceIter = it
        self.sequences = None

    def setTokenizerFactory(self, tf):
        self.tokenizerFactory = tf

    def _tokenize(self, s):
        if isinstance(s, (list, tuple)):
            return list(s)
        return self.tokenizerFactory.create(s).getTokens()

    def _load_sequences(self):
        if self.sequences is not None:
            return
        it = self.sentenceIter
        if it is None:
            raise ValueError("Word2Vec needs a sentence iterator (Builder.iterate)")
        if isinstance(it, SentenceIterator):
            it.reset()
            sents = []
            while it.hasNext():
                sents.append(it.nextSentence())
        else:
            sents = list(it)
        self.sequences = [self._tokenize(s) for s in sents]


class ParagraphVectors(Word2Vec):
    """Doc2Vec: every document label is an extra syn0 row trained by PV-DBOW or PV-DM."""

    class Builder(_BaseBuilder):
        def __init__(self, conf=None):
            super().__init__(conf)
            self.c.sequenceLearningAlgorithm = "dbow"
            self.c.trainElementsVectors = False
            self._docs = None

        def trainWordVectors(self, v):
            self.c.trainElementsVectors = bool(v)
            return self

        def labelsSource(self, s):
            self._labels_source = s
            return self

        def labels(self, ls):
            self._labels_source = LabelsSource(list(ls))
            return self

        def build(self):
            m = ParagraphVectors(self.c)
            m.sentenceIter = self._iter
            m.tokenizerFactory = self._tf or DefaultTokenizerFactory()
            m.labelsSource = self._labels_source
            return self._finish(m)

    def __init__(self, conf=None):
        super().__init__(conf)
        self.labelsSource = None

    def _load_sequences(self):
        if self.sequences is not None:
            return
        it = self.sentenceIter
        seqs, labs = [], []
        if isinstance(it, LabelAwareIterator):
            it.reset()
            while it.hasNextDocument():
                d = it.nextDocument()
                seqs.append(self._tokenize(d.content))
                labs.append(list(d.labels))
            if self.labelsSource is None:
                self.labelsSource = it.getLabelsSource()
        elif isinstance(it, SentenceIterator):
            src = self.labelsSource or LabelsSource("DOC_%d")
            it.reset()
            while it.hasNext():
                seqs.append(self._tokenize(it.nextSentence()))
                labs.append([src.nextLabel()])
            self.labelsSource = src
        else:
            for item in it:
                if hasattr(item, "content"):
                    seqs.append(self._tokenize(item.content))
                    labs.append(list(item.labels))
                else:
                    content, lab = item
                    seqs.append(self._tokenize(content))
                    labs.append([lab] if isinstance(lab, str) else list(lab))
        self.sequences, self.seq_labels = seqs, labs
        if self.labelsSource is None:
            self.labelsSource = LabelsSource([])
        for ls in labs:
            for l in ls:
                self.labelsSource.storeLabel(l)

    def getLabelsSource(self):
        return self.labelsSource

    def _label_rows(self):
        V = self.vocabCache
        labels = [l for l in self.labelsSource.getLabels() if V.indexOf(l) >= 0]
        idx = torch.as_tensor([V.indexOf(l) for l in labels], dtype=torch.long, device=self._lookup.device)
        return labels, idx

    def inferVector(self, document, learningRate=None, minLearningRate=None, iterations=None):
        """Train a fresh vector for an unseen document against the frozen model (ParagraphVectors.inferVector)."""
        c = self.conf
        lr = c.learningRate if learningRate is None else learningRate
        mlr = c.minLearningRate if minLearningRate is None else minLearningRate
        its = iterations or max(5, c.iterations * c.epochs)
        toks = self._tokenize(document)
        V = self.vocabCache
        idx = np.array([V.indexOf(t) for t in toks if V.indexOf(t) >= 0 and not V.wordFor(t).special],
                       dtype=np.int32)
        dev = self._lookup.device
        D = self._lookup.vectorLength
        g = torch.Generator().manual_seed(zlib.crc32(" ".join(toks).encode()) % (2 ** 31))  # stable across processes
        vec = ((torch.rand(1, D, generator=g) - 0.5) / D).to(dev)
        if len(idx) == 0:
            return vec.reshape(-1)
        eng = EmbeddingEngine(self._lookup, 1)
        base = self._lookup.negative > 0 and self._lookup.syn1Neg is not None
        out_flags = (F_HS if self._lookup.useHS else 0) | (F_NS if base else 0)
        seq_algo = _algo_name(c.sequenceLearningAlgorithm)
        seed_box = [int(c.seed) or 1]
        for it in range(its):
            a = lr - (lr - mlr) * it / max(1, its)
            if seq_algo == "dm":
                items = eng._batch(idx, np.array([0, len(idx)], np.int64), None, None, None, c.window, M_CBOW,
                                   seed_box, a, a, 0, 0)
                grad = torch.zeros_like(vec)
                eng._apply(M_CBOW, items, out_flags, extra=vec, extra_grad=grad)
                vec += grad
            else:
                items = eng._batch(idx, np.array([0, len(idx)], np.int64), np.zeros(1, np.int32),
                                   np.array([0, 1], np.int64), None, c.window, M_DBOW, seed_box, a, a, 0, 0)
                eng._apply(M_DBOW, items, out_flags | F_UPD_IN, syn0=vec)
        return vec.reshape(-1)

    def _as_vector(self, doc):
        if isinstance(doc, (np.ndarray, torch.Tensor)):
            return torch.as_tensor(doc, dtype=self._lookup.syn0.dtype, device=self._lookup.device).reshape(-1)
        if hasattr(doc, "content"):
            doc = doc.content
        return self.inferVector(doc)

    def nearestLabels(self, document, topN=5):
        v = self._as_vector(document)
        labels, idx = self._label_rows()
        rows = self._lookup.syn0[idx]
        sims = torch.nn.functional.cosine_similarity(rows, v.reshape(1, -1), dim=1)
        top = torch.topk(sims, min(topN, len(labels))).indices.cpu().tolist()
        return [labels[i] for i in top]

    def predict(self, document):
        r = self.nearestLabels(document, 1)
        return r[0] if r else None

    def predictSeveral(self, document, limit):
        return self.nearestLabels(document, limit)

    def similarityToLabel(self, document, label):
        v = self._as_vector(document)
        i = self.vocabCache.indexOf(label)
        if i < 0:
            return float("nan")
        return float(torch.nn.functional.cosine_similarity(self._lookup.syn0[i].reshape(1, -1), v.reshape(1, -1)))


_ = (AbstractCache,)
