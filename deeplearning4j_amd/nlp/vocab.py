"""Vocabulary: elements, cache, constructor and Huffman coding.

Reference: NLP:models/word2vec/VocabWord.java, models/sequencevectors/sequence/SequenceElement.java,
models/word2vec/wordstore/inmemory/AbstractCache.java (VocabCache API), wordstore/VocabConstructor.java,
models/word2vec/Huffman.java (word2vec.c CreateBinaryTree, MAX_CODE_LENGTH 40).
Huffman codes/points are materialised as dense [V, maxc] arrays for the native kernels.
"""
import numpy as np

MAX_CODE_LENGTH = 40


class SequenceElement:
    def __init__(self, label, frequency=1.0, special=False):
        if isinstance(frequency, str) and not isinstance(label, str):   # reference order VocabWord(frequency, word)
            label, frequency = frequency, label
        self.label = label
        self.elementFrequency = float(frequency)
        self.sequencesCount = 0
        self.index = -1
        self.codes = []
        self.points = []
        self.special = special          # labels (documents) in ParagraphVectors
        self.isLabel = special

    def getLabel(self):
        return self.label

    def getWord(self):
        return self.label

    def getIndex(self):
        return self.index

    def setIndex(self, i):
        self.index = i

    def getElementFrequency(self):
        return self.elementFrequency

    def increaseElementFrequency(self, by=1.0):
        self.elementFrequency += by

    def setElementFrequency(self, f):
        self.elementFrequency = float(f)

    def getSequencesCount(self):
        return self.sequencesCount

    def getCodes(self):
        return self.codes

    def getPoints(self):
        return self.points

    def getCodeLength(self):
        return len(self.codes)

    def setSpecial(self, s):
        self.special = s

    def isSpecial(self):
        return self.special

    def __repr__(self):
        return f"{type(self).__name__}({self.label!r}, freq={self.elementFrequency}, idx={self.index})"

    def __eq__(self, other):
        # same element = same class and label (reference SequenceElement.equals)
        return type(other) is type(self) and other.label == self.label

    def __hash__(self):
        return hash(self.label)

    def toJSON(self):
        import json
        return json.dumps({"@class": type(self).__name__, "label": self.label,
                           "elementFrequency": self.elementFrequency, "sequencesCount": self.sequencesCount,
                           "index": self.index, "codes": list(self.codes), "points": list(self.points),
                           "special": bool(self.special)})

    @classmethod
    def fromJSON(cls, s):
        import json
        d = json.loads(s)
        e = cls(d["label"], d.get("elementFrequency", 1.0), d.get("special", False))
        e.sequencesCount, e.index = d.get("sequencesCount", 0), d.get("index", -1)
        e.codes, e.points = list(d.get("codes", [])), list(d.get("points", []))
        return e


class VocabWord(SequenceElement):
    pass


class AbstractElementFactory:
    """JSON (de)serialiser for one element class (reference models/sequencevectors/serialization/
    AbstractElementFactory.java), used by the vocabulary writers."""

    def __init__(self, cls):
        self.cls = cls

    def serialize(self, element):
        return element.toJSON()

    def deserialize(self, s):
        return self.cls.fromJSON(s)


class AbstractCache:
    """In-memory VocabCache: label <-> element <-> index, counts, document frequencies."""

    class Builder:
        def __init__(self):
            pass

        def hugeModelExpected(self, b):
            return self

        def minElementFrequency(self, f):
            return self

        def build(self):
            return AbstractCache()

    def __init__(self):
        self._by_label = {}
        self._by_index = []
        self.totalWordCount = 0.0
        self.numDocs = 0

    # --- building
    def addToken(self, element):
        if not element.special:
            self.totalWordCount += element.elementFrequency
        if element.label in self._by_label:
            e = self._by_label[element.label]
            e.increaseElementFrequency(element.elementFrequency)
            return False
        self._by_label[element.label] = element
        return True

    def incrementWordCount(self, word, by=1):
        e = self._by_label.get(word)
        if e is None:
            e = VocabWord(word, 0.0)
            self._by_label[word] = e
        e.increaseElementFrequency(by)
        self.totalWordCount += by

    def addWordToIndex(self, index, label):
        e = self._by_label.get(label)
        if e is None:               # unseen word: added with frequency 1 (reference InMemoryLookupCache)
            e = VocabWord(label, 1.0)
            self._by_label[label] = e
        e.index = index
        while len(self._by_index) <= index:
            self._by_index.append(None)
        self._by_index[index] = e

    def putVocabWord(self, word):
        if word not in self._by_label:
            self._by_label[word] = VocabWord(word, 0.0)

    def removeElement(self, label):
        e = self._by_label.pop(label, None)
        if e is not None and not e.special:
            self.totalWordCount -= e.elementFrequency
        if e is not None and 0 <= e.index < len(self._by_index) and self._by_index[e.index] is e:
            self._by_index[e.index] = None

    def updateWordsOccurrences(self):
        self.totalWordCount = sum(e.elementFrequency for e in self._by_label.values() if not e.special)

    def reindex(self, order):
        """Assign indices 0..n-1 following ``order`` (list of labels); drops everything else."""
        self._by_index = []
        keep = {}
        for i, lab in enumerate(order):
            e = self._by_label[lab]
            e.index = i
            keep[lab] = e
            self._by_index.append(e)
        self._by_label = keep

    # --- queries
    def containsWord(self, w):
        return w in self._by_label

    def containsElement(self, e):
        return e.label in self._by_label

    def wordFor(self, w):
        return self._by_label.get(w)

    tokenFor = wordFor
    elementFor = wordFor

    def indexOf(self, w):
        e = self._by_label.get(w)
        return -1 if e is None else e.index

    def wordAtIndex(self, i):
        e = self._by_index[i] if 0 <= i < len(self._by_index) else None
        return None if e is None else e.label

    def elementAtIndex(self, i):
        return self._by_index[i]

    def numWords(self):
        return len(self._by_index) if self._by_index else len(self._by_label)

    def words(self):
        return [e.label for e in self._by_index] if self._by_index else list(self._by_label)

    def vocabWords(self):
        return list(self._by_index) if self._by_index else list(self._by_label.values())

    tokens = vocabWords

    def wordFrequency(self, w):
        e = self._by_label.get(w)
        return 0 if e is None else int(e.elementFrequency)

    def docAppearedIn(self, w):
        e = self._by_label.get(w)
        return 0 if e is None else e.sequencesCount

    def incrementDocCount(self, w, by=1):
        e = self._by_label.get(w)
        if e is not None:
            e.sequencesCount += by

    def totalWordOccurrences(self):
        return int(self.totalWordCount)

    def totalNumberOfDocs(self):
        return self.numDocs

    def incrementTotalDocCount(self, by=1):
        self.numDocs += by

    def setTotalDocCount(self, n):
        self.numDocs = n

    def __len__(self):
        return self.numWords()


InMemoryLookupCache = AbstractCache


class VocabConstructor:
    """Builds the vocabulary from element sequences: counts, min-frequency / stop-word filtering (labels are
    always kept), index assignment by descending frequency, Huffman coding (VocabConstructor.java)."""

    def __init__(self, minElementFrequency=5, stopWords=None, useUnknown=False, unk="UNK"):
        self.minFreq = minElementFrequency
        self.stop = set(stopWords or [])
        self.useUnknown = useUnknown
        self.unk = unk

    def buildJointVocabulary(self, sequences, labels_per_seq=None, cache=None, buildHuffman=True):
        cache = AbstractCache() if cache is None else cache
        counts = {}
        docs = {}
        ndocs = 0
        for k, seq in enumerate(sequences):
            ndocs += 1
            seen = set()
            for t in seq:
                if t in self.stop:
                    continue
                counts[t] = counts.get(t, 0) + 1
                if t not in seen:
                    seen.add(t)
                    docs[t] = docs.get(t, 0) + 1
        labels = {}
        if labels_per_seq is not None:
            for ls in labels_per_seq:
                for l in ls:
                    labels.setdefault(l, None)
        return self.buildFromCounts(counts, docs, ndocs, list(labels), cache, buildHuffman)

    def buildFromCounts(self, counts, docs, ndocs, labels=(), cache=None, buildHuffman=True):
        """Vocabulary from (merged) element counts / document counts — the reduce step of the distributed
        text pipeline (dl4j-spark-nlp TextPipeline + WordFreqAccumulator)."""
        cache = AbstractCache() if cache is None else cache
        labels = list(labels)
        lset = set(labels)
        words = [w for w, c in counts.items() if c >= self.minFreq and w not in lset and w not in self.stop]
        dropped = sum(c for w, c in counts.items() if c < self.minFreq)
        words.sort(key=lambda w: (-counts[w], w))
        for w in words:
            e = VocabWord(w, counts[w])
            e.sequencesCount = docs.get(w, 0)
            cache.addToken(e)
        if self.useUnknown and dropped > 0:
            e = VocabWord(self.unk, dropped)
            cache.addToken(e)
            words.append(self.unk)
        for l in labels:
            e = VocabWord(l, 1.0, special=True)
            cache.addToken(e)
        cache.reindex(words + labels)
        cache.setTotalDocCount(ndocs)
        cache.updateWordsOccurrences()
        if buildHuffman:
            Huffman(cache.vocabWords()).build().applyIndexes(cache)
        return cache


class Huffman:
    """word2vec.c CreateBinaryTree over element frequencies (elements must be in index order)."""

    def __init__(self, elements):
        self.elements = list(elements)

    def build(self):
        V = len(self.elements)
        self.codes = [[] for _ in range(V)]
        self.points = [[] for _ in range(V)]
        if V < 2:
            return self
        # two-pointer merge over counts sorted descending (index order is already by frequency for words;
        # labels come last with frequency 1); sort defensively for arbitrary caches
        order = sorted(range(V), key=lambda i: -self.elements[i].elementFrequency)
        count = np.empty(2 * V, dtype=np.float64)
        count[:V] = [self.elements[i].elementFrequency for i in order]
        count[V:] = 1e30
        binary = np.zeros(2 * V, dtype=np.int8)
        parent = np.zeros(2 * V, dtype=np.int64)
        pos1, pos2 = V - 1, V
        for a in range(V - 1):
            mins = []
            for _ in range(2):
                if pos1 >= 0 and count[pos1] < count[pos2]:
                    mins.append(pos1)
                    pos1 -= 1
                else:
                    mins.append(pos2)
                    pos2 += 1
            count[V + a] = count[mins[0]] + count[mins[1]]
            parent[mins[0]] = V + a
            parent[mins[1]] = V + a
            binary[mins[1]] = 1
        root = 2 * V - 2
        for r, orig in enumerate(order):
            code, point = [], []
            b = r
            while b != root:
                code.append(int(binary[b]))
                point.append(b)
                b = parent[b]
                if len(code) > MAX_CODE_LENGTH:
                    break
            self.codes[orig] = code[::-1]
            pts = [root - V]
            for p in point[::-1][:-1]:          # inner nodes from the root's child down; the leaf is excluded
                pts.append(int(p) - V)
            self.points[orig] = pts[:len(self.codes[orig])]
        return self

    def applyIndexes(self, cache):
        for i, e in enumerate(self.elements):
            e.codes = self.codes[i]
            e.points = self.points[i]
        if not any(x is not None for x in cache._by_index):
            # an unindexed cache takes the Huffman order: most frequent element first (reference Huffman.applyIndexes)
            order = sorted(range(len(self.elements)), key=lambda i: -self.elements[i].elementFrequency)
            for rank, i in enumerate(order):
                cache.addWordToIndex(rank, self.elements[i].label)
        return cache


def huffman_arrays(cache):
    """Dense [V, maxc] uint8 codes, int32 points, int32 code lengths for the native kernels."""
    els = cache.vocabWords()
    V = len(els)
    maxc = max([len(e.codes) for e in els] + [1])
    codes = np.zeros((V, maxc), dtype=np.uint8)
    points = np.zeros((V, maxc), dtype=np.int32)
    lens = np.zeros(V, dtype=np.int32)
    for i, e in enumerate(els):
        L = len(e.codes)
        lens[i] = L
        if L:
            codes[i, :L] = e.codes
            points[i, :L] = e.points
    return codes, points, lens, maxc
