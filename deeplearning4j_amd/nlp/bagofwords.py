"""Bag-of-words / TF-IDF vectorizers and the CNN sentence iterator.

Reference: NLP:bagofwords/vectorizer/BagOfWordsVectorizer.java, TfidfVectorizer.java (tf = count/docLength,
idf = log10(totalDocs/docFreq), MathUtils.java:258-286), NLP:iterator/CnnSentenceDataSetIterator.java
(word vectors stacked into [mb, 1, maxLen, D] (sentences along height) or [mb, 1, D, maxLen], one-hot labels,
feature mask [mb, maxLen] for variable-length sentences).
"""
import math

import numpy as np
import torch

from ..datasets.dataset import DataSet, DataSetIterator
from .text import DefaultTokenizerFactory, LabelAwareIterator, SentenceIterator
from .vocab import VocabConstructor


class BaseTextVectorizer:
    class Builder:
        def __init__(self):
            self.tf = DefaultTokenizerFactory()
            self.it = None
            self.minFreq = 1
            self.stop = []
            self.vocab = None

        def setTokenizerFactory(self, tf): self.tf = tf; return self  # noqa: E704
        def setIterator(self, it): self.it = it; return self  # noqa: E704
        def setMinWordFrequency(self, v): self.minFreq = int(v); return self  # noqa: E704
        def setStopWords(self, s): self.stop = list(s); return self  # noqa: E704
        def setVocab(self, v): self.vocab = v; return self  # noqa: E704
        def allowParallelTokenization(self, v): return self  # noqa: E704

        def build(self):
            v = self.TARGET()
            v.tf, v.it, v.minFreq, v.stop, v.vocabCache = self.tf, self.it, self.minFreq, self.stop, self.vocab
            return v

    def __init__(self):
        self.tf = DefaultTokenizerFactory()
        self.it = None
        self.minFreq = 1
        self.stop = []
        self.vocabCache = None
        self.labels = []

    def _docs(self):
        it = self.it
        out = []
        if isinstance(it, LabelAwareIterator):
            it.reset()
            while it.hasNextDocument():
                d = it.nextDocument()
                out.append((d.content, d.labels))
        elif isinstance(it, SentenceIterator):
            it.reset()
            while it.hasNext():
                out.append((it.nextSentence(), []))
        else:
            out = [(x, []) if isinstance(x, str) else (x[0], [x[1]]) for x in it]
        return out

    def tokens(self, text):
        return self.tf.create(text).getTokens()

    def fit(self):
        docs = self._docs()
        seqs = [self.tokens(t) for t, _ in docs]
        self.labels = sorted({l for _, ls in docs for l in ls})
        self.vocabCache = VocabConstructor(self.minFreq, self.stop).buildJointVocabulary(seqs, buildHuffman=False)
        return self

    def getVocabCache(self):
        return self.vocabCache

    def _label_vec(self, label):
        y = torch.zeros(1, max(1, len(self.labels)))
        if label in self.labels:
            y[0, self.labels.index(label)] = 1.0
        return y

    def vectorize(self, text, label):
        return DataSet(self.transform(text), self._label_vec(label))


class BagOfWordsVectorizer(BaseTextVectorizer):
    def transform(self, text):
        toks = self.tokens(text) if isinstance(text, str) else list(text)
        v = torch.zeros(1, self.vocabCache.numWords())
        for t in toks:
            i = self.vocabCache.indexOf(t)
            if i >= 0:
                v[0, i] += 1.0
        return v


class TfidfVectorizer(BaseTextVectorizer):
    def tfidfWord(self, word, wordCount, documentLength):
        return self.tfForWord(wordCount, documentLength) * self.idfForWord(word)

    @staticmethod
    def tfForWord(count, docLength):
        return count / docLength if docLength else 0.0

    def idfForWord(self, word):
        n = self.vocabCache.totalNumberOfDocs()
        df = self.vocabCache.docAppearedIn(word)
        return math.log10(n / df) if n and df else 0.0

    def transform(self, text):
        toks = self.tokens(text) if isinstance(text, str) else list(text)
        v = torch.zeros(1, self.vocabCache.numWords())
        counts = {}
        for t in toks:
            counts[t] = counts.get(t, 0) + 1
        for t, c in counts.items():
            i = self.vocabCache.indexOf(t)
            if i >= 0:
                v[0, i] = self.tfidfWord(t, c, len(toks))
        return v


TfidfVectorizer.Builder = type("Builder", (BaseTextVectorizer.Builder,), {"TARGET": TfidfVectorizer})
BagOfWordsVectorizer.Builder = type("Builder", (BaseTextVectorizer.Builder,), {"TARGET": BagOfWordsVectorizer})


class LabeledSentenceProvider:
    def hasNext(self):
        raise NotImplementedError

    def nextSentence(self):
        raise NotImplementedError

    def reset(self):
        pass

    def totalNumSentences(self):
        raise NotImplementedError

    def allLabels(self):
        raise NotImplementedError


class CollectionLabeledSentenceProvider(LabeledSentenceProvider):
    def __init__(self, sentences, labels, seed=None):
        assert len(sentences) == len(labels)
        self.s, self.l = list(sentences), list(labels)
        self.order = np.arange(len(self.s))
        if seed is not None:
            np.random.RandomState(seed).shuffle(self.order)
        self._i = 0
        self._labels = sorted(set(self.l))

    def hasNext(self):
        return self._i < len(self.s)

    def nextSentence(self):
        k = self.order[self._i]
        self._i += 1
        return self.s[k], self.l[k]

    def reset(self):
        self._i = 0

    def totalNumSentences(self):
        return len(self.s)

    def allLabels(self):
        return list(self._labels)


class CnnSentenceDataSetIterator(DataSetIterator):
    class Builder:
        def __init__(self):
            self.kw = dict(provider=None, wordVectors=None, tf=DefaultTokenizerFactory(), unknown="RemoveWord",
                           maxLen=-1, mb=32, alongHeight=True, normalized=True)

        def sentenceProvider(self, p): self.kw["provider"] = p; return self  # noqa: E704
        def wordVectors(self, w): self.kw["wordVectors"] = w; return self  # noqa: E704
        def tokenizerFactory(self, t): self.kw["tf"] = t; return self  # noqa: E704
        def unknownWordHandling(self, u): self.kw["unknown"] = str(u); return self  # noqa: E704
        def maxSentenceLength(self, n): self.kw["maxLen"] = int(n); return self  # noqa: E704
        def minibatchSize(self, n): self.kw["mb"] = int(n); return self  # noqa: E704
        def sentencesAlongHeight(self, b): self.kw["alongHeight"] = bool(b); return self  # noqa: E704
        def useNormalizedWordVectors(self, b): self.kw["normalized"] = bool(b); return self  # noqa: E704

        def build(self):
            return CnnSentenceDataSetIterator(**self.kw)

    def __init__(self, provider, wordVectors, tf, unknown, maxLen, mb, alongHeight, normalized):
        self.p, self.wv, self.tf = provider, wordVectors, tf
        self.unknown, self.maxLen, self.mb = unknown, maxLen, mb
        self.alongHeight, self.normalized = alongHeight, normalized
        self.labels = provider.allLabels()
        self.D = wordVectors.getLayerSize()
        self._unk = None

    def _vec(self, w):
        m = self.wv.getWordVectorMatrixNormalized(w) if self.normalized else self.wv.getWordVectorMatrix(w)
        return None if m is None else m.reshape(-1).float().cpu()

    def _tokens(self, s):
        toks = self.tf.create(s).getTokens()
        if self.unknown == "RemoveWord":
            toks = [t for t in toks if self.wv.hasWord(t)]
        return toks

    def hasNext(self):
        return self.p.hasNext()

    def reset(self):
        self.p.reset()

    def batch(self):
        return self.mb

    def totalOutcomes(self):
        return len(self.labels)

    def getLabels(self):
        return list(self.labels)

    def next(self, num=None):
        n = num or self.mb
        sents = []
        while len(sents) < n and self.p.hasNext():
            s, l = self.p.nextSentence()
            sents.append((self._tokens(s), l))
        L = max([len(t) for t, _ in sents] + [1])
        if self.maxLen > 0:
            L = min(L, self.maxLen)
        B = len(sents)
        feats = torch.zeros(B, 1, L, self.D) if self.alongHeight else torch.zeros(B, 1, self.D, L)
        labels = torch.zeros(B, len(self.labels))
        mask = torch.zeros(B, L)
        for i, (toks, lab) in enumerate(sents):
            toks = toks[:L]
            for j, t in enumerate(toks):
                v = self._vec(t)
                if v is None:
                    v = torch.zeros(self.D)
                if self.alongHeight:
                    feats[i, 0, j] = v
                else:
                    feats[i, 0, :, j] = v
            mask[i, :len(toks)] = 1.0
            labels[i, self.labels.index(lab)] = 1.0
        ds = DataSet(feats, labels, mask if any(len(t) < L for t, _ in sents) else None, None)
        return self._pp(ds)
