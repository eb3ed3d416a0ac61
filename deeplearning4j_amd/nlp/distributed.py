"""Distributed Word2Vec / ParagraphVectors training over torch.distributed — the replacement for dl4j-spark-nlp's
``SparkWord2Vec`` (deeplearning4j-scaleout/spark/dl4j-spark-nlp/.../word2vec/Word2Vec.java, TextPipeline,
WordFreqAccumulator, FirstIterationFunction / SecondIterationFunction) and the Spark-NLP sequence-vectors path.

Pipeline (one process per GPU, RCCL over xGMI; gloo on CPU):
1. **Text pipeline** — every rank tokenizes its own shard of the corpus and counts element / document frequencies;
   the counters are all-gathered and merged, and every rank builds the identical vocabulary + Huffman tree from the
   merged counts (``VocabConstructor.buildFromCounts``).
2. **Training** — every rank initialises the same lookup table (same seed), trains one epoch on its shard with the
   native embedding engine (gfx950 skip-gram/CBOW kernels), then syn0 / syn1 / syn1Neg are averaged with one
   all-reduce per table (parameter averaging, as the Spark implementation folds partition results). The learning
   rate decays linearly across the global epoch schedule.
"""
import collections

import torch
import torch.distributed as dist

from .vocab import VocabConstructor


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def merge_counts(local_counts, local_docs, local_ndocs):
    """All-gather and merge (counts, doc counts, #docs) dicts across ranks."""
    world, _ = _world()
    if world == 1:
        return dict(local_counts), dict(local_docs), int(local_ndocs)
    objs = [None] * world
    dist.all_gather_object(objs, (dict(local_counts), dict(local_docs), int(local_ndocs)))
    counts, docs, nd = collections.Counter(), collections.Counter(), 0
    for c, d, n in objs:
        counts.update(c)
        docs.update(d)
        nd += n
    return dict(counts), dict(docs), nd


def count_sequences(sequences, stop=()):
    stop = set(stop or ())
    counts, docs = collections.Counter(), collections.Counter()
    n = 0
    for seq in sequences:
        n += 1
        seen = set()
        for t in seq:
            if t in stop:
                continue
            counts[t] += 1
            if t not in seen:
                seen.add(t)
                docs[t] += 1
    return counts, docs, n


def average_tables(lookup):
    """In-place mean of syn0 / syn1 / syn1Neg across ranks (one all-reduce per table)."""
    world, _ = _world()
    if world == 1:
        return
    for name in ("syn0", "syn1", "syn1Neg"):
        t = getattr(lookup, name, None)
        if t is None:
            continue
        if dist.get_backend() == "nccl" and not t.is_cuda:
            buf = t.cuda()
            dist.all_reduce(buf)
            t.copy_(buf.cpu())
        else:
            dist.all_reduce(t)
        t.div_(world)
    if hasattr(lookup, "invalidate"):
        lookup.invalidate()


class DistributedWord2Vec:
    """Data-parallel Word2Vec / ParagraphVectors. ``model`` is a configured (not yet fitted) Word2Vec or
    ParagraphVectors whose iterator yields THIS rank's shard. ``fit()`` trains it in place and returns it."""

    def __init__(self, model, averageEvery=1):
        self.model = model
        self.averageEvery = max(1, int(averageEvery))

    def _build_global_vocab(self):
        m = self.model
        m._load_sequences()
        c = m.conf
        counts, docs, nd = count_sequences(m.sequences, c.stopList)
        counts, docs, nd = merge_counts(counts, docs, nd)
        labels = []
        if m.seq_labels is not None:
            world, _ = _world()
            local = sorted({l for ls in m.seq_labels for l in ls})
            if world > 1:
                objs = [None] * world
                dist.all_gather_object(objs, local)
                local = sorted({l for o in objs for l in o})
            labels = local
        vc = VocabConstructor(c.minWordFrequency, c.stopList, c.useUnknown, c.UNK)
        m.vocabCache = vc.buildFromCounts(counts, docs, nd, labels)
        m.setVocab(m.vocabCache)
        c.vocabSize = m.vocabCache.numWords()

    def fit(self):
        m = self.model
        c = m.conf
        self._build_global_vocab()
        m.resetWeights()                          # same seed on every rank -> identical initial tables
        epochs = max(1, c.epochs)
        lr0, lr_min = c.learningRate, c.minLearningRate
        try:
            c.epochs = 1
            for e in range(epochs):
                # linear decay over the global schedule, split into per-epoch segments
                c.learningRate = lr0 - (lr0 - lr_min) * e / epochs
                c.minLearningRate = lr0 - (lr0 - lr_min) * (e + 1) / epochs
                m.fit()
                if (e + 1) % self.averageEvery == 0 or e == epochs - 1:
                    average_tables(m._lookup)
        finally:
            c.epochs, c.learningRate, c.minLearningRate = epochs, lr0, lr_min
        return m


SparkWord2Vec = DistributedWord2Vec
