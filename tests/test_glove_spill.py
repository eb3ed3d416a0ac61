"""GloVe co-occurrence counting under a memory cap (reference NLP:models/glove/AbstractCoOccurrences.java:55-104,
185-266, 387-520 and count/{Binary,ASCII}CoOccurrence{Reader,Writer}.java): the native counter spills sorted runs
when its map fills and merges them into one table equal to the unbounded count; the reference's binary and ASCII
record formats round-trip; GloVe trains over the memory-mapped merged table. CPU."""
import os

import numpy as np

from deeplearning4j_amd.nlp import CollectionSentenceIterator
from deeplearning4j_amd.nlp.glove import (ASCIICoOccurrenceReader, ASCIICoOccurrenceWriter, BinaryCoOccurrenceReader,
                                          BinaryCoOccurrenceWriter, CoOccurrenceCounter, Glove, cooccurrences)

A = [f"alpha{i}" for i in range(20)]
B = [f"beta{i}" for i in range(20)]


def _corpus(n=1500, seed=0, length=12):
    rng = np.random.RandomState(seed)
    return [" ".join(rng.choice(A if k % 2 == 0 else B, length)) for k in range(n)]


def _seqs(n=400, V=300, seed=1):
    rng = np.random.RandomState(seed)
    return [rng.randint(0, V, size=rng.randint(3, 30)).astype(np.int32) for _ in range(n)]


def test_spilled_count_equals_unbounded(tmp_path):
    seqs = _seqs()
    i0, j0, x0 = cooccurrences(seqs, 5, True)
    c = CoOccurrenceCounter(5, True, maxEntries=2000, workDir=str(tmp_path))
    for a in range(0, len(seqs), 37):
        c.add(seqs[a:a + 37])
    assert c.spills() >= 5
    t = c.finish()
    assert len(t) == len(i0)
    np.testing.assert_array_equal(np.asarray(t["i"]), i0)
    np.testing.assert_array_equal(np.asarray(t["j"]), j0)
    np.testing.assert_allclose(np.asarray(t["x"]), x0, rtol=1e-5)
    runs = [f for f in os.listdir(tmp_path) if f.startswith("cooc_run_")]
    assert runs == []                                   # run files removed after the merge
    c.close()


def test_memory_cap_in_bytes_and_asymmetric(tmp_path):
    seqs = _seqs(200, 50, 3)
    c = CoOccurrenceCounter(3, False, maxMemoryBytes=64 * 1024 * 2, workDir=str(tmp_path))   # 1024 pairs
    c.add(seqs)
    t = c.finish()
    i0, j0, x0 = cooccurrences(seqs, 3, False)
    assert c.spills() >= 1 and len(t) == len(i0)
    np.testing.assert_allclose(np.asarray(t["x"]), x0, rtol=1e-5)
    c.close()


def test_reference_record_formats_round_trip(tmp_path):
    i, j, x = cooccurrences(_seqs(50, 30, 4), 4, True)
    w = BinaryCoOccurrenceWriter(str(tmp_path / "c.bin"))
    w.writeArrays(i[:-1], j[:-1], x[:-1])
    w.writeObject(int(i[-1]), int(j[-1]), float(x[-1]))
    w.finish()
    assert os.path.getsize(tmp_path / "c.bin") == 16 * len(i)      # big-endian int, int, double per record
    r = BinaryCoOccurrenceReader(str(tmp_path / "c.bin"))
    assert r.nextObject() == (int(i[0]), int(j[0]), float(x[0]))
    bi, bj, bx = r.arrays()
    np.testing.assert_array_equal(bi, i)
    np.testing.assert_array_equal(bx, x)
    aw = ASCIICoOccurrenceWriter(str(tmp_path / "c.txt"))
    for a, b, v in zip(i[:10], j[:10], x[:10]):
        aw.writeObject(a, b, v)
    aw.finish()
    ar = ASCIICoOccurrenceReader(str(tmp_path / "c.txt"))
    got = []
    while ar.hasMoreObjects():
        got.append(ar.nextObject())
    ar.finish()
    assert got == [(int(a), int(b), float(v)) for a, b, v in zip(i[:10], j[:10], x[:10])]


def test_glove_trains_over_spilled_table():
    g = Glove.Builder().iterate(CollectionSentenceIterator(_corpus())).minWordFrequency(1).layerSize(24) \
        .epochs(15).windowSize(4).seed(1).device("cpu").build()
    g.maxCoOccurrences = 300                            # 40-word vocabulary: ~1.6k pairs -> several spills
    g.streamBlock = 256
    g.fit()
    assert g.coOccurrenceSpills >= 3
    assert g.lossHistory[-1] < g.lossHistory[0] * 0.1
    s_in = np.mean([g.similarity("alpha0", w) for w in A[1:]])
    s_out = np.mean([g.similarity("alpha0", w) for w in B])
    assert s_in > s_out + 0.3
    g2 = Glove.Builder().iterate(CollectionSentenceIterator(_corpus(200))).minWordFrequency(1).layerSize(8) \
        .maxMemory(1).epochs(2).windowSize(2).seed(1).device("cpu").build()
    assert g2.maxMemoryBytes == float(1 << 30)
    g2.fit()
