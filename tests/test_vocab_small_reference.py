"""Vocabulary ports, after the reference's VocabWordFactoryTest / AbstractElementFactoryTest
(deeplearning4j-nlp/src/test/java/org/deeplearning4j/models/sequencevectors/serialization/), AbstractCacheTest
(.../models/word2vec/wordstore/inmemory/AbstractCacheTest.java) and LabelsSourceTest (.../text/documentiterator/
LabelsSourceTest.java): elements round-trip through JSON and the element factory, the cache counts words and
occurrences, removes elements, lists labels and takes Huffman indexes (most frequent first), and LabelsSource
generates / replays labels and counts them. CPU."""
import deeplearning4j_amd.nlp as N
from deeplearning4j_amd.nlp.vocab import AbstractCache, AbstractElementFactory, Huffman, VocabWord


def test_element_factory_deserialize_and_serialize():
    word = VocabWord(1, "word")
    f = AbstractElementFactory(VocabWord)
    assert f.deserialize(word.toJSON()) == word
    w2 = f.deserialize(f.serialize(word))
    assert w2 == word and w2.getElementFrequency() == 1.0


def _cache():
    c = AbstractCache.Builder().build()
    c.addToken(VocabWord(1.0, "word"))
    c.addToken(VocabWord(2.0, "test"))
    c.addToken(VocabWord(3.0, "tester"))
    return c


def test_cache_num_words_and_occurrences():
    c = AbstractCache.Builder().build()
    c.addToken(VocabWord(1.0, "word"))
    c.addToken(VocabWord(1.0, "test"))
    assert c.numWords() == 2
    c = _cache()
    assert c.numWords() == 3 and c.totalWordOccurrences() == 6


def test_cache_huffman():
    c = _cache()
    h = Huffman(c.tokens())
    h.build()
    h.applyIndexes(c)
    assert [c.wordAtIndex(i) for i in range(3)] == ["tester", "test", "word"]
    assert c.tokenFor("tester").getIndex() == 0


def test_cache_removal_and_labels():
    c = _cache()
    c.removeElement("tester")
    assert c.numWords() == 2 and c.totalWordOccurrences() == 3
    words = _cache().words()
    assert len(words) == 3 and {"word", "test", "tester"} <= set(words)


def test_labels_source():
    assert N.LabelsSource("SENTENCE_").nextLabel() == "SENTENCE_0"
    assert N.LabelsSource("SENTENCE_%d_HAHA").nextLabel() == "SENTENCE_0_HAHA"
    g = N.LabelsSource(["LABEL0", "LABEL1", "LABEL2"])
    assert [g.nextLabel() for _ in range(3)] == ["LABEL0", "LABEL1", "LABEL2"]
    assert g.getNumberOfLabelsUsed() == 3
    g = N.LabelsSource("SENTENCE_")
    assert [g.nextLabel() for _ in range(5)] == [f"SENTENCE_{i}" for i in range(5)]
    assert g.getNumberOfLabelsUsed() == 5
    g.reset()
    assert g.getNumberOfLabelsUsed() == 5
