"""NLP + graph embeddings (reference test strategy: NLP Word2VecTests / ParagraphVectorsTest / GloveTest /
WordVectorSerializerTest, deeplearning4j-graph TestDeepWalk / TestGraphHuffman / TestGraphLoading).

No text corpora ship with the reference snapshot (raw_sentences.txt lives in dl4j-test-resources), so the corpora
here are synthetic with a planted structure: two disjoint topics whose words only co-occur within their topic.
Trained embeddings must separate the topics; exact vectors are "parity unpinned" (Hogwild training).
"""
import os

import numpy as np
import pytest
import torch

from deeplearning4j_amd.nlp import (CollectionSentenceIterator, CommonPreprocessor, DefaultTokenizerFactory,
                                    EndingPreProcessor, LabelledDocument, NGramTokenizerFactory, ParagraphVectors,
                                    SimpleLabelAwareIterator, VocabConstructor, Word2Vec)
from deeplearning4j_amd.nlp.bagofwords import (BagOfWordsVectorizer, CnnSentenceDataSetIterator,
                                               CollectionLabeledSentenceProvider, TfidfVectorizer)
from deeplearning4j_amd.nlp.glove import Glove, cooccurrences
from deeplearning4j_amd.nlp.serializer import WordVectorSerializer
from _ref_fixtures import path as _ref_path

A = [f"alpha{i}" for i in range(20)]
B = [f"beta{i}" for i in range(20)]


def _corpus(n=2000, seed=0, length=12):
    rng = np.random.RandomState(seed)
    return [" ".join(rng.choice(A if k % 2 == 0 else B, length)) for k in range(n)]


def _separation(m):
    s_in = np.mean([m.similarity("alpha0", w) for w in A[1:]])
    s_out = np.mean([m.similarity("alpha0", w) for w in B])
    return s_in, s_out


def test_tokenizers_and_preprocessors():
    tf = DefaultTokenizerFactory()
    tf.setTokenPreProcessor(CommonPreprocessor())
    assert tf.create("Hello, World! It's 42 (ok).").getTokens() == ["hello", "world", "its", "ok"]
    assert EndingPreProcessor().preProcess("jumping") == "jump"
    ng = NGramTokenizerFactory(DefaultTokenizerFactory(), 1, 2)
    assert ng.create("a b c").getTokens() == ["a", "b", "c", "a b", "b c"]


def test_vocab_and_huffman():
    seqs = [["a"] * 5 + ["b"] * 3 + ["c"] * 2 + ["d"]]
    v = VocabConstructor(1).buildJointVocabulary(seqs)
    assert v.words() == ["a", "b", "c", "d"]
    # word2vec.c: most frequent word gets the shortest code, points start at the root (V-2)
    assert [len(e.codes) for e in v.vocabWords()] == [1, 2, 3, 3]
    assert all(e.points[0] == 2 for e in v.vocabWords())
    v2 = VocabConstructor(2).buildJointVocabulary(seqs)
    assert v2.words() == ["a", "b", "c"]


@pytest.mark.parametrize("algo,hs,neg", [("SkipGram", True, 0), ("SkipGram", False, 5), ("CBOW", True, 0),
                                         ("CBOW", False, 5)])
def test_word2vec_topics(algo, hs, neg):
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(32).windowSize(4).seed(42).epochs(2) \
        .elementsLearningAlgorithm(algo).useHierarchicSoftmax(hs).negativeSample(neg) \
        .iterate(CollectionSentenceIterator(_corpus())).device("cpu").build()
    w2v.fit()
    s_in, s_out = _separation(w2v)
    assert s_in > s_out + 0.3, (s_in, s_out)
    near = w2v.wordsNearest("alpha0", 5)
    assert len(near) == 5 and all(w.startswith("alpha") for w in near)
    assert "alpha0" not in near


def test_word2vec_subsampling_and_analogy_api():
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(16).windowSize(3).seed(1).sampling(1e-3) \
        .iterate(CollectionSentenceIterator(_corpus(500))).device("cpu").build()
    w2v.fit()
    assert w2v.getWordVector("alpha1").shape == (16,)
    assert w2v.getWordVectorsMean(["alpha1", "alpha2"]).shape == (1, 16)
    assert len(w2v.wordsNearest(["alpha1", "alpha2"], ["beta1"], 3)) == 3
    assert len(w2v.wordsNearestSum("alpha1", 4)) == 4
    assert w2v.similarWordsInVocabTo("alpha1", 0.9) == ["alpha1"] or "alpha1" in w2v.similarWordsInVocabTo("alpha1", 0.9)


@pytest.mark.parametrize("algo", ["dbow", "dm"])
def test_paragraph_vectors(algo):
    rng = np.random.RandomState(0)
    docs = [LabelledDocument(" ".join(rng.choice(A if k % 2 == 0 else B, 15)), ["TA" if k % 2 == 0 else "TB"])
            for k in range(400)]
    pv = ParagraphVectors.Builder().minWordFrequency(1).layerSize(32).windowSize(4).seed(42).epochs(5) \
        .sequenceLearningAlgorithm(algo).trainWordVectors(True).iterate(SimpleLabelAwareIterator(docs)) \
        .device("cpu").build()
    pv.fit()
    ta = " ".join(rng.choice(A, 15))
    tb = " ".join(rng.choice(B, 15))
    assert pv.predict(ta) == "TA" and pv.predict(tb) == "TB"
    assert pv.similarityToLabel(ta, "TA") > pv.similarityToLabel(ta, "TB")
    assert sorted(pv.getLabelsSource().getLabels()) == ["TA", "TB"]
    # labels are not returned as words
    assert all(not w.startswith("T") for w in pv.wordsNearest("alpha0", 10))


def test_glove():
    i, j, x = cooccurrences([np.array([0, 1, 2], np.int32)], 2, True)
    got = {(a, b): c for a, b, c in zip(i.tolist(), j.tolist(), x.tolist())}
    assert got == {(1, 0): 1.0, (0, 1): 1.0, (2, 1): 1.0, (1, 2): 1.0, (2, 0): 0.5, (0, 2): 0.5}
    g = Glove.Builder().iterate(CollectionSentenceIterator(_corpus())).minWordFrequency(1).layerSize(24) \
        .epochs(15).windowSize(4).seed(1).device("cpu").build()
    g.fit()
    assert g.lossHistory[-1] < g.lossHistory[0] * 0.1
    s_in, s_out = _separation(g)
    assert s_in > s_out + 0.3


def test_serializer_roundtrips(tmp_path):
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(8).windowSize(2).seed(3).negativeSample(3) \
        .iterate(CollectionSentenceIterator(_corpus(200))).device("cpu").build()
    w2v.fit()
    p = str(tmp_path / "w2v.zip")
    WordVectorSerializer.writeWord2VecModel(w2v, p)
    r = WordVectorSerializer.readWord2VecModel(p)
    assert r.vocab().words() == w2v.vocab().words()
    assert torch.allclose(r.lookupTable().syn0, w2v.lookupTable().syn0, atol=1e-6)
    assert torch.allclose(r.lookupTable().syn1Neg, w2v.lookupTable().syn1Neg, atol=1e-6)
    assert r.vocab().wordFor("alpha3").codes == w2v.vocab().wordFor("alpha3").codes
    assert abs(r.similarity("alpha0", "alpha1") - w2v.similarity("alpha0", "alpha1")) < 1e-5
    # continued training of a restored model works
    r.sentenceIter = CollectionSentenceIterator(_corpus(50))
    r.sequences = None
    t = str(tmp_path / "v.txt")
    WordVectorSerializer.writeWordVectors(w2v, t)
    s = WordVectorSerializer.loadTxtVectors(t)
    assert np.allclose(s.getWordVector("beta2"), w2v.getWordVector("beta2"), atol=1e-6)
    b = str(tmp_path / "v.bin")
    WordVectorSerializer.writeBinaryModel(w2v, b)
    s2 = WordVectorSerializer.readBinaryModel(b)
    assert np.allclose(s2.getWordVector("beta2"), w2v.getWordVector("beta2"), atol=1e-6)
    assert WordVectorSerializer.loadStaticModel(p).vocab().numWords() == w2v.vocab().numWords()
    # plain "word v1 v2" text without header (GloVe text format)
    g = tmp_path / "glove.txt"
    g.write_text("cat 1 0 0\ndog 0.9 0.1 0\ncar 0 0 1\n")
    gv = WordVectorSerializer.loadTxtVectors(str(g))
    assert gv.wordsNearest("cat", 1) == ["dog"]
    vc = str(tmp_path / "vocab.json")
    WordVectorSerializer.writeVocabCache(w2v.vocab(), vc)
    assert WordVectorSerializer.readVocabCache(vc).words() == w2v.vocab().words()


def test_paragraph_vectors_serializer(tmp_path):
    docs = [LabelledDocument(" ".join(_corpus(1, k)[0].split()), [f"D{k}"]) for k in range(20)]
    pv = ParagraphVectors.Builder().minWordFrequency(1).layerSize(8).seed(1).iterate(SimpleLabelAwareIterator(docs)) \
        .device("cpu").build()
    pv.fit()
    p = str(tmp_path / "pv.zip")
    WordVectorSerializer.writeParagraphVectors(pv, p)
    r = WordVectorSerializer.readParagraphVectors(p)
    assert sorted(r.getLabelsSource().getLabels()) == sorted(pv.getLabelsSource().getLabels())
    assert r.nearestLabels(docs[3].content, 3)


def test_bag_of_words_tfidf_and_cnn_iterator():
    docs = [LabelledDocument("the cat sat", ["pos"]), LabelledDocument("the dog ran", ["neg"])]
    bow = BagOfWordsVectorizer.Builder().setIterator(SimpleLabelAwareIterator(docs)).build().fit()
    v = bow.transform("the cat cat")
    assert v[0, bow.getVocabCache().indexOf("cat")] == 2 and v[0, bow.getVocabCache().indexOf("the")] == 1
    tf = TfidfVectorizer.Builder().setIterator(SimpleLabelAwareIterator(docs)).build().fit()
    t = tf.transform("the cat")
    assert t[0, tf.getVocabCache().indexOf("the")] == 0.0          # appears in every doc: idf 0
    assert abs(float(t[0, tf.getVocabCache().indexOf("cat")]) - 0.5 * np.log10(2)) < 1e-6
    ds = tf.vectorize("the dog", "neg")
    assert ds.labels.shape == (1, 2)
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(8).seed(1) \
        .iterate(CollectionSentenceIterator(_corpus(100))).device("cpu").build()
    w2v.fit()
    prov = CollectionLabeledSentenceProvider(["alpha1 alpha2 alpha3", "beta1 unknownword"], ["a", "b"])
    it = CnnSentenceDataSetIterator.Builder().sentenceProvider(prov).wordVectors(w2v).minibatchSize(2).build()
    d = it.next()
    assert d.features.shape == (2, 1, 3, 8) and d.labels.tolist() == [[1, 0], [0, 1]]
    assert d.featuresMask.tolist() == [[1, 1, 1], [1, 0, 0]]


R = _ref_path("deeplearning4j-graph/src/test/resources") + "/"


@pytest.mark.skipif(not os.path.isdir(R), reason="reference graph fixtures not present")
def test_graph_loading_and_walks():
    from deeplearning4j_amd.graph import (GraphLoader, NoEdgeHandling, NoEdgesException, RandomWalkIterator,
                                          WeightedRandomWalkIterator, Graph)
    g = GraphLoader.loadUndirectedGraphEdgeListFile(R + "testgraph_7vertices.txt", 7)
    assert g.numVertices() == 7
    assert sorted(g.getConnectedVertexIndices(4)) == [1, 2, 3, 5, 6]
    it = RandomWalkIterator(g, 8, 12345)
    walks = [it.next().indices() for _ in range(7)]
    assert not it.hasNext()
    assert sorted(w[0] for w in walks) == list(range(7))
    for w in walks:
        assert len(w) == 9
        for a, b in zip(w[:-1], w[1:]):
            assert b in g.getConnectedVertexIndices(a)
    gw = GraphLoader.loadWeightedEdgeListFile(R + "WeightedGraph.txt", 9, ",", True)
    assert [(e.to, e.value) for e in gw.getEdgesOut(1)] == [(2, 12.0), (4, 14.0)]
    wit = WeightedRandomWalkIterator(gw, 20, 7)
    while wit.hasNext():
        w = wit.next().indices()
        for a, b in zip(w[:-1], w[1:]):
            assert b in gw.getConnectedVertexIndices(a)
    # directed graph with a sink: self loops, or an exception when requested
    d = Graph(3)
    d.addEdge(0, 1, None, True)
    w = RandomWalkIterator(d, 4, 1).all_walks()
    assert (w[w[:, 0] == 1] == 1).all()
    with pytest.raises(NoEdgesException):
        RandomWalkIterator(d, 4, 1, NoEdgeHandling.EXCEPTION_ON_DISCONNECTED).all_walks()


def test_graph_huffman():
    from deeplearning4j_amd.graph import GraphHuffman
    h = GraphHuffman(7).buildTree([1, 2, 3, 4, 5, 6, 7])
    lens = [h.getCodeLength(i) for i in range(7)]
    assert lens[6] == 2 and lens[0] == 4
    codes = {h.getCodeString(i) for i in range(7)}
    assert len(codes) == 7
    for a in codes:                      # prefix-free
        for b in codes:
            assert a == b or not b.startswith(a)
    assert all(h.getPathInnerNodes(i)[0] == 0 for i in range(7))


@pytest.mark.skipif(not os.path.isdir(R), reason="reference graph fixtures not present")
def test_deepwalk(tmp_path):
    from deeplearning4j_amd.graph import DeepWalk, GraphLoader, GraphVectorSerializer
    g = GraphLoader.loadUndirectedGraphEdgeListFile(R + "graph13.txt", 13)
    dw = DeepWalk.Builder().vectorSize(16).windowSize(2).learningRate(0.05).seed(1).device("cpu").build()
    dw.initialize(g)
    s0 = dw.lookupTable().calculateScore(0, 1)
    for _ in range(40):
        dw.fit(g, 10)
    assert dw.lookupTable().calculateScore(0, 1) < s0
    assert dw.similarity(0, 1) > dw.similarity(0, 12)
    p = str(tmp_path / "g.txt")
    GraphVectorSerializer.writeGraphVectors(dw, p)
    r = GraphVectorSerializer.loadTxtVectors(p)
    assert torch.allclose(r.getVertexVector(5), dw.getVertexVector(5).cpu(), atol=1e-6)
