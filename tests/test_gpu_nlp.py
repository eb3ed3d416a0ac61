"""gfx950 embedding kernels (csrc/embeddings.hip) vs the C++ CPU applier (csrc/runtime/embeddings.cpp).

Items are applied one per launch on both sides, so the (otherwise Hogwild) update order is identical and the
results must agree to float rounding (__expf vs expf). Also: a Word2Vec / ParagraphVectors / GloVe / DeepWalk fit
entirely on the GPU separates planted topics.
"""
import copy

import numpy as np
import pytest
import torch

from deeplearning4j_amd.nlp import CollectionSentenceIterator, Word2Vec
from deeplearning4j_amd.nlp.embeddings import (EmbeddingEngine, F_HS, F_NS, F_UPD_IN, F_UPD_OUT, M_CBOW, M_SG)

pytestmark = pytest.mark.gpu

A = [f"alpha{i}" for i in range(20)]
B = [f"beta{i}" for i in range(20)]


def _corpus(n=2000, seed=0):
    rng = np.random.RandomState(seed)
    return [" ".join(rng.choice(A if k % 2 == 0 else B, 12)) for k in range(n)]


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _model(D, neg):
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(D).windowSize(3).seed(5).negativeSample(neg) \
        .iterate(CollectionSentenceIterator(_corpus(300))).device("cpu").build()
    w2v.fit()                                # non-trivial syn1/syn1neg state
    return w2v


@pytest.mark.parametrize("D", [48, 100, 300])
@pytest.mark.parametrize("mode", [M_SG, M_CBOW])
def test_w2v_kernel_matches_cpu(cuda, D, mode):
    w2v = _model(D, 4)
    cpu_t = w2v.lookupTable()
    gpu_t = copy.copy(cpu_t)
    gpu_t.device = cuda
    for n in ("syn0", "syn1", "syn1Neg"):
        setattr(gpu_t, n, getattr(cpu_t, n).clone())
    cpu_t2 = copy.copy(cpu_t)
    for n in ("syn0", "syn1", "syn1Neg"):
        setattr(cpu_t2, n, getattr(cpu_t, n).clone())
    gpu_t.to(cuda)
    e_cpu, e_gpu = EmbeddingEngine(cpu_t2, 1), EmbeddingEngine(gpu_t)
    seqs, _ = w2v._index_sequences()
    items = e_cpu._batch(np.concatenate(seqs[:6]).astype(np.int32), np.array([0] + list(np.cumsum(
        [len(s) for s in seqs[:6]])), np.int64), None, None, None, 3, mode, [7], 0.05, 0.05, 0, 0)
    n = len(items[1])
    assert n > 20
    flags = F_HS | F_NS | F_UPD_IN | F_UPD_OUT
    for k in range(n):                      # one item per launch: identical update order on both sides
        if mode == M_SG:
            one = (items[0][k:k + 1], items[1][k:k + 1], items[2][k:k + 1], None, None, 0)
        else:
            c0, c1 = items[3][k], items[3][k + 1]
            one = (None, items[1][k:k + 1], items[2][k:k + 1], np.array([0, c1 - c0], np.int32),
                   items[4][c0:c1].copy(), 0)
        e_cpu._apply(mode, one, flags)
        e_gpu._apply(mode, one, flags)
    torch.cuda.synchronize()
    for nme in ("syn0", "syn1", "syn1Neg"):
        g = getattr(gpu_t, nme).cpu()
        c = getattr(cpu_t2, nme)
        assert not torch.equal(c, getattr(cpu_t, nme)), f"{nme} unchanged"
        torch.testing.assert_close(g, c, rtol=1e-4, atol=2e-5)


def test_glove_kernel_matches_cpu(cuda):
    from deeplearning4j_amd.nlp.embeddings import _np_ptr, _t_ptr
    from deeplearning4j_amd.nlp.glove import cooccurrences
    from deeplearning4j_amd.ops import native, runtime as RT
    import ctypes
    from deeplearning4j_amd.nlp import glove as G  # noqa: F401  (registers signatures)
    rng = np.random.RandomState(0)
    seqs = [rng.randint(0, 30, 20).astype(np.int32) for _ in range(20)]
    ei, ej, ex = cooccurrences(seqs, 3)
    V, D = 30, 70
    W = (torch.rand(V, D, generator=torch.Generator().manual_seed(1)) - 0.5) / D
    b, hW, hb = torch.zeros(V), torch.zeros(V, D), torch.zeros(V)
    Wg, bg, hWg, hbg = (t.clone().to(cuda) for t in (W, b, hW, hb))
    lib = native.load()
    native.register_sig("dl4j_glove", [ctypes.c_void_p] * 3 + [ctypes.c_longlong] + [ctypes.c_void_p] * 4 +
                        [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                         ctypes.c_int, ctypes.c_void_p])
    rt = RT.load()
    dev_e = [torch.from_numpy(a).to(cuda) for a in (ei, ej, ex)]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for k in range(min(200, len(ei))):
        rt.rt_glove_apply(_np_ptr(ei[k:k + 1]), _np_ptr(ej[k:k + 1]), _np_ptr(ex[k:k + 1]), 1, _t_ptr(W), _t_ptr(b),
                          _t_ptr(hW), _t_ptr(hb), D, 0.05, 100.0, 0.75, 1)
        assert lib.dl4j_glove(_t_ptr(dev_e[0][k:]), _t_ptr(dev_e[1][k:]), _t_ptr(dev_e[2][k:]), 1, _t_ptr(Wg),
                              _t_ptr(bg), _t_ptr(hWg), _t_ptr(hbg), D, 0.05, 100.0, 0.75, None, 0, s) == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(Wg.cpu(), W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bg.cpu(), b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("algo", ["SkipGram", "CBOW"])
def test_word2vec_on_gpu(cuda, algo):
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(64).windowSize(4).seed(42).epochs(2).negativeSample(5) \
        .elementsLearningAlgorithm(algo).iterate(CollectionSentenceIterator(_corpus())).device(cuda).build()
    w2v.fit()
    assert w2v.lookupTable().syn0.is_cuda
    s_in = np.mean([w2v.similarity("alpha0", w) for w in A[1:]])
    s_out = np.mean([w2v.similarity("alpha0", w) for w in B])
    assert s_in > s_out + 0.3
    assert all(w.startswith("alpha") for w in w2v.wordsNearest("alpha0", 5))


def test_glove_on_gpu(cuda):
    from deeplearning4j_amd.nlp.glove import Glove
    g = Glove.Builder().iterate(CollectionSentenceIterator(_corpus())).minWordFrequency(1).layerSize(24) \
        .epochs(15).windowSize(4).seed(1).device(cuda).build()
    g.fit()
    assert g.lossHistory[-1] < g.lossHistory[0] * 0.1
    s_in = np.mean([g.similarity("alpha0", w) for w in A[1:]])
    s_out = np.mean([g.similarity("alpha0", w) for w in B])
    assert s_in > s_out + 0.3


def test_paragraph_vectors_and_deepwalk_on_gpu(cuda):
    from deeplearning4j_amd.nlp import LabelledDocument, ParagraphVectors, SimpleLabelAwareIterator
    from deeplearning4j_amd.graph import DeepWalk, Graph
    rng = np.random.RandomState(0)
    docs = [LabelledDocument(" ".join(rng.choice(A if k % 2 == 0 else B, 15)), ["TA" if k % 2 == 0 else "TB"])
            for k in range(400)]
    for algo in ("dbow", "dm"):
        pv = ParagraphVectors.Builder().minWordFrequency(1).layerSize(32).windowSize(4).seed(42).epochs(5) \
            .sequenceLearningAlgorithm(algo).trainWordVectors(True).iterate(SimpleLabelAwareIterator(docs)) \
            .device(cuda).build()
        pv.fit()
        assert pv.predict(" ".join(rng.choice(A, 15))) == "TA"
        assert pv.predict(" ".join(rng.choice(B, 15))) == "TB"
    g = Graph(20)
    for i in range(10):                      # two 10-cliques joined by one edge
        for j in range(i + 1, 10):
            g.addEdge(i, j)
            g.addEdge(10 + i, 10 + j)
    g.addEdge(0, 10)
    dw = DeepWalk.Builder().vectorSize(32).windowSize(2).learningRate(0.05).seed(1).device(cuda).build()
    dw.initialize(g)
    for _ in range(30):
        dw.fit(g, 12)
    assert dw.similarity(3, 4) > dw.similarity(3, 15)
