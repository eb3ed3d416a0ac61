"""Graphs and DeepWalk vertex embeddings.

Reference: deeplearning4j-graph — graph/Graph.java (adjacency lists, directed/undirected edges, multi-edges),
data/GraphLoader.java (edge-list files, weighted edge lists, vertex files), iterator/RandomWalkIterator.java +
WeightedRandomWalkIterator.java (NoEdgeHandling), models/deepwalk/GraphHuffman.java (Huffman tree over vertex
degrees, preorder inner-node numbering), models/deepwalk/DeepWalk.java (skip-gram over walks, window pairs
(walk[mid] -> walk[pos]) for mid in [w, len-w)), models/embeddings/InMemoryGraphLookupTable.java (vertex vectors
and inner-node vectors both uniform (r-0.5)/D; hierarchical softmax SGD), models/loader/GraphVectorSerializer.java.
MI355X path: walks come from the threaded C++ walker (csrc/runtime/graphwalk.cpp); pair updates run on the
gfx950 skip-gram kernel (csrc/embeddings.hip) when the vectors live on a GPU, or the threaded C++ applier.
"""
import ctypes
import heapq
import os

import numpy as np
import torch

from ..nlp.embeddings import EmbeddingEngine, F_HS, F_UPD_IN, F_UPD_OUT, InMemoryLookupTable, M_SG
from ..ops import runtime as RT

c_void_p, c_int, c_ll, c_ull = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong
RT.register("rt_random_walks", [c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_int, c_ull, c_int, c_void_p, c_int],
            c_ll)


class NoEdgesException(Exception):
    pass


class Vertex:
    def __init__(self, idx, value=None):
        self.idx, self.value = idx, value

    def vertexID(self):
        return self.idx

    def getValue(self):
        return self.value

    def __repr__(self):
        return f"Vertex({self.idx}, {self.value!r})"

    def __eq__(self, o):
        return isinstance(o, Vertex) and (self.idx, self.value) == (o.idx, o.value)

    def __hash__(self):
        return hash(self.idx)


class Edge:
    def __init__(self, frm, to, value=None, directed=False):
        self.frm, self.to, self.value, self.directed = frm, to, value, directed

    def getFrom(self):
        return self.frm

    def getTo(self):
        return self.to

    def getValue(self):
        return self.value

    def isDirected(self):
        return self.directed

    def __repr__(self):
        return f"Edge({self.frm}{'->' if self.directed else '--'}{self.to}, {self.value!r})"

    def __eq__(self, o):
        return isinstance(o, Edge) and (self.frm, self.to, self.value, self.directed) == \
            (o.frm, o.to, o.value, o.directed)

    def __hash__(self):
        return hash((self.frm, self.to))


class NoEdgeHandling:
    SELF_LOOP_ON_DISCONNECTED = "SELF_LOOP_ON_DISCONNECTED"
    EXCEPTION_ON_DISCONNECTED = "EXCEPTION_ON_DISCONNECTED"


class Graph:
    """Adjacency-list graph over vertices 0..n-1 (IGraph API)."""

    def __init__(self, vertices, allowMultipleEdges=False):
        if isinstance(vertices, int):
            vertices = [Vertex(i, None) for i in range(vertices)]
        self.vertices = list(vertices)
        self.allowMultiple = allowMultipleEdges
        self.edges = [[] for _ in self.vertices]
        self._csr = None

    def __eq__(self, o):
        return isinstance(o, Graph) and self.vertices == o.vertices and self.edges == o.edges

    __hash__ = None

    def numVertices(self):
        return len(self.vertices)

    def getVertex(self, idx):
        return self.vertices[idx]

    def getVertices(self, frm=0, to=None):
        return self.vertices[frm:(len(self.vertices) if to is None else to + 1)]

    def addEdge(self, frm, to=None, value=None, directed=False):
        e = frm if isinstance(frm, Edge) else Edge(frm, to, value, directed)
        if not self.allowMultiple and any(x.to == e.to for x in self.edges[e.frm]):
            return
        self.edges[e.frm].append(e)
        if not e.directed and e.frm != e.to:
            self.edges[e.to].append(Edge(e.to, e.frm, e.value, False))
        self._csr = None

    def getEdgesOut(self, v):
        return list(self.edges[v])

    def getVertexDegree(self, v):
        return len(self.edges[v])

    def getConnectedVertexIndices(self, v):
        return [e.to for e in self.edges[v]]

    def getConnectedVertices(self, v):
        return [self.vertices[e.to] for e in self.edges[v]]

    def getRandomConnectedVertex(self, v, rng):
        es = self.edges[v]
        if not es:
            raise NoEdgesException(f"vertex {v} has no edges")
        return self.vertices[es[rng.randint(len(es))].to]

    def csr(self, weighted=False):
        if self._csr is None:
            n = self.numVertices()
            offs = np.zeros(n + 1, dtype=np.int64)
            offs[1:] = np.cumsum([len(es) for es in self.edges])
            nbr = np.array([e.to for es in self.edges for e in es], dtype=np.int32)
            w = np.array([float(e.value) if e.value is not None else 1.0 for es in self.edges for e in es],
                         dtype=np.float32)
            self._csr = (offs, nbr if len(nbr) else np.zeros(1, np.int32), w if len(w) else np.ones(1, np.float32))
        offs, nbr, w = self._csr
        return offs, nbr, (w if weighted else None)


class GraphLoader:
    @staticmethod
    def _lines(path, ignore=("//",)):
        with open(path, encoding="utf-8") as fh:
            for ln in fh:
                ln = ln.strip()
                if not ln or any(ln.startswith(p) for p in ignore):
                    continue
                yield ln

    @staticmethod
    def loadUndirectedGraphEdgeListFile(path, numVertices, delim=",", allowMultipleEdges=False):
        g = Graph(numVertices, allowMultipleEdges)
        for ln in GraphLoader._lines(path):
            a, b = ln.split(delim)[:2]
            g.addEdge(int(a), int(b), None, False)
        return g

    @staticmethod
    def loadWeightedEdgeListFile(path, numVertices, delim=",", directed=False, allowMultipleEdges=False,
                                 ignoreLinesStartingWith=("//",)):
        if isinstance(allowMultipleEdges, (list, tuple, str)):   # reference overload (path, n, delim, directed, ignore)
            allowMultipleEdges, ignoreLinesStartingWith = False, allowMultipleEdges
        if isinstance(ignoreLinesStartingWith, str):
            ignoreLinesStartingWith = (ignoreLinesStartingWith,)
        g = Graph([StringVertexFactory().create(i) for i in range(numVertices)], allowMultipleEdges)
        for ln in GraphLoader._lines(path, ignoreLinesStartingWith):
            a, b, w = ln.split(delim)[:3]
            g.addEdge(int(a), int(b), float(w), directed)
        return g

    @staticmethod
    def loadGraph(vertexFile, edgeFile, delim=",", directed=False, allowMultipleEdges=False):
        if isinstance(edgeFile, EdgeLineProcessor):
            # reference overload loadGraph(path, EdgeLineProcessor, VertexFactory, numVertices, allowMultipleEdges)
            proc, factory, n = edgeFile, delim, directed
            g = Graph([factory.create(i) for i in range(int(n))], bool(allowMultipleEdges))
            with open(vertexFile, encoding="utf-8") as fh:
                for ln in fh:
                    e = proc.processLine(ln.rstrip("\n"))
                    if e is not None:
                        g.addEdge(e.getFrom(), e.getTo(), e.getValue(), e.isDirected())
            return g
        verts = []
        for ln in GraphLoader._lines(vertexFile):
            i, v = ln.split(delim, 1)
            verts.append(Vertex(int(i), v))
        verts.sort(key=lambda v: v.idx)
        g = Graph(verts)
        for ln in GraphLoader._lines(edgeFile):
            a, b = ln.split(delim)[:2]
            g.addEdge(int(a), int(b), None, directed)
        return g


class EdgeLineProcessor:
    """Turns one line of an edge-list file into an Edge, or None for comment / blank lines."""

    def processLine(self, line):
        raise NotImplementedError


class WeightedEdgeLineProcessor(EdgeLineProcessor):
    """"from<delim>to<delim>weight" lines (reference graph/data/impl/WeightedEdgeLineProcessor.java)."""

    def __init__(self, delim=",", directed=False, ignoreLinesStartingWith=("//",)):
        self.delim, self.directed = delim, bool(directed)
        self.ignore = (ignoreLinesStartingWith,) if isinstance(ignoreLinesStartingWith, str) else \
            tuple(ignoreLinesStartingWith or ())

    def processLine(self, line):
        ln = line.strip()
        if not ln or any(ln.startswith(p) for p in self.ignore):
            return None
        a, b, w = ln.split(self.delim)[:3]
        return Edge(int(a), int(b), float(w), self.directed)


class DelimitedEdgeLineProcessor(EdgeLineProcessor):
    """Unweighted "from<delim>to" lines (reference DelimitedEdgeLineProcessor.java)."""

    def __init__(self, delim=",", directed=False, ignoreLinesStartingWith=("//",)):
        self.delim, self.directed = delim, bool(directed)
        self.ignore = (ignoreLinesStartingWith,) if isinstance(ignoreLinesStartingWith, str) else \
            tuple(ignoreLinesStartingWith or ())

    def processLine(self, line):
        ln = line.strip()
        if not ln or any(ln.startswith(p) for p in self.ignore):
            return None
        a, b = ln.split(self.delim)[:2]
        return Edge(int(a), int(b), None, self.directed)


class StringVertexFactory:
    """Vertex i carries the string form of i (reference graph/vertexfactory/StringVertexFactory.java)."""

    def __init__(self, fmt=None):
        self.fmt = fmt

    def create(self, idx):
        return Vertex(idx, (self.fmt % idx) if self.fmt else str(idx))


class VertexSequence:
    def __init__(self, graph, idxs):
        self.graph, self.idxs, self._i = graph, list(idxs), 0

    def sequenceLength(self):
        return len(self.idxs)

    def hasNext(self):
        return self._i < len(self.idxs)

    def next(self):
        v = self.graph.getVertex(self.idxs[self._i])
        self._i += 1
        return v

    def indices(self):
        return list(self.idxs)


class RandomWalkIterator:
    """One walk of ``walkLength`` steps from every vertex, start order shuffled per reset."""

    WEIGHTED = False

    def __init__(self, graph, walkLength, rngSeed=12345, mode=NoEdgeHandling.SELF_LOOP_ON_DISCONNECTED,
                 firstVertex=0, lastVertex=None):
        self.g, self.L, self.seed, self.mode = graph, int(walkLength), int(rngSeed), mode
        self.first = firstVertex
        self.last = graph.numVertices() if lastVertex is None else lastVertex
        self._epoch = 0
        self.reset()

    def walkLength(self):
        return self.L

    def all_walks(self):
        """All walks of this pass as an int32 [nWalks, walkLength+1] array (native walker)."""
        rng = np.random.RandomState((self.seed + self._epoch) & 0x7FFFFFFF)
        starts = np.arange(self.first, self.last, dtype=np.int32)
        rng.shuffle(starts)
        offs, nbr, w = self.g.csr(self.WEIGHTED)
        out = np.empty((len(starts), self.L + 1), dtype=np.int32)
        rt = RT.load()
        no_edge = 1 if self.mode == NoEdgeHandling.EXCEPTION_ON_DISCONNECTED else 0
        r = rt.rt_random_walks(ctypes.c_void_p(offs.ctypes.data), ctypes.c_void_p(nbr.ctypes.data),
                               None if w is None else ctypes.c_void_p(w.ctypes.data),
                               ctypes.c_void_p(starts.ctypes.data), len(starts), self.L,
                               (self.seed * 1000003 + self._epoch) & 0xFFFFFFFFFFFFFFFF, no_edge,
                               ctypes.c_void_p(out.ctypes.data), min(8, os.cpu_count() or 1))
        if r < 0:
            raise NoEdgesException(f"vertex {starts[-r - 1]} (walk start) reached a vertex with no edges")
        return out

    def reset(self):
        self._walks = None
        self._i = 0
        self._epoch += 1

    def hasNext(self):
        if self._walks is None:
            self._walks = self.all_walks()
        return self._i < len(self._walks)

    def next(self):
        if self._walks is None:
            self._walks = self.all_walks()
        w = self._walks[self._i]
        self._i += 1
        return VertexSequence(self.g, w)


class WeightedRandomWalkIterator(RandomWalkIterator):
    """Next vertex drawn with probability proportional to the edge weight."""
    WEIGHTED = True


class GraphHuffman:
    """Huffman tree over vertex degrees; codes as bit lists, inner nodes numbered in preorder."""

    def __init__(self, nVertices, maxCodeLength=64):
        self.n = nVertices
        self.maxc = maxCodeLength
        self.codes = [[] for _ in range(nVertices)]
        self.paths = [[] for _ in range(nVertices)]

    def buildTree(self, degrees):
        heap = [(int(d), i, ("leaf", i)) for i, d in enumerate(degrees)]
        heapq.heapify(heap)
        k = len(heap)
        while len(heap) > 1:
            c1, _, a = heapq.heappop(heap)
            c2, _, b = heapq.heappop(heap)
            heapq.heappush(heap, (c1 + c2, k, ("inner", a, b)))
            k += 1
        root = heap[0][2]
        counter = [-1]
        stack = [(root, [], [])]
        while stack:
            node, code, path = stack.pop()
            if node[0] == "leaf":
                if len(code) > self.maxc:
                    raise RuntimeError(f"code length exceeds {self.maxc}")
                self.codes[node[1]] = code
                self.paths[node[1]] = path
                continue
            counter[0] += 1
            idx = counter[0]
            # preorder: left subtree first -> push right then left
            stack.append((node[2], code + [1], path + [idx]))
            stack.append((node[1], code + [0], path + [idx]))
        return self

    def getCodeLength(self, v):
        return len(self.codes[v])

    def getCode(self, v):
        return sum(b << i for i, b in enumerate(self.codes[v]))

    def getCodeString(self, v):
        return "".join(str(b) for b in self.codes[v])

    def getPathInnerNodes(self, v):
        return list(self.paths[v])


class _GraphTable(InMemoryLookupTable):
    def __init__(self, huffman, nVertices, vectorSize, learningRate, seed, device):
        super().__init__(None, vectorSize, seed, True, 0.0, device)
        self.tree = huffman
        self.n = nVertices
        self.learningRate = learningRate
        self.resetWeights()

    def resetWeights(self, reset=True):
        n, D = self.n, self.vectorLength
        g = torch.Generator().manual_seed(int(self.seed) & 0x7FFFFFFF)
        self.syn0 = ((torch.rand(n, D, generator=g) - 0.5) / D).to(self.device)
        self.syn1 = ((torch.rand(max(1, n - 1), D, generator=g) - 0.5) / D).to(self.device)
        self.syn1Neg = None
        maxc = max([len(c) for c in self.tree.codes] + [1])
        codes = np.zeros((n, maxc), np.uint8)
        points = np.zeros((n, maxc), np.int32)
        lens = np.zeros(n, np.int32)
        for v in range(n):
            L = len(self.tree.codes[v])
            lens[v] = L
            codes[v, :L] = [1 - b for b in self.tree.codes[v]]   # DeepWalk: bit 1 = sigmoid(+dot) -> w2v code 0
            points[v, :L] = self.tree.paths[v]
        self.codes_np, self.points_np, self.codelen_np, self.maxc = codes, points, lens, maxc
        self.codes = torch.from_numpy(codes).to(self.device)
        self.points = torch.from_numpy(points).to(self.device)
        self.codelen = torch.from_numpy(lens).to(self.device)
        self.table_np = np.zeros(1, np.int32)
        self.table = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._norm = None

    # GraphVectorLookupTable API
    def getVertexVectors(self):
        return self.syn0

    def setVertexVectors(self, v):
        self.syn0 = torch.as_tensor(v, dtype=torch.float32).to(self.device)
        self._norm = None

    def getOutWeights(self):
        return self.syn1

    def vectorSize(self):
        return self.vectorLength

    def getNumVertices(self):
        return self.n

    def getVector(self, i):
        return self.syn0[i]

    def calculateProb(self, first, second):
        vec = self.syn0[first].double()
        p = 1.0
        for b, node in zip(self.tree.codes[second], self.tree.paths[second]):
            d = float((self.syn1[node].double() * vec).sum())
            p *= 1.0 / (1.0 + np.exp(-d)) if b else 1.0 / (1.0 + np.exp(d))
        return p

    def calculateScore(self, first, second):
        return -np.log(self.calculateProb(first, second))


class GraphVectorsImpl:
    def __init__(self, graph=None, table=None):
        self.graph = graph
        self._table = table

    def lookupTable(self):
        return self._table

    def numVertices(self):
        return self._table.n

    def getVectorSize(self):
        return self._table.vectorLength

    def getVertexVector(self, v):
        idx = v.vertexID() if isinstance(v, Vertex) else int(v)
        return self._table.syn0[idx]

    def similarity(self, a, b):
        va, vb = self.getVertexVector(a), self.getVertexVector(b)
        return float(torch.nn.functional.cosine_similarity(va.reshape(1, -1), vb.reshape(1, -1)))

    def verticesNearest(self, v, top):
        idx = v.vertexID() if isinstance(v, Vertex) else int(v)
        n = self._table.normalized()
        sims = n @ n[idx]
        sims[idx] = -float("inf")
        return torch.topk(sims, min(top, sims.shape[0] - 1)).indices.cpu().tolist()


class DeepWalk(GraphVectorsImpl):
    class Builder:
        def __init__(self):
            self._vs, self._seed, self._lr, self._ws, self._dev = 100, 12345, 0.01, 2, None

        def vectorSize(self, v): self._vs = int(v); return self  # noqa: E704
        def learningRate(self, v): self._lr = float(v); return self  # noqa: E704
        def windowSize(self, v): self._ws = int(v); return self  # noqa: E704
        def seed(self, v): self._seed = int(v); return self  # noqa: E704
        def device(self, d): self._dev = d; return self  # noqa: E704

        def build(self):
            d = DeepWalk()
            d.vectorSize, d.seed, d.learningRate, d.windowSize, d.device = self._vs, self._seed, self._lr, \
                self._ws, self._dev
            return d

    def __init__(self):
        super().__init__()
        self.vectorSize, self.seed, self.learningRate, self.windowSize = 100, 12345, 0.01, 2
        self.device = None
        self.initCalled = False
        self.walkCounter = 0

    def _dev(self):
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

    def initialize(self, graph_or_degrees):
        if isinstance(graph_or_degrees, Graph):
            self.graph = graph_or_degrees
            degrees = [graph_or_degrees.getVertexDegree(i) for i in range(graph_or_degrees.numVertices())]
        else:
            degrees = list(graph_or_degrees)
        gh = GraphHuffman(len(degrees)).buildTree(degrees)
        self._table = _GraphTable(gh, len(degrees), self.vectorSize, self.learningRate, self.seed, self._dev())
        self.initCalled = True
        return self

    def setLearningRate(self, lr):
        self.learningRate = lr
        if self._table is not None:
            self._table.learningRate = lr

    def _pairs(self, walks):
        w = self.windowSize
        W = np.asarray(walks, dtype=np.int32)
        L = W.shape[1]
        if L <= 2 * w:
            return np.zeros(0, np.int32), np.zeros(0, np.int32)
        mids = np.arange(w, L - w)
        offs = np.array([o for o in range(-w, w + 1) if o != 0])
        ins = np.repeat(W[:, mids], len(offs), axis=1)
        tgt = W[:, (mids[:, None] + offs[None, :]).reshape(-1)]
        return ins.reshape(-1).astype(np.int32), tgt.reshape(-1).astype(np.int32)

    def fit(self, graph_or_iter, walkLength=None):
        if isinstance(graph_or_iter, Graph):
            if not self.initCalled:
                self.initialize(graph_or_iter)
            it = RandomWalkIterator(graph_or_iter, walkLength, self.seed + self.walkCounter)
        else:
            it = graph_or_iter
            if not self.initCalled:
                raise RuntimeError("DeepWalk not initialized (call initialize before fit)")
        walks = it.all_walks() if hasattr(it, "all_walks") else np.array(
            [s.indices() for s in _drain(it)], dtype=np.int32)
        ins, tgt = self._pairs(walks)
        alpha = np.full(len(ins), self.learningRate, dtype=np.float32)
        eng = EmbeddingEngine(self._table)
        eng._apply(M_SG, (ins, tgt, alpha, None, None, 0), F_HS | F_UPD_IN | F_UPD_OUT)
        self._table.invalidate()
        self.walkCounter += len(walks)
        return self


def _drain(it):
    while it.hasNext():
        yield it.next()


class GraphVectorSerializer:
    """Text format: ``<vertexIdx>\\t<v1>\\t<v2>...`` per line (GraphVectorSerializer.java)."""

    @staticmethod
    def writeGraphVectors(deepwalk, path):
        V = deepwalk.lookupTable().syn0.detach().cpu().double().numpy()
        with open(path, "w", encoding="utf-8") as fh:
            for i, row in enumerate(V):
                fh.write(str(i) + "\t" + "\t".join(repr(float(x)) for x in row) + "\n")

    @staticmethod
    def loadTxtVectors(path):
        rows = []
        with open(path, encoding="utf-8") as fh:
            for ln in fh:
                p = ln.rstrip("\n").split("\t")
                rows.append((int(p[0]), np.array(p[1:], dtype=np.float32)))
        rows.sort(key=lambda r: r[0])
        n, D = len(rows), len(rows[0][1])
        gh = GraphHuffman(n).buildTree([1] * n)
        t = _GraphTable(gh, n, D, 0.01, 1, "cpu")
        t.syn0 = torch.from_numpy(np.stack([r[1] for r in rows]))
        return GraphVectorsImpl(None, t)
