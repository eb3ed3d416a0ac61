"""SequenceVectors graph walkers and the graph -> sequence transformer (reference deeplearning4j-nlp
models/sequencevectors/graph/walkers/impl/{RandomWalker,WeightedWalker,PopularityWalker,NearestVertexWalker}.java,
graph/enums/*.java, transformers/impl/GraphTransformer.java).

Each walker produces one ``Sequence`` per start vertex per pass (start order optionally shuffled by ``reset``); the
GraphTransformer iterates a walker and numbers the sequences; ``SequenceVectors.Builder().iterate(transformer)``
(nlp/word2vec.py) trains vertex embeddings on them — the reference's Node2Vec / DeepWalk-on-SequenceVectors route.

Differences from the reference, on purpose:
* ``FORWARD_PREFERRED`` moves to an unvisited neighbour when one exists (the reference leaves ``startPosition``
  unchanged in that branch, i.e. stays put);
* ``NearestVertexWalker``'s sampling modes are separate (the reference's switch falls through from MAX_POPULARITY
  into the later cases) and MIN_POPULARITY starts from the last vertex, not one past it;
* the walkers draw from one seeded ``numpy.random.RandomState`` (the reference mixes java.util.Random and
  RandomUtils), so sequences are reproducible per seed but not equal to the reference's.
The walkers run on the host: they are sequential pointer chasing; DeepWalk's bulk walks use the threaded native walker
(graph/__init__.py ``RandomWalkIterator``).
"""
import enum

import numpy as np

from . import NoEdgesException


class WalkDirection(enum.Enum):
    RANDOM = "RANDOM"
    FORWARD_ONLY = "FORWARD_ONLY"
    FORWARD_UNIQUE = "FORWARD_UNIQUE"
    FORWARD_PREFERRED = "FORWARD_PREFERRED"


class NoEdgeHandling(enum.Enum):
    SELF_LOOP_ON_DISCONNECTED = "SELF_LOOP_ON_DISCONNECTED"
    EXCEPTION_ON_DISCONNECTED = "EXCEPTION_ON_DISCONNECTED"
    PADDING_ON_DISCONNECTED = "PADDING_ON_DISCONNECTED"
    CUTOFF_ON_DISCONNECTED = "CUTOFF_ON_DISCONNECTED"
    RESTART_ON_DISCONNECTED = "RESTART_ON_DISCONNECTED"


class PopularityMode(enum.Enum):
    MAXIMUM = "MAXIMUM"
    AVERAGE = "AVERAGE"
    MINIMUM = "MINIMUM"


class SpreadSpectrum(enum.Enum):
    PLAIN = "PLAIN"
    PROPORTIONAL = "PROPORTIONAL"


class SamplingMode(enum.Enum):
    RANDOM = "RANDOM"
    MAX_POPULARITY = "MAX_POPULARITY"
    MEDIAN_POPULARITY = "MEDIAN_POPULARITY"
    MIN_POPULARITY = "MIN_POPULARITY"


def _label(v):
    val = v.getValue()
    return str(v.vertexID()) if val is None else str(getattr(val, "label", val))


class Sequence:
    """Walk output: element labels in visit order, optional sequence label(s) and id (SequenceVectors' Sequence)."""

    def __init__(self, elements=None, label=None):
        self.elements = list(elements or [])
        self.labels = [] if label is None else [label]
        self.sequenceId = -1

    def addElement(self, e):
        self.elements.append(e)

    def addElements(self, es):
        self.elements.extend(es)

    def getElements(self):
        return list(self.elements)

    def size(self):
        return len(self.elements)

    def getElementByLabel(self, label):
        return label if label in self.elements else None

    def setSequenceLabel(self, label):
        self.labels = [label]

    def getSequenceLabel(self):
        return self.labels[0] if self.labels else None

    def getSequenceLabels(self):
        return list(self.labels) if self.labels else None

    def setSequenceId(self, i):
        self.sequenceId = int(i)

    def getSequenceId(self):
        return self.sequenceId

    def __len__(self):
        return len(self.elements)

    def __repr__(self):
        return f"Sequence({self.elements}, labels={self.labels})"


class RandomWalker:
    """Uniform random walks of ``walkLength`` vertices from every vertex (RandomWalker.java:70-220) with the four
    walk directions, the no-edge policies and an optional restart probability ``alpha`` (jump back to the start)."""

    def __init__(self, graph, walkLength=5, noEdgeHandling=NoEdgeHandling.RESTART_ON_DISCONNECTED,
                 walkDirection=WalkDirection.FORWARD_ONLY, alpha=0.0, seed=0):
        self.sourceGraph = graph
        self.walkLength = int(walkLength)
        self.noEdgeHandling = noEdgeHandling
        self.walkDirection = walkDirection
        self.alpha = float(alpha)
        self.seed = int(seed)
        self.rng = np.random.RandomState(self.seed & 0x7FFFFFFF)
        self.order = np.arange(graph.numVertices())
        if self.seed != 0:
            self.rng.shuffle(self.order)
        self.position = 0

    def getSourceGraph(self):
        return self.sourceGraph

    def hasNext(self):
        return self.position < self.sourceGraph.numVertices()

    def isLabelEnabled(self):
        return False

    def reset(self, shuffle=False):
        self.position = 0
        if shuffle:
            self.rng.shuffle(self.order)

    def _no_edge(self, cur, start):
        """Next vertex when the walk is stuck at ``cur``: (vertex, stop)."""
        h = self.noEdgeHandling
        if h == NoEdgeHandling.CUTOFF_ON_DISCONNECTED:
            return cur, True
        if h == NoEdgeHandling.EXCEPTION_ON_DISCONNECTED:
            raise NoEdgesException(f"No more edges at vertex [{cur}]")
        if h == NoEdgeHandling.SELF_LOOP_ON_DISCONNECTED:
            return cur, False
        if h == NoEdgeHandling.RESTART_ON_DISCONNECTED:
            return start, False
        raise NotImplementedError(f"NoEdgeHandling mode [{h.value}] not implemented")

    def _pick(self, hops):
        return int(hops[self.rng.randint(len(hops))])

    def next(self):
        g = self.sourceGraph
        start = int(self.order[self.position])
        self.position += 1
        seq = Sequence()
        visited = []
        cur, last = start, -1
        for _ in range(self.walkLength):
            v = g.getVertex(cur)
            seq.addElement(_label(v))
            visited.append(cur)
            if self.alpha > 0 and last != start and last != -1 and self.alpha > self.rng.random_sample():
                cur, last = start, cur
                continue
            nbrs = g.getConnectedVertexIndices(cur)
            d = self.walkDirection
            if d == WalkDirection.RANDOM:
                if not nbrs:
                    nxt, stop = self._no_edge(cur, start)
                else:
                    nxt, stop = self._pick(nbrs), False
            elif d == WalkDirection.FORWARD_ONLY:
                hops = [n for n in nbrs if n != last]
                nxt, stop = (self._pick(hops), False) if hops else self._no_edge(cur, start)
            elif d == WalkDirection.FORWARD_UNIQUE:
                hops = [n for n in nbrs if n not in visited]
                nxt, stop = (self._pick(hops), False) if hops else self._no_edge(cur, start)
            elif d == WalkDirection.FORWARD_PREFERRED:
                hops = [n for n in nbrs if n not in visited] or [n for n in nbrs if n != last]
                nxt, stop = (self._pick(hops), False) if hops else self._no_edge(cur, start)
            else:
                raise NotImplementedError(f"Unknown WalkDirection [{d}]")
            if stop:
                break
            last, cur = cur, nxt
        return seq

    class Builder:
        def __init__(self, graph):
            self.kw = {"graph": graph}

        def setWalkLength(self, n):
            self.kw["walkLength"] = n
            return self

        def setNoEdgeHandling(self, h):
            self.kw["noEdgeHandling"] = h
            return self

        def setSeed(self, s):
            self.kw["seed"] = s
            return self

        def setWalkDirection(self, d):
            self.kw["walkDirection"] = d
            return self

        def setRestartProbability(self, a):
            self.kw["alpha"] = a
            return self

        def _cls(self):
            return RandomWalker

        def build(self):
            return self._cls()(**self.kw)


class WeightedWalker(RandomWalker):
    """Next vertex drawn with probability proportional to the outgoing edge weights (WeightedWalker.java:46-119)."""

    def next(self):
        g = self.sourceGraph
        start = int(self.order[self.position])
        self.position += 1
        seq = Sequence()
        cur, last = start, -1
        for _ in range(self.walkLength):
            if self.alpha > 0 and last != start and last != -1 and self.alpha > self.rng.random_sample():
                cur, last = start, -1
                continue
            seq.addElement(_label(g.getVertex(cur)))
            edges = g.getEdgesOut(cur)
            if not edges:
                nxt, stop = self._no_edge(cur, start)
                if stop:
                    break
                cur = nxt
                continue
            w = np.array([float(e.getValue()) if e.getValue() is not None else 1.0 for e in edges])
            thr = self.rng.random_sample() * w.sum()
            k = int(min(np.searchsorted(np.cumsum(w), thr, side="left"), len(edges) - 1))
            e = edges[k]
            cur = e.getTo() if (e.isDirected() or e.getFrom() == cur) else e.getFrom()
            last = cur
        return seq

    class Builder(RandomWalker.Builder):
        def _cls(self):
            return WeightedWalker


class PopularityWalker(RandomWalker):
    """Walks that prefer neighbours by popularity (degree): the unvisited neighbours sorted by degree (descending),
    a window of ``spread`` of them at the top (MAXIMUM), middle (AVERAGE) or bottom (MINIMUM), then a uniform pick in
    that window (PLAIN) or one proportional to degree (PROPORTIONAL) (PopularityWalker.java:60-190)."""

    def __init__(self, graph, popularityMode=PopularityMode.MAXIMUM, spread=10, spectrum=SpreadSpectrum.PLAIN, **kw):
        super().__init__(graph, **kw)
        self.popularityMode, self.spread, self.spectrum = popularityMode, int(spread), spectrum

    def next(self):
        g = self.sourceGraph
        start = int(self.order[self.position])
        self.position += 1
        seq = Sequence()
        visited = []
        cur, last = start, -1
        for _ in range(self.walkLength):
            seq.addElement(_label(g.getVertex(cur)))
            visited.append(cur)
            if self.alpha > 0 and last != start and last != -1 and self.alpha > self.rng.random_sample():
                cur = start
                continue
            conns = [n for n in g.getConnectedVertexIndices(cur) if n not in visited]
            if not conns:
                nxt, stop = self._no_edge(cur, start)
                if stop:
                    break
                cur = nxt
                continue
            # stable sort by degree, most popular first (the reference's priority queue order)
            conns.sort(key=lambda n: -g.getVertexDegree(n))
            cs = min(self.spread, len(conns))
            if self.popularityMode == PopularityMode.MAXIMUM:
                lo, hi = 0, cs - 1
            elif self.popularityMode == PopularityMode.MINIMUM:
                lo, hi = len(conns) - cs, len(conns) - 1
            else:
                mid = len(conns) // 2
                lo, hi = max(0, mid - cs // 2), min(len(conns) - 1, mid + cs // 2)
            window = conns[lo:hi + 1]
            if self.spectrum == SpreadSpectrum.PLAIN:
                nxt = window[self.rng.randint(len(window))]
            else:
                w = np.array([g.getVertexDegree(n) for n in window], dtype=np.float64)
                p = w / w.sum() if w.sum() > 0 else np.full(len(w), 1.0 / len(w))
                nxt = window[int(min(np.searchsorted(np.cumsum(p), self.rng.random_sample(), side="right"),
                                     len(window) - 1))]
            last, cur = cur, int(nxt)
        return seq

    class Builder(RandomWalker.Builder):
        def setPopularityMode(self, m):
            self.kw["popularityMode"] = m
            return self

        def setPopularitySpread(self, n):
            self.kw["spread"] = n
            return self

        def setSpreadSpectrum(self, s):
            self.kw["spectrum"] = s
            return self

        def _cls(self):
            return PopularityWalker


class NearestVertexWalker:
    """One labelled sequence per vertex: its neighbours (all, or ``walkLength`` of them sampled RANDOM / by
    MAX / MEDIAN / MIN popularity), recursively expanded to ``depth`` hops without duplicates; the sequence label is
    the vertex itself (NearestVertexWalker.java:63-170) — ParagraphVectors-style training over graph
    neighbourhoods."""

    def __init__(self, graph, walkLength=0, seed=0, samplingMode=SamplingMode.RANDOM, depth=1):
        self.sourceGraph = graph
        self.walkLength, self.seed, self.samplingMode, self.depth = int(walkLength), int(seed), samplingMode, \
            int(depth)
        self.rng = np.random.RandomState(self.seed & 0x7FFFFFFF)
        self.order = np.arange(graph.numVertices())
        if self.seed != 0:
            self.rng.shuffle(self.order)
        self.position = 0

    def getSourceGraph(self):
        return self.sourceGraph

    def hasNext(self):
        return self.position < len(self.order)

    def isLabelEnabled(self):
        return True

    def reset(self, shuffle=False):
        self.position = 0
        if shuffle:
            self.rng.shuffle(self.order)

    def next(self):
        v = int(self.order[self.position])
        self.position += 1
        return self._walk(v, 1)

    def _by_popularity(self, nbrs):
        g = self.sourceGraph
        return sorted(nbrs, key=lambda n: -g.getVertexDegree(n))

    def _walk(self, v, cdepth):
        g = self.sourceGraph
        seq = Sequence(label=_label(g.getVertex(v)))
        nbrs = g.getConnectedVertexIndices(v)
        if self.walkLength == 0:
            seq.addElements(_label(g.getVertex(n)) for n in nbrs)
            return seq
        m, L = self.samplingMode, self.walkLength
        if m == SamplingMode.RANDOM:
            picked = list(nbrs) if len(nbrs) <= L else [nbrs[i] for i in self.rng.choice(len(nbrs), L, replace=False)]
        else:
            srt = self._by_popularity(nbrs)
            if m == SamplingMode.MAX_POPULARITY:
                picked = srt[:L]
            elif m == SamplingMode.MEDIAN_POPULARITY:
                s0 = max(0, len(srt) // 2 - L // 2)
                picked = srt[s0:s0 + L]
            else:
                picked = srt[::-1][:L]
        for n in picked:
            lab = _label(g.getVertex(n))
            if seq.getElementByLabel(lab) is None:
                seq.addElement(lab)
            if self.depth > 1 and cdepth < self.depth:
                for e in self._walk(n, cdepth + 1).getElements():
                    if seq.getElementByLabel(e) is None:
                        seq.addElement(e)
        return seq

    class Builder:
        def __init__(self, graph):
            self.kw = {"graph": graph}

        def setSeed(self, s):
            self.kw["seed"] = s
            return self

        def setWalkLength(self, n):
            self.kw["walkLength"] = n
            return self

        def setDepth(self, d):
            self.kw["depth"] = d
            return self

        def setSamplingMode(self, m):
            self.kw["samplingMode"] = m
            return self

        def build(self):
            return NearestVertexWalker(**self.kw)


class GraphTransformer:
    """Iterable of walker sequences (GraphTransformer.java): each ``iter()`` resets the walker (shuffling its start
    order when ``shuffle``), numbers the sequences, and labels them through ``labelsProvider`` when the walker is
    label-enabled and produced none."""

    def __init__(self, walker, shuffle=True, labelsProvider=None):
        self.walker, self.shuffle, self.labelsProvider = walker, bool(shuffle), labelsProvider
        self.sourceGraph = walker.getSourceGraph()

    def __iter__(self):
        self.walker.reset(self.shuffle)
        n = 0
        while self.walker.hasNext():
            s = self.walker.next()
            s.setSequenceId(n)
            if self.walker.isLabelEnabled() and s.getSequenceLabels() is None and self.labelsProvider is not None:
                s.setSequenceLabel(self.labelsProvider(n))
            n += 1
            yield s

    def vertexFrequencies(self):
        """Element frequencies as the reference's initialize() assigns them: the vertex degree."""
        g = self.sourceGraph
        return {_label(g.getVertex(i)): g.getVertexDegree(i) for i in range(g.numVertices())}

    class Builder:
        def __init__(self, walker=None):
            self._walker, self._shuffle, self._labels = walker, True, None

        def setGraphWalker(self, w):
            self._walker = w
            return self

        def shuffleOnReset(self, v):
            self._shuffle = bool(v)
            return self

        def setLabelsProvider(self, p):
            self._labels = p
            return self

        def build(self):
            if self._walker is None:
                raise ValueError("GraphTransformer needs a GraphWalker")
            return GraphTransformer(self._walker, self._shuffle, self._labels)
