"""Text processing: tokenizers, token pre-processors, sentence / document iterators, stop words.

Reference: NLP:text/tokenization/** (DefaultTokenizer, NGramTokenizer, CommonPreprocessor/StringCleaning,
EndingPreProcessor, LowCasePreProcessor), NLP:text/sentenceiterator/** (BasicLineIterator, CollectionSentenceIterator,
FileSentenceIterator, LineSentenceIterator, AggregatingSentenceIterator, MutipleEpochsSentenceIterator),
NLP:text/documentiterator/** (LabelledDocument, LabelAwareIterator, BasicLabelAwareIterator, SimpleLabelAwareIterator,
FileLabelAwareIterator, FilenamesLabelAwareIterator, LabelsSource), NLP:text/stopwords/StopWords.java.
Tokenization is host work; it feeds the native batcher (csrc/runtime/embeddings.cpp).
"""
import os
import re
import threading
import queue

_PUNCT = re.compile(r"[\d\.:,\"'\(\)\[\]|/?!;]+")


# ------------------------------------------------------------------------------------------ pre-processors
class TokenPreProcess:
    def preProcess(self, token):
        return token


class CommonPreprocessor(TokenPreProcess):
    """Strip digits and ASCII punctuation ``0-9.:,"'()[]|/?!;`` then lower-case (CommonPreprocessor.java)."""

    def preProcess(self, token):
        return _PUNCT.sub("", token).lower()


class LowCasePreProcessor(TokenPreProcess):
    def preProcess(self, token):
        return token.lower()


class EndingPreProcessor(TokenPreProcess):
    """Crude suffix stripping: s (not ss), trailing '.', ed, ing, ly (EndingPreProcessor.java)."""

    def preProcess(self, token):
        if token.endswith("s") and not token.endswith("ss"):
            token = token[:-1]
        for suf in (".", "ed", "ing", "ly"):
            if token.endswith(suf):
                token = token[:-len(suf)]
        return token


class StringCleaning:
    @staticmethod
    def stripPunct(s):
        return _PUNCT.sub("", s)


class SentencePreProcessor:
    def preProcess(self, sentence):
        return sentence


# ------------------------------------------------------------------------------------------ tokenizers
class Tokenizer:
    def __init__(self, tokens, pre=None):
        self._raw = tokens
        self._pre = pre
        self._i = 0

    def setTokenPreProcessor(self, pre):
        self._pre = pre

    def _proc(self, t):
        return self._pre.preProcess(t) if self._pre is not None else t

    def hasMoreTokens(self):
        return self._i < len(self._raw)

    def countTokens(self):
        return len(self._raw)

    def nextToken(self):
        t = self._raw[self._i]
        self._i += 1
        return self._proc(t)

    def getTokens(self):
        out = []
        for t in self._raw:
            p = self._proc(t)
            if p is not None and p != "":
                out.append(p)
        return out


class DefaultTokenizer(Tokenizer):
    """Whitespace tokenization (java.util.StringTokenizer semantics: space, tab, newline, CR, form feed)."""

    def __init__(self, text, pre=None):
        super().__init__(re.split(r"[ \t\n\r\f]+", text.strip()) if text.strip() else [], pre)


class NGramTokenizer(Tokenizer):
    """All n-grams (minN..maxN, joined by a space) over the pre-processed base tokens (NGramTokenizer.java)."""

    def __init__(self, base, minN, maxN):
        toks = base.getTokens()
        out = []
        for n in range(minN, maxN + 1):
            for i in range(len(toks) - n + 1):
                out.append(" ".join(toks[i:i + n]))
        super().__init__(out, None)


class TokenizerFactory:
    def __init__(self):
        self.pre = None

    def create(self, text):
        raise NotImplementedError

    def setTokenPreProcessor(self, pre):
        self.pre = pre

    def getTokenPreProcessor(self):
        return self.pre


class DefaultTokenizerFactory(TokenizerFactory):
    def create(self, text):
        if hasattr(text, "read"):
            text = text.read()
            if isinstance(text, bytes):
                text = text.decode("utf-8")
        return DefaultTokenizer(text, self.pre)


class NGramTokenizerFactory(TokenizerFactory):
    def __init__(self, base=None, minN=1, maxN=1):
        super().__init__()
        self.base = base or DefaultTokenizerFactory()
        self.minN, self.maxN = minN, maxN

    def setTokenPreProcessor(self, pre):
        self.pre = pre
        self.base.setTokenPreProcessor(pre)

    def create(self, text):
        return NGramTokenizer(self.base.create(text), self.minN, self.maxN)


# ------------------------------------------------------------------------------------------ stop words
STOP_WORDS = frozenset("""a about above after again against all am an and any are as at be because been before being
below between both but by can could did do does doing down during each few for from further had has have having he
her here hers herself him himself his how i if in into is it its itself just me more most my myself no nor not now of
off on once only or other our ours ourselves out over own same she should so some such than that the their theirs
them themselves then there these they this those through to too under until up very was we were what when where
which while who whom why will with would you your yours yourself yourselves""".split())


class StopWords:
    @staticmethod
    def getStopWords():
        return sorted(STOP_WORDS)


# ------------------------------------------------------------------------------------------ sentence iterators
class SentenceIterator:
    def __init__(self):
        self.preProcessor = None

    def setPreProcessor(self, p):
        self.preProcessor = p

    def getPreProcessor(self):
        return self.preProcessor

    def _pp(self, s):
        return self.preProcessor.preProcess(s) if self.preProcessor is not None else s

    def hasNext(self):
        raise NotImplementedError

    def nextSentence(self):
        raise NotImplementedError

    def reset(self):
        pass

    def finish(self):
        pass

    def __iter__(self):
        self.reset()
        while self.hasNext():
            yield self.nextSentence()


class CollectionSentenceIterator(SentenceIterator):
    def __init__(self, sentences, preProcessor=None):
        super().__init__()
        self.sentences = list(sentences)
        self.preProcessor = preProcessor
        self._i = 0

    def hasNext(self):
        return self._i < len(self.sentences)

    def nextSentence(self):
        s = self.sentences[self._i]
        self._i += 1
        return self._pp(s)

    def reset(self):
        self._i = 0


class BasicLineIterator(SentenceIterator):
    """One sentence per non-empty line of a file path or an open binary / text stream (streamed; a stream is
    rewound on reset)."""

    def __init__(self, path):
        super().__init__()
        self.path = path
        self._fh = None
        self._next = None

    def _open(self):
        if hasattr(self.path, "read"):
            import io
            self.path.seek(0)
            return self.path if isinstance(self.path, io.TextIOBase) else io.TextIOWrapper(self.path, "utf-8")
        return open(self.path, encoding="utf-8")

    def _advance(self):
        while True:
            line = self._fh.readline()
            if not line:
                self._next = None
                return
            line = line.rstrip("\r\n")
            if line.strip():
                self._next = line
                return

    def reset(self):
        if self._fh is not None and not hasattr(self.path, "read"):
            self._fh.close()
        if self._fh is not None and hasattr(self.path, "read") and self._fh is not self.path:
            self._fh.detach()                          # keep the caller's stream open
        self._fh = self._open()
        self._advance()

    def hasNext(self):
        if self._fh is None:
            self.reset()
        return self._next is not None

    def nextSentence(self):
        if self._fh is None:
            self.reset()
        s = self._next
        self._advance()
        return self._pp(s)

    def finish(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None


LineSentenceIterator = BasicLineIterator


class FileSentenceIterator(SentenceIterator):
    """Every line of every file under a directory (or a single file)."""

    def __init__(self, path, preProcessor=None):
        super().__init__()
        self.preProcessor = preProcessor
        if os.path.isdir(path):
            self.files = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(path) for f in fs)
        else:
            self.files = [path]
        self.reset()

    def reset(self):
        self._lines = []
        for f in self.files:
            with open(f, encoding="utf-8", errors="replace") as fh:
                self._lines.extend(l.rstrip("\r\n") for l in fh if l.strip())
        self._i = 0

    def hasNext(self):
        return self._i < len(self._lines)

    def nextSentence(self):
        s = self._lines[self._i]
        self._i += 1
        return self._pp(s)


class StreamLineIterator(BasicLineIterator):
    """Lines of an input stream read ahead in blocks of ``fetchSize`` (reference text/sentenceiterator/
    StreamLineIterator.java); blank lines are skipped."""

    def __init__(self, stream, fetchSize=10000):
        super().__init__(stream)
        self.fetchSize = int(fetchSize)

    class Builder:
        def __init__(self, stream):
            self._s, self._n, self._pp_ = stream, 10000, None

        def setFetchSize(self, n):
            self._n = int(n)
            return self

        def setPreProcessor(self, p):
            self._pp_ = p
            return self

        def build(self):
            it = StreamLineIterator(self._s, self._n)
            it.preProcessor = self._pp_
            return it


class AggregatingSentenceIterator(SentenceIterator):
    def __init__(self, iterators, preProcessor=None):
        super().__init__()
        self.its = list(iterators)
        self.preProcessor = preProcessor
        self._k = 0

    def reset(self):
        for it in self.its:
            it.reset()
        self._k = 0

    def hasNext(self):
        while self._k < len(self.its):
            if self.its[self._k].hasNext():
                return True
            self._k += 1
        return False

    def nextSentence(self):
        self.hasNext()
        return self._pp(self.its[self._k].nextSentence())

    class Builder:
        """Reference AggregatingSentenceIterator.Builder: addSentenceIterator(...) / addSentenceIterators(list) /
        addSentencePreProcessor(p).build()."""

        def __init__(self):
            self._its, self._pp_ = [], None

        def addSentenceIterator(self, it):
            self._its.append(it)
            return self

        def addSentenceIterators(self, its):
            self._its.extend(its)
            return self

        def addSentencePreProcessor(self, p):
            self._pp_ = p
            return self

        def build(self):
            return AggregatingSentenceIterator(self._its, self._pp_)


class MutipleEpochsSentenceIterator(SentenceIterator):
    def __init__(self, base, epochs):
        super().__init__()
        self.base, self.epochs, self._e = base, epochs, 0

    def reset(self):
        self.base.reset()
        self._e = 0

    def hasNext(self):
        if self.base.hasNext():
            return True
        if self._e + 1 < self.epochs:
            self._e += 1
            self.base.reset()
            return self.base.hasNext()
        return False

    def nextSentence(self):
        return self.base.nextSentence()


class PrefetchingSentenceIterator(SentenceIterator):
    """Background-thread prefetch of another iterator's sentences (PrefetchingSentenceIterator.java)."""

    def __init__(self, base, fetchSize=10000):
        super().__init__()
        self.base, self.size = base, fetchSize
        self._q = None
        self._next = None

    def _run(self, q):
        self.base.reset()
        while self.base.hasNext():
            q.put(self.base.nextSentence())
        q.put(StopIteration)

    def reset(self):
        self._q = queue.Queue(self.size)
        threading.Thread(target=self._run, args=(self._q,), daemon=True).start()
        self._next = self._q.get()

    def hasNext(self):
        if self._q is None:
            self.reset()
        return self._next is not StopIteration

    def nextSentence(self):
        s = self._next
        self._next = self._q.get()
        return self._pp(s)


# ------------------------------------------------------------------------------------------ documents / labels
class LabelledDocument:
    def __init__(self, content=None, labels=None, referencedContent=None):
        self.content = content
        self.labels = list(labels or [])
        self.referencedContent = referencedContent

    def getContent(self):
        return self.content

    def setContent(self, c):
        self.content = c

    def getLabels(self):
        return self.labels

    def getLabel(self):
        return self.labels[0] if self.labels else None

    def addLabel(self, l):
        self.labels.append(l)

    def setLabels(self, ls):
        self.labels = list(ls)


class LabelsSource:
    """Label generator/collector: either a fixed list or a template like ``"DOC_%d"`` (LabelsSource.java)."""

    def __init__(self, template_or_labels="DOC_%d"):
        if isinstance(template_or_labels, (list, tuple)):
            self.template, self.labels = None, list(template_or_labels)
        else:
            self.template, self.labels = template_or_labels, []
        self.counter = 0
        self._seen = set(self.labels)

    def nextLabel(self):
        if self.template is not None:
            # "%d" templates are formatted; any other string gets the counter appended (reference LabelsSource)
            lab = self.template % self.counter if "%d" in self.template else f"{self.template}{self.counter}"
            self.counter += 1
            self.storeLabel(lab)
            return lab
        lab = self.labels[self.counter]
        self.counter += 1
        return lab

    def storeLabel(self, lab):
        if lab not in self._seen:
            self._seen.add(lab)
            self.labels.append(lab)

    def getLabels(self):
        return list(self.labels)

    def indexOf(self, lab):
        return self.labels.index(lab)

    def reset(self):
        self.counter = 0

    def getNumberOfLabelsUsed(self):
        return len(self.labels)


class LabelAwareIterator:
    def hasNextDocument(self):
        raise NotImplementedError

    def nextDocument(self):
        raise NotImplementedError

    def reset(self):
        pass

    def getLabelsSource(self):
        return self.labelsSource

    def shutdown(self):
        pass

    def __iter__(self):
        self.reset()
        while self.hasNextDocument():
            yield self.nextDocument()


class SimpleLabelAwareIterator(LabelAwareIterator):
    def __init__(self, documents):
        self.docs = list(documents)
        self.labelsSource = LabelsSource([])
        for d in self.docs:
            for l in d.labels:
                self.labelsSource.storeLabel(l)
        self._i = 0

    def hasNextDocument(self):
        return self._i < len(self.docs)

    def nextDocument(self):
        d = self.docs[self._i]
        self._i += 1
        return d

    def reset(self):
        self._i = 0


class BasicLabelAwareIterator(LabelAwareIterator):
    """Wraps a SentenceIterator (each sentence a document, labelled from a LabelsSource template) or another
    LabelAwareIterator (BasicLabelAwareIterator.java)."""

    class Builder:
        def __init__(self, source):
            self.source = source
            self.labels = LabelsSource("DOC_%d")

        def setLabelTemplate(self, t):
            self.labels = LabelsSource(t)
            return self

        def setLabelsSource(self, s):
            self.labels = s
            return self

        def build(self):
            return BasicLabelAwareIterator(self.source, self.labels)

    def __init__(self, source, labelsSource=None):
        self.source = source
        self.labelsSource = labelsSource or LabelsSource("DOC_%d")
        self.reset()

    def reset(self):
        self.source.reset()
        self.labelsSource.reset()

    def hasNextDocument(self):
        return self.source.hasNextDocument() if isinstance(self.source, LabelAwareIterator) else self.source.hasNext()

    def nextDocument(self):
        if isinstance(self.source, LabelAwareIterator):
            d = self.source.nextDocument()
            for l in d.labels:
                self.labelsSource.storeLabel(l)
            return d
        return LabelledDocument(self.source.nextSentence(), [self.labelsSource.nextLabel()])


class FileLabelAwareIterator(LabelAwareIterator):
    """Documents from ``root/<label>/<file>``: one document per file, labelled by its parent directory."""

    class Builder:
        def __init__(self):
            self.roots = []

        def addSourceFolder(self, p):
            self.roots.append(p)
            return self

        def build(self):
            return FileLabelAwareIterator(self.roots)

    def __init__(self, roots):
        self.files = []
        for r in roots:
            for lab in sorted(os.listdir(r)):
                d = os.path.join(r, lab)
                if os.path.isdir(d):
                    for f in sorted(os.listdir(d)):
                        self.files.append((os.path.join(d, f), lab))
        self.labelsSource = LabelsSource(sorted({l for _, l in self.files}))
        self._i = 0

    def hasNextDocument(self):
        return self._i < len(self.files)

    def nextDocument(self):
        p, lab = self.files[self._i]
        self._i += 1
        with open(p, encoding="utf-8", errors="replace") as fh:
            return LabelledDocument(fh.read(), [lab])

    def reset(self):
        self._i = 0


class FilenamesLabelAwareIterator(FileLabelAwareIterator):
    """Documents from files in folders, labelled by their file name."""

    def __init__(self, roots):
        self.files = []
        for r in roots:
            for dp, _, fs in os.walk(r):
                for f in sorted(fs):
                    self.files.append((os.path.join(dp, f), f))
        self.labelsSource = LabelsSource([l for _, l in self.files])
        self._i = 0


class ContextLabelRetriever:
    """Inline span labels (reference deeplearning4j-nlp-uima/.../util/ContextLabelRetriever.java): in
    "<POS> great film </POS> overall" the tokens between <LABEL> and </LABEL> carry LABEL and every other run of
    tokens carries "none"; returns (the sentence without the tags, {(firstToken, endToken): label})."""

    @staticmethod
    def stringWithLabels(sentence, tokenizerFactory):
        import re
        tokens = tokenizerFactory.create(sentence).getTokens()
        words, spans = [], {}
        label, start = None, 0

        def close(lab):
            if len(words) > start:
                spans[(start, len(words))] = lab
        for t in tokens:
            m = re.fullmatch(r"<(/?)([^<>/\s]+)>", t)
            if m and not m.group(1):                  # opening tag: close the running "none" span
                close("none")
                label, start = m.group(2), len(words)
            elif m and m.group(1):                    # closing tag
                if label != m.group(2):
                    raise ValueError(f"closing tag </{m.group(2)}> does not match <{label}>")
                close(label)
                label, start = None, len(words)
            else:
                words.append(t)
        if label is not None:
            raise ValueError(f"unclosed label <{label}>")
        close("none")
        return " ".join(words), spans
