"""WordVectorSerializer: the reference's embedding file formats.

Reference: NLP:models/embeddings/loader/WordVectorSerializer.java
  * text vectors (writeWordVectors:339): header ``"<numWords> <layerSize> <numDocs>"`` then ``B64:<base64 label> v1 v2
    ...`` per line; loadTxtVectors also accepts plain ``word v1 v2 ...`` (GloVe / word2vec text) with or without header
  * Google word2vec binary (readBinaryModel): ``"<V> <D>\\n"`` then per word ``word<space>`` + D little-endian float32
    (+ optional newline)
  * full Word2Vec zip (writeWord2VecModel:450): syn0.txt, syn1.txt, syn1Neg.txt, codes.txt, huffman.txt,
    frequencies.txt, config.json; ParagraphVectors zip adds labels.txt
  * vocab cache (writeVocabCache:2031): JSON lines
All readers are plain parsers (text / struct); nothing is deserialized by executing code.
"""
import base64
import io
import json
import struct
import zipfile

import numpy as np
import torch

from .embeddings import InMemoryLookupTable, WordVectorsImpl
from .vocab import AbstractCache, VocabWord


def encodeB64(word):
    return "B64:" + base64.b64encode(word.encode("utf-8")).decode("ascii")


def decodeB64(word):
    if word.startswith("B64:"):
        return base64.b64decode(word[4:]).decode("utf-8")
    return word


def _fmt_row(v):
    return " ".join(repr(float(x)) for x in v)


class StaticWord2Vec(WordVectorsImpl):
    """Read-only vectors (loadStaticModel)."""


class WordVectorSerializer:
    encodeB64 = staticmethod(encodeB64)
    decodeB64 = staticmethod(decodeB64)

    # ------------------------------------------------------------------ text vectors
    @staticmethod
    def writeWordVectors(vectors, path):
        """Text format with header; labels B64-encoded (the reference's writeWordVectors(lookupTable, file))."""
        table = vectors.lookupTable() if hasattr(vectors, "lookupTable") else vectors
        vocab = table.vocab
        syn0 = table.syn0.detach().cpu().double().numpy()
        out = io.StringIO()
        out.write(f"{vocab.numWords()} {table.vectorLength} {vocab.totalNumberOfDocs()}\n")
        for i, e in enumerate(vocab.vocabWords()):
            out.write(encodeB64(e.label) + " " + _fmt_row(syn0[i]) + "\n")
        data = out.getvalue()
        if hasattr(path, "write"):
            path.write(data.encode("utf-8") if "b" in getattr(path, "mode", "") else data)
        else:
            with open(path, "w", encoding="utf-8") as fh:
                fh.write(data)

    @staticmethod
    def loadTxt(path):
        vocab = AbstractCache()
        rows, labels = [], []
        with open(path, encoding="utf-8") as fh:
            first = fh.readline()
            parts = first.split()
            header = len(parts) in (2, 3) and all(p.lstrip("-").isdigit() for p in parts)
            lines = fh if header else _chain([first], fh)
            for line in lines:
                p = line.rstrip("\n").split(" ")
                if len(p) < 2:
                    continue
                labels.append(decodeB64(p[0]))
                rows.append(np.array(p[1:], dtype=np.float32))
        for i, l in enumerate(labels):
            e = VocabWord(l, 1.0)
            vocab.addToken(e)
        vocab.reindex(labels)
        table = InMemoryLookupTable(vocab, rows[0].shape[0] if rows else 0, useHierarchicSoftmax=False)
        table.syn0 = torch.from_numpy(np.stack(rows)) if rows else torch.zeros(0, 0)
        return table, vocab

    @staticmethod
    def loadTxtVectors(path):
        table, vocab = WordVectorSerializer.loadTxt(path)
        return StaticWord2Vec(table, vocab)

    # ------------------------------------------------------------------ google binary
    @staticmethod
    def writeBinaryModel(vectors, path):
        table = vectors.lookupTable()
        syn0 = table.syn0.detach().cpu().float().numpy()
        with open(path, "wb") as fh:
            fh.write(f"{syn0.shape[0]} {syn0.shape[1]}\n".encode())
            for i, e in enumerate(table.vocab.vocabWords()):
                fh.write(e.label.encode("utf-8") + b" ")
                fh.write(syn0[i].astype("<f4").tobytes())
                fh.write(b"\n")

    @staticmethod
    def readBinaryModel(path, linebreaks=True, normalize=False):
        with open(path, "rb") as fh:
            V, D = (int(x) for x in fh.readline().split())
            labels, rows = [], np.empty((V, D), dtype=np.float32)
            for i in range(V):
                w = bytearray()
                while True:
                    ch = fh.read(1)
                    if ch == b" " or ch == b"":
                        break
                    if ch != b"\n":
                        w += ch
                labels.append(w.decode("utf-8", errors="replace"))
                rows[i] = np.frombuffer(fh.read(4 * D), dtype="<f4")
        if normalize:
            rows /= np.maximum(np.linalg.norm(rows, axis=1, keepdims=True), 1e-12)
        vocab = AbstractCache()
        for l in labels:
            vocab.addToken(VocabWord(l, 1.0))
        vocab.reindex(labels)
        table = InMemoryLookupTable(vocab, D, useHierarchicSoftmax=False)
        table.syn0 = torch.from_numpy(rows)
        return StaticWord2Vec(table, vocab)

    loadGoogleModel = readBinaryModel

    @staticmethod
    def loadStaticModel(path):
        with open(path, "rb") as fh:
            head = fh.read(4)
        if head[:2] == b"PK":
            return WordVectorSerializer.readWord2VecModel(path)
        try:
            return WordVectorSerializer.loadTxtVectors(path)
        except (UnicodeDecodeError, ValueError):
            return WordVectorSerializer.readBinaryModel(path)

    # ------------------------------------------------------------------ full zip models
    @staticmethod
    def _matrix_txt(t):
        if t is None:
            return ""
        a = t.detach().cpu().double().numpy()
        return "".join(_fmt_row(r) + "\n" for r in a)

    @staticmethod
    def writeWord2VecModel(vectors, path, extra=None):
        table = vectors.lookupTable()
        vocab = vectors.vocab()
        with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
            buf = io.StringIO()
            WordVectorSerializer.writeWordVectors(table, buf)
            z.writestr("syn0.txt", buf.getvalue())
            z.writestr("syn1.txt", WordVectorSerializer._matrix_txt(table.syn1))
            z.writestr("syn1Neg.txt", WordVectorSerializer._matrix_txt(table.syn1Neg))
            z.writestr("codes.txt", "".join(encodeB64(e.label) + "".join(f" {c}" for c in e.codes) + "\n"
                                           for e in vocab.vocabWords()))
            z.writestr("huffman.txt", "".join(encodeB64(e.label) + "".join(f" {p}" for p in e.points) + "\n"
                                             for e in vocab.vocabWords()))
            z.writestr("frequencies.txt", "".join(
                f"{encodeB64(e.label)} {e.elementFrequency} {e.sequencesCount}\n" for e in vocab.vocabWords()))
            z.writestr("config.json", vectors.getConfiguration().toJson())
            if extra:
                for k, v in extra.items():
                    z.writestr(k, v)

    @staticmethod
    def writeParagraphVectors(vectors, path):
        labels = "".join(encodeB64(e.label) + "\n" for e in vectors.vocab().vocabWords() if e.special)
        WordVectorSerializer.writeWord2VecModel(vectors, path, {"labels.txt": labels})

    @staticmethod
    def _read_zip(path, cls):
        from .word2vec import VectorsConfiguration
        with zipfile.ZipFile(path) as z:
            names = set(z.namelist())
            conf = VectorsConfiguration.fromJson(z.read("config.json").decode()) if "config.json" in names \
                else VectorsConfiguration()
            lines = z.read("syn0.txt").decode("utf-8").splitlines()
            hdr = lines[0].split()
            ndocs = int(hdr[2]) if len(hdr) > 2 else 0
            labels, rows = [], []
            for ln in lines[1:]:
                p = ln.split(" ")
                labels.append(decodeB64(p[0]))
                rows.append(np.array(p[1:], dtype=np.float32))
            D = rows[0].shape[0] if rows else conf.layersSize
            special = set()
            if "labels.txt" in names:
                special = {decodeB64(l.strip()) for l in z.read("labels.txt").decode().splitlines() if l.strip()}
            vocab = AbstractCache()
            freq = {}
            if "frequencies.txt" in names:
                for ln in z.read("frequencies.txt").decode().splitlines():
                    p = ln.split(" ")
                    freq[decodeB64(p[0])] = (float(p[1]), int(float(p[2])) if len(p) > 2 else 0)
            for l in labels:
                e = VocabWord(l, freq.get(l, (1.0, 0))[0], special=l in special)
                e.sequencesCount = freq.get(l, (1.0, 0))[1]
                vocab.addToken(e)
            vocab.reindex(labels)
            vocab.setTotalDocCount(ndocs)
            vocab.updateWordsOccurrences()
            for fname, attr, conv in (("codes.txt", "codes", int), ("huffman.txt", "points", int)):
                if fname in names:
                    for ln in z.read(fname).decode().splitlines():
                        p = ln.split(" ")
                        e = vocab.wordFor(decodeB64(p[0]))
                        if e is not None:
                            setattr(e, attr, [conv(x) for x in p[1:] if x != ""])

            def mat(n):
                if n not in names:
                    return None
                txt = z.read(n).decode().strip()
                if not txt:
                    return None
                return torch.from_numpy(np.array([r.split(" ") for r in txt.splitlines()], dtype=np.float32))
            syn1, syn1neg = mat("syn1.txt"), mat("syn1Neg.txt")
        m = cls(conf)
        table = InMemoryLookupTable(vocab, D, conf.seed or 12345, syn1 is not None, conf.negative)
        table.syn0 = torch.from_numpy(np.stack(rows)) if rows else torch.zeros(0, D)
        table.syn1 = syn1
        table.syn1Neg = syn1neg
        if syn1neg is not None:
            table.initNegative()
            table.syn1Neg = syn1neg
        table._arrays()
        m._lookup = table
        m.vocabCache = vocab
        m.setVocab(vocab)
        m.device = "cpu"
        return m

    @staticmethod
    def readWord2VecModel(path, extendedModel=True):
        from .word2vec import Word2Vec
        return WordVectorSerializer._read_zip(path, Word2Vec)

    readWord2Vec = readWord2VecModel

    @staticmethod
    def readParagraphVectors(path):
        from .text import LabelsSource
        from .word2vec import ParagraphVectors
        m = WordVectorSerializer._read_zip(path, ParagraphVectors)
        m.labelsSource = LabelsSource([e.label for e in m.vocabCache.vocabWords() if e.special])
        return m

    # ------------------------------------------------------------------ vocab cache
    @staticmethod
    def writeVocabCache(vocab, path):
        with open(path, "w", encoding="utf-8") as fh:
            for e in vocab.vocabWords():
                fh.write(json.dumps({"word": e.label, "frequency": e.elementFrequency, "index": e.index,
                                     "special": e.special, "docs": e.sequencesCount, "codes": e.codes,
                                     "points": e.points}) + "\n")
            fh.write(json.dumps({"__meta__": True, "docs": vocab.totalNumberOfDocs()}) + "\n")

    @staticmethod
    def readVocabCache(path):
        vocab = AbstractCache()
        order = []
        ndocs = 0
        with open(path, encoding="utf-8") as fh:
            for line in fh:
                d = json.loads(line)
                if d.get("__meta__"):
                    ndocs = d["docs"]
                    continue
                e = VocabWord(d["word"], d["frequency"], special=d.get("special", False))
                e.sequencesCount = d.get("docs", 0)
                e.codes, e.points = d.get("codes", []), d.get("points", [])
                vocab.addToken(e)
                order.append((d["index"], d["word"]))
        vocab.reindex([w for _, w in sorted(order)])
        vocab.setTotalDocCount(ndocs)
        vocab.updateWordsOccurrences()
        return vocab

    @staticmethod
    def writeTsneFormat(vectors, coords, path):
        """CSV ``x,y,word`` of 2-D t-SNE coordinates (writeTsneFormat)."""
        c = coords.detach().cpu().numpy() if isinstance(coords, torch.Tensor) else np.asarray(coords)
        with open(path, "w", encoding="utf-8") as fh:
            for i, w in enumerate(vectors.vocab().words()):
                fh.write(",".join(repr(float(v)) for v in c[i]) + "," + w + "\n")


def _chain(a, b):
    yield from a
    yield from b


_ = struct
