"""Lattice (Viterbi) morphological analyser for Japanese, the algorithm of the reference's vendored Kuromoji
(deeplearning4j-nlp-japanese: com/atilika/kuromoji/viterbi/ViterbiBuilder.java, ViterbiSearcher.java,
dict/CharacterDefinitions.java, dict/UnknownDictionary.java, dict/UserDictionary.java, TokenizerBase.Mode).

* A lexicon maps surface strings to entries (left context id, right context id, word cost, features); a connection
  matrix gives the cost of every (right id of the previous word, left id of the next word) pair. The best analysis is
  the minimum-cost path through the lattice of every lexicon match at every position, between BOS and EOS.
* Unknown words come from the character categories of ``char.def`` (INVOKE: also when the lexicon matches, GROUP: one
  candidate for the whole same-category run, LENGTH: candidates of 1..n characters) with the per-category entries of
  ``unk.def``.
* A user dictionary (``surface,segmentation,readings,part-of-speech`` lines) forces its segmentation and features.
* SEARCH mode adds Kuromoji's length penalty for long kanji / other tokens, which decompounds them.

Dictionaries: ``Lexicon.from_mecab_dir`` reads the standard MeCab / IPADIC source files (``*.csv``, ``matrix.def``,
``char.def``, ``unk.def``); ``Lexicon.from_features_corpus`` estimates a lexicon and connection costs (negative
log-probabilities of an HMM over part-of-speech classes) from a tokenized ``surface<TAB>features`` corpus. The IPADIC
dictionary itself is not in this image, so the default factory uses a small built-in lexicon of function words and
unknown-word processing; load a real dictionary for full-quality analysis.
"""
import glob
import math
import os
import unicodedata

# ------------------------------------------------------------------------------------------------ characters
# Built-in category table (code point ranges) used when no char.def is given.
_BUILTIN_CATEGORIES = {          # name: (invoke, group, length)
    "DEFAULT": (0, 1, 0), "SPACE": (0, 1, 0), "KANJI": (0, 0, 2), "SYMBOL": (1, 1, 0), "NUMERIC": (1, 1, 0),
    "ALPHA": (1, 1, 0), "HIRAGANA": (0, 1, 2), "KATAKANA": (1, 1, 2), "KANJINUMERIC": (1, 1, 0), "GREEK": (1, 1, 0),
    "CYRILLIC": (1, 1, 0),
}
_BUILTIN_RANGES = [
    (0x0020, 0x0020, ["SPACE"]), (0x00D0, 0x00D0, ["SPACE"]), (0x0009, 0x000B, ["SPACE"]), (0x3000, 0x3000, ["SPACE"]),
    (0x0030, 0x0039, ["NUMERIC"]), (0xFF10, 0xFF19, ["NUMERIC"]),
    (0x0041, 0x005A, ["ALPHA"]), (0x0061, 0x007A, ["ALPHA"]), (0xFF21, 0xFF3A, ["ALPHA"]), (0xFF41, 0xFF5A, ["ALPHA"]),
    (0x0021, 0x002F, ["SYMBOL"]), (0x003A, 0x0040, ["SYMBOL"]), (0x005B, 0x0060, ["SYMBOL"]),
    (0x007B, 0x007E, ["SYMBOL"]), (0x3001, 0x303F, ["SYMBOL"]), (0xFF01, 0xFF0F, ["SYMBOL"]),
    (0xFF1A, 0xFF20, ["SYMBOL"]), (0xFF3B, 0xFF40, ["SYMBOL"]), (0xFF5B, 0xFF65, ["SYMBOL"]),
    (0x2000, 0x206F, ["SYMBOL"]), (0x25A0, 0x25FF, ["SYMBOL"]),
    (0x0391, 0x03C9, ["GREEK"]), (0x0401, 0x044F, ["CYRILLIC"]),
    (0x3041, 0x309F, ["HIRAGANA"]), (0x30A1, 0x30FF, ["KATAKANA"]), (0x31F0, 0x31FF, ["KATAKANA"]),
    (0xFF66, 0xFF9D, ["KATAKANA"]), (0x30FC, 0x30FC, ["KATAKANA", "HIRAGANA"]),
    (0x2E80, 0x2FDF, ["KANJI"]), (0x3005, 0x3007, ["KANJI"]), (0x3400, 0x4DBF, ["KANJI"]),
    (0x4E00, 0x9FFF, ["KANJI"]), (0xF900, 0xFAFF, ["KANJI"]),
    (0x4E00, 0x4E00, ["KANJINUMERIC", "KANJI"]), (0x4E8C, 0x4E8C, ["KANJINUMERIC", "KANJI"]),
    (0x4E09, 0x4E09, ["KANJINUMERIC", "KANJI"]), (0x56DB, 0x56DB, ["KANJINUMERIC", "KANJI"]),
    (0x4E94, 0x4E94, ["KANJINUMERIC", "KANJI"]), (0x516D, 0x516D, ["KANJINUMERIC", "KANJI"]),
    (0x4E03, 0x4E03, ["KANJINUMERIC", "KANJI"]), (0x516B, 0x516B, ["KANJINUMERIC", "KANJI"]),
    (0x4E5D, 0x4E5D, ["KANJINUMERIC", "KANJI"]), (0x5341, 0x5341, ["KANJINUMERIC", "KANJI"]),
    (0x767E, 0x767E, ["KANJINUMERIC", "KANJI"]), (0x5343, 0x5343, ["KANJINUMERIC", "KANJI"]),
    (0x4E07, 0x4E07, ["KANJINUMERIC", "KANJI"]), (0x5104, 0x5104, ["KANJINUMERIC", "KANJI"]),
    (0x5146, 0x5146, ["KANJINUMERIC", "KANJI"]),
]


class CharacterDefinitions:
    """Category of every code point plus each category's (invoke, group, length) rule (char.def)."""

    def __init__(self, categories=None, ranges=None):
        self.categories = dict(categories or _BUILTIN_CATEGORIES)
        self.ranges = list(ranges or _BUILTIN_RANGES)
        self._cache = {}

    @staticmethod
    def parse(text):
        cats, ranges = {}, []
        for raw in text.splitlines():
            line = raw.split("#", 1)[0].strip()
            if not line:
                continue
            p = line.split()
            if p[0].startswith("0x"):
                lo, _, hi = p[0].partition("..")
                ranges.append((int(lo, 16), int(hi or lo, 16), p[1:]))
            elif len(p) >= 4:
                cats[p[0]] = (int(p[1]), int(p[2]), int(p[3]))
        return CharacterDefinitions(cats, ranges)

    def lookup(self, ch):
        """Categories of one character, most specific (last matching range) first."""
        c = self._cache.get(ch)
        if c is None:
            cp = ord(ch)
            c = ["DEFAULT"]
            for lo, hi, names in self.ranges:          # later ranges refine earlier ones, as in char.def
                if lo <= cp <= hi:
                    c = [n for n in names if n in self.categories] or c
            self._cache[ch] = c
        return c

    def category(self, ch):
        return self.lookup(ch)[0]


# ------------------------------------------------------------------------------------------------ dictionaries
class Entry:
    __slots__ = ("surface", "left", "right", "cost", "features", "kind")

    def __init__(self, surface, left, right, cost, features, kind="known"):
        self.surface, self.left, self.right, self.cost = surface, int(left), int(right), int(cost)
        self.features, self.kind = list(features), kind


class ConnectionCosts:
    def __init__(self, table=None, default=0):
        self.table = dict(table or {})
        self.default = default

    def get(self, right, left):
        return self.table.get((right, left), self.default)

    @staticmethod
    def parse_matrix_def(text):
        lines = [ln.split() for ln in text.splitlines() if ln.strip()]
        t = {(int(a), int(b)): int(c) for a, b, c in (ln for ln in lines[1:] if len(ln) == 3)}
        return ConnectionCosts(t)


class Lexicon:
    def __init__(self, entries, connections, chardef=None, unknown=None):
        self.by_surface = {}
        for e in entries:
            self.by_surface.setdefault(e.surface, []).append(e)
        self.max_len = max((len(s) for s in self.by_surface), default=1)
        self.connections = connections
        self.chardef = chardef or CharacterDefinitions()
        self.unknown = unknown or {}          # category -> [Entry]

    def lookup(self, text, pos):
        """(length, entries) of every lexicon surface starting at ``pos``."""
        out = []
        for n in range(1, min(self.max_len, len(text) - pos) + 1):
            es = self.by_surface.get(text[pos:pos + n])
            if es:
                out.append((n, es))
        return out

    # -- loaders
    @staticmethod
    def parse_unk_def(text):
        unk = {}
        for raw in text.splitlines():
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            p = line.split(",")
            unk.setdefault(p[0], []).append(Entry(p[0], p[1], p[2], p[3], p[4:], "unknown"))
        return unk

    @staticmethod
    def from_mecab_dir(path, encoding="euc-jp"):
        """MeCab / IPADIC source dictionary: every ``*.csv`` (surface,left,right,cost,features...), ``matrix.def``,
        ``char.def`` and ``unk.def`` (the files Kuromoji's DictionaryCompiler reads)."""
        def read(name):
            with open(os.path.join(path, name), "rb") as fh:
                return fh.read().decode(encoding, errors="replace")
        entries = []
        for f in sorted(glob.glob(os.path.join(path, "*.csv"))):
            with open(f, "rb") as fh:
                for line in fh.read().decode(encoding, errors="replace").splitlines():
                    p = line.split(",")
                    if len(p) >= 4:
                        entries.append(Entry(p[0], p[1], p[2], p[3], p[4:]))
        return Lexicon(entries, ConnectionCosts.parse_matrix_def(read("matrix.def")),
                       CharacterDefinitions.parse(read("char.def")), Lexicon.parse_unk_def(read("unk.def")))

    @staticmethod
    def from_features_corpus(lines, chardef=None, unknown_text=None, scale=100.0, smoothing=0.5):
        """Estimate a lexicon from tokenized ``surface<TAB>f1,f2,...`` lines (one sentence boundary per blank line /
        sentence-final punctuation). Context ids are part-of-speech classes (the first six features); word cost =
        -scale*log P(surface | class), connection cost = -scale*log P(class | previous class) (add-``smoothing``)."""
        cls_id, counts, trans, cls_n = {"BOS/EOS": 0}, {}, {}, {}
        prev = 0
        for raw in lines:
            line = raw.rstrip("\n")
            if not line.strip():
                trans[(prev, 0)] = trans.get((prev, 0), 0) + 1
                prev = 0
                continue
            if "\t" not in line:
                continue
            surf, feats = line.split("\t", 1)
            f = feats.split(",")
            key = tuple(f[:6])
            c = cls_id.setdefault(key, len(cls_id))
            counts[(surf, c, feats)] = counts.get((surf, c, feats), 0) + 1
            cls_n[c] = cls_n.get(c, 0) + 1
            trans[(prev, c)] = trans.get((prev, c), 0) + 1
            prev = c
            if surf in ("。", "．", "！", "？"):
                trans[(prev, 0)] = trans.get((prev, 0), 0) + 1
                prev = 0
        trans[(prev, 0)] = trans.get((prev, 0), 0) + 1
        ncls = len(cls_id)
        out_n = {}
        for (a, _), n in trans.items():
            out_n[a] = out_n.get(a, 0) + n
        table = {}
        for a in range(ncls):
            tot = out_n.get(a, 0) + smoothing * ncls
            for b in range(ncls):
                table[(a, b)] = int(round(-scale * math.log((trans.get((a, b), 0) + smoothing) / tot)))
        entries = [Entry(s, c, c, int(round(-scale * math.log(n / cls_n[c]))), feats.split(","))
                   for (s, c, feats), n in counts.items()]
        unk = {}
        if unknown_text is not None:
            for cat, es in Lexicon.parse_unk_def(unknown_text).items():
                for e in es:
                    key = tuple(e.features[:6])
                    c = cls_id.get(key)
                    if c is None:
                        continue
                    # ipadic unknown-word costs are on another scale: rank them above the rarest known word
                    unk.setdefault(cat, []).append(Entry(cat, c, c, int(scale * 12 + e.cost / 100), e.features,
                                                         "unknown"))
        # a noun class for categories unk.def did not map
        noun = next((c for k, c in cls_id.items() if k[:2] == ("名詞", "一般")), 1)
        for cat in (chardef or CharacterDefinitions()).categories:
            unk.setdefault(cat, [Entry(cat, noun, noun, int(scale * 14), ["名詞", "一般", "*", "*", "*", "*", "*"],
                                       "unknown")])
        lex = Lexicon(entries, ConnectionCosts(table, int(scale * 10)), chardef, unk)
        lex.classes = cls_id
        # search-mode penalties are IPADIC-unit constants: express them in this lexicon's cost units (the ratio of
        # its unknown-katakana cost to IPADIC's 9461, the unit Kuromoji's 1700-per-character penalty is set against)
        kata = unk.get("KATAKANA")
        lex.penalty_scale = (min(e.cost for e in kata) / 9461.0) if kata else scale / 700.0
        return lex


class UserDictionary:
    """``surface,segmentation,readings,part-of-speech`` (Kuromoji's user dictionary format)."""

    def __init__(self, entries=()):
        self.entries = {}
        for surface, seg, readings, pos in entries:
            self.entries[surface] = (seg.split(), readings.split(), pos)
        self.max_len = max((len(s) for s in self.entries), default=0)

    @staticmethod
    def parse(text):
        rows = []
        for raw in text.splitlines():
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            p = [x.strip() for x in line.split(",")]
            if len(p) >= 4:
                rows.append((p[0], p[1], p[2], p[3]))
        return UserDictionary(rows)

    def match(self, text, pos):
        out = []
        for n in range(1, min(self.max_len, len(text) - pos) + 1):
            e = self.entries.get(text[pos:pos + n])
            if e:
                out.append((n, e))
        return out


# ------------------------------------------------------------------------------------------------ tokens / search
class Token:
    def __init__(self, surface, position, features, kind="known"):
        self.surface, self.position, self.features, self.kind = surface, position, list(features), kind

    def getSurface(self):
        return self.surface

    def getPosition(self):
        return self.position

    def getAllFeatures(self):
        return ",".join(self.features)

    def getAllFeaturesArray(self):
        return list(self.features)

    def _f(self, i):
        return self.features[i] if i < len(self.features) else "*"

    def getPartOfSpeechLevel1(self):
        return self._f(0)

    def getPartOfSpeechLevel2(self):
        return self._f(1)

    def getBaseForm(self):
        b = self._f(6)
        return self.surface if b == "*" else b

    def getReading(self):
        return self._f(7)

    def getPronunciation(self):
        return self._f(8)

    def isKnown(self):
        return self.kind in ("known", "user")

    def isUser(self):
        return self.kind == "user"

    def __repr__(self):
        return f"{self.surface}\t{self.getAllFeatures()}"


class Mode:
    NORMAL, SEARCH, EXTENDED = "NORMAL", "SEARCH", "EXTENDED"


class LatticeTokenizer:
    """Kuromoji-style tokenizer over a ``Lexicon`` (+ optional ``UserDictionary``)."""
    # search-mode penalties (Kuromoji TokenizerBase defaults)
    KANJI_LEN, KANJI_PENALTY, OTHER_LEN, OTHER_PENALTY = 2, 3000, 7, 1700

    def __init__(self, lexicon, user=None, mode=Mode.NORMAL):
        self.lex, self.user, self.mode = lexicon, user, mode

    def _unknown(self, text, pos, has_known):
        cd = self.lex.chardef
        ch = text[pos]
        out = []
        for cat in cd.lookup(ch)[:1]:
            invoke, group, length = cd.categories.get(cat, (0, 1, 0))
            if has_known and not invoke:
                continue
            ents = self.lex.unknown.get(cat) or self.lex.unknown.get("DEFAULT") or []
            lens = set()
            if group:
                n = 1
                while pos + n < len(text) and cat in cd.lookup(text[pos + n]) and n < 1024:
                    n += 1
                lens.add(n)
            for n in range(1, length + 1):
                if pos + n <= len(text) and all(cat in cd.lookup(c) for c in text[pos:pos + n]):
                    lens.add(n)
            if not lens:
                lens.add(1)
            for n in lens:
                for e in ents:
                    out.append((n, Entry(text[pos:pos + n], e.left, e.right, e.cost, e.features, "unknown")))
        return out

    def _penalty(self, surf):
        if self.mode == Mode.NORMAL:
            return 0
        n = len(surf)
        cd = self.lex.chardef
        k = getattr(self.lex, "penalty_scale", 1.0)        # lexicon cost units per IPADIC cost unit
        if all(cd.category(c) == "KANJI" for c in surf):
            return k * (n - self.KANJI_LEN) * self.KANJI_PENALTY if n > self.KANJI_LEN else 0
        return k * (n - self.OTHER_LEN) * self.OTHER_PENALTY if n > self.OTHER_LEN else 0

    def _analyze(self, text):
        N = len(text)
        # ends[i]: nodes ending at i: (cost_so_far, right_id, start, entry_or_user, back_index)
        INF = float("inf")
        ends = [[] for _ in range(N + 1)]
        ends[0].append((0, 0, -1, None, None))
        conn = self.lex.connections
        for i in range(N):
            if not ends[i]:
                continue
            cands = []
            user = self.user.match(text, i) if self.user else []
            for n, (seg, readings, pos) in user:
                cands.append((n, ("user", seg, readings, pos), 0, 0, -100000 * n))
            known = self.lex.lookup(text, i)
            for n, es in known:
                for e in es:
                    cands.append((n, e, e.left, e.right, e.cost))
            if text[i].isspace() and not known:
                pass
            for n, e in self._unknown(text, i, bool(known)):
                cands.append((n, e, e.left, e.right, e.cost))
            for n, node, left, right, wcost in cands:
                surf = text[i:i + n]
                best, bj = INF, None
                for j, (c, r, _, _, _) in enumerate(ends[i]):
                    v = c + conn.get(r, left)
                    if v < best:
                        best, bj = v, j
                ends[i + n].append((best + wcost + self._penalty(surf), right, i, node, bj))
        best, bj = INF, None
        for j, (c, r, _, _, _) in enumerate(ends[N]):
            v = c + conn.get(r, 0)
            if v < best:
                best, bj = v, j
        path, i, j = [], N, bj
        while j is not None and i > 0:
            _, _, start, node, back = ends[i][j]
            path.append((start, i, node))
            i, j = start, back
        return path[::-1]

    def tokenize(self, text):
        text = unicodedata.normalize("NFC", text)
        toks = []
        for start, end, node in self._analyze(text):
            if isinstance(node, tuple) and node[0] == "user":
                _, seg, readings, pos = node
                p = start
                for k, s in enumerate(seg):
                    rd = readings[k] if k < len(readings) else "*"
                    toks.append(Token(s, p, [pos, "*", "*", "*", "*", "*", "*", rd, "*"], "user"))
                    p += len(s)
            else:
                toks.append(Token(text[start:end], start, node.features, node.kind))
        return toks


# ------------------------------------------------------------------------------------------------ built-in lexicon
# A small lexicon of closed-class words (particles, auxiliaries, copula, common inflection endings and a few
# high-frequency nouns) with hand-set costs; content words come from unknown-word processing. Features follow IPADIC
# (POS1,POS2,POS3,POS4,conj-type,conj-form,base,reading,pronunciation).
_P = "助詞"
_BUILTIN_WORDS = [
    ("は", _P, "係助詞", "ハ", 300), ("が", _P, "格助詞", "ガ", 300), ("を", _P, "格助詞", "ヲ", 300),
    ("に", _P, "格助詞", "ニ", 300), ("へ", _P, "格助詞", "ヘ", 300), ("で", _P, "格助詞", "デ", 400),
    ("と", _P, "格助詞", "ト", 350), ("も", _P, "係助詞", "モ", 350), ("の", _P, "連体化", "ノ", 300),
    ("や", _P, "並立助詞", "ヤ", 450), ("から", _P, "格助詞", "カラ", 350), ("まで", _P, "副助詞", "マデ", 400),
    ("より", _P, "格助詞", "ヨリ", 450), ("か", _P, "副助詞／並立助詞／終助詞", "カ", 450),
    ("ね", _P, "終助詞", "ネ", 500), ("よ", _P, "終助詞", "ヨ", 500), ("て", _P, "接続助詞", "テ", 350),
    ("ば", _P, "接続助詞", "バ", 450), ("けど", _P, "接続助詞", "ケド", 450), ("だけ", _P, "副助詞", "ダケ", 450),
]
_BUILTIN_AUX = [  # surface, conj type, conj form, base, reading, cost
    ("な", "特殊・ダ", "体言接続", "だ", "ナ", 450), ("だ", "特殊・ダ", "基本形", "だ", "ダ", 400),
    ("です", "特殊・デス", "基本形", "です", "デス", 400), ("た", "特殊・タ", "基本形", "た", "タ", 300),
    ("ます", "特殊・マス", "基本形", "ます", "マス", 350), ("まし", "特殊・マス", "連用形", "ます", "マシ", 400),
    ("ない", "特殊・ナイ", "基本形", "ない", "ナイ", 450), ("ませ", "特殊・マス", "未然形", "ます", "マセ", 450),
    ("ん", "不変化型", "基本形", "ん", "ン", 500),
]
_BUILTIN_OTHER = [  # surface, features, cost: pronouns, formal nouns, the light verb and punctuation
    ("彼", ["名詞", "代名詞", "一般", "*", "*", "*", "彼", "カレ", "カレ"], 500),
    ("私", ["名詞", "代名詞", "一般", "*", "*", "*", "私", "ワタシ", "ワタシ"], 500),
    ("これ", ["名詞", "代名詞", "一般", "*", "*", "*", "これ", "コレ", "コレ"], 500),
    ("それ", ["名詞", "代名詞", "一般", "*", "*", "*", "それ", "ソレ", "ソレ"], 500),
    ("こと", ["名詞", "非自立", "一般", "*", "*", "*", "こと", "コト", "コト"], 500),
    ("もの", ["名詞", "非自立", "一般", "*", "*", "*", "もの", "モノ", "モノ"], 500),
    ("する", ["動詞", "自立", "*", "*", "サ変・スル", "基本形", "する", "スル", "スル"], 500),
    ("し", ["動詞", "自立", "*", "*", "サ変・スル", "連用形", "する", "シ", "シ"], 550),
    ("い", ["動詞", "非自立", "*", "*", "一段", "連用形", "いる", "イ", "イ"], 700),
    ("いる", ["動詞", "非自立", "*", "*", "一段", "基本形", "いる", "イル", "イル"], 600),
    ("ある", ["動詞", "自立", "*", "*", "五段・ラ行", "基本形", "ある", "アル", "アル"], 600),
    ("。", ["記号", "句点", "*", "*", "*", "*", "。", "。", "。"], 100),
    ("、", ["記号", "読点", "*", "*", "*", "*", "、", "、", "、"], 100),
]
_BUILTIN_CLASSES = ["BOS/EOS", "名詞", "助詞", "助動詞", "動詞", "形容詞", "記号", "副詞", "連体詞", "接続詞"]
# connection costs between the coarse classes above (row: previous, column: next); low = likely
_BUILTIN_CONN = {
    "BOS/EOS": {"名詞": 0, "動詞": 200, "形容詞": 200, "副詞": 200, "連体詞": 300, "接続詞": 300, "記号": 300},
    "名詞": {"助詞": 0, "助動詞": 200, "名詞": 600, "BOS/EOS": 300, "記号": 100, "動詞": 500},
    "助詞": {"名詞": 0, "動詞": 100, "形容詞": 200, "副詞": 200, "BOS/EOS": 400, "記号": 200, "助詞": 600},
    "助動詞": {"BOS/EOS": 0, "記号": 0, "名詞": 200, "助詞": 300, "助動詞": 200},
    "動詞": {"助動詞": 0, "助詞": 100, "動詞": 200, "BOS/EOS": 300, "名詞": 400, "記号": 300},
    "形容詞": {"名詞": 0, "助詞": 200, "助動詞": 200, "BOS/EOS": 300, "記号": 200},
    "記号": {"BOS/EOS": 0, "名詞": 100, "記号": 200, "動詞": 300, "副詞": 300},
}


def builtin_lexicon():
    cid = {c: i for i, c in enumerate(_BUILTIN_CLASSES)}
    es = []
    for s, p1, p2, rd, cost in _BUILTIN_WORDS:
        es.append(Entry(s, cid[p1], cid[p1], cost, [p1, p2, "*", "*", "*", "*", s, rd, rd]))
    for s, ct, cf, base, rd, cost in _BUILTIN_AUX:
        es.append(Entry(s, cid["助動詞"], cid["助動詞"], cost, ["助動詞", "*", "*", "*", ct, cf, base, rd, rd]))
    for s, f, cost in _BUILTIN_OTHER:
        es.append(Entry(s, cid[f[0]], cid[f[0]], cost, f))
    table = {}
    for a, row in _BUILTIN_CONN.items():
        for b, c in row.items():
            table[(cid[a], cid[b])] = c
    noun = cid["名詞"]
    unk = {cat: [Entry(cat, noun, noun, 900 if cat in ("KANJI", "KATAKANA", "ALPHA", "NUMERIC") else 1500,
                       ["名詞", "一般" if cat != "SYMBOL" else "サ変接続", "*", "*", "*", "*", "*"], "unknown")]
           for cat in _BUILTIN_CATEGORIES}
    unk["SYMBOL"] = [Entry("SYMBOL", cid["記号"], cid["記号"], 800, ["記号", "一般", "*", "*", "*", "*", "*"],
                           "unknown")]
    unk["HIRAGANA"] = [Entry("HIRAGANA", noun, noun, 2500, ["名詞", "一般", "*", "*", "*", "*", "*"], "unknown")]
    return Lexicon(es, ConnectionCosts(table, 800), CharacterDefinitions(), unk)
