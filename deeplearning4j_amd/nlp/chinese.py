"""Dictionary-based Chinese word segmentation (reference deeplearning4j-nlp-chinese: ChineseTokenizer over ansj_seg's
ToAnalysis, org/ansj/library/DATDictionary.java core dictionary, DicLibrary user words, Term natures).

Design: a word lattice over each Han run (every dictionary word starting at every position, plus the single character
as the fallback edge), scored with unigram log-probabilities log((freq + 1) / total) and solved by dynamic programming
right to left (the best segmentation of the suffix is known when a position is visited). Latin words, digit runs
(with a decimal point / thousands comma inside) and full-width forms (NFKC) form single tokens; punctuation is a token
of its own; whitespace separates.

Dictionaries:
  * ``CoreDictionary.from_ansj_core(path)`` reads ansj's ``core.dic`` dump (tab-separated
    ``id, word, base, check, status, {nature=freq, ...}``; status 2/3 rows are words, status 1 rows are prefixes only).
  * ``CoreDictionary.from_user_library(text)`` reads ansj userLibrary lines ``word [TAB nature [TAB freq]]``.
  * ``builtin_dictionary()`` holds a small set of closed-class words (pronouns, particles, conjunctions, measure
    words) so the segmenter is usable without a dictionary file; ``DL4J_AMD_ZH_DICT`` names a core.dic to load.
The dictionary data is read from files, nothing is vendored here.
"""
import math
import os
import unicodedata

__all__ = ["Term", "CoreDictionary", "Segmenter", "builtin_dictionary"]


class Term:
    """One segmented word with its part-of-speech nature (ansj Term: getName / getNatureStr / getOffe)."""
    __slots__ = ("name", "nature", "offset")

    def __init__(self, name, nature, offset):
        self.name, self.nature, self.offset = name, nature, offset

    def getName(self):
        return self.name

    def getNatureStr(self):
        return self.nature

    def getOffe(self):
        return self.offset

    def __repr__(self):
        return f"{self.name}/{self.nature}"


class CoreDictionary:
    """word -> (frequency, dominant nature); ``max_len`` bounds the lattice edges per position."""

    def __init__(self):
        self.words = {}
        self.total = 0
        self.max_len = 1

    def add(self, word, freq=1, nature="n"):
        if not word:
            return
        old = self.words.get(word)
        if old is not None:
            self.total -= old[0]
        self.words[word] = (int(freq), nature)
        self.total += int(freq)
        self.max_len = max(self.max_len, len(word))

    def __contains__(self, w):
        return w in self.words

    def __len__(self):
        return len(self.words)

    def logp(self, word):
        f = self.words.get(word)
        return math.log(((f[0] if f else 0) + 1.0) / (self.total + len(self.words) + 1.0))

    def nature(self, word, default="nw"):
        f = self.words.get(word)
        return f[1] if f else default

    @staticmethod
    def _natures(field):
        field = field.strip()
        if not field or field == "null":
            return None
        out = {}
        for part in field.strip("{}").split(","):
            if "=" in part:
                k, v = part.split("=", 1)
                try:
                    out[k.strip()] = int(v)
                except ValueError:
                    continue
        return out or None

    @classmethod
    def from_ansj_core(cls, path):
        d = cls()
        with open(path, encoding="utf-8") as fh:
            for line in fh:
                cols = line.rstrip("\n").split("\t")
                if len(cols) < 6:
                    continue
                try:
                    status = int(cols[4])
                except ValueError:
                    continue
                if status not in (2, 3):             # 1: prefix of longer words only; 4/5: char classes
                    continue
                nat = cls._natures(cols[5])
                if nat is None:
                    continue
                best = max(nat.items(), key=lambda kv: kv[1])[0]
                d.add(cols[1], sum(nat.values()), best)
        return d

    def load_user_library(self, text, default_freq=1000):
        """ansj userLibrary lines: ``word``, ``word TAB nature`` or ``word TAB nature TAB freq`` (user words win ties
        against core words through their default frequency)."""
        for line in text.splitlines():
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            cols = line.split("\t") if "\t" in line else line.split()
            word = cols[0]
            nature = cols[1] if len(cols) > 1 else "userDefine"
            freq = int(cols[2]) if len(cols) > 2 and cols[2].lstrip("-").isdigit() else default_freq
            self.add(word, freq, nature)
        return self

    @classmethod
    def from_user_library(cls, text, default_freq=1000):
        return cls().load_user_library(text, default_freq)


# closed-class words: enough for particles / pronouns / conjunctions / measure words to come out as words without a
# dictionary file (frequencies are coarse ranks, not corpus counts)
_BUILTIN = {
    "u": "的 了 着 过 得 地 之 所",
    "r": "我 你 他 她 它 我们 你们 他们 她们 它们 自己 这 那 这个 那个 这些 那些 这里 那里 什么 怎么 哪里 谁 咱们 大家",
    "c": "和 与 或 或者 但 但是 而 而且 因为 所以 如果 虽然 然后 并且 还是 以及 及 跟 同",
    "p": "在 从 向 对 把 被 给 为 为了 比 让 关于 按照 通过 根据 由于 除了",
    "d": "不 没 没有 很 也 都 就 才 又 再 还 更 最 太 已经 正在 曾经 非常 只 一起 一直",
    "q": "个 些 种 次 件 本 条 张 位 年 月 日 天",
    "m": "一 二 三 四 五 六 七 八 九 十 百 千 万 亿 两 几",
    "v": "是 有 说 要 会 能 可以 去 来 到 做 看 想 知道 觉得",
    "y": "吗 呢 吧 啊 呀",
}


def builtin_dictionary():
    d = CoreDictionary()
    for rank, (nat, words) in enumerate(_BUILTIN.items()):
        for w in words.split():
            d.add(w, 1000 - rank, nat)
    return d


def _kind(ch):
    if "一" <= ch <= "鿿" or "㐀" <= ch <= "䶿" or "豈" <= ch <= "﫿":
        return "han"
    if ch.isdigit():
        return "digit"
    if ch.isalpha():
        return "latin"
    if ch.isspace():
        return "space"
    return "punct"


class Segmenter:
    """Maximum-probability segmentation over a CoreDictionary (plus optional user dictionary, consulted first)."""

    def __init__(self, dictionary=None, userDictionary=None):
        if dictionary is None:
            p = os.environ.get("DL4J_AMD_ZH_DICT")
            dictionary = CoreDictionary.from_ansj_core(p) if p else builtin_dictionary()
        self.dic = dictionary
        self.user = userDictionary

    def _lookup(self, w):
        if self.user is not None and w in self.user:        # user words scored on the core dictionary's scale
            f, nat = self.user.words[w]
            return math.log((f + 1.0) / (self.dic.total + len(self.dic.words) + 1.0)), nat
        if w in self.dic:
            return self.dic.logp(w), self.dic.nature(w)
        return None

    def _han(self, run, base):
        n = len(run)
        max_len = max(self.dic.max_len, self.user.max_len if self.user is not None else 1)
        unk = self.dic.logp("\x00") - 4.0                # an out-of-dictionary character costs more than any word
        best = [0.0] * (n + 1)
        nxt = [n] * (n + 1)
        nat = [None] * (n + 1)
        for i in range(n - 1, -1, -1):
            b, bj, bn = -math.inf, i + 1, "nw"
            for j in range(i + 1, min(n, i + max_len) + 1):
                hit = self._lookup(run[i:j])
                if hit is None:
                    if j == i + 1:
                        hit = (unk, "nw")
                    else:
                        continue
                s = hit[0] + best[j]
                if s > b:
                    b, bj, bn = s, j, hit[1]
            best[i], nxt[i], nat[i] = b, bj, bn
        out, i = [], 0
        while i < n:
            out.append(Term(run[i:nxt[i]], nat[i], base + i))
            i = nxt[i]
        return out

    def terms(self, text):
        text = unicodedata.normalize("NFKC", text)
        out, i, n = [], 0, len(text)
        while i < n:
            k = _kind(text[i])
            j = i + 1
            if k == "han":
                while j < n and _kind(text[j]) == "han":
                    j += 1
                out.extend(self._han(text[i:j], i))
            elif k == "digit":
                while j < n and (_kind(text[j]) == "digit" or (text[j] in ".," and j + 1 < n
                                                               and _kind(text[j + 1]) == "digit")):
                    j += 1
                out.append(Term(text[i:j], "m", i))
            elif k == "latin":
                while j < n and _kind(text[j]) in ("latin", "digit"):
                    j += 1
                out.append(Term(text[i:j], "en", i))
            elif k == "punct":
                out.append(Term(text[i], "w", i))
            i = j
        return out

    def segment(self, text):
        return [t.name for t in self.terms(text)]
