"""Korean morphological segmentation (reference deeplearning4j-nlp-korean KoreanTokenizer over twitter-korean-text's
TwitterKoreanProcessor.tokenize: nouns split out of compounds, josa (postpositions) and predicate endings as tokens
of their own, e.g. ``최초의`` -> ``최초 의``, ``라이브러리입니다`` -> ``라이브러리 입니 다``).

Each whitespace-separated eojeol is decomposed by dynamic programming over a small grammar:

    eojeol := stem+ [josa]  |  stem* predicate eomi

stem edges are dictionary nouns (cost -log p) or an unknown Hangul chunk (a fixed cost plus a per-syllable cost, so
unknown material stays in one piece unless dictionary words explain it better); josa, predicate stems (copula /
ha-da / doe-da forms) and eomi come from closed lists. Non-Hangul runs (latin, digits) are tokens; punctuation comes
out as Punctuation tokens, which the TokenizerFactory's word list leaves out.

The noun dictionary is data: ``KoreanDictionary.from_file(path)`` (one noun per line, optional TAB frequency) or
``DL4J_AMD_KO_DICT``; a small built-in set of pronouns / bound nouns works without one. twitter-korean-text's own
dictionary is not in the reference tree, so token-for-token parity with it is unpinned.
"""
import math
import os
import unicodedata

__all__ = ["KoreanDictionary", "KoreanAnalyzer", "KoreanToken"]

JOSA = ("으로써", "으로서", "에게서", "한테서", "으로", "에서", "에게", "한테", "까지", "부터", "보다", "처럼", "마다", "조차",
        "은", "는", "이", "가", "을", "를", "에", "의", "도", "로", "와", "과", "만", "랑", "께")
PREDICATE = ("입니", "이었", "이에", "였", "합니", "했", "하", "됩니", "되었", "됐", "습니", "있습니", "없습니")
_COPULA = ("입니", "이었", "이에", "였")
EOMI = ("습니다", "니다", "다", "요", "까", "고", "며", "면", "서", "지만", "는데")

_BUILTIN_NOUNS = ("나 너 저 우리 저희 그 그녀 이것 그것 저것 여기 거기 저기 것 수 때 곳 등 중 년 월 일 사람 오늘 내일 어제 "
                  "지금 학교 회사 집 문제 세계")


class KoreanToken:
    __slots__ = ("text", "pos", "offset")

    def __init__(self, text, pos, offset):
        self.text, self.pos, self.offset = text, pos, offset

    def getText(self):
        return self.text

    def getPos(self):
        return self.pos

    def __repr__(self):
        return f"{self.text}/{self.pos}"


class KoreanDictionary:
    def __init__(self, words=None):
        self.freq = {}
        self.total = 0
        self.max_len = 1
        for w in words or ():
            self.add(w)

    def add(self, word, freq=100):
        if word:
            self.total += int(freq) - self.freq.get(word, 0)
            self.freq[word] = int(freq)
            self.max_len = max(self.max_len, len(word))

    def __contains__(self, w):
        return w in self.freq

    def cost(self, w):
        return -math.log((self.freq[w] + 1.0) / (self.total + len(self.freq) + 1.0))

    @classmethod
    def from_file(cls, path):
        d = cls()
        with open(path, encoding="utf-8") as fh:
            for line in fh:
                cols = line.strip().split("\t")
                if cols and cols[0] and not cols[0].startswith("#"):
                    d.add(cols[0], int(cols[1]) if len(cols) > 1 and cols[1].isdigit() else 100)
        return d

    @classmethod
    def builtin(cls):
        return cls(_BUILTIN_NOUNS.split())


def _hangul(ch):
    return "가" <= ch <= "힣" or "ᄀ" <= ch <= "ᇿ" or "㄰" <= ch <= "㆏"


_JOSA_COST, _PRED_COST, _EOMI_COST = 1.0, 1.0, 0.5


class KoreanAnalyzer:
    def __init__(self, dictionary=None, unknown_base=14.0, unknown_per_char=1.5):
        if dictionary is None:
            p = os.environ.get("DL4J_AMD_KO_DICT")
            dictionary = KoreanDictionary.from_file(p) if p else KoreanDictionary.builtin()
        self.dic = dictionary
        self.ub, self.up = unknown_base, unknown_per_char

    def _eojeol(self, w, base):
        """Best decomposition of one Hangul word. State after position j: 0 = stems so far (josa / predicate may
        follow), 1 = after a predicate stem (only eomi may follow), 2 = closed (josa or eomi consumed)."""
        n = len(w)
        INF = math.inf
        best = [[INF] * 3 for _ in range(n + 1)]
        back = [[None] * 3 for _ in range(n + 1)]
        best[0][0] = 0.0
        for i in range(n):
            for st in range(3):
                c0 = best[i][st]
                if c0 == INF:
                    continue
                if st == 0:
                    for j in range(i + 1, n + 1):
                        piece = w[i:j]
                        if piece in self.dic:
                            self._relax(best, back, j, 0, c0 + self.dic.cost(piece), i, st, piece, "Noun")
                        self._relax(best, back, j, 0, c0 + self.ub + self.up * (j - i), i, st, piece, "Noun*")
                    if i > 0:
                        for s in JOSA:
                            if w.startswith(s, i) and i + len(s) == n:
                                self._relax(best, back, n, 2, c0 + _JOSA_COST, i, st, s, "Josa")
                    for s in PREDICATE:
                        if w.startswith(s, i):
                            pos = "Adjective" if s in _COPULA else "Verb"
                            self._relax(best, back, i + len(s), 1, c0 + _PRED_COST, i, st, s, pos)
                elif st == 1:
                    for s in EOMI:
                        if w.startswith(s, i) and i + len(s) == n:
                            self._relax(best, back, n, 2, c0 + _EOMI_COST, i, st, s, "Eomi")
        end = min((best[n][s], s) for s in (0, 2))
        if end[0] == INF:
            return [KoreanToken(w, "Noun*", base)]
        out, j, st = [], n, end[1]
        while j > 0:
            i, pst, piece, pos = back[j][st]
            out.append(KoreanToken(piece, "Noun" if pos == "Noun*" else pos, base + i))
            j, st = i, pst
        return out[::-1]

    @staticmethod
    def _relax(best, back, j, st, c, i, pst, piece, pos):
        if c < best[j][st]:
            best[j][st] = c
            back[j][st] = (i, pst, piece, pos)

    def tokenize(self, text):
        text = unicodedata.normalize("NFC", text)
        out, i, n = [], 0, len(text)
        while i < n:
            ch = text[i]
            j = i + 1
            if _hangul(ch):
                while j < n and _hangul(text[j]):
                    j += 1
                out.extend(self._eojeol(text[i:j], i))
            elif ch.isalnum():
                while j < n and text[j].isalnum() and not _hangul(text[j]):
                    j += 1
                out.append(KoreanToken(text[i:j], "Number" if text[i:j].isdigit() else "Alpha", i))
            elif not ch.isspace():
                out.append(KoreanToken(ch, "Punctuation", i))
            i = j
        return out
