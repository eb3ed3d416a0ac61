"""Language-specific tokenizers and pre-processors (SURVEY §2.9 "Tokenizers": deeplearning4j-nlp-uima
StemmingPreprocessor / PoS tokenizers, deeplearning4j-nlp-japanese (Kuromoji), -chinese (ansj), -korean), plus a
BERT WordPiece tokenizer for the transformer path.

Japanese: the lattice / Viterbi morphological analyser of ``nlp/kuromoji.py`` (Kuromoji's algorithm; MeCab/IPADIC
dictionaries load from their source files, a small built-in lexicon otherwise).
* Chinese: maximum-probability word lattice over an ansj core dictionary (``nlp/chinese.py``; core.dic read from its
  file, a built-in closed-class dictionary otherwise).
* Korean: eojeol decomposition into nouns, josa, predicate stems and endings (``nlp/korean.py``).
The Porter stemmer (English) is the algorithm behind the UIMA module's StemmingPreprocessor.
"""
import os
import re
import unicodedata

from .text import TokenPreProcess, Tokenizer, TokenizerFactory


# ------------------------------------------------------------------------------------------------ Porter stemmer
class PorterStemmer:
    """M. F. Porter, "An algorithm for suffix stripping" (1980)."""

    _V = "aeiou"

    def _cons(self, w, i):
        c = w[i]
        if c in self._V:
            return False
        if c == "y":
            return i == 0 or not self._cons(w, i - 1)
        return True

    def _m(self, stem):
        n, i, L = 0, 0, len(stem)
        while i < L and self._cons(stem, i):
            i += 1
        while i < L:
            while i < L and not self._cons(stem, i):
                i += 1
            if i >= L:
                break
            n += 1
            while i < L and self._cons(stem, i):
                i += 1
        return n

    def _has_vowel(self, stem):
        return any(not self._cons(stem, i) for i in range(len(stem)))

    def _double_c(self, w):
        return len(w) >= 2 and w[-1] == w[-2] and self._cons(w, len(w) - 1)

    def _cvc(self, w):
        if len(w) < 3:
            return False
        return (self._cons(w, len(w) - 3) and not self._cons(w, len(w) - 2) and self._cons(w, len(w) - 1)
                and w[-1] not in "wxy")

    def _replace(self, w, suffixes, cond):
        for suf, rep in suffixes:
            if w.endswith(suf):
                stem = w[:len(w) - len(suf)]
                return (stem + rep) if cond(stem) else w
        return w

    def stem(self, w):
        w = w.lower()
        if len(w) <= 2:
            return w
        # step 1a
        if w.endswith("sses"):
            w = w[:-2]
        elif w.endswith("ies"):
            w = w[:-2]
        elif w.endswith("ss"):
            pass
        elif w.endswith("s"):
            w = w[:-1]
        # step 1b
        flag = False
        if w.endswith("eed"):
            if self._m(w[:-3]) > 0:
                w = w[:-1]
        elif w.endswith("ed") and self._has_vowel(w[:-2]):
            w, flag = w[:-2], True
        elif w.endswith("ing") and self._has_vowel(w[:-3]):
            w, flag = w[:-3], True
        if flag:
            if w.endswith(("at", "bl", "iz")):
                w += "e"
            elif self._double_c(w) and w[-1] not in "lsz":
                w = w[:-1]
            elif self._m(w) == 1 and self._cvc(w):
                w += "e"
        # step 1c
        if w.endswith("y") and self._has_vowel(w[:-1]):
            w = w[:-1] + "i"
        # step 2
        w = self._replace(w, [("ational", "ate"), ("tional", "tion"), ("enci", "ence"), ("anci", "ance"),
                              ("izer", "ize"), ("abli", "able"), ("alli", "al"), ("entli", "ent"), ("eli", "e"),
                              ("ousli", "ous"), ("ization", "ize"), ("ation", "ate"), ("ator", "ate"),
                              ("alism", "al"), ("iveness", "ive"), ("fulness", "ful"), ("ousness", "ous"),
                              ("aliti", "al"), ("iviti", "ive"), ("biliti", "ble")], lambda s: self._m(s) > 0)
        # step 3
        w = self._replace(w, [("icate", "ic"), ("ative", ""), ("alize", "al"), ("iciti", "ic"), ("ical", "ic"),
                              ("ful", ""), ("ness", "")], lambda s: self._m(s) > 0)
        # step 4
        for suf in ("al", "ance", "ence", "er", "ic", "able", "ible", "ant", "ement", "ment", "ent", "ion", "ou",
                    "ism", "ate", "iti", "ous", "ive", "ize"):
            if w.endswith(suf):
                stem = w[:len(w) - len(suf)]
                if self._m(stem) > 1 and (suf != "ion" or stem.endswith(("s", "t"))):
                    w = stem
                break
        # step 5
        if w.endswith("e"):
            stem = w[:-1]
            if self._m(stem) > 1 or (self._m(stem) == 1 and not self._cvc(stem)):
                w = stem
        if self._m(w) > 1 and self._double_c(w) and w.endswith("l"):
            w = w[:-1]
        return w


class StemmingPreprocessor(TokenPreProcess):
    """CommonPreprocessor-style cleaning (lower case, strip punctuation/digits) followed by Porter stemming."""

    _strip = re.compile(r"[\d\.:,\"'\(\)\[\]|/?!;]+")

    def __init__(self):
        self.stemmer = PorterStemmer()

    def preProcess(self, token):
        t = self._strip.sub("", token.lower())
        return self.stemmer.stem(t) if t else t


# ------------------------------------------------------------------------------------------------ CJK / Korean
def _script(ch):
    o = ord(ch)
    if 0x3040 <= o <= 0x309F:
        return "hira"
    if 0x30A0 <= o <= 0x30FF or 0x31F0 <= o <= 0x31FF:
        return "kata"
    if 0x4E00 <= o <= 0x9FFF or 0x3400 <= o <= 0x4DBF or 0xF900 <= o <= 0xFAFF:
        return "han"
    if 0xAC00 <= o <= 0xD7AF:
        return "hangul"
    if ch.isdigit():
        return "digit"
    if ch.isalpha():
        return "latin"
    if ch.isspace():
        return "space"
    return "punct"


class _SegmentingFactory(TokenizerFactory):
    def segment(self, text):
        raise NotImplementedError

    def create(self, text):
        if hasattr(text, "read"):
            text = text.read()
            if isinstance(text, bytes):
                text = text.decode("utf-8")
        return Tokenizer(self.segment(text), self.pre)


class JapaneseTokenizerFactory(_SegmentingFactory):
    """Morphological analysis on the lattice / Viterbi analyser of ``nlp/kuromoji.py`` (reference
    deeplearning4j-nlp-japanese JapaneseTokenizerFactory / JapaneseTokenizer, Kuromoji IPADIC tokenizer).

    useBaseForm: emit each token's dictionary form (``驚い`` -> ``驚く``). lexicon: a ``kuromoji.Lexicon`` (default:
    the MeCab/IPADIC directory named by ``DL4J_AMD_JA_DICT`` when set, else the small built-in lexicon).
    userDictionary: a ``kuromoji.UserDictionary`` or its text. mode: ``kuromoji.Mode.NORMAL`` / ``SEARCH``."""

    def __init__(self, useBaseForm=False, lexicon=None, userDictionary=None, mode="NORMAL"):
        super().__init__()
        from . import kuromoji as K
        if lexicon is None:
            d = os.environ.get("DL4J_AMD_JA_DICT")
            lexicon = K.Lexicon.from_mecab_dir(d) if d else K.builtin_lexicon()
        if isinstance(userDictionary, str):
            userDictionary = K.UserDictionary.parse(userDictionary)
        self.useBaseForm = useBaseForm
        self.analyzer = K.LatticeTokenizer(lexicon, userDictionary, mode)

    def tokens(self, text):
        """The analyser's Token objects (surface, features, base form, reading)."""
        return self.analyzer.tokenize(text)

    def segment(self, text):
        out = []
        for t in self.analyzer.tokenize(text):
            if t.surface.isspace():
                continue
            out.append(t.getBaseForm() if self.useBaseForm else t.surface)
        return out


class ChineseTokenizerFactory(_SegmentingFactory):
    """Maximum-probability word segmentation over a word dictionary (``nlp/chinese.py``; reference
    deeplearning4j-nlp-chinese ChineseTokenizerFactory / ChineseTokenizer over ansj ToAnalysis).

    dictionary: a ``chinese.CoreDictionary`` or a path to an ansj ``core.dic`` (default: ``DL4J_AMD_ZH_DICT`` when
    set, else the small built-in closed-class dictionary). userDictionary: a ``CoreDictionary`` or userLibrary text
    (``word TAB nature TAB freq`` lines)."""

    def __init__(self, dictionary=None, userDictionary=None):
        super().__init__()
        from . import chinese as Z
        if isinstance(dictionary, str):
            dictionary = Z.CoreDictionary.from_ansj_core(dictionary)
        if isinstance(userDictionary, str):
            userDictionary = Z.CoreDictionary.from_user_library(userDictionary)
        self.segmenter = Z.Segmenter(dictionary, userDictionary)

    def terms(self, text):
        """Segmented words with their natures (ansj Term)."""
        return self.segmenter.terms(text)

    def segment(self, text):
        return self.segmenter.segment(text)


class KoreanTokenizerFactory(_SegmentingFactory):
    """Eojeol decomposition into nouns, josa, predicate stems and endings (``nlp/korean.py``; reference
    deeplearning4j-nlp-korean KoreanTokenizerFactory over twitter-korean-text). dictionary: a
    ``korean.KoreanDictionary``, a path to a noun list, or an iterable of nouns (default: ``DL4J_AMD_KO_DICT`` when
    set, else the built-in pronoun / bound-noun set)."""

    def __init__(self, dictionary=None):
        super().__init__()
        from . import korean as K
        if isinstance(dictionary, str):
            dictionary = K.KoreanDictionary.from_file(dictionary)
        elif dictionary is not None and not isinstance(dictionary, K.KoreanDictionary):
            dictionary = K.KoreanDictionary(dictionary)
        self.analyzer = K.KoreanAnalyzer(dictionary)

    def tokens(self, text):
        return self.analyzer.tokenize(text)

    def segment(self, text):
        return [t.text for t in self.analyzer.tokenize(text) if t.pos != "Punctuation"]


# ------------------------------------------------------------------------------------------------ BERT WordPiece
class BertWordPieceTokenizerFactory(_SegmentingFactory):
    """BERT basic tokenization (lower-casing, accent stripping, punctuation split, CJK chars as words) followed by
    greedy longest-match-first WordPiece over ``vocab`` (dict token -> id, or a vocab.txt path)."""

    def __init__(self, vocab, lowerCase=True, unk="[UNK]", maxCharsPerWord=100):
        super().__init__()
        if isinstance(vocab, str):
            with open(vocab, encoding="utf-8") as fh:
                vocab = {line.rstrip("\n"): i for i, line in enumerate(fh)}
        self.vocab = dict(vocab)
        self.lowerCase = lowerCase
        self.unk = unk
        self.maxChars = maxCharsPerWord

    def _basic(self, text):
        text = unicodedata.normalize("NFC", text)
        if self.lowerCase:
            text = "".join(c for c in unicodedata.normalize("NFD", text.lower()) if unicodedata.category(c) != "Mn")
        out, cur = [], ""
        for ch in text:
            cat = unicodedata.category(ch)
            if ch.isspace():
                if cur:
                    out.append(cur)
                cur = ""
            elif cat.startswith("P") or (33 <= ord(ch) <= 47) or (58 <= ord(ch) <= 64) or (91 <= ord(ch) <= 96) or \
                    (123 <= ord(ch) <= 126) or _script(ch) == "han":
                if cur:
                    out.append(cur)
                cur = ""
                out.append(ch)
            elif cat in ("Cc", "Cf"):
                continue
            else:
                cur += ch
        if cur:
            out.append(cur)
        return out

    def _wordpiece(self, word):
        if len(word) > self.maxChars:
            return [self.unk]
        pieces, start = [], 0
        while start < len(word):
            end, found = len(word), None
            while start < end:
                sub = word[start:end] if start == 0 else "##" + word[start:end]
                if sub in self.vocab:
                    found = sub
                    break
                end -= 1
            if found is None:
                return [self.unk]
            pieces.append(found)
            start = end
        return pieces

    def segment(self, text):
        return [p for w in self._basic(text) for p in self._wordpiece(w)]

    def encode(self, text, maxLength=None, addSpecial=True):
        ids = [self.vocab.get(t, self.vocab.get(self.unk, 0)) for t in self.segment(text)]
        if addSpecial:
            cls, sep = self.vocab.get("[CLS]"), self.vocab.get("[SEP]")
            if cls is not None and sep is not None:
                ids = [cls] + ids + [sep]
        if maxLength is not None:
            ids = ids[:maxLength]
        return ids
