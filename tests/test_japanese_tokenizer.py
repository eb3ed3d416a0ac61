"""Japanese morphological analysis (reference deeplearning4j-nlp-japanese: JapaneseTokenizerTest.java, Kuromoji's
UserDictionaryTokenizerTest / TokenizerTest). The IPADIC dictionary is not in this image: the lattice analyser is
checked with a lexicon + connection costs estimated from the reference's own tokenized test corpus
(bocchan-ipadic-features.txt, the expected Kuromoji/IPADIC output for bocchan.txt) and evaluated on a HELD-OUT corpus
(jawikisentences-ipadic-features.txt, produced with the reference's userdict.txt). Exact IPADIC parity is unpinned."""
import os

import pytest

from deeplearning4j_amd.nlp import kuromoji as K
from deeplearning4j_amd.nlp.tokenization_ext import JapaneseTokenizerFactory
from _ref_fixtures import path as _ref_path

RES = _ref_path("deeplearning4j-nlp-parent/deeplearning4j-nlp-japanese/src/test/resources")
need_res = pytest.mark.skipif(not os.path.isdir(RES), reason="reference Kuromoji test resources not present")


@pytest.fixture(scope="module")
def trained():
    with open(os.path.join(RES, "bocchan-ipadic-features.txt"), encoding="utf-8") as fh:
        lines = fh.read().splitlines()
    with open(os.path.join(RES, "char.def"), "rb") as fh:
        cd = K.CharacterDefinitions.parse(fh.read().decode("euc-jp", errors="replace"))
    with open(os.path.join(RES, "unk.def"), "rb") as fh:
        unk = fh.read().decode("euc-jp", errors="replace")
    return K.Lexicon.from_features_corpus(lines, cd, unk)


def _gold(path):
    toks = []
    with open(path, encoding="utf-8") as fh:
        for line in fh.read().splitlines():
            if "\t" in line:
                s, f = line.split("\t", 1)
                toks.append((s, f))
    return toks


def _spans(surfaces):
    out, p = set(), 0
    for s in surfaces:
        out.add((p, p + len(s)))
        p += len(s)
    return out


def test_char_def_and_unknown_words():
    cd = K.CharacterDefinitions()
    assert cd.category("漢") == "KANJI" and cd.category("カ") == "KATAKANA" and cd.category("a") == "ALPHA"
    assert cd.lookup("一")[0] == "KANJINUMERIC"
    tok = K.LatticeTokenizer(K.builtin_lexicon())
    out = [t.surface for t in tok.tokenize("私はコンピュータを使う")]
    assert out[:3] == ["私", "は", "コンピュータ"] and "を" in out       # katakana run grouped as one unknown word


def test_builtin_factory_api():
    tf = JapaneseTokenizerFactory()
    t = tf.create("これは本です。")
    toks = t.getTokens()
    assert toks[:2] == ["これ", "は"] and toks[-2:] == ["です", "。"]
    assert t.countTokens() == len(toks)


@need_res
def test_heldout_segmentation_and_tagging(trained):
    """Lexicon from bocchan, evaluated on the Wikipedia sentences: segmentation F1 and POS accuracy on matched tokens."""
    gold = _gold(os.path.join(RES, "jawikisentences-ipadic-features.txt"))
    with open(os.path.join(RES, "userdict.txt"), encoding="utf-8") as fh:
        user = K.UserDictionary.parse(fh.read())
    text = "".join(s for s, _ in gold)
    toks = K.LatticeTokenizer(trained, user).tokenize(text)
    assert "".join(t.surface for t in toks) == text
    g, p = _spans(s for s, _ in gold), _spans(t.surface for t in toks)
    tp = len(g & p)
    f1 = 2 * tp / (len(g) + len(p))
    gpos = {sp: f.split(",")[0] for sp, (_, f) in zip(sorted(g), gold)}
    ppos = {(t.position, t.position + len(t.surface)): t.getPartOfSpeechLevel1() for t in toks}
    acc = sum(gpos[s] == ppos[s] for s in g & p) / max(1, tp)
    print(f"held-out segmentation F1 {f1:.3f}, POS accuracy {acc:.3f} ({len(gold)} gold tokens)")
    assert f1 > 0.75 and acc > 0.8


@need_res
def test_user_dictionary_forces_segmentation(trained):
    """UserDictionaryTokenizerTest: a user entry's segmentation, readings and part of speech win."""
    with open(os.path.join(RES, "userdict.txt"), encoding="utf-8") as fh:
        user = K.UserDictionary.parse(fh.read())
    toks = K.LatticeTokenizer(trained, user).tokenize("関西国際空港に行った")
    assert [t.surface for t in toks[:3]] == ["関西", "国際", "空港"]
    assert toks[0].getPartOfSpeechLevel1() == "テスト名詞" and toks[0].getReading() == "カンサイ" and toks[0].isUser()
    toks = K.LatticeTokenizer(trained, user).tokenize("朝青龍")
    assert len(toks) == 1 and toks[0].getReading() == "アサショウリュウ"


@need_res
def test_reference_japanese_tokenizer_scenarios(trained):
    """JapaneseTokenizerTest: "黒い瞳の綺麗な女の子" and the base form of a conjugated verb ("驚いた" -> "驚く")."""
    tf = JapaneseTokenizerFactory(lexicon=trained)
    toks = tf.create("黒い瞳の綺麗な女の子").getTokens()
    print("tokens:", toks)
    assert toks[0] == "黒い" and "の" in toks and "な" in toks
    base = JapaneseTokenizerFactory(useBaseForm=True, lexicon=trained).create("驚いた彼は道を走っていった。")
    assert base.nextToken() == "驚く"


@need_res
def test_search_mode_decompounds(trained):
    """SEARCH mode's length penalty never produces longer kanji tokens than NORMAL mode."""
    text = "関西国際空港株式会社代表取締役社長"
    n = K.LatticeTokenizer(trained, mode=K.Mode.NORMAL).tokenize(text)
    s = K.LatticeTokenizer(trained, mode=K.Mode.SEARCH).tokenize(text)
    assert "".join(t.surface for t in s) == text
    assert max(len(t.surface) for t in s) <= max(len(t.surface) for t in n) and len(s) >= len(n)


def _search_cases():
    cases = []
    with open(os.path.join(RES, "search-segmentation-tests.txt"), encoding="utf-8") as fh:
        for line in fh.read().splitlines():
            if not line.strip() or line.startswith("#"):
                continue
            text, exp = line.split("\t")
            cases.append((text, exp.split(" ")))
    return cases


@need_res
def test_search_segmentation_fixture(trained):
    """Kuromoji's search-segmentation-tests.txt (45 decompounding cases). Its header says the expectations depend on
    IPADIC, which is not in this image: with the corpus-estimated lexicon the dictionary words the splits need
    (関西, 国際, ソフトウェア, ...) are unknown, so exact parity is UNPINNED. Pinned here: every case loads and
    tokenizes in SEARCH mode back to its text; SEARCH mode's penalties are in the lexicon's own cost units, so it
    does not break unknown katakana runs into arbitrary pieces (span F1 >= NORMAL's); and the measured span F1 does
    not regress (0.277 at the time of writing)."""
    cases = _search_cases()
    assert len(cases) == 45
    f1 = {}
    for mode in (K.Mode.NORMAL, K.Mode.SEARCH):
        tok = K.LatticeTokenizer(trained, mode=mode)
        tp = fp = fn = 0
        for text, exp in cases:
            got = [t.surface for t in tok.tokenize(text)]
            assert "".join(got) == text
            a, b = _spans(got), _spans(exp)
            tp, fp, fn = tp + len(a & b), fp + len(a - b), fn + len(b - a)
        p, r = tp / (tp + fp), tp / (tp + fn)
        f1[mode] = 2 * p * r / (p + r)
    print("search-segmentation span F1:", f1)
    assert f1[K.Mode.SEARCH] >= f1[K.Mode.NORMAL] - 1e-9
    assert f1[K.Mode.SEARCH] >= 0.27


def test_search_mode_heuristic_on_fixture_case():
    """The first fixture case with the dictionary words it needs (IPADIC-like costs, penalty scale 1): NORMAL keeps
    the cheap whole-word entry 関西国際空港, SEARCH's kanji-length penalty ((6 - 2) x 3000) splits it into
    関西 国際 空港 exactly as the fixture expects."""
    noun = 1
    feats = ["名詞", "固有名詞", "組織", "*", "*", "*", "*", "*", "*"]
    words = {"関西国際空港": 4000, "関西": 3000, "国際": 3000, "空港": 3000}
    es = [K.Entry(w, noun, noun, c, feats) for w, c in words.items()]
    lex = K.Lexicon(es, K.ConnectionCosts({(0, 1): 0, (1, 1): 0, (1, 0): 0}, 5000), K.CharacterDefinitions(),
                    {cat: [K.Entry(cat, noun, noun, 20000, feats, "unknown")] for cat in K._BUILTIN_CATEGORIES})
    normal = [t.surface for t in K.LatticeTokenizer(lex, mode=K.Mode.NORMAL).tokenize("関西国際空港")]
    search = [t.surface for t in K.LatticeTokenizer(lex, mode=K.Mode.SEARCH).tokenize("関西国際空港")]
    assert normal == ["関西国際空港"]
    assert search == ["関西", "国際", "空港"]
    if os.path.isdir(RES):
        assert _search_cases()[0] == ("関西国際空港", search)
