"""Chinese tokenizer (reference deeplearning4j-nlp-chinese ChineseTokenizerTest.testChineseTokenizer: the sentence
"青山绿水和伟大的科学家让世界更美好和平" segments into exactly the reference's ten words when the reference's own ansj core
dictionary is loaded). Without the reference tree the dictionary-backed cases skip; the rest run on the built-in
dictionary."""
import os

import pytest

from deeplearning4j_amd.nlp import chinese as Z
from deeplearning4j_amd.nlp.tokenization_ext import ChineseTokenizerFactory
from _ref_fixtures import path as _ref_path

CORE = _ref_path("deeplearning4j-nlp-parent/deeplearning4j-nlp-chinese/src/main/resources/core.dic")
need_core = pytest.mark.skipif(not os.path.exists(CORE), reason="reference core.dic not present")


@pytest.fixture(scope="module")
def core_factory():
    return ChineseTokenizerFactory(CORE)


@need_core
def test_reference_sentence(core_factory):
    text = "青山绿水和伟大的科学家让世界更美好和平"
    expect = ["青山绿水", "和", "伟大", "的", "科学家", "让", "世界", "更", "美好", "和平"]
    tok = core_factory.create(text)
    assert tok.countTokens() == len(expect)
    assert [tok.nextToken() for _ in range(len(expect))] == expect


@need_core
def test_terms_natures_numbers_latin(core_factory):
    terms = core_factory.terms("2017年我在北京大学学习计算机科学，价格3,999.50元。GPU是MI355X")
    names = [t.getName() for t in terms]
    assert names == ["2017", "年", "我", "在", "北京大学", "学习", "计算机", "科学", ",",
                     "价格", "3,999.50", "元", "。", "GPU", "是", "MI355X"]
    nat = {t.getName(): t.getNatureStr() for t in terms}
    assert nat["2017"] == "m" and nat["GPU"] == "en" and nat["。"] == "w"
    assert nat["学习"].startswith("v") and nat["计算机"].startswith("n")
    # offsets index the NFKC-normalized text; the full-width comma normalizes to ","
    assert terms[4].getOffe() == 7


@need_core
def test_user_dictionary_word_wins(core_factory):
    text = "我们研究深度学习框架的性能"
    base = core_factory.segment(text)
    assert "深度学习框架" not in base
    f = ChineseTokenizerFactory(core_factory.segmenter.dic, userDictionary="深度学习框架\tn\t1000\n")
    seg = f.segment(text)
    assert "深度学习框架" in seg
    assert "".join(seg) == text
    assert {t.getName(): t.getNatureStr() for t in f.terms(text)}["深度学习框架"] == "n"


def test_builtin_dictionary_closed_class_words():
    f = ChineseTokenizerFactory()
    seg = f.segment("我们和他们在这里")
    assert seg == ["我们", "和", "他们", "在", "这里"]
    # unknown Han characters come out one per token, never dropped
    seg = f.segment("我们研究算法")
    assert seg[0] == "我们" and "".join(seg) == "我们研究算法"


def test_dictionary_scoring_prefers_probable_path():
    d = Z.CoreDictionary()
    for w, fr in [("研究", 50), ("研究生", 20), ("生命", 40), ("命", 5), ("起源", 30), ("生", 5)]:
        d.add(w, fr, "n")
    seg = Z.Segmenter(d).segment("研究生命起源")
    assert seg == ["研究", "生命", "起源"]
    d.add("研究生", 5000, "n")
    d.add("命起", 3000, "n")
    assert Z.Segmenter(d).segment("研究生命起源")[0] == "研究生"


def test_user_library_parser_and_fullwidth():
    d = Z.CoreDictionary.from_user_library("# comment\n机器学习\tn\t300\n深度\ta\n")
    assert d.words["机器学习"] == (300, "n") and d.words["深度"][1] == "a"
    seg = Z.Segmenter(Z.builtin_dictionary(), d).segment("ＡＢＣ１２３机器学习")
    assert seg == ["ABC123", "机器学习"]


# ------------------------------------------------------------------------------------------------ Korean
def test_korean_reference_sentence_with_noun_dictionary():
    """reference KoreanTokenizerTest: with twitter-korean-text's nouns (딥 and 러닝 are separate dictionary nouns there)
    the sentence splits exactly as the reference expects; without them the unknown compound stays whole."""
    from deeplearning4j_amd.nlp.korean import KoreanDictionary
    from deeplearning4j_amd.nlp.tokenization_ext import KoreanTokenizerFactory
    text = "세계 최초의 상용 수준 오픈소스 딥러닝 라이브러리입니다"
    expect = ["세계", "최초", "의", "상용", "수준", "오픈소스", "딥", "러닝", "라이브러리", "입니", "다"]
    d = KoreanDictionary.builtin()
    for w in ("최초", "상용", "수준", "오픈소스", "딥", "러닝", "라이브러리"):
        d.add(w)
    tok = KoreanTokenizerFactory(d).create(text)
    assert tok.countTokens() == len(expect)
    assert [tok.nextToken() for _ in range(len(expect))] == expect
    plain = KoreanTokenizerFactory().segment(text)
    assert plain == ["세계", "최초", "의", "상용", "수준", "오픈소스", "딥러닝", "라이브러리", "입니", "다"]


def test_korean_pos_and_mixed_script():
    from deeplearning4j_amd.nlp.tokenization_ext import KoreanTokenizerFactory
    toks = KoreanTokenizerFactory().tokens("우리는 GPU 8개로 학습했다.")
    assert [(t.getText(), t.getPos()) for t in toks] == [
        ("우리", "Noun"), ("는", "Josa"), ("GPU", "Alpha"), ("8", "Number"), ("개", "Noun"), ("로", "Josa"),
        ("학습", "Noun"), ("했", "Verb"), ("다", "Eomi"), (".", "Punctuation")]
    assert KoreanTokenizerFactory().segment("나는 학교에 갑니다") == ["나", "는", "학교", "에", "갑니다"]
