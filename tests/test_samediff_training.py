"""SameDiff graphs recorded at definition time: replay for new placeholder values (``output``) and training with a
TrainingConfig (``fit``: the reverse pass over the recorded ops + the fused updater), incl. the LSTM layer op."""
import torch

from deeplearning4j_amd import Adam, DataSet
from deeplearning4j_amd.samediff import SameDiff, TrainingConfig


def _linear_graph():
    sd = SameDiff.create()
    x = sd.placeHolder("x", torch.zeros(4, 3))
    y = sd.placeHolder("y", torch.zeros(4, 2))
    w = sd.var("w", torch.randn(3, 2, generator=torch.Generator().manual_seed(1)) * 0.1)
    b = sd.var("b", torch.zeros(2))
    z = sd.nn().linear("z", x, w, b)
    sd.loss().meanSquaredError("loss", y, z)
    return sd


def test_output_replays_for_new_placeholders():
    sd = _linear_graph()
    X = torch.randn(7, 3)
    got = sd.output({"x": X}, "z")["z"]
    w, b = sd.getVariable("w").value, sd.getVariable("b").value
    assert torch.allclose(got, X @ w + b)


def test_fit_linear_regression_converges():
    sd = _linear_graph()
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(0.05)).dataSetFeatureMapping("x")
                         .dataSetLabelMapping("y").build())
    g = torch.Generator().manual_seed(0)
    X = torch.randn(64, 3, generator=g)
    Y = X @ torch.tensor([[1.0, -1.0], [0.5, 2.0], [0.0, 1.0]])
    first = sd.fit(DataSet(X, Y))
    for _ in range(200):
        last = sd.fit(DataSet(X, Y))
    assert last < 1e-3 * first
    assert sd.iterationCount == 201


def test_samediff_lstm_char_model_trains_cpu():
    mb, nIn, T, H, nOut = 4, 6, 5, 8, 6
    g = torch.Generator().manual_seed(2)
    sd = SameDiff.create()
    x = sd.placeHolder("x", torch.zeros(mb, nIn, T))
    y = sd.placeHolder("y", torch.zeros(mb, T, nOut))
    W = sd.var("W", torch.randn(nIn, 4 * H, generator=g) * 0.3)
    RW = sd.var("RW", torch.randn(H, 4 * H + 3, generator=g) * 0.1)
    b = sd.var("b", torch.zeros(4 * H))
    Wo = sd.var("Wo", torch.randn(H, nOut, generator=g) * 0.3)
    h = sd.rnn().lstmLayer("h", x, W, RW, b, peephole=True)
    logits = sd.mmul("logits", h.permute(0, 2, 1), Wo)
    sd.loss().softmaxCrossEntropy("loss", y, logits)
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(0.03)).dataSetFeatureMapping("x")
                         .dataSetLabelMapping("y").build())
    idx = torch.randint(0, nOut, (mb, T + 1), generator=g)
    X = torch.nn.functional.one_hot(idx[:, :-1], nIn).permute(0, 2, 1).float()
    Y = torch.nn.functional.one_hot(idx[:, 1:], nOut).float()
    losses = [sd.fit(DataSet(X, Y)) for _ in range(60)]
    assert losses[-1] < 0.5 * losses[0]


def test_bert_samediff_import_matches_transformers():
    """BERT imported as a SameDiff graph == HuggingFace BertForSequenceClassification (random init, no download),
    then one SameDiff fit step lowers the loss on the same batch."""
    import pytest
    transformers = pytest.importorskip("transformers")
    from deeplearning4j_amd.modelimport.bert import importBertSameDiff
    cfg = transformers.BertConfig(vocab_size=60, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                                  intermediate_size=48, max_position_embeddings=24, num_labels=3)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(cfg).eval()
    sd = importBertSameDiff(hf.state_dict(), cfg.to_dict(), seqLen=10)
    gen = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 60, (4, 10), generator=gen)
    am = torch.ones(4, 10, dtype=torch.long)
    am[1, 7:] = 0
    am[3, 4:] = 0
    with torch.no_grad():
        ref = torch.softmax(hf(input_ids=ids, attention_mask=am).logits, dim=-1)
    got = sd.output({"input_ids": ids, "attention_mask": am.float()}, "probabilities")["probabilities"]
    assert torch.allclose(got, ref, atol=2e-5), (got - ref).abs().max()
    from deeplearning4j_amd import Adam, MultiDataSet
    sd.setTrainingConfig(TrainingConfig.builder().updater(Adam(1e-3)).dataSetFeatureMapping("input_ids",
                                                                                            "attention_mask")
                         .dataSetLabelMapping("labels").build())
    y = torch.nn.functional.one_hot(torch.tensor([0, 1, 2, 1]), 3).float()
    mds = MultiDataSet([ids, am.float()], [y])
    l0 = sd.fit(mds)
    for _ in range(5):
        l1 = sd.fit(mds)
    assert l1 < l0
