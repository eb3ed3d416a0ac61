"""Transformer layers (BERT config): fp64 gradient checks of the hand-written backward of the encoder block, the
embedding and pooler layers (masked and causal), and a tiny BertBase fit. Reference test strategy: gradient checks
for every layer type (NNT:gradientcheck/*)."""
import pytest
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd.gradientcheck import checkGradients
from deeplearning4j_amd.models import BertBase


def _graph(causal=False, T=6, V=11, E=16, H=4, F=24, layers=2, nl=3):
    g = (NeuralNetConfiguration.Builder().seed(7).dataType(DataType.DOUBLE).updater(NoOp())
         .weightInit(NormalDistribution(0.0, 0.5)).graphBuilder())
    g.addInputs("tokens")
    g.addLayer("emb", BertEmbeddingLayer.Builder().nIn(V).nOut(E).maxPositions(T + 2).inputLength(T).build(), "tokens")
    prev = "emb"
    for i in range(layers):
        g.addLayer(f"enc{i}", TransformerEncoderLayer.Builder().nIn(E).nOut(E).nHeads(H).ffnSize(F).causal(causal)
                   .build(), prev)
        prev = f"enc{i}"
    g.addLayer("pool", BertPoolerLayer.Builder().nIn(E).nOut(E).build(), prev)
    g.addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).activation(Activation.SOFTMAX).nIn(E).nOut(nl).build(),
               "pool")
    g.setOutputs("out")
    net = ComputationGraph(g.build())
    net.init(device="cpu")
    return net


def _data(B=3, T=6, V=11, nl=3, seed=0):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randint(0, V, (B, T), generator=gen)
    y = torch.zeros(B, nl, dtype=torch.float64)
    y[torch.arange(B), torch.randint(0, nl, (B,), generator=gen)] = 1
    return x, y


@pytest.mark.parametrize("causal", [False, True])
def test_transformer_block_gradients(causal):
    net = _graph(causal=causal)
    x, y = _data()
    assert checkGradients(net, input=[x], labels=[y], print_results=True, subset=400)


def test_transformer_block_gradients_with_padding_mask():
    net = _graph()
    x, y = _data()
    mask = torch.ones(3, 6, dtype=torch.float64)
    mask[0, 4:] = 0
    mask[2, 2:] = 0
    assert checkGradients(net, input=[x], labels=[y], inputMask=[mask], print_results=True, subset=400)


def test_bert_base_tiny_fits_and_serializes(tmp_path):
    net = BertBase(numLabels=2, inputShape=[12], vocabSize=50, hidden=32, layers=2, heads=2, ffn=64,
                   maxPositions=16, learningRate=1e-2).init(device="cpu")
    gen = torch.Generator().manual_seed(1)
    x = torch.randint(0, 50, (16, 12), generator=gen)
    lab = (x[:, 0] % 2).long()                                # label = parity of the first token: learnable
    y = torch.nn.functional.one_hot(lab, 2).float()
    s0 = None
    for _ in range(60):
        net.fit([x], [y])
        s0 = s0 if s0 is not None else net.score()
    assert net.score() < s0 * 0.7
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    p = str(tmp_path / "bert.zip")
    ModelSerializer.writeModel(net, p, True)
    net2 = ModelSerializer.restoreComputationGraph(p)
    assert torch.allclose(net2.outputSingle(x), net.outputSingle(x), atol=1e-5)


def test_hf_bert_import_matches_transformers_forward(tmp_path):
    """Parity pinned to HuggingFace transformers' BertForSequenceClassification (random init, no download)."""
    transformers = pytest.importorskip("transformers")
    cfg = transformers.BertConfig(vocab_size=60, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                                  intermediate_size=48, max_position_embeddings=24, num_labels=3)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(cfg).eval()
    from deeplearning4j_amd.modelimport.bert import importBert
    net = importBert(hf.state_dict(), cfg.to_dict(), seqLen=10, device="cpu")
    gen = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 60, (4, 10), generator=gen)
    am = torch.ones(4, 10, dtype=torch.long)
    am[1, 7:] = 0
    am[3, 4:] = 0
    with torch.no_grad():
        ref = torch.softmax(hf(input_ids=ids, attention_mask=am).logits, dim=-1)
    got = net.output(ids, masks=[am.float()])[0]
    assert torch.allclose(got, ref, atol=2e-5), (got - ref).abs().max()
    # safetensors round trip of the same checkpoint
    from safetensors.torch import save_file
    p = tmp_path / "model.safetensors"
    save_file({k: v.contiguous() for k, v in hf.state_dict().items()}, str(p))
    (tmp_path / "config.json").write_text(cfg.to_json_string())
    net2 = importBert(str(tmp_path), seqLen=10, device="cpu")
    assert torch.allclose(net2.output(ids, masks=[am.float()])[0], ref, atol=2e-5)
