"""BERT import: HuggingFace-format BERT checkpoints (``BertModel`` / ``BertForSequenceClassification`` state dicts,
``.safetensors`` or torch ``.bin`` loaded with ``weights_only=True``, plus ``config.json``) -> the BertBase
ComputationGraph of :mod:`deeplearning4j_amd.models`.

This is the model-import path behind BASELINE.json's "BERT-base SameDiff import" config: the reference imports
TensorFlow/ONNX graphs into SameDiff; here the transformer graph is a native ComputationGraph (fused encoder-block
layers running the flash-attention / LayerNorm HIP kernels) and the importer maps tensors by name:

  embeddings.{word,position,token_type}_embeddings.weight -> embeddings/{Wword,Wpos,Wtype}
  embeddings.LayerNorm                                     -> embeddings/{lng,lnb}
  encoder.layer.i.attention.self.{query,key,value}         -> encoder_i/Wqkv (= [Wqᵀ | Wkᵀ | Wvᵀ]), bqkv
  encoder.layer.i.attention.output.dense / .LayerNorm      -> encoder_i/{Wo,bo} / {ln1g,ln1b}
  encoder.layer.i.intermediate.dense, output.dense         -> encoder_i/{W1,b1}, {W2,b2}
  encoder.layer.i.output.LayerNorm                         -> encoder_i/{ln2g,ln2b}
  pooler.dense, classifier                                 -> pooler/{W,b}, classifier/{W,b}
(torch Linear weights are [out, in]; DL4J layers store [in, out], hence the transposes.)
"""
import json
import os

import torch


def _load_state(src):
    if isinstance(src, dict):
        return dict(src)
    if os.path.isdir(src):
        for name in ("model.safetensors", "pytorch_model.bin"):
            p = os.path.join(src, name)
            if os.path.exists(p):
                return _load_state(p)
        raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin in {src}")
    if src.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(src)
    return torch.load(src, map_location="cpu", weights_only=True)


def _load_config(cfg, src):
    if isinstance(cfg, dict):
        return cfg
    if cfg is None and isinstance(src, str):
        d = src if os.path.isdir(src) else os.path.dirname(src)
        cfg = os.path.join(d, "config.json")
    if hasattr(cfg, "to_dict"):
        return cfg.to_dict()
    with open(cfg) as fh:
        return json.load(fh)


def importBert(src, config=None, numLabels=None, seqLen=128, device=None, dataType=None):
    """Build a BertBase graph with the checkpoint's hyper-parameters and copy its weights. ``numLabels`` defaults to
    the checkpoint's classifier size (2 when there is none; the classifier then keeps its random init)."""
    from ..models import BertBase
    from ..nn.conf import DataType
    sd = _load_state(src)
    sd = {(k[5:] if k.startswith("bert.") else k): v for k, v in sd.items()}
    cfg = _load_config(config, src)
    if numLabels is None:
        numLabels = sd["classifier.weight"].shape[0] if "classifier.weight" in sd else 2
    model = BertBase(numLabels=numLabels, inputShape=[seqLen], vocabSize=cfg["vocab_size"], hidden=cfg["hidden_size"],
                     layers=cfg["num_hidden_layers"], heads=cfg["num_attention_heads"], ffn=cfg["intermediate_size"],
                     maxPositions=cfg["max_position_embeddings"], dataType=dataType or DataType.FLOAT)
    conf = model.conf()
    eps = float(cfg.get("layer_norm_eps", 1e-12))
    for name, v in conf.vertices.items():
        lc = getattr(v, "layerConf", None)
        lc = getattr(lc, "layer", lc)
        if lc is not None and hasattr(lc, "layerNormEps"):
            lc.layerNormEps = eps
    if cfg.get("hidden_act", "gelu") not in ("gelu", "gelu_new", "gelu_python"):
        raise ValueError(f"unsupported hidden_act {cfg.get('hidden_act')}")
    from ..nn.graph import ComputationGraph
    net = ComputationGraph(conf)
    net.init(device=device)
    copy_bert_weights(net, sd, cfg["num_hidden_layers"])
    return net


def copy_bert_weights(net, sd, layers):
    def put(key, t):
        dst = net.getParam(key)
        with torch.no_grad():
            dst.copy_(t.reshape(dst.shape).to(dst.dtype))

    put("embeddings_Wword", sd["embeddings.word_embeddings.weight"])
    put("embeddings_Wpos", sd["embeddings.position_embeddings.weight"])
    put("embeddings_Wtype", sd["embeddings.token_type_embeddings.weight"])
    put("embeddings_lng", sd["embeddings.LayerNorm.weight"])
    put("embeddings_lnb", sd["embeddings.LayerNorm.bias"])
    for i in range(layers):
        p = f"encoder.layer.{i}."
        a = p + "attention."
        wq, wk, wv = (sd[a + f"self.{n}.weight"] for n in ("query", "key", "value"))
        bq, bk, bv = (sd[a + f"self.{n}.bias"] for n in ("query", "key", "value"))
        e = f"encoder_{i}_"
        put(e + "Wqkv", torch.cat([wq.t(), wk.t(), wv.t()], dim=1))
        put(e + "bqkv", torch.cat([bq, bk, bv]))
        put(e + "Wo", sd[a + "output.dense.weight"].t())
        put(e + "bo", sd[a + "output.dense.bias"])
        put(e + "ln1g", sd[a + "output.LayerNorm.weight"])
        put(e + "ln1b", sd[a + "output.LayerNorm.bias"])
        put(e + "W1", sd[p + "intermediate.dense.weight"].t())
        put(e + "b1", sd[p + "intermediate.dense.bias"])
        put(e + "W2", sd[p + "output.dense.weight"].t())
        put(e + "b2", sd[p + "output.dense.bias"])
        put(e + "ln2g", sd[p + "output.LayerNorm.weight"])
        put(e + "ln2b", sd[p + "output.LayerNorm.bias"])
    if "pooler.dense.weight" in sd:
        put("pooler_W", sd["pooler.dense.weight"].t())
        put("pooler_b", sd["pooler.dense.bias"])
    if "classifier.weight" in sd:
        put("classifier_W", sd["classifier.weight"].t())
        put("classifier_b", sd["classifier.bias"])
    net.sync_shadow()
    return net


def importBertSameDiff(src, config=None, numLabels=None, seqLen=128, device=None, dtype=torch.float32, batch=1):
    """Import a HuggingFace BERT checkpoint as a SameDiff graph (BASELINE.json "BERT-base SameDiff import").

    Placeholders ``input_ids`` [B, T] (int), ``attention_mask`` [B, T] (1 = token, 0 = padding) and ``labels``
    [B, numLabels] (one-hot). Outputs ``probabilities`` and the loss variable ``loss``
    (softmax cross entropy). The encoder uses the same fused ops as the ComputationGraph import: one fused QKV
    projection per layer, ``nn().fusedSelfAttention`` (flash-attention kernel), ``nn().layerNorm`` (LayerNorm
    kernel) and GELU. Train it with ``setTrainingConfig`` + ``fit`` (mapping features -> input_ids, attention_mask;
    labels -> labels)."""
    from ..samediff import SameDiff
    sd_ = _load_state(src)
    sd_ = {(k[5:] if k.startswith("bert.") else k): v for k, v in sd_.items()}
    cfg = _load_config(config, src)
    if numLabels is None:
        numLabels = sd_["classifier.weight"].shape[0] if "classifier.weight" in sd_ else 2
    dev = torch.device(device) if device is not None else torch.device("cpu")
    E, L, nh = cfg["hidden_size"], cfg["num_hidden_layers"], cfg["num_attention_heads"]
    eps = float(cfg.get("layer_norm_eps", 1e-12))

    def w(t):
        return t.detach().to(dtype).to(dev).contiguous()

    g = SameDiff.create()
    ids = g.placeHolder("input_ids", torch.zeros(batch, seqLen, dtype=torch.long, device=dev))
    am = g.placeHolder("attention_mask", torch.ones(batch, seqLen, device=dev))
    labels = g.placeHolder("labels", torch.zeros(batch, numLabels, dtype=dtype, device=dev))
    wword = g.var("embeddings_Wword", w(sd_["embeddings.word_embeddings.weight"]))
    wpos = g.var("embeddings_Wpos", w(sd_["embeddings.position_embeddings.weight"]))
    wtype = g.var("embeddings_Wtype", w(sd_["embeddings.token_type_embeddings.weight"]))
    x = g.gather("emb_word", wword, ids)
    x = x.add("emb_pos", wpos.get(slice(0, seqLen)))
    x = x.add("emb_type", wtype.get(slice(0, 1)))               # token type 0 for every position
    x = g.nn().layerNorm("emb_ln", x, g.var("embeddings_lng", w(sd_["embeddings.LayerNorm.weight"])),
                         g.var("embeddings_lnb", w(sd_["embeddings.LayerNorm.bias"])), eps)
    for i in range(L):
        p = f"encoder.layer.{i}."
        a = p + "attention."
        e = f"encoder_{i}_"
        wqkv = torch.cat([sd_[a + f"self.{n}.weight"].t() for n in ("query", "key", "value")], dim=1)
        bqkv = torch.cat([sd_[a + f"self.{n}.bias"] for n in ("query", "key", "value")])
        qkv = g.nn().linear(e + "qkv", x, g.var(e + "Wqkv", w(wqkv)), g.var(e + "bqkv", w(bqkv)))
        att = g.nn().fusedSelfAttention(e + "attn", qkv, nh, am)
        o = g.nn().linear(e + "attn_out", att, g.var(e + "Wo", w(sd_[a + "output.dense.weight"].t())),
                          g.var(e + "bo", w(sd_[a + "output.dense.bias"])))
        x = g.nn().layerNorm(e + "ln1", o.add(e + "res1", x), g.var(e + "ln1g", w(sd_[a + "output.LayerNorm.weight"])),
                             g.var(e + "ln1b", w(sd_[a + "output.LayerNorm.bias"])), eps)
        hdn = g.nn().gelu(e + "gelu", g.nn().linear(e + "ffn1", x, g.var(e + "W1", w(sd_[p + "intermediate.dense.weight"].t())),
                                                    g.var(e + "b1", w(sd_[p + "intermediate.dense.bias"]))))
        f2 = g.nn().linear(e + "ffn2", hdn, g.var(e + "W2", w(sd_[p + "output.dense.weight"].t())),
                           g.var(e + "b2", w(sd_[p + "output.dense.bias"])))
        x = g.nn().layerNorm(e + "ln2", f2.add(e + "res2", x), g.var(e + "ln2g", w(sd_[p + "output.LayerNorm.weight"])),
                             g.var(e + "ln2b", w(sd_[p + "output.LayerNorm.bias"])), eps)
    cls = x.get(slice(None), 0)
    if "pooler.dense.weight" in sd_:
        pw, pb = sd_["pooler.dense.weight"].t(), sd_["pooler.dense.bias"]
    else:
        pw, pb = torch.eye(E), torch.zeros(E)
    pooled = g.nn().tanh("pooled", g.nn().linear("pooler", cls, g.var("pooler_W", w(pw)), g.var("pooler_b", w(pb))))
    if "classifier.weight" in sd_:
        cw, cb = sd_["classifier.weight"].t(), sd_["classifier.bias"]
    else:
        gen = torch.Generator().manual_seed(0)
        cw, cb = torch.randn(E, numLabels, generator=gen) * 0.02, torch.zeros(numLabels)
    logits = g.nn().linear("logits", pooled, g.var("classifier_W", w(cw)), g.var("classifier_b", w(cb)))
    g.nn().softmax("probabilities", logits)
    g.loss().softmaxCrossEntropy("loss", labels, logits)
    return g
