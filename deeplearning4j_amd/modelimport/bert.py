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
