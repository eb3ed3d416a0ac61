"""configuration.json in DL4J's own Jackson schema (reference NN:nn/conf/MultiLayerConfiguration.java:120-200,
NN:nn/conf/NeuralNetConfiguration.java:94, NN:nn/conf/layers/Layer.java:54-90).

Fixtures: tests/fixtures/dl4j_json/*.json are configurations printed by the reference itself — extracted verbatim
from the output cells of the reference's own tutorial notebooks (dl4j-examples/tutorials/01, 11). No DL4J model
ZIPs exist in the reference tree, so ZIP-level interop beyond these configurations remains unpinned.
"""
import json
import os

import torch

from deeplearning4j_amd.nn.conf.network import ComputationGraphConfiguration, MultiLayerConfiguration

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "dl4j_json")


def _read(name):
    with open(os.path.join(FIX, name)) as f:
        return f.read()


def test_reference_mlp_configs_parse_and_run():
    from deeplearning4j_amd.nn.conf.activations import ActivationLReLU, ActivationReLU, ActivationSoftmax
    from deeplearning4j_amd.nn.conf.layers import DenseLayer, OutputLayer
    from deeplearning4j_amd.nn.conf.losses import LossMCXENT
    from deeplearning4j_amd.nn.conf.updaters import Nesterovs, Sgd
    from deeplearning4j_amd.nn.multilayer import MultiLayerNetwork
    c = MultiLayerConfiguration.fromJson(_read("01_1.json"))
    assert [type(l) for l in c.confs] == [DenseLayer, OutputLayer]
    assert (c.confs[0].nIn, c.confs[0].nOut, c.confs[1].nOut) == (784, 100, 10)
    assert isinstance(c.confs[0].activation, ActivationReLU) and isinstance(c.confs[0].updater, Nesterovs)
    assert c.confs[0].updater.momentum == 0.9
    c2 = MultiLayerConfiguration.fromJson(_read("11_3.json"))
    assert isinstance(c2.confs[0].activation, ActivationLReLU) and c2.confs[0].activation.alpha == 0.01
    assert isinstance(c2.confs[1].activation, ActivationSoftmax) and isinstance(c2.confs[1].lossFn, LossMCXENT)
    assert isinstance(c2.confs[0].updater, Sgd)
    assert c2.seed == json.loads(_read("11_3.json"))["confs"][0]["seed"]
    net = MultiLayerNetwork(c2)
    net.init()
    assert net.numParams() == 784 * 250 + 250 + 250 * 10 + 10
    out = net.output(torch.rand(3, 784))
    assert out.shape == (3, 10) and torch.allclose(out.sum(1), torch.ones(3), atol=1e-5)


def test_reference_graph_config_parse_and_run():
    from deeplearning4j_amd.nn.graph.computation_graph import ComputationGraph
    c = ComputationGraphConfiguration.fromJson(_read("01_2.json"))
    assert c.networkInputs == ["input"] and c.networkOutputs == ["out1", "out2"]
    assert c.vertexInputs["out2"] == ["L1"]
    net = ComputationGraph(c)
    net.init()
    outs = net.output(torch.rand(4, 3))
    assert len(outs) == 2 and outs[0].shape == (4, 3)


def _layer_key(nnc):
    return next(iter(nnc["layer"]))


def test_written_schema_is_jackson_wrapper_objects():
    from deeplearning4j_amd.models import LeNet, TextGenerationLSTM
    d = json.loads(LeNet(numLabels=10).conf().toJson())
    keys = [_layer_key(c) for c in d["confs"]]
    assert keys[0] == "convolution" and "subsampling" in keys and keys[-1] == "output"
    conv = d["confs"][0]["layer"]["convolution"]
    assert "nin" in conv and "nout" in conv and "activationFn" in conv and "iupdater" in conv
    assert conv["iupdater"]["@class"].startswith("org.nd4j.linalg.learning.config.")
    assert list(d["confs"][-1]["layer"]["output"]["lossFn"]) == ["NegativeLogLikelihood"] or \
        list(d["confs"][-1]["layer"]["output"]["lossFn"])[0] in ("MCXENT", "NegativeLogLikelihood")
    for c in d["confs"]:
        assert {"seed", "optimizationAlgo", "miniBatch", "minimize", "layer", "variables"} <= set(c)
    d = json.loads(TextGenerationLSTM(totalUniqueCharacters=77).conf().toJson())
    assert _layer_key(d["confs"][0]) == "gravesLSTM" and _layer_key(d["confs"][-1]) == "rnnoutput"
    assert d["backpropType"] == "TruncatedBPTT"


def test_round_trip_zoo_configs():
    from deeplearning4j_amd.models import LeNet, ResNet50, TextGenerationLSTM
    for m in (LeNet(numLabels=10), TextGenerationLSTM(totalUniqueCharacters=77), ResNet50(numLabels=10)):
        conf = m.conf()
        back = type(conf).fromJson(conf.toJson())
        assert back == conf, type(m).__name__
    d = json.loads(ResNet50(numLabels=10).conf().toJson())
    v = d["vertices"]["res2a_branch2a"]["LayerVertex"]
    assert _layer_key(v["layerConf"]) == "convolution" and v["outputVertex"] is False
    assert "ElementWiseVertex" in json.dumps(d["vertices"])


def test_legacy_updater_and_loss_fields():
    """Pre-1.0 configs: updater enum + hyperparameters, lossFunction enum, dropOut probability."""
    from deeplearning4j_amd.nn.conf.losses import LossMCXENT
    from deeplearning4j_amd.nn.conf.updaters import Adam
    d = json.loads(_read("11_3.json"))
    for c in d["confs"]:
        body = next(iter(c["layer"].values()))
        body.pop("iupdater")
        body.update({"updater": "ADAM", "learningRate": 0.02, "adamMeanDecay": 0.8, "adamVarDecay": 0.99,
                     "dropOut": 0.5})
        body.pop("lossFn", None)
    conf = MultiLayerConfiguration.fromJson(json.dumps(d))
    u = conf.confs[0].updater
    assert isinstance(u, Adam) and (u.learningRate, u.beta1, u.beta2) == (0.02, 0.8, 0.99)
    assert isinstance(conf.confs[1].lossFn, LossMCXENT)
    assert conf.confs[0].idropout is not None


def test_previous_tagged_format_still_reads():
    from deeplearning4j_amd.models import LeNet
    conf = LeNet(numLabels=10).conf()
    old = json.dumps(conf.to_dict())
    assert MultiLayerConfiguration.fromJson(old) == conf


def test_model_serializer_zip_holds_dl4j_configuration(tmp_path):
    import zipfile
    from deeplearning4j_amd.models import LeNet
    from deeplearning4j_amd.utils.model_serializer import ModelSerializer
    net = LeNet(numLabels=10).init()
    p = str(tmp_path / "lenet.zip")
    ModelSerializer.writeModel(net, p, True)
    with zipfile.ZipFile(p) as z:
        cfg = json.loads(z.read("configuration.json"))
    assert "confs" in cfg and _layer_key(cfg["confs"][0]) == "convolution"
    back = ModelSerializer.restoreMultiLayerNetwork(p, True)
    assert torch.equal(back.params(), net.params())
    x = torch.rand(2, 1, 28, 28)
    assert torch.allclose(back.output(x), net.output(x))
