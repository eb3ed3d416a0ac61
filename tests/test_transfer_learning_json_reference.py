"""FineTuneConfiguration JSON / YAML, after the reference's TestTransferLearningJson
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/transferlearning/TestTransferLearningJson.java:18-34): the
configuration (activation, backprop flag, updater and bias updater) round-trips through JSON and YAML to an equal
object that serialises to the same text. CPU."""
import deeplearning4j_amd as D


def test_json_yaml():
    c = (D.FineTuneConfiguration.Builder().activation(D.Activation.ELU).backprop(True).updater(D.AdaGrad(1.0))
         .biasUpdater(D.AdaGrad(10.0)).build())
    as_json, as_yaml = c.toJson(), c.toYaml()
    from_json, from_yaml = D.FineTuneConfiguration.fromJson(as_json), D.FineTuneConfiguration.fromYaml(as_yaml)
    assert c == from_json and c == from_yaml
    assert from_json.toJson() == as_json
    assert from_yaml.toYaml() == as_yaml
