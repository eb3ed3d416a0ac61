"""User-defined input preprocessors, after the reference's CustomPreprocessorTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/preprocessor/CustomPreprocessorTest.java:25-70): a
subclass of InputPreProcessor is registered for (de)serialisation by being defined, and a MultiLayerConfiguration
using it round-trips through JSON and YAML to an equal configuration whose preprocessor is that class. CPU."""
import deeplearning4j_amd as D
from deeplearning4j_amd.nn.conf.base import lookup
from deeplearning4j_amd.nn.conf.preprocessors import InputPreProcessor


class MyCustomPreprocessor(InputPreProcessor):
    """Reference conf/preprocessor/custom/MyCustomPreprocessor: adds 1 forward, passes epsilons through."""

    def preProcess(self, x, miniBatchSize, training=False):
        return x + 1.0

    def backprop(self, eps, miniBatchSize):
        return eps

    def getOutputType(self, inputType):
        return inputType


def test_custom_preprocessor():
    assert lookup("MyCustomPreprocessor") is MyCustomPreprocessor, "not registered for deserialisation"
    conf = (D.NeuralNetConfiguration.Builder().list()
            .layer(0, D.DenseLayer.Builder().nIn(10).nOut(10).build())
            .layer(1, D.OutputLayer.Builder(D.LossFunction.MCXENT).nIn(10).nOut(10).build())
            .inputPreProcessor(0, MyCustomPreprocessor()).pretrain(False).backprop(True).build())
    from_json = D.MultiLayerConfiguration.fromJson(conf.toJson())
    assert from_json == conf
    assert D.MultiLayerConfiguration.fromYaml(conf.toYaml()) == conf
    assert isinstance(from_json.getInputPreProcess(0), MyCustomPreprocessor)
