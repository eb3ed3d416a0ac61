"""ParallelWrapperMain end to end, after the reference's ParallelWrapperMainTest
(deeplearning4j-scaleout/deeplearning4j-scaleout-parallelwrapper/src/test/java/org/deeplearning4j/parallelism/main/
ParallelWrapperMainTest.java:25-81): the LeNet-style MNIST network (Nesterovs, l2 5e-4, conv 5x5 x20 / max pool /
conv 5x5 x50 / max pool / dense 500 / softmax 10) is written without its updater, and the CLI entry point restores it,
trains from an iterator-provider factory named on the command line, reports to a UI server given by --uiUrl, and
writes the trained model to --modelOutputPath. MNIST is not available offline: the factory yields MNIST-shaped
synthetic batches (parity of the flow, not of the numbers). fp32, CPU, one process."""
import json
import sys
import urllib.request

import torch

import deeplearning4j_amd as D
from deeplearning4j_amd.nn.conf.inputs import InputType
from deeplearning4j_amd.parallel.main import main
from deeplearning4j_amd.utils.model_serializer import ModelSerializer

FACTORY = '''
import torch
from deeplearning4j_amd import DataSet, ListDataSetIterator


class MnistDataSetIteratorProviderFactory:
    """The reference test's provider factory: create() returns the training iterator (synthetic MNIST shapes)."""

    def create(self):
        g = torch.Generator().manual_seed(12345)
        out = []
        for _ in range(3):
            x = torch.rand(16, 784, generator=g)
            y = torch.zeros(16, 10)
            y[torch.arange(16), torch.randint(0, 10, (16,), generator=g)] = 1.0
            out.append(DataSet(x, y))
        return ListDataSetIterator(out)
'''


def _lenet():
    conf = (D.NeuralNetConfiguration.Builder().seed(123).l2(0.0005).weightInit(D.WeightInit.XAVIER)
            .updater(D.Nesterovs(0.01, 0.9)).list()
            .layer(0, D.ConvolutionLayer.Builder(5, 5).nIn(1).stride(1, 1).nOut(20).activation(D.Activation.IDENTITY)
                   .build())
            .layer(1, D.SubsamplingLayer.Builder(D.SubsamplingLayer.PoolingType.MAX).kernelSize(2, 2).stride(2, 2)
                   .build())
            .layer(2, D.ConvolutionLayer.Builder(5, 5).stride(1, 1).nOut(50).activation(D.Activation.IDENTITY).build())
            .layer(3, D.SubsamplingLayer.Builder(D.SubsamplingLayer.PoolingType.MAX).kernelSize(2, 2).stride(2, 2)
                   .build())
            .layer(4, D.DenseLayer.Builder().activation(D.Activation.RELU).nOut(500).build())
            .layer(5, D.OutputLayer.Builder(D.LossFunctions.LossFunction.NEGATIVELOGLIKELIHOOD).nOut(10)
                   .activation(D.Activation.SOFTMAX).build())
            .backprop(True).pretrain(False).setInputType(InputType.convolutionalFlat(28, 28, 1)).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    return net


def test_run_parallel_wrapper_main(tmp_path):
    from deeplearning4j_amd.ui.server import UIServer
    (tmp_path / "pwmain_mnist_factory.py").write_text(FACTORY)
    sys.path.insert(0, str(tmp_path))
    ui = UIServer(port=0).start()
    try:
        ui.enableRemoteListener()
        model = _lenet()
        p0 = model.params().clone()
        ModelSerializer.writeModel(model, str(tmp_path / "tmpmodel.zip"), False)
        out = main(["--modelPath", str(tmp_path / "tmpmodel.zip"),
                    "--dataSetIteratorFactoryClazz", "pwmain_mnist_factory:MnistDataSetIteratorProviderFactory",
                    "--modelOutputPath", str(tmp_path / "tmpmodel.bin"),
                    "--uiUrl", ui.getAddress().replace("http://", "")])
        assert out.getIterationCount() == 3
        restored = ModelSerializer.restoreMultiLayerNetwork(str(tmp_path / "tmpmodel.bin"))
        assert torch.equal(restored.params(), out.params())
        assert not torch.equal(restored.params(), p0)
        sessions = json.loads(urllib.request.urlopen(ui.getAddress() + "/api/sessions", timeout=10).read())
        assert sessions and ui.remote_storage.getNumUpdateRecordsFor(sessions[0]) >= 1
    finally:
        ui.stop()
        sys.path.remove(str(tmp_path))
