"""Estimator / model wrappers over tabular data frames — the replacement for dl4j-spark-ml (SURVEY §2.9:
``SparkDl4jNetwork`` / ``SparkDl4jModel`` / ``AutoEncoder`` wrappers, dl4j-spark-ml/src/main/spark-2/scala/
org/deeplearning4j/spark/ml/impl/SparkDl4jNetwork.scala, AutoEncoderWrapper.scala).

The reference's Spark ML pipeline stages take a ``Dataset[Row]`` with a features vector column and a label column,
train through ``SparkDl4jMultiLayer`` (a TrainingMaster) and return a model whose ``transform`` appends a
prediction column. Here the data frame is a pandas DataFrame (one local partition per rank; under torchrun every
rank passes its own partition and training runs through the same TrainingMasters as
:mod:`deeplearning4j_amd.parallel.cluster`, i.e. RCCL parameter averaging / gradient sharing).
"""
import numpy as np
import torch


def _features(df, col):
    v = df[col].to_numpy()
    if v.dtype == object:
        return np.stack([np.asarray(r, dtype=np.float32) for r in v])
    return v.astype(np.float32).reshape(len(v), -1)


class _Params:
    def __init__(self):
        self.featuresCol = "features"
        self.labelCol = "label"
        self.predictionCol = "prediction"

    def setFeaturesCol(self, c):
        self.featuresCol = c
        return self

    def setLabelCol(self, c):
        self.labelCol = c
        return self

    def setPredictionCol(self, c):
        self.predictionCol = c
        return self


class SparkDl4jNetwork(_Params):
    """Estimator: ``fit(df) -> SparkDl4jModel``. ``numLabels`` > 0 = classification (label column holds class
    indices, one-hot encoded for training), 0 = regression (label column holds scalars or vectors)."""

    def __init__(self, multiLayerConfiguration, numLabels, trainingMaster=None, epochs=1, listeners=(),
                 collectStats=False, batchSize=32, device=None):
        super().__init__()
        self.conf = multiLayerConfiguration
        self.numLabels = int(numLabels)
        self.trainingMaster = trainingMaster
        self.epochs = int(epochs)
        self.listeners = list(listeners)
        self.collectStats = collectStats
        self.batchSize = int(batchSize)
        self.device = device

    def _datasets(self, df):
        from ..datasets import DataSet
        x = torch.from_numpy(_features(df, self.featuresCol))
        lab = df[self.labelCol].to_numpy()
        if self.numLabels > 0:
            y = torch.zeros(len(lab), self.numLabels)
            y[torch.arange(len(lab)), torch.as_tensor(lab.astype(np.int64))] = 1.0
        else:
            y = torch.from_numpy(_features(df, self.labelCol))
        return [DataSet(x[i:i + self.batchSize], y[i:i + self.batchSize]) for i in range(0, len(x), self.batchSize)]

    def fit(self, df):
        from ..datasets import ListDataSetIterator
        from ..nn.conf import MultiLayerConfiguration
        from ..nn.multilayer import MultiLayerNetwork
        net = MultiLayerNetwork(MultiLayerConfiguration.fromJson(self.conf.toJson()))   # fresh copy per fit
        net.init(device=self.device)
        if self.listeners:
            net.setListeners(self.listeners)
        stats = None
        if self.trainingMaster is not None:
            from .cluster import SparkDl4jMultiLayer
            SparkDl4jMultiLayer(None, net, self.trainingMaster).fit(self._datasets(df), self.epochs)
            stats = getattr(self.trainingMaster, "stats", None) if self.collectStats else None
        else:
            it = ListDataSetIterator(self._datasets(df), self.batchSize)
            for _ in range(self.epochs):
                it.reset()
                net.fit(it)
        m = SparkDl4jModel(net, self.numLabels)
        m.featuresCol, m.labelCol, m.predictionCol = self.featuresCol, self.labelCol, self.predictionCol
        m.trainingStats = stats
        return m


class SparkDl4jModel(_Params):
    """Fitted model: ``transform(df)`` appends the prediction column (argmax class for classification, the output
    vector/scalar for regression); ``predict`` / ``output`` work on single feature vectors."""

    def __init__(self, network, numLabels=0):
        super().__init__()
        self.network = network
        self.numLabels = int(numLabels)
        self.trainingStats = None

    def output(self, vector):
        x = torch.as_tensor(np.asarray(vector, dtype=np.float32)).reshape(1, -1)
        return self.network.output(x)[0].cpu()

    def predict(self, vector):
        o = self.output(vector)
        return float(torch.argmax(o)) if self.numLabels > 0 else (float(o[0]) if o.numel() == 1 else o.numpy())

    def transform(self, df):
        x = torch.from_numpy(_features(df, self.featuresCol))
        out = self.network.output(x).cpu()
        df = df.copy()
        if self.numLabels > 0:
            df[self.predictionCol] = torch.argmax(out, dim=1).double().numpy()
        elif out.shape[1] == 1:
            df[self.predictionCol] = out[:, 0].double().numpy()
        else:
            df[self.predictionCol] = list(out.numpy())
        return df

    def getNetwork(self):
        return self.network

    def getTrainingStats(self):
        return self.trainingStats


class AutoEncoder(_Params):
    """Unsupervised estimator: trains the network to reconstruct its input; the fitted model's ``transform``
    appends the activations of ``compressedLayer`` (the code) as the output column (AutoEncoderWrapper.scala)."""

    def __init__(self, multiLayerConfiguration, compressedLayer, epochs=1, batchSize=32, device=None):
        super().__init__()
        self.conf = multiLayerConfiguration
        self.compressedLayer = int(compressedLayer)
        self.epochs = int(epochs)
        self.batchSize = int(batchSize)
        self.device = device
        self.inputCol = "features"
        self.outputCol = "compressed"

    def setInputCol(self, c):
        self.inputCol = c
        return self

    def setOutputCol(self, c):
        self.outputCol = c
        return self

    def fit(self, df):
        from ..datasets import DataSet, ListDataSetIterator
        from ..nn.multilayer import MultiLayerNetwork
        net = MultiLayerNetwork(self.conf)
        net.init(device=self.device)
        x = torch.from_numpy(_features(df, self.inputCol))
        batches = [DataSet(x[i:i + self.batchSize], x[i:i + self.batchSize]) for i in range(0, len(x), self.batchSize)]
        it = ListDataSetIterator(batches, self.batchSize)
        for _ in range(self.epochs):
            it.reset()
            net.fit(it)
        m = AutoEncoderModel(net, self.compressedLayer)
        m.inputCol, m.outputCol = self.inputCol, self.outputCol
        return m


class AutoEncoderModel:
    def __init__(self, network, compressedLayer):
        self.network = network
        self.compressedLayer = compressedLayer
        self.inputCol = "features"
        self.outputCol = "compressed"

    def encode(self, x):
        with torch.no_grad():
            acts = self.network.feedForwardToLayer(self.compressedLayer, torch.as_tensor(x, dtype=torch.float32))
        return acts[-1].float().cpu()

    def transform(self, df):
        code = self.encode(torch.from_numpy(_features(df, self.inputCol)))
        df = df.copy()
        df[self.outputCol] = list(code.numpy())
        return df
