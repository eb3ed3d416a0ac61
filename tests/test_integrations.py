"""Feature-parity integrations from SURVEY §2.9: streaming/serving routes (dl4j-streaming), Spark-ML-style
estimators (dl4j-spark-ml), S3 object store + provisioning API (deeplearning4j-aws), language tokenizers
(nlp-uima/japanese/chinese/korean), distributed Word2Vec (dl4j-spark-nlp)."""
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd import aws, streaming
from deeplearning4j_amd.parallel.ml import AutoEncoder, SparkDl4jNetwork
from deeplearning4j_amd.utils.model_serializer import ModelSerializer

import _dist_workers as W


def _conf(nin=4, nout=3, seed=3):
    return (NeuralNetConfiguration.Builder().seed(seed).updater(Adam(0.05)).list()
            .layer(0, DenseLayer.Builder().nIn(nin).nOut(16).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(16).nOut(nout).activation(Activation.SOFTMAX)
                   .build()).build())


def _net():
    n = MultiLayerNetwork(_conf())
    n.init(device="cpu")
    return n


# ------------------------------------------------------------------------------------------------ streaming
def test_ndarray_pubsub_roundtrip_and_route():
    broker = streaming.Broker()
    out = streaming.NDArrayConsumer("doubled", broker)
    route = streaming.NDArrayPubSubRoute("raw", "doubled", transform=lambda a: a * 2, broker=broker).start()
    try:
        x = torch.arange(12, dtype=torch.float32).reshape(3, 4)
        streaming.NDArrayPublisher("raw", broker).publish(x)
        got = out.getINDArray(timeout=5)
        assert torch.equal(got, x * 2)
        s = streaming.NDArrayType.toBase64(x)
        assert torch.equal(streaming.NDArrayType.fromBase64(s), x)
    finally:
        route.stop()


def test_serve_route_from_model_zip(tmp_path):
    net = _net()
    p = str(tmp_path / "m.zip")
    ModelSerializer.writeModel(net, p, False)
    broker = streaming.Broker()
    outq = streaming.NDArrayConsumer("predictions", broker)
    route = streaming.DL4jServeRouteBuilder().modelUri(p).consumingTopic("features").outputTopic("predictions") \
        .broker(broker).build().start()
    try:
        x = torch.randn(5, 4)
        streaming.NDArrayPublisher("features", broker).publish(x)
        y = outq.getINDArray(timeout=10)
        assert y.shape == (5, 3)
        assert torch.allclose(y, net.output(x), atol=1e-5)
    finally:
        route.stop()


def test_csv_record_converters():
    recs = ["1,2,3,0", "4,5,6,2"]
    ds = streaming.CSVRecordToDataSet().convert(recs, 3)
    assert ds.features.shape == (2, 3) and ds.labels[1, 2] == 1
    assert streaming.CSVRecordToINDArray().convert(recs).shape == (2, 4)


def test_http_model_server():
    from fastapi.testclient import TestClient
    net = _net()
    srv = streaming.ModelServer(net, batchLimit=8)
    try:
        c = TestClient(srv.app)
        assert c.get("/health").json()["status"] == "ok"
        x = torch.randn(3, 4)
        r = c.post("/predict", json={"array": x.tolist()}).json()
        assert np.allclose(np.array(r["array"]), net.output(x).numpy(), atol=1e-5)
        r2 = c.post("/predict", json={"ndarray": streaming.NDArrayType.toBase64(x)}).json()
        assert torch.allclose(streaming.NDArrayType.fromBase64(r2["ndarray"]), net.output(x), atol=1e-5)
        assert c.post("/predict", json={}).status_code == 400
    finally:
        srv.shutdown()


# ------------------------------------------------------------------------------------------------ spark-ml style
def _frame(n=256, seed=0):
    g = np.random.RandomState(seed)
    x = g.randn(n, 4).astype(np.float32)
    lab = (x[:, 0] + x[:, 1] > 0).astype(int) + (x[:, 2] > 0.8).astype(int)
    return pd.DataFrame({"features": list(x), "label": lab})


def test_estimator_fit_transform():
    df = _frame()
    est = SparkDl4jNetwork(_conf(), numLabels=3, epochs=30, batchSize=32).setPredictionCol("pred")
    model = est.fit(df)
    out = model.transform(df)
    acc = (out["pred"].to_numpy() == df["label"].to_numpy()).mean()
    assert acc > 0.78, acc
    assert model.predict(df["features"][0]) in (0.0, 1.0, 2.0)


def test_estimator_with_training_master():
    from deeplearning4j_amd.parallel import ParameterAveragingTrainingMaster
    tm = ParameterAveragingTrainingMaster.Builder(32).averagingFrequency(2).build()
    m = SparkDl4jNetwork(_conf(), numLabels=3, trainingMaster=tm, epochs=2).fit(_frame(128))
    assert "prediction" in m.transform(_frame(16, 1)).columns


def test_autoencoder_estimator():
    conf = (NeuralNetConfiguration.Builder().seed(1).updater(Adam(0.02)).list()
            .layer(0, DenseLayer.Builder().nIn(4).nOut(2).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MSE).nIn(2).nOut(4).activation(Activation.IDENTITY).build())
            .build())
    df = _frame(64)
    m = AutoEncoder(conf, compressedLayer=0, epochs=3).setOutputCol("code").fit(df)
    out = m.transform(df)
    assert np.asarray(out["code"][0]).shape == (2,)


# ------------------------------------------------------------------------------------------------ aws
def test_s3_local_object_store_and_dataset_iterator(tmp_path):
    root = str(tmp_path / "s3")
    os.makedirs(root)
    up = aws.S3Uploader(root=root)
    up.createBucket("data")
    f = tmp_path / "hello.txt"
    f.write_text("hi")
    assert up.upload(str(f), "data", "dir/hello.txt") == "s3://data/dir/hello.txt"
    down = aws.S3Downloader(root=root)
    assert down.keysForBucket("data") == ["dir/hello.txt"]
    assert open(down.download("data", "dir/hello.txt", str(tmp_path / "o.txt"))).read() == "hi"
    for i in range(3):
        aws.save_dataset_to_bucket(DataSet(torch.full((2, 4), float(i)), torch.zeros(2, 3)), "batches",
                                   f"b{i}.bin", up)
    it = aws.BaseS3DataSetIterator("batches", down)
    vals = [float(ds.features[0, 0]) for ds in it]
    assert vals == [0.0, 1.0, 2.0]
    with pytest.raises(ValueError):
        down.objectForKey("data", "../../etc/passwd")


def test_aws_object_store_unavailable_is_explicit(monkeypatch):
    monkeypatch.delenv("DL4J_AMD_S3_ROOT", raising=False)
    if aws._boto3() is None:
        with pytest.raises(aws.AwsUnavailable):
            aws.S3Downloader()
    assert "--nproc-per-node 8" in aws.ClusterSetup(None).launch_command(2, "10.0.0.1")


# ------------------------------------------------------------------------------------------------ tokenizers
def test_language_tokenizers():
    from deeplearning4j_amd.nlp import DefaultTokenizerFactory
    from deeplearning4j_amd.nlp.tokenization_ext import (BertWordPieceTokenizerFactory, ChineseTokenizerFactory,
                                                          JapaneseTokenizerFactory, KoreanTokenizerFactory,
                                                          PorterStemmer, StemmingPreprocessor)
    p = PorterStemmer()
    assert [p.stem(w) for w in ("caresses", "ponies", "hopping", "relational", "agreed")] == \
        ["caress", "poni", "hop", "relat", "agre"]
    tf = DefaultTokenizerFactory()
    tf.setTokenPreProcessor(StemmingPreprocessor())
    assert tf.create("Running dogs, jumped!").getTokens() == ["run", "dog", "jump"]
    assert JapaneseTokenizerFactory().create("私は東京へ行きました").getTokens()[:4] == ["私", "は", "東京", "へ"]
    assert ChineseTokenizerFactory().create("我爱北京 ok").getTokens() == ["我", "爱", "北", "京", "ok"]
    assert KoreanTokenizerFactory().create("나는 학교에 갑니다").getTokens() == ["나", "는", "학교", "에", "갑니다"]
    v = {t: i for i, t in enumerate(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "un", "##aff", "##able", "hi", "!"])}
    b = BertWordPieceTokenizerFactory(v)
    assert b.create("Unaffable hi! zzz").getTokens() == ["un", "##aff", "##able", "hi", "!", "[UNK]"]
    assert b.encode("unaffable") == [2, 4, 5, 6, 3]


# ------------------------------------------------------------------------------------------------ spark-nlp
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_distributed_word2vec_gloo(tmp_path):
    path = str(tmp_path / "w2v.pt")
    mp.spawn(W.run_w2v, args=(2, _port(), path), nprocs=2, join=True)
    r = torch.load(path, weights_only=True)
    assert r["same"], "averaged tables differ across ranks"
    assert r["n"] == 20
    assert r["in"] > r["out"] + 0.2, r
