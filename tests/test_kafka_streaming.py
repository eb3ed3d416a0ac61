"""Streaming over the Kafka wire protocol (reference dl4j-streaming: NDArrayPublisher / NDArrayConsumer over Camel
kafka: endpoints, routes/DL4jServeRouteBuilder.java:48-92). The client speaks Metadata v1 / Produce v3 / Fetch v4 /
ListOffsets v1 with RecordBatch v2; here it runs against the in-tree protocol-level broker (no Kafka in the image)."""
import torch

from deeplearning4j_amd import *  # noqa: F401,F403
from deeplearning4j_amd import streaming
from deeplearning4j_amd.streaming import kafka as K
from deeplearning4j_amd.utils.model_serializer import ModelSerializer


def test_crc32c_known_values():
    assert K.crc32c(b"123456789") == 0xE3069283            # the CRC-32C check value
    assert K.crc32c(b"") == 0
    assert K.crc32c(bytes(32)) == 0x8A9136AA                 # RFC 3720 B.4: 32 bytes of zeros


def test_record_batch_roundtrip_and_corruption():
    recs = [(None, b"a"), (b"k", b"x" * 300), (b"", None)]
    b = K.encode_record_batch(recs, base_offset=41, base_timestamp=1234)
    assert b[16] == 2                                         # magic after base offset, length, leader epoch
    out = K.decode_record_batches(b + b[:20])                # a trailing partial batch is ignored
    assert out == [(41, None, b"a"), (42, b"k", b"x" * 300), (43, b"", None)]
    bad = bytearray(b)
    bad[-1] ^= 0xFF
    try:
        K.decode_record_batches(bytes(bad))
        raise AssertionError("corruption not detected")
    except ValueError:
        pass


def test_produce_fetch_offsets_metadata():
    srv = K.MiniKafkaServer().start()
    kb = K.KafkaBroker(srv.bootstrap)
    try:
        md = kb.metadata(["t1"])
        assert md["t1"][0] == 0 and md["t1"][1] == {0: 1}
        assert kb.list_offset("t1") == 0
        assert kb.produce("t1", ["m0", "m1"]) == 0
        assert kb.produce("t1", ["m2"]) == 2
        assert kb.list_offset("t1") == 3 and kb.list_offset("t1", latest=False) == 0
        recs, hw = kb.fetch("t1", 1, max_wait_ms=0)
        assert hw == 3 and [(o, v) for o, _, v in recs] == [(1, b"m1"), (2, b"m2")]
        recs, _ = kb.fetch("t1", 3, max_wait_ms=20)          # long poll with nothing new: empty
        assert recs == []
    finally:
        kb.close()
        srv.stop()


def test_ndarray_pubsub_route_over_kafka():
    srv = K.MiniKafkaServer().start()
    kb = K.KafkaBroker(srv.bootstrap)
    try:
        out = streaming.NDArrayConsumer("doubled", kb)
        route = streaming.NDArrayPubSubRoute("raw", "doubled", transform=lambda a: a * 2, broker=kb).start()
        try:
            xs = [torch.arange(12, dtype=torch.float32).reshape(3, 4) + i for i in range(3)]
            streaming.NDArrayPublisher("raw", kb).publish(xs)
            got = out.getArrays(3, timeout=10)
            for g, x in zip(got, xs):
                assert torch.equal(g, x * 2)
        finally:
            route.stop()
            out.close()
    finally:
        kb.close()
        srv.stop()


def test_serve_route_over_kafka(tmp_path):
    net = MultiLayerNetwork(NeuralNetConfiguration.Builder().seed(3).list()
                            .layer(0, DenseLayer.Builder().nIn(4).nOut(8).activation(Activation.TANH).build())
                            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(8).nOut(3)
                                   .activation(Activation.SOFTMAX).build()).build())
    net.init(device="cpu")
    p = str(tmp_path / "m.zip")
    ModelSerializer.writeModel(net, p, False)
    srv = K.MiniKafkaServer().start()
    kb = K.KafkaBroker(srv.bootstrap)
    try:
        outq = streaming.NDArrayConsumer("predictions", kb)
        route = (streaming.DL4jServeRouteBuilder().modelUri(p).consumingTopic("features").outputTopic("predictions")
                 .broker(kb).build().start())
        try:
            x = torch.randn(5, 4)
            streaming.NDArrayPublisher("features", kb).publish(x)
            y = outq.getINDArray(timeout=10)
            assert torch.allclose(y, net.output(x), atol=1e-5)
        finally:
            route.stop()
            outq.close()
    finally:
        kb.close()
        srv.stop()
