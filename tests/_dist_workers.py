"""Worker bodies for the multi-process (gloo, world_size 2) data-parallel tests in test_parallel.py."""
import os

import torch
import torch.distributed as dist


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def make_net(updater):
    from deeplearning4j_amd import (Activation, DenseLayer, LossFunction, MultiLayerNetwork, NeuralNetConfiguration,
                                    OutputLayer)
    conf = (NeuralNetConfiguration.Builder().seed(11).updater(updater).l2(1e-3).list()
            .layer(0, DenseLayer.Builder().nIn(5).nOut(12).activation(Activation.TANH).build())
            .layer(1, OutputLayer.Builder(LossFunction.MCXENT).nIn(12).nOut(3).activation(Activation.SOFTMAX).build())
            .build())
    net = MultiLayerNetwork(conf)
    net.init(device=torch.device("cpu"))
    return net


def make_batches(n_batches, bs, seed=5):
    from deeplearning4j_amd import DataSet
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        x = torch.randn(bs, 5, generator=g)
        y = torch.zeros(bs, 3)
        y[torch.arange(bs), torch.randint(0, 3, (bs,), generator=g)] = 1
        out.append(DataSet(x, y))
    return out


def run_mode(rank, world, port, mode, result_path):
    _setup(rank, world, port)
    from deeplearning4j_amd import Adam, ListDataSetIterator
    from deeplearning4j_amd.parallel import EncodedGradientsAccumulator, ParallelWrapper, TrainingMode
    net = make_net(Adam(0.01) if mode != "encoded" else Adam(0.5))
    if rank == 1:                                   # replicas must be synchronised from rank 0 by the wrapper
        with torch.no_grad():
            net.flattenedParams.add_(1.0)
    batches = make_batches(8, 8)
    it = ListDataSetIterator(batches, 8)
    b = ParallelWrapper.Builder(net)
    if mode == "shared":
        b.trainingMode(TrainingMode.SHARED_GRADIENTS)
    elif mode == "averaging":
        b.trainingMode(TrainingMode.AVERAGING).averagingFrequency(2).averageUpdaters(True)
    elif mode == "encoded":
        b.gradientsAccumulator(EncodedGradientsAccumulator(threshold=1e-3))
    elif mode in ("ctx_default", "ctx_sym", "ctx_ps"):
        from deeplearning4j_amd.parallel import (DefaultTrainerContext, ParameterServerTrainerContext,
                                                 SymmetricTrainerContext)
        ctx = {"ctx_default": DefaultTrainerContext(), "ctx_sym": SymmetricTrainerContext(),
               "ctx_ps": ParameterServerTrainerContext()}[mode]
        b.trainerFactory(ctx).averagingFrequency(2)
    pw = b.build()
    pw.fit(it, 2)
    p = net.params().clone()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        torch.save({"params": [t.clone() for t in gathered], "iters": net.getIterationCount()}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def run_cluster(rank, world, port, master, result_path):
    """Cluster training masters (the dl4j-spark replacement) on a gloo process group."""
    _setup(rank, world, port)
    from deeplearning4j_amd import Adam
    from deeplearning4j_amd.parallel.cluster import (ParameterAveragingTrainingMaster, SharedTrainingMaster,
                                                     SparkDl4jMultiLayer, StatsUtils)
    net = make_net(Adam(0.01))
    if rank == 1:
        with torch.no_grad():
            net.flattenedParams.add_(1.0)
    if master == "paramavg":
        tm = ParameterAveragingTrainingMaster.Builder(1).batchSizePerWorker(8).averagingFrequency(2) \
            .collectTrainingStats(True).build()
    else:
        tm = SharedTrainingMaster.Builder(1e-3).batchSizePerWorker(8).build()
    spark = SparkDl4jMultiLayer(None, net, tm)
    data = make_batches(8, 8)
    spark.fit(data, 2)
    ev = spark.evaluate(data)
    score = spark.calculateScore(data)
    p = net.params().clone()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        if master == "paramavg":
            StatsUtils.exportStatsAsHtml(tm.getTrainingStats(), result_path + ".html")
        torch.save({"params": [t.clone() for t in gathered], "n_eval": int(ev.getNumRowCounter()),
                    "score": score, "acc": float(ev.accuracy())}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def run_w2v(rank, world, port, result_path):
    """Distributed Word2Vec: each rank trains on its shard; the averaged tables must be identical on both ranks and
    still separate the two topic clusters of the synthetic corpus."""
    _setup(rank, world, port)
    import numpy as np
    from deeplearning4j_amd.nlp import CollectionSentenceIterator, Word2Vec
    from deeplearning4j_amd.nlp.distributed import DistributedWord2Vec
    rng = np.random.RandomState(3)
    A = [f"alpha{i}" for i in range(10)]
    B = [f"beta{i}" for i in range(10)]
    corpus = [" ".join(rng.choice(A if k % 2 == 0 else B, 12)) for k in range(600)]
    shard = corpus[rank::world]
    w2v = Word2Vec.Builder().minWordFrequency(1).layerSize(24).windowSize(4).seed(7).epochs(3) \
        .iterate(CollectionSentenceIterator(shard)).device("cpu").build()
    DistributedWord2Vec(w2v).fit()
    syn0 = w2v.lookupTable().getSyn0().clone()
    gathered = [torch.empty_like(syn0) for _ in range(world)]
    dist.all_gather(gathered, syn0)
    if rank == 0:
        same = all(torch.equal(gathered[0], g) for g in gathered[1:])
        sim_in = w2v.similarity("alpha1", "alpha2")
        sim_out = w2v.similarity("alpha1", "beta2")
        torch.save({"same": same, "in": sim_in, "out": sim_out, "n": w2v.vocab().numWords()}, result_path)
    dist.destroy_process_group()


def run_es_parallel(rank, world, port, result_path):
    """EarlyStoppingParallelTrainer over 2 gloo ranks: replicas must end identical and agree on termination."""
    _setup(rank, world, port)
    from deeplearning4j_amd import Adam, ListDataSetIterator
    from deeplearning4j_amd.earlystopping import (DataSetLossCalculator, EarlyStoppingConfiguration,
                                                  EarlyStoppingParallelTrainer, InMemoryModelSaver,
                                                  MaxEpochsTerminationCondition)
    net = make_net(Adam(0.02))
    train = ListDataSetIterator(make_batches(7, 8), 8)          # 7 batches: trailing partial group dropped
    val = ListDataSetIterator(make_batches(2, 16, seed=9), 16)
    conf = (EarlyStoppingConfiguration.Builder().epochTerminationConditions(MaxEpochsTerminationCondition(3))
            .scoreCalculator(DataSetLossCalculator(val, True)).modelSaver(InMemoryModelSaver()).build())
    res = EarlyStoppingParallelTrainer(conf, net, train).fit()
    p = net.params().clone()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        torch.save({"params": [t.clone() for t in gathered], "iters": net.getIterationCount(),
                    "epochs": res.getTotalEpochs(), "scores": dict(res.getScoreVsEpoch())}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def make_cg(seed=3, device=None, dtype=None):
    """Residual conv ComputationGraph (no BatchNorm, so DP-2 equals one process at 2x batch exactly). ``dtype``
    (a DataType) sets the network compute dtype; bf16 puts c2 on the MFMA conv kernels and its weight gradient on
    the overlap stream."""
    from deeplearning4j_amd import Activation, Adam, LossFunction, NeuralNetConfiguration
    from deeplearning4j_amd.nn.conf.graph import ElementWiseVertex
    from deeplearning4j_amd.nn.conf.inputs import InputType
    from deeplearning4j_amd.nn.conf.layers import ConvolutionLayer, GlobalPoolingLayer, OutputLayer
    from deeplearning4j_amd.nn.graph.computation_graph import ComputationGraph
    b = NeuralNetConfiguration.Builder().seed(seed).updater(Adam(0.01))
    if dtype is not None:
        b = b.dataType(dtype)
    conf = (b.graphBuilder()
            .addInputs("in")
            .addLayer("c1", ConvolutionLayer.Builder(3, 3).nIn(3).nOut(8).padding(1, 1)
                      .activation(Activation.RELU).build(), "in")
            .addLayer("c2", ConvolutionLayer.Builder(3, 3).nIn(8).nOut(8).padding(1, 1)
                      .activation(Activation.IDENTITY).build(), "c1")
            .addVertex("add", ElementWiseVertex(ElementWiseVertex.Op.Add), "c1", "c2")
            .addLayer("gap", GlobalPoolingLayer.Builder().build(), "add")
            .addLayer("out", OutputLayer.Builder(LossFunction.MCXENT).nIn(8).nOut(4)
                      .activation(Activation.SOFTMAX).build(), "gap")
            .setOutputs("out").setInputTypes(InputType.convolutional(8, 8, 3)).build())
    net = ComputationGraph(conf)
    net.init(device=device or torch.device("cpu"))
    return net


def make_image_batches(n, bs, seed=21):
    from deeplearning4j_amd import DataSet
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        x = torch.randn(bs, 3, 8, 8, generator=g)
        y = torch.zeros(bs, 4)
        y[torch.arange(bs), torch.randint(0, 4, (bs,), generator=g)] = 1
        out.append(DataSet(x, y))
    return out


def run_cg_shared(rank, world, port, result_path):
    """SHARED_GRADIENTS on a ComputationGraph with small buckets (several all-reduces overlapped with backward)."""
    _setup(rank, world, port)
    from deeplearning4j_amd.parallel import ParallelWrapper, TrainingMode
    net = make_cg()
    if rank == 1:
        with torch.no_grad():
            net.flattenedParams.add_(0.5)
    pw = ParallelWrapper.Builder(net).trainingMode(TrainingMode.SHARED_GRADIENTS).bucketSizeMB(0.0005).build()
    pw.fit(make_image_batches(6, 4), 1)
    p = net.params().clone()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        torch.save({"params": [t.clone() for t in gathered], "nbuckets": len(pw.accumulator._buckets)}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def make_samediff(seed=4):
    from deeplearning4j_amd import Sgd
    from deeplearning4j_amd.samediff import SameDiff, TrainingConfig
    g = torch.Generator().manual_seed(seed)
    sd = SameDiff.create()
    x = sd.placeHolder("x", torch.zeros(4, 6))
    y = sd.placeHolder("y", torch.zeros(4, 3))
    w0 = sd.var("w0", torch.randn(6, 8, generator=g) * 0.4)
    b0 = sd.var("b0", torch.zeros(8))
    w1 = sd.var("w1", torch.randn(8, 3, generator=g) * 0.4)
    h = sd.nn().tanh(sd.nn().linear(x, w0, b0))
    sd.loss().softmaxCrossEntropy("loss", y, h.mmul(w1))
    sd.setTrainingConfig(TrainingConfig.builder().updater(Sgd(0.2)).dataSetFeatureMapping("x")
                         .dataSetLabelMapping("y").build())
    return sd


def samediff_batches(n=5, bs=8, seed=9):
    from deeplearning4j_amd import DataSet
    g = torch.Generator().manual_seed(seed)
    return [DataSet(torch.randn(bs, 6, generator=g),
                    torch.nn.functional.one_hot(torch.randint(0, 3, (bs,), generator=g), 3).float()) for _ in range(n)]


def run_samediff_dp(rank, world, port, result_path):
    """SameDiff fit with the flat gradient all-reduced across ranks (samediff.SameDiff._allreduce)."""
    _setup(rank, world, port)
    from deeplearning4j_amd import DataSet
    sd = make_samediff()
    for ds in samediff_batches():
        h = ds.features.shape[0] // world
        sd.fit(DataSet(ds.features[rank * h:(rank + 1) * h], ds.labels[rank * h:(rank + 1) * h]))
    p = torch.cat([v.value.reshape(-1) for v in sd.trainableVariables()])
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        torch.save({"params": [t.clone() for t in gathered],
                    "nbuckets": len(sd._train_state["dp"].buckets)}, result_path)
    dist.barrier()
    dist.destroy_process_group()


def simulate_averaging(make, batches, world, freq, epochs, average_updaters=True):
    """Reference semantics of AVERAGING (PW:ParallelWrapper.java:316-376) computed in one process: ``world``
    replicas from the same init, replica r fits batches r, r+W, ... of each epoch, and after every ``freq`` rounds
    parameters (+ updater state) are replaced by their mean; a final average if the last round was not one."""
    reps = [make() for _ in range(world)]
    base = reps[0].params().clone()
    for n in reps[1:]:
        n.setParams(base.clone())
    rnd = 0
    nr = len(batches) // world
    for _ in range(epochs):
        for k in range(nr):
            for r in range(world):
                reps[r].fit(batches[k * world + r])
            rnd += 1
            if rnd % freq == 0:
                _avg(reps, average_updaters)
    if rnd % freq:
        _avg(reps, average_updaters)
    return reps[0].params().clone()


def _avg(reps, average_updaters):
    p = sum(n.params() for n in reps) / len(reps)
    for n in reps:
        n.setParams(p.clone())
    if average_updaters:
        st = sum(n.updater.getStateViewArray() for n in reps) / len(reps)
        for n in reps:
            n.updater.getStateViewArray().copy_(st)


def run_mode4(rank, world, port, mode, result_path):
    """world-4 gloo runs: AVERAGING with averagingFrequency 3 (12 batches = 3 rounds per epoch, 2 epochs) and the
    encoded (threshold) update sharing."""
    _setup(rank, world, port)
    from deeplearning4j_amd import Adam, ListDataSetIterator
    from deeplearning4j_amd.parallel import EncodedGradientsAccumulator, ParallelWrapper, TrainingMode
    net = make_net(Adam(0.01) if mode != "encoded" else Adam(0.5))
    batches = make_batches(12, 8)
    it = ListDataSetIterator(batches, 8)
    b = ParallelWrapper.Builder(net)
    if mode == "averaging3":
        b.trainingMode(TrainingMode.AVERAGING).averagingFrequency(3).averageUpdaters(True)
    elif mode == "encoded":
        b.gradientsAccumulator(EncodedGradientsAccumulator(threshold=1e-3))
    pw = b.build()
    pw.fit(it, 2)
    p = net.params().clone()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p)
    if rank == 0:
        torch.save({"params": [t.clone() for t in gathered], "iters": net.getIterationCount()}, result_path)
    dist.barrier()
    dist.destroy_process_group()
