"""Network conversions (reference NN:nn/multilayer/MultiLayerNetwork.toComputationGraph ->
NN:util/NetworkUtils.java toComputationGraph)."""
import copy

from ..nn.conf.graph import LayerVertex
from ..nn.conf.network import ComputationGraphConfiguration


def to_computation_graph(mln):
    """The same network as a ComputationGraph: vertices ``layer0 .. layerN-1`` chained from input ``in`` with the
    MLN's input preprocessors, identical flat parameter layout (the chain's topological order is the layer order),
    parameters and updater state copied."""
    from ..nn.graph.computation_graph import ComputationGraph
    conf = mln.conf
    n = len(conf.confs)
    names = [f"layer{i}" for i in range(n)]
    vertices, inputs = {}, {}
    for i, lc in enumerate(conf.confs):
        lc = copy.deepcopy(lc)
        if lc.layerName is None:
            lc.layerName = names[i]
        vertices[names[i]] = LayerVertex(layerConf=lc, preProcessor=copy.deepcopy(conf.inputPreProcessors.get(i)))
        inputs[names[i]] = ["in" if i == 0 else names[i - 1]]
    cg_conf = ComputationGraphConfiguration(
        vertices=vertices, vertexInputs=inputs, networkInputs=["in"], networkOutputs=[names[-1]],
        backprop=conf.backprop, pretrain=conf.pretrain, backpropType=conf.backpropType,
        tbpttFwdLength=conf.tbpttFwdLength, tbpttBackLength=conf.tbpttBackLength,
        globalConf=copy.deepcopy(conf.globalConf), iterationCount=conf.iterationCount, epochCount=conf.epochCount,
        inputTypes=[conf.inputType] if getattr(conf, "inputType", None) is not None else None)
    cg = ComputationGraph(cg_conf)
    if not mln.initCalled:
        mln.init()
    cg.init(mln.params().detach().clone().reshape(-1), device=mln.device)
    st = mln.updater.getStateViewArray() if mln.updater is not None else None
    if st is not None and st.numel() > 0:
        cg.updater.setStateViewArray(st.clone())
    return cg
