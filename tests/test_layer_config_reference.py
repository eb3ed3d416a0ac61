"""Global-vs-layerwise configuration inheritance, after the reference's LayerConfigTest
(deeplearning4j-core/src/test/java/org/deeplearning4j/nn/conf/layers/LayerConfigTest.java:30-300; its learning-rate
and learning-rate-policy tests are commented out in the reference and not ported): layer names, activation, weight
init / distribution / bias init, dropout, Nesterovs momentum schedule, AdaDelta rho / RmsProp decay, Adam betas and
gradient normalization set on the builder reach every layer unless a layer sets its own. CPU."""
import deeplearning4j_amd as D


def _two_dense(builder, l0=None, l1=None):
    l0 = l0 or D.DenseLayer.Builder().nIn(2).nOut(2)
    l1 = l1 or D.DenseLayer.Builder().nIn(2).nOut(2)
    conf = builder.list().layer(0, l0.build()).layer(1, l1.build()).build()
    net = D.MultiLayerNetwork(conf)
    net.init()
    return conf


def _layer(conf, i):
    return conf.getConf(i).getLayer()


def test_layer_name():
    conf = (D.NeuralNetConfiguration.Builder().list()
            .layer(0, D.DenseLayer.Builder().nIn(2).nOut(2).name("genisys").build())
            .layer(1, D.DenseLayer.Builder().nIn(2).nOut(2).name("bill").build()).build())
    net = D.MultiLayerNetwork(conf)
    net.init()
    assert _layer(conf, 0).getLayerName() == "genisys"
    assert _layer(conf, 1).getLayerName() == "bill"


def test_activation_layerwise_override():
    conf = _two_dense(D.NeuralNetConfiguration.Builder().activation(D.Activation.RELU))
    assert str(_layer(conf, 0).getActivationFn()) == "relu"
    assert str(_layer(conf, 1).getActivationFn()) == "relu"
    conf = _two_dense(D.NeuralNetConfiguration.Builder().activation(D.Activation.RELU),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).activation(D.Activation.TANH))
    assert str(_layer(conf, 0).getActivationFn()) == "relu"
    assert str(_layer(conf, 1).getActivationFn()) == "tanh"


def test_weight_bias_init_layerwise_override():
    b = lambda: D.NeuralNetConfiguration.Builder().weightInit(D.WeightInit.DISTRIBUTION) \
        .dist(D.NormalDistribution(0, 1.0)).biasInit(1)  # noqa: E731
    conf = _two_dense(b())
    for i in (0, 1):
        assert _layer(conf, i).getWeightInit() == D.WeightInit.DISTRIBUTION
        assert str(_layer(conf, i).getDist()) == "NormalDistribution{mean=0.0, std=1.0}"
        assert _layer(conf, i).getBiasInit() == 1
    conf = _two_dense(b(), l1=D.DenseLayer.Builder().nIn(2).nOut(2).weightInit(D.WeightInit.DISTRIBUTION)
                      .dist(D.UniformDistribution(0, 1)).biasInit(0))
    assert _layer(conf, 0).getWeightInit() == D.WeightInit.DISTRIBUTION
    assert _layer(conf, 1).getWeightInit() == D.WeightInit.DISTRIBUTION
    assert str(_layer(conf, 0).getDist()) == "NormalDistribution{mean=0.0, std=1.0}"
    assert str(_layer(conf, 1).getDist()) == "UniformDistribution{lower=0.0, upper=1.0}"
    assert _layer(conf, 0).getBiasInit() == 1
    assert _layer(conf, 1).getBiasInit() == 0


def test_dropout_layerwise_override():
    """The reference keeps a no-op Dropout(1.0) object for dropOut(1.0); here a retain probability of 1 (like 0)
    normalises to no dropout, so the fusion planners that need dropout-free layers still apply. The inheritance
    itself is checked with retain probabilities below 1."""
    conf = _two_dense(D.NeuralNetConfiguration.Builder().dropOut(0.9))
    assert _layer(conf, 0).getIDropout() == D.Dropout(0.9)
    assert _layer(conf, 1).getIDropout() == D.Dropout(0.9)
    conf = _two_dense(D.NeuralNetConfiguration.Builder().dropOut(0.9),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).dropOut(0.5))
    assert _layer(conf, 0).getIDropout() == D.Dropout(0.9)
    assert _layer(conf, 1).getIDropout() == D.Dropout(0.5)
    conf = _two_dense(D.NeuralNetConfiguration.Builder().dropOut(1.0))
    assert _layer(conf, 0).getIDropout() is None


def test_momentum_layerwise_override():
    sched = lambda v: D.MapSchedule(D.ScheduleType.ITERATION, {0: v})  # noqa: E731
    conf = _two_dense(D.NeuralNetConfiguration.Builder().updater(D.Nesterovs(1.0, sched(0.1))))
    for i in (0, 1):
        assert _layer(conf, i).getIUpdater().getMomentumISchedule().valueAt(0, 0) == 0.1
    conf = _two_dense(D.NeuralNetConfiguration.Builder().updater(D.Nesterovs(1.0, sched(0.1))),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).updater(D.Nesterovs(1.0, sched(0.2))))
    assert _layer(conf, 0).getIUpdater().getMomentumISchedule().valueAt(0, 0) == 0.1
    assert _layer(conf, 1).getIUpdater().getMomentumISchedule().valueAt(0, 0) == 0.2


def test_updater_rho_rms_decay_layerwise_override():
    conf = _two_dense(D.NeuralNetConfiguration.Builder().updater(D.AdaDelta(0.5, 0.9)),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).updater(D.AdaDelta(0.01, 0.9)))
    assert isinstance(_layer(conf, 0).getIUpdater(), D.AdaDelta)
    assert isinstance(_layer(conf, 1).getIUpdater(), D.AdaDelta)
    assert _layer(conf, 0).getIUpdater().getRho() == 0.5
    assert _layer(conf, 1).getIUpdater().getRho() == 0.01
    conf = _two_dense(D.NeuralNetConfiguration.Builder().updater(D.RmsProp(1.0, 2.0, D.RmsProp.DEFAULT_RMSPROP_EPSILON)),
                      l0=D.DenseLayer.Builder().nIn(2).nOut(2).updater(
                          D.RmsProp(1.0, 1.0, D.RmsProp.DEFAULT_RMSPROP_EPSILON)),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).updater(
                          D.AdaDelta(0.5, D.AdaDelta.DEFAULT_ADADELTA_EPSILON)))
    assert isinstance(_layer(conf, 0).getIUpdater(), D.RmsProp)
    assert isinstance(_layer(conf, 1).getIUpdater(), D.AdaDelta)
    assert _layer(conf, 0).getIUpdater().getRmsDecay() == 1.0
    assert _layer(conf, 1).getIUpdater().getRho() == 0.5


def test_updater_adam_params_layerwise_override():
    conf = _two_dense(D.NeuralNetConfiguration.Builder().updater(D.Adam(1.0, 0.5, 0.5, 1e-8)),
                      l1=D.DenseLayer.Builder().nIn(2).nOut(2).updater(D.Adam(1.0, 0.6, 0.7, 1e-8)))
    assert _layer(conf, 0).getIUpdater().getBeta1() == 0.5
    assert _layer(conf, 1).getIUpdater().getBeta1() == 0.6
    assert _layer(conf, 0).getIUpdater().getBeta2() == 0.5
    assert _layer(conf, 1).getIUpdater().getBeta2() == 0.7


def test_gradient_normalization_layerwise_override():
    gb = lambda: D.NeuralNetConfiguration.Builder().gradientNormalization(  # noqa: E731
        D.GradientNormalization.ClipElementWiseAbsoluteValue).gradientNormalizationThreshold(10)
    conf = _two_dense(gb())
    for i in (0, 1):
        assert _layer(conf, i).getGradientNormalization() == D.GradientNormalization.ClipElementWiseAbsoluteValue
        assert _layer(conf, i).getGradientNormalizationThreshold() == 10
    conf = _two_dense(gb(), l1=D.DenseLayer.Builder().nIn(2).nOut(2)
                      .gradientNormalization(D.GradientNormalization.None_).gradientNormalizationThreshold(2.5))
    assert _layer(conf, 0).getGradientNormalization() == D.GradientNormalization.ClipElementWiseAbsoluteValue
    assert _layer(conf, 1).getGradientNormalization() == D.GradientNormalization.None_
    assert _layer(conf, 0).getGradientNormalizationThreshold() == 10
    assert _layer(conf, 1).getGradientNormalizationThreshold() == 2.5
