"""Configuration and input validation (reference CORET:exceptions/TestInvalidConfigurations.java and
TestInvalidInput.java; NN:nn/conf/layers/LayerValidation.java, NN:nn/layers/BaseLayer.java preOutput checks).

``validate_network_conf(confs)`` runs when a network is initialised (after nIn inference from the InputType);
``check_layer_input(conf, x, where)`` runs on the host before each layer's forward: shape comparisons only, no
device synchronisation (embedding index ranges are checked for host tensors only)."""
from ...exceptions import DL4JInvalidConfigException, DL4JInvalidInputException


def _name(conf, where):
    n = getattr(conf, "layerName", None)
    return f"layer {where}" + (f" ({n})" if n else "") + f", {type(conf).__name__}"


def _sized(conf):
    """Layers whose parameters are sized by nIn / nOut (both must be positive once the network is built)."""
    from .layers import (BaseOutputLayer, BaseRecurrentLayer, ConvolutionLayer, DenseLayer, EmbeddingLayer)
    return isinstance(conf, (DenseLayer, BaseOutputLayer, BaseRecurrentLayer, ConvolutionLayer, EmbeddingLayer))


def validate_layer_conf(conf, where):
    if _sized(conf):
        nin, nout = getattr(conf, "nIn", None), getattr(conf, "nOut", None)
        if not nin or nin <= 0:
            raise DL4JInvalidConfigException(f"{_name(conf, where)}: nIn = {nin} (must be > 0; set nIn or give the "
                                             f"network an InputType so it can be inferred)")
        if not nout or nout <= 0:
            raise DL4JInvalidConfigException(f"{_name(conf, where)}: nOut = {nout} (must be > 0)")
    inner = getattr(conf, "underlying", None)
    if inner is not None and hasattr(inner, "nIn"):
        validate_layer_conf(inner, where)


def validate_network_conf(confs):
    for i, c in (confs.items() if isinstance(confs, dict) else enumerate(confs)):
        validate_layer_conf(c, i)


def validate_kernel_geometry(conf, ndim=2):
    """Builder-time check of a convolution / subsampling layer (reference ConvolutionUtils.validateCnnKernelStridePadding:
    IllegalStateException): exactly ``ndim`` kernel / stride / padding values, kernel and stride > 0, padding >= 0."""
    for field, lo in (("kernelSize", 1), ("stride", 1), ("padding", 0), ("dilation", 1)):
        v = getattr(conf, field, None)
        if v is None:
            continue
        v = list(v) if isinstance(v, (list, tuple)) else [v]
        if len(v) != ndim:
            raise DL4JInvalidConfigException(f"{type(conf).__name__}: {field} needs {ndim} values, got {v}")
        if any(int(a) < lo for a in v):
            raise DL4JInvalidConfigException(f"{type(conf).__name__}: invalid {field} {v} (values must be "
                                             f"{'>= 0' if lo == 0 else '> 0'})")


def check_layer_input(conf, x, where):
    """Shape checks of a layer's input against its configuration; raises DL4JInvalidInputException."""
    from .layers import (BaseOutputLayer, BaseRecurrentLayer, BaseWrapperLayer, BatchNormalization,
                         Convolution1DLayer, ConvolutionLayer, DenseLayer, EmbeddingLayer, EmbeddingSequenceLayer,
                         Subsampling1DLayer, SubsamplingLayer)
    nin = getattr(conf, "nIn", None)
    if isinstance(conf, Convolution1DLayer) or isinstance(conf, Subsampling1DLayer):
        if x.dim() != 3:
            raise DL4JInvalidInputException(f"{_name(conf, where)}: expected a rank 3 [minibatch, channels, time] "
                                            f"input, got shape {tuple(x.shape)}")
        if isinstance(conf, Convolution1DLayer) and nin and x.shape[1] != nin:
            raise DL4JInvalidInputException(f"{_name(conf, where)}: input has {x.shape[1]} channels, layer nIn = "
                                            f"{nin}")
        _check_spatial(conf, (x.shape[2],), where)
        return
    if isinstance(conf, (ConvolutionLayer, SubsamplingLayer)):
        if x.dim() != 4:
            raise DL4JInvalidInputException(
                f"{_name(conf, where)}: expected a rank 4 [minibatch, channels, height, width] input, got shape "
                f"{tuple(x.shape)} (a flattened image needs InputType.convolutionalFlat or a preprocessor)")
        if isinstance(conf, ConvolutionLayer) and nin and x.shape[1] != nin:
            raise DL4JInvalidInputException(f"{_name(conf, where)}: input depth {x.shape[1]} does not match the "
                                            f"layer's nIn (depth) {nin}")
        _check_spatial(conf, (x.shape[2], x.shape[3]), where)
        return
    if isinstance(conf, EmbeddingLayer):
        if isinstance(conf, EmbeddingSequenceLayer):
            if x.dim() not in (2, 3) or (x.dim() == 3 and x.shape[1] != 1):
                raise DL4JInvalidInputException(f"{_name(conf, where)}: expected [minibatch, T] or [minibatch, 1, T] "
                                                f"indices, got shape {tuple(x.shape)}")
        elif not (x.dim() == 1 or (x.dim() == 2 and x.shape[1] == 1)):
            raise DL4JInvalidInputException(f"{_name(conf, where)}: expected [minibatch, 1] indices, got shape "
                                            f"{tuple(x.shape)}")
        if nin and not x.is_cuda and x.numel():
            lo, hi = float(x.min()), float(x.max())
            if lo < 0 or hi >= nin:
                raise DL4JInvalidInputException(f"{_name(conf, where)}: index {int(hi if hi >= nin else lo)} outside "
                                                f"[0, nIn = {nin})")
        return
    if isinstance(conf, BaseRecurrentLayer):
        if x.dim() not in (2, 3):
            raise DL4JInvalidInputException(f"{_name(conf, where)}: expected a rank 3 [minibatch, size, time] "
                                            f"input, got shape {tuple(x.shape)}")
        if nin and x.shape[1] != nin:
            raise DL4JInvalidInputException(f"{_name(conf, where)}: input size {x.shape[1]} does not match the "
                                            f"layer's nIn {nin}")
        return
    if isinstance(conf, BaseWrapperLayer) and conf.underlying is not None:
        check_layer_input(conf.underlying, x, where)
        return
    if isinstance(conf, (DenseLayer, BaseOutputLayer)) and nin and x.dim() in (2, 3) and x.shape[1] != nin:
        raise DL4JInvalidInputException(f"{_name(conf, where)}: input has {x.shape[1]} features, layer nIn = {nin}")
    if isinstance(conf, BatchNormalization) and nin and x.dim() >= 2 and x.shape[1] != nin:
        raise DL4JInvalidInputException(f"{_name(conf, where)}: input has {x.shape[1]} channels, layer nIn = {nin}")


def _check_spatial(conf, sizes, where):
    """Output size of every spatial dim under the layer's ConvolutionMode (reference ConvolutionUtils.getOutputSize:
    DL4JInvalidInputException for data smaller than the kernel or, in Strict mode, sizes the stride does not
    divide). Transposed convolutions grow their input and are not checked here."""
    from .enums import ConvolutionMode
    from .layers import Deconvolution2D, conv_out_size
    if isinstance(conf, Deconvolution2D):
        return
    mode = conf.convolutionMode or ConvolutionMode.Truncate
    for d, n in enumerate(sizes):
        try:
            conv_out_size(int(n), conf.kernelSize[d], conf.stride[d], conf.padding[d], conf.dilation[d], mode)
        except DL4JInvalidConfigException as e:
            raise DL4JInvalidInputException(f"{_name(conf, where)}: input size {tuple(sizes)} is invalid for this "
                                            f"layer: {e}") from None


def check_labels(conf, labels, where):
    """Label width vs the output layer's nOut (reference: IllegalArgumentException from the loss function)."""
    nout = getattr(conf, "nOut", None)
    if labels is None or not nout or labels.dim() < 2:
        return
    if labels.shape[1] != nout:
        raise ValueError(f"{_name(conf, where)}: labels have {labels.shape[1]} columns, the output layer has "
                         f"nOut = {nout}")
