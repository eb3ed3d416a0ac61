"""DL4J exception hierarchy (reference NN:exception/DL4JException.java, DL4JInvalidConfigException.java,
DL4JInvalidInputException.java): configuration errors found when a network is built / initialised and input errors
found when data reaches a layer, each naming the layer and the offending sizes. Both also derive from ValueError, so
code that catches the Python convention keeps working."""


class DL4JException(RuntimeError):
    """Base of the framework's own exceptions."""


class DL4JInvalidConfigException(DL4JException, ValueError):
    """A configuration that cannot work (nIn / nOut of 0, non-positive kernel or stride, negative padding,
    ConvolutionMode.Strict with sizes that do not divide, an input smaller than the kernel)."""


class DL4JInvalidInputException(DL4JException, ValueError):
    """Data that does not match the network (feature count vs nIn, rank of a CNN / RNN input, label width vs nOut,
    embedding indices outside [0, nIn))."""


class InvalidInputTypeException(DL4JInvalidConfigException):
    """An InputType that a layer cannot take, found while shapes are inferred at build time (reference
    nn/conf/inputs/InvalidInputTypeException.java), e.g. a convolution kernel larger than the padded input."""


class UnsupportedOperationException(DL4JException, NotImplementedError):
    """java.lang.UnsupportedOperationException: a configured feature the engine refuses (e.g. HESSIAN_FREE)."""


class IllegalStateException(DL4JException, ValueError):
    """java.lang.IllegalStateException: an array whose shape contradicts the state a component was configured with
    (e.g. a CNN-to-feed-forward preprocessor fed [mb, C, W, H] instead of [mb, C, H, W])."""
