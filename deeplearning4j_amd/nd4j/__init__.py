"""ND4J-compatible array API (``INDArray``, ``Nd4j``, ``NDArrayIndex``, ``Transforms``, ``AffinityManager``)."""
from .factory import AffinityManager, Nd4j  # noqa: F401
from .ndarray import INDArray, NDArrayIndex, Transforms  # noqa: F401
