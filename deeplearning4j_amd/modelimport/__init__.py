"""Model import: Keras 1.x/2.x HDF5/JSON models (keras.py) read through a dependency-free HDF5 parser (hdf5.py)."""
from .keras import (InvalidKerasConfigurationException, KerasLayer, KerasModel, KerasModelImport,  # noqa: F401
                    UnsupportedKerasConfigurationException, space_to_depth_mapper)
