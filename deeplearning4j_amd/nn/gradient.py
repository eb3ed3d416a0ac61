"""Gradient container (reference nn/gradient/{Gradient,DefaultGradient}.java): an ordered map
variable-name -> gradient view (keys "<layerIdx>_<param>" in MLN, "<vertexName>_<param>" in CG)."""
from collections import OrderedDict


class Gradient:
    def __init__(self, flat=None):
        self._map = OrderedDict()
        self._flat = flat

    def gradientForVariable(self):
        return self._map

    def setGradientFor(self, key, arr, order=None):
        self._map[key] = arr
        return arr

    def getGradientFor(self, key):
        return self._map.get(key)

    def gradient(self):
        return self._flat

    def setFlattenedGradient(self, flat):
        self._flat = flat

    def clear(self):
        self._map.clear()

    def __getitem__(self, k):
        return self._map[k]

    def __contains__(self, k):
        return k in self._map

    def keys(self):
        return self._map.keys()

    def items(self):
        return self._map.items()


DefaultGradient = Gradient
