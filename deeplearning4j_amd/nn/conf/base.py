"""Serializable configuration objects + DL4J-style fluent builders.

The reference serialises every config (layers, vertices, preprocessors, updaters, activations, losses,
distributions) with Jackson polymorphic subtypes found by classpath scan
(reference nn/conf/NeuralNetConfiguration.java:343-520). Here every config class registers itself in a
global registry under its simple class name and serialises as ``{"@class": Name, ...fields}``;
``from_dict`` resolves the name back through the registry (custom user subclasses register
themselves the same way, which replaces the classpath scan).

Every config class gets an auto-generated ``Builder`` so reference-style code ports verbatim::

    DenseLayer.Builder().nIn(784).nOut(100).activation(Activation.RELU).build()
    ConvolutionLayer.Builder([5, 5], [1, 1]).nOut(20).build()
"""
import copy
import enum
import json

_REGISTRY = {}


def register(cls):
    _REGISTRY[cls.__name__] = cls
    return cls


def lookup(name):
    if name not in _REGISTRY:
        raise KeyError(f"Unknown config class {name!r} (is the module defining it imported?)")
    return _REGISTRY[name]


def _encode(v):
    if isinstance(v, Config):
        return v.to_dict()
    if isinstance(v, enum.Enum):
        return {"@enum": type(v).__name__, "value": v.name}
    if isinstance(v, (list, tuple)):
        return [_encode(x) for x in v]
    if isinstance(v, dict):
        return {"@map": [[_encode(k), _encode(x)] for k, x in v.items()]}
    if isinstance(v, float) and v != v:
        return {"@float": "nan"}
    return v


_ENUMS = {}


def register_enum(cls):
    _ENUMS[cls.__name__] = cls
    return cls


def _decode(v):
    if isinstance(v, dict):
        if "@class" in v:
            return lookup(v["@class"]).from_dict(v)
        if "@enum" in v:
            return _ENUMS[v["@enum"]][v["value"]]
        if "@map" in v:
            return {(_decode(k) if not isinstance(k, list) else tuple(_decode(k))): _decode(x)
                    for k, x in v["@map"]}
        if "@float" in v:
            return float(v["@float"])
        return {k: _decode(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_decode(x) for x in v]
    return v


class _AutoBuilder:
    """Generic fluent builder: every DL4J builder method ``foo(x)`` sets field ``foo``."""

    def __init__(self, cls, *args, **kw):
        object.__setattr__(self, "_cls", cls)
        object.__setattr__(self, "_kw", {})
        if args:
            cls._builder_positional(self._kw, *args)
        for k, v in kw.items():
            self._set(k, v)

    def _set(self, name, value):
        cls = self._cls
        name = cls._ALIASES.get(name, name)
        if name not in cls._all_fields():
            raise AttributeError(f"{cls.__name__}.Builder has no property {name!r}")
        dist_field = {"weightInit": "dist", "weightInitRecurrent": "distRecurrent"}.get(name)
        if dist_field is not None and dist_field in cls._all_fields():
            from .weights import Distribution, WeightInit
            if isinstance(value, Distribution):       # layer.weightInit(dist) == dist(d) + WeightInit.DISTRIBUTION
                self._kw[dist_field] = value
                value = WeightInit.DISTRIBUTION
        conv = cls._CONVERTERS.get(name)
        self._kw[name] = conv(value) if conv else value

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)

        def setter(*vals, **kw):
            if kw:
                raise TypeError("builder setters take positional values only")
            if len(vals) == 0:
                val = True
            elif len(vals) == 1:
                val = vals[0]
            else:
                val = list(vals)
            hook = getattr(self._cls, "_builder_hook_" + name, None)
            if hook is not None:
                hook(self._kw, val)
            else:
                self._set(name, val)
            return self
        return setter

    def build(self):
        return self._cls(**self._kw)


class _BuilderDescriptor:
    def __get__(self, obj, cls):
        def make(*args, **kw):
            return _AutoBuilder(cls, *args, **kw)
        return make


class Config:
    """Base of every serialisable config. Subclasses declare ``FIELDS = {name: default}``."""
    FIELDS = {}
    _ALIASES = {}
    _CONVERTERS = {}
    Builder = _BuilderDescriptor()

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        register(cls)
        cls._fields_cache = None

    @classmethod
    def _all_fields(cls):
        if cls.__dict__.get("_fields_cache") is None:
            fields = {}
            for klass in reversed(cls.__mro__):
                fields.update(getattr(klass, "FIELDS", {}) if "FIELDS" in klass.__dict__ else {})
            cls._fields_cache = fields
        return cls._fields_cache

    @classmethod
    def _builder_positional(cls, kw, *args):
        raise TypeError(f"{cls.__name__}.Builder takes no positional arguments")

    def __init__(self, **kw):
        fields = self._all_fields()
        for k, d in fields.items():
            setattr(self, k, copy.deepcopy(d))
        for k, v in kw.items():
            k = self._ALIASES.get(k, k)
            if k not in fields:
                raise TypeError(f"{type(self).__name__} has no property {k!r}")
            dist_field = {"weightInit": "dist", "weightInitRecurrent": "distRecurrent"}.get(k)
            if dist_field in fields and dist_field not in kw:
                from .weights import Distribution, WeightInit
                if isinstance(v, Distribution):
                    setattr(self, dist_field, v)
                    v = WeightInit.DISTRIBUTION
            conv = self._CONVERTERS.get(k)
            setattr(self, k, conv(v) if conv and v is not None else v)
        self._post_init()

    def _post_init(self):
        pass

    _GETTER_ALIASES = {"IUpdater": "updater", "ActivationFn": "activation", "LossFn": "lossFn",
                       "LossFunction": "lossFn", "Dist": "dist"}

    def __getattr__(self, name):
        """Java-style getters for every field (``getL2()``, ``getIUpdater()``, ``getMomentum()``, ``isX()``), as the
        reference's Lombok-generated accessors. Only reached when normal attribute lookup fails."""
        if name.startswith("_") or not (name.startswith("get") or name.startswith("is") or name.startswith("set")) \
                or len(name) < 3:
            raise AttributeError(name)
        setter = name.startswith("set")
        stem = name[3:] if name.startswith(("get", "set")) else name[2:]
        if not stem:
            raise AttributeError(name)
        fields = type(self)._all_fields()
        field = self._GETTER_ALIASES.get(stem)
        if field is None:
            for cand in (stem[0].lower() + stem[1:], stem, stem.lower()):
                cand = self._ALIASES.get(cand, cand)
                if cand in fields:
                    field = cand
                    break
        if field is None or field not in fields:
            raise AttributeError(f"{type(self).__name__} has no attribute {name!r}")
        if setter:
            conv = self._CONVERTERS.get(field)

            def _set(v):
                setattr(self, field, conv(v) if conv and v is not None else v)
            return _set
        return lambda: self.__dict__.get(field)

    # --- serde -------------------------------------------------------------------------------
    def to_dict(self):
        d = {"@class": type(self).__name__}
        for k in sorted(self._all_fields()):
            d[k] = _encode(getattr(self, k))
        return d

    @classmethod
    def from_dict(cls, d):
        obj = cls.__new__(cls)
        fields = cls._all_fields()
        for k, dflt in fields.items():
            setattr(obj, k, copy.deepcopy(dflt))
        for k, v in d.items():
            if k == "@class":
                continue
            if k in fields:          # ignore unknown properties (reference: FAIL_ON_UNKNOWN_PROPERTIES=false)
                setattr(obj, k, _decode(v))
        obj._post_init()
        return obj

    def toJson(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True)

    @classmethod
    def fromJson(cls, s):
        return _decode(json.loads(s))

    def clone(self):
        return copy.deepcopy(self)

    def __eq__(self, other):
        return type(self) is type(other) and self.to_dict() == other.to_dict()

    def __hash__(self):
        return hash(json.dumps(self.to_dict(), sort_keys=True, default=str))

    def __repr__(self):
        items = ", ".join(f"{k}={getattr(self, k)!r}" for k in sorted(self._all_fields())
                          if getattr(self, k) is not None)
        return f"{type(self).__name__}({items})"


def int_pair(v):
    if v is None:
        return None
    if isinstance(v, int):
        return [v, v]
    return [int(x) for x in v]


def int_list(v):
    if v is None:
        return None
    if isinstance(v, int):
        return [v]
    return [int(x) for x in v]
