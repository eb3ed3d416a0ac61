"""ModelSerializer: the reference's checkpoint ZIP format (reference NN:util/ModelSerializer.java:51-690).

ZIP entries:
  configuration.json   network configuration JSON (includes iteration/epoch counts)
  coefficients.bin     flat parameters [1, P], ND4J binary format (utils.nd4j_io)
  updaterState.bin     flat updater state [1, S] (optional; exact Adam/RmsProp resume)
  normalizer.bin       data normalizer (optional)
  noParams.marker      present when the network has no parameters
Extras written by this framework (ignored by readers that do not know them):
  rngState.bin         torch RNG state (optional, for exact resume)
"""
import io
import json
import os
import zipfile

import torch

from . import nd4j_io

CONFIG = "configuration.json"
COEFFS = "coefficients.bin"
UPDATER = "updaterState.bin"
NORMALIZER = "normalizer.bin"
NO_PARAMS = "noParams.marker"
PREPROCESSOR = "preprocessor.bin"


def _open_out(f):
    if isinstance(f, (str, os.PathLike)):
        return open(f, "wb"), True
    return f, False


def _config_from_json(text):
    """configuration.json in DL4J's Jackson schema (nn/conf/dl4j_json.py) or this framework's earlier tagged form."""
    from ..nn.conf.base import _decode
    from ..nn.conf.dl4j_json import from_json, is_dl4j_format
    d = json.loads(text)
    return from_json(d) if is_dl4j_format(d) else _decode(d)


class ModelSerializer:
    @staticmethod
    def writeModel(model, f, saveUpdater=True, dataNormalization=None):
        fh, close = _open_out(f)
        try:
            with zipfile.ZipFile(fh, "w", zipfile.ZIP_DEFLATED) as z:
                z.writestr(CONFIG, model.conf.toJson())
                if model.numParams() > 0:
                    z.writestr(COEFFS, nd4j_io.to_bytes(model.params()))
                else:
                    z.writestr(NO_PARAMS, b"")
                if saveUpdater and model.updater is not None and model.updater.state is not None and \
                        model.updater.state.numel() > 0:
                    z.writestr(UPDATER, nd4j_io.to_bytes(model.updater.getStateViewArray()))
                if dataNormalization is not None:
                    z.writestr(NORMALIZER, dataNormalization.to_bytes())
        finally:
            if close:
                fh.close()

    # --------------------------------------------------------------------------------- restore
    @staticmethod
    def _read(f):
        if isinstance(f, (str, os.PathLike)):
            with open(f, "rb") as fh:
                data = fh.read()
        else:
            data = f.read()
        return zipfile.ZipFile(io.BytesIO(data))

    @staticmethod
    def _restore(f, loadUpdater, kind, device=None):
        z = ModelSerializer._read(f)
        names = set(z.namelist())
        if CONFIG not in names:
            raise ValueError("Invalid model file: no configuration.json")
        cfg = _config_from_json(z.read(CONFIG).decode("utf-8"))
        from ..nn.conf.network import ComputationGraphConfiguration, MultiLayerConfiguration
        if kind == "mln" and not isinstance(cfg, MultiLayerConfiguration):
            raise ValueError("File does not contain a MultiLayerNetwork (use restoreComputationGraph)")
        if kind == "cg" and not isinstance(cfg, ComputationGraphConfiguration):
            raise ValueError("File does not contain a ComputationGraph (use restoreMultiLayerNetwork)")
        params = None
        if COEFFS in names:
            params = nd4j_io.from_bytes(z.read(COEFFS)).reshape(-1)
        if isinstance(cfg, MultiLayerConfiguration):
            from ..nn.multilayer import MultiLayerNetwork
            net = MultiLayerNetwork(cfg)
        else:
            from ..nn.graph import ComputationGraph
            net = ComputationGraph(cfg)
        net.init(params, device=device)
        if loadUpdater and UPDATER in names:
            net.updater.setStateViewArray(nd4j_io.from_bytes(z.read(UPDATER)))
        net._normalizer = None
        if NORMALIZER in names:
            from ..datasets.normalizers import DataNormalization
            net._normalizer = DataNormalization.from_bytes(z.read(NORMALIZER))
        return net

    @staticmethod
    def restoreMultiLayerNetwork(f, loadUpdater=True, device=None):
        return ModelSerializer._restore(f, loadUpdater, "mln", device)

    @staticmethod
    def restoreComputationGraph(f, loadUpdater=True, device=None):
        return ModelSerializer._restore(f, loadUpdater, "cg", device)

    @staticmethod
    def restoreModel(f, loadUpdater=True, device=None):
        return ModelSerializer._restore(f, loadUpdater, None, device)

    @staticmethod
    def restoreMultiLayerNetworkAndNormalizer(f, loadUpdater=True, device=None):
        net = ModelSerializer.restoreMultiLayerNetwork(f, loadUpdater, device)
        return net, net._normalizer

    @staticmethod
    def restoreComputationGraphAndNormalizer(f, loadUpdater=True, device=None):
        net = ModelSerializer.restoreComputationGraph(f, loadUpdater, device)
        return net, net._normalizer

    @staticmethod
    def restoreNormalizerFromFile(f):
        z = ModelSerializer._read(f)
        if NORMALIZER not in z.namelist():
            return None
        from ..datasets.normalizers import DataNormalization
        return DataNormalization.from_bytes(z.read(NORMALIZER))

    @staticmethod
    def addNormalizerToModel(path, normalizer):
        """Append/replace normalizer.bin inside an existing model zip (reference :690)."""
        with open(path, "rb") as fh:
            old = zipfile.ZipFile(io.BytesIO(fh.read()))
        with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
            for n in old.namelist():
                if n != NORMALIZER:
                    z.writestr(n, old.read(n))
            z.writestr(NORMALIZER, normalizer.to_bytes())

    @staticmethod
    def writeParamsAndConfig(model):
        return model.conf.toJson(), model.params().detach().cpu().clone()


def _guess_bytes(head):
    if head[:2] == b"PK":
        return "dl4j"
    if head[:8] == b"\x89HDF\r\n\x1a\n":
        return "keras"
    if head.lstrip()[:1] in (b"{", b"["):
        return "json"
    return "unknown"


def guess_model_type(path):
    """ModelGuesser (reference CORE:util/ModelGuesser.java:20): DL4J zip vs config JSON vs Keras h5."""
    with open(path, "rb") as fh:
        head = fh.read(8)
    return _guess_bytes(head)


def _source_bytes(src):
    """(bytes, path-or-None) of a path or a readable binary stream."""
    if isinstance(src, (str, os.PathLike)):
        with open(src, "rb") as fh:
            return fh.read(), str(src)
    return src.read(), None


class ModelGuesser:
    """Load a model, configuration or normalizer without knowing its format (reference util/ModelGuesser.java):
    DL4J model zips, Keras HDF5 files and configuration JSON, from a path or an input stream."""

    @staticmethod
    def loadModelGuess(src):
        data, path = _source_bytes(src)
        t = _guess_bytes(data[:8])
        if t == "dl4j":
            return ModelSerializer.restoreModel(io.BytesIO(data))
        if t == "keras":
            from ..modelimport.keras import KerasModelImport
            if path is None:
                import tempfile
                with tempfile.NamedTemporaryFile(suffix=".h5", delete=False) as tf:
                    tf.write(data)
                    path = tf.name
                try:
                    return KerasModelImport.importKerasModelAndWeights(path)
                finally:
                    os.unlink(path)
            return KerasModelImport.importKerasModelAndWeights(path)
        raise ValueError(f"Unable to guess model type of {path or 'the stream'}")

    @staticmethod
    def loadConfigGuess(src):
        data, _ = _source_bytes(src)
        return _config_from_json(data.decode("utf-8"))

    @staticmethod
    def loadNormalizer(src):
        """The normalizer stored inside a DL4J model zip (None when it has none)."""
        data, _ = _source_bytes(src)
        return ModelSerializer.restoreNormalizerFromFile(io.BytesIO(data))


_ = torch
