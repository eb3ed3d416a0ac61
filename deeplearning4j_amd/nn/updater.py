"""Network updater: UpdaterBlocks over the flat gradient + one fused update kernel.

Reference: nn/updater/BaseMultiLayerUpdater.java:54-161 (block grouping: contiguous (layer,param)
pairs with equal updater config share one block and one contiguous state slice), :223-309 (update
order), :322-382 (gradient normalization preApply), UpdaterBlock.java:142-193.
"""
import math

import torch

from ..nn.conf.enums import GradientNormalization
from ..nn.conf.updaters import NoOp
from ..ops.update import (GN_CLIP_ELEM, GN_CLIP_L2_LAYER, GN_CLIP_L2_PARAM, GN_NONE, GN_RENORM_LAYER,
                          GN_RENORM_PARAM, Segment, UpdatePlan, fused_update, pre_apply)
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


def updater_configs_equal(a, b):
    """Reference UpdaterUtils.updaterConfigurationsEquals: same class and identical hyperparameters."""
    if a is None or b is None:
        return a is b
    return type(a) is type(b) and a.to_dict() == b.to_dict()


class ParamEntry:
    __slots__ = ("layer_idx", "layer_name", "key", "p_off", "n", "updater", "l1", "l2", "layer")

    def __init__(self, layer_idx, layer_name, key, p_off, n, updater, l1, l2, layer):
        self.layer_idx, self.layer_name, self.key, self.p_off, self.n = layer_idx, layer_name, key, p_off, n
        self.updater, self.l1, self.l2, self.layer = updater, l1, l2, layer


class UpdaterBlock:
    def __init__(self, p_start, p_end, st_off, updater, entries):
        self.paramOffsetStart, self.paramOffsetEnd = p_start, p_end
        self.st_off = st_off
        self.updater = updater
        self.entries = entries

    def getLayersAndVariablesInBlock(self):
        return [(e.layer_name, e.key) for e in self.entries]

    def getGradientUpdater(self):
        return self.updater

    @property
    def stateSize(self):
        return self.updater.stateSize(self.paramOffsetEnd - self.paramOffsetStart)


class NetworkUpdater:
    """Shared implementation of MultiLayerUpdater / ComputationGraphUpdater."""

    def __init__(self, net, entries):
        self.net = net
        self.entries = entries
        self.blocks = []
        cur = []
        st = 0
        for e in entries:
            if cur and updater_configs_equal(cur[-1].updater, e.updater) and cur[-1].p_off + cur[-1].n == e.p_off:
                cur.append(e)
            else:
                if cur:
                    self._close(cur, st)
                    st += self.blocks[-1].stateSize
                cur = [e]
        if cur:
            self._close(cur, st)
            st += self.blocks[-1].stateSize
        self.state_size = st
        self._gn_layers = self._collect_gn()
        gn_of = {}
        G = GradientNormalization
        codes = {G.RenormalizeL2PerLayer: GN_RENORM_LAYER, G.RenormalizeL2PerParamType: GN_RENORM_PARAM,
                 G.ClipElementWiseAbsoluteValue: GN_CLIP_ELEM, G.ClipL2PerLayer: GN_CLIP_L2_LAYER,
                 G.ClipL2PerParamType: GN_CLIP_L2_PARAM}
        for name, (gn, thr, ents) in self._gn_layers.items():
            code = codes.get(gn, GN_NONE)
            per_layer = code in (GN_RENORM_LAYER, GN_CLIP_L2_LAYER)
            for e in ents:
                if not isinstance(e.updater, NoOp):     # BN running statistics etc. are not normalised
                    gn_of[id(e)] = (code, float(thr), name if per_layer else None)
        segs = []
        for bi, b in enumerate(self.blocks):
            for e in b.entries:
                code, thr, grp = gn_of.get(id(e), (GN_NONE, 1.0, None))
                segs.append(Segment(e.p_off, e.n, b.st_off, e.p_off - b.paramOffsetStart,
                                    b.paramOffsetEnd - b.paramOffsetStart, b.updater, e.l1, e.l2, bi,
                                    code, thr, grp))
        self.plan = UpdatePlan(segs, [(b.paramOffsetStart, b.paramOffsetEnd, b.st_off, b.updater)
                                      for b in self.blocks])
        self.state = None

    def _close(self, cur, st):
        self.blocks.append(UpdaterBlock(cur[0].p_off, cur[-1].p_off + cur[-1].n, st, cur[0].updater, list(cur)))

    def init_state(self, device, dtype):
        self.state = torch.zeros(max(self.state_size, 1), dtype=dtype, device=device)[:self.state_size]

    def getStateViewArray(self):
        return self.state.reshape(1, -1)

    def setStateViewArray(self, arr):
        with torch.no_grad():
            self.state.copy_(arr.reshape(-1).to(self.state.dtype))

    def getUpdaterBlocks(self):
        return self.blocks

    def _collect_gn(self):
        out = {}
        for e in self.entries:
            conf = e.layer.conf
            gn = getattr(conf, "gradientNormalization", None)
            if gn is None and hasattr(conf, "underlying"):
                gn = getattr(conf.underlying, "gradientNormalization", None)
            if gn is not None and gn != GradientNormalization.None_:
                thr = getattr(conf, "gradientNormalizationThreshold", None) or \
                    getattr(getattr(conf, "underlying", None), "gradientNormalizationThreshold", 1.0) or 1.0
                out.setdefault(e.layer_name, (gn, thr, []))[2].append(e)
        return out

    def preApply(self, grad):
        """Per-layer gradient normalization / clipping (reference BaseMultiLayerUpdater.java:322-382). ``update``
        does not call this on the GPU: the fused updater kernel applies the same scaling in its own pass."""
        pre_apply(self.plan, grad)

    def update(self, params, grad, iteration, epoch, batch_size, shadow=None, reg_out=None):
        """Apply the whole update (preApply -> updater -> l1/l2 -> /batch -> params -= u) in place; the gradient
        normalization runs inside fused_update (kernel pass on the GPU, ``pre_apply`` on the host path).

        Called as ``update(model, gradient, iteration, epoch, batchSize)`` (the reference's Updater.update), the
        Gradient is turned into the update in place instead -- the parameters stay as they are and the updater state
        advances -- so a gradient computed by one network can be applied to another (params -= gradient)."""
        if hasattr(grad, "gradient") and callable(getattr(params, "params", None)):
            flat_g = grad.gradient()
            gmap = keys = None
            pflat = params.params().reshape(-1)
            if flat_g is None:
                # same element layout as the flat parameter vector: each variable lands where its parameter view
                # sits in it (f-order weight views included)
                gmap, keys = self._map_keys(params, grad)
                table = params.paramTable()
                flat_g = torch.zeros_like(pflat)
                base = pflat.storage_offset()
                views = {k: flat_g.as_strided(table[k].shape, table[k].stride(), table[k].storage_offset() - base)
                         for k in keys}
                for k in keys:
                    views[k].copy_(gmap[k].reshape(table[k].shape))
            flat_g = flat_g.reshape(-1)
            p = pflat.detach().clone()
            before = p.clone()
            fused_update(self.plan, p, flat_g.detach().clone().to(p.dtype), self.state, iteration, epoch,
                         batch_size, self.net.conf.globalConf.get("miniBatch", True), None)
            upd = before - p
            if gmap is None:
                flat_g.copy_(upd.to(flat_g.dtype))
            else:
                flat_g.copy_(upd.to(flat_g.dtype))
                for k in keys:
                    gmap[k].copy_(views[k].reshape(gmap[k].shape))
            return
        fused_update(self.plan, params, grad, self.state, iteration, epoch, batch_size,
                     self.net.conf.globalConf.get("miniBatch", True), shadow, reg_out=reg_out)

    @staticmethod
    def _map_keys(model, grad):
        """Parameter keys of a Gradient built only with setGradientFor (no flattened view), in the model's flat
        parameter order (paramTable), or a ValueError naming what is missing."""
        gmap = grad.gradientForVariable() if hasattr(grad, "gradientForVariable") else {}
        keys = list(model.paramTable().keys())
        missing = [k for k in keys if k not in gmap]
        if missing:
            raise ValueError(f"Gradient has no flattened view and no entry for parameter(s) {missing[:4]}")
        return gmap, keys

    def update_range(self, params, grad, iteration, epoch, batch_size, lo, hi):
        """Update only the parameters in the flat range [lo, hi) (layer-wise pretraining): the fused update
        runs over everything, then parameters and updater state outside the range are restored."""
        keep_p = params.clone()
        keep_s = self.state.clone() if self.state is not None else None
        self.update(params, grad, iteration, epoch, batch_size)
        inside = torch.zeros(params.numel(), dtype=torch.bool, device=params.device)
        inside[lo:hi] = True
        params.copy_(torch.where(inside, params, keep_p))
        if keep_s is not None and keep_s.numel():
            smask = torch.zeros(keep_s.numel(), dtype=torch.bool, device=keep_s.device)
            for sg in self.plan.segments:
                if lo <= sg.p_off < hi and sg.block_n > 0:
                    comps = sg.updater.stateSize(sg.block_n) // sg.block_n
                    for c in range(comps):
                        a = sg.st_off + c * sg.block_n + sg.in_block
                        smask[a:a + sg.n] = True
            self.state.copy_(torch.where(smask, self.state, keep_s))

    # learning-rate control (reference MultiLayerNetwork.setLearningRate :3411-3459)
    def setLearningRate(self, lr, layer_name=None):
        for b in self.blocks:
            for e in b.entries:
                if layer_name is None or e.layer_name == layer_name:
                    if hasattr(e.updater, "learningRate"):
                        e.updater.learningRate = lr
                        e.updater.learningRateSchedule = None


def build_entries(layer_list):
    """layer_list: [(idx, name, layer_impl, p_off)] in flat order -> ParamEntry list."""
    entries = []
    for idx, name, layer, off in layer_list:
        conf = layer.conf
        o = off
        for spec in conf.param_specs():
            upd = conf.updaterFor(spec.key) if spec.trainable else NoOp()
            if upd is None:
                from ..nn.conf.updaters import Sgd
                upd = Sgd(1e-3)
            entries.append(ParamEntry(idx, name, spec.key, o, spec.numel, upd, conf.l1For(spec.key),
                                      conf.l2For(spec.key), layer))
            o += spec.numel
    return entries


_ = math
