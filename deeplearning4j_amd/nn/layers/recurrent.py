"""Recurrent runtime layers: LSTM, GravesLSTM (peepholes), GravesBidirectionalLSTM, SimpleRnn,
Bidirectional, LastTimeStep.

LSTM math = reference nn/layers/recurrent/LSTMHelpers.java (forward :189-358, backward :392-690):
gate blocks in the 4H axis are [a (cell input, layer activation) | f (forget) | o (output) |
g (input-modulation)], peepholes (Graves) are RW columns 4H (wFF), 4H+1 (wOO), 4H+2 (wGG):
    a = act(z_a); f = gate(z_f + wFF*c_prev); g = gate(z_g + wGG*c_prev)
    c = f*c_prev + g*a; o = gate(z_o + wOO*c); h = o*act(c)
MI355X structure: ONE big input-projection GEMM for all T steps ([T*mb, nIn] x [nIn, 4H]), then on GPU ONE
launch of the whole-sequence recurrent kernel (csrc/lstm.hip: MFMA h·RW + fused gates, cell state in registers;
the HIP replacement of the cuDNN LSTMHelper); the per-step torch loop below is the CPU/fp64 reference path.
Backward runs the mirrored sequence kernel, then accumulates dW, dRW and dX as single big GEMMs. TBPTT stops the
backward time loop at ``tbpttBackLength`` steps (LSTMHelpers.java:484).
"""
import torch

from ... import ops
from ..conf.activations import ActivationSigmoid, ActivationTanH
from .base import LayerImpl, copy_grad_, matmul, weight_grad_
from deeplearning4j_amd.nn.util.dtypes import acc as _acc, acc_dtype  # noqa: E402


def _native_ok(x, W, act, gate_act, H):
    """Whole-sequence HIP kernels apply: GPU tensor, tanh/sigmoid (the cuDNN helper's own restriction,
    CudnnLSTMHelper.java:174-190 — peepholes are supported here), kernel-supported H/dtype."""
    from ...ops import rnn_native
    return (x.is_cuda and isinstance(act, ActivationTanH) and isinstance(gate_act, ActivationSigmoid)
            and rnn_native.supported(H, W.dtype) and ops.use_native(x, "lstm"))


def _time_major_rows(x, dt):
    """[mb, nIn, T] -> [T*mb, nIn] rows in the compute dtype. On the GPU, when that takes a copy anyway (a cast, a
    non-trivial permute, or nIn % 8 != 0), ONE launch permutes + casts + zero-pads the last dimension to a multiple of
    8 (ops/nd4j_kernels.cast_pad_last): the rows are then a ``kz_view`` GEMM operand read in place by x·W and by
    dW = xᵀ·dz (no padded copies inside the GEMMs)."""
    mb, nIn, T = x.shape
    xp = x.permute(2, 0, 1)
    if x.is_cuda and dt in (torch.bfloat16, torch.float16) and (nIn % 8 or x.dtype != dt or not xp.is_contiguous()):
        from ...memory import arena
        from ...ops import nd4j_kernels as K
        from ...ops.gemm import kz_view
        K8 = (nIn + 7) // 8 * 8
        buf = arena.empty((T, mb, K8), dt, x.device)
        if K.cast_pad_last(xp, dt, K8, out=buf) is not None:
            rows = buf.reshape(T * mb, K8)
            return kz_view(rows, nIn) if K8 != nIn else rows
    return xp.reshape(T * mb, nIn).to(dt)


def _lstm_fwd(x, W, RW, b, h0, c0, H, peephole, act, gate_act, mask, need_cache):
    """x: [mb, nIn, T]. Returns out [mb, H, T], (hT, cT), cache."""
    mb, nIn, T = x.shape
    dt = W.dtype
    _adt = acc_dtype(W)
    xt = _time_major_rows(x, dt)
    zx = matmul(xt, W, bias=b).reshape(T, mb, 4 * H)          # input projection, all steps (bias in the epilogue)
    if _native_ok(x, W, act, gate_act, H):
        from ...ops import rnn_native
        # both packed images of RW (+ fp32 peepholes) in one launch; the backward pass reuses them
        packs = rnn_native.pack_rw(RW, H, peephole, need_bwd=need_cache)
        r = rnn_native.lstm_seq_fwd(zx, RW, H, peephole, h0, c0, mask, need_cache, packs=packs, out16=True)
        if r is not None:
            out_tmh, hT, cT, gates, call, o16 = r
            # compute dtype (DL4J casts input to the net dtype); the kernel wrote the 16-bit copy itself
            out = o16.permute(1, 2, 0) if o16 is not None else out_tmh.permute(1, 2, 0).to(dt)
            cache = None
            if need_cache:
                cache = {"native": True, "gates": gates, "call": call, "out": out_tmh, "h0": h0, "c0": c0,
                         "xt": xt, "packs": packs}
            return out, (hT, cT), cache
    RWg = RW[:, :4 * H]
    if peephole:
        wFF, wOO, wGG = _acc(RW[:, 4 * H]), _acc(RW[:, 4 * H + 1]), _acc(RW[:, 4 * H + 2])
    h = torch.zeros(mb, H, dtype=_adt, device=x.device) if h0 is None else _acc(h0)
    c = torch.zeros(mb, H, dtype=_adt, device=x.device) if c0 is None else _acc(c0)
    outs = []
    cache = {"z": [], "a": [], "f": [], "g": [], "o": [], "c": [], "c_prev": [], "h_prev": [], "cact": []} \
        if need_cache else None
    for t in range(T):
        z = _acc(zx[t]) + _acc(matmul(h.to(dt), RWg))
        za, zf, zo, zg = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
        if peephole:
            zf = zf + c * wFF
            zg = zg + c * wGG
        a = act.getActivation(za, True)
        f = gate_act.getActivation(zf, True)
        g = gate_act.getActivation(zg, True)
        c_new = f * c + g * a
        if peephole:
            zo = zo + c_new * wOO
        o = gate_act.getActivation(zo, True)
        cact = act.getActivation(c_new, True)
        h_new = o * cact
        z = torch.cat([za, zf, zo, zg], dim=1)
        if mask is not None:
            m = _acc(mask[:, t]).reshape(-1, 1)
            h_new = h_new * m
            c_new = c_new * m
        if need_cache:
            cache["z"].append(z)
            cache["a"].append(a)
            cache["f"].append(f)
            cache["g"].append(g)
            cache["o"].append(o)
            cache["c"].append(c_new)
            cache["c_prev"].append(c)
            cache["h_prev"].append(h)
            cache["cact"].append(cact)
        h, c = h_new, c_new
        outs.append(h)
    out = torch.stack(outs, dim=2).to(dt)
    if need_cache:
        cache["xt"] = xt
    return out, (h, c), cache


def _lstm_weight_grads(dzf2, xt, hprev, W, H, peephole, peep_grads, grads_prefix, grads, T, mb):
    """The big library GEMMs after the time loop: dW = xᵀ·dz, dRW = hprevᵀ·dz (+ peephole columns), db = Σdz,
    dX = dz·Wᵀ (LSTMHelpers.java:616-676)."""
    dt = W.dtype
    if dzf2.is_cuda and dt == torch.bfloat16:
        # mixed precision: bf16 operands, fp32 accumulation straight into the fp32 gradient views
        from .transformer import _bsum, _wgrad
        dzb = dzf2.to(dt)
        _wgrad(grads[grads_prefix + "W"], xt.to(dt), dzb)
        hb = hprev.reshape(T * mb, H).to(dt)
        gRW = grads[grads_prefix + "RW"]
        if peephole:
            dRW = matmul(hb.t(), dzb, out_dtype=torch.float32)
            copy_grad_(gRW, torch.cat([dRW] + [g.reshape(-1, 1) for g in peep_grads], dim=1))
        else:
            _wgrad(gRW, hb, dzb)
        _bsum(grads[grads_prefix + "b"], dzf2)
        return matmul(dzb, W.t()).reshape(T, mb, -1).permute(1, 2, 0)
    weight_grad_(grads[grads_prefix + "W"], _acc(xt).t(), dzf2)
    dRW = matmul(hprev.reshape(T * mb, H).t(), dzf2)
    if peephole:
        dRW = torch.cat([dRW] + [g.reshape(-1, 1) for g in peep_grads], dim=1)
    copy_grad_(grads[grads_prefix + "RW"], dRW)
    copy_grad_(grads[grads_prefix + "b"], dzf2.sum(dim=0))
    return matmul(dzf2.to(dt), W.t()).reshape(T, mb, -1).permute(1, 2, 0)


def _lstm_bwd_native(eps, cache, W, RW, H, peephole, mask, tbptt_back, grads_prefix, grads, dh_last, dc_last,
                     need_dx=True):
    from ...ops import rnn_native
    mb, _, T = eps.shape
    t_end = max(0, T - tbptt_back) if tbptt_back else 0
    r = rnn_native.lstm_seq_bwd(eps.permute(2, 0, 1), cache["gates"], cache["call"], cache["c0"], RW, H, peephole,
                                mask, dh_last, dc_last, t_end, packs=cache.get("packs"))
    if r is None:
        return None
    dz, dh0, dc0 = r
    return _native_weight_grads(dz, cache, W, H, peephole, grads_prefix, grads, need_dx, dh0, dc0)


def _native_weight_grads(dz, cache, W, H, peephole, grads_prefix, grads, need_dx, dh0, dc0):
    """Weight / bias / peephole gradients (and dL/dinput when ``need_dx``) from the sequence kernels' gate deltas
    dz [T, mb, 4H] fp32 (LSTMHelpers.java:616-676)."""
    from ...ops import rnn_native
    T, mb = dz.shape[0], dz.shape[1]
    out = cache["out"]                                                # [T, mb, H] fp32
    dev = dz.device
    if W.dtype in (torch.bfloat16, torch.float16):
        prep = rnn_native.lstm_bwd_prep(dz, out, cache["h0"], cache["call"], cache["c0"], peephole, W.dtype)
        if prep is not None:
            # one fused glue launch, then the three GEMMs write fp32 gradients straight into the flat views
            from .transformer import _wgrad
            dzb, hpb, db, dpeep = prep
            _wgrad(grads[grads_prefix + "W"], cache["xt"].to(W.dtype), dzb)
            gRW = grads[grads_prefix + "RW"]
            if peephole:
                _wgrad(gRW[:, :4 * H], hpb, dzb)
                gRW[:, 4 * H:].copy_(dpeep.t())
            else:
                _wgrad(gRW, hpb, dzb)
            copy_grad_(grads[grads_prefix + "b"], db)
            if not need_dx:                              # first layer: dL/dinput is never read
                return None, dh0, dc0
            return matmul(dzb, W.t()).reshape(T, mb, -1).permute(1, 2, 0), dh0, dc0
    h0 = torch.zeros(1, mb, H, device=dev) if cache["h0"] is None else _acc(cache["h0"]).reshape(1, mb, H)
    hprev = torch.cat([h0.to(out.dtype), out[:-1]], dim=0)
    peep_grads = None
    if peephole:
        c0 = torch.zeros(1, mb, H, device=dev) if cache["c0"] is None else _acc(cache["c0"]).reshape(1, mb, H)
        call = cache["call"]
        cprev = torch.cat([c0.to(call.dtype), call[:-1]], dim=0)
        dzf, dzo, dzg = dz[:, :, H:2 * H], dz[:, :, 2 * H:3 * H], dz[:, :, 3 * H:]
        peep_grads = [(dzf * cprev).sum(dim=(0, 1)), (dzo * call).sum(dim=(0, 1)), (dzg * cprev).sum(dim=(0, 1))]
    dx = _lstm_weight_grads(dz.reshape(T * mb, 4 * H), cache["xt"], hprev, W, H, peephole, peep_grads,
                            grads_prefix, grads, T, mb)
    return dx, dh0, dc0


def _lstm_bwd(eps, cache, W, RW, H, peephole, act, gate_act, mask, tbptt_back, grads_prefix, grads, dh_last=None,
              dc_last=None, need_dx=True):
    """eps: [mb, H, T]. Writes dW/dRW/db into grads views; returns eps_in [mb, nIn, T] (None possible when
    ``need_dx`` is False)."""
    if cache.get("native"):
        r = _lstm_bwd_native(eps, cache, W, RW, H, peephole, mask, tbptt_back, grads_prefix, grads, dh_last, dc_last,
                             need_dx)
        if r is not None:
            return r
        raise RuntimeError("native LSTM forward cache but the backward kernel rejected the shape")
    mb, _, T = eps.shape
    _adt = acc_dtype(W)
    RWg = _acc(RW[:, :4 * H])
    if peephole:
        wFF, wOO, wGG = _acc(RW[:, 4 * H]), _acc(RW[:, 4 * H + 1]), _acc(RW[:, 4 * H + 2])
        dwFF = torch.zeros(H, device=eps.device, dtype=_adt)
        dwOO = torch.zeros(H, device=eps.device, dtype=_adt)
        dwGG = torch.zeros(H, device=eps.device, dtype=_adt)
    dh_next = torch.zeros(mb, H, device=eps.device, dtype=_adt) if dh_last is None else _acc(dh_last)
    dc_next = torch.zeros(mb, H, device=eps.device, dtype=_adt) if dc_last is None else _acc(dc_last)
    dz_all = torch.zeros(T, mb, 4 * H, device=eps.device, dtype=_adt)
    t_end = max(0, T - tbptt_back) if tbptt_back else 0
    e = _acc(eps)
    for t in range(T - 1, t_end - 1, -1):
        dh = e[:, :, t] + dh_next
        dc = dc_next
        if mask is not None:
            m = _acc(mask[:, t]).reshape(-1, 1)
            dh = dh * m
            dc = dc * m
        z = cache["z"][t]
        a, f, g, o = cache["a"][t], cache["f"][t], cache["g"][t], cache["o"][t]
        c, c_prev, cact = cache["c"][t], cache["c_prev"][t], cache["cact"][t]
        za, zf, zo, zg = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
        do = dh * cact
        dzo = gate_act.backprop(zo, do)
        dc = dc + act.backprop(c, dh * o)
        if peephole:
            dc = dc + dzo * wOO
        dzf = gate_act.backprop(zf, dc * c_prev)
        dzg = gate_act.backprop(zg, dc * a)
        dza = act.backprop(za, dc * g)
        dc_next = dc * f
        if peephole:
            dc_next = dc_next + dzf * wFF + dzg * wGG
            dwFF += (dzf * c_prev).sum(dim=0)
            dwGG += (dzg * c_prev).sum(dim=0)
            dwOO += (dzo * c).sum(dim=0)
        dz = torch.cat([dza, dzf, dzo, dzg], dim=1)
        dz_all[t] = dz
        dh_next = matmul(dz, RWg.t())
    hprev = torch.stack(cache["h_prev"], 0)                       # [T, mb, H]
    dx = _lstm_weight_grads(dz_all.reshape(T * mb, 4 * H), cache["xt"], hprev, W, H, peephole,
                            [dwFF, dwOO, dwGG] if peephole else None, grads_prefix, grads, T, mb)
    return dx, dh_next, dc_next


class BaseRecurrentImpl(LayerImpl):
    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.stateMap = {}
        self.tBpttStateMap = {}

    def type(self):
        return "RECURRENT"

    def rnnClearPreviousState(self):
        self.stateMap = {}
        self.tBpttStateMap = {}

    def _check_state_mb(self, x):
        """rnnTimeStep continues the stored state, so the minibatch size cannot change between calls without
        rnnClearPreviousState() (reference TestInvalidInput.testInvalidRnnTimeStep: DL4JInvalidInputException)."""
        h = self.stateMap.get("prevAct")
        if h is not None and h.shape[0] != x.shape[0]:
            from ...exceptions import DL4JInvalidInputException
            raise DL4JInvalidInputException(
                f"rnnTimeStep on layer {self.index} ({type(self.conf).__name__}): minibatch size {x.shape[0]} differs "
                f"from the stored state's {h.shape[0]}; call rnnClearPreviousState() before changing it")

    def rnnGetPreviousState(self):
        return dict(self.stateMap)

    def rnnSetPreviousState(self, s):
        self.stateMap = dict(s)

    def rnnGetTBPTTState(self):
        return dict(self.tBpttStateMap)

    def rnnSetTBPTTState(self, s):
        self.tBpttStateMap = dict(s)


class LSTMImpl(BaseRecurrentImpl):
    PEEPHOLE = False
    # the feature mask leaves an LSTM in the Passthrough state: layers above still see it, but an output layer no
    # longer masks its score with it (reference GravesLSTM/LSTM.feedForwardMaskArray, RnnOutputLayer:204-216)
    MASK_PASSTHROUGH = True
    GRADS_OVERWRITE = True        # W / RW / b gradient views are written whole every backward (no accumulation)

    def _run(self, x, training, h0, c0, need_cache, mask):
        H = self.conf.nOut
        return _lstm_fwd(x, self.W("W"), self.W("RW"), self.Wbias("b"), h0, c0, H, self.PEEPHOLE, self.conf.activation,
                         self.conf.gateActivationFn, mask, need_cache)

    def activate(self, x, training=False, mask=None, stored_state=False, store_last_for_tbptt=False):
        if x.dim() == 2:
            x = x.unsqueeze(2)
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        self.maskArray = mask
        h0 = c0 = None
        if stored_state:
            h0, c0 = self.tBpttStateMap.get("prevAct"), self.tBpttStateMap.get("prevMem")
        pend = getattr(self, "_stack_pending", None)
        self._stack_pending = None
        if pend is not None and pend[0] is x:
            out, (h, c), cache = pend[1]              # computed by the layer below in one stacked launch
        else:
            nxt = getattr(self, "_stack_next", None)
            r = self._stack_forward(nxt, x, h0, c0, mask, stored_state, training) if nxt is not None else None
            if r is None:
                r = self._run(x, training, h0, c0, training, mask)
            out, (h, c), cache = r
        self._cache = cache
        if store_last_for_tbptt:
            self.tBpttStateMap = {"prevAct": h.detach(), "prevMem": c.detach()}
        return out

    # ---- pipelined two-layer stack (csrc/lstm_coop.hip lstm_fwd_stack2 / lstm_bwd_stack2)
    def _stack_forward(self, nxt, x, h0, c0, mask, stored_state, need_cache):
        """This layer and ``nxt`` (planned by MultiLayerNetwork._plan_fusions) in ONE launch: layer 2 runs step t
        while this layer runs step t+1, and layer 2's input projection happens inside the recurrence. Returns this
        layer's (out, (hT, cT), cache) and leaves layer 2's result pending for its activate; None when the stack
        kernel does not apply (both layers then run on their own)."""
        from ...ops import rnn_native
        H = self.conf.nOut
        W1, RW1, W2, RW2 = self.W("W"), self.W("RW"), nxt.W("W"), nxt.W("RW")
        T = x.shape[2]
        if not (_native_ok(x, W1, self.conf.activation, self.conf.gateActivationFn, H)
                and rnn_native.stack2_supported(H, W1.dtype, T) and W2.dtype == W1.dtype
                and tuple(W2.shape) == (H, 4 * H)):
            return None
        mb = x.shape[0]
        xt = _time_major_rows(x, W1.dtype)
        zx1 = matmul(xt, W1, bias=self.Wbias("b")).reshape(T, mb, 4 * H)
        p1 = rnn_native.pack_rw(RW1, H, self.PEEPHOLE, need_bwd=need_cache)
        p2 = rnn_native.pack_rw(RW2, H, nxt.PEEPHOLE, need_bwd=need_cache)
        pw = rnn_native.pack_rw(W2, H, False, need_bwd=need_cache)
        if p1 is None or p2 is None or pw is None:
            return None
        h02 = c02 = None
        if stored_state:
            h02, c02 = nxt.tBpttStateMap.get("prevAct"), nxt.tBpttStateMap.get("prevMem")
        r = rnn_native.lstm2_seq_fwd(zx1, p1, p2, pw, nxt.Wbias("b").reshape(-1), H, (h0, h02), (c0, c02), mask,
                                     need_cache)
        if r is None:
            return None
        (o1, hT1, cT1, g1, ca1, s1), (o2, hT2, cT2, g2, ca2, s2) = r
        out1, out2 = s1.permute(1, 2, 0), s2.permute(1, 2, 0)
        c1 = c2 = None
        if need_cache:
            tag = object()                                 # pairs the two caches of one launch
            c1 = {"native": True, "gates": g1, "call": ca1, "out": o1, "h0": h0, "c0": c0, "xt": xt, "packs": p1,
                  "stack": tag}
            c2 = {"native": True, "gates": g2, "call": ca2, "out": o2, "h0": h02, "c0": c02,
                  "xt": s1.reshape(T * mb, H), "packs": p2, "w2pack": pw, "stack": tag}
        nxt._stack_pending = (out1, (out2, (hT2, cT2), c2))
        return out1, (hT1, cT1), c1

    def _stack_backward(self, prev, eps, tbptt_back):
        """Both layers' backward time loops in ONE launch (this layer's eps feeds the layer below inside the
        kernel); this layer's weight gradients here, the layer below's gate deltas handed to its backprop."""
        from ...ops import rnn_native
        c2, c1 = self._cache, prev._cache
        H = self.conf.nOut
        mb, _, T = eps.shape
        t_end = max(0, T - tbptt_back) if tbptt_back else 0
        r = rnn_native.lstm2_seq_bwd(eps.permute(2, 0, 1), c1, c2, c1["packs"], c2["packs"], c2["w2pack"], H,
                                     self.maskArray, t_end)
        if r is None:
            return None
        dz1, dz2, st1, st2 = r
        _native_weight_grads(dz2, c2, self.W("W"), H, self.PEEPHOLE, "", self.grads, False, *st2)
        prev._stack_dz = (dz1, st1, c2["stack"])
        # the layer below takes its gate deltas from _stack_dz: a zero-cost placeholder stands in for its epsilon.
        # It is marked, so that a layer below that does NOT find the matching _stack_dz (its cache was replaced by a
        # re-run forward in between) raises instead of silently training on a zero gradient.
        from ...ops import nd4j_kernels as NK
        ph = NK.zero_(torch.empty((), dtype=eps.dtype, device=eps.device)).expand(mb, H, T)
        ph._dl4j_stack_placeholder = True
        return self.make_gradient(), ph

    def rnnTimeStep(self, x, mask=None):
        self._check_state_mb(x)
        is2d = x.dim() == 2
        if is2d:
            x = x.unsqueeze(2)
        out, (h, c), _ = self._run(x, False, self.stateMap.get("prevAct"), self.stateMap.get("prevMem"), False, mask)
        self.stateMap = {"prevAct": h, "prevMem": c}
        return out[:, :, 0] if is2d else out

    def backpropGradient(self, eps, tbptt_back=None):
        if eps.dim() == 2:
            eps = eps.unsqueeze(2)
        H = self.conf.nOut
        need_dx = getattr(self, "need_input_grad", True)
        sdz = getattr(self, "_stack_dz", None)
        self._stack_dz = None
        prev = getattr(self, "_stack_prev", None)
        if sdz is not None and self._cache is not None and sdz[2] is self._cache.get("stack"):
            # gate deltas from the stacked launch of the layer above (eps is its placeholder)
            dx, _, _ = _native_weight_grads(sdz[0], self._cache, self.W("W"), H, self.PEEPHOLE, "", self.grads,
                                            need_dx, *sdz[1])
            if dx is None:
                return self.make_gradient(), None
            return self.make_gradient(), self.backpropDropOut(dx.to(eps.dtype))
        if getattr(eps, "_dl4j_stack_placeholder", False):
            raise RuntimeError(f"LSTM layer {self.conf.layerName!r}: received the stacked-launch epsilon placeholder "
                               "without the matching gate deltas (the forward was re-run between the two layers' "
                               "backprops); run forward and backward of the stack together")
        if prev is not None and self._cache is not None and self._cache.get("stack") is not None and \
                prev._cache is not None and prev._cache.get("stack") is self._cache["stack"]:
            r = self._stack_backward(prev, eps, tbptt_back)
            if r is not None:
                return r
        dx, _, _ = _lstm_bwd(eps, self._cache, self.W("W"), self.W("RW"), H, self.PEEPHOLE, self.conf.activation,
                             self.conf.gateActivationFn, self.maskArray, tbptt_back, "", self.grads,
                             need_dx=need_dx)
        if dx is None:
            return self.make_gradient(), None
        return self.make_gradient(), self.backpropDropOut(dx.to(eps.dtype))


class GravesLSTMImpl(LSTMImpl):
    PEEPHOLE = True


class GravesBidirectionalLSTMImpl(BaseRecurrentImpl):
    def activate(self, x, training=False, mask=None, **kw):
        from ..util.time_series import reverse_time_series
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        self.maskArray = mask
        H = self.conf.nOut
        a, ga = self.conf.activation, self.conf.gateActivationFn
        fw, _, self._cf = _lstm_fwd(x, self.W("WF"), self.W("RWF"), self.W("bF"), None, None, H, True, a, ga, mask,
                                    training)
        xr = reverse_time_series(x, mask)
        mr = reverse_time_series(mask, mask) if mask is not None else None
        bw, _, self._cb = _lstm_fwd(xr, self.W("WB"), self.W("RWB"), self.W("bB"), None, None, H, True, a, ga, mr,
                                    training)
        self._mr = mr
        return fw + reverse_time_series(bw, mask)

    def backpropGradient(self, eps, tbptt_back=None):
        from ..util.time_series import reverse_time_series
        H = self.conf.nOut
        a, ga = self.conf.activation, self.conf.gateActivationFn
        dxf, _, _ = _lstm_bwd(eps, self._cf, self.W("WF"), self.W("RWF"), H, True, a, ga, self.maskArray, tbptt_back,
                              "", {"W": self.grads["WF"], "RW": self.grads["RWF"], "b": self.grads["bF"]})
        er = reverse_time_series(eps, self.maskArray)
        dxb, _, _ = _lstm_bwd(er, self._cb, self.W("WB"), self.W("RWB"), H, True, a, ga, self._mr, tbptt_back, "",
                              {"W": self.grads["WB"], "RW": self.grads["RWB"], "b": self.grads["bB"]})
        return self.make_gradient(), self.backpropDropOut((dxf + reverse_time_series(dxb, self.maskArray))
                                                          .to(eps.dtype))

    def rnnTimeStep(self, x, mask=None):
        raise NotImplementedError("GravesBidirectionalLSTM does not support rnnTimeStep (needs the full sequence)")


class SimpleRnnImpl(BaseRecurrentImpl):
    def _fwd(self, x, h0, mask, need_cache):
        mb, nIn, T = x.shape
        _adt = acc_dtype(self.W("W"))
        W, RW, b = self.W("W"), self.W("RW"), self.W("b")
        dt = W.dtype
        xt = x.permute(2, 0, 1).reshape(T * mb, nIn).to(dt)
        zx = matmul(xt, W, bias=b).reshape(T, mb, -1)
        h = torch.zeros(mb, self.conf.nOut, device=x.device, dtype=_adt) if h0 is None else _acc(h0)
        zs, hs, outs = [], [], []
        for t in range(T):
            z = _acc(zx[t]) + _acc(matmul(h.to(dt), RW))
            hn = self.conf.activation.getActivation(z, True)
            if mask is not None:
                hn = hn * _acc(mask[:, t]).reshape(-1, 1)
            zs.append(z)
            hs.append(h)
            h = hn
            outs.append(h)
        self._c = {"z": zs, "hprev": hs, "xt": xt} if need_cache else None
        return torch.stack(outs, 2).to(x.dtype), h

    def activate(self, x, training=False, mask=None, stored_state=False, store_last_for_tbptt=False):
        if x.dim() == 2:
            x = x.unsqueeze(2)
        self.training = training
        x = self.applyDropOutIfNecessary(x, training)
        self.input = x
        self.maskArray = mask
        h0 = self.tBpttStateMap.get("prevAct") if stored_state else None
        out, h = self._fwd(x, h0, mask, training)
        if store_last_for_tbptt:
            self.tBpttStateMap = {"prevAct": h.detach()}
        return out

    def rnnTimeStep(self, x, mask=None):
        self._check_state_mb(x)
        is2d = x.dim() == 2
        if is2d:
            x = x.unsqueeze(2)
        out, h = self._fwd(x, self.stateMap.get("prevAct"), mask, False)
        self.stateMap = {"prevAct": h}
        return out[:, :, 0] if is2d else out

    def backpropGradient(self, eps, tbptt_back=None):
        mb, H, T = eps.shape
        _adt = acc_dtype(self.W("W"))
        RW = _acc(self.W("RW"))
        c = self._c
        dh_next = torch.zeros(mb, H, device=eps.device, dtype=_adt)
        dz_all = torch.zeros(T, mb, H, device=eps.device, dtype=_adt)
        t_end = max(0, T - tbptt_back) if tbptt_back else 0
        for t in range(T - 1, t_end - 1, -1):
            dh = _acc(eps[:, :, t]) + dh_next
            if self.maskArray is not None:
                dh = dh * _acc(self.maskArray[:, t]).reshape(-1, 1)
            dz = self.conf.activation.backprop(c["z"][t], dh)
            dz_all[t] = dz
            dh_next = matmul(dz, RW.t())
        dzf = dz_all.reshape(T * mb, H)
        weight_grad_(self.grads["W"], _acc(c["xt"]).t(), dzf)
        weight_grad_(self.grads["RW"], torch.stack(c["hprev"], 0).reshape(T * mb, H).t(), dzf)
        copy_grad_(self.grads["b"], dzf.sum(0))
        dx = matmul(dzf.to(self.W("W").dtype), self.W("W").t()).reshape(T, mb, -1).permute(1, 2, 0)
        return self.make_gradient(), self.backpropDropOut(dx.to(eps.dtype))


class _SubView(LayerImpl):
    """A child layer sharing a prefix-filtered view of the parent's params/grads."""


class BidirectionalImpl(BaseRecurrentImpl):
    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.fwd = conf.underlying.instantiate(index=index, net=net)
        self.bwd = conf.underlying.instantiate(index=index, net=net)

    def bind(self):
        for d, layer in (("f", self.fwd), ("b", self.bwd)):
            layer.params = {k[1:]: v for k, v in self.params.items() if k.startswith(d)}
            layer.cparams = {k[1:]: v for k, v in self.cparams.items() if k.startswith(d)}
            layer.grads = {k[1:]: v for k, v in self.grads.items() if k.startswith(d)}

    def activate(self, x, training=False, mask=None, **kw):
        from ..util.time_series import reverse_time_series
        self.bind()
        self.maskArray = mask
        of = self.fwd.activate(x, training, mask)
        xr = reverse_time_series(x, mask)
        ob = reverse_time_series(self.bwd.activate(xr, training, reverse_time_series(mask, mask) if mask is not None
                                                   else None), mask)
        self._of, self._ob = of, ob
        m = self.conf.mode.upper()
        if m == "CONCAT":
            return torch.cat([of, ob], dim=1)
        if m == "ADD":
            return of + ob
        if m == "MUL":
            return of * ob
        if m == "AVERAGE":
            return (of + ob) / 2
        raise ValueError(m)

    def backpropGradient(self, eps, tbptt_back=None):
        from ..util.time_series import reverse_time_series
        m = self.conf.mode.upper()
        if m == "CONCAT":
            n = self._of.shape[1]
            ef, eb = eps[:, :n], eps[:, n:]
        elif m == "ADD":
            ef = eb = eps
        elif m == "MUL":
            ef, eb = eps * self._ob, eps * self._of
        else:
            ef = eb = eps / 2
        _, dxf = self.fwd.backpropGradient(ef)
        _, dxb = self.bwd.backpropGradient(reverse_time_series(eb, self.maskArray))
        return self.make_gradient(), dxf + reverse_time_series(dxb, self.maskArray)

    def rnnClearPreviousState(self):
        self.fwd.rnnClearPreviousState() if hasattr(self.fwd, "rnnClearPreviousState") else None
        self.bwd.rnnClearPreviousState() if hasattr(self.bwd, "rnnClearPreviousState") else None


class LastTimeStepImpl(LayerImpl):
    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.inner = conf.underlying.instantiate(index=index, net=net)

    def bind(self):
        self.inner.params, self.inner.cparams, self.inner.grads = self.params, self.cparams, self.grads

    def getUnderlying(self):
        self.bind()
        return self.inner

    def activate(self, x, training=False, mask=None, **kw):
        from ..util.time_series import last_time_step
        self.bind()
        out = self.inner.activate(x, training, mask)
        self._shape = out.shape
        self.maskArray = mask
        if mask is None:
            self._idx = None
            return out[:, :, -1]
        self._idx = mask.reshape(mask.shape[0], -1).sum(dim=1).long().clamp(min=1) - 1
        return last_time_step(out, mask)

    def backpropGradient(self, eps, tbptt_back=None):
        g = torch.zeros(self._shape, dtype=eps.dtype, device=eps.device)
        if self._idx is None:
            g[:, :, -1] = eps
        else:
            g[torch.arange(self._shape[0], device=eps.device), :, self._idx] = eps
        return self.inner.backpropGradient(g)

    def feedForwardMaskArray(self, mask, state, mb):
        self.maskArray = mask
        return None, state

    def rnnClearPreviousState(self):
        if hasattr(self.inner, "rnnClearPreviousState"):
            self.inner.rnnClearPreviousState()
