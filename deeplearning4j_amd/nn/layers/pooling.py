"""GlobalPoolingLayer: masked MAX/AVG/SUM/PNORM over time (RNN) or space (CNN)
(reference nn/layers/pooling/GlobalPoolingLayer.java, nn/util/MaskedReductionUtil.java:39-53)."""
import torch

from ..conf.enums import PoolingType
from .base import LayerImpl
from deeplearning4j_amd.nn.util.dtypes import acc as _acc  # noqa: E402


class GlobalPoolingLayerImpl(LayerImpl):
    def _dims(self, x):
        if self.conf.poolingDimensions:
            return tuple(self.conf.poolingDimensions)
        return (2,) if x.dim() == 3 else (2, 3)

    def _nhwc_fast(self, x, mask, dims, pt):
        """AVG/SUM over H,W of a channels-last 4-D tensor: reduce the contiguous [N, H*W, C] view in fp32 without
        materialising an fp32 copy (the generic path converts the whole activation and reduces over strided dims)."""
        return (x.dim() == 4 and mask is None and dims == (2, 3) and pt in (PoolingType.AVG, PoolingType.SUM)
                and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous())

    @staticmethod
    def _cnn_mask(mask, x):
        """A [mb, H] or [mb, W] mask over CNN activations whose other spatial size is 1 (reference
        MaskedReductionUtil.maskedPoolingConvolution), or a [mb, 1, H, W] mask, as [mb, 1, H, W]."""
        n, _, h, w = x.shape
        if mask.dim() == 4:
            return mask.expand(n, 1, h, w)
        if mask.dim() == 2 and mask.shape[1] == w and (h == 1 or mask.shape[1] != h):
            return mask.reshape(n, 1, 1, w).expand(n, 1, h, w)
        if mask.dim() == 2 and mask.shape[1] == h:
            return mask.reshape(n, 1, h, 1).expand(n, 1, h, w)
        raise ValueError(f"GlobalPooling: a mask of shape {tuple(mask.shape)} does not fit CNN activations "
                         f"{tuple(x.shape)}; use [mb, H] with W == 1 or [mb, W] with H == 1")

    def activate(self, x, training=False, mask=None):
        self.input = x
        dims = self._dims(x)
        pt = self.conf.poolingType
        if self._nhwc_fast(x, mask, dims, pt):
            n, c, h, w = x.shape
            v = x.permute(0, 2, 3, 1).reshape(n, h * w, c)
            out = v.sum(dim=1, dtype=_acc(x[:0]).dtype)
            if pt == PoolingType.AVG:
                out = out / (h * w)
            self._fast = (n, c, h, w)
            self._mask = None
            self._keep_shape = (n, c, 1, 1)
            out = out.reshape(n, c, 1, 1)
            if self.conf.collapseDimensions:
                out = out.reshape(n, c)
            return out.to(x.dtype)
        self._fast = None
        xf = _acc(x)
        m = None
        if mask is not None and x.dim() == 3:
            m = _acc(mask).unsqueeze(1)                                  # [mb,1,T]
        elif mask is not None and x.dim() == 4:
            m = self._cnn_mask(_acc(mask), x)                           # [mb,1,H,W]
        self._mask = m
        if pt == PoolingType.MAX:
            xm = xf if m is None else xf.masked_fill(m == 0, float("-inf"))
            out = xm.amax(dim=dims, keepdim=True)
            self._argmask = (xm == out)
            cnt = self._argmask.sum(dim=dims, keepdim=True).clamp(min=1)
            self._argmask = _acc(self._argmask) / cnt
        elif pt == PoolingType.AVG:
            if m is None:
                out = xf.mean(dim=dims, keepdim=True)
                self._n = 1
                for d in dims:
                    self._n *= x.shape[d]
            else:
                self._n = m.sum(dim=dims, keepdim=True).clamp(min=1)
                out = (xf * m).sum(dim=dims, keepdim=True) / self._n
        elif pt == PoolingType.SUM:
            out = (xf if m is None else xf * m).sum(dim=dims, keepdim=True)
        elif pt == PoolingType.PNORM:
            p = self.conf.pnorm
            xa = torch.abs(xf) ** p
            if m is not None:
                xa = xa * m
            out = xa.sum(dim=dims, keepdim=True) ** (1.0 / p)
            self._pn = out
        else:
            raise ValueError(pt)
        self._keep_shape = out.shape
        if self.conf.collapseDimensions:
            out = out.reshape(out.shape[0], out.shape[1])
        return out.to(x.dtype)

    def backpropGradient(self, eps):
        x = self.input
        pt = self.conf.poolingType
        if getattr(self, "_fast", None) is not None:
            n, c, h, w = self._fast
            e = _acc(eps).reshape(n, 1, 1, c)
            if pt == PoolingType.AVG:
                e = e / (h * w)
            g = e.to(eps.dtype).expand(n, h, w, c).contiguous().permute(0, 3, 1, 2)   # channels-last, one write
            return self.make_gradient(), g
        e = _acc(eps).reshape(self._keep_shape)
        if pt == PoolingType.MAX:
            g = e * self._argmask
        elif pt == PoolingType.AVG:
            g = (e / self._n).expand(x.shape).clone()
            if self._mask is not None:
                g = g * self._mask
        elif pt == PoolingType.SUM:
            g = e.expand(x.shape).clone()
            if self._mask is not None:
                g = g * self._mask
        else:
            p = self.conf.pnorm
            xf = _acc(x)
            g = e * torch.abs(xf) ** (p - 1) * torch.sign(xf) * torch.clamp(self._pn, min=1e-12) ** (1 - p)
            if self._mask is not None:
                g = g * self._mask
        return self.make_gradient(), g.to(eps.dtype)

    def feedForwardMaskArray(self, mask, state, mb):
        self.maskArray = mask
        return None, state
