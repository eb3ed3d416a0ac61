"""YOLOv2 output layer + detection utilities (reference nn/layers/objdetect/Yolo2OutputLayer.java,
YoloUtils.java, DetectedObject.java).

Input  [mb, B*(5+C), H, W]: per anchor box b: (tx, ty, tw, th, tc, class logits...).
Labels [mb, 4+C, H, W]: (x1, y1, x2, y2) of the object whose centre falls in cell (h, w), in grid units,
followed by the one-hot class; all-zero where no object.
Loss (reference computeBackpropGradientAndScore): responsible box = argmax IOU over the B anchors in cells
with an object; lambdaCoord * [L2(xy) + L2(sqrt wh)] + L2(conf vs IOU) + lambdaNoObj * L2(conf vs 0) for
non-responsible boxes + class loss (softmax, L2 by default) for responsible boxes; divided by minibatch.
The input gradient is derived by hand (reference computeBackpropGradientAndScore :256-340 and
calculateIOULabelPredicted :364-480): position / size / class terms come from the configured loss functions'
computeGradient, the confidence label IOU contributes the dIOU/d(xy), dIOU/d(wh) path through the
intersection / union geometry, and sigmoid / exp(prior) / softmax are backpropagated in closed form.
One deliberate difference: the reference's dLc/dIOU = 2 (IOU - conf) (1_obj + lambdaNoObj 1_noobj) also charges
no-object anchors, whose confidence label is 0 and therefore independent of the IOU; here only the responsible
anchor's term is kept, which is the exact derivative of the score (tests/test_explicit_backward.py gradient-checks
the layer in fp64).
"""
import torch

from ..conf.activations import ActivationIdentity, ActivationSoftmax
from ..conf.losses import LossL2
from .base import LayerImpl


def _priors(conf, device, dtype):
    bb = conf.boundingBoxes
    if bb is None:
        raise ValueError("Yolo2OutputLayer requires boundingBoxes (anchor priors [B, 2] in grid units)")
    t = torch.as_tensor(bb, dtype=dtype, device=device).reshape(-1, 2)
    return t


def yolo_activate(boundingBoxes, x):
    """[mb, B*(5+C), H, W] -> same shape with sigmoid(xy), prior*exp(wh), sigmoid(conf), softmax(classes)."""
    mb, ch, H, W = x.shape
    pri = torch.as_tensor(boundingBoxes, dtype=x.dtype, device=x.device).reshape(-1, 2)
    B = pri.shape[0]
    C = ch // B - 5
    x5 = x.reshape(mb, B, 5 + C, H, W)
    xy = torch.sigmoid(x5[:, :, 0:2])
    wh = torch.exp(x5[:, :, 2:4]) * pri.reshape(1, B, 2, 1, 1)
    conf = torch.sigmoid(x5[:, :, 4:5])
    cls = torch.softmax(x5[:, :, 5:], dim=2)
    return torch.cat([xy, wh, conf, cls], dim=2).reshape(mb, ch, H, W)


class DetectedObject:
    def __init__(self, exampleNumber, centerX, centerY, width, height, classPredictions, confidence):
        self.exampleNumber, self.centerX, self.centerY = exampleNumber, centerX, centerY
        self.width, self.height = width, height
        self.classPredictions, self.confidence = classPredictions, confidence

    def getPredictedClass(self):
        return int(torch.argmax(self.classPredictions))

    def getTopLeftXY(self):
        return self.centerX - self.width / 2, self.centerY - self.height / 2

    def getBottomRightXY(self):
        return self.centerX + self.width / 2, self.centerY + self.height / 2

    def __repr__(self):
        return (f"DetectedObject(exampleNumber={self.exampleNumber}, centerX={self.centerX:.3f}, centerY="
                f"{self.centerY:.3f}, width={self.width:.3f}, height={self.height:.3f}, confidence="
                f"{self.confidence:.3f}, predictedClass={self.getPredictedClass()})")


class YoloUtils:
    activate = staticmethod(yolo_activate)

    @staticmethod
    def iou(a, b):
        ax1, ay1 = a.getTopLeftXY()
        ax2, ay2 = a.getBottomRightXY()
        bx1, by1 = b.getTopLeftXY()
        bx2, by2 = b.getBottomRightXY()
        iw = max(0.0, min(ax2, bx2) - max(ax1, bx1))
        ih = max(0.0, min(ay2, by2) - max(ay1, by1))
        inter = iw * ih
        union = a.width * a.height + b.width * b.height - inter
        return inter / union if union > 0 else 0.0

    @staticmethod
    def nms(objects, iouThreshold):
        """Greedy per-class non-max suppression (YoloUtils.nms)."""
        keep = []
        for o in sorted(objects, key=lambda d: -d.confidence):
            if all(o.getPredictedClass() != k.getPredictedClass() or YoloUtils.iou(o, k) < iouThreshold
                   for k in keep):
                keep.append(o)
        return keep

    @staticmethod
    def getPredictedObjects(boundingBoxPriors, networkOutput, confThreshold, nmsThreshold=0.0):
        """Objects whose confidence >= threshold from an ACTIVATED output; coordinates in grid units."""
        out = networkOutput
        mb, ch, H, W = out.shape
        pri = torch.as_tensor(boundingBoxPriors).reshape(-1, 2)
        B = pri.shape[0]
        C = ch // B - 5
        o5 = out.reshape(mb, B, 5 + C, H, W).detach().float().cpu()
        conf = o5[:, :, 4]
        idx = (conf >= confThreshold).nonzero()
        res = []
        for e, b, h, w in idx.tolist():
            v = o5[e, b, :, h, w]
            res.append(DetectedObject(e, w + float(v[0]), h + float(v[1]), float(v[2]), float(v[3]), v[5:].clone(),
                                      float(v[4])))
        if nmsThreshold > 0:
            res = YoloUtils.nms(res, nmsThreshold)
        return res


class Yolo2OutputLayerImpl(LayerImpl):
    def __init__(self, conf, index=0, net=None):
        super().__init__(conf, index, net)
        self.labels = None

    def setLabels(self, labels):
        self.labels = labels

    def getLabels(self):
        return self.labels

    def activate(self, x, training=False, mask=None, **kw):
        self.input = x
        self._cache = None
        return yolo_activate(self.conf.boundingBoxes, x)

    def _loss(self, x, labels, need_grad=False):
        """Score of one minibatch (summed over examples); with ``need_grad`` also dScore/dx."""
        c = self.conf
        mb, ch, H, W = x.shape
        pri = _priors(c, x.device, x.dtype)
        B = pri.shape[0]
        C = ch // B - 5
        lab = labels.to(x.dtype)
        tl, br = lab[:, 0:2], lab[:, 2:4]
        cls_lab = lab[:, 4:]
        obj = (cls_lab.sum(1) > 0).to(x.dtype)                           # [mb, H, W]
        center = (tl + br) * 0.5
        center_in = center - torch.floor(center)                          # [mb, 2, H, W]
        wh_lab_sqrt = (br - tl).clamp_min(0).sqrt()
        x5 = x.reshape(mb, B, 5 + C, H, W)
        pxy = torch.sigmoid(x5[:, :, 0:2])                                # [mb, B, 2, H, W]
        pwh = torch.exp(x5[:, :, 2:4]) * pri.reshape(1, B, 2, 1, 1)
        pconf = torch.sigmoid(x5[:, :, 4])                                # [mb, B, H, W]
        # IOU of every anchor's predicted box with the cell's label box (grid units)
        gy, gx = torch.meshgrid(torch.arange(H, device=x.device, dtype=x.dtype),
                                torch.arange(W, device=x.device, dtype=x.dtype), indexing="ij")
        grid = torch.stack([gx, gy], 0).reshape(1, 1, 2, H, W)
        pc = pxy + grid
        ptl, pbr = pc - 0.5 * pwh, pc + 0.5 * pwh
        ltl, lbr = tl.unsqueeze(1), br.unsqueeze(1)
        itl = torch.maximum(ptl, ltl)
        ibr = torch.minimum(pbr, lbr)
        iwh = (ibr - itl).clamp_min(0)
        obj1 = obj.unsqueeze(1)
        inter = iwh[:, :, 0] * iwh[:, :, 1] * obj1
        area_p = pwh[:, :, 0] * pwh[:, :, 1]
        area_l = ((br - tl)[:, 0] * (br - tl)[:, 1]).unsqueeze(1)
        union = area_p + area_l - inter
        valid = (union > 0).to(x.dtype) * obj1
        iou = inter / union.clamp_min(1e-12) * valid
        resp = torch.nn.functional.one_hot(iou.argmax(1), B).permute(0, 3, 1, 2).to(x.dtype)
        resp = resp * obj1                                                # mask1_ij_obj [mb, B, H, W]
        noresp = 1 - resp
        l2 = c.lossPositionScale if getattr(c, "lossPositionScale", None) is not None else LossL2()
        lcls = c.lossClassPredictions if getattr(c, "lossClassPredictions", None) is not None else LossL2()
        ident = ActivationIdentity()
        soft = ActivationSoftmax()

        def flat(t):   # [mb, B, k, H, W] -> [mb*B*H*W, k]
            return t.permute(0, 1, 3, 4, 2).reshape(-1, t.shape[2])

        def unflat(t):
            return t.reshape(mb, B, H, W, -1).permute(0, 1, 4, 2, 3)
        m2 = resp.reshape(-1, 1)
        nr2 = noresp.reshape(-1, 1)
        rep = lambda t: t.unsqueeze(1).expand(mb, B, *t.shape[1:])  # noqa: E731
        psq = pwh.sqrt()
        pos = l2.computeScore(flat(rep(center_in)), flat(pxy), ident, m2, False)
        size = l2.computeScore(flat(rep(wh_lab_sqrt)), flat(psq), ident, m2, False)
        label_conf = (iou * resp).reshape(-1, 1)
        pc2 = pconf.reshape(-1, 1)
        lc = LossL2()
        lam = c.lambdaNoObj
        conf_loss = lc.computeScore(label_conf, pc2, ident, m2, False) + \
            lam * lc.computeScore(label_conf, pc2, ident, nr2, False)
        cls_loss = lcls.computeScore(flat(rep(cls_lab)), flat(x5[:, :, 5:]), soft, m2, False)
        loss = c.lambdaCoord * (pos + size) + conf_loss + cls_loss
        if not need_grad:
            return loss
        lcd = c.lambdaCoord
        g_xy = lcd * unflat(l2.computeGradient(flat(rep(center_in)), flat(pxy), ident, m2))
        g_wh = lcd * unflat(l2.computeGradient(flat(rep(wh_lab_sqrt)), flat(psq), ident, m2)) * 0.5 / psq
        g_conf = (lc.computeGradient(label_conf, pc2, ident, m2) +
                  lam * lc.computeGradient(label_conf, pc2, ident, nr2)).reshape(mb, B, H, W)
        # confidence label = IOU on the responsible anchor: d/dlabel = -d/dconf of the (label - conf)^2 terms
        g_iou = -g_conf * resp
        u2 = union.clamp_min(1e-12) ** 2
        g_inter = g_iou * valid * (union + inter) / u2                    # d(inter / (A + L - inter))/d inter
        g_area = -g_iou * valid * inter / u2
        pos_w = ((ibr - itl) >= 0).to(x.dtype)                            # clamp_min(0) passes gradient at >= 0
        g_iwh = torch.stack([g_inter * iwh[:, :, 1], g_inter * iwh[:, :, 0]], 2) * obj1.unsqueeze(2) * pos_w

        def sel(a, b, lt):                                                # share of d min/max going to ``a``
            return (a < b).to(x.dtype) + 0.5 * (a == b).to(x.dtype) if lt else \
                (a > b).to(x.dtype) + 0.5 * (a == b).to(x.dtype)
        g_pbr = g_iwh * sel(pbr, lbr, True)
        g_ptl = -g_iwh * sel(ptl, ltl, False)
        g_xy = g_xy + g_pbr + g_ptl
        g_wh = g_wh + 0.5 * (g_pbr - g_ptl) + torch.stack([g_area * pwh[:, :, 1], g_area * pwh[:, :, 0]], 2)
        d_xy = g_xy * pxy * (1 - pxy)
        d_wh = g_wh * pwh
        d_c = (g_conf * pconf * (1 - pconf)).unsqueeze(2)
        d_cls = unflat(lcls.computeGradient(flat(rep(cls_lab)), flat(x5[:, :, 5:]), soft, m2))
        dx = torch.cat([d_xy, d_wh, d_c, d_cls.to(x.dtype)], 2).reshape(mb, ch, H, W)
        return loss, dx

    def _compute(self):
        if self._cache is not None:
            return self._cache
        dt = torch.float64 if self.input.dtype == torch.float64 else torch.float32
        with torch.no_grad():
            loss, g = self._loss(self.input.detach().to(dt), self.labels.to(self.input.device), need_grad=True)
        self._cache = (loss, g)
        return self._cache

    def computeScore(self, fullNetworkL1=0.0, fullNetworkL2=0.0, training=True):
        loss, _ = self._compute()
        return (loss + fullNetworkL1 + fullNetworkL2) / self.input.shape[0]

    def computeScoreForExamples(self, fullNetworkL1=0.0, fullNetworkL2=0.0):
        out = []
        for i in range(self.input.shape[0]):
            with torch.no_grad():
                xi = self.input[i:i + 1]
                out.append(self._loss(xi if xi.dtype == torch.float64 else xi.float(),
                                      self.labels[i:i + 1].to(self.input.device)))
        return torch.stack(out) + (fullNetworkL1 + fullNetworkL2)

    def backpropGradient(self, eps=None, **kw):
        _, g = self._compute()
        return self.make_gradient(), g.to(self.input.dtype)

    def getPredictedObjects(self, networkOutput, threshold, nmsThreshold=0.0):
        return YoloUtils.getPredictedObjects(self.conf.boundingBoxes, networkOutput, threshold, nmsThreshold)

    def clear(self):
        super().clear()
        self.labels = None
        self._cache = None
