"""YOLOv2 output layer + detection utilities (reference nn/layers/objdetect/Yolo2OutputLayer.java,
YoloUtils.java, DetectedObject.java).

Input  [mb, B*(5+C), H, W]: per anchor box b: (tx, ty, tw, th, tc, class logits...).
Labels [mb, 4+C, H, W]: (x1, y1, x2, y2) of the object whose centre falls in cell (h, w), in grid units,
followed by the one-hot class; all-zero where no object.
Loss (reference computeBackpropGradientAndScore): responsible box = argmax IOU over the B anchors in cells
with an object; lambdaCoord * [L2(xy) + L2(sqrt wh)] + L2(conf vs IOU) + lambdaNoObj * L2(conf vs 0) for
non-responsible boxes + class loss (softmax, L2 by default) for responsible boxes; divided by minibatch.
The gradient is obtained by autograd through the same expression (it includes the dIOU/dxy, dIOU/dwh terms
the reference derives by hand, restricted to responsible boxes because the no-object label is 0).
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

    def _loss(self, x, labels):
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
        itl = torch.maximum(ptl, tl.unsqueeze(1))
        ibr = torch.minimum(pbr, br.unsqueeze(1))
        iwh = (ibr - itl).clamp_min(0)
        inter = iwh[:, :, 0] * iwh[:, :, 1] * obj.unsqueeze(1)
        area_p = pwh[:, :, 0] * pwh[:, :, 1]
        area_l = ((br - tl)[:, 0] * (br - tl)[:, 1]).unsqueeze(1)
        union = area_p + area_l - inter
        iou = torch.where(union > 0, inter / union.clamp_min(1e-12), torch.zeros_like(inter)) * obj.unsqueeze(1)
        resp = torch.nn.functional.one_hot(iou.detach().argmax(1), B).permute(0, 3, 1, 2).to(x.dtype)
        resp = resp * obj.unsqueeze(1)                                    # mask1_ij_obj [mb, B, H, W]
        noresp = 1 - resp
        l2 = c.lossPositionScale if getattr(c, "lossPositionScale", None) is not None else LossL2()
        lcls = c.lossClassPredictions if getattr(c, "lossClassPredictions", None) is not None else LossL2()
        ident = ActivationIdentity()

        def flat(t):   # [mb, B, k, H, W] -> [mb*B*H*W, k]
            return t.permute(0, 1, 3, 4, 2).reshape(-1, t.shape[2])
        m2 = resp.reshape(-1, 1)
        rep = lambda t: t.unsqueeze(1).expand(mb, B, *t.shape[1:])  # noqa: E731
        pos = l2.computeScore(flat(rep(center_in)), flat(pxy), ident, m2, False)
        size = l2.computeScore(flat(rep(wh_lab_sqrt)), flat(pwh.sqrt()), ident, m2, False)
        label_conf = (iou * resp).reshape(-1, 1)
        pc2 = pconf.reshape(-1, 1)
        lc = LossL2()
        conf_loss = lc.computeScore(label_conf, pc2, ident, m2, False) + \
            c.lambdaNoObj * lc.computeScore(label_conf, pc2, ident, noresp.reshape(-1, 1), False)
        cls_loss = lcls.computeScore(flat(rep(cls_lab)), flat(x5[:, :, 5:]), ActivationSoftmax(), m2, False)
        return c.lambdaCoord * (pos + size) + conf_loss + cls_loss

    def _compute(self):
        if self._cache is not None:
            return self._cache
        dt = torch.float64 if self.input.dtype == torch.float64 else torch.float32
        x = self.input.detach().to(dt).requires_grad_(True)
        with torch.enable_grad():
            loss = self._loss(x, self.labels.to(x.device))
            (g,) = torch.autograd.grad(loss, [x])
        self._cache = (loss.detach(), g)
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
