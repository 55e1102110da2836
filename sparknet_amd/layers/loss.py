"""Loss and output layers: SoftmaxWithLoss, Softmax, Accuracy, EuclideanLoss,
SigmoidCrossEntropyLoss, HingeLoss, MultinomialLogisticLoss, InfogainLoss,
ContrastiveLoss.

References: caffe/src/caffe/layers/{softmax_loss,softmax,accuracy,euclidean_loss,
sigmoid_cross_entropy_loss,hinge_loss,multinomial_logistic_loss,infogain_loss,
contrastive_loss,loss}_layer.{cpp,cu}.

The reference synchronises with the host for every loss scalar (cublasSasum/Sdot,
softmax_loss_layer.cu:51-54); here losses stay on device as 0-d tensors and the
fused softmax-cross-entropy kernel produces loss, normaliser and probabilities in one
launch (``ops.hip.softmax_loss_forward``).
"""
from __future__ import annotations

import torch

from .. import ops
from ..core.layer import Layer, register


def _prod(dims) -> int:
    n = 1
    for d in dims:
        n *= int(d)
    return n


def rows_view(blob, axis, diff=False):
    """[outer*inner, channels] view of a blob along ``axis`` (Caffe's outer-major, inner-minor
    row order: softmax_loss_layer.cpp:36-37 canonicalises any axis).  A 4-D blob's storage
    is NHWC: axis 1 is already channels-last; any other axis goes through the logical NCHW
    layout first."""
    t = blob.diff if diff else blob.data
    axis = blob.canonical_axis(axis)
    if blob.is_image:
        if axis == 1:
            return t.reshape(-1, blob.shape[1])
        t = _lh().nhwc_to_nchw(t) if t.is_cuda else t.permute(0, 3, 1, 2)
    elif axis == len(blob.shape) - 1 or blob.count_range(axis + 1) == 1:
        return t.reshape(-1, blob.shape[axis])
    # generic: move axis last ([outer][A][inner] -> [outer][inner][A])
    outer, A, inner = _prod(blob.shape[:axis]), blob.shape[axis], _prod(blob.shape[axis + 1:])
    if inner == 1:
        return t.reshape(-1, A)
    if t.is_cuda:
        return _lh().transpose(t.contiguous(), outer, A, inner).reshape(-1, A)
    return t.reshape(outer, A, inner).permute(0, 2, 1).reshape(-1, A)


def rows_view_back(rows, blob, axis):
    """Inverse of :func:`rows_view` for a result in the [rows, A] layout."""
    axis = blob.canonical_axis(axis)
    if (blob.is_image and axis == 1) or (not blob.is_image and (
            axis == len(blob.shape) - 1 or blob.count_range(axis + 1) == 1)):
        return rows.reshape(blob.data.shape)
    outer, A, inner = _prod(blob.shape[:axis]), blob.shape[axis], _prod(blob.shape[axis + 1:])
    if inner == 1:
        t = rows
    elif rows.is_cuda:
        t = _lh().transpose(rows.contiguous().reshape(outer, inner, A), outer, inner, A)
    else:
        t = rows.reshape(outer, inner, A).permute(0, 2, 1)
    if not blob.is_image:
        return t.reshape(blob.data.shape)
    N, C_, H, W = blob.shape
    if rows.is_cuda:
        return _lh().nchw_to_nhwc(t.contiguous().reshape(N, C_, H * W), N, C_, H, W)
    return t.reshape(N, C_, H, W).permute(0, 2, 3, 1).contiguous()


def _lh():
    from ..ops import layers_hip
    return layers_hip


def _sample_rows(blob, diff=False):
    """[N, count / N] in Caffe's logical per-sample order (NHWC images are transposed)."""
    t = blob.diff if diff else blob.data
    N = blob.shape[0] if blob.shape else 1
    if blob.is_image and blob.shape[2] * blob.shape[3] > 1:
        t = _lh().nhwc_to_nchw(t)
    return t.reshape(N, -1)


def _sample_rows_back(g, blob):
    """Inverse of :func:`_sample_rows` for a gradient."""
    if blob.is_image and blob.shape[2] * blob.shape[3] > 1:
        N, C_, H, W = blob.shape
        return _lh().nchw_to_nhwc(g.reshape(N, C_, H * W), N, C_, H, W)
    return g.reshape(blob.data.shape)


class _RowLossGPU:
    """Shared GPU path of the row-structured losses: per-row terms in one HIP kernel, a
    deterministic device sum (no host sync), gradients in one HIP kernel."""

    kind = ""

    def _gpu_label(self, bottoms):
        return bottoms[1].data.reshape(-1).float() if len(bottoms) > 1 else None

    def gpu_forward(self, x, t, label, H=None, margin=0.0, legacy=False):
        lh = _lh()
        M = x.shape[0]
        self._ws = lh.loss_rows_fwd(self.kind, x, t, label, H, M, x.shape[1], margin, legacy)
        return lh.loss_sum(self._ws, M, 1.0 / M)

    def gpu_backward(self, x, t, label, lw, H=None, margin=0.0, legacy=False):
        M = x.shape[0]
        return _lh().loss_rows_bwd(self.kind, x, t, label, H, M, x.shape[1], lw, 1.0 / M, 1.0, self._ws, margin,
                                   legacy)


class LossLayer(Layer):
    is_loss = True
    auto_top_blobs = True   # loss_layer.hpp: AutoTopBlobs() -> anonymous loss top
    min_bottoms = 2
    exact_tops = -1
    min_tops = 1

    def reshape(self, bottoms, tops):
        tops[0].reshape((), torch.float32)

    def allow_force_backward(self, bottom_id: int) -> bool:
        """Labels / targets never get a forced gradient (loss_layer.hpp AllowForceBackward)."""
        return bottom_id != 1


@register("SoftmaxWithLoss")
class SoftmaxWithLossLayer(LossLayer):
    exact_bottoms = 2
    max_tops = 2

    def layer_setup(self, bottoms, tops):
        lp = self.lp.loss_param
        self.ignore_label = lp.ignore_label if lp.HasField("ignore_label") else None
        self.normalize = lp.normalize
        self.axis = bottoms[0].canonical_axis(self.lp.softmax_param.axis)

    def reshape(self, bottoms, tops):
        tops[0].reshape((), torch.float32)
        b = bottoms[0]
        outer = b.count_range(0, self.axis)
        inner = b.count_range(self.axis + 1)
        if outer * inner != bottoms[1].count:
            raise ValueError("Number of labels must match number of predictions")
        self.outer = outer
        if len(tops) > 1:
            tops[1].reshape(b.shape, self.dtype)

    def forward(self, bottoms, tops):
        x2 = rows_view(bottoms[0], self.axis)
        loss, prob, norm = ops.softmax_loss_forward(x2, bottoms[1].data, self.ignore_label,
                                                    self.normalize, self.outer)
        self.prob, self.norm = prob, norm
        tops[0].data = loss.reshape(())
        if len(tops) > 1:
            tops[1].data = rows_view_back(prob, bottoms[0], self.axis).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if len(propagate_down) > 1 and propagate_down[1]:
            raise ValueError("SoftmaxWithLoss cannot backpropagate to label inputs")
        if propagate_down[0]:
            g = ops.softmax_loss_backward(self.prob, bottoms[1].data, tops[0].diff, self.norm,
                                          self.ignore_label, bottoms[0].dtype)
            bottoms[0].diff = rows_view_back(g, bottoms[0], self.axis).to(bottoms[0].dtype)


@register("Softmax")
class SoftmaxLayer(Layer):
    exact_bottoms = 1
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        self.axis = bottoms[0].canonical_axis(self.lp.softmax_param.axis)

    def reshape(self, bottoms, tops):
        tops[0].reshape(bottoms[0].shape, self.dtype)

    def forward(self, bottoms, tops):
        b = bottoms[0]
        tops[0].data = rows_view_back(ops.softmax_forward(rows_view(b, self.axis)), b, self.axis).to(self.dtype)

    def backward(self, tops, propagate_down, bottoms):
        if not propagate_down[0]:
            return
        t, b = tops[0], bottoms[0]
        g = ops.softmax_backward(rows_view(t, self.axis, diff=True), rows_view(t, self.axis))
        b.diff = rows_view_back(g, b, self.axis).to(b.dtype)


@register("Accuracy")
class AccuracyLayer(Layer):
    exact_bottoms = 2
    exact_tops = 1

    def layer_setup(self, bottoms, tops):
        p = self.lp.accuracy_param
        self.top_k = int(p.top_k)
        self.axis = bottoms[0].canonical_axis(p.axis)
        self.ignore_label = p.ignore_label if p.HasField("ignore_label") else None

    def reshape(self, bottoms, tops):
        tops[0].reshape((), torch.float32)

    def forward(self, bottoms, tops):
        x2 = rows_view(bottoms[0], self.axis)
        tops[0].data = ops.accuracy(x2, bottoms[1].data, self.top_k, self.ignore_label).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if any(propagate_down):
            raise NotImplementedError("Accuracy has no backward")


@register("EuclideanLoss")
class EuclideanLossLayer(LossLayer, _RowLossGPU):
    exact_bottoms = 2
    kind = "Euclidean"

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            a, b = bottoms[0].data.reshape(bottoms[0].shape[0], -1), bottoms[1].data.reshape(bottoms[0].shape[0], -1)
            tops[0].data = self.gpu_forward(a, b, None).reshape(())
            return
        self.d = bottoms[0].data.float() - bottoms[1].data.float()
        n = bottoms[0].shape[0]
        tops[0].data = ((self.d * self.d).sum() / n / 2.0).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        n = bottoms[0].shape[0]
        if tops[0].diff.is_cuda:
            rows = [bottoms[i].data.reshape(n, -1) for i in range(2)]
            for i in range(2):
                if propagate_down[i]:  # d/dx_i of |x_0 - x_1|^2 / 2N = (x_i - x_other) / N
                    g = self.gpu_backward(rows[i], rows[1 - i], None, tops[0].diff)
                    bottoms[i].diff = g.reshape(bottoms[i].data.shape)
            return
        lw = tops[0].diff.float()
        for i in range(2):
            if propagate_down[i]:
                sign = 1.0 if i == 0 else -1.0
                bottoms[i].diff = (self.d * (sign * lw / n)).to(bottoms[i].dtype)


@register("SigmoidCrossEntropyLoss")
class SigmoidCrossEntropyLossLayer(LossLayer, _RowLossGPU):
    exact_bottoms = 2
    kind = "SigmoidXent"

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            x, t = _sample_rows(bottoms[0]), _sample_rows(bottoms[1])
            tops[0].data = self.gpu_forward(x, t.reshape(x.shape), None).reshape(())
            return
        x = bottoms[0].data.float()
        t = bottoms[1].data.float().reshape(x.shape)
        self.sig = torch.sigmoid(x)
        loss = -(x * (t - (x >= 0).float()) - torch.log1p(torch.exp(x - 2 * x * (x >= 0).float())))
        tops[0].data = (loss.sum() / bottoms[0].shape[0]).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if len(propagate_down) > 1 and propagate_down[1]:
            raise ValueError("SigmoidCrossEntropyLoss cannot backpropagate to label inputs")
        if propagate_down[0] and tops[0].diff.is_cuda:
            x, t = _sample_rows(bottoms[0]), _sample_rows(bottoms[1])
            g = self.gpu_backward(x, t.reshape(x.shape), None, tops[0].diff)
            bottoms[0].diff = _sample_rows_back(g, bottoms[0])
            return
        if propagate_down[0]:
            t = bottoms[1].data.float().reshape(self.sig.shape)
            g = (self.sig - t) * (tops[0].diff.float() / bottoms[0].shape[0])
            bottoms[0].diff = g.to(bottoms[0].dtype)


@register("HingeLoss")
class HingeLossLayer(LossLayer, _RowLossGPU):
    exact_bottoms = 2

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            self.kind = "HingeL2" if int(self.lp.hinge_loss_param.norm) == 2 else "HingeL1"
            tops[0].data = self.gpu_forward(_sample_rows(bottoms[0]), None, self._gpu_label(bottoms)).reshape(())
            return
        x = rows_view(bottoms[0], 1).float()
        lab = bottoms[1].data.reshape(-1).long()
        sign = -torch.ones_like(x)
        sign.scatter_(1, lab[:, None], 1.0)
        self.m = torch.clamp(1 - sign * x, min=0)
        self.sign = sign
        l2 = int(self.lp.hinge_loss_param.norm) == 2
        self.l2 = l2
        v = (self.m * self.m).sum() if l2 else self.m.sum()
        tops[0].data = (v / x.shape[0]).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and tops[0].diff.is_cuda:
            g = self.gpu_backward(_sample_rows(bottoms[0]), None, self._gpu_label(bottoms), tops[0].diff)
            bottoms[0].diff = _sample_rows_back(g, bottoms[0])
            return
        if propagate_down[0]:
            n = self.m.shape[0]
            g = -self.sign * ((2 * self.m) if self.l2 else (self.m > 0).float())
            g = g * (tops[0].diff.float() / n)
            bottoms[0].diff = g.reshape(bottoms[0].data.shape).to(bottoms[0].dtype)


@register("MultinomialLogisticLoss")
class MultinomialLogisticLossLayer(LossLayer, _RowLossGPU):
    exact_bottoms = 2
    kind = "Multinomial"

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            tops[0].data = self.gpu_forward(_sample_rows(bottoms[0]), None, self._gpu_label(bottoms)).reshape(())
            return
        p = rows_view(bottoms[0], 1).float()
        lab = bottoms[1].data.reshape(-1).long()
        self.pl = p.gather(1, lab[:, None]).clamp_min(1e-20)
        tops[0].data = (-torch.log(self.pl).sum() / p.shape[0]).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and tops[0].diff.is_cuda:
            g = self.gpu_backward(_sample_rows(bottoms[0]), None, self._gpu_label(bottoms), tops[0].diff)
            bottoms[0].diff = _sample_rows_back(g, bottoms[0])
            return
        if propagate_down[0]:
            p = rows_view(bottoms[0], 1).float()
            lab = bottoms[1].data.reshape(-1).long()
            g = torch.zeros_like(p)
            g.scatter_(1, lab[:, None], -1.0 / self.pl)
            g = g * (tops[0].diff.float() / p.shape[0])
            bottoms[0].diff = g.reshape(bottoms[0].data.shape).to(bottoms[0].dtype)


@register("InfogainLoss")
class InfogainLossLayer(LossLayer, _RowLossGPU):
    min_bottoms = 2
    max_bottoms = 3
    kind = "Infogain"

    def _gpu_H(self, bottoms, dim):
        H = self.H if self.H is not None else bottoms[2].data
        return H.reshape(dim, -1).float().contiguous()

    def layer_setup(self, bottoms, tops):
        self.H = None
        if len(bottoms) < 3:
            from ..core.net import blob_proto_to_tensor
            from .. import proto
            src = self.lp.infogain_loss_param.source
            self.H = blob_proto_to_tensor(proto.read_binary(src, proto.BlobProto)).reshape(
                bottoms[0].shape[1], -1).to(self.device)

    def forward(self, bottoms, tops):
        if bottoms[0].data.is_cuda:
            x = _sample_rows(bottoms[0])
            self._Hg = self._gpu_H(bottoms, x.shape[1])
            tops[0].data = self.gpu_forward(x, None, self._gpu_label(bottoms), self._Hg).reshape(())
            return
        p = rows_view(bottoms[0], 1).float()
        H = self.H if self.H is not None else bottoms[2].data.float().reshape(p.shape[1], -1)
        lab = bottoms[1].data.reshape(-1).long()
        self.Hl = H[lab]
        self.p = p.clamp_min(1e-20)
        tops[0].data = (-(self.Hl * torch.log(self.p)).sum() / p.shape[0]).reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if propagate_down[0] and tops[0].diff.is_cuda:
            g = self.gpu_backward(_sample_rows(bottoms[0]), None, self._gpu_label(bottoms), tops[0].diff, self._Hg)
            bottoms[0].diff = _sample_rows_back(g, bottoms[0])
            return
        if propagate_down[0]:
            g = -self.Hl / self.p * (tops[0].diff.float() / self.p.shape[0])
            bottoms[0].diff = g.reshape(bottoms[0].data.shape).to(bottoms[0].dtype)


@register("ContrastiveLoss")
class ContrastiveLossLayer(LossLayer, _RowLossGPU):
    exact_bottoms = 3
    kind = "Contrastive"

    def forward(self, bottoms, tops):
        p = self.lp.contrastive_loss_param
        if bottoms[0].data.is_cuda:
            n = bottoms[0].shape[0]
            a, b = bottoms[0].data.reshape(n, -1), bottoms[1].data.reshape(n, -1)
            self._y = bottoms[2].data.reshape(-1).float()
            tops[0].data = self.gpu_forward(a, b, self._y, None, p.margin, p.legacy_version).reshape(())
            return
        a = bottoms[0].data.float().reshape(bottoms[0].shape[0], -1)
        b = bottoms[1].data.float().reshape(a.shape)
        y = bottoms[2].data.float().reshape(-1)
        self.diff = a - b
        self.d2 = (self.diff * self.diff).sum(1)
        self.margin, self.legacy = p.margin, p.legacy_version
        if self.legacy:
            neg = torch.clamp(self.margin - self.d2, min=0)
        else:
            neg = torch.clamp(self.margin - torch.sqrt(self.d2), min=0) ** 2
        self.y = y
        loss = torch.where(y > 0, self.d2, neg).sum() / a.shape[0] / 2.0
        tops[0].data = loss.reshape(())

    def backward(self, tops, propagate_down, bottoms):
        if tops[0].diff.is_cuda:
            p = self.lp.contrastive_loss_param
            n = bottoms[0].shape[0]
            rows = [bottoms[i].data.reshape(n, -1) for i in range(2)]
            for i in range(2):
                if propagate_down[i]:  # gradient of bottom i: coef * (x_i - x_other) * lw / N
                    g = self.gpu_backward(rows[i], rows[1 - i], self._y, tops[0].diff, None, p.margin,
                                          p.legacy_version)
                    bottoms[i].diff = g.reshape(bottoms[i].data.shape)
            return
        n = self.diff.shape[0]
        lw = tops[0].diff.float() / n
        if self.legacy:
            negc = -(self.margin - self.d2 > 0).float()
        else:
            dist = torch.sqrt(self.d2)
            mdist = self.margin - dist
            negc = -(mdist > 0).float() * mdist / (dist + 1e-4)
        coef = torch.where(self.y > 0, torch.ones_like(self.d2), negc)[:, None]
        for i, sign in ((0, 1.0), (1, -1.0)):
            if propagate_down[i]:
                g = sign * lw * coef * self.diff
                bottoms[i].diff = g.reshape(bottoms[i].data.shape).to(bottoms[i].dtype)
