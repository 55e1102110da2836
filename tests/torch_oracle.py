"""Independent NCHW PyTorch (fp64 autograd) interpreter for Caffe NetParameters.

Used as the oracle for whole-net tests: it never touches sparknet_amd's layers, layouts
or kernels — only the NetParameter, Caffe-layout weights and the inputs.
"""
import math

import torch
import torch.nn.functional as F


def _kp(cp):
    if cp.HasField("kernel_h"):
        k = (cp.kernel_h, cp.kernel_w)
    else:
        k = (cp.kernel_size[0],) * 2
    s = (cp.stride_h, cp.stride_w) if cp.HasField("stride_h") else ((cp.stride[0],) * 2 if len(cp.stride) else (1, 1))
    p = (cp.pad_h, cp.pad_w) if cp.HasField("pad_h") else ((cp.pad[0],) * 2 if len(cp.pad) else (0, 0))
    return k, s, p


def _pool(x, pp):
    if pp.global_pooling:
        k, s, p = (x.shape[2], x.shape[3]), (1, 1), (0, 0)
    else:
        k = (pp.kernel_h, pp.kernel_w) if pp.HasField("kernel_h") else (pp.kernel_size,) * 2
        s = (pp.stride_h, pp.stride_w) if pp.HasField("stride_h") else (pp.stride,) * 2
        p = (pp.pad_h, pp.pad_w) if pp.HasField("pad_h") else (pp.pad,) * 2
    H, W = x.shape[2:]
    P = int(math.ceil((H + 2 * p[0] - k[0]) / s[0])) + 1
    Q = int(math.ceil((W + 2 * p[1] - k[1]) / s[1])) + 1
    if p[0] and (P - 1) * s[0] >= H + p[0]:
        P -= 1
    if p[1] and (Q - 1) * s[1] >= W + p[1]:
        Q -= 1
    out = []
    for i in range(P):
        row = []
        for j in range(Q):
            hs, ws = i * s[0] - p[0], j * s[1] - p[1]
            he, we = min(hs + k[0], H + p[0]), min(ws + k[1], W + p[1])
            size = (he - hs) * (we - ws)
            h0, w0, h1, w1 = max(hs, 0), max(ws, 0), min(he, H), min(we, W)
            win = x[:, :, h0:h1, w0:w1]
            if pp.pool == 0:
                row.append(win.amax(dim=(2, 3)))
            else:
                row.append(win.sum(dim=(2, 3)) / size)
        out.append(torch.stack(row, -1))
    return torch.stack(out, -2)


def _lrn(x, p):
    size, a, b, k = p.local_size, p.alpha, p.beta, p.k
    pre = (size - 1) // 2
    if p.norm_region == 1:
        sq = F.avg_pool2d(x * x, size, 1, pre, count_include_pad=True)
        return x * (1 + a * sq) ** (-b)
    sq = F.pad(x * x, (0, 0, 0, 0, pre, size - pre - 1))
    s = sum(sq[:, i:i + x.shape[1]] for i in range(size))
    return x * (k + a / size * s) ** (-b)


def run(netparam, phase, weights: dict, inputs: dict):
    """Returns (total loss, dict of output tensors, dict name->list of leaf weight tensors)."""
    from sparknet_amd.core.net import filter_net
    from sparknet_amd import proto
    n = proto.copy(netparam)
    n.state.phase = phase
    n = filter_net(n)
    blobs = {k: v.double() for k, v in inputs.items()}
    leaves = {}
    total = 0.0
    outs = {}
    for l in n.layer:
        t = l.type
        if t in ("JavaData", "DummyData", "Input"):
            continue
        bots = [blobs[b] for b in l.bottom]
        w = None
        if l.name in weights:
            w = [x.double().clone().requires_grad_(True) for x in weights[l.name]]
            leaves[l.name] = w
        if t == "Convolution":
            cp = l.convolution_param
            k, s, p = _kp(cp)
            y = F.conv2d(bots[0], w[0], w[1] if len(w) > 1 else None, s, p, groups=cp.group)
        elif t == "InnerProduct":
            x = bots[0].reshape(bots[0].shape[0], -1)
            y = x @ w[0].t() + (w[1] if len(w) > 1 else 0)
        elif t == "ReLU":
            y = F.relu(bots[0])
        elif t == "Pooling":
            y = _pool(bots[0], l.pooling_param)
        elif t == "LRN":
            y = _lrn(bots[0], l.lrn_param)
        elif t == "Dropout":
            y = bots[0]
        elif t == "Concat":
            y = torch.cat(bots, 1)
        elif t == "SoftmaxWithLoss":
            lab = bots[1].reshape(-1).long()
            y = F.cross_entropy(bots[0].reshape(bots[0].shape[0], -1), lab)
            lw = l.loss_weight[0] if len(l.loss_weight) else 1.0
            total = total + lw * y
        elif t == "Accuracy":
            lab = bots[1].reshape(-1).long()
            y = (bots[0].argmax(1) == lab).double().mean()
        elif t == "EuclideanLoss":
            d = bots[0] - bots[1]
            y = (d * d).sum() / bots[0].shape[0] / 2
            total = total + y
        else:
            raise NotImplementedError(t)
        blobs[l.top[0]] = y
        outs[l.top[0]] = y
    return total, outs, leaves
