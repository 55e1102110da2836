"""Windowed detection over a TEST-phase net (caffe/python/caffe/detector.py:23-216):
crops (optionally with R-CNN context padding) are warped to the net input, preprocessed
by the io.Transformer and classified in one ``forward_all``.

Windows are ``(ymin, xmin, ymax, xmax)``. ``detect_selective_search`` needs the external
``selective_search_ijcv_with_python`` MATLAB bridge, which is not part of this
environment; it raises ImportError unless that module is importable."""
from __future__ import annotations

import os

import numpy as np

from .. import proto
from . import io as caffe_io
from .net import Net


class Detector(Net):
    def __init__(self, model_file, pretrained_file, mean=None, input_scale=None, raw_scale=None,
                 channel_swap=None, context_pad=None):
        super().__init__(model_file, pretrained_file, proto.TEST)
        in_ = self.inputs[0]
        self.transformer = caffe_io.Transformer({in_: self.blobs[in_].shape})
        self.transformer.set_transpose(in_, (2, 0, 1))
        if mean is not None:
            self.transformer.set_mean(in_, mean)
        if input_scale is not None:
            self.transformer.set_input_scale(in_, input_scale)
        if raw_scale is not None:
            self.transformer.set_raw_scale(in_, raw_scale)
        if channel_swap is not None:
            self.transformer.set_channel_swap(in_, channel_swap)
        self.configure_crop(context_pad)

    def detect_windows(self, images_windows):
        """[(image filename, windows)] -> [{'window', 'prediction', 'filename'}]."""
        images_windows = [(f, list(ws)) for f, ws in images_windows]
        crops = []
        for fname, windows in images_windows:
            image = caffe_io.load_image(fname).astype(np.float32)
            crops.extend(self.crop(image, np.asarray(w)) for w in windows)
        in_ = self.inputs[0]
        batch = np.stack([self.transformer.preprocess(in_, c) for c in crops]).astype(np.float32)
        out = self.forward_all(**{in_: batch})
        preds = out[self.outputs[0]]
        preds = preds.reshape(preds.shape[0], -1)
        dets, ix = [], 0
        for fname, windows in images_windows:
            for w in windows:
                dets.append({"window": w, "prediction": preds[ix], "filename": fname})
                ix += 1
        return dets

    def detect_selective_search(self, image_fnames):
        import selective_search_ijcv_with_python as selective_search  # external, optional
        image_fnames = [os.path.abspath(f) for f in image_fnames]
        windows = selective_search.get_windows(image_fnames, cmd="selective_search_rcnn")
        return self.detect_windows(zip(image_fnames, windows))

    def crop(self, im, window):
        """H x W x K crop of ``window``; with context padding the box is grown so that a
        ``context_pad``-pixel border of the net input is context, out-of-image parts are
        filled with the (unprocessed-space) mean."""
        y0, x0, y1, x1 = (int(v) for v in window[:4])
        if not self.context_pad:
            return im[y0:y1, x0:x1]
        size = int(self.blobs[self.inputs[0]].shape[3])  # square input assumed, as upstream
        grow = size / (size - 2.0 * self.context_pad)
        hh, hw = (y1 - y0 + 1) / 2.0, (x1 - x0 + 1) / 2.0
        cy, cx = y0 + hh, x0 + hw
        box = np.round(np.array([cy - hh * grow, cx - hw * grow, cy + hh * grow, cx + hw * grow]))
        sh, sw = size / (box[2] - box[0] + 1), size / (box[3] - box[1] + 1)
        pad_y, pad_x = int(round(max(0.0, -box[0]) * sh)), int(round(max(0.0, -box[1]) * sw))
        ih, iw = im.shape[:2]
        box = np.clip(box, 0.0, [ih, iw, ih, iw])
        ch, cw = box[2] - box[0] + 1, box[3] - box[1] + 1
        if ch <= 0 or cw <= 0:
            raise ValueError(f"window {window} lies outside the image")
        crop_h = min(int(round(ch * sh)), size - pad_y)
        crop_w = min(int(round(cw * sw)), size - pad_x)
        b = box.astype(int)
        ctx = caffe_io.resize_image(im[b[0]:b[2], b[1]:b[3]], (crop_h, crop_w))
        out = np.array(np.broadcast_to(self.crop_mean, tuple(self.crop_dims)), dtype=np.float32)
        out[pad_y:pad_y + crop_h, pad_x:pad_x + crop_w] = ctx
        return out

    def configure_crop(self, context_pad):
        """Crop dims (H, W, K) and, with context padding, the mean mapped back to the raw
        input space (inverse transpose, inverse channel swap, divided by raw_scale)."""
        in_ = self.inputs[0]
        tpose = self.transformer.transpose[in_]
        inv = [tpose.index(i) for i in range(len(tpose))]
        self.crop_dims = np.array(self.blobs[in_].shape[1:])[inv]
        self.context_pad = context_pad
        if not context_pad:
            return
        mean = self.transformer.mean.get(in_)
        if mean is None:
            self.crop_mean = np.zeros(tuple(self.crop_dims), dtype=np.float32)
            return
        m = np.array(mean, dtype=np.float32).transpose(inv)
        swap = self.transformer.channel_swap.get(in_)
        if swap is not None:
            m = m[:, :, [list(swap).index(i) for i in range(m.shape[2])]]
        raw = self.transformer.raw_scale.get(in_)
        if raw is not None:
            m = m / raw
        self.crop_mean = m
