"""Image classifier over a TEST-phase net (caffe/python/caffe/classifier.py): resize to
``image_dims``, centre crop or 10-crop oversampling, the io.Transformer preprocessing,
batched forward, mean of the 10 crop predictions."""
from __future__ import annotations

import numpy as np

from .. import proto
from . import io as caffe_io
from .net import Net


class Classifier(Net):
    def __init__(self, model_file, pretrained_file, image_dims=None, mean=None, input_scale=None,
                 raw_scale=None, channel_swap=None):
        super().__init__(model_file, pretrained_file, proto.TEST)
        in_ = self.inputs[0]
        shape = self.blobs[in_].shape
        self.transformer = caffe_io.Transformer({in_: shape})
        self.transformer.set_transpose(in_, (2, 0, 1))
        if mean is not None:
            self.transformer.set_mean(in_, mean)
        if input_scale is not None:
            self.transformer.set_input_scale(in_, input_scale)
        if raw_scale is not None:
            self.transformer.set_raw_scale(in_, raw_scale)
        if channel_swap is not None:
            self.transformer.set_channel_swap(in_, channel_swap)
        self.crop_dims = np.array(shape[2:])
        self.image_dims = np.array(image_dims if image_dims is not None else self.crop_dims)

    def predict(self, inputs, oversample: bool = True) -> np.ndarray:
        """(N x classes) probabilities for a list of H x W x K images."""
        imgs = np.zeros((len(inputs), int(self.image_dims[0]), int(self.image_dims[1]), inputs[0].shape[2]),
                        dtype=np.float32)
        for i, im in enumerate(inputs):
            imgs[i] = caffe_io.resize_image(im, self.image_dims)
        if oversample:
            crops = caffe_io.oversample(imgs, self.crop_dims)
        else:
            c = self.image_dims / 2.0
            lo = (c - self.crop_dims / 2.0).astype(int)
            hi = lo + self.crop_dims
            crops = imgs[:, lo[0]:hi[0], lo[1]:hi[1], :]
        in_ = self.inputs[0]
        batch = np.stack([self.transformer.preprocess(in_, x) for x in crops])
        pred = self.forward_all(**{in_: batch})[self.outputs[0]]
        pred = pred.reshape(pred.shape[0], -1)
        if oversample:
            pred = pred.reshape(len(pred) // 10, 10, -1).mean(1)
        return pred
