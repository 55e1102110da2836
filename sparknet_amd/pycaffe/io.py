"""pycaffe ``caffe.io`` equivalents (caffe/python/caffe/io.py): BlobProto / Datum <->
ndarray conversion, the input ``Transformer`` (transpose, channel swap, raw scale, mean,
input scale), image loading / resizing and 10-crop oversampling.

Images are decoded with PIL (the reference used skimage, not installed here); resizing of
1- and 3-channel images is bilinear through PIL on float32 planes, other channel counts
use scipy's ``ndimage.zoom`` like the reference.
"""
from __future__ import annotations

import numpy as np

from .. import proto


# ---- proto / datum / ndarray conversion -----------------------------------------------

def blobproto_to_array(blob, return_diff: bool = False) -> np.ndarray:
    """BlobProto -> ndarray (legacy num/channels/height/width or the N-d shape)."""
    data = np.array(blob.diff if return_diff else blob.data, dtype=np.float32)
    if blob.HasField("num") or blob.HasField("channels") or blob.HasField("height") or blob.HasField("width"):
        return data.reshape(blob.num, blob.channels, blob.height, blob.width)
    return data.reshape(tuple(blob.shape.dim))


def array_to_blobproto(arr: np.ndarray, diff: np.ndarray | None = None):
    blob = proto.BlobProto()
    blob.shape.dim.extend(int(d) for d in arr.shape)
    blob.data.extend(np.asarray(arr, np.float64).reshape(-1).tolist())
    if diff is not None:
        blob.diff.extend(np.asarray(diff, np.float64).reshape(-1).tolist())
    return blob


def arraylist_to_blobprotovector_str(arraylist) -> bytes:
    vec = proto.BlobProtoVector()
    vec.blobs.extend(array_to_blobproto(a) for a in arraylist)
    return vec.SerializeToString()


arraylist_to_blobprotovecor_str = arraylist_to_blobprotovector_str  # the reference's spelling


def blobprotovector_str_to_arraylist(s: bytes) -> list[np.ndarray]:
    vec = proto.BlobProtoVector()
    vec.ParseFromString(s)
    return [blobproto_to_array(b) for b in vec.blobs]


def array_to_datum(arr: np.ndarray, label: int = 0):
    """3-D array -> Datum: uint8 arrays as the byte ``data`` field, others as float_data."""
    if arr.ndim != 3:
        raise ValueError("Incorrect array shape.")
    d = proto.Datum()
    d.channels, d.height, d.width = (int(s) for s in arr.shape)
    if arr.dtype == np.uint8:
        d.data = np.ascontiguousarray(arr).tobytes()
    else:
        d.float_data.extend(np.asarray(arr, np.float32).reshape(-1).tolist())
    d.label = int(label)
    return d


def datum_to_array(datum) -> np.ndarray:
    if len(datum.data):
        return np.frombuffer(datum.data, dtype=np.uint8).reshape(datum.channels, datum.height, datum.width)
    return np.array(datum.float_data, dtype=np.float32).reshape(datum.channels, datum.height, datum.width)


# ---- pre-processing -------------------------------------------------------------------

class Transformer:
    """Format H' x W' x K images for a net input of shape (N, K, H, W)."""

    def __init__(self, inputs: dict):
        self.inputs = {k: tuple(v) for k, v in inputs.items()}
        self.transpose, self.channel_swap, self.raw_scale, self.mean, self.input_scale = {}, {}, {}, {}, {}

    def _check(self, in_):
        if in_ not in self.inputs:
            raise ValueError(f"{in_} is not one of the net inputs: {list(self.inputs)}")

    def preprocess(self, in_, data) -> np.ndarray:
        """convert to float32, resize to the input H x W, transpose (e.g. HWC -> CHW), swap
        channels, scale raw values, subtract the mean, scale the result."""
        self._check(in_)
        x = np.asarray(data, dtype=np.float32)
        in_dims = self.inputs[in_][2:]
        if x.shape[:2] != tuple(in_dims):
            x = resize_image(x, in_dims)
        if in_ in self.transpose:
            x = x.transpose(self.transpose[in_])
        if in_ in self.channel_swap:
            x = x[list(self.channel_swap[in_]), :, :]
        x = np.array(x, dtype=np.float32)
        if in_ in self.raw_scale:
            x *= self.raw_scale[in_]
        if in_ in self.mean:
            x -= self.mean[in_]
        if in_ in self.input_scale:
            x *= self.input_scale[in_]
        return x

    def deprocess(self, in_, data) -> np.ndarray:
        self._check(in_)
        x = np.array(data, dtype=np.float32).squeeze()
        if in_ in self.input_scale:
            x /= self.input_scale[in_]
        if in_ in self.mean:
            x += self.mean[in_]
        if in_ in self.raw_scale:
            x /= self.raw_scale[in_]
        if in_ in self.channel_swap:
            x = x[np.argsort(self.channel_swap[in_]), :, :]
        if in_ in self.transpose:
            x = x.transpose(np.argsort(self.transpose[in_]))
        return x

    def set_transpose(self, in_, order):
        self._check(in_)
        if len(order) != len(self.inputs[in_]) - 1:
            raise ValueError("Transpose order needs to have the same number of dimensions as the input.")
        self.transpose[in_] = tuple(order)

    def set_channel_swap(self, in_, order):
        self._check(in_)
        if len(order) != self.inputs[in_][1]:
            raise ValueError("Channel swap needs to have the same number of dimensions as the input channels.")
        self.channel_swap[in_] = tuple(order)

    def set_raw_scale(self, in_, scale):
        self._check(in_)
        self.raw_scale[in_] = scale

    def set_mean(self, in_, mean):
        """Per-channel (K,) or elementwise (K, H, W) / (H, W) mean."""
        self._check(in_)
        mean = np.asarray(mean, dtype=np.float32)
        if mean.ndim == 1:
            if mean.shape[0] != self.inputs[in_][1]:
                raise ValueError("Mean channels incompatible with input.")
            mean = mean[:, None, None]
        else:
            ms = mean.shape if mean.ndim == 3 else (1,) + mean.shape
            if len(ms) != 3:
                raise ValueError("Mean shape invalid")
            if tuple(ms) != tuple(self.inputs[in_][1:]):
                raise ValueError("Mean shape incompatible with input shape.")
        self.mean[in_] = mean

    def set_input_scale(self, in_, scale):
        self._check(in_)
        self.input_scale[in_] = scale


# ---- image IO -----------------------------------------------------------------------

def load_image(filename: str, color: bool = True) -> np.ndarray:
    """H x W x 3 (RGB) or H x W x 1 float32 image in [0, 1]."""
    from PIL import Image
    im = Image.open(filename)
    if color:
        arr = np.asarray(im.convert("RGB"), dtype=np.float32) / 255.0
    else:
        arr = np.asarray(im.convert("L"), dtype=np.float32)[:, :, None] / 255.0
    return arr


def resize_image(im: np.ndarray, new_dims, interp_order: int = 1) -> np.ndarray:
    """Resize an H x W x K array to new_dims = (height, width), preserving its value range."""
    im = np.asarray(im, dtype=np.float32)
    h, w = int(new_dims[0]), int(new_dims[1])
    if im.shape[-1] in (1, 3):
        from PIL import Image
        resample = Image.BILINEAR if interp_order == 1 else (Image.NEAREST if interp_order == 0 else Image.BICUBIC)
        planes = [np.asarray(Image.fromarray(im[:, :, k], mode="F").resize((w, h), resample), dtype=np.float32)
                  for k in range(im.shape[-1])]
        return np.stack(planes, axis=-1)
    from scipy.ndimage import zoom
    scale = (h / im.shape[0], w / im.shape[1], 1.0)
    return zoom(im, scale, order=interp_order).astype(np.float32)


def oversample(images, crop_dims) -> np.ndarray:
    """The 4 corner + centre crops of each image and their mirrors: (10 N) x h x w x K."""
    images = [np.asarray(im) for im in images]
    im_shape = np.array(images[0].shape)
    crop_dims = np.array(crop_dims)
    center = im_shape[:2] / 2.0
    crops_ix = []
    for i in (0, im_shape[0] - crop_dims[0]):
        for j in (0, im_shape[1] - crop_dims[1]):
            crops_ix.append((i, j, i + crop_dims[0], j + crop_dims[1]))
    c = np.concatenate([center - crop_dims / 2.0, center + crop_dims / 2.0]).astype(int)
    crops_ix.append(tuple(c))
    crops = np.empty((10 * len(images), crop_dims[0], crop_dims[1], im_shape[-1]), dtype=np.float32)
    ix = 0
    for im in images:
        for (a, b, c_, d) in crops_ix:
            crops[ix] = im[a:c_, b:d, :]
            ix += 1
        crops[ix:ix + 5] = crops[ix - 5:ix, :, ::-1, :]  # mirrors
        ix += 5
    return crops
