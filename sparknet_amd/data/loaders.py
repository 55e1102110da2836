"""Dataset loaders.

* :class:`CifarLoader` — CIFAR-10 binary batches (src/main/scala/loaders/CifarLoader.scala:
  15-85): 5 ``data_batch_*.bin`` + ``test_batch.bin``, records of 1 label byte + 3072 bytes
  (planar RGB 32x32), train set shuffled with a seeded permutation.  numpy memory maps,
  no per-record objects.
* :class:`ImageNetLoader` — ImageNet from local tar shards or JPEG directories plus a
  label file (src/main/scala/loaders/ImageNetLoader.scala:25-96 read the tars from S3;
  there is no network here, so the same tar format is read from disk), decoded and
  resized with PIL (ScaleAndConvert.scala:16-27) into planar uint8 batches.
* :func:`compute_mean` — dataset mean image (ComputeMean.scala:8-85), optionally
  all-reduced across ranks, written as a BlobProto ``.binaryproto``.
"""
from __future__ import annotations

import io
import os
import tarfile

import numpy as np
import torch

CIFAR_RECORD = 1 + 3 * 32 * 32


class CifarLoader:
    def __init__(self, path: str, seed: int = 0, shuffle: bool = True):
        train_files = [os.path.join(path, f"data_batch_{i}.bin") for i in range(1, 6)]
        test_file = os.path.join(path, "test_batch.bin")
        self.train_images, self.train_labels = self._read([f for f in train_files if os.path.exists(f)])
        self.test_images, self.test_labels = self._read([test_file] if os.path.exists(test_file) else [])
        if shuffle and len(self.train_labels):
            perm = np.random.default_rng(seed).permutation(len(self.train_labels))
            self.train_images = self.train_images[perm]
            self.train_labels = self.train_labels[perm]

    @staticmethod
    def _read(files):
        if not files:
            return np.zeros((0, 3, 32, 32), np.uint8), np.zeros((0,), np.int32)
        recs = np.concatenate([np.fromfile(f, dtype=np.uint8).reshape(-1, CIFAR_RECORD) for f in files])
        labels = recs[:, 0].astype(np.int32)
        images = recs[:, 1:].reshape(-1, 3, 32, 32)
        return np.ascontiguousarray(images), labels

    def mean_image(self) -> np.ndarray:
        return self.train_images.reshape(len(self.train_images), -1).mean(0).reshape(3, 32, 32)

    def tensors(self, train: bool = True):
        im, lab = (self.train_images, self.train_labels) if train else (self.test_images, self.test_labels)
        return torch.from_numpy(im), torch.from_numpy(lab)


def write_synthetic_cifar(path: str, n_train: int = 500, n_test: int = 100, seed: int = 0) -> None:
    """Write CIFAR-format binary files with random content (tests / offline demos)."""
    rng = np.random.default_rng(seed)
    os.makedirs(path, exist_ok=True)

    def rec(n):
        r = np.empty((n, CIFAR_RECORD), np.uint8)
        r[:, 0] = rng.integers(0, 10, n)
        r[:, 1:] = rng.integers(0, 256, (n, CIFAR_RECORD - 1))
        return r
    per = max(1, n_train // 5)
    for i in range(1, 6):
        rec(per).tofile(os.path.join(path, f"data_batch_{i}.bin"))
    rec(n_test).tofile(os.path.join(path, "test_batch.bin"))


def decode_resize(data: bytes, size: tuple[int, int]) -> np.ndarray | None:
    """JPEG -> planar uint8 (3, H, W), resized (ScaleAndConvert.convertImage); None if
    undecodable (the reference skips such images)."""
    from PIL import Image
    try:
        im = Image.open(io.BytesIO(data)).convert("RGB").resize((size[1], size[0]), Image.BILINEAR)
    except Exception:
        return None
    return np.ascontiguousarray(np.asarray(im, dtype=np.uint8).transpose(2, 0, 1))


class ImageNetLoader:
    """Iterate (planar uint8 image, label) from tar shards or a directory tree, local or
    on S3 (ImageNetLoader.scala:21-96: list the shards under a prefix, read the labels
    file ``path label`` keyed by file name, stream each tar).  ``root`` / ``labels_file``
    may be ``s3://bucket/prefix`` URLs (see :mod:`sparknet_amd.data.s3`)."""

    def __init__(self, root: str, labels_file: str | None = None, size=(256, 256), s3_client=None):
        self.root = root
        self.size = size
        self.labels = {}
        self._s3 = s3_client
        if labels_file:
            for line in self._read_text(labels_file).splitlines():
                parts = line.split()
                if len(parts) >= 2:
                    self.labels[os.path.basename(parts[0])] = int(parts[1])

    def _client(self):
        if self._s3 is None:
            from .s3 import S3Client
            self._s3 = S3Client()
        return self._s3

    def _read_text(self, path: str) -> str:
        if path.startswith("s3://"):
            from .s3 import parse_url
            with self._client().get_object(*parse_url(path)) as r:
                return r.read().decode()
        with open(path) as f:
            return f.read()

    def files(self) -> list[str]:
        """The shard files (tars / images) in a stable order."""
        if self.root.startswith("s3://"):
            from .s3 import parse_url
            bucket, prefix = parse_url(self.root)
            return [f"s3://{bucket}/{k}" for k in sorted(self._client().list_objects(bucket, prefix))
                    if not k.endswith("/")]
        if os.path.isdir(self.root):
            out = []
            for dirpath, _, files in os.walk(self.root):
                out += [os.path.join(dirpath, fn) for fn in files
                        if fn.endswith(".tar") or fn.lower().endswith((".jpg", ".jpeg", ".png"))]
            return sorted(out)
        return [self.root]

    def _open(self, path: str):
        if path.startswith("s3://"):
            from .s3 import parse_url
            return self._client().get_object(*parse_url(path))
        return open(path, "rb")

    def _members(self, files):
        for p in files:
            if p.endswith(".tar"):
                with self._open(p) as fh, tarfile.open(fileobj=fh, mode="r|*") as tf:
                    for m in tf:
                        if m.isfile():
                            yield os.path.basename(m.name), tf.extractfile(m).read()
            else:
                with self._open(p) as fh:
                    yield os.path.basename(p), fh.read()

    def __iter__(self):
        yield from self._decoded(self.files())

    def _decoded(self, files):
        for name, data in self._members(files):
            img = decode_resize(data, self.size)
            if img is None:
                continue
            yield img, self.labels.get(name, 0)

    def minibatches(self, batch: int, shard: tuple[int, int] = (0, 1)):
        """Full minibatches only (the remainder is dropped, ScaleAndConvert.scala:45-70).
        With at least ``world`` shard files each rank reads only its files (the
        reference's one-partition-per-file RDD); otherwise images are dealt round-robin."""
        rank, world = shard
        files = self.files()
        by_file = len(files) >= world > 1
        stream = self._decoded(files[rank::world] if by_file else files)
        imgs, labs = [], []
        for i, (img, lab) in enumerate(stream):
            if not by_file and i % world != rank:
                continue
            imgs.append(img)
            labs.append(lab)
            if len(imgs) == batch:
                yield torch.from_numpy(np.stack(imgs)), torch.tensor(labs, dtype=torch.int32)
                imgs, labs = [], []


def compute_mean(batches, comm=None) -> np.ndarray:
    """Mean image over uint8 batches (int64 partial sums, then an all-reduce across ranks:
    ComputeMean.scala's per-partition sums + driver reduce)."""
    total = None
    count = 0
    for x in batches:
        x = torch.as_tensor(x)
        s = x.to(torch.int64).sum(0)
        total = s if total is None else total + s
        count += x.shape[0]
    t = torch.cat([total.reshape(-1).double(), torch.tensor([float(count)], dtype=torch.float64)])
    if comm is not None and comm.world_size > 1:
        import torch.distributed as dist
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = t.to(dev)
        dist.all_reduce(t)
        t = t.cpu()
    return (t[:-1] / t[-1]).reshape(total.shape).float().numpy()


def write_mean_binaryproto(mean: np.ndarray, path: str) -> None:
    """ComputeMean.writeMeanToBinaryProto -> save_mean_image (libccaffe/ccaffe.cpp)."""
    from .. import proto
    bp = proto.BlobProto(num=1, channels=mean.shape[0], height=mean.shape[1], width=mean.shape[2])
    bp.data.extend(np.asarray(mean, np.float32).reshape(-1).tolist())
    proto.write_binary(path, bp)


def read_mean_binaryproto(path: str) -> np.ndarray:
    from .. import proto
    from ..core.net import blob_proto_to_tensor
    t = blob_proto_to_tensor(proto.read_binary(path, proto.BlobProto))
    return t.reshape(t.shape[-3:]).numpy() if t.dim() == 4 else t.numpy()
