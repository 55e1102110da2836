"""Python handle on the native minibatch pipeline (``csrc/runtime/loader.cpp``,
``libsn_runtime.so``).

The C++ side owns the record sources (memory-mapped CIFAR-style fixed-size record files,
caller-provided host arrays, or a synthetic generator), the sampler (per-epoch shuffle,
sequential cursor, or SparkNet's random window of ``tau`` consecutive minibatches per
round — src/main/scala/libs/MinibatchSampler.scala:18-58), the worker threads and a
ring of pinned (hipHostMalloc) slots; :meth:`NativeLoader.next_to_device` issues the
H2D copy on the caller's stream and returns immediately.  Python only hands over
pointers — nothing on the per-sample path runs in the interpreter.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ..ops import _lib

SOURCE_FILES, SOURCE_MEMORY, SOURCE_SYNTHETIC = 0, 1, 2
SAMPLER_SHUFFLE, SAMPLER_SEQUENTIAL, SAMPLER_WINDOW = 0, 1, 2


class SnLoaderConfig(C.Structure):
    _fields_ = [("source", C.c_int), ("paths", C.c_char_p),
                ("header_bytes", C.c_longlong), ("record_bytes", C.c_longlong),
                ("label_offset", C.c_longlong), ("label_bytes", C.c_longlong), ("image_offset", C.c_longlong),
                ("mem_images", C.c_void_p), ("mem_labels", C.c_void_p), ("mem_count", C.c_longlong),
                ("image_bytes", C.c_longlong), ("batch", C.c_int), ("sampler", C.c_int), ("tau", C.c_int),
                ("rank", C.c_int), ("world", C.c_int), ("seed", C.c_ulonglong),
                ("slots", C.c_int), ("threads", C.c_int), ("pinned", C.c_int), ("classes", C.c_int),
                ("synthetic_count", C.c_longlong), ("first_batch", C.c_longlong)]


class SnLoaderStats(C.Structure):
    _fields_ = [("batches_filled", C.c_longlong), ("batches_consumed", C.c_longlong),
                ("fill_seconds", C.c_double), ("consumer_wait_seconds", C.c_double),
                ("shard_samples", C.c_longlong), ("batches_per_epoch", C.c_longlong)]


_ERRORS = {1: "bad batch/slots/threads", 2: "bad rank/world", 3: "window sampler needs tau >= 1",
           4: "bad record layout or memory source", 5: "unknown source", 6: "shard smaller than one batch",
           7: "tau exceeds the batches in the shard", 8: "host allocation failed", 9: "event creation failed",
           20: "cannot open a record file", 21: "mmap failed"}


def _rt():
    lib = _lib.runtime()
    if not getattr(lib, "_sn_loader_typed", False):
        lib.sn_loader_create.argtypes = [C.POINTER(SnLoaderConfig), C.POINTER(C.c_int)]
        lib.sn_loader_create.restype = C.c_void_p
        lib.sn_loader_acquire.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        lib.sn_loader_acquire.restype = C.c_longlong
        lib.sn_loader_copy_async.argtypes = [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.sn_loader_copy_async.restype = C.c_int
        lib.sn_loader_release.argtypes = [C.c_void_p, C.c_longlong]
        lib.sn_loader_release.restype = C.c_int
        lib.sn_loader_stats.argtypes = [C.c_void_p, C.POINTER(SnLoaderStats)]
        lib.sn_loader_stats.restype = None
        lib.sn_loader_batch_indices.argtypes = [C.c_void_p, C.c_longlong, C.POINTER(C.c_longlong)]
        lib.sn_loader_batch_indices.restype = None
        lib.sn_loader_destroy.argtypes = [C.c_void_p]
        lib.sn_loader_destroy.restype = None
        lib._sn_loader_typed = True
    return lib


class NativeLoader:
    """Minibatches of uint8 planar images [B, C, H, W] + int32 labels [B]."""

    def __init__(self, shape, batch: int, *, source: int = SOURCE_SYNTHETIC, paths=None,
                 record=None, images: np.ndarray | None = None, labels: np.ndarray | None = None,
                 sampler: int = SAMPLER_SHUFFLE, tau: int = 1, rank: int = 0, world: int = 1, seed: int = 0,
                 slots: int = 4, threads: int = 2, pinned: bool | None = None, classes: int = 1000,
                 synthetic_count: int | None = None, first_batch: int = 0):
        c, h, w = (int(v) for v in shape)
        self.shape = (int(batch), c, h, w)
        self.batch = int(batch)
        self.image_bytes = c * h * w
        if pinned is None:
            import torch
            pinned = torch.cuda.is_available()
        self.pinned = bool(pinned)
        cfg = SnLoaderConfig()
        cfg.source = source
        self._keep = []
        if source == SOURCE_FILES:
            if isinstance(paths, (str, bytes)):
                paths = [paths]
            self._paths = "\n".join(str(p) for p in paths).encode()
            cfg.paths = self._paths
            header, rec, loff, lbytes, ioff = record
            cfg.header_bytes, cfg.record_bytes = header, rec
            cfg.label_offset, cfg.label_bytes, cfg.image_offset = loff, lbytes, ioff
        elif source == SOURCE_MEMORY:
            imgs = np.ascontiguousarray(images, dtype=np.uint8).reshape(len(images), -1)
            labs = np.ascontiguousarray(labels, dtype=np.int32).reshape(-1)
            if imgs.shape[1] != self.image_bytes or len(labs) != len(imgs):
                raise ValueError("images/labels do not match the sample shape")
            self._keep = [imgs, labs]  # the C++ side reads them in place
            cfg.mem_images = imgs.ctypes.data
            cfg.mem_labels = labs.ctypes.data
            cfg.mem_count = len(imgs)
        cfg.image_bytes = self.image_bytes
        cfg.batch, cfg.sampler, cfg.tau = self.batch, sampler, tau
        cfg.rank, cfg.world, cfg.seed = rank, world, seed
        cfg.slots, cfg.threads, cfg.pinned = slots, threads, int(self.pinned)
        cfg.classes = classes
        cfg.synthetic_count = synthetic_count or 0
        cfg.first_batch = int(first_batch)  # resume: batch sequence continues from here
        err = C.c_int(0)
        self._lib = _rt()
        self._h = self._lib.sn_loader_create(C.byref(cfg), C.byref(err))
        if not self._h:
            raise RuntimeError(f"sn_loader_create failed ({err.value}: {_ERRORS.get(err.value, '?')})")

    # -- constructors for the reference's on-disk formats ------------------------------
    @classmethod
    def cifar10(cls, paths, batch: int, **kw) -> "NativeLoader":
        """CIFAR-10 binary batches (CifarLoader.scala:15-85): [label u8][3072 u8 planar RGB]."""
        return cls((3, 32, 32), batch, source=SOURCE_FILES, paths=paths, record=(0, 3073, 0, 1, 1), **kw)

    @classmethod
    def cifar100(cls, paths, batch: int, **kw) -> "NativeLoader":
        """CIFAR-100 binary: [coarse u8][fine u8][3072 u8]; the fine label is used."""
        return cls((3, 32, 32), batch, source=SOURCE_FILES, paths=paths, record=(0, 3074, 1, 1, 2), **kw)

    # -- consumption ----------------------------------------------------------------------
    def _acquire(self):
        img, lab = C.c_void_p(), C.c_void_p()
        seq = self._lib.sn_loader_acquire(self._h, C.byref(img), C.byref(lab))
        if seq < 0:
            raise RuntimeError("loader stopped")
        return seq, img.value, lab.value

    def next_host(self):
        """(seq, images uint8 [B,C,H,W], labels int32 [B]) as numpy copies."""
        seq, ip, lp = self._acquire()
        imgs = np.ctypeslib.as_array(C.cast(ip, C.POINTER(C.c_uint8)), shape=(self.batch * self.image_bytes,))
        labs = np.ctypeslib.as_array(C.cast(lp, C.POINTER(C.c_int32)), shape=(self.batch,))
        out = imgs.copy().reshape(self.shape), labs.copy()
        self._check(self._lib.sn_loader_release(self._h, seq), "release")
        return (seq,) + out

    def next_to_device(self, dev_images, dev_labels, stream) -> int:
        """H2D copy of the next batch into device tensors on ``stream`` (a torch stream or
        raw hipStream_t); the slot is recycled once that copy has completed."""
        assert dev_images.numel() == self.batch * self.image_bytes and dev_labels.numel() == self.batch
        st = getattr(stream, "cuda_stream", stream)
        seq, _, _ = self._acquire()
        self._check(self._lib.sn_loader_copy_async(self._h, seq, C.c_void_p(dev_images.data_ptr()),
                                                   C.c_void_p(dev_labels.data_ptr()), C.c_void_p(st)), "copy")
        self._check(self._lib.sn_loader_release(self._h, seq), "release")
        return seq

    def batch_indices(self, seq: int) -> list[int]:
        buf = (C.c_longlong * self.batch)()
        self._lib.sn_loader_batch_indices(self._h, seq, buf)
        return list(buf)

    def stats(self) -> dict:
        s = SnLoaderStats()
        self._lib.sn_loader_stats(self._h, C.byref(s))
        return {f: getattr(s, f) for f, _ in SnLoaderStats._fields_}

    @staticmethod
    def _check(rc, what):
        if rc != 0:
            raise RuntimeError(f"sn_loader {what} failed ({rc})")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.sn_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
