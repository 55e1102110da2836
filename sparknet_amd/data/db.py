"""Datum record database (CreateDB / Data-layer path).

The reference writes Caffe ``Datum`` records into LevelDB / LMDB
(src/main/scala/preprocessing/CreateDB.scala:13-50 via libccaffe create_db/write_to_db/
commit_db_txn, caffe/src/caffe/util/db_{leveldb,lmdb}.cpp).  Neither library exists in
this environment, so the same records go into an append-only SNDB file:
``b"SNDB1\\n"`` then ``[uint32 little-endian length][serialized Datum]`` repeated.  Keys
are implicit (insertion order), which is all the Data layer's sequential cursor needs.
"""
from __future__ import annotations

import os
import struct

import numpy as np

from .. import proto

MAGIC = b"SNDB1\n"


class DatumWriter:
    def __init__(self, path: str, commit_every: int = 1000):
        self.f = open(path, "wb")
        self.f.write(MAGIC)
        self.commit_every = commit_every
        self.pending = 0
        self.count = 0

    def put(self, datum) -> None:
        b = datum.SerializeToString()
        self.f.write(struct.pack("<I", len(b)))
        self.f.write(b)
        self.pending += 1
        self.count += 1
        if self.pending >= self.commit_every:
            self.commit()

    def put_image(self, chw_uint8: np.ndarray, label: int) -> None:
        c, h, w = chw_uint8.shape
        self.put(proto.Datum(channels=c, height=h, width=w, data=np.ascontiguousarray(chw_uint8).tobytes(),
                             label=int(label)))

    def commit(self) -> None:
        self.f.flush()
        self.pending = 0

    def close(self) -> None:
        self.commit()
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class DatumReader:
    """Sequential cursor that wraps around at the end (Caffe DataReader semantics)."""

    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            data = f.read()
        if not data.startswith(MAGIC):
            raise ValueError(f"{path}: not an SNDB file")
        self.offsets = []
        pos = len(MAGIC)
        while pos + 4 <= len(data):
            (n,) = struct.unpack_from("<I", data, pos)
            self.offsets.append((pos + 4, n))
            pos += 4 + n
        self.data = data
        self.i = 0
        if not self.offsets:
            raise ValueError(f"{path}: empty database")

    def __len__(self):
        return len(self.offsets)

    def get(self, idx: int):
        off, n = self.offsets[idx]
        d = proto.Datum()
        d.ParseFromString(self.data[off:off + n])
        return d

    def peek(self):
        return self.get(self.i)

    def next(self):
        d = self.get(self.i)
        self.i = (self.i + 1) % len(self.offsets)
        return d


def datum_to_array(d) -> np.ndarray:
    if d.data:
        return np.frombuffer(d.data, dtype=np.uint8).reshape(d.channels, d.height, d.width)
    return np.asarray(d.float_data, np.float32).reshape(d.channels, d.height, d.width)


def create_db(path: str, images, labels, commit_every: int = 1000) -> int:
    """CreateDB.makeDBFromPartition: write (image, label) pairs."""
    with DatumWriter(path, commit_every) as w:
        for im, lab in zip(images, labels):
            w.put_image(np.asarray(im, np.uint8), int(lab))
        return w.count


def exists(path: str) -> bool:
    return os.path.exists(path)
