"""Datum record databases (CreateDB / Data-layer path; caffe/src/caffe/util/db.cpp).

The reference writes Caffe ``Datum`` records into LevelDB or LMDB
(src/main/scala/preprocessing/CreateDB.scala:13-50 via libccaffe create_db/write_to_db/
commit_db_txn, caffe/src/caffe/util/db_{leveldb,lmdb}.cpp) and the Data layer reads
them back with a forward cursor in key order.  Three backends, all on-disk compatible
formats implemented here (the libraries are not installed):

* ``lmdb``    — :mod:`sparknet_amd.data.lmdb` (``<dir>/data.mdb``);
* ``leveldb`` — :mod:`sparknet_amd.data.leveldb` (tables + logs + MANIFEST); each
  ``commit()`` appends the transaction to the write-ahead log as one WriteBatch, like
  LevelDB's ``Write``; ``close()`` compacts into sorted tables;
* ``sndb``    — an append-only record file (``b"SNDB1\\n"`` then
  ``[uint32 length][serialized Datum]``...), the native loader's mmap format.

Transactions of the LMDB writer are buffered and the environment is bulk-written at
``close()``.
"""
from __future__ import annotations

import os
import struct

import numpy as np

from .. import proto

MAGIC = b"SNDB1\n"


class DatumWriter:
    """db::GetDB(backend)->Open(NEW) + NewTransaction/Put/Commit (db.hpp)."""

    def __init__(self, path: str, commit_every: int = 1000, backend: str = "sndb"):
        self.backend = backend.lower()
        if self.backend not in ("sndb", "lmdb", "leveldb"):
            raise ValueError(f"unknown DB backend {backend!r}")
        self.path = path
        self.commit_every = commit_every
        self.pending = 0
        self.count = 0
        self._txn: list[tuple[bytes, bytes]] = []
        self._all: list[tuple[bytes, bytes]] = []
        self._seq = 1
        if self.backend == "sndb":
            self.f = open(path, "wb")
            self.f.write(MAGIC)
        elif self.backend == "leveldb":
            import shutil
            if os.path.isdir(path):
                shutil.rmtree(path)
            os.makedirs(path)
            self._log = os.path.join(path, "000002.log")

    def put(self, datum, key: str | bytes | None = None) -> None:
        b = datum.SerializeToString()
        if self.backend == "sndb":
            self.f.write(struct.pack("<I", len(b)))
            self.f.write(b)
        else:
            k = key if key is not None else f"{self.count:08d}"
            self._txn.append((k.encode() if isinstance(k, str) else bytes(k), b))
        self.pending += 1
        self.count += 1
        if self.pending >= self.commit_every:
            self.commit()

    def put_image(self, chw_uint8: np.ndarray, label: int, key: str | bytes | None = None) -> None:
        c, h, w = chw_uint8.shape
        self.put(proto.Datum(channels=c, height=h, width=w, data=np.ascontiguousarray(chw_uint8).tobytes(),
                             label=int(label)), key)

    def commit(self) -> None:
        if self.backend == "sndb":
            self.f.flush()
        elif self._txn:
            if self.backend == "leveldb":
                from .leveldb import append_batch_log
                append_batch_log(self._log, self._txn, self._seq)
                self._seq += len(self._txn)
            self._all += self._txn
            self._txn = []
        self.pending = 0

    def close(self) -> None:
        self.commit()
        if self.backend == "sndb":
            self.f.close()
        elif self.backend == "lmdb":
            from .lmdb import write_lmdb
            write_lmdb(self.path, self._all)
        else:
            from .leveldb import write_leveldb
            os.remove(self._log)
            write_leveldb(self.path, self._all)
        self._all = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def detect_backend(path: str) -> str:
    if os.path.isdir(path):
        if os.path.exists(os.path.join(path, "data.mdb")):
            return "lmdb"
        if os.path.exists(os.path.join(path, "CURRENT")) or any(
                n.endswith((".ldb", ".sst", ".log")) for n in os.listdir(path)):
            return "leveldb"
        raise ValueError(f"{path}: no LMDB or LevelDB database in this directory")
    with open(path, "rb") as f:
        head = f.read(len(MAGIC))
    if head == MAGIC:
        return "sndb"
    return "lmdb"                                   # MDB_NOSUBDIR single-file environment


class DatumReader:
    """Forward cursor in key order that wraps around at the end (Caffe DataReader /
    db::Cursor semantics); ``get(i)`` gives random access for samplers."""

    def __init__(self, path: str, backend: str | None = None):
        self.path = path
        self.backend = (backend or detect_backend(path)).lower()
        if self.backend == "sndb":
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
            self._bytes = lambda i: data[self.offsets[i][0]:self.offsets[i][0] + self.offsets[i][1]]
            self.keys = [f"{i:08d}".encode() for i in range(len(self.offsets))]
        elif self.backend == "lmdb":
            from .lmdb import LMDBReader
            self._env = LMDBReader(path)
            self.offsets = [(start, n) for _, start, n in self._env.index()]
            self.keys = [bytes(k) for k in self._env.keys()]
            self._bytes = lambda i: self._env.value_at(*self.offsets[i])
        elif self.backend == "leveldb":
            from .leveldb import read_leveldb
            kv = read_leveldb(path)
            self.keys = [k for k, _ in kv]
            vals = [v for _, v in kv]
            self.offsets = [(i, len(v)) for i, v in enumerate(vals)]
            self._bytes = lambda i: vals[i]
        else:
            raise ValueError(f"unknown DB backend {self.backend!r}")
        self.i = 0
        if not self.offsets:
            raise ValueError(f"{path}: empty database")

    def __len__(self):
        return len(self.offsets)

    def get(self, idx: int):
        d = proto.Datum()
        d.ParseFromString(bytes(self._bytes(idx)))
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


def create_db(path: str, images, labels, commit_every: int = 1000, backend: str = "sndb",
              decimal_keys: bool = False) -> int:
    """CreateDB.makeDBFromPartition (CreateDB.scala:13-32): write (image, label) pairs;
    ``decimal_keys`` reproduces SparkNet's ``counter.toString`` keys (which LMDB and
    LevelDB then order lexicographically), otherwise keys are zero-padded."""
    with DatumWriter(path, commit_every, backend) as w:
        for i, (im, lab) in enumerate(zip(images, labels)):
            w.put_image(np.asarray(im, np.uint8), int(lab), str(i) if decimal_keys else None)
        return w.count


def exists(path: str) -> bool:
    return os.path.exists(path)
