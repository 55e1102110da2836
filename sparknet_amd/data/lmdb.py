"""LMDB environment codec (no liblmdb in this environment).

Caffe's ``db_lmdb.cpp`` (caffe/src/caffe/util/db_lmdb.cpp, caffe/include/caffe/util/
db_lmdb.hpp) stores Datum records in the main database of an LMDB environment
(``<dir>/data.mdb``) and reads them back with a forward cursor in key order.  This module
implements that file format directly:

* :class:`LMDBReader` memory-maps ``data.mdb``, picks the newer of the two meta pages and
  walks the main B+tree in key order (branch / leaf / overflow pages; 32- and 64-bit page
  numbers of the 64-bit layout);
* :func:`write_lmdb` bulk-loads sorted key/value pairs into a fresh environment (leaf
  pages packed left to right, values larger than the node limit on overflow pages, branch
  levels built bottom-up, both meta pages pointing at the tree) — the layout liblmdb's
  cursor walks.

Keys compare bytewise (liblmdb's default ``memcmp`` order, shorter key first on ties).
Only what Caffe uses is supported: the unnamed main database, no DUPSORT.
"""
from __future__ import annotations

import mmap
import os
import struct

PAGEHDRSZ = 16
P_BRANCH, P_LEAF, P_OVERFLOW, P_META, P_LEAF2 = 0x01, 0x02, 0x04, 0x08, 0x20
F_BIGDATA, F_SUBDATA, F_DUPDATA = 0x01, 0x02, 0x04
MDB_MAGIC = 0xBEEFC0DE
MDB_DATA_VERSION = 1
P_INVALID = 0xFFFFFFFFFFFFFFFF
MAX_KEY = 511
_DB = struct.Struct("<IHHQQQQQ")          # MDB_db: pad, flags, depth, branch, leaf, overflow, entries, root
_META_HEAD = struct.Struct("<IIQQ")       # magic, version, address, mapsize


def _data_file(path: str) -> str:
    return os.path.join(path, "data.mdb") if os.path.isdir(path) else path


class LMDBReader:
    """Read-only cursor over the main database, in key order."""

    def __init__(self, path: str):
        self.path = _data_file(path)
        self._fh = open(self.path, "rb")
        self.mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        metas = []
        psize = self._meta(0)[0]
        for pg in (0, 1):
            metas.append(self._meta(pg * psize))
        self.psize, self.db, self.txnid = max(metas, key=lambda m: m[2])

    def _meta(self, off: int):
        mm = self.mm
        flags = struct.unpack_from("<H", mm, off + 10)[0]
        if not flags & P_META:
            raise ValueError(f"{self.path}: not an LMDB environment (no meta page at {off})")
        magic, version, _, _ = _META_HEAD.unpack_from(mm, off + PAGEHDRSZ)
        if magic != MDB_MAGIC:
            raise ValueError(f"{self.path}: bad LMDB magic {magic:#x}")
        if version != MDB_DATA_VERSION:
            raise ValueError(f"{self.path}: unsupported LMDB data version {version}")
        p = off + PAGEHDRSZ + _META_HEAD.size
        free = _DB.unpack_from(mm, p)
        main = _DB.unpack_from(mm, p + _DB.size)
        txnid = struct.unpack_from("<Q", mm, p + 2 * _DB.size + 8)[0]
        return free[0], main, txnid               # free.md_pad holds the page size

    @property
    def entries(self) -> int:
        return self.db[6]

    def __len__(self) -> int:
        return self.entries

    def _nodes(self, pgno: int):
        base = pgno * self.psize
        mm = self.mm
        flags, lower = struct.unpack_from("<HH", mm, base + 10)
        if flags & P_LEAF2:
            raise ValueError("LMDB DUPFIXED pages are not supported")
        n = (lower - PAGEHDRSZ) >> 1
        for i in range(n):
            ptr = struct.unpack_from("<H", mm, base + PAGEHDRSZ + 2 * i)[0]
            yield flags, base + ptr

    def _walk(self, pgno: int):
        mm = self.mm
        for flags, node in self._nodes(pgno):
            lo, hi, nflags, ksize = struct.unpack_from("<HHHH", mm, node)
            if flags & P_BRANCH:
                yield from self._walk(lo | (hi << 16) | (nflags << 32))
                continue
            key = mm[node + 8:node + 8 + ksize]
            dsize = lo | (hi << 16)
            if nflags & (F_SUBDATA | F_DUPDATA):
                raise ValueError("LMDB sub-databases / DUPSORT are not supported")
            if nflags & F_BIGDATA:
                opg = struct.unpack_from("<Q", mm, node + 8 + ksize)[0]
                start = opg * self.psize + PAGEHDRSZ
            else:
                start = node + 8 + ksize
            yield key, start, dsize

    def keys(self):
        for k, _, _ in self._iter_raw():
            yield k

    def _iter_raw(self):
        root = self.db[7]
        if root == P_INVALID or self.entries == 0:
            return
        yield from self._walk(root)

    def items(self):
        """(key, value) pairs in key order; values are copied out of the map."""
        for k, start, n in self._iter_raw():
            yield k, self.mm[start:start + n]

    def index(self):
        """[(key, offset, size)] — cheap random access for samplers."""
        return list(self._iter_raw())

    def value_at(self, start: int, n: int) -> bytes:
        return self.mm[start:start + n]

    def close(self) -> None:
        self.mm.close()
        self._fh.close()


# ---------------------------------------------------------------------------------------------
def _node_bytes(key: bytes, lo: int, hi: int, flags: int, payload: bytes) -> bytes:
    b = struct.pack("<HHHH", lo, hi, flags, len(key)) + key + payload
    return b + (b"\0" if len(b) & 1 else b"")


class _PageWriter:
    def __init__(self, fh, psize: int):
        self.fh, self.psize = fh, psize
        self.next_pg = 2
        self.counts = {"branch": 0, "leaf": 0, "overflow": 0}

    def put(self, pgno: int, data: bytes) -> None:
        self.fh.seek(pgno * self.psize)
        self.fh.write(data)

    def overflow(self, value: bytes) -> int:
        n = (PAGEHDRSZ + len(value) + self.psize - 1) // self.psize
        pg = self.next_pg
        self.next_pg += n
        hdr = struct.pack("<QHHI", pg, 0, P_OVERFLOW, n)
        self.put(pg, (hdr + value).ljust(n * self.psize, b"\0"))
        self.counts["overflow"] += n
        return pg

    def page(self, nodes: list[bytes], flags: int) -> int:
        pg = self.next_pg
        self.next_pg += 1
        buf = bytearray(self.psize)
        upper = self.psize
        for i, nd in enumerate(nodes):
            upper -= len(nd)
            buf[upper:upper + len(nd)] = nd
            struct.pack_into("<H", buf, PAGEHDRSZ + 2 * i, upper)
        struct.pack_into("<QHHHH", buf, 0, pg, 0, flags, PAGEHDRSZ + 2 * len(nodes), upper)
        self.put(pg, bytes(buf))
        self.counts["branch" if flags & P_BRANCH else "leaf"] += 1
        return pg


def write_lmdb(path: str, items, psize: int = 4096) -> int:
    """Create ``path/data.mdb`` holding ``items`` (an iterable of (key, value) bytes,
    in any order; duplicate keys keep the last value).  Returns the entry count."""
    os.makedirs(path, exist_ok=True)
    data = {}
    for k, v in items:
        k = bytes(k)
        if not 0 < len(k) <= MAX_KEY:
            raise ValueError(f"LMDB keys must be 1..{MAX_KEY} bytes")
        data[k] = bytes(v)
    keys = sorted(data)
    nodemax = (((psize - PAGEHDRSZ) // 2) & ~1) - 2
    fname = _data_file(path)
    with open(fname + ".tmp", "wb") as fh:
        w = _PageWriter(fh, psize)
        level: list[tuple[bytes, int]] = []       # (first key, pgno) of each page
        cur: list[bytes] = []
        used = PAGEHDRSZ
        first = None
        for k in keys:
            v = data[k]
            if 8 + len(k) + len(v) > nodemax:
                nd = _node_bytes(k, len(v) & 0xFFFF, len(v) >> 16, F_BIGDATA, struct.pack("<Q", w.overflow(v)))
            else:
                nd = _node_bytes(k, len(v) & 0xFFFF, len(v) >> 16, 0, v)
            if cur and used + 2 + len(nd) > psize:
                level.append((first, w.page(cur, P_LEAF)))
                cur, used = [], PAGEHDRSZ
            if not cur:
                first = k
            cur.append(nd)
            used += 2 + len(nd)
        if cur:
            level.append((first, w.page(cur, P_LEAF)))
        depth = 1 if level else 0
        while len(level) > 1:
            nxt, cur, used = [], [], PAGEHDRSZ
            for k, pg in level:
                key = b"" if not cur else k       # leftmost key of a branch page is implicit
                nd = _node_bytes(key, pg & 0xFFFF, (pg >> 16) & 0xFFFF, (pg >> 32) & 0xFFFF, b"")
                if cur and used + 2 + len(nd) > psize:
                    nxt.append((first, w.page(cur, P_BRANCH)))
                    cur, used = [], PAGEHDRSZ
                    nd = _node_bytes(b"", pg & 0xFFFF, (pg >> 16) & 0xFFFF, (pg >> 32) & 0xFFFF, b"")
                if not cur:
                    first = k
                cur.append(nd)
                used += 2 + len(nd)
            nxt.append((first, w.page(cur, P_BRANCH)))
            level = nxt
            depth += 1
        root = level[0][1] if level else P_INVALID
        last_pg = w.next_pg - 1
        mapsize = max(w.next_pg * psize, 1 << 20)
        free_db = _DB.pack(psize, 0, 0, 0, 0, 0, 0, P_INVALID)
        main_db = _DB.pack(0, 0, depth, w.counts["branch"], w.counts["leaf"], w.counts["overflow"], len(keys), root)
        for pg in (0, 1):
            meta = (struct.pack("<QHHHH", pg, 0, P_META, 0, 0) + _META_HEAD.pack(MDB_MAGIC, MDB_DATA_VERSION, 0, mapsize)
                    + free_db + main_db + struct.pack("<QQ", last_pg, 1))
            w.put(pg, meta.ljust(psize, b"\0"))
        fh.truncate(w.next_pg * psize)
    os.replace(fname + ".tmp", fname)
    return len(keys)
