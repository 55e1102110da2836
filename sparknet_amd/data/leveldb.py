"""LevelDB database codec (no libleveldb in this environment).

Caffe's default Data-layer backend (``DataParameter.backend = LEVELDB``,
caffe/src/caffe/util/db_leveldb.cpp) and SparkNet's CifarDBApp / CreateDB
(src/main/scala/preprocessing/CreateDB.scala:13-50) keep Datum records in a LevelDB
directory.  This module reads and writes that on-disk format directly:

* reader — every table file (``*.ldb`` / ``*.sst``: data blocks with prefix-compressed
  keys and restart arrays, uncompressed or Snappy-compressed, located through the index
  block named by the 48-byte footer) and every write-ahead log (``*.log``: 32 KiB blocks
  of CRC-framed records carrying WriteBatches) is decoded; internal keys
  (``user_key | seq << 8 | type``) are merged so the newest entry of each user key wins
  and deletions hide older values;
* writer — one or more sorted, non-overlapping tables, a MANIFEST holding the
  VersionEdit that installs them, ``CURRENT`` and an empty log: the state LevelDB itself
  leaves after a bulk load and compaction.

Block and record checksums are CRC32C (masked as LevelDB does); the reader verifies them.
"""
from __future__ import annotations

import os
import struct

# ---------------------------------------------------------------------------------------------
# CRC32C (Castagnoli), LevelDB masking
# ---------------------------------------------------------------------------------------------
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def _crc32c_py(data: bytes, crc: int = 0) -> int:
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _native_crc():
    try:
        import ctypes as C
        from ..build_native import RUNTIME_LIB
        path = str(RUNTIME_LIB)
        if not os.path.exists(path):
            return None
        lib = C.CDLL(path)
        fn = lib.sn_crc32c
        fn.restype = C.c_uint32
        fn.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
        return lambda data, crc=0: fn(bytes(data), len(data), crc)
    except (OSError, AttributeError, ImportError):
        return None


crc32c = _native_crc() or _crc32c_py
_MASK_DELTA = 0xA282EAD8


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    r = (m - _MASK_DELTA) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------------------------------
# varints / snappy
# ---------------------------------------------------------------------------------------------
def put_varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def get_varint(b, p: int) -> tuple[int, int]:
    result = shift = 0
    while True:
        c = b[p]
        p += 1
        result |= (c & 0x7F) << shift
        if c < 0x80:
            return result, p
        shift += 7


def snappy_decompress(src: bytes) -> bytes:
    n, p = get_varint(src, 0)
    out = bytearray()
    end = len(src)
    while p < end:
        tag = src[p]
        p += 1
        kind = tag & 3
        if kind == 0:                               # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[p:p + nb], "little")
                p += nb
            ln += 1
            out += src[p:p + ln]
            p += ln
            continue
        if kind == 1:
            ln = 4 + ((tag >> 2) & 7)
            off = ((tag >> 5) << 8) | src[p]
            p += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[p:p + 2], "little")
            p += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[p:p + 4], "little")
            p += 4
        if off == 0 or off > len(out):
            raise ValueError("corrupt snappy stream")
        start = len(out) - off
        if off >= ln:
            out += out[start:start + ln]
        else:                                       # overlapping copy
            for i in range(ln):
                out.append(out[start + i])
    if len(out) != n:
        raise ValueError("corrupt snappy stream (length mismatch)")
    return bytes(out)


# ---------------------------------------------------------------------------------------------
# table format
# ---------------------------------------------------------------------------------------------
TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER = 48
TYPE_DELETION, TYPE_VALUE = 0, 1


def _read_block(buf, off: int, size: int, verify: bool = True) -> bytes:
    data = bytes(buf[off:off + size])
    ctype = buf[off + size]
    if verify:
        want = unmask_crc(struct.unpack_from("<I", buf, off + size + 1)[0])
        if crc32c(data + bytes([ctype])) != want:
            raise ValueError("LevelDB block checksum mismatch")
    if ctype == 1:
        return snappy_decompress(data)
    if ctype != 0:
        raise ValueError(f"unsupported LevelDB block compression {ctype}")
    return data


def _block_entries(block: bytes):
    nrestarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * nrestarts
    p = 0
    key = b""
    while p < limit:
        shared, p = get_varint(block, p)
        nonshared, p = get_varint(block, p)
        vlen, p = get_varint(block, p)
        key = key[:shared] + block[p:p + nonshared]
        p += nonshared
        yield key, block[p:p + vlen]
        p += vlen


def read_table(path: str, verify: bool = True):
    """All (internal key, value) entries of one table file, in order."""
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < FOOTER or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != TABLE_MAGIC:
        raise ValueError(f"{path}: not a LevelDB table")
    p = len(buf) - FOOTER
    _, p = get_varint(buf, p)                       # metaindex handle
    _, p = get_varint(buf, p)
    ioff, p = get_varint(buf, p)
    isize, p = get_varint(buf, p)
    for _, handle in _block_entries(_read_block(buf, ioff, isize, verify)):
        boff, q = get_varint(handle, 0)
        bsize, _ = get_varint(handle, q)
        yield from _block_entries(_read_block(buf, boff, bsize, verify))


class _BlockBuilder:
    def __init__(self, restart_interval: int = 16):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""
        self.interval = restart_interval

    def add(self, key: bytes, value: bytes) -> None:
        shared = 0
        if self.counter < self.interval:
            m = min(len(self.last), len(key))
            while shared < m and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += put_varint(shared) + put_varint(len(key) - shared) + put_varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def empty(self) -> bool:
        return not self.buf


class _TableWriter:
    def __init__(self, path: str, block_size: int = 65536):
        self.f = open(path, "wb")
        self.off = 0
        self.block = _BlockBuilder()
        self.index = _BlockBuilder(restart_interval=1)
        self.block_size = block_size
        self.last_key = None

    def _write_block(self, contents: bytes) -> bytes:
        trailer = bytes([0]) + struct.pack("<I", mask_crc(crc32c(contents + b"\0")))
        self.f.write(contents + trailer)
        handle = put_varint(self.off) + put_varint(len(contents))
        self.off += len(contents) + 5
        return handle

    def add(self, ikey: bytes, value: bytes) -> None:
        self.block.add(ikey, value)
        self.last_key = ikey
        if self.block.size() >= self.block_size:
            self._flush()

    def _flush(self) -> None:
        if self.block.empty():
            return
        self.index.add(self.last_key, self._write_block(self.block.finish()))
        self.block = _BlockBuilder()

    def finish(self) -> int:
        self._flush()
        meta = self._write_block(_BlockBuilder().finish())
        index = self._write_block(self.index.finish())
        footer = (meta + index).ljust(40, b"\0") + struct.pack("<Q", TABLE_MAGIC)
        self.f.write(footer)
        self.off += len(footer)
        self.f.close()
        return self.off


# ---------------------------------------------------------------------------------------------
# log format (write-ahead logs and MANIFEST)
# ---------------------------------------------------------------------------------------------
LOG_BLOCK = 32768
FULL, FIRST, MIDDLE, LAST = 1, 2, 3, 4


def read_log_records(path: str, verify: bool = True):
    with open(path, "rb") as f:
        buf = f.read()
    p, n = 0, len(buf)
    frag = bytearray()
    while p + 7 <= n:
        left = LOG_BLOCK - p % LOG_BLOCK
        if left < 7:
            p += left
            continue
        crc, ln, typ = struct.unpack_from("<IHB", buf, p)
        if typ == 0 and ln == 0:                    # zero padding / preallocated tail
            p += left
            continue
        data = buf[p + 7:p + 7 + ln]
        if verify and crc32c(bytes([typ]) + data) != unmask_crc(crc):
            raise ValueError(f"{path}: log record checksum mismatch")
        p += 7 + ln
        if typ == FULL:
            yield bytes(data)
        elif typ == FIRST:
            frag = bytearray(data)
        elif typ == MIDDLE:
            frag += data
        elif typ == LAST:
            frag += data
            yield bytes(frag)
            frag = bytearray()


class _LogWriter:
    def __init__(self, path: str, append: bool = False):
        self.f = open(path, "ab" if append else "wb")
        self.off = self.f.tell()

    def add(self, record: bytes) -> None:
        p = 0
        first = True
        while True:
            left = LOG_BLOCK - self.off % LOG_BLOCK
            if left < 7:
                self.f.write(b"\0" * left)
                self.off += left
                left = LOG_BLOCK
            avail = left - 7
            chunk = record[p:p + avail]
            p += len(chunk)
            end = p >= len(record)
            typ = FULL if first and end else FIRST if first else LAST if end else MIDDLE
            crc = mask_crc(crc32c(bytes([typ]) + chunk))
            self.f.write(struct.pack("<IHB", crc, len(chunk), typ) + chunk)
            self.off += 7 + len(chunk)
            first = False
            if end:
                return

    def close(self) -> None:
        self.f.close()


def _batch_entries(rec: bytes):
    seq = struct.unpack_from("<Q", rec, 0)[0]
    count = struct.unpack_from("<I", rec, 8)[0]
    p = 12
    for i in range(count):
        tag = rec[p]
        p += 1
        kl, p = get_varint(rec, p)
        key = rec[p:p + kl]
        p += kl
        if tag == TYPE_VALUE:
            vl, p = get_varint(rec, p)
            val = rec[p:p + vl]
            p += vl
        else:
            val = None
        yield key, seq + i, tag, val


# ---------------------------------------------------------------------------------------------
# database
# ---------------------------------------------------------------------------------------------
def _live_tables(path: str):
    """Table numbers named by the MANIFEST that CURRENT points to (files that compaction
    obsoleted but did not delete are ignored); ``None`` when there is no manifest."""
    cur = os.path.join(path, "CURRENT")
    if not os.path.exists(cur):
        return None
    with open(cur) as f:
        manifest = os.path.join(path, f.read().strip())
    live: set[int] = set()
    for rec in read_log_records(manifest):
        p = 0
        while p < len(rec):
            tag, p = get_varint(rec, p)
            if tag == 1:                            # comparator
                ln, p = get_varint(rec, p)
                p += ln
            elif tag in (2, 3, 4, 9):               # log / next file / last seq / prev log
                _, p = get_varint(rec, p)
            elif tag == 5:                          # compact pointer
                _, p = get_varint(rec, p)
                ln, p = get_varint(rec, p)
                p += ln
            elif tag == 6:                          # deleted file
                _, p = get_varint(rec, p)
                num, p = get_varint(rec, p)
                live.discard(num)
            elif tag == 7:                          # new file
                _, p = get_varint(rec, p)
                num, p = get_varint(rec, p)
                _, p = get_varint(rec, p)
                for _ in range(2):
                    ln, p = get_varint(rec, p)
                    p += ln
                live.add(num)
            else:
                raise ValueError(f"unknown MANIFEST tag {tag}")
    return live


def read_leveldb(path: str, verify: bool = True) -> list[tuple[bytes, bytes]]:
    """The live (key, value) pairs of a LevelDB directory, sorted by key."""
    live = _live_tables(path)
    newest: dict[bytes, tuple[int, int, bytes | None]] = {}

    def offer(key, seq, typ, val):
        old = newest.get(key)
        if old is None or seq > old[0]:
            newest[key] = (seq, typ, val)

    for name in sorted(os.listdir(path)):
        stem, ext = os.path.splitext(name)
        full = os.path.join(path, name)
        if ext in (".ldb", ".sst") and stem.isdigit():
            if live is not None and int(stem) not in live:
                continue
            for ikey, val in read_table(full, verify):
                tag = struct.unpack("<Q", ikey[-8:])[0]
                offer(ikey[:-8], tag >> 8, tag & 0xFF, val)
        elif ext == ".log" and stem.isdigit():
            for rec in read_log_records(full, verify):
                for key, seq, typ, val in _batch_entries(rec):
                    offer(key, seq, typ, val)
    return [(k, v[2]) for k, v in sorted(newest.items()) if v[1] == TYPE_VALUE]


def write_leveldb(path: str, items, table_bytes: int = 64 << 20) -> int:
    """Bulk-load ``items`` (key, value) into a new LevelDB directory; returns the count."""
    os.makedirs(path, exist_ok=True)
    data = {}
    for k, v in items:
        data[bytes(k)] = bytes(v)
    keys = sorted(data)
    tables = []                                      # (number, size, smallest, largest)
    num = 3
    seq = 0
    tw, first, size_est = None, None, 0
    for k in keys:
        if tw is None:
            tw = _TableWriter(os.path.join(path, f"{num:06d}.ldb"))
            first, size_est = None, 0
        seq += 1
        ikey = k + struct.pack("<Q", (seq << 8) | TYPE_VALUE)
        tw.add(ikey, data[k])
        first = first or ikey
        size_est += len(ikey) + len(data[k])
        if size_est >= table_bytes:
            tables.append((num, tw.finish(), first, ikey))
            tw, num = None, num + 1
    if tw is not None:
        tables.append((num, tw.finish(), first, ikey))
        num += 1
    edit = bytearray()
    cmp_name = b"leveldb.BytewiseComparator"
    edit += put_varint(1) + put_varint(len(cmp_name)) + cmp_name
    edit += put_varint(2) + put_varint(2)            # log number
    edit += put_varint(3) + put_varint(num)          # next file number
    edit += put_varint(4) + put_varint(seq)          # last sequence
    level = 0 if len(tables) == 1 else 6             # sorted, disjoint tables fit one level
    for tnum, tsize, small, large in tables:
        edit += put_varint(7) + put_varint(level) + put_varint(tnum) + put_varint(tsize)
        edit += put_varint(len(small)) + small + put_varint(len(large)) + large
    lw = _LogWriter(os.path.join(path, "MANIFEST-000001"))
    lw.add(bytes(edit))
    lw.close()
    open(os.path.join(path, "000002.log"), "wb").close()
    with open(os.path.join(path, "CURRENT.tmp"), "w") as f:
        f.write("MANIFEST-000001\n")
    os.replace(os.path.join(path, "CURRENT.tmp"), os.path.join(path, "CURRENT"))
    return len(keys)


def append_batch_log(path: str, puts, first_seq: int = 1) -> None:
    """Append one WriteBatch record (``puts``: (key, value-or-None for deletion)) to a
    write-ahead log, as LevelDB's ``DB::Write`` does before acknowledging a commit."""
    rec = bytearray(struct.pack("<QI", first_seq, len(puts)))
    for k, v in puts:
        if v is None:
            rec += bytes([TYPE_DELETION]) + put_varint(len(k)) + k
        else:
            rec += bytes([TYPE_VALUE]) + put_varint(len(k)) + k + put_varint(len(v)) + v
    lw = _LogWriter(path, append=True)
    lw.add(bytes(rec))
    lw.close()
