"""Self-contained HDF5 codec (no libhdf5 / h5py in this environment).

Replaces the reference's libhdf5 dependency (caffe/src/caffe/util/hdf5.cpp:1-187,
SURVEY §2 C18) for the three places Caffe uses HDF5:

* ``snapshot_format: HDF5`` model and solver snapshots (net.cpp:861-980,
  sgd_solver.cpp:277-343): groups ``data/<layer>/<i>`` (+ ``diff``), datasets ``iter``,
  ``learned_net``, ``current_step`` and ``history/<i>``;
* the ``HDF5Data`` layer (hdf5_data_layer.cpp:26-160): one dataset per top, rows along
  axis 0;
* the ``HDF5Output`` layer (hdf5_output_layer.cpp:15-60): ``data`` and ``label``.

Reader: superblock v0-v3, object headers v1 and v2, old-style (symbol table / B-tree v1 /
local heap) and compact (link message) groups, contiguous / compact / chunked (B-tree v1
index) layouts, the deflate, shuffle and fletcher32 filters, integer / float / fixed
string types.  That covers files written by libhdf5 with its default (earliest) format,
which is what Caffe and h5py produce — including the reference's fixtures
(caffe/src/caffe/test/test_data/sample_data.h5, sample_data_2_gzip.h5, solver_data.h5).

Writer: superblock v0, v1 object headers, symbol-table groups and contiguous datasets —
the same structures libhdf5 writes by default.
"""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF

# object header message types
MSG_NIL, MSG_DATASPACE, MSG_LINKINFO, MSG_DATATYPE, MSG_FILL_OLD, MSG_FILL = 0x0, 0x1, 0x2, 0x3, 0x4, 0x5
MSG_LINK, MSG_LAYOUT, MSG_FILTERS, MSG_CONT, MSG_SYMTAB = 0x6, 0x8, 0xB, 0x10, 0x11


class HDF5Error(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# reader
# ---------------------------------------------------------------------------------------------
class _Buf:
    def __init__(self, data: bytes, osz: int = 8, lsz: int = 8):
        self.b = data
        self.osz, self.lsz = osz, lsz

    def u(self, pos: int, n: int) -> int:
        return int.from_bytes(self.b[pos:pos + n], "little")

    def off(self, pos: int) -> int:
        v = self.u(pos, self.osz)
        return UNDEF if v == (1 << (8 * self.osz)) - 1 else v

    def off_bytes(self, msg: bytes, p: int) -> int:
        """Offset-sized field inside a message body."""
        v = int.from_bytes(msg[p:p + self.osz], "little")
        return UNDEF if v == (1 << (8 * self.osz)) - 1 else v

    def ln(self, pos: int) -> int:
        return self.u(pos, self.lsz)

    def cstr(self, pos: int) -> str:
        end = self.b.index(b"\0", pos)
        return self.b[pos:end].decode("utf-8")


def _dtype(msg: bytes):
    """Datatype message -> (numpy dtype, class)."""
    cls = msg[0] & 0x0F
    bits0 = msg[1]
    size = int.from_bytes(msg[4:8], "little")
    order = ">" if bits0 & 1 else "<"
    if cls == 0:    # fixed point
        signed = bool(bits0 & 0x08)
        return np.dtype(f"{order}{'i' if signed else 'u'}{size}"), cls
    if cls == 1:    # floating point
        if size not in (2, 4, 8):
            raise HDF5Error(f"unsupported float size {size}")
        return np.dtype(f"{order}f{size}"), cls
    if cls == 3:    # fixed-length string
        return np.dtype(f"S{size}"), cls
    raise HDF5Error(f"unsupported HDF5 datatype class {cls}")


def _dataspace(msg: bytes, lsz: int):
    ver, nd, flags = msg[0], msg[1], msg[2]
    if ver == 1:
        p = 8
    elif ver == 2:
        if msg[3] == 2:          # null dataspace
            return None
        p = 4
    else:
        raise HDF5Error(f"unsupported dataspace version {ver}")
    return tuple(int.from_bytes(msg[p + i * lsz:p + (i + 1) * lsz], "little") for i in range(nd))


def _filters(msg: bytes):
    ver, n = msg[0], msg[1]
    out = []
    p = 8 if ver == 1 else 2
    for _ in range(n):
        fid = int.from_bytes(msg[p:p + 2], "little")
        p += 2
        name_len = 0
        if ver == 1 or fid >= 256:
            name_len = int.from_bytes(msg[p:p + 2], "little")
            p += 2
        flags = int.from_bytes(msg[p:p + 2], "little")
        nvals = int.from_bytes(msg[p + 2:p + 4], "little")
        p += 4
        if ver == 1:
            name_len = (name_len + 7) & ~7
        p += name_len
        vals = [int.from_bytes(msg[p + 4 * i:p + 4 * i + 4], "little") for i in range(nvals)]
        p += 4 * nvals
        if ver == 1 and nvals % 2:
            p += 4
        out.append((fid, flags, vals))
    return out


def _unfilter(raw: bytes, filters, mask: int, elem: int) -> bytes:
    for i in range(len(filters) - 1, -1, -1):
        if mask & (1 << i):
            continue
        fid = filters[i][0]
        if fid == 1:
            raw = zlib.decompress(raw)
        elif fid == 2:           # shuffle: bytes grouped by significance
            a = np.frombuffer(raw, np.uint8)
            n = len(a) // elem
            body = a[:n * elem].reshape(elem, n).T.reshape(-1)
            raw = body.tobytes() + a[n * elem:].tobytes()
        elif fid == 3:           # fletcher32: trailing checksum
            raw = raw[:-4]
        else:
            raise HDF5Error(f"unsupported HDF5 filter id {fid}")
    return raw


class Dataset:
    def __init__(self, f: "File", name: str, msgs: dict):
        self._f, self.name = f, name
        if MSG_DATATYPE not in msgs or MSG_LAYOUT not in msgs:
            raise HDF5Error(f"{name}: not a dataset")
        self.dtype, self.type_class = _dtype(msgs[MSG_DATATYPE][0])
        ds = msgs.get(MSG_DATASPACE)
        self.shape = _dataspace(ds[0], f.buf.lsz) if ds else ()
        self._layout = msgs[MSG_LAYOUT][0]
        self._filters = _filters(msgs[MSG_FILTERS][0]) if MSG_FILTERS in msgs else []

    @property
    def ndim(self) -> int:
        return len(self.shape)

    def read(self) -> np.ndarray:
        buf, lay = self._f.buf, self._layout
        n = int(np.prod(self.shape)) if self.shape else 1
        nbytes = n * self.dtype.itemsize
        ver = lay[0]
        if ver != 3:
            if ver in (1, 2):
                return self._read_v12(lay, n)
            raise HDF5Error(f"{self.name}: unsupported layout version {ver}")
        cls = lay[1]
        if cls == 0:                                     # compact
            size = int.from_bytes(lay[2:4], "little")
            raw = lay[4:4 + size]
        elif cls == 1:                                   # contiguous
            addr = buf.off_bytes(lay, 2)
            if addr == UNDEF:
                return np.zeros(self.shape, self.dtype)
            raw = buf.b[addr:addr + nbytes]
        elif cls == 2:                                   # chunked, B-tree v1 index
            rank = lay[2]
            addr = buf.off_bytes(lay, 3)
            p = 3 + buf.osz
            cdims = [int.from_bytes(lay[p + 4 * i:p + 4 * i + 4], "little") for i in range(rank)]
            return self._read_chunked(addr, cdims[:-1])
        else:
            raise HDF5Error(f"{self.name}: unsupported layout class {cls}")
        return np.frombuffer(bytes(raw[:nbytes]), self.dtype).reshape(self.shape).copy()

    def _read_v12(self, lay, n):
        buf = self._f.buf
        nd, cls = lay[1], lay[2]
        p = 8
        if cls != 0:
            addr = buf.off_bytes(lay, p)
            p += buf.osz
        dims = [int.from_bytes(lay[p + 4 * i:p + 4 * i + 4], "little") for i in range(nd)]
        p += 4 * nd
        if cls == 1:
            raw = buf.b[addr:addr + n * self.dtype.itemsize]
        elif cls == 0:
            size = int.from_bytes(lay[p:p + 4], "little")
            raw = lay[p + 4:p + 4 + size]
        else:
            return self._read_chunked(addr, dims[:-1] if len(dims) > len(self.shape) else dims)
        return np.frombuffer(bytes(raw), self.dtype).reshape(self.shape).copy()

    def _read_chunked(self, addr: int, cdims):
        buf = self._f.buf
        out = np.zeros(self.shape, self.dtype)
        rank = len(self.shape)
        elem = self.dtype.itemsize
        for size, mask, offs, caddr in self._f._chunk_leaves(addr, rank + 1):
            raw = _unfilter(bytes(buf.b[caddr:caddr + size]), self._filters, mask, elem)
            chunk = np.frombuffer(raw[:int(np.prod(cdims)) * elem], self.dtype).reshape(cdims)
            sl_out = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, self.shape))
            sl_in = tuple(slice(0, s.stop - s.start) for s in sl_out)
            out[sl_out] = chunk[sl_in]
        return out

    def __array__(self, dtype=None, copy=None):
        a = self.read()
        return a.astype(dtype) if dtype is not None else a


class Group:
    def __init__(self, f: "File", name: str, links: dict):
        self._f, self.name, self._links = f, name, links

    def keys(self):
        """Link names in name order (H5_INDEX_NAME iteration, hdf5.cpp:171-186)."""
        return sorted(self._links)

    def __len__(self):
        return len(self._links)

    def __contains__(self, key):
        return self._resolve(key) is not None

    def __iter__(self):
        return iter(self.keys())

    def _resolve(self, path: str):
        parts = [p for p in path.split("/") if p]
        node = self
        for p in parts:
            if not isinstance(node, Group) or p not in node._links:
                return None
            node = node._f._object(node._links[p], f"{node.name.rstrip('/')}/{p}")
        return node

    def __getitem__(self, path: str):
        node = self._resolve(path)
        if node is None:
            raise KeyError(f"{path!r} not found in HDF5 group {self.name!r}")
        return node

    def items(self):
        return [(k, self[k]) for k in self.keys()]


class File(Group):
    """Read-only HDF5 file: ``File(path)["group/dataset"].read()``."""

    def __init__(self, path: str):
        with open(path, "rb") as fh:
            data = fh.read()
        base = None
        for cand in (0, 512, 1024, 2048, 4096):
            if data[cand:cand + 8] == SIGNATURE:
                base = cand
                break
        if base is None:
            raise HDF5Error(f"{path}: not an HDF5 file")
        ver = data[base + 8]
        if ver in (0, 1):
            osz, lsz = data[base + 13], data[base + 14]
            buf = _Buf(data, osz, lsz)
            p = base + 24 + (4 if ver == 1 else 0)
            root_entry = p + 4 * osz
            root_addr = buf.off(root_entry + osz)
        elif ver in (2, 3):
            osz, lsz = data[base + 9], data[base + 10]
            buf = _Buf(data, osz, lsz)
            root_addr = buf.off(base + 12 + 3 * osz)
        else:
            raise HDF5Error(f"{path}: unsupported superblock version {ver}")
        self.buf, self.path = buf, path
        self._cache: dict = {}
        root = self._object(root_addr, "/")
        if not isinstance(root, Group):
            raise HDF5Error(f"{path}: root object is not a group")
        super().__init__(self, "/", root._links)

    # -- object headers ----------------------------------------------------------------------
    def _messages(self, addr: int) -> dict:
        b = self.buf
        msgs: dict = {}
        if b.b[addr:addr + 4] == b"OHDR":
            self._messages_v2(addr, msgs)
            return msgs
        if b.b[addr] != 1:
            raise HDF5Error(f"unsupported object header version {b.b[addr]} at {addr}")
        nmsgs = b.u(addr + 2, 2)
        size = b.u(addr + 8, 4)
        blocks = [(addr + 16, size)]
        seen = 0
        while blocks and seen < nmsgs:
            start, size = blocks.pop(0)
            p, end = start, start + size
            while p + 8 <= end and seen < nmsgs:
                mtype, msize, mflags = b.u(p, 2), b.u(p + 2, 2), b.b[p + 4]
                body = bytes(b.b[p + 8:p + 8 + msize])
                seen += 1
                if mflags & 0x02:
                    raise HDF5Error("shared object header messages are not supported")
                if mtype == MSG_CONT:
                    blocks.append((b.off(p + 8), b.ln(p + 8 + b.osz)))
                else:
                    msgs.setdefault(mtype, []).append(body)
                p += 8 + msize
        return msgs

    def _messages_v2(self, addr: int, msgs: dict) -> None:
        b = self.buf
        flags = b.b[addr + 5]
        p = addr + 6
        if flags & 0x20:
            p += 16
        if flags & 0x10:
            p += 4
        szw = 1 << (flags & 3)
        size = b.u(p, szw)
        p += szw
        blocks = [(p, p + size)]
        while blocks:
            start, end = blocks.pop(0)
            q = start
            while q + 4 <= end:
                mtype, msize, mflags = b.b[q], b.u(q + 1, 2), b.b[q + 3]
                q += 4
                if flags & 0x04:
                    q += 2
                body = bytes(b.b[q:q + msize])
                if mflags & 0x02:
                    raise HDF5Error("shared object header messages are not supported")
                if mtype == MSG_CONT:
                    caddr, clen = b.off(q), b.ln(q + b.osz)
                    if b.b[caddr:caddr + 4] != b"OCHK":
                        raise HDF5Error("bad continuation block")
                    blocks.append((caddr + 4, caddr + clen - 4))
                elif mtype != MSG_NIL:
                    msgs.setdefault(mtype, []).append(body)
                q += msize

    def _object(self, addr: int, name: str):
        if addr in self._cache:
            return self._cache[addr]
        msgs = self._messages(addr)
        if MSG_SYMTAB in msgs:
            m = msgs[MSG_SYMTAB][0]
            links = self._symtab_links(self.buf.off_bytes(m, 0), self.buf.off_bytes(m, self.buf.osz))
            obj = Group(self, name, links)
        elif MSG_LINK in msgs or (MSG_LINKINFO in msgs and MSG_LAYOUT not in msgs):
            links = {}
            for m in msgs.get(MSG_LINK, []):
                k, v = self._link(m)
                if v is not None:
                    links[k] = v
            if MSG_LINKINFO in msgs:
                li = msgs[MSG_LINKINFO][0]
                p = 2 + (8 if li[1] & 1 else 0)
                if self.buf.off_bytes(li, p) != UNDEF:
                    raise HDF5Error("dense (fractal-heap) link storage is not supported")
            obj = Group(self, name, links)
        else:
            obj = Dataset(self, name, msgs)
        self._cache[addr] = obj
        return obj

    def _link(self, m: bytes):
        flags = m[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = m[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nsz = 1 << (flags & 3)
        nlen = int.from_bytes(m[p:p + nsz], "little")
        p += nsz
        name = m[p:p + nlen].decode("utf-8")
        p += nlen
        if ltype != 0:
            return name, None                       # soft / external links are skipped
        return name, self.buf.off_bytes(m, p)

    def _symtab_links(self, btree: int, heap: int) -> dict:
        b = self.buf
        if b.b[heap:heap + 4] != b"HEAP":
            raise HDF5Error("bad local heap")
        heap_data = b.off(heap + 8 + 2 * b.lsz)
        links = {}

        def walk(node):
            if b.b[node:node + 4] != b"TREE":
                raise HDF5Error("bad group B-tree node")
            level, used = b.b[node + 5], b.u(node + 6, 2)
            p = node + 8 + 2 * b.osz
            for i in range(used):
                child = b.off(p + b.lsz)
                p += b.lsz + b.osz
                if level > 0:
                    walk(child)
                else:
                    if b.b[child:child + 4] != b"SNOD":
                        raise HDF5Error("bad symbol table node")
                    n = b.u(child + 6, 2)
                    e = child + 8
                    esz = 2 * b.osz + 24
                    for j in range(n):
                        nm = b.cstr(heap_data + b.off(e + j * esz))
                        links[nm] = b.off(e + j * esz + b.osz)
        walk(btree)
        return links

    def _chunk_leaves(self, node: int, ndims: int):
        b = self.buf
        if b.b[node:node + 4] != b"TREE" or b.b[node + 4] != 1:
            raise HDF5Error("bad chunk B-tree node")
        level, used = b.b[node + 5], b.u(node + 6, 2)
        ksz = 8 + 8 * ndims
        p = node + 8 + 2 * b.osz
        for _ in range(used):
            size, mask = b.u(p, 4), b.u(p + 4, 4)
            offs = [b.u(p + 8 + 8 * d, 8) for d in range(ndims - 1)]
            child = b.off(p + ksz)
            if level > 0:
                yield from self._chunk_leaves(child, ndims)
            else:
                yield size, mask, offs, child
            p += ksz + b.osz


# ---------------------------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------------------------
def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "f":
        size = dt.itemsize
        sign, exp_loc, exp_sz, man_sz, bias = {2: (15, 10, 5, 10, 15), 4: (31, 23, 8, 23, 127),
                                               8: (63, 52, 11, 52, 1023)}[size]
        head = bytes([0x11, 0x20, sign, 0]) + struct.pack("<I", size)
        return head + struct.pack("<HHBBBBI", 0, 8 * size, exp_loc, exp_sz, 0, man_sz, bias)
    if dt.kind in "iu":
        head = bytes([0x10, 0x08 if dt.kind == "i" else 0, 0, 0]) + struct.pack("<I", dt.itemsize)
        return head + struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "S":
        return bytes([0x13, 0, 0, 0]) + struct.pack("<I", dt.itemsize)
    raise HDF5Error(f"cannot write dtype {dt}")


class _Writer:
    """Builds a file bottom-up; objects are appended after the superblock."""

    GROUP_INTERNAL_K = 16

    def __init__(self, leaf_k: int):
        self.leaf_k = leaf_k
        self.out = bytearray(b"\0" * 96)

    def alloc(self, data: bytes) -> int:
        addr = len(self.out)
        self.out += _pad8(data)
        return addr

    @staticmethod
    def _header(msgs) -> bytes:
        body = b""
        for mtype, data in msgs:
            data = _pad8(data)
            body += struct.pack("<HHB3x", mtype, len(data), 1 if mtype == MSG_DATATYPE else 0) + data
        return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body

    def dataset(self, arr: np.ndarray) -> int:
        arr = np.asarray(arr, order="C")
        if arr.dtype.byteorder == ">":
            arr = arr.astype(arr.dtype.newbyteorder("<"))
        raw = arr.tobytes()
        daddr = self.alloc(raw) if raw else UNDEF
        space = struct.pack("<BBBB4x", 1, arr.ndim, 0, 0) + b"".join(struct.pack("<Q", d) for d in arr.shape)
        fill = bytes([2, 2, 2, 0])
        layout = struct.pack("<BBQQ", 3, 1, daddr, len(raw))
        return self.alloc(self._header([(MSG_DATASPACE, space), (MSG_DATATYPE, _dtype_msg(arr.dtype)),
                                        (MSG_FILL, fill), (MSG_LAYOUT, layout)]))

    def group(self, children: dict) -> tuple[int, int, int]:
        """Returns (object header addr, btree addr, heap addr)."""
        entries = []
        for name in sorted(children, key=lambda s: s.encode()):
            v = children[name]
            if isinstance(v, dict):
                oh, bt, hp = self.group(v)
                entries.append((name, oh, 1, bt, hp))
            else:
                entries.append((name, self.dataset(_as_array(v)), 0, 0, 0))
        # local heap: offset 0 is the empty string
        heap_data = bytearray(b"\0" * 8)
        offs = []
        for name, *_ in entries:
            offs.append(len(heap_data))
            heap_data += _pad8(name.encode() + b"\0")
        heap_data += b"\0" * 16                     # keep a free block like libhdf5 does
        seg = self.alloc(bytes(heap_data))
        heap = self.alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_data), UNDEF, seg))
        # symbol table node (capacity 2K)
        cap = 2 * self.leaf_k
        snod = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(entries)))
        for (name, oh, cache, bt, hp), off in zip(entries, offs):
            snod += struct.pack("<QQII", off, oh, cache, 0)
            snod += struct.pack("<QQ", bt, hp) if cache == 1 else b"\0" * 16
        snod += b"\0" * (40 * (cap - len(entries)))
        snod_addr = self.alloc(bytes(snod))
        # group B-tree: one leaf child; keys = heap offsets of "" and of the last name
        k2 = 2 * self.GROUP_INTERNAL_K
        tree = bytearray(b"TREE" + bytes([0, 0]) + struct.pack("<H", 1) + struct.pack("<QQ", UNDEF, UNDEF))
        tree += struct.pack("<QQQ", 0, snod_addr, offs[-1] if offs else 0)
        tree += b"\0" * (8 * (k2 - 1) + 8 * (k2 - 1))
        btree = self.alloc(bytes(tree))
        oh = self.alloc(self._header([(MSG_SYMTAB, struct.pack("<QQ", btree, heap))]))
        return oh, btree, heap

    def finish(self, root: tuple[int, int, int]) -> bytes:
        oh, bt, hp = root
        eof = len(self.out)
        sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", self.leaf_k, self.GROUP_INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", bt, hp)
        assert len(sb) == 96
        self.out[:96] = sb
        return bytes(self.out)


def _as_array(v) -> np.ndarray:
    if isinstance(v, str):
        return np.array(v.encode() + b"\0", dtype=f"S{len(v.encode()) + 1}")
    if isinstance(v, bytes):
        return np.array(v + b"\0", dtype=f"S{len(v) + 1}")
    try:
        import torch
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
    except ImportError:       # pragma: no cover
        pass
    return np.asarray(v)


def _max_children(tree: dict) -> int:
    m = len(tree)
    for v in tree.values():
        if isinstance(v, dict):
            m = max(m, _max_children(v))
    return m


def write(path: str, tree: dict) -> None:
    """Write a nested ``{name: array | str | dict}`` tree as an HDF5 file (atomically)."""
    leaf_k = max(4, (_max_children(tree) + 1) // 2)
    w = _Writer(leaf_k)
    data = w.finish(w.group(tree))
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def read_string(ds: Dataset) -> str:
    """hdf5_load_string (hdf5.cpp:125-137)."""
    a = ds.read()
    v = a.reshape(-1)[0] if a.ndim else a[()]
    return bytes(v).split(b"\0", 1)[0].decode()


def read_int(ds: Dataset) -> int:
    """hdf5_load_int (hdf5.cpp:147-153)."""
    return int(ds.read().reshape(-1)[0])
