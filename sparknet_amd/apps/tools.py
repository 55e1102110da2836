"""Caffe's dataset / model tools (caffe/tools/*.cpp, caffe/tools/extra/parse_log.py) as
one command line:

    python -m sparknet_amd.apps.tools convert_imageset [flags] ROOT/ LISTFILE DB
    python -m sparknet_amd.apps.tools compute_image_mean [--backend B] DB [MEAN.binaryproto]
    python -m sparknet_amd.apps.tools extract_features WEIGHTS PROTOTXT BLOBS DBS NUM_BATCHES [--gpu]
    python -m sparknet_amd.apps.tools upgrade_net_proto_text IN OUT
    python -m sparknet_amd.apps.tools upgrade_net_proto_binary IN OUT
    python -m sparknet_amd.apps.tools upgrade_solver_proto_text IN OUT
    python -m sparknet_amd.apps.tools parse_log LOGFILE OUTDIR

Images are decoded with PIL (the reference needs OpenCV).  DB backends: lmdb, leveldb
(on-disk formats implemented in sparknet_amd.data) or sndb.
"""
from __future__ import annotations

import argparse
import io
import math
import os
import random
import re
import sys

import numpy as np

from .. import proto
from ..data.db import DatumReader, DatumWriter


# ---- convert_imageset (caffe/tools/convert_imageset.cpp) -------------------------------

def read_image_to_datum(path: str, label: int, height: int = 0, width: int = 0, is_color: bool = True,
                        encode_type: str = ""):
    """ReadImageToDatum (caffe/src/caffe/util/io.cpp): decode, optional resize, CHW uint8
    (BGR channel order like OpenCV) — or, with ``encode_type``, the (re-)encoded bytes."""
    from PIL import Image
    try:
        im = Image.open(path)
        im = im.convert("RGB" if is_color else "L")
    except Exception:
        return None
    if height > 0 and width > 0:
        im = im.resize((width, height), Image.BILINEAR)
    d = proto.Datum(label=int(label))
    if encode_type:
        fmt = {"jpg": "JPEG", "jpeg": "JPEG", "png": "PNG", "bmp": "BMP"}.get(encode_type.lstrip(".").lower())
        if fmt is None:
            return None
        buf = io.BytesIO()
        im.save(buf, format=fmt)
        d.data = buf.getvalue()
        d.encoded = True
        return d
    a = np.asarray(im, dtype=np.uint8)
    a = a[:, :, ::-1].transpose(2, 0, 1) if a.ndim == 3 else a[None]
    d.channels, d.height, d.width = (int(s) for s in a.shape)
    d.data = np.ascontiguousarray(a).tobytes()
    return d


def convert_imageset(root: str, listfile: str, db: str, gray=False, shuffle=False, backend="lmdb",
                     resize_width=0, resize_height=0, check_size=False, encoded=False, encode_type="",
                     seed: int = 0) -> int:
    lines = []
    with open(listfile) as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 2:
                lines.append((parts[0], int(parts[1])))
    if shuffle:
        random.Random(seed).shuffle(lines)
    count, size = 0, None
    with DatumWriter(db, commit_every=1000, backend=backend) as w:
        for i, (fn, label) in enumerate(lines):
            enc = encode_type
            if encoded and not enc:
                enc = os.path.splitext(fn)[1].lower()
            d = read_image_to_datum(os.path.join(root, fn), label, max(0, resize_height), max(0, resize_width),
                                    not gray, enc)
            if d is None:
                continue
            if check_size and not d.encoded:
                n = d.channels * d.height * d.width
                if size is None:
                    size = n
                elif n != size:
                    raise ValueError(f"Incorrect data field size {n} (expected {size}) for {fn}")
            w.put(d, f"{i:08d}_{fn}")
            count += 1
    return count


# ---- compute_image_mean (caffe/tools/compute_image_mean.cpp) ----------------------------

def datum_pixels(d) -> np.ndarray:
    if d.encoded:
        from PIL import Image
        im = Image.open(io.BytesIO(d.data))
        a = np.asarray(im.convert("RGB" if im.mode != "L" else "L"), dtype=np.uint8)
        return a[:, :, ::-1].transpose(2, 0, 1).astype(np.float64) if a.ndim == 3 else a[None].astype(np.float64)
    if len(d.data):
        return np.frombuffer(d.data, np.uint8).reshape(d.channels, d.height, d.width).astype(np.float64)
    return np.asarray(d.float_data, np.float64).reshape(d.channels, d.height, d.width)


def compute_image_mean(db: str, out: str | None = None, backend: str | None = None) -> np.ndarray:
    r = DatumReader(db, backend)
    total = None
    for i in range(len(r)):
        x = datum_pixels(r.get(i))
        if total is None:
            total = np.zeros_like(x)
        elif x.shape != total.shape:
            raise ValueError("Incorrect data field size")
        total += x
    mean = (total / len(r)).astype(np.float32)
    if out:
        bp = proto.BlobProto(num=1, channels=mean.shape[0], height=mean.shape[1], width=mean.shape[2])
        bp.data.extend(mean.reshape(-1).tolist())
        proto.write_binary(out, bp)
    return mean


# ---- extract_features (caffe/tools/extract_features.cpp) --------------------------------

def extract_features(weights: str, prototxt: str, blob_names: list[str], dbs: list[str], num_batches: int,
                     backend: str = "lmdb", device: str = "cpu") -> int:
    """Forward the TEST net ``num_batches`` times and store every image's feature vector of
    each named blob as a float Datum (key = running image index)."""
    from ..core.net import Net
    if len(blob_names) != len(dbs):
        raise ValueError("the number of blob names and datasets must be equal")
    net = Net(proto.read_net(prototxt), phase=proto.TEST, device=device)
    net.copy_trained_layers_from(weights)
    net.sync_compute()
    for b in blob_names:
        if not net.has_blob(b):
            raise ValueError(f"Unknown feature blob name {b} in the network {prototxt}")
    writers = [DatumWriter(p, commit_every=1000, backend=backend) for p in dbs]
    n = 0
    try:
        for _ in range(num_batches):
            net.forward()
            for name, w in zip(blob_names, writers):
                t = net.blob_by_name(name).nchw().float().cpu()
                feats = t.reshape(t.shape[0], -1).numpy()
                per = t.shape[1:] if t.dim() == 4 else (feats.shape[1], 1, 1)
                for j in range(feats.shape[0]):
                    d = proto.Datum(channels=int(per[0]), height=int(per[1]) if len(per) > 1 else 1,
                                    width=int(per[2]) if len(per) > 2 else 1)
                    d.float_data.extend(feats[j].tolist())
                    w.put(d, f"{n + j:010d}")
            n += feats.shape[0]
    finally:
        for w in writers:
            w.close()
    return n


# ---- proto upgrades (caffe/tools/upgrade_*.cpp) ----------------------------------------

def upgrade_net_proto(inp: str, out: str, binary_out: bool) -> None:
    from ..proto.upgrade import upgrade_net
    net = proto.read_net(inp) if not inp.endswith((".prototxt", ".txt")) else upgrade_net(proto.read_prototxt(inp))
    (proto.write_binary if binary_out else proto.write_prototxt)(out, net)


def upgrade_solver_proto(inp: str, out: str) -> None:
    from ..proto.upgrade import upgrade_solver
    proto.write_prototxt(out, upgrade_solver(proto.read_solver(inp)))


# ---- parse_log (caffe/tools/extra/parse_log.py) -----------------------------------------

_RE_ITER = re.compile(r"Iteration (\d+)")
_RE_TRAIN = re.compile(r"Train net output #(\d+): (\S+) = ([\.\deE+-]+)")
_RE_TEST = re.compile(r"Test net output #(\d+): (\S+) = ([\.\deE+-]+)")
_RE_LOSS = re.compile(r"Iteration (\d+), loss = ([\.\deE+-]+)")
_RE_LR = re.compile(r"lr = ([-+]?[0-9]*\.?[0-9]+([eE]?[-+]?[0-9]+)?)")
_RE_GLOG = re.compile(r"^[IWEF](\d{2})(\d{2}) (\d{2}):(\d{2}):(\d{2}\.\d+)")
_RE_SN = re.compile(r"^(\d+\.\d+)(?:, i = \d+)?: ")


def _seconds(line: str):
    m = _RE_GLOG.match(line)
    if m:
        mon, day, h, mi, s = m.groups()
        return ((int(day) * 24 + int(h)) * 60 + int(mi)) * 60 + float(s)
    m = _RE_SN.match(line)
    return float(m.group(1)) if m else None


def parse_log(path: str):
    """(train rows, test rows): dicts with NumIters, Seconds, LearningRate and one column
    per net output, from Caffe glog logs or this framework's training logs."""
    train, test = [], []
    it, lr, t0 = -1, float("nan"), None

    def row_for(rows, seconds):
        if not rows or rows[-1]["NumIters"] != it:
            rows.append({"NumIters": it, "Seconds": seconds, "LearningRate": lr})
        return rows[-1]

    with open(path) as f:
        for line in f:
            sec = _seconds(line)
            if sec is not None:
                t0 = sec if t0 is None else t0
                sec -= t0
            m = _RE_ITER.search(line)
            if m:
                it = int(m.group(1))
            m = _RE_LR.search(line)
            if m:
                lr = float(m.group(1))
                for rows in (train, test):
                    if rows and rows[-1]["NumIters"] == it and math.isnan(rows[-1]["LearningRate"]):
                        rows[-1]["LearningRate"] = lr
            m = _RE_LOSS.search(line)
            if m and it >= 0:
                row_for(train, sec)["loss"] = float(m.group(2))
            m = _RE_TRAIN.search(line)
            if m and it >= 0:
                row_for(train, sec)[m.group(2)] = float(m.group(3))
            m = _RE_TEST.search(line)
            if m and it >= 0:
                row_for(test, sec)[m.group(2)] = float(m.group(3))
    return train, test


def write_parsed_log(path: str, outdir: str, delimiter: str = ",") -> tuple[str, str]:
    import csv
    train, test = parse_log(path)
    base = os.path.join(outdir, os.path.basename(path))
    outs = []
    for rows, ext in ((train, ".train"), (test, ".test")):
        fn = base + ext
        keys = []
        for r in rows:
            keys += [k for k in r if k not in keys]
        with open(fn, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys or ["NumIters"], delimiter=delimiter)
            w.writeheader()
            w.writerows(rows)
        outs.append(fn)
    return outs[0], outs[1]


# ---- CLI ------------------------------------------------------------------------------

def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="sparknet_amd.apps.tools")
    sub = ap.add_subparsers(dest="tool", required=True)
    c = sub.add_parser("convert_imageset")
    c.add_argument("root")
    c.add_argument("listfile")
    c.add_argument("db")
    c.add_argument("--gray", action="store_true")
    c.add_argument("--shuffle", action="store_true")
    c.add_argument("--backend", default="lmdb")
    c.add_argument("--resize_width", type=int, default=0)
    c.add_argument("--resize_height", type=int, default=0)
    c.add_argument("--check_size", action="store_true")
    c.add_argument("--encoded", action="store_true")
    c.add_argument("--encode_type", default="")
    m = sub.add_parser("compute_image_mean")
    m.add_argument("db")
    m.add_argument("out", nargs="?")
    m.add_argument("--backend", default=None)
    e = sub.add_parser("extract_features")
    e.add_argument("weights")
    e.add_argument("prototxt")
    e.add_argument("blobs")
    e.add_argument("dbs")
    e.add_argument("num_batches", type=int)
    e.add_argument("--backend", default="lmdb")
    e.add_argument("--gpu", action="store_true")
    for name in ("upgrade_net_proto_text", "upgrade_net_proto_binary", "upgrade_solver_proto_text"):
        u = sub.add_parser(name)
        u.add_argument("inp")
        u.add_argument("out")
    p = sub.add_parser("parse_log")
    p.add_argument("logfile")
    p.add_argument("outdir")
    p.add_argument("--delimiter", default=",")
    a = ap.parse_args(argv)
    if a.tool == "convert_imageset":
        n = convert_imageset(a.root, a.listfile, a.db, a.gray, a.shuffle, a.backend, a.resize_width,
                             a.resize_height, a.check_size, a.encoded, a.encode_type)
        print(f"Processed {n} files.")
    elif a.tool == "compute_image_mean":
        mean = compute_image_mean(a.db, a.out, a.backend)
        for c_, v in enumerate(mean.reshape(mean.shape[0], -1).mean(1)):
            print(f"mean_value channel [{c_}]: {v:.4f}")
    elif a.tool == "extract_features":
        n = extract_features(a.weights, a.prototxt, a.blobs.split(","), a.dbs.split(","), a.num_batches,
                             a.backend, "cuda" if a.gpu else "cpu")
        print(f"Extracted features of {n} query images.")
    elif a.tool == "upgrade_net_proto_text":
        upgrade_net_proto(a.inp, a.out, False)
    elif a.tool == "upgrade_net_proto_binary":
        upgrade_net_proto(a.inp, a.out, True)
    elif a.tool == "upgrade_solver_proto_text":
        upgrade_solver_proto(a.inp, a.out)
    elif a.tool == "parse_log":
        print(*write_parsed_log(a.logfile, a.outdir, a.delimiter))
    return 0


if __name__ == "__main__":
    sys.exit(main())
