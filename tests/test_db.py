"""Datum databases: LMDB and LevelDB codecs, the Data layer over every backend, and the
DB apps (CreateDB / CifarDBApp / ImageNetRunDBApp flow).

Format parity with liblmdb / libleveldb is parity unpinned (neither library nor a
fixture database exists here; the reference ships none): the codecs are checked by
round trips, by structural invariants of the formats (page / block layouts, checksums,
snappy and CRC32C test vectors) and by LevelDB's log-recovery semantics."""
import os
import random
import struct

import numpy as np
import pytest
import torch

from sparknet_amd import proto
from sparknet_amd.core.net import Net
from sparknet_amd.data import leveldb as L
from sparknet_amd.data.db import DatumReader, DatumWriter, create_db, detect_backend
from sparknet_amd.data.lmdb import PAGEHDRSZ, P_BRANCH, LMDBReader, write_lmdb


def _items(n, seed=0):
    rnd = random.Random(seed)
    return {str(i).encode(): os.urandom(rnd.choice([0, 7, 300, 2030, 2100, 5000, 13000])) for i in range(n)}


def test_lmdb_roundtrip_multilevel(tmp_path):
    items = _items(3000)
    n = write_lmdb(str(tmp_path / "db"), items.items())
    assert n == 3000
    r = LMDBReader(str(tmp_path / "db"))
    assert r.entries == 3000 and r.db[2] >= 2          # depth: branch level(s) above leaves
    got = list(r.items())
    assert [k for k, _ in got] == sorted(items)        # memcmp order: "10" < "2"
    assert all(bytes(v) == items[bytes(k)] for k, v in got)
    # structural invariants of the root branch page
    root = r.db[7]
    base = root * r.psize
    flags, lower, upper = struct.unpack_from("<HHH", r.mm, base + 10)
    assert flags & P_BRANCH and PAGEHDRSZ < lower <= upper <= r.psize
    first_node = struct.unpack_from("<H", r.mm, base + PAGEHDRSZ)[0]
    assert struct.unpack_from("<H", r.mm, base + first_node + 6)[0] == 0   # implicit leftmost key
    r.close()


def test_lmdb_empty_and_single(tmp_path):
    write_lmdb(str(tmp_path / "e"), [])
    assert list(LMDBReader(str(tmp_path / "e")).items()) == []
    write_lmdb(str(tmp_path / "s"), [(b"k", b"v")])
    assert [(bytes(k), bytes(v)) for k, v in LMDBReader(str(tmp_path / "s")).items()] == [(b"k", b"v")]


def test_crc32c_and_snappy_vectors():
    assert L.crc32c(b"123456789") == 0xE3069283
    assert L._crc32c_py(b"123456789") == 0xE3069283
    assert L.unmask_crc(L.mask_crc(0x12345678)) == 0x12345678
    # "abc" literal then an overlapping 9-byte copy at offset 3
    assert L.snappy_decompress(b"\x0c\x08abc\x15\x03") == b"abcabcabcabc"
    lit = bytes(range(200))
    # long literal (tag 60 => one length byte), then a 2-byte-offset copy of 64 bytes
    stream = L.put_varint(264) + bytes([60 << 2, 199]) + lit + bytes([(63 << 2) | 2]) + struct.pack("<H", 200)
    assert L.snappy_decompress(stream) == lit + lit[:64]


def test_leveldb_roundtrip_tables(tmp_path):
    items = _items(2500, seed=1)
    L.write_leveldb(str(tmp_path / "db"), items.items(), table_bytes=4 << 20)
    files = os.listdir(tmp_path / "db")
    assert "CURRENT" in files and any(f.endswith(".ldb") for f in files)
    assert sum(f.endswith(".ldb") for f in files) > 1      # split into several tables
    got = L.read_leveldb(str(tmp_path / "db"))
    assert [k for k, _ in got] == sorted(items)
    assert all(v == items[k] for k, v in got)


def test_leveldb_log_recovery_and_deletes(tmp_path):
    d = str(tmp_path / "db")
    L.write_leveldb(d, [(b"a", b"1"), (b"b", b"2"), (b"c", b"3")])
    # newer writes sitting in a log (not yet compacted): overwrite, delete, insert
    L.append_batch_log(os.path.join(d, "000002.log"), [(b"b", b"22"), (b"c", None), (b"d", b"4")], first_seq=10)
    assert L.read_leveldb(d) == [(b"a", b"1"), (b"b", b"22"), (b"d", b"4")]
    # a corrupted record is detected
    with open(os.path.join(d, "000002.log"), "r+b") as f:
        f.seek(12)
        f.write(b"\xff")
    with pytest.raises(ValueError):
        L.read_leveldb(d)


def test_leveldb_large_record_spans_log_blocks(tmp_path):
    big = os.urandom(100_000)                          # > 3 log blocks: FIRST/MIDDLE/LAST
    path = str(tmp_path / "x.log")
    L.append_batch_log(path, [(b"k", big)])
    recs = list(L.read_log_records(path))
    assert len(recs) == 1 and list(L._batch_entries(recs[0]))[0][3] == big


@pytest.mark.parametrize("backend", ["sndb", "lmdb", "leveldb"])
def test_datum_writer_reader_and_data_layer(tmp_path, backend):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (30, 3, 8, 8), dtype=np.uint8)
    labels = rng.integers(0, 10, 30)
    path = str(tmp_path / f"db_{backend}")
    with DatumWriter(path, commit_every=7, backend=backend) as w:
        for i, (im, lab) in enumerate(zip(imgs, labels)):
            w.put_image(im, int(lab))
    assert detect_backend(path) == backend
    r = DatumReader(path)
    assert len(r) == 30
    for i in (0, 13, 29):
        d = r.get(i)
        assert d.label == labels[i]
        assert np.frombuffer(d.data, np.uint8).reshape(3, 8, 8).tolist() == imgs[i].tolist()
    txt = (f'name: "d" layer {{ name: "data" type: "Data" top: "data" top: "label" data_param {{ '
           f'source: "{path}" batch_size: 4 backend: {"LMDB" if backend == "lmdb" else "LEVELDB"} }} '
           f'transform_param {{ scale: 0.5 }} }}')
    net = Net(proto.parse_prototxt(txt), phase=proto.TRAIN)
    net.forward()
    x = net.blobs[net.blob_names.index("data")].nchw()
    assert torch.allclose(x, torch.from_numpy(imgs[:4]).float() * 0.5)
    assert net.blobs[net.blob_names.index("label")].data.tolist() == labels[:4].astype(float).tolist()


def test_decimal_keys_follow_key_order(tmp_path):
    """SparkNet's CreateDB keys are counter.toString; key order puts "10" before "2"."""
    imgs = np.arange(12, dtype=np.uint8).reshape(12, 1, 1, 1)
    create_db(str(tmp_path / "k"), imgs, np.arange(12), backend="lmdb", decimal_keys=True)
    r = DatumReader(str(tmp_path / "k"))
    assert [k.decode() for k in r.keys][:4] == ["0", "1", "10", "11"]
    assert [r.get(i).label for i in range(4)] == [0, 1, 10, 11]


@pytest.mark.parametrize("backend", ["leveldb", "lmdb"])
def test_db_app_create_and_train(tmp_path, backend):
    from sparknet_amd.apps import db_app
    out = str(tmp_path / "dbs")
    info = db_app.main(["create", "--dataset", "cifar", "--synthetic", "--synthetic-train", "400",
                        "--synthetic-test", "200", "--out", out, "--backend", backend, "--cpu",
                        "--log-dir", str(tmp_path)])
    assert info["n_train"] == 400 and os.path.exists(os.path.join(out, "mean.binaryproto"))
    assert open(os.path.join(out, "num_test_batches.txt")).read().split() == ["2"]
    solver, hist = db_app.main(["train", "--dataset", "cifar", "--db", out, "--backend", backend, "--rounds", "2",
                                "--tau", "2", "--test-every", "1", "--cpu", "--batch", "20", "--test-batch", "100",
                                "--log-dir", str(tmp_path)])
    assert solver.iter == 4 and len(hist) == 2
    assert 0.0 <= hist[0][1]["accuracy"] <= 100.0
