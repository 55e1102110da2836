"""HDF5 codec, HDF5Data / HDF5Output layers and HDF5 snapshots.

Reader parity is pinned by the reference's own fixture files
(caffe/src/caffe/test/test_data/{sample_data,sample_data_2_gzip,solver_data}.h5, written
by h5py/libhdf5 per generate_sample_data.py) and the expectations of
caffe/src/caffe/test/test_hdf5data_layer.cpp:55-139.  The writer is checked by round
trips through the reader; byte-level interop of written files with libhdf5 is parity
unpinned here (no libhdf5 / h5py in this environment)."""
import os

import numpy as np
import pytest
import torch

from sparknet_amd import proto
from sparknet_amd.core.net import Net
from sparknet_amd.core.solver import Solver
from sparknet_amd.utils import hdf5

FIX = "/root/reference/caffe/src/caffe/test/test_data"
need_fixtures = pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures not present")


@need_fixtures
def test_read_reference_fixtures():
    f = hdf5.File(f"{FIX}/sample_data.h5")
    assert f.keys() == ["data", "label", "label2"]
    data = f["data"].read()
    assert data.shape == (10, 8, 6, 5) and data.dtype == np.float32
    np.testing.assert_array_equal(data, np.arange(2400, dtype=np.float32).reshape(10, 8, 6, 5))
    np.testing.assert_array_equal(f["label"].read(), 1 + np.arange(10, dtype=np.float32)[:, None])
    np.testing.assert_array_equal(f["label2"].read(), 2 + np.arange(10, dtype=np.float32)[:, None])
    g = hdf5.File(f"{FIX}/sample_data_2_gzip.h5")         # chunked + deflate
    np.testing.assert_array_equal(g["data"].read(), data + 2400)
    lab = g["label"].read()
    assert lab.dtype == np.uint8
    np.testing.assert_array_equal(lab, 1 + np.arange(10, dtype=np.uint8)[:, None])
    s = hdf5.File(f"{FIX}/solver_data.h5")
    assert s["data"].shape == (8, 3, 10, 10) and s["targets"].shape == (8, 1)
    assert np.isfinite(s["data"].read()).all()


def test_writer_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    tree = {
        "f32": rng.standard_normal((3, 4, 5)).astype(np.float32),
        "f64": rng.standard_normal(7),
        "i32": np.array([42], np.int32),
        "u8": np.arange(12, dtype=np.uint8).reshape(3, 4),
        "name": "snapshot_iter_10.caffemodel.h5",
        "scalar": np.float32(2.5),
        "empty": np.zeros((0, 3), np.float32),
        "grp": {f"layer{i:02d}": {"0": np.full((2, 2), i, np.float32), "1": np.array([i], np.float32)}
                for i in range(23)},                   # > 2K entries per symbol-table node
    }
    path = str(tmp_path / "rt.h5")
    hdf5.write(path, tree)
    f = hdf5.File(path)
    assert f.keys() == sorted(tree)
    for k in ("f32", "f64", "i32", "u8"):
        got = f[k].read()
        assert got.dtype == tree[k].dtype
        np.testing.assert_array_equal(got, tree[k])
    assert hdf5.read_string(f["name"]) == tree["name"]
    assert f["scalar"].shape == () and float(f["scalar"].read()) == 2.5
    assert f["empty"].read().shape == (0, 3)
    assert len(f["grp"]) == 23
    np.testing.assert_array_equal(f["grp/layer17/0"].read(), np.full((2, 2), 17, np.float32))
    assert "grp/layer05/1" in f and "grp/nope" not in f


@need_fixtures
def test_hdf5_data_layer_matches_reference_test(tmp_path):
    lst = tmp_path / "list.txt"
    lst.write_text(f"{FIX}/sample_data.h5\n{FIX}/sample_data_2_gzip.h5\n")
    net = Net(proto.parse_prototxt(
        f'name: "h" layer {{ name: "d" type: "HDF5Data" top: "data" top: "label" top: "label2" '
        f'hdf5_data_param {{ source: "{lst}" batch_size: 5 }} }}'), phase=proto.TRAIN)
    data, label, label2 = (net.blobs[net.blob_names.index(n)] for n in ("data", "label", "label2"))
    assert data.shape == (5, 8, 6, 5) and label.shape == (5, 1) and label2.shape == (5, 1)
    ds = 8 * 6 * 5
    for it in range(10):
        net.forward()
        lo = 1 + (0 if it % 2 == 0 else 5)
        np.testing.assert_array_equal(label.data.reshape(-1).numpy(), np.arange(lo, lo + 5))
        np.testing.assert_array_equal(label2.data.reshape(-1).numpy(), np.arange(lo + 1, lo + 6))
        off = (0 if it % 4 < 2 else 2400) + (0 if it % 2 == 0 else 5 * ds)
        np.testing.assert_array_equal(data.nchw().reshape(-1).numpy(), np.arange(off, off + 5 * ds))


@need_fixtures
def test_hdf5_data_layer_shuffle_covers_rows(tmp_path):
    lst = tmp_path / "list.txt"
    lst.write_text(f"{FIX}/sample_data.h5\n")
    net = Net(proto.parse_prototxt(
        f'name: "h" layer {{ name: "d" type: "HDF5Data" top: "data" top: "label" '
        f'hdf5_data_param {{ source: "{lst}" batch_size: 5 shuffle: true }} }}'), phase=proto.TRAIN)
    data, label = net.blobs[net.blob_names.index("data")], net.blobs[net.blob_names.index("label")]
    seen = []
    for _ in range(2):
        net.forward()
        lab = label.data.reshape(-1).numpy()
        # data rows stay paired with their labels
        np.testing.assert_array_equal(data.nchw()[:, 0, 0, 0].numpy(), (lab - 1) * 240)
        seen += lab.tolist()
    assert sorted(seen) == list(range(1, 11))


def test_hdf5_output_layer(tmp_path):
    out = tmp_path / "out.h5"
    net = Net(proto.parse_prototxt(
        'name: "o" layer { name: "in" type: "DummyData" top: "x" top: "y" dummy_data_param { '
        'shape { dim: 3 dim: 2 dim: 4 dim: 4 } shape { dim: 3 dim: 1 } data_filler { type: "gaussian" } } } '
        f'layer {{ name: "w" type: "HDF5Output" bottom: "x" bottom: "y" '
        f'hdf5_output_param {{ file_name: "{out}" }} }}'), phase=proto.TEST)
    net.forward()
    f = hdf5.File(str(out))
    x = net.blobs[net.blob_names.index("x")].nchw().numpy()
    np.testing.assert_array_equal(f["data"].read(), x)
    assert f["label"].read().shape == (3, 1)


SOLVER = """
base_lr: 0.05 momentum: 0.9 weight_decay: 0.001 lr_policy: "step" gamma: 0.5 stepsize: 3
snapshot_format: HDF5 random_seed: 7
net_param {
  name: "n" force_backward: true
  layer { name: "d" type: "DummyData" top: "x" top: "t" dummy_data_param {
    shape { dim: 4 dim: 3 dim: 5 dim: 5 } shape { dim: 4 dim: 2 }
    data_filler { type: "constant" value: 0.5 } data_filler { type: "constant" value: 1 } } }
  layer { name: "c" type: "Convolution" bottom: "x" top: "c" convolution_param { num_output: 4 kernel_size: 3
    weight_filler { type: "gaussian" std: 0.1 } bias_filler { type: "constant" value: 0.1 } } }
  layer { name: "ip" type: "InnerProduct" bottom: "c" top: "y" param { name: "shared_w" } param { }
    inner_product_param { num_output: 2 weight_filler { type: "gaussian" std: 0.1 } } }
  layer { name: "loss" type: "EuclideanLoss" bottom: "y" bottom: "t" top: "l" }
}
"""


def test_hdf5_snapshot_resume_is_exact(tmp_path):
    sp = proto.parse_prototxt(SOLVER, proto.SolverParameter)
    sp.snapshot_prefix = str(tmp_path / "snap")
    a = Solver(sp)
    a.step(4)
    model, state = a.snapshot()
    assert model.endswith("_iter_4.caffemodel.h5") and state.endswith("_iter_4.solverstate.h5")
    f = hdf5.File(state)
    assert hdf5.read_int(f["iter"]) == 4 and hdf5.read_string(f["learned_net"]) == model
    assert len(f["history"]) == len(a.net.learnable_params)
    m = hdf5.File(model)
    assert m["data"].keys() == ["c", "d", "ip", "loss"] and m["data/ip"].keys() == ["0", "1"]
    a.step(3)
    b = Solver(sp)
    b.restore(state)
    assert b.iter == 4
    b.step(3)
    assert torch.equal(a.net.flat_data, b.net.flat_data)


def test_hdf5_weights_via_copy_trained_layers(tmp_path):
    sp = proto.parse_prototxt(SOLVER, proto.SolverParameter)
    a = Solver(sp)
    a.step(2)
    path = str(tmp_path / "w.caffemodel.h5")
    a.net.to_hdf5(path, write_diff=True)
    assert "diff" in hdf5.File(path)
    sp.random_seed = 99
    b = Solver(sp)
    assert not torch.equal(a.net.flat_data, b.net.flat_data)
    b.net.copy_trained_layers_from(path)
    assert torch.equal(a.net.flat_data, b.net.flat_data)


@need_fixtures
def test_train_from_hdf5_solver_data(tmp_path):
    """The reference's GradientBasedSolver fixture net (test_gradient_based_solver.cpp:
    HDF5Data over solver_data.h5 -> InnerProduct -> EuclideanLoss) trains end to end."""
    lst = tmp_path / "solver_list.txt"
    lst.write_text(f"{FIX}/solver_data.h5\n")
    sp = proto.parse_prototxt(f"""
      base_lr: 0.01 momentum: 0.9 lr_policy: "fixed" random_seed: 1
      net_param {{ name: "TestNetwork"
        layer {{ name: "data" type: "HDF5Data" top: "data" top: "targets"
                 hdf5_data_param {{ source: "{lst}" batch_size: 4 }} }}
        layer {{ name: "innerprod" type: "InnerProduct" bottom: "data" top: "innerprod"
                 inner_product_param {{ num_output: 1 weight_filler {{ type: "gaussian" std: 1.0 }}
                 bias_filler {{ type: "gaussian" std: 1.0 }} }} }}
        layer {{ name: "loss" type: "EuclideanLoss" bottom: "innerprod" bottom: "targets" }} }}""",
                              proto.SolverParameter)
    s = Solver(sp)
    first = float(s.net.forward())
    s.step(40)
    assert float(s.net.forward()) < 0.5 * first
