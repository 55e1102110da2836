"""Dataset / model tools (sparknet_amd.apps.tools) — caffe/tools/{convert_imageset,
compute_image_mean,extract_features,upgrade_*}.cpp and tools/extra/parse_log.py."""
import numpy as np
import pytest

from sparknet_amd import proto
from sparknet_amd.apps import tools
from sparknet_amd.data.db import DatumReader


def _images(tmp_path, n=6, size=(10, 12)):
    from PIL import Image
    rng = np.random.default_rng(0)
    root = tmp_path / "imgs"
    root.mkdir()
    lines, arrays = [], []
    for i in range(n):
        a = rng.integers(0, 256, (size[0], size[1], 3), dtype=np.uint8)
        Image.fromarray(a).save(root / f"im{i}.png")
        lines.append(f"im{i}.png {i % 3}")
        arrays.append(a)
    lf = tmp_path / "list.txt"
    lf.write_text("\n".join(lines) + "\n")
    return str(root) + "/", str(lf), arrays


@pytest.mark.parametrize("backend", ["lmdb", "leveldb", "sndb"])
def test_convert_imageset_and_mean(tmp_path, backend):
    root, lf, arrays = _images(tmp_path)
    db = str(tmp_path / f"db_{backend}")
    assert tools.convert_imageset(root, lf, db, backend=backend, check_size=True) == 6
    r = DatumReader(db)
    assert len(r) == 6
    d = r.get(2)
    assert (d.channels, d.height, d.width, d.label) == (3, 10, 12, 2)
    chw_bgr = arrays[2][:, :, ::-1].transpose(2, 0, 1)
    assert np.array_equal(np.frombuffer(d.data, np.uint8).reshape(3, 10, 12), chw_bgr)
    out = str(tmp_path / "mean.binaryproto")
    mean = tools.compute_image_mean(db, out)
    ref = np.mean([a[:, :, ::-1].transpose(2, 0, 1).astype(np.float64) for a in arrays], axis=0)
    assert np.allclose(mean, ref, atol=1e-4)
    bp = proto.read_binary(out, proto.BlobProto)
    assert (bp.channels, bp.height, bp.width) == (3, 10, 12)


def test_convert_imageset_resize_encoded(tmp_path):
    root, lf, _ = _images(tmp_path)
    db = str(tmp_path / "enc")
    tools.convert_imageset(root, lf, db, backend="lmdb", resize_width=8, resize_height=6, encode_type="png",
                           shuffle=True)
    r = DatumReader(db)
    d = r.get(0)
    assert d.encoded and tools.datum_pixels(d).shape == (3, 6, 8)
    assert tools.compute_image_mean(db).shape == (3, 6, 8)


def test_extract_features(tmp_path):
    net = tmp_path / "feat.prototxt"
    net.write_text("""name: 'f'
      layer { name: 'data' type: 'DummyData' top: 'data'
        dummy_data_param { shape { dim: 4 dim: 3 dim: 5 dim: 5 } data_filler { type: 'gaussian' } } }
      layer { name: 'ip' type: 'InnerProduct' bottom: 'data' top: 'ip'
        inner_product_param { num_output: 7 weight_filler { type: 'gaussian' std: 0.1 } } }""")
    from sparknet_amd.core.net import Net
    n = Net(proto.read_net(str(net)), phase=proto.TEST)
    w = str(tmp_path / "f.caffemodel")
    proto.write_binary(w, n.to_proto())
    dbs = [str(tmp_path / "ip_db"), str(tmp_path / "data_db")]
    assert tools.extract_features(w, str(net), ["ip", "data"], dbs, 2, backend="sndb") == 8
    r = DatumReader(dbs[0])
    assert len(r) == 8 and len(r.get(0).float_data) == 7
    r2 = DatumReader(dbs[1])
    d = r2.get(3)
    assert (d.channels, d.height, d.width) == (3, 5, 5)


def test_upgrade_tools(tmp_path):
    v1 = tmp_path / "v1.prototxt"
    v1.write_text("""name: 'old'
      layers { name: 'ip' type: INNER_PRODUCT bottom: 'data' top: 'ip' blobs_lr: 2 weight_decay: 0
               inner_product_param { num_output: 3 } }""")
    out = tmp_path / "v2.prototxt"
    tools.upgrade_net_proto(str(v1), str(out), binary_out=False)
    net = proto.read_prototxt(str(out))
    assert len(net.layers) == 0 and net.layer[0].type == "InnerProduct" and net.layer[0].param[0].lr_mult == 2
    sv = tmp_path / "s.prototxt"
    sv.write_text("base_lr: 0.1 solver_type: NESTEROV")
    so = tmp_path / "s2.prototxt"
    tools.upgrade_solver_proto(str(sv), str(so))
    sp = proto.read_solver(str(so))
    assert sp.type == "Nesterov" and not sp.HasField("solver_type")


def test_parse_log(tmp_path):
    log = tmp_path / "caffe.log"
    log.write_text("""I1016 10:00:00.000000  1 solver.cpp:1] Iteration 0, Testing net (#0)
I1016 10:00:01.000000  1 solver.cpp:2]     Test net output #0: accuracy = 0.1
I1016 10:00:02.000000  1 solver.cpp:3] Iteration 0, loss = 2.3
I1016 10:00:02.000000  1 solver.cpp:4]     Train net output #0: loss = 2.3 (* 1 = 2.3 loss)
I1016 10:00:02.000000  1 sgd_solver.cpp:5] Iteration 0, lr = 0.01
I1016 10:00:12.500000  1 solver.cpp:3] Iteration 100, loss = 1.5
I1016 10:00:12.500000  1 sgd_solver.cpp:5] Iteration 100, lr = 0.01
""")
    train, test = tools.parse_log(str(log))
    assert [r["NumIters"] for r in train] == [0, 100]
    assert train[1]["loss"] == 1.5 and abs(train[1]["Seconds"] - 12.5) < 1e-6 and train[1]["LearningRate"] == 0.01
    assert test[0]["accuracy"] == 0.1
    tr, te = tools.write_parsed_log(str(log), str(tmp_path))
    assert open(tr).readline().startswith("NumIters")


def test_window_data_layer(tmp_path):
    """WindowData (window_data_layer.cpp): bg windows first, fg after; constant images make
    the warped crops exact; context padding past the image edge leaves a zero border."""
    from PIL import Image
    from sparknet_amd.core.net import Net
    for i, v in enumerate((40, 200)):
        Image.fromarray(np.full((20, 30, 3), v, np.uint8)).save(tmp_path / f"w{i}.png")
    wf = tmp_path / "windows.txt"
    wf.write_text("# 0\nw0.png\n3 20 30\n2\n1 0.9 2 3 12 15\n0 0.1 0 0 29 19\n"
                  "# 1\nw1.png\n3 20 30\n1\n2 0.7 5 5 25 15\n")

    def net(pad, mean_value=10.0):
        txt = f"""name: 'w'
          layer {{ name: 'd' type: 'WindowData' top: 'data' top: 'label'
            transform_param {{ crop_size: 8 mirror: true mean_value: {mean_value} }}
            window_data_param {{ source: '{wf}' root_folder: '{tmp_path}/' batch_size: 8
              fg_fraction: 0.5 scale: 0.5 context_pad: {pad} }} }}"""
        return Net(proto.parse_prototxt(txt), phase=proto.TRAIN, seed=3)

    n = net(0)
    n.forward()
    data = n.blob_by_name("data").nchw().float().numpy()
    lab = n.blob_by_name("label").data.float().numpy()
    assert data.shape == (8, 3, 8, 8)
    assert (lab[:4] == 0).all() and set(lab[4:].tolist()) <= {1.0, 2.0}
    for k in range(8):
        v = {0: 40, 1: 40, 2: 200}[int(lab[k])] if lab[k] else 40
        assert np.allclose(data[k], (v - 10.0) * 0.5)
    n = net(2)
    n.forward()
    data = n.blob_by_name("data").nchw().float().numpy()
    lab = n.blob_by_name("label").data.float().numpy()
    bg = data[:4]  # full-image background window grown by the context: zero border
    # window grows to x -15..45, y -10..30: a 4x4 patch at offset (2, 2) either way
    assert np.allclose(bg[:, :, 2:6, 2:6], (40 - 10.0) * 0.5)
    assert (bg[:, :, :2] == 0).all() and (bg[:, :, 6:] == 0).all()
    assert (bg[:, :, :, :2] == 0).all() and (bg[:, :, :, 6:] == 0).all()
