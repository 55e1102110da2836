"""libsn_core — the C ABI replacing SparkNet's libccaffe (libccaffe/ccaffe.cpp:22-296).
A C host program (tests/native/core_demo.c) trains through it with callback-fed data,
tests, and round-trips flat weights and a .caffemodel; the same library is also driven
from Python through ctypes (interpreter already running, GIL handed over)."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from sparknet_amd import build_native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sparknet_amd", "lib")
SOLVER = os.path.join(ROOT, "tests", "native", "core_solver.prototxt")


@pytest.fixture(scope="module")
def core_lib():
    out = build_native.build()
    assert "core" in out
    return out["core"]


def _c_host_program(tmp_path, device):
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "core_demo"
    r = subprocess.run(["gcc", "-std=c11", "-O1", f"-I{ROOT}/csrc/core", f"{ROOT}/tests/native/core_demo.c",
                        f"-L{LIB}", "-lsn_core", f"-Wl,-rpath,{LIB}", "-lm", "-o", str(exe)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ)
    if device < 0:
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    db = tmp_path / "demo_db"
    r = subprocess.run([str(exe), SOLVER, str(tmp_path / "w.caffemodel"), str(device), str(db)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout, r.stderr[-3000:])
    if device < 0:
        assert "native=0" in r.stdout
    assert "layers=7 layer2=conv1" in r.stdout and "callbacks=15" in r.stdout
    assert "weights2=2" in r.stdout and "blob0=data" in r.stdout
    from sparknet_amd.data.db import DatumReader
    from sparknet_amd.data.loaders import read_mean_binaryproto
    rd = DatumReader(str(db))
    assert len(rd) == 5 and [rd.get(i).label for i in range(5)] == [0, 1, 2, 3, 4]
    assert list(rd.get(3).data[:2]) == [144, 145]
    assert read_mean_binaryproto(str(db) + ".mean.binaryproto").reshape(-1).tolist() == [1.0, 2.0, 3.0]
    return r.stdout


def test_c_host_program(core_lib, tmp_path):
    _c_host_program(tmp_path, -1)


@pytest.mark.gpu
def test_c_host_program_gpu_native_step(core_lib, tmp_path):
    """The same C host program on the GPU: sn_solver_step captures one iteration and runs
    the remaining ones in the native C++ loop (sn_native_iterations > 0)."""
    out = _c_host_program(tmp_path, 0)
    assert "native=2" in out, out
    # step, test, forward, get / set weights: zero interpreter entries
    assert "steady_py=0 " in out, out



CB = C.CFUNCTYPE(None, C.POINTER(C.c_float), C.c_int, C.c_int, C.POINTER(C.c_int), C.c_void_p)


def test_ctypes_inside_python(core_lib, tmp_path):
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_num_params.restype = C.c_longlong
    for f in ("sn_set_device", "sn_load_solver_from_protobuf", "sn_set_train_data_callback", "sn_solver_step",
              "sn_get_weights", "sn_parse_solver_prototxt"):
        getattr(lib, f).restype = C.c_int
    st = C.c_void_p(lib.sn_create_state())
    assert st.value, lib.sn_last_error()
    buf, n = C.c_char_p(), C.c_int()
    assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
    assert lib.sn_set_device(st, -1) == 0
    assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()
    seen = []

    def fill(p, batch, nd, shape, user):
        cnt = int(np.prod([shape[i] for i in range(nd)]))
        arr = np.ctypeslib.as_array(p, shape=(cnt,))
        arr[:] = np.linspace(-1, 1, cnt, dtype=np.float32) if nd == 4 else (np.arange(cnt) % 3)
        seen.append(nd)

    cb = CB(fill)
    assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
    assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
    assert lib.sn_solver_step(st, 3) == 0, lib.sn_last_error()
    assert sorted(set(seen)) == [2, 4] and len(seen) == 6
    nparam = lib.sn_num_params(st)
    w = (C.c_float * nparam)()
    assert lib.sn_get_weights(st, w, C.c_longlong(nparam)) == 0
    assert np.isfinite(np.frombuffer(w, dtype=np.float32)).all()
    lib.sn_free(buf)
    lib.sn_destroy_state(st)


def test_native_param_blob_verbs_match_python(core_lib, monkeypatch):
    """sn_blob_num_axes / axis_shape / get / set on layer parameters run natively off the
    weights plan (flat buffer offsets + the conv weights' [K][R][S][C] -> [K][C][R][S]
    conversion) and agree with the Python path (SN_NATIVE_STEP=0) on every parameter of
    every layer, data and diff; a native set is what the Python path reads back."""
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_python_entries.restype = C.c_longlong
    st = C.c_void_p(lib.sn_create_state())
    buf, n = C.c_char_p(), C.c_int()
    assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
    assert lib.sn_set_device(st, -1) == 0
    assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()

    def fill(p, batch, nd, shape, user):
        cnt = int(np.prod([shape[i] for i in range(nd)]))
        arr = np.ctypeslib.as_array(p, shape=(cnt,))
        arr[:] = np.cos(0.11 * np.arange(cnt)).astype(np.float32) if nd == 4 else (np.arange(cnt) % 3)

    cb = CB(fill)
    assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
    assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
    assert lib.sn_solver_step(st, 2) == 0, lib.sn_last_error()
    rng = np.random.default_rng(3)

    def blob(layer, index, native):
        monkeypatch.setenv("SN_NATIVE_STEP", "1" if native else "0")
        axes = lib.sn_blob_num_axes(st, layer, index)
        shape = [lib.sn_blob_axis_shape(st, layer, index, a) for a in range(axes)]
        return axes, shape

    def get(layer, index, diff, cnt, native):
        monkeypatch.setenv("SN_NATIVE_STEP", "1" if native else "0")
        out = (C.c_float * cnt)()
        assert lib.sn_blob_get(st, layer, index, diff, out, C.c_longlong(cnt)) == 0, lib.sn_last_error()
        return np.frombuffer(out, dtype=np.float32).copy()

    checked = 0
    for layer in range(lib.sn_num_layers(st)):
        for index in range(lib.sn_num_layer_weights(st, layer)):
            axes, shape = blob(layer, index, False)
            assert blob(layer, index, True) == (axes, shape)
            cnt = int(np.prod(shape))
            for diff in (0, 1):
                np.testing.assert_array_equal(get(layer, index, diff, cnt, True), get(layer, index, diff, cnt, False))
            vals = rng.standard_normal(cnt).astype(np.float32)
            monkeypatch.setenv("SN_NATIVE_STEP", "1")
            py0 = lib.sn_python_entries()
            assert lib.sn_blob_set(st, layer, index, 0, vals.ctypes.data_as(C.POINTER(C.c_float)),
                                   C.c_longlong(cnt)) == 0, lib.sn_last_error()
            assert lib.sn_python_entries() == py0  # the plan exists: no interpreter entry
            np.testing.assert_array_equal(get(layer, index, 0, cnt, False), vals)
            small = (C.c_float * 1)()
            monkeypatch.setenv("SN_NATIVE_STEP", "1")
            if cnt > 1:
                assert lib.sn_blob_get(st, layer, index, 0, small, C.c_longlong(1)) != 0
                assert b"buffer holds 1 floats" in lib.sn_last_error()
            checked += 1
    assert checked >= 4
    lib.sn_free(buf)
    lib.sn_destroy_state(st)


def _ctypes_train(core_lib, device, iters, native):
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_num_params.restype = C.c_longlong
    lib.sn_native_iterations.restype = C.c_longlong
    os.environ["SN_NATIVE_STEP"] = "1" if native else "0"
    try:
        st = C.c_void_p(lib.sn_create_state())
        buf, n = C.c_char_p(), C.c_int()
        assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
        assert lib.sn_set_device(st, device) == 0
        assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()
        calls = [0]

        def fill(p, batch, nd, shape, user):
            cnt = int(np.prod([shape[i] for i in range(nd)]))
            arr = np.ctypeslib.as_array(p, shape=(cnt,))
            if nd == 4:
                arr[:] = np.sin(0.37 * (np.arange(cnt) + 13 * calls[0])).astype(np.float32)
                calls[0] += 1
            else:
                arr[:] = (np.arange(cnt) + calls[0]) % 3

        cb = CB(fill)
        assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
        assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
        assert lib.sn_solver_step(st, iters) == 0, lib.sn_last_error()
        nparam = lib.sn_num_params(st)
        w = (C.c_float * nparam)()
        assert lib.sn_get_weights(st, w, C.c_longlong(nparam)) == 0
        nat = lib.sn_native_iterations(st)
        lib.sn_free(buf)
        lib.sn_destroy_state(st)
        return np.frombuffer(w, dtype=np.float32).copy(), nat, calls[0]
    finally:
        os.environ.pop("SN_NATIVE_STEP", None)


@pytest.mark.gpu
def test_native_step_matches_python_step(core_lib):
    """20 iterations through the native C++ step loop (after its 3 capture iterations) end
    at the same weights as 20 iterations of the Python solver fed by the same callbacks."""
    w_py, nat_py, calls_py = _ctypes_train(core_lib, 0, 20, native=False)
    w_nat, nat, calls_nat = _ctypes_train(core_lib, 0, 20, native=True)
    assert nat_py == 0 and nat == 17 and calls_py == calls_nat == 20
    err = np.abs(w_nat - w_py).max() / (np.abs(w_py).max() + 1e-12)
    assert err < 2e-2, err


def _ctypes_eval(core_lib, native_verbs):
    """Python-path training (SN_NATIVE_STEP=0), then sn_solver_test / sn_forward /
    sn_get_weights twice each with the native verbs on or off."""
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_num_params.restype = C.c_longlong
    lib.sn_python_entries.restype = C.c_longlong
    lib.sn_get_test_score.restype = C.c_float
    os.environ["SN_NATIVE_STEP"] = "0"
    try:
        st = C.c_void_p(lib.sn_create_state())
        buf, n = C.c_char_p(), C.c_int()
        assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
        assert lib.sn_set_device(st, 0) == 0
        assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()
        calls = [0]

        def fill(p, batch, nd, shape, user):
            cnt = int(np.prod([shape[i] for i in range(nd)]))
            arr = np.ctypeslib.as_array(p, shape=(cnt,))
            if nd == 4:
                arr[:] = np.cos(0.29 * (np.arange(cnt) + 7 * calls[0])).astype(np.float32)
                calls[0] += 1
            else:
                arr[:] = (np.arange(cnt) + calls[0]) % 3

        cb = CB(fill)
        for t in (0, 1):
            f = lib.sn_set_test_data_callback if t else lib.sn_set_train_data_callback
            assert f(st, 0, cb, None) == 0 and f(st, 1, cb, None) == 0
        assert lib.sn_solver_step(st, 6) == 0, lib.sn_last_error()
        os.environ["SN_NATIVE_STEP"] = "1" if native_verbs else "0"
        nparam = lib.sn_num_params(st)
        w = (C.c_float * nparam)()
        scores, losses, py = [], [], []
        for _ in range(2):
            py.append(lib.sn_python_entries())
            assert lib.sn_solver_test(st, 3) == 1, lib.sn_last_error()
            scores.append(lib.sn_get_test_score(st, 0))
            loss = C.c_float()
            assert lib.sn_forward(st, C.byref(loss)) == 0, lib.sn_last_error()
            losses.append(loss.value)
            assert lib.sn_get_weights(st, w, C.c_longlong(nparam)) == 0
            assert lib.sn_set_weights(st, w, C.c_longlong(nparam)) == 0
        py.append(lib.sn_python_entries())
        lib.sn_free(buf)
        lib.sn_destroy_state(st)
        return scores, losses, np.frombuffer(w, dtype=np.float32).copy(), py[2] - py[1], calls[0]
    finally:
        os.environ.pop("SN_NATIVE_STEP", None)


@pytest.mark.gpu
def test_native_test_forward_weights_match_python(core_lib):
    """The captured forward-only graphs (sn_forward, sn_solver_test) and the hipMemcpy
    weight verbs give what the Python verbs give, with no interpreter entry once built."""
    s_py, l_py, w_py, py_py, c_py = _ctypes_eval(core_lib, False)
    s_nat, l_nat, w_nat, py_nat, c_nat = _ctypes_eval(core_lib, True)
    assert c_py == c_nat == 6 + 2 * (3 + 1)
    assert py_py > 0 and py_nat == 0
    np.testing.assert_allclose(s_nat, s_py, rtol=1e-3)
    np.testing.assert_allclose(l_nat, l_py, rtol=1e-3)
    assert np.array_equal(w_nat, w_py)


def _blob(lib, st, layer, index, diff):
    nd = lib.sn_blob_num_axes(st, layer, index)
    cnt = int(np.prod([lib.sn_blob_axis_shape(st, layer, index, a) for a in range(nd)])) if nd > 0 else 1
    buf = (C.c_float * cnt)()
    assert lib.sn_blob_get(st, layer, index, diff, buf, C.c_longlong(cnt)) == 0, lib.sn_last_error()
    return np.frombuffer(buf, dtype=np.float32).copy()


def _ctypes_fwd_bwd(core_lib, native_verbs):
    """sn_forward -> sn_backward -> blob / parameter-gradient reads, on the first call and
    again after an intervening sn_solver_step (a captured forward plan must
    leave the net's blobs holding a real forward, and be dropped once a step rebinds them)."""
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    os.environ["SN_NATIVE_STEP"] = "0"
    try:
        st = C.c_void_p(lib.sn_create_state())
        buf, n = C.c_char_p(), C.c_int()
        assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
        assert lib.sn_set_device(st, 0) == 0
        assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()
        calls = [0]

        def fill(p, batch, nd, shape, user):
            cnt = int(np.prod([shape[i] for i in range(nd)]))
            arr = np.ctypeslib.as_array(p, shape=(cnt,))
            if nd == 4:
                arr[:] = np.cos(0.31 * (np.arange(cnt) + 5 * calls[0])).astype(np.float32)
                calls[0] += 1
            else:
                arr[:] = (np.arange(cnt) + calls[0]) % 3
        cb = CB(fill)
        assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
        assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
        assert lib.sn_solver_step(st, 3) == 0, lib.sn_last_error()
        os.environ["SN_NATIVE_STEP"] = "1" if native_verbs else "0"
        out = []
        for rnd in range(3):
            for _ in range(2):  # the first sn_forward builds the plan, the second replays it
                loss = C.c_float()
                assert lib.sn_forward(st, C.byref(loss)) == 0, lib.sn_last_error()
                assert lib.sn_backward(st) == 0, lib.sn_last_error()
                out.append((loss.value, _blob(lib, st, -1, 4, 0), _blob(lib, st, -1, 3, 0),
                            _blob(lib, st, 5, 0, 1), _blob(lib, st, 2, 0, 1)))
            assert lib.sn_solver_step(st, 2 if rnd == 0 else 5) == 0, lib.sn_last_error()
        lib.sn_free(buf)
        lib.sn_destroy_state(st)
        return out, calls[0]
    finally:
        os.environ.pop("SN_NATIVE_STEP", None)


@pytest.mark.gpu
def test_native_forward_then_backward_and_blob_reads(core_lib):
    py, c_py = _ctypes_fwd_bwd(core_lib, False)
    nat, c_nat = _ctypes_fwd_bwd(core_lib, True)
    assert c_py == c_nat
    for a, b in zip(py, nat):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-3)
        for x, y in zip(a[1:], b[1:]):
            assert np.isfinite(y).all()
            np.testing.assert_allclose(y, x, rtol=2e-2, atol=2e-2 * (np.abs(x).max() + 1e-6))


def _bn_stats_after_forwards(core_lib, native_verbs, forwards=3):
    """3 Python-path steps of a net with a train-phase BatchNorm, then `forwards` sn_forward
    calls (the first one builds the native plan when native_verbs is on): the BN running
    mean / variance / factor after each call."""
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    os.environ["SN_NATIVE_STEP"] = "0"
    try:
        st = C.c_void_p(lib.sn_create_state())
        buf, n = C.c_char_p(), C.c_int()
        solver = os.path.join(ROOT, "tests", "native", "core_solver_bn.prototxt")
        assert lib.sn_parse_solver_prototxt(solver.encode(), C.byref(buf), C.byref(n)) == 0
        assert lib.sn_set_device(st, 0) == 0
        assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()

        def fill(p, batch, nd, shape, user):
            cnt = int(np.prod([shape[i] for i in range(nd)]))
            arr = np.ctypeslib.as_array(p, shape=(cnt,))
            arr[:] = np.cos(0.23 * np.arange(cnt)).astype(np.float32) if nd == 4 else np.arange(cnt) % 3
        cb = CB(fill)
        assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
        assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
        assert lib.sn_solver_step(st, 3) == 0, lib.sn_last_error()
        os.environ["SN_NATIVE_STEP"] = "1" if native_verbs else "0"
        out = []
        for _ in range(forwards):
            loss = C.c_float()
            assert lib.sn_forward(st, C.byref(loss)) == 0, lib.sn_last_error()
            out.append([_blob(lib, st, 3, i, 0) for i in range(3)])  # layer 3 = bn1
        lib.sn_free(buf)
        lib.sn_destroy_state(st)
        return out
    finally:
        os.environ.pop("SN_NATIVE_STEP", None)


@pytest.mark.gpu
def test_native_forward_plan_updates_batchnorm_stats_once(core_lib):
    """building the captured forward plan replays the forward once after the
    eager forward; a train-phase BatchNorm must still update its running statistics once
    per sn_forward (Caffe: once per Forward, batch_norm_layer.cpp:104-121)."""
    py = _bn_stats_after_forwards(core_lib, False)
    nat = _bn_stats_after_forwards(core_lib, True)
    for a, b in zip(py, nat):
        # the moving-average factor counts the updates exactly
        assert float(b[2][0]) == pytest.approx(float(a[2][0]), rel=1e-6), (a[2], b[2])
        for x, y in zip(a[:2], b[:2]):
            np.testing.assert_allclose(y, x, rtol=2e-2, atol=1e-3 * (np.abs(x).max() + 1e-6))


def test_native_caffemodel_io_matches_python(core_lib, tmp_path, monkeypatch):
    """sn_save_weights_to_file / sn_load_weights_from_file read and write .caffemodel files in
    C++ (protobuf wire format, Net::ToProto / CopyTrainedLayersFrom semantics, net.cpp:816-858)
    once the weights plan exists: no interpreter entry; the native file holds the same blobs as
    the Python writer's, each reader loads the other's file, legacy 4-D blob dims load, and
    shape / blob-count mismatches fail with Caffe's messages."""
    from sparknet_amd import proto
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_num_params.restype = C.c_longlong
    lib.sn_python_entries.restype = C.c_longlong
    st = C.c_void_p(lib.sn_create_state())
    buf, n = C.c_char_p(), C.c_int()
    assert lib.sn_parse_solver_prototxt(SOLVER.encode(), C.byref(buf), C.byref(n)) == 0
    assert lib.sn_set_device(st, -1) == 0
    assert lib.sn_load_solver_from_protobuf(st, buf, n) == 0, lib.sn_last_error()

    def fill(p, batch, nd, shape, user):
        cnt = int(np.prod([shape[i] for i in range(nd)]))
        arr = np.ctypeslib.as_array(p, shape=(cnt,))
        arr[:] = np.sin(0.07 * np.arange(cnt)).astype(np.float32) if nd == 4 else (np.arange(cnt) % 3)

    cb = CB(fill)
    assert lib.sn_set_train_data_callback(st, 0, cb, None) == 0
    assert lib.sn_set_train_data_callback(st, 1, cb, None) == 0
    assert lib.sn_solver_step(st, 2) == 0, lib.sn_last_error()
    nparam = lib.sn_num_params(st)
    w0 = (C.c_float * nparam)()
    assert lib.sn_get_weights(st, w0, C.c_longlong(nparam)) == 0  # builds the weights plan
    zeros = (C.c_float * nparam)()

    def weights():
        out = (C.c_float * nparam)()
        assert lib.sn_get_weights(st, out, C.c_longlong(nparam)) == 0
        return np.frombuffer(out, dtype=np.float32).copy()

    ref = np.frombuffer(w0, dtype=np.float32).copy()
    nat, py = str(tmp_path / "native.caffemodel"), str(tmp_path / "python.caffemodel")
    monkeypatch.setenv("SN_NATIVE_STEP", "1")
    e0 = lib.sn_python_entries()
    assert lib.sn_save_weights_to_file(st, nat.encode()) == 0, lib.sn_last_error()
    assert lib.sn_python_entries() == e0
    monkeypatch.setenv("SN_NATIVE_STEP", "0")
    assert lib.sn_save_weights_to_file(st, py.encode()) == 0, lib.sn_last_error()
    a, b = proto.read_net(nat), proto.read_net(py)
    blobs_b = {l.name: l.blobs for l in b.layer}
    assert [l.name for l in a.layer] == [l.name for l in b.layer]
    assert [l.type for l in a.layer] == [l.type for l in b.layer]
    checked = 0
    for la in a.layer:
        assert len(la.blobs) == len(blobs_b[la.name])
        for x, y in zip(la.blobs, blobs_b[la.name]):
            assert list(x.shape.dim) == list(y.shape.dim)
            np.testing.assert_array_equal(np.asarray(x.data, np.float32), np.asarray(y.data, np.float32))
            checked += 1
    assert checked >= 4
    # each reader loads the other's file
    for reader_native, path in ((True, py), (False, nat), (True, nat)):
        assert lib.sn_set_weights(st, zeros, C.c_longlong(nparam)) == 0
        monkeypatch.setenv("SN_NATIVE_STEP", "1" if reader_native else "0")
        e0 = lib.sn_python_entries()
        assert lib.sn_load_weights_from_file(st, path.encode()) == 0, lib.sn_last_error()
        if reader_native:
            assert lib.sn_python_entries() == e0
        np.testing.assert_array_equal(weights(), ref)
    monkeypatch.setenv("SN_NATIVE_STEP", "1")
    # legacy (num, channels, height, width) dims: the 4-D weights load; a 2-D blob pads to (1, 1, r, c)
    leg = proto.read_net(py)
    for layer in leg.layer:
        for bp in layer.blobs:
            dims = [1] * (4 - len(bp.shape.dim)) + list(bp.shape.dim)
            bp.ClearField("shape")
            bp.num, bp.channels, bp.height, bp.width = dims
    proto.write_binary(str(tmp_path / "legacy.caffemodel"), leg)
    assert lib.sn_set_weights(st, zeros, C.c_longlong(nparam)) == 0
    assert lib.sn_load_weights_from_file(st, str(tmp_path / "legacy.caffemodel").encode()) == 0, lib.sn_last_error()
    np.testing.assert_array_equal(weights(), ref)
    # mismatches: Caffe's messages
    bad = proto.read_net(py)
    lyr = next(l for l in bad.layer if len(l.blobs))
    lyr.blobs[0].shape.dim[0] += 1
    proto.write_binary(str(tmp_path / "bad_shape.caffemodel"), bad)
    assert lib.sn_load_weights_from_file(st, str(tmp_path / "bad_shape.caffemodel").encode()) != 0
    assert b"shape mismatch" in lib.sn_last_error() and lyr.name.encode() in lib.sn_last_error()
    bad = proto.read_net(py)
    lyr = next(l for l in bad.layer if len(l.blobs))
    del lyr.blobs[-1]
    proto.write_binary(str(tmp_path / "bad_count.caffemodel"), bad)
    assert lib.sn_load_weights_from_file(st, str(tmp_path / "bad_count.caffemodel").encode()) != 0
    assert b"Incompatible number of blobs" in lib.sn_last_error()
    (tmp_path / "trunc.caffemodel").write_bytes(open(py, "rb").read()[:-7])
    assert lib.sn_load_weights_from_file(st, str(tmp_path / "trunc.caffemodel").encode()) != 0
    lib.sn_free(buf)
    lib.sn_destroy_state(st)


@pytest.mark.parametrize("backend", ["lmdb", "sndb"])
def test_native_db_verbs_byte_equal_python(core_lib, tmp_path, monkeypatch, backend):
    """sn_create_db / sn_write_to_db / sn_commit_db_txn / sn_close_db write LMDB environments
    and sndb record files in C++ (no interpreter entry) that are byte-identical to the Python
    writers' (SN_NATIVE_STEP=0): explicit, automatic and duplicate keys, values past an LMDB
    page (overflow pages) and enough records for a two-level B+tree; sn_save_mean_image too."""
    from sparknet_amd.data.db import DatumReader
    lib = C.CDLL(core_lib)
    lib.sn_create_state.restype = C.c_void_p
    lib.sn_last_error.restype = C.c_char_p
    lib.sn_python_entries.restype = C.c_longlong
    st = C.c_void_p(lib.sn_create_state())
    rng = np.random.default_rng(7)
    recs = []
    for i in range(400):
        c, h, w = (3, 40, 40) if i % 97 == 5 else (3, 4, 4)  # 4800-byte images span overflow pages
        key = b"" if i % 5 == 0 else (b"k%05d" % (i % 350))       # auto keys, and duplicates of k00000..
        recs.append((rng.integers(0, 256, c * h * w, dtype=np.uint8).tobytes(), int(i % 10 - 2), c, h, w, key))
    out = {}
    for native in (True, False):
        monkeypatch.setenv("SN_NATIVE_STEP", "1" if native else "0")
        path = str(tmp_path / f"{backend}_{int(native)}")
        e0 = lib.sn_python_entries()
        assert lib.sn_create_db(st, path.encode(), backend.encode()) == 0, lib.sn_last_error()
        for i, (img, label, c, h, w, key) in enumerate(recs):
            assert lib.sn_write_to_db(st, img, label, c, h, w, key) == 0, lib.sn_last_error()
            if i % 150 == 149:
                assert lib.sn_commit_db_txn(st) == 0
        assert lib.sn_close_db(st) == 0, lib.sn_last_error()
        mean = np.linspace(-1, 1, 12, dtype=np.float32)
        mpath = path + ".mean.binaryproto"
        assert lib.sn_save_mean_image(mean.ctypes.data_as(C.POINTER(C.c_float)), 3, 2, 2, mpath.encode()) == 0
        if native:
            assert lib.sn_python_entries() == e0
        f = os.path.join(path, "data.mdb") if backend == "lmdb" else path
        out[native] = (open(f, "rb").read(), open(mpath, "rb").read())
        rd = DatumReader(path)
        assert len(rd) == (len({k for *_, k in recs if k} | {b"%08d" % i for i, r in enumerate(recs) if not r[5]})
                           if backend == "lmdb" else len(recs))
    assert out[True][0] == out[False][0]
    assert out[True][1] != b"" and out[True][1] == out[False][1]
    lib.sn_destroy_state(st)
