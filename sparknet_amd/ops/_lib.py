"""ctypes bindings of the native kernel library (``libsn_kernels.so``).

torch is imported first so that its HIP runtime (SONAME ``libamdhip64.so.7``) is the one
our library binds to — there is exactly one HIP runtime per process and our kernels
launch on torch's current stream (graph-capturable).

On a machine with a GPU the library MUST load: ``kernels()`` raises instead of silently
falling back to PyTorch ops.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_LIBDIR = Path(__file__).resolve().parent.parent / "lib"
# SN_DEBUG_SYNC=1: synchronise after every native launch and name the failing kernel
# (Caffe's CUDA_POST_KERNEL_CHECK under a blocking-launch debug mode)
DEBUG_SYNC = os.environ.get("SN_DEBUG_SYNC", "0") == "1"
_kern = None
_rt = None


class SnConvGeom(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("N", "H", "W", "C", "P", "Q", "R", "S", "sh", "sw", "ph", "pw", "dh", "dw", "Cg")]


class SnOperand(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("ld", C.c_longlong), ("gstride", C.c_longlong),
                ("g", SnConvGeom)]


class SnGemmArgs(C.Structure):
    _fields_ = [("M", C.c_int), ("N", C.c_int), ("K", C.c_int),
                ("groups", C.c_int), ("splits", C.c_int), ("kchunk", C.c_int),
                ("a_mc", C.c_int), ("a_mode", C.c_int), ("b_mc", C.c_int), ("b_mode", C.c_int),
                ("epi", C.c_int),
                ("A", SnOperand), ("B", SnOperand),
                ("C", C.c_void_p), ("ldc", C.c_longlong), ("c_gstride", C.c_longlong),
                ("c_split_stride", C.c_longlong),
                ("bias", C.c_void_p), ("relu", C.c_int), ("tile", C.c_int), ("gate", C.c_void_p),
                ("fp8", C.c_int), ("deq_a", C.c_void_p), ("deq_b", C.c_void_p), ("raster_n", C.c_int),
                ("ones_col", C.c_int), ("bias_out", C.c_void_p), ("bias_acc", C.c_int),
                ("sgd_w", C.c_void_p), ("sgd_h", C.c_void_p), ("sgd_shadow", C.c_void_p), ("sgd_hyper", C.c_void_p),
                ("sgd_lr_mult", C.c_float), ("sgd_decay_mult", C.c_float), ("sgd_flags", C.c_int),
                ("drop_rng", C.c_void_p), ("drop_stream", C.c_int), ("drop_thr", C.c_uint),
                ("drop_scale", C.c_float), ("gate_scale", C.c_float), ("lds_store", C.c_int),
                ("q_out", C.c_void_p), ("q_ld", C.c_longlong), ("q_gstride", C.c_longlong), ("q_slot", C.c_void_p),
                ("q_e5m2", C.c_int), ("q_part", C.c_void_p)]


def lib_path(name: str = "libsn_kernels.so") -> Path:
    if name == "libsn_kernels.so" and os.environ.get("SN_KERNEL_LIB"):  # A/B of two kernel builds
        return Path(os.environ["SN_KERNEL_LIB"])
    return _LIBDIR / name


def available() -> bool:
    return lib_path().exists()


def kernels():
    """Load (once) and return the kernel library.  Builds it if missing."""
    global _kern
    if _kern is None:
        p = lib_path()
        if not p.exists():
            from .. import build_native
            build_native.build()
        _kern = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
        _kern.sn_gemm.argtypes = [C.POINTER(SnGemmArgs), C.c_void_p]
        _kern.sn_gemm.restype = C.c_int
    return _kern


def runtime():
    global _rt
    if _rt is None:
        p = lib_path("libsn_runtime.so")
        if not p.exists():
            from .. import build_native
            build_native.build()
        _rt = C.CDLL(str(p))
    return _rt


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"sparknet_amd kernel '{what}' failed with code {rc}")


def call(name: str, *args):
    """Call ``sn_<name>(..., stream)`` with ctypes-converted args on the current stream."""
    fn = getattr(kernels(), "sn_" + name)
    conv = []
    for a in args:
        if isinstance(a, torch.Tensor):
            conv.append(C.c_void_p(a.data_ptr()))
        elif a is None:
            conv.append(C.c_void_p(0))
        elif isinstance(a, bool):
            conv.append(C.c_int(int(a)))
        elif isinstance(a, int):
            conv.append(C.c_longlong(a))
        elif isinstance(a, float):
            conv.append(C.c_float(a))
        else:
            conv.append(a)
    conv.append(C.c_void_p(stream_ptr()))
    fn.restype = C.c_int
    check(fn(*conv), name)
    if DEBUG_SYNC:
        debug_sync(name)


def debug_sync(name: str) -> None:
    try:
        torch.cuda.synchronize()
    except RuntimeError as e:  # a fault inside the kernel surfaces here
        raise RuntimeError(f"sparknet_amd kernel '{name}' faulted: {e}") from e


def loaded_libraries() -> list[str]:
    """Which sparknet native libraries are mapped into this process (for diagnostics)."""
    out = []
    try:
        with open(f"/proc/{os.getpid()}/maps") as f:
            for line in f:
                if "libsn_" in line or "libamdhip64" in line:
                    path = line.split()[-1]
                    if path not in out:
                        out.append(path)
    except OSError:
        pass
    return out
