"""In-tree builder for the native parts of sparknet_amd.

Three shared libraries are produced inside the package (so they travel with the repo
snapshot to a GPU box and are what the Python processes load):

* ``sparknet_amd/lib/libsn_kernels.so`` — every ``csrc/kernels/*.hip`` file compiled by
  hipcc for gfx950 (MFMA GEMM / implicit-GEMM conv, pooling, LRN, dropout, softmax-loss,
  fused solver updates, data augmentation ...).  C ABI, launched through ctypes on
  torch's current HIP stream.
* ``sparknet_amd/lib/libsn_runtime.so`` — host C++ runtime (``csrc/runtime/*.cpp``):
  the native minibatch pipeline (mmap'd record sources, samplers, worker threads,
  pinned ring, async H2D copies).
* ``sparknet_amd/lib/libsn_core.so`` — the C ABI over the engine (``csrc/core``), the
  counterpart of SparkNet's libccaffe for C / C++ / JVM (JNA) hosts.

The builder is incremental (mtime based) and compiles translation units in parallel.
``python -m sparknet_amd.build_native`` or ``__graft_entry__.build()`` drive it.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "lib"
OBJDIR = ROOT / "build" / "obj"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("SN_OFFLOAD_ARCH", "gfx950")

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    f"-I{CSRC / 'kernels'}",
]
# host C++ runtime: g++ against the HIP runtime API (hipHostMalloc / hipMemcpyAsync /
# events); the HIP platform macro selects the AMD backend of the runtime headers.
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", f"-I{CSRC / 'runtime'}",
             "-D__HIP_PLATFORM_AMD__=1", f"-I{ROCM}/include"]
RUNTIME_LINK = [f"-L{ROCM}/lib", "-lamdhip64", f"-Wl,-rpath,{ROCM}/lib"]

KERNEL_LIB = LIBDIR / "libsn_kernels.so"
RUNTIME_LIB = LIBDIR / "libsn_runtime.so"
CORE_LIB = LIBDIR / "libsn_core.so"


def _python_flags() -> tuple[list[str], list[str]]:
    """Compile / link flags for embedding CPython (libsn_core)."""
    import sysconfig
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR") or "/usr/lib"
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    return [f"-I{inc}"], [f"-L{libdir}", f"-lpython{ver}", f"-Wl,-rpath,{libdir}", "-ldl"]


def _deps(src: Path) -> list[Path]:
    hdrs = [h for d in ("kernels", "runtime", "core") for h in (CSRC / d).glob("*.h")]
    return [src] + hdrs


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> subprocess.CompletedProcess:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _resources(stderr: str) -> dict:
    """{kernel symbol: {"vgpr", "agpr", "scratch", "vgpr_spill", "occupancy"}} from the
    compiler's kernel-resource-usage remarks (scratch > 0 = the kernel spills or keeps a
    private array in scratch memory — a register-pressure regression in a K-loop)."""
    out, cur = {}, None
    fields = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "VGPRs Spill": "vgpr_spill",
              "Occupancy [waves/SIMD]": "occupancy"}
    for line in stderr.splitlines():
        if "remark:" not in line or "kernel-resource-usage" not in line:
            continue
        body = line.split("remark:", 1)[1].rsplit("[-Rpass", 1)[0].strip()
        if body.startswith("Function Name:"):
            cur = body.split(":", 1)[1].strip()
            out[cur] = {}
        elif cur is not None and ":" in body:
            k, v = body.rsplit(":", 1)
            if k.strip() in fields:
                try:
                    out[cur][fields[k.strip()]] = int(v.strip())
                except ValueError:
                    pass
    return out


def _compile(src: Path, hip: bool, extra: list[str] | None = None) -> Path:
    obj = OBJDIR / (src.parent.name + "_" + src.stem + (".hip.o" if hip else ".cpp.o"))
    rep = obj.with_suffix(".resources.json")
    # a HIP object is rebuilt when its resource report is missing or older than it, so the
    # spill guard (tests/test_kernel_resources.py) always reads the report of the shipped code
    if _stale(obj, _deps(src)) or (hip and (not rep.exists() or rep.stat().st_mtime < obj.stat().st_mtime)):
        obj.parent.mkdir(parents=True, exist_ok=True)
        if hip:
            cmd = [HIPCC, *HIP_FLAGS, "-Rpass-analysis=kernel-resource-usage", "-c", str(src), "-o", str(obj)]
        else:
            cmd = ["g++", *CXX_FLAGS, *(extra or []), "-c", str(src), "-o", str(obj)]
        r = _run(cmd)
        if hip:  # per-kernel register / scratch report (tests/test_kernel_resources.py)
            rep.write_text(json.dumps(_resources(r.stderr), indent=0, sort_keys=True))
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> dict:
    """Compile and link both libraries; returns {name: path}."""
    if force and OBJDIR.exists():
        for f in OBJDIR.glob("*.o"):
            f.unlink()
    LIBDIR.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    cpp_srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    core_srcs = sorted((CSRC / "core").glob("*.cpp"))
    py_inc, py_link = _python_flags()
    with cf.ThreadPoolExecutor(jobs) as ex:
        hip_objs = list(ex.map(lambda s: _compile(s, True), hip_srcs))
        cpp_objs = list(ex.map(lambda s: _compile(s, False), cpp_srcs))
        core_objs = list(ex.map(lambda s: _compile(s, False, [*py_inc, f"-I{CSRC / 'core'}", "-D__HIP_PLATFORM_AMD__=1",
                                                              f"-I{ROCM}/include"]), core_srcs))
    out = {}
    if hip_objs:
        if force or _stale(KERNEL_LIB, hip_objs):
            _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, hip_objs),
                  "-o", str(KERNEL_LIB)])
        out["kernels"] = str(KERNEL_LIB)
    if cpp_objs:
        if force or _stale(RUNTIME_LIB, cpp_objs):
            _run(["g++", "-shared", "-fPIC", "-pthread", *map(str, cpp_objs), *RUNTIME_LINK, "-o",
                  str(RUNTIME_LIB)])
        out["runtime"] = str(RUNTIME_LIB)
    if core_objs:
        if force or _stale(CORE_LIB, core_objs):
            _run(["g++", "-shared", "-fPIC", "-pthread", *map(str, core_objs), *py_link, *RUNTIME_LINK, "-ldl",
                  "-o", str(CORE_LIB)])
        out["core"] = str(CORE_LIB)
    if verbose:
        print(out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
