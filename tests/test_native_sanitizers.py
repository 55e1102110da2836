"""Sanitizer builds of the native host runtime: the loader's worker / ring
protocol (csrc/runtime/loader.cpp) is compiled with ThreadSanitizer and with
AddressSanitizer + UBSan into a host-only stress driver (tests/native/loader_stress.cpp,
unpinned ring, 1-8 worker threads, all samplers, early destroy) that must run clean."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_loader_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    exe = tmp_path / ("loader_" + san.split(",")[0])
    cmd = ["g++", "-std=c++17", "-g", "-O1", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-Werror=unused-result",
           "-D__HIP_PLATFORM_AMD__=1", f"-I{ROCM}/include", os.path.join(ROOT, "csrc/runtime/loader.cpp"),
           os.path.join(ROOT, "tests/native/loader_stress.cpp"), f"-L{ROCM}/lib", "-lamdhip64",
           f"-Wl,-rpath,{ROCM}/lib", "-pthread", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    if "ThreadSanitizer: unexpected memory mapping" in r.stderr:
        # TSan's shadow layout does not accept this host's address-space layout (high-entropy
        # mmap randomisation, or another runtime preloaded into the process): an environment
        # limit, not a finding
        pytest.skip("ThreadSanitizer cannot map its shadow memory on this host")
    assert r.returncode == 0 and "bad=0" in r.stdout, (r.stdout[-1000:], r.stderr[-3000:])
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
