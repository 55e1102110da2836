"""Second capture probe: which node kinds on a forked side stream break hipStreamEndCapture.
Stops at the first failing case (a crash ends the GPU work of the call)."""
import subprocess
import sys

PRE = ("import sys, os; sys.path.insert(0, os.getcwd())\nimport torch\nfrom sparknet_amd.ops import hip\n"
       "g=torch.cuda.CUDAGraph(); s=torch.cuda.Stream()\n"
       "x=torch.randn(4096,device='cuda').bfloat16(); y=torch.empty_like(x)\n"
       "hip.relu_forward(x); torch.cuda.synchronize()\n")
CASES = {
    "sn_kernel_side": """
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    with torch.cuda.stream(s): z=hip.relu_forward(x)
    m.wait_stream(s)
""",
    "memcpy_side": """
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    with torch.cuda.stream(s): y.copy_(x)
    m.wait_stream(s)
""",
    "memcpy_side_after_main": """
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); x.add_(1); e=torch.cuda.Event(); e.record(m); s.wait_event(e)
    with torch.cuda.stream(s): y.copy_(x)
    e2=torch.cuda.Event(); e2.record(s); m.wait_event(e2); x.add_(y)
""",
    "memset_side": """
import ctypes
rt=ctypes.CDLL('libamdhip64.so')
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    rc=rt.hipMemsetAsync(ctypes.c_void_p(y.data_ptr()), 0, ctypes.c_size_t(8192), ctypes.c_void_p(s.cuda_stream))
    m.wait_stream(s)
""",
    "side_only_first_node": """
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    with torch.cuda.stream(s): z=hip.relu_forward(x); w=hip.relu_forward(z)
    e=torch.cuda.Event(); e.record(s); m.wait_event(e); u=hip.relu_forward(w)
""",
}

if __name__ == "__main__":
    for name, body in CASES.items():
        code = PRE + body + "g.replay(); torch.cuda.synchronize(); print('ok')\n"
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        tail = r.stderr.strip().splitlines()[-2:] if r.returncode else ""
        print(f"{name}: rc={r.returncode} {r.stdout.strip()} {tail}", flush=True)
        if r.returncode:
            break
