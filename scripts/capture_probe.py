"""Probe which multi-stream hipGraph capture patterns work on this ROCm build (each case
runs in its own subprocess so a crash is attributed)."""
import subprocess
import sys

CASES = {
    "fork_work_join": """
s=torch.cuda.Stream(); x=torch.ones(1024,device='cuda')
with torch.cuda.graph(g):
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s): x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
""",
    "fork_empty_join": """
s=torch.cuda.Stream(); x=torch.ones(1024,device='cuda')
with torch.cuda.graph(g):
    s.wait_stream(torch.cuda.current_stream())
    x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
""",
    "event_chain": """
s=torch.cuda.Stream(); x=torch.ones(1024,device='cuda'); y=torch.ones(1024,device='cuda')
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    x.add_(1); e=torch.cuda.Event(); e.record(m)
    with torch.cuda.stream(s): y.add_(1)
    s.wait_event(e)
    with torch.cuda.stream(s): y.add_(x)
    e2=torch.cuda.Event(); e2.record(s); m.wait_event(e2); x.add_(y)
    m.wait_stream(s)
""",
    "event_record_nowork": """
s=torch.cuda.Stream(); x=torch.ones(1024,device='cuda')
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    e=torch.cuda.Event(); e.record(s); m.wait_event(e); x.add_(1)
    m.wait_stream(s)
""",
    "alloc_on_side": """
s=torch.cuda.Stream(); x=torch.ones(1024,device='cuda')
with torch.cuda.graph(g):
    m=torch.cuda.current_stream(); s.wait_stream(m)
    with torch.cuda.stream(s):
        t=torch.empty(4096,device='cuda'); t.fill_(2); x.add_(t[:1024])
    m.wait_stream(s)
""",
    "four_streams": """
ss=[torch.cuda.Stream() for _ in range(3)]; xs=[torch.ones(1024,device='cuda') for _ in range(4)]
with torch.cuda.graph(g):
    m=torch.cuda.current_stream()
    for s in ss: s.wait_stream(m)
    xs[0].add_(1)
    for s,x in zip(ss,xs[1:]):
        with torch.cuda.stream(s): x.add_(1)
    for s in ss: m.wait_stream(s)
""",
}

if __name__ == "__main__":
    for name, body in CASES.items():
        code = ("import torch\ng=torch.cuda.CUDAGraph()\n" + body +
                "g.replay(); torch.cuda.synchronize(); print('ok')\n")
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        print(f"{name}: rc={r.returncode} {r.stdout.strip()} {r.stderr.strip().splitlines()[-1:] if r.returncode else ''}",
              flush=True)
