#!/bin/bash
# RCCL rehearsal on one GPU: bench.py under torch.distributed.run --nproc-per-node 1 with SN_COMM_FORCE=1,
# so the nccl (RCCL) process group, broadcast, averaging all-reduces and comm diagnostics all run
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
SN_COMM_FORCE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 20 --warmup 5 --verify-average > gpurun_out/rccl1.json 2> gpurun_out/rccl1.err || { tail -30 gpurun_out/rccl1.err; exit 5; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/rccl1.json").read().splitlines() if l.startswith("{")][-1])
keep = {k: d.get(k) for k in ("value", "n_gpus", "rccl_world", "comm_backend", "average_buckets", "averages_in_window",
                               "allreduce_ms_per_average", "avg_payload_mb", "avg_check", "comm_bench")}
keep["diag"] = {k: v for k, v in d.get("diag", {}).items() if k != "rccl_log_rank0"}
keep["rccl_log_lines"] = (d.get("diag", {}).get("rccl_log_rank0") or "")[:600] if isinstance(d.get("diag", {}).get("rccl_log_rank0"), str) else d.get("diag", {}).get("rccl_log_rank0")
print(json.dumps(keep, indent=1))
PY
