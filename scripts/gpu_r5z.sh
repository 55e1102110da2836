#!/bin/bash
# distributed-path rehearsal on one GPU (gloo, ranks sharing the card): bench.py launched the
# way the driver launches the scaling runs, 2 and 4 ranks, with the cross-rank average check
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --share-gpu --steps 6 --warmup 2 --verify-average > gpurun_out/share$n.json 2> gpurun_out/share$n.err || { tail -30 gpurun_out/share$n.err; exit 5; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/share$n.json').read().strip().splitlines()[-1]); print($n, d['value'], d['n_gpus'], d['config']['parallelism'], d.get('avg_check'), d.get('averages_in_window'))"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_multirank_gpu.py -m gpu > gpurun_out/multirank.log 2>&1; rc=$?; tail -2 gpurun_out/multirank.log; exit $rc
