#!/bin/bash
# same-box step traces, packed conv1 on / off, and the host-side cost of a step
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for v in 0 1; do
  rm -rf gpurun_out/prof_pk$v
  SN_CONV_PACKED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pk$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_pk$v.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_pk$v.log; exit 5; }
  python3 scripts/prof_summary.py gpurun_out/prof_pk$v > gpurun_out/prof_pk${v}_summary.txt 2>&1
  echo "packed=$v: $(tail -1 gpurun_out/prof_pk${v}_summary.txt) bench-under-trace: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_pk$v.log)"
done
timeout -k 10 300 python -u bench.py --host-profile > gpurun_out/hostprof.jsonl 2> gpurun_out/hostprof.err || { tail -5 gpurun_out/hostprof.err; exit 4; }
grep "us/step" gpurun_out/hostprof.err
