# CaffeNet b256 bench.py at 1 / 2 / 3 / 4 branch streams, alternating, two reps (the default is 3)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/streams_cn.txt
for rep in 1 2; do for ns in 1 2 3 4; do
  timeout -k 10 200 python bench.py --model caffenet --streams $ns --steps 50 --warmup 10 2>/dev/null > gpurun_out/streams_one.json || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/streams_one.json').read().strip().splitlines()[-1]); print('streams', $ns, d['value'], d['ms_per_step'])" | tee -a gpurun_out/streams_cn.txt
done; done
