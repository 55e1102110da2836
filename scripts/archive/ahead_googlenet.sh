set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
  for d in 2 3 4 0; do
    SN_MAX_AHEAD=$d timeout -k 10 300 python bench.py --model googlenet --steps 30 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('googlenet max_ahead $d', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
for d in 2 3; do
  SN_MAX_AHEAD=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('caffenet max_ahead $d', d['value'], d['ms_per_step'], flush=True)" || exit 1
done
