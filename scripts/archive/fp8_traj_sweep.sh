set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "--lr 0.002 --noise 0.5 --steps 300 --window 30" "--lr 0.001 --noise 0.5 --steps 400 --window 40"; do
  echo "== $cfg"
  timeout -k 10 500 python -u scripts/fp8_trajectory.py $cfg 2>gpurun_out/fp8_trajectory.err | tee -a gpurun_out/fp8_trajectory2.txt || { echo "trajectory failed"; tail -20 gpurun_out/fp8_trajectory.err; exit 1; }
done
