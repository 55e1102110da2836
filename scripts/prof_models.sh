cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for m in vgg16 googlenet; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python3 bench.py --model $m --steps 6 --warmup 3 > gpurun_out/prof_$m.log 2>&1 || exit 1
  python scripts/prof_summary.py gpurun_out/prof_$m all > gpurun_out/prof_${m}_summary.txt 2>&1
done
timeout -k 10 200 python bench.py --model vgg16 --dtype fp8 --steps 20 --warmup 5 > gpurun_out/vgg_fp8.log 2>&1
timeout -k 10 200 python bench.py --model cifar10_quick --steps 200 --warmup 20 > gpurun_out/cq.log 2>&1
