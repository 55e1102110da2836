# Interleaved A/B of bench.py variants on one box: bash scripts/ab_bench.sh "<flags A>" "<flags B>" [rounds]
A="$1"; B="$2"; R="${3:-2}"
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  timeout -k 10 200 python bench.py $A > gpurun_out/ab_A_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $B > gpurun_out/ab_B_$i.log 2>&1 || exit 1
  echo "A[$A] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_A_$i.log)  B[$B] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_B_$i.log)"
done
