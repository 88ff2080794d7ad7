set -o pipefail
for rep in 1 2; do
for e in "X=0" "SRR_BIGBLOCK=0"; do
  for m in "" "--no-pipeline"; do
    env $e timeout -k 10 120 python bench.py --no-cpu-baseline --scene s1 --steps 30 --warmup 3 $m > gpurun_out/c1bb.log 2>&1 || { tail -3 gpurun_out/c1bb.log; exit 1; }
    echo "$e $m rep $rep: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"trace_ms_per_launch": [0-9.]*' gpurun_out/c1bb.log | tr '\n' ' ')"
  done
done
done
