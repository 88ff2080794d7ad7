set -o pipefail
L=$PWD/simple-raytracing-render_amd
O=gpurun_out
for rep in 1 2 3; do
  for e in "run:X=0" "run2:SRR_LIB=$L/exp_run2.so" "prev:SRR_LIB=$L/exp_prev.so" "prev2:SRR_LIB=$L/exp_prev2.so"; do
    name=${e%%:*}; envs=${e#*:}
    env ${envs//;/ } timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/r4rep.$name.$rep.log 2>&1 || { echo "$name failed"; tail -3 $O/r4rep.$name.$rep.log; exit 1; }
    echo "$name rep $rep: $(grep -o '"value": [0-9.]*' $O/r4rep.$name.$rep.log)"
  done
done
