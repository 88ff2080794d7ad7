#!/bin/bash
# PMC passes on a short bench run (kernel-trace only, no sys/hip trace), via gpurun
TAG=${1:-pmc}
shift
ARGS="$@"
R=$PWD
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/$TAG.counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$TAG.p$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > $R/gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/$TAG.p$i.log; }
done
ls $R/gpurun_out/$TAG.p*/
