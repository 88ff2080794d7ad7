#!/bin/bash
# Memory-latency counters on one bench frame (kernel-trace PMC passes only)
TAG=${1:-pmc3}; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS" \
           "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ" \
           "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$TAG.p$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; grep -v "^W2026\|^    @" $R/gpurun_out/$TAG.p$i.log | tail -3; }
done
python $R/tools/pmc_sum.py $R/gpurun_out/$TAG
