#!/bin/bash
# Texture-address / L1 (TA, TCP) counters of k_paths, one rocprofv3 --pmc pass per group
# (kernel trace only): is the vector-memory pipe the walk's limit?
#   bash tools/pmc_ta.sh TAG [bench.py args...]     (run on the GPU box)
TAG=${1:-ta}; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TA_TA_BUSY TA_TOTAL_WAVEFRONTS GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES" \
           "TCP_TOTAL_ACCESSES TCP_CACHE_MISS TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" \
           "TCP_TCP_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/$TAG.p$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/$TAG.p$i.log; exit 1; }
done
cd $R && python tools/counters.py gpurun_out/$TAG k_paths > gpurun_out/$TAG.json 2>&1; cat gpurun_out/$TAG.json | head -40
