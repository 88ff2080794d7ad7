#!/bin/bash
# PMC passes (kernel-trace only) on one bench frame; per-kernel sums via tools/pmc_sum.py
TAG=${1:-pmc2}; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES" \
           "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_TCP_LATENCY" \
           "TCC_HIT_sum TCC_MISS_sum" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/$TAG.p$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $R/gpurun_out/$TAG.p$i.log; exit 1; }
done
python $R/tools/pmc_sum.py $R/gpurun_out/$TAG
