#!/bin/bash
# Issue / occupancy / wait / instruction-mix / HBM counters for k_paths on one
# bench frame: one rocprofv3 --pmc pass per counter group (kernel trace only),
# then tools/counters.py reduces them to profiles-ready JSON.
#   bash tools/counters.sh TAG [bench.py args...]     (run on the GPU box)
TAG=${1:-cnt}; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/gpurun_out/$TAG.p$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; grep -v "^W2026\|^    @" $R/gpurun_out/$TAG.p$i.log | tail -3; exit 1; }
done
cd $R && python tools/counters.py gpurun_out/$TAG k_paths > gpurun_out/$TAG.json && cat gpurun_out/$TAG.json
