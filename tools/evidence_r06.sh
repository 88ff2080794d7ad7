#!/bin/bash
# Round-6 evidence on one GPU box (run via gpurun from the repo root), in stages:
#   bash tools/evidence_r06.sh counters [cfg..] -> gpurun_out/r06cnt_<cfg>.json (tools/counters_all.sh)
#   bash tools/evidence_r06.sh configs          -> every config's bench line (tools/configs.sh -> r06cfg.jsonl)
#   bash tools/evidence_r06.sh final            -> GPU tests, smoke(), default bench line (cpu_baseline),
#                                                  rocprofv3 --kernel-trace --stats of the same command
#   bash tools/evidence_r06.sh phases           -> k_paths phase timing per config (diagnostics build)
#   bash tools/evidence_r06.sh multi            -> shard balance (two frames in flight), the C-ABI
#                                                  multi-device bench rehearsed on one GPU, the wavefront engine
set -o pipefail
R=$PWD; O=$R/gpurun_out
case "$1" in
  counters)
    shift
    bash tools/counters_all.sh r06cnt "$@"
    ;;
  configs)
    bash tools/configs.sh r06cfg
    ;;
  final)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/r06final.tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -1 $O/r06final.tests.log; [ $rc -eq 0 ] || exit 1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06final.smoke.log 2>&1 || { tail -5 $O/r06final.smoke.log; exit 1; }
    tail -1 $O/r06final.smoke.log
    timeout -k 10 600 python bench.py > $O/r06final.bench.log 2>&1 || { tail -5 $O/r06final.bench.log; exit 1; }
    grep '^{' $O/r06final.bench.log | cut -c1-200
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r06final.prof -o run --output-format csv -- \
      python $R/bench.py --no-cpu-baseline > $O/r06final.prof.log 2>&1 || { tail -5 $O/r06final.prof.log; exit 1; }
    grep '^{' $O/r06final.prof.log | cut -c1-200
    python $R/tools/stats.py $O/r06final.prof
    ;;
  phases)
    shift
    bash tools/phases.sh r06ph ${@:-c2 c3 c4 c5 c4r}
    ;;
  multi)
    timeout -k 10 600 python tools/shard_balance.py --scene s2 --tile 1 --pipeline 8 > $O/r06sb_s2.json 2> $O/r06sb_s2.log || { tail -3 $O/r06sb_s2.log; exit 1; }
    tail -1 $O/r06sb_s2.json | cut -c1-300
    timeout -k 10 600 python tools/shard_balance.py --scene s4 --tile 1 --pipeline 3 > $O/r06sb_s4.json 2> $O/r06sb_s4.log || { tail -3 $O/r06sb_s4.log; exit 1; }
    tail -1 $O/r06sb_s4.json | cut -c1-300
    timeout -k 10 300 python bench.py --host capi --gpus 3 --rehearse --steps 3 --no-cpu-baseline > $O/r06capi3.log 2>&1 || { tail -3 $O/r06capi3.log; exit 1; }
    grep '^{' $O/r06capi3.log | cut -c1-200
    for sc in s2 s4_real; do
      SRR_ENGINE=wave timeout -k 10 600 python bench.py --scene $sc --no-pipeline --no-cpu-baseline --steps 1 --warmup 1 > $O/r06wave_$sc.log 2>&1 || { tail -3 $O/r06wave_$sc.log; exit 1; }
      grep '^{' $O/r06wave_$sc.log | cut -c1-200
    done
    ;;
  *) echo "usage: $0 counters|configs|final|phases|multi"; exit 2;;
esac
