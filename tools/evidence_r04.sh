#!/bin/bash
# Round-4 evidence on one GPU box (run via gpurun from the repo root), in stages:
#   bash tools/evidence_r04.sh counters   -> gpurun_out/r04cnt_<cfg>.json  (tools/counters.sh per config)
#   bash tools/evidence_r04.sh final      -> GPU tests, smoke(), default bench line (cpu_baseline),
#                                            rocprofv3 --kernel-trace --stats of the same command
#   bash tools/evidence_r04.sh configs    -> every config's bench line (tools/configs.sh)
set -o pipefail
R=$PWD; O=$R/gpurun_out
case "$1" in
  counters)
    # the frames are cut to 256 spp where a full one takes seconds: counters.py records the
    # profiled frame's world rays, and bench.py prices the counts per world ray
    shift
    want=" $* "  # optional subset of config tags
    while read -r tag args; do
      [ -z "$tag" ] && continue
      [ "$want" != "  " ] && [[ "$want" != *" $tag "* ]] && continue
      bash tools/counters.sh r04cnt_$tag $args > $O/r04cnt_$tag.log 2>&1 || { echo "counters $tag failed"; tail -5 $O/r04cnt_$tag.log; exit 1; }
      echo "$tag: $(python -c "import json; d=json.load(open('$O/r04cnt_$tag.json')); print(d['ms_per_launch_profiled'], 'ms', d.get('valu_lane_utilisation'), 'lanes', d['hbm']['total_bytes'], 'B', d['world_rays_per_launch'], 'rays')")"
    done <<'CFG'
s2 --scene s2
s1 --scene s1
s3 --scene s3
s3_metal --scene s3_metal
s4 --scene s4 --spp 256
s5 --scene s5 --spp 256
s2_d100 --scene s2 --divs 100
s4_real --scene s4_real --spp 256
CFG
    ;;
  final)
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/r04final.tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -1 $O/r04final.tests.log; [ $rc -eq 0 ] || exit 1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04final.smoke.log 2>&1 || { tail -5 $O/r04final.smoke.log; exit 1; }
    tail -1 $O/r04final.smoke.log
    timeout -k 10 600 python bench.py > $O/r04final.bench.log 2>&1 || { tail -5 $O/r04final.bench.log; exit 1; }
    grep '^{' $O/r04final.bench.log | cut -c1-200
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04final.prof -o run --output-format csv -- \
      python $R/bench.py --no-cpu-baseline > $O/r04final.prof.log 2>&1 || { tail -5 $O/r04final.prof.log; exit 1; }
    grep '^{' $O/r04final.prof.log | cut -c1-200
    python $R/tools/stats.py $O/r04final.prof
    ;;
  configs)
    bash tools/configs.sh
    ;;
  *) echo "usage: $0 counters|final|configs"; exit 2;;
esac
