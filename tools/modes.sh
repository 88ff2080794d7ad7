#!/bin/bash
# per traversal mode: counted run (visits per ray) then timed run
TAG=${1:-modes}; shift
for m in "$@"; do
  SRR_TRAVERSAL=$m timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --count-visits > gpurun_out/$TAG.$m.count.log 2>&1 || { echo "count $m failed"; tail -3 gpurun_out/$TAG.$m.count.log; exit 1; }
  SRR_TRAVERSAL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.$m.log 2>&1 || { echo "bench $m failed"; exit 1; }
  python - "$m" gpurun_out/$TAG.$m.count.log gpurun_out/$TAG.$m.log <<'PY'
import json, sys
c = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
b = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
v = c["visits"]
print(f"{sys.argv[1]:10s} value {b['value']:8.1f} ms/step {b['ms_per_step']:7.1f} trace/launch {b['roofline']['trace_ms_per_launch']:.4f} "
      f"rays {b['config']['world_rays_per_step']} boxes/ray {v['box_tests_per_ray']:.2f} tris/ray {v['tri_tests_per_ray']:.2f} ovf {v['stack_overflows']}")
PY
done
