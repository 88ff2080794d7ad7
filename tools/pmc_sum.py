"""Per-kernel sums of rocprofv3 --pmc passes: python tools/pmc_sum.py PREFIX"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + ".p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("srr::dev::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:6]:
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:34s} {x:14.4g}")
