"""Busy/idle analysis of a rocprofv3 kernel trace: union of kernel intervals."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1] + '/run_kernel_trace.csv')))
# restrict to the last bench step: kernels after the last k_finish but one
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
fin = [i for i, x in enumerate(iv) if 'k_finish' in x[2]]
if len(fin) >= 2:
    iv = iv[fin[-2] + 1: fin[-1] + 1]
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy = 0; cur_s, cur_e = iv[0][0], iv[0][1]
for s, e, _ in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s; cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1-t0)/1e6:.1f} ms, busy {busy/1e6:.1f} ms ({100*busy/(t1-t0):.1f}%)")
tot = collections.defaultdict(float); cnt = collections.Counter()
for s, e, n in iv:
    k = n.split('(')[0].replace('void ', '').replace('srr::dev::', '')
    tot[k] += (e - s) / 1e6; cnt[k] += 1
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]:
    print(f"  {k:40s} {v:8.1f} ms  x{cnt[k]}")
