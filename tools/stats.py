import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
for r in rows[:9]:
    n = r['Name']
    n = n.split('(')[0].replace('void ', '').replace('srr::dev::', '')
    print(f"{n:28s} calls={r['Calls']:>6s} total_ms={int(r['TotalDurationNs'])/1e6:8.2f} avg_us={float(r['AverageNs'])/1e3:8.1f} {float(r['Percentage']):5.1f}%")
