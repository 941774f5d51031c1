"""Print the top kernels of a rocprofv3 kernel_stats.csv."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for r in rows[:n]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} tot%={float(r['Percentage']):6.2f}")
