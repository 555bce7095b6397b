"""Print a rocprofv3 kernel_stats.csv as 'name calls avg_us total_ms' rows (top 14)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    name = r["Name"].split("(")[0][-48:]
    print(f"{name:48s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us {float(r['TotalDurationNs']) / 1e6:9.3f} ms")
