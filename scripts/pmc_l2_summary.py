"""L2 (TCC) hit rate per kernel from rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum counter CSVs:
    python scripts/pmc_l2_summary.py <dir> [<dir> ...]"""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    agg = defaultdict(lambda: defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", r.get("Kernel-Name", "?")).split("(")[0][-40:]
            cn = r.get("Counter_Name", r.get("Counter-Name"))
            agg[name][cn] += float(r.get("Counter_Value", r.get("Counter-Value", 0)))
    print(f"== {d}")
    for name, c in sorted(agg.items(), key=lambda kv: -(kv[1]["TCC_HIT_sum"] + kv[1]["TCC_MISS_sum"])):
        h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
        if h + m > 0:
            print(f"  {name:40s} hit {100 * h / (h + m):5.1f} %  (hits {h:.3g}, misses {m:.3g})")
