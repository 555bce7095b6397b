"""Summarise rocprofv3 --pmc counter_collection CSVs written by scripts/gpu_pmc.sh:
mean counter value per dispatch, per kernel and grid size (MB for *_SIZE counters, which
rocprofv3 reports in KB)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for path in sorted(glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            short = name.split("(")[0].replace("void ", "")[:60]
            grid = row.get("Grid_Size", "")
            acc[(row.get("Counter_Name", "?"), short, grid)].append(float(row.get("Counter_Value", "nan")))
    print(f"== {os.path.relpath(path, root)}")
    for (cn, k, g), xs in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
        mean = sum(xs) / len(xs)
        unit = f"{mean / 1024:10.2f} MB" if cn.endswith("_SIZE") else f"{mean:12.0f}"
        print(f"{cn:12s} {unit}  n={len(xs):4d}  grid={g:>9s}  {k}")
