"""Per-kernel summary of a rocprofv3 rocpd database (ROCm 7 default output):
    python scripts/dbstats.py <results.db> [N]  -> name, calls, total ms, avg us, % of kernel time."""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = c.execute(f"select {name}, count(*), sum(end-start) from kernels group by {name} order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':90s} {'calls':>8s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for n, k, t in rows[:top]:
    n = n if len(n) <= 88 else n[:85] + "..."
    print(f"{n:90s} {k:8d} {t / 1e6:10.3f} {t / k / 1e3:9.2f} {100 * t / tot:6.2f}")
print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")
