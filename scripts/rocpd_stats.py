"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db,
what rocprofv3 writes when no --output-format is given): calls, total and
mean duration per kernel name, the --stats summary's columns.
usage: python scripts/rocpd_stats.py DB [name-filter] [--csv]"""
import sqlite3
import sys

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                 f"from kernels group by {name} order by sum(end - start) desc").fetchall()
print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs")
for n, k, tot, avg, mn, mx in rows:
    if flt and flt not in n:
        continue
    short = n if len(n) < 140 else n[:137] + "..."
    print(f'"{short}",{k},{tot},{avg:.0f},{mn},{mx}')
