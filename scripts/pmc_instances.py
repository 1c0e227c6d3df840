"""Per-instance PMC values from rocprofv3 rocpd databases (run_results.db):
rocpd keeps one pmc_events row per counter instance (TCC: 16 channels x 8
XCDs = 128 rows per dispatch).  For every dispatch of kernels matching a
filter: duration, the total, and the spread over the instances (min / max /
coefficient of variation, and the per-XCD sums).
usage: python scripts/pmc_instances.py FILTER DB [DB ...]"""
import sqlite3
import sys

import numpy as np

flt = sys.argv[1]
for db in sys.argv[2:]:
    c = sqlite3.connect(db)
    rows = c.execute("select event_id, name, duration, counter_name, counter_value from pmc_events order by id").fetchall()
    by = {}
    for ev, name, dur, cn, v in rows:
        if flt in name:
            by.setdefault((ev, cn), [name, dur, []])[2].append(v)
    print(f"# {db}")
    for (ev, cn), (name, dur, vals) in sorted(by.items()):
        a = np.array(vals)
        line = (f"  dispatch {ev:4d} {cn:16s} {dur / 1e6:7.3f} ms  n={a.size:3d} total={a.sum():.4g} "
                f"min={a.min():.4g} max={a.max():.4g} cv={a.std() / a.mean() if a.mean() else 0:.4f}")
        if a.size == 128:
            x = a.reshape(8, 16) if True else a
            xs = x.sum(axis=1)
            line += f" xcd_cv={xs.std() / xs.mean():.4f} chan_max/mean={(x / x.mean(axis=1, keepdims=True)).max():.3f}"
        print(line)
