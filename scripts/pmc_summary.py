"""Summarise rocprofv3 --pmc passes (counter_collection.csv per pass dir) into
per-kernel means.  usage: pmc_summary.py DIR [DIR ...]"""
import csv, glob, sys
from collections import defaultdict

acc = defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.replace("(anonymous namespace)::", "").replace("void ", "")
            short = short.split("(")[0].split("<")[0].split("::")[-1]
            acc[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, cname), v in sorted(acc.items()):
    if k.startswith("__amd") or k in ("k_generate", "k_fold", "k_write_init", "k_zero_count"):
        continue
    print(f"{k:22s} {cname:24s} dispatches={len(v):3d} mean={sum(v) / len(v):.5g}")
