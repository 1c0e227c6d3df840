"""Summarise rocprofv3 --pmc passes (counter_collection.csv per pass dir) into
per-kernel means and maxima (one row per template instantiation).
usage: pmc_summary.py DIR [DIR ...]"""
import csv, glob, sys, zlib
from collections import defaultdict

acc = defaultdict(list)
args = {}
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.replace("(anonymous namespace)::", "").replace("void ", "")
            full = short.split("(")[0]
            short = full.split("<")[0].split("::")[-1]
            # instantiations are told apart by their template arguments
            # (e.g. the 9-bit and the byte onesweep pass, plain and
            # persistent grids): short name + a tag of the argument list
            tag = format(zlib.crc32(full.encode()) % 4096, "03x") if "<" in full else ""
            acc[(short, tag, r["Counter_Name"])].append(float(r["Counter_Value"]))
            args.setdefault((short, tag), full[len(full.split("<")[0]):][:160])
for (k, tag, cname), v in sorted(acc.items()):
    if k.startswith("__amd") or k in ("k_generate", "k_fold", "k_write_init", "k_zero_count"):
        continue
    print(f"{k + (' #' + tag if tag else ''):28s} {cname:24s} dispatches={len(v):3d} mean={sum(v) / len(v):.5g} "
          f"max={max(v):.5g}")
print()
for (k, tag), a in sorted(args.items()):
    if tag:
        print(f"#{tag} {k}{a}")
