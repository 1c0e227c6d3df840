"""GPU half of the k_mw_merge miscompile reproducer (round 6; the libraries
come from scripts/diag/mw_repro_build.sh): lease r5/ad's failing case --
float64 keys, p = 2 runs of random lengths (numpy default_rng(2)), standard
normals with zeros of both signs, ascending -- and p = 3 / 8, through the
commit-8a18d38 merge built at the default bound and at 8 waves per SIMD,
and through the shipped library and its variant builds.  Prints the
mismatch count per build and dtype; a key written in its ordered-bit form
shows as ~bits of the expected key (negative doubles)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import hpx_amd as hpx  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_merge_sort import merge_runs_with, rnd  # noqa: E402

tgt = hpx.target(0)
libs = {"r05_8a18d38_default": "scripts/diag/mw_old/default/libhpxhip.so",
        "r05_8a18d38_minw8": "scripts/diag/mw_old/minw8/libhpxhip.so",
        "shipped": "hpx_amd/libhpxhip.so",
        "variant_mw512": "hpx_amd/variants/mw512/libhpxhip.so",
        "variant_mwminw4": "hpx_amd/variants/mwminw4/libhpxhip.so"}
bad_total = {}
for name, rel in libs.items():
    path = os.path.join(ROOT, rel)
    for dt in (np.float64, np.uint64, np.int32):
        for p in (2, 3, 8):
            rng = np.random.default_rng(p)
            lens = rng.integers(0, 300000, p)
            runs = [O.sort(np.asarray(rnd(dt, int(n), 10 + j), dt)) for j, n in enumerate(lens)]
            got = merge_runs_with(path, tgt, runs, dt, False)
            exp = O.sort(np.concatenate(runs))
            ub = np.uint64 if np.dtype(dt).itemsize == 8 else np.uint32
            bad = np.nonzero(got.view(ub) != exp.view(ub))[0]
            msg = f"{name:22s} {np.dtype(dt).name:8s} p={p} n={int(lens.sum()):7d} mismatches={bad.size}"
            if bad.size:
                i = bad[0]
                g, e = got.view(ub)[i], exp.view(ub)[i]
                msg += f" first={i} got={got[i]!r} exp={exp[i]!r} got==~exp:{bool(g == ~e)}"
                flip = np.count_nonzero(got.view(ub)[bad] == ~exp.view(ub)[bad])
                msg += f" (~exp at {flip}/{bad.size})"
            print(msg, flush=True)
            bad_total[name] = bad_total.get(name, 0) + int(bad.size)
print("summary", bad_total, flush=True)
# the shipped library and its variants must be exact; the old builds are the evidence
sys.exit(1 if any(bad_total[k] for k in ("shipped", "variant_mw512", "variant_mwminw4")) else 0)
