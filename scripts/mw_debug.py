"""Debug: the failing merge_runs case (float64, p = 2, random shape, desc=False)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import hpx_amd as hpx
from hpx_amd import segmented as S
from hpx_amd.compute import dtype_code
from oracle import oracle as O
from test_gpu_merge_sort import rnd, _merge_runs

tgt = hpx.target(0)
for dt in (np.float64, np.uint64):
    for p in (2,):
        rng = np.random.default_rng(p)
        lens = rng.integers(0, 300000, p)
        runs = [O.sort(np.asarray(rnd(dt, int(n), 10 + j), dt)) for j, n in enumerate(lens)]
        for lead in (3, 0, 4):
            got = _merge_runs(tgt, runs, dt, False, lead=lead)
            exp = O.sort(np.concatenate(runs))
            bad = np.nonzero(got.view(np.uint64) != exp.view(np.uint64))[0]
            print(dt.__name__, "lead", lead, "lens", lens, "mismatches", bad.size, flush=True)
            if bad.size:
                i = bad[0]
                print(" first", i, "last", bad[-1])
                print(" got", got[max(0, i - 3):i + 5])
                print(" exp", exp[max(0, i - 3):i + 5])
                print(" got bits", [hex(x) for x in got.view(np.uint64)[max(0, i - 3):i + 5]])
