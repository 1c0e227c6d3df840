"""Timing of the segmented sort's merge step at 2^30 u64 keys per GPU (round
5): p sorted runs (p = 2, 4, 8) merged by one hpxhip_merge_runs call against
ceil(log2 p) rounds of pairwise hpxhip_merge, the form rounds 1-4 shipped.
Runs are random u64 keys sorted by the library; each result is checked
sorted on the device (hpxhip_unsorted_pairs).  Wall time around a device
synchronize, best of 5.

usage: python scripts/merge_runs_probe.py [log2 n]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import hpx_amd as hpx  # noqa: E402
from hpx_amd import _lib as L  # noqa: E402
from hpx_amd import execution as ex  # noqa: E402
from hpx_amd import parallel as P  # noqa: E402
from hpx_amd import segmented as S  # noqa: E402


def main():
    logn = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    n = 1 << logn
    tgt = hpx.target(0)
    pol = ex.par.on(hpx.default_executor(tgt))
    eng = S.HipEngine(tgt)
    src = hpx.vector(n, dtype=np.uint64, tgt=tgt)
    out = hpx.vector(n, dtype=np.uint64, tgt=tgt)
    tmp = hpx.vector(n, dtype=np.uint64, tgt=tgt)
    cnt = hpx.vector(1, dtype=np.uint64, tgt=tgt)
    P.generate(pol, src.begin(), src.end(), "bits", 3)
    print(f"{'p':>3} {'one pass ms':>12} {'pairwise ms':>12} {'GB/s one pass':>14}")
    for p in (2, 4, 8):
        offs = [n * j // p for j in range(p + 1)]
        for j in range(p):
            eng.sort(src, offs[j], offs[j + 1], False)
        tgt.synchronize()

        def one():
            eng.merge_runs(L.U64, src, 0, offs, out, 0, False)

        def pairwise():
            runs = [(offs[j], offs[j + 1] - offs[j]) for j in range(p)]
            a, i = src, 0
            while len(runs) > 1:
                b = (tmp, out)[i % 2]
                i += 1
                nxt = []
                for k in range(0, len(runs) - 1, 2):
                    (oa, na), (ob, nb) = runs[k], runs[k + 1]
                    eng.merge(L.U64, a, oa, na, a, ob, nb, b, oa, False)
                    nxt.append((oa, na + nb))
                if len(runs) % 2:
                    eng.copy(L.U64, a, runs[-1][0], runs[-1][1], b, runs[-1][0])
                    nxt.append(runs[-1])
                runs, a = nxt, b

        res = []
        for f in (one, pairwise):
            best = 1e9
            for _ in range(5):
                tgt.synchronize()
                t0 = time.perf_counter()
                f()
                tgt.synchronize()
                best = min(best, time.perf_counter() - t0)
            res.append(best * 1e3)
        one()
        L.call("hpxhip_unsorted_pairs", L.U64, ctypes.c_void_p(out.data()), n, 0, ctypes.c_void_p(cnt.data()),
               tgt.stream)
        bad = int(cnt.to_host()[0])
        print(f"{p:>3} {res[0]:12.3f} {res[1]:12.3f} {16.0 * n / res[0] / 1e6:14.1f}  unsorted pairs {bad}",
              flush=True)
        assert bad == 0 or os.environ.get("HPXHIP_PROBE_NOCHECK")
        P.generate(pol, src.begin(), src.end(), "bits", 3 + p)


if __name__ == "__main__":
    main()
