"""Per-kernel durations of bench.py's timed step, from a rocprofv3
--kernel-trace of the bench (run_kernel_trace.csv).

The --stats summary averages every launch of a kernel in the process; the
step's triad shares its kernel (k_binary with the triad functor) with the
STREAM row's triad, which runs later on freshly allocated arrays.  This
script takes the launches in dispatch order and keeps the step's: the first
warmup + steps launches of each step kernel (triad, transform_reduce,
inclusive_scan), of which the last `steps` are the timed ones -- the launches
behind bench.py's kernels_ms and roofline.achieved.

usage: python scripts/step_kernel_stats.py TRACE_CSV [--warmup 3] [--steps 10]
"""
import argparse
import csv
import statistics

STEP_KERNELS = (
    ("triad", lambda name: name.startswith("void (anonymous namespace)::k_binary<double, double, double, "
                                           "hpxhip::binary_fn<1, double>")),
    ("transform_reduce", lambda name: "k_reduce<" in name and "long" in name and "k_reduce_partials" not in name),
    ("inclusive_scan", lambda name: "k_scan<long" in name),
)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for label, match in STEP_KERNELS:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if match(r["Kernel_Name"])]
        step = d[:a.warmup + a.steps]
        timed = step[a.warmup:]
        if not timed:
            print(f"{label:18s} no launches matched")
            continue
        print(f"{label:18s} launches {len(d):3d}  timed step launches {len(timed):2d}: mean {statistics.mean(timed):.4f} ms"
              f"  min {min(timed):.4f}  max {max(timed):.4f}   (all launches of the kernel: mean "
              f"{statistics.mean(d):.4f} ms)")


if __name__ == "__main__":
    main()
