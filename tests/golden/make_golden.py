"""Generate the golden fixtures under tests/golden/ from the CLOSED FORMS and
data recipes written in the reference's own known-answer tests.

The expected outputs here are computed by the formulas the reference tests
assert (not by the oracle), so that tests/test_oracle_golden.py pins the
oracle against an independent statement, and the GPU parity tests pin the
kernels against the same vectors.  Randomised reference tests (seeded at run
time there) are instantiated with a fixed seed recorded in index.json.

Run:  python tests/golden/make_golden.py   (writes *.npz + index.json)
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MASK64 = (1 << 64) - 1


def tri(n):
    # exclusive_scan_validate.cpp:37-39 check_n_triangle
    return 0 if n < 0 else n * (n + 1) // 2


def main():
    index = []

    def save(name, meta, **arrays):
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        meta = dict(meta, name=name, file=name + ".npz")
        index.append(meta)

    # --- exclusive_scan_validate.cpp:46-131 (INITIAL_VAL 50, ARRAY_SIZE 10000, FILL_VALUE 10)
    n = 10000
    a = np.arange(0, n, dtype=np.int32)
    save("exclusive_scan_validate_count0",
         {"ref": "tests/unit/parallel/algorithms/exclusive_scan_validate.cpp:53-72",
          "algo": "exclusive_scan", "dtype": "int32", "init": 50, "op": "plus",
          "in_place_too": True},
         input=a, expected=np.array([50 + tri(i - 1) for i in range(n)], np.int32))
    a = np.arange(1, n, dtype=np.int32)  # counting_iterator(1) .. (ARRAY_SIZE): 9999 elements
    save("exclusive_scan_validate_count1",
         {"ref": "tests/unit/parallel/algorithms/exclusive_scan_validate.cpp:75-102",
          "algo": "exclusive_scan", "dtype": "int32", "init": 50, "op": "plus", "in_place_too": True},
         input=a, expected=np.array([50 + tri(i) for i in range(a.size)], np.int32))
    a = np.full(n, 10, np.int32)
    save("exclusive_scan_validate_const",
         {"ref": "tests/unit/parallel/algorithms/exclusive_scan_validate.cpp:104-131",
          "algo": "exclusive_scan", "dtype": "int32", "init": 50, "op": "plus", "in_place_too": True},
         input=a, expected=np.array([50 + 10 * i for i in range(n)], np.int32))

    # --- inclusive_scan_tests.hpp:63-88 test_inclusive_scan1: 10007 x size_t(1), init 0
    c = np.ones(10007, np.uint64)
    save("inclusive_scan1",
         {"ref": "tests/unit/parallel/algorithms/inclusive_scan_tests.hpp:63-88",
          "algo": "inclusive_scan", "dtype": "uint64", "init": 0, "op": "plus"},
         input=c, expected=np.arange(1, 10008, dtype=np.uint64))

    # --- inclusive_scan_tests.hpp:26-60 benchmark: doubles all 1.0, std::equal (bit-exact);
    #     the reference uses 1e8 elements, the fixture stores the closed form at 2^16
    m = 1 << 16
    save("inclusive_scan_benchmark_ones",
         {"ref": "tests/unit/parallel/algorithms/inclusive_scan_tests.hpp:26-60",
          "algo": "inclusive_scan", "dtype": "float64", "init": 0.0, "op": "plus",
          "note": "reference size 1e8; closed form out[i] = i + 1"},
         input=np.ones(m, np.float64), expected=np.arange(1, m + 1, dtype=np.float64))

    # --- copyif_random.cpp:27-63: first half iota(dis(gen)), second half -1, pred !(i<0)
    rng = np.random.default_rng(0xC0FF1F)
    start = int(rng.integers(0, 2**31 - 1 - 10007))
    c = np.empty(10007, np.int32)
    half = c.size // 2
    c[:half] = np.arange(start, start + half, dtype=np.int64).astype(np.int32)
    c[half:] = -1
    save("copyif_random",
         {"ref": "tests/unit/parallel/algorithms/copyif_random.cpp:27-63",
          "algo": "copy_if", "dtype": "int32", "pred": "not_less_than", "arg": 0, "seed_start": start},
         input=c, expected=c[:half].copy())

    # --- partitioned_vector_reduce.cpp:47-76: 10007 x T(1), init T(1), plus -> T(num + 1)
    for dt in ("int32", "float64"):
        save(f"partitioned_vector_reduce_{dt}",
             {"ref": "tests/unit/parallel/segmented_algorithms/partitioned_vector_reduce.cpp:47-76",
              "algo": "reduce", "dtype": dt, "init": 1, "op": "plus", "segmented": True},
             input=np.ones(10007, dt), expected=np.array([10008], dt))

    # --- transform_reduce.cpp:23-69: size_t iota(rand()), multiplies of (v, v) tuples, init (1,1)
    start = int(np.random.default_rng(0x7EED).integers(0, 2**31 - 1))
    c = np.arange(start, start + 10007, dtype=np.uint64)
    prod = 1
    for v in range(start, start + 10007):
        prod = (prod * v) & MASK64
    save("transform_reduce_product",
         {"ref": "tests/unit/parallel/algorithms/transform_reduce.cpp:23-69",
          "algo": "transform_reduce", "dtype": "uint64", "init": 1, "op": "multiplies",
          "conv": "identity", "seed_start": start},
         input=c, expected=np.array([prod], np.uint64))

    # --- transform_compute.cu:28-90: A, B = iota(dis(gen)) with dis(2,101), N=100, C = int(a + 3.0*b)
    rng = np.random.default_rng(0x7AA)
    a0, b0 = int(rng.integers(2, 102)), int(rng.integers(2, 102))
    A = np.arange(a0, a0 + 100, dtype=np.int32)
    B = np.arange(b0, b0 + 100, dtype=np.int32)
    C = np.array([int(float(x) + 3.0 * float(y)) for x, y in zip(A.tolist(), B.tolist())], np.int32)
    save("transform_compute",
         {"ref": "tests/unit/computeapi/cuda/transform_compute.cu:28-90",
          "algo": "transform_binary", "dtype": "int32", "compute": "float64", "kind": "triad",
          "scalar": 3.0},
         input=A, input2=B, expected=C)

    # --- for_each_compute.cu:28-70: i += 5 over N = 100 ints; the input is
    # std::iota(h_A.begin(), h_A.end(), dis(gen)) with dis = uniform int in
    # [2, 101] (for_each_compute.cu:62-67): 100 consecutive ints from that start
    rng = np.random.default_rng(0xF0E)
    start = int(rng.integers(2, 102))
    A = np.arange(start, start + 100, dtype=np.int32)
    save("for_each_compute",
         {"ref": "tests/unit/computeapi/cuda/for_each_compute.cu:28-51",
          "algo": "for_each", "dtype": "int32", "kind": "add_scalar", "scalar": 5},
         input=A, expected=(A + 5).astype(np.int32))

    # --- stream.cpp:82-133 check_results closed form (a = 2a warm-up, then `iterations` loops)
    for iters in (1, 2, 10):
        aj, bj, cj = 1.0, 2.0, 0.0
        aj = 2.0 * aj
        scalar = 3.0
        for _ in range(iters):
            cj = aj
            bj = scalar * cj
            cj = aj + bj
            aj = bj + scalar * cj
        save(f"stream_check_{iters}",
             {"ref": "tests/performance/local/stream.cpp:82-133", "algo": "stream", "iterations": iters,
              "scalar": 3.0},
             expected=np.array([aj, bj, cj], np.float64))

    # --- 1d_stencil_1.cpp:41-72 with U0[i] = i (1d_stencil_4.cpp:64-66): the interior of a linear
    #     ramp is a fixed point (l - 2m + r == 0 exactly), only the wrap region moves.  Closed form
    #     of the first step: next[0] = 0 + 0.5*((nx-1) - 0 + 1), next[nx-1] = (nx-1) + 0.5*((nx-2) - 2(nx-1) + 0)
    nx = 1000
    u = np.arange(nx, dtype=np.float64)
    nxt = u.copy()
    nxt[0] = 0.0 + 0.5 * ((nx - 1) - 2 * 0.0 + 1.0)
    nxt[-1] = (nx - 1) + 0.5 * ((nx - 2) - 2 * (nx - 1) + 0.0)
    save("stencil_ramp_step1",
         {"ref": "examples/1d_stencil/1d_stencil_1.cpp:41-72", "algo": "stencil", "nx": nx, "nt": 1,
          "k": 0.5, "dt": 1.0, "dx": 1.0},
         input=u, expected=nxt)

    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print(f"wrote {len(index)} fixtures")


if __name__ == "__main__":
    main()
