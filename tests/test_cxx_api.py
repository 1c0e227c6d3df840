"""C++ drop-in layer (include/hpx/...): header-only mirror of HPX 1.4.0's
compute API and parallel algorithms over the C ABI.

CPU: the headers compile with plain g++, and a function object with no
device mapping is rejected at compile time (no silent host fallback).
GPU: the C++ test programs under tests/cxx/ -- restatements of the
reference's computeapi tests, known-answer algorithm tests and STREAM --
run against the HIP library and must report zero HPX_TEST failures.
"""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cxx", "bin")
CXX = ["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include")]


def _compile(src: str):
    with tempfile.NamedTemporaryFile("w", suffix=".cpp", delete=False) as f:
        f.write(src)
        path = f.name
    try:
        return subprocess.run(CXX + [path], capture_output=True, text=True, timeout=120)
    finally:
        os.unlink(path)


def test_headers_compile_with_host_compiler():
    r = _compile("""
#include <hpx/hpx.hpp>
#include <hpx/include/parallel_for_each.hpp>
#include <hpx/include/parallel_scan.hpp>
namespace fn = hpx::compute::hip::functional;
void f(hpx::compute::vector<double>& a, hpx::compute::vector<double>& b) {
    hpx::compute::hip::default_executor exec;
    auto p = hpx::parallel::execution::par.on(exec);
    hpx::parallel::fill(p, a.begin(), a.end(), 1.0);
    hpx::parallel::transform(p, a.begin(), a.end(), b.begin(), b.end(), a.begin(), fn::triad_step<double>{3.0});
    double s = hpx::parallel::reduce(p, a.begin(), a.end(), 0.0);
    hpx::future<double> fs = hpx::parallel::reduce(hpx::parallel::execution::par(hpx::parallel::execution::task).on(exec),
                                                   a.begin(), a.end(), s);
    hpx::parallel::inclusive_scan(p, a.begin(), a.end(), b.begin());
    hpx::parallel::sort(p, a.begin(), a.end(), std::greater<double>());
    (void)fs;
}
""")
    assert r.returncode == 0, r.stderr


def test_closure_algorithms_need_hipcc():
    """A lambda conv / op / pred / comp in a host-compiled TU is rejected at
    compile time with the way out named (no host fallback)."""
    for call in ("hpx::parallel::transform_reduce(p, a.begin(), a.end(), 0, std::plus<>(), [](int x) { return x * 2; });",
                 "hpx::parallel::reduce(p, a.begin(), a.end(), 0, [](int x, int y) { return x + y; });",
                 "hpx::parallel::inclusive_scan(p, a.begin(), a.end(), a.begin(), [](int x, int y) { return x + y; });",
                 "hpx::parallel::copy_if(p, a.begin(), a.end(), a.begin(), [](int x) { return x > 0; });",
                 "hpx::parallel::sort(p, a.begin(), a.end(), [](int x, int y) { return x > y; });"):
        r = _compile(f"""
#include <hpx/hpx.hpp>
void f(hpx::compute::vector<int>& a) {{
    hpx::compute::hip::default_executor exec;
    auto p = hpx::parallel::execution::par.on(exec);
    {call}
}}
""")
        assert r.returncode != 0, call
        assert "compile the translation unit with hipcc" in r.stderr, (call, r.stderr[-2000:])


def test_unmapped_functor_is_a_compile_error():
    r = _compile("""
#include <hpx/hpx.hpp>
void f(hpx::compute::vector<int>& a) {
    hpx::parallel::for_each(hpx::parallel::execution::par, a.begin(), a.end(), [](int& i) { i *= 7; });
}
""")
    assert r.returncode != 0
    assert "traits::unary" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("prog,args", [
    ("compute_api", ["12345"]),
    ("algorithms_known_answer", ["20260101"]),
    ("stream_hip", ["--vector_size", str(1 << 26), "--iterations", "10"]),
    ("for_loop_merge", []),
    ("device_closures", ["4242"]),
    ("closure_algorithms", ["777"]),
    ("closure_algorithms", ["778", "--big"]),
    ("partitioned_vector", []),
    ("stencil_partitioned", []),
    ("call_overhead", []),
    ("exception_list", []),
    ("dataflow_stencil", []),
    ("futures", []),
])
def test_cxx_program(prog, args):
    exe = os.path.join(BIN, prog)
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (run `make cxxtests` / __graft_entry__.build())")
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert f"{prog}: all tests passed" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("targets", [1, 3])
def test_cxx_drop_in_bench_program(targets):
    """tests/cxx/bench_targets (bench.py's `cxx_drop_in` row) at small sizes:
    the step (triad + reduce + inclusive_scan under par(task)) and the heat
    ring over a partitioned_vector of `targets` HIP targets on one device,
    its own checks (reduce == scan's last == n, triad == 7, the heat ring's
    sum conserved) and one JSON line."""
    import json
    exe = os.path.join(BIN, "bench_targets")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (run `make cxxtests` / __graft_entry__.build())")
    r = subprocess.run([exe, "--targets", str(targets), "--logn", "20", "--heat-logn", "14", "--steps", "3",
                        "--warmup", "1", "--heat-steps", "37"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    row = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"cxx_drop_in"')][-1])["cxx_drop_in"]
    assert row["checks_ok"] and row["heat"]["sum_conserved"], row
    assert row["targets"] == targets and row["elements_per_target"] == 1 << 20 and row["ms_per_step"] > 0


def test_futures_compose_on_host():
    """hpx::future / shared_future / dataflow / unwrapping / when_all /
    wait_all / sliding_semaphore on host values (the restated lcos unit
    tests, tests/cxx/futures.cpp): no device work, so it runs without a GPU;
    the completion engine's thread runs the continuations."""
    exe = os.path.join(BIN, "futures")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "tests/cxx/bin/futures"], check=True, capture_output=True, timeout=600)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "futures: all tests passed" in r.stdout


def test_par_unseq_error_terminates():
    """handle_exception_impl<parallel_unsequenced_policy> (parallel/
    exception_list.hpp:138-158): an algorithm error under par_unseq calls
    std::terminate.  The failure (a reversed range over an empty vector) is
    raised before any device call, so this runs without a GPU."""
    exe = os.path.join(BIN, "exception_list")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (run `make cxxtests`)")
    r = subprocess.run([exe, "unseq"], capture_output=True, text=True, timeout=120)
    assert r.returncode == -6, (r.returncode, r.stdout, r.stderr)
    assert "returned" not in r.stdout and "negative range" in r.stderr
