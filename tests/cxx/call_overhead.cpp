// call_overhead.cpp -- what one call through the C++ drop-in layer costs on
// the host (round-1 review: "every par.on(exec) call creates and destroys a
// stream and result-slot buffers; no C++-side timing exists").  Targets now
// take their streams and result slots from per-device pools, so a call is the
// policy copy + the C-ABI enqueue (+ the completion for task policies).
//
// Measured on small vectors (4096 doubles: the kernel is a few microseconds,
// so host time dominates), per call, after warm-up:
//   * transform(par.on(exec)) -- synchronous: enqueue + stream wait;
//   * transform(par(task).on(exec)) + get();
//   * reduce(par.on(exec)) -- includes the result's D2H copy;
//   * reduce(par(task).on(exec)) with the policy built inline each time (the
//     temporary-policy case that was a use-after-free in round 1);
//   * 64 reduce futures in flight, then when_all().get() (per call);
//   * the raw C-ABI hpxhip_transform_binary enqueue for comparison.
// Prints one line per case; exit status 0 unless a result is wrong.
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

using executor_type = hpx::compute::hip::default_executor;
using alloc_t = hpx::compute::hip::allocator<double>;
using dvec = hpx::compute::vector<double, alloc_t>;
namespace fn = hpx::compute::hip::functional;
namespace ex = hpx::parallel::execution;

template <typename F>
double us_per_call(int reps, F&& f) {
    for (int i = 0; i < 16; ++i) f();  // warm-up: pools filled, code objects loaded
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int hpx_main(int, char**) {
    hpx::compute::hip::target t;
    alloc_t alloc(t);
    executor_type exec(t);
    const std::size_t n = 4096;
    dvec a(n, 1.0, alloc), b(n, 2.0, alloc), c(n, 0.0, alloc);
    const int reps = 2000;

    const double sync_tr = us_per_call(reps, [&] {
        hpx::parallel::transform(ex::par.on(exec), b.begin(), b.end(), c.begin(), a.begin(),
                                 fn::triad_step<double>{3.0});
    });
    const double task_tr = us_per_call(reps, [&] {
        hpx::parallel::transform(ex::par(ex::task).on(exec), b.begin(), b.end(), c.begin(), a.begin(),
                                 fn::triad_step<double>{3.0})
            .get();
    });
    double s = 0;
    const double sync_red = us_per_call(reps, [&] { s = hpx::parallel::reduce(ex::par.on(exec), b.begin(), b.end(), 0.0); });
    HPX_TEST_EQ(s, 2.0 * double(n));
    const double task_red = us_per_call(reps, [&] {
        s = hpx::parallel::reduce(ex::par(ex::task).on(executor_type(t)), b.begin(), b.end(), 0.0).get();
    });
    HPX_TEST_EQ(s, 2.0 * double(n));
    const int batch = 64;
    const double many = us_per_call(reps / batch, [&] {
                            std::vector<hpx::future<double>> fs;
                            fs.reserve(batch);
                            auto pol = ex::par(ex::task).on(exec);
                            for (int i = 0; i < batch; ++i) fs.push_back(hpx::parallel::reduce(pol, b.begin(), b.end(), 0.0));
                            auto all = hpx::when_all(std::move(fs)).get();
                            s = all[batch - 1].get();
                        }) /
                        batch;
    HPX_TEST_EQ(s, 2.0 * double(n));
    double three = 3.0;
    auto stream = exec.target().native_handle().get_stream();
    const double raw = us_per_call(reps, [&] {
        hpxhip_transform_binary(HPXHIP_F64, HPXHIP_F64, HPXHIP_F64, HPXHIP_B_TRIAD, &three, b.data(), c.data(),
                                a.data(), n, stream);
    });
    exec.target().synchronize();
    HPX_TEST_EQ(double(a[n - 1]), 2.0);  // a = b + 3 c with b = 2, c = 0

    // sort(par(task)) returns once the device-planned sort is enqueued
    // (sort.hpp:251-276); a reduce queued behind it on the same stream sees
    // the sorted keys.  2^27 u64 keys: the device takes milliseconds, the
    // call must return in far less.
    using ualloc_t = hpx::compute::hip::allocator<uint64_t>;
    const std::size_t nk = std::size_t(1) << 27;
    hpx::compute::vector<uint64_t, ualloc_t> keys(nk, ualloc_t(t));
    double sort_call_us = 1e30, sort_total_us = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        hpxhip_generate(HPXHIP_U64, HPXHIP_GEN_BITS, 77 + rep, 0, 0, keys.data(), nk, stream);
        // the keys are written on exec's own stream; the policies below hold
        // copies of exec, whose targets have streams of their own
        exec.target().synchronize();
        const uint64_t sum0 = hpx::parallel::reduce(ex::par.on(exec), keys.begin(), keys.end(), uint64_t(0));
        // one policy object: its executor's target (a copy of exec's, so its
        // own stream, cuda_target.cpp:203-211) orders the three calls
        auto tpol = ex::par(ex::task).on(exec);
        const auto t0 = std::chrono::steady_clock::now();
        auto fs = hpx::parallel::sort(tpol, keys.begin(), keys.end());
        const auto t1 = std::chrono::steady_clock::now();
        auto fr = hpx::parallel::reduce(tpol, keys.begin(), keys.end(), uint64_t(0));
        auto fo = hpx::parallel::is_sorted(tpol, keys.begin(), keys.end());
        HPX_TEST(fs.get() == keys.end());
        const uint64_t sr = fr.get();
        HPX_TEST_EQ(sr, sum0);
        HPX_TEST(fo.get());
        if (sr != sum0) {
            const uint64_t again = hpx::parallel::reduce(ex::par.on(exec), keys.begin(), keys.end(), uint64_t(0));
            std::printf("rep %d: sum0 %llu, task reduce after sort %llu, sync reduce afterwards %llu\n", rep,
                        (unsigned long long)sum0, (unsigned long long)sr, (unsigned long long)again);
        }
        const auto t2 = std::chrono::steady_clock::now();
        sort_call_us = std::min(sort_call_us, std::chrono::duration<double, std::micro>(t1 - t0).count());
        sort_total_us = std::min(sort_total_us, std::chrono::duration<double, std::micro>(t2 - t0).count());
    }
    HPX_TEST(sort_call_us < 0.25 * sort_total_us);  // the call did not wait for the device

    std::printf("C++ layer host time per call, %zu doubles (us):\n", n);
    std::printf("  transform par.on(exec)                 %8.2f\n", sync_tr);
    std::printf("  transform par(task).on(exec) + get     %8.2f\n", task_tr);
    std::printf("  reduce par.on(exec)                    %8.2f\n", sync_red);
    std::printf("  reduce par(task).on(inline exec) + get %8.2f\n", task_red);
    std::printf("  reduce x64 futures + when_all, per call %7.2f\n", many);
    std::printf("  raw C ABI enqueue (transform_binary)   %8.2f\n", raw);
    std::printf("sort(par(task)) of 2^27 u64 keys: call returns after %.1f us, sort + reduce + is_sorted done "
                "after %.1f us\n",
                sort_call_us, sort_total_us);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::printf("call_overhead: all tests passed\n");
    return errors;
}
