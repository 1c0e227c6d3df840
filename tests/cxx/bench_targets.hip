// The C++ drop-in path as an HPX program calls it, timed:
// hpx::partitioned_vector over hip::target_layout(targets) with one partition
// per target -- examples/compute/cuda/partitioned_vector.cu:38-49,
// hpx/compute/cuda/target_distribution_policy.hpp:37-218 -- running
//   the step       STREAM triad (f64) + reduce (int64) + inclusive_scan (int64)
//                  over the partitions, each algorithm under par(task), the
//                  reduce future taken after the scan is enqueued (as bench.py's
//                  step does through the Python layer);
//   the heat ring  hip::heat_solver (1d_stencil_8 over the partitions: halos
//                  between targets, fused passes of 16 steps).
// Targets: every local GPU (get_local_targets), or --targets T: T targets
// cycled over the local GPUs -- on one GPU, T targets on device 0, each with
// its own stream, so every cross-target hand-off (carries, halos, stream
// marks) still runs, without peer copies.  Elements: --logn per target (weak).
// Prints one JSON line (the keys of bench.py's step line: ms_per_step, GB/s,
// per-algorithm ms) and checks every result (reduce == scan's last == n,
// triad == 7, heat sum conserved).
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/include/partitioned_vector.hpp>
#include <hpx/parallel/heat_solver.hpp>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;
namespace fn = hpx::compute::hip::functional;

template <typename T>
using pvec = hpx::partitioned_vector<T, hpx::compute::vector<T, hip::allocator<T>>>;

namespace {
int arg_int(int argc, char** argv, char const* name, int dflt) {
    for (int i = 1; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], name)) return std::atoi(argv[i + 1]);
    return dflt;
}
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void sync_all(std::vector<hip::target> const& ts) {
    for (auto const& t : ts) t.synchronize();
}
template <typename T>
void sync_parts(pvec<T> const& v) {
    for (std::size_t j = 0; j != v.get_num_partitions(); ++j) v.get_partition(j).target.synchronize();
}
}  // namespace

int g_argc;
char** g_argv;

int hpx_main(int, char**) {
    const int logn = arg_int(g_argc, g_argv, "--logn", 30);
    const int steps = arg_int(g_argc, g_argv, "--steps", 10);
    const int warmup = arg_int(g_argc, g_argv, "--warmup", 3);
    const int heat_logn = arg_int(g_argc, g_argv, "--heat-logn", 28);
    const int heat_steps = arg_int(g_argc, g_argv, "--heat-steps", 100);
    const auto local = hip::get_local_targets();
    const int ntargets = arg_int(g_argc, g_argv, "--targets", static_cast<int>(local.size()));
    std::vector<hip::target> targets;
    for (int i = 0; i < ntargets; ++i) targets.emplace_back(local[i % local.size()].device());
    const auto policy = hip::target_layout(targets);

    const std::size_t per = std::size_t(1) << logn;
    const std::size_t n = per * targets.size();
    double el = 0, ms_triad = 0, ms_reduce = 0, ms_scan = 0;
    bool ok = false;
    {  // the step's vectors, freed before the heat ring
    pvec<double> a(n, policy), b(n, 1.0, policy), c(n, 2.0, policy);
    pvec<int64_t> x(n, int64_t(1), policy), y(n, policy);
    sync_parts(b);
    sync_parts(c);
    sync_parts(x);

    auto tpol = ex::par(ex::task);
    int64_t r = 0;
    auto step = [&] {
        auto f1 = hpx::parallel::transform(tpol, b.begin(), b.end(), c.begin(), a.begin(), fn::triad_step<double>{3.0});
        auto f2 = hpx::parallel::reduce(tpol, x.begin(), x.end(), int64_t(0), std::plus<int64_t>());
        auto f3 = hpx::parallel::inclusive_scan(tpol, x.begin(), x.end(), y.begin(), std::plus<int64_t>(), int64_t(0));
        f1.get();
        r = f2.get();
        f3.get();
    };
    for (int i = 0; i < warmup; ++i) step();
    sync_all(targets);
    const double t0 = now_s();
    for (int i = 0; i < steps; ++i) step();
    sync_all(targets);
    el = now_s() - t0;

    // per-algorithm wall times (each alone, synchronised)
    auto alone = [&](auto&& f) {
        f();
        sync_all(targets);
        double best = 1e30;
        for (int i = 0; i < 3; ++i) {
            const double s = now_s();
            f();
            sync_all(targets);
            best = std::min(best, now_s() - s);
        }
        return best * 1e3;
    };
    ms_triad = alone([&] {
        hpx::parallel::transform(ex::par, b.begin(), b.end(), c.begin(), a.begin(), fn::triad_step<double>{3.0});
    });
    ms_reduce = alone([&] { r = hpx::parallel::reduce(ex::par, x.begin(), x.end(), int64_t(0)); });
    ms_scan = alone([&] {
        hpx::parallel::inclusive_scan(ex::par, x.begin(), x.end(), y.begin(), std::plus<int64_t>(), int64_t(0));
    });

    // checks: reduce == n, scan's last == n (and across the first partition
    // boundary), a few triad values == 7
    ok = r == static_cast<int64_t>(n) && int64_t(y[n - 1]) == static_cast<int64_t>(n) &&
         int64_t(y[per - 1]) == static_cast<int64_t>(per) &&
         (n == per || int64_t(y[per]) == static_cast<int64_t>(per + 1)) && double(a[0]) == 7.0 &&
         double(a[n - 1]) == 7.0 && double(a[n / 2]) == 7.0;
    }

    // 1d_stencil_8 heat ring over the targets
    const std::size_t nx = (std::size_t(1) << heat_logn) * targets.size();
    double heat_ms = 0;
    bool heat_ok = true;
    {
        hip::heat_solver hs(nx, policy);
        hs.do_work(16);
        sync_all(targets);
        const double s = now_s();
        hs.do_work(static_cast<std::size_t>(heat_steps));
        sync_all(targets);
        heat_ms = (now_s() - s) * 1e3;
        // the ramp's sum is conserved by the periodic update up to rounding
        const std::vector<double> u = hs.to_host();
        double sum = 0, comp = 0;  // compensated: 2^28 plain additions alone drift by ~1e-8
        for (double v : u) {
            const double y = v - comp, t = sum + y;
            comp = (t - sum) - y;
            sum = t;
        }
        const double want = 0.5 * double(nx) * double(nx - 1);
        heat_ok = std::fabs(sum - want) <= 1e-9 * want;
    }

    const double ms_step = 1e3 * el / steps;
    const double bytes = 48.0 * double(n);  // triad 24 + reduce 8 + scan 16 B per element
    std::printf(
        "{\"cxx_drop_in\": {\"path\": \"partitioned_vector over hip::target_layout(targets), include/hpx\", "
        "\"targets\": %zu, \"devices\": %zu, \"partitions\": %zu, \"elements_per_target\": %zu, \"steps\": %d, "
        "\"warmup\": %d, \"ms_per_step\": %.4f, \"gbs\": %.1f, \"gbs_per_target\": %.1f, "
        "\"alone_ms\": {\"triad\": %.4f, \"reduce\": %.4f, \"inclusive_scan\": %.4f}, "
        "\"heat\": {\"points\": %zu, \"steps\": %d, \"ms\": %.3f, \"gpoint_steps_per_s\": %.2f, \"sum_conserved\": %s}, "
        "\"checks_ok\": %s}}\n",
        targets.size(), local.size(), targets.size(), per, steps, warmup, ms_step, bytes / (ms_step * 1e-3) / 1e9,
        bytes / (ms_step * 1e-3) / 1e9 / double(targets.size()), ms_triad, ms_reduce, ms_scan, nx, heat_steps, heat_ms,
        double(nx) * heat_steps / (heat_ms * 1e-3) / 1e9, heat_ok ? "true" : "false", ok ? "true" : "false");
    std::fflush(stdout);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    g_argc = argc;
    g_argv = argv;
    return hpx::init(argc, argv);
}
