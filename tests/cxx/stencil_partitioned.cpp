// 1d_stencil_8 on HIP targets through the C++ layer: hpx::compute::hip::
// heat_solver (include/hpx/parallel/heat_solver.hpp) over a
// partitioned_vector, checked bit for bit against the serial example
// (1d_stencil_1.cpp:41-72: U0[i] = i, periodic ring, k = 0.5, dt = dx = 1)
// computed here on the host:
//   - partitions: one per target, 3, 7 (uneven, some neighbours on the same
//     target), and more partitions than points per partition allows fused
//     passes of 16 (small partitions force shorter passes);
//   - step counts that are not multiples of the fused pass (1, 15, 33, 100);
//   - a random initial state (the ramp is a steady state away from the seam).
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/include/partitioned_vector.hpp>
#include <hpx/parallel/heat_solver.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <chrono>
#include <cstdint>
#include <iostream>
#include <random>
#include <vector>

namespace hip = hpx::compute::hip;

// 1d_stencil_1.cpp:41-72 (space-time loop with two buffers)
std::vector<double> serial(std::vector<double> u, std::size_t nt, double k = 0.5, double dt = 1.0, double dx = 1.0) {
    const std::size_t n = u.size();
    std::vector<double> v(n);
    for (std::size_t t = 0; t != nt; ++t) {
        for (std::size_t i = 0; i != n; ++i) {
            const double l = u[(i + n - 1) % n], m = u[i], r = u[(i + 1) % n];
            v[i] = m + (k * dt / (dx * dx)) * (l - 2 * m + r);
        }
        u.swap(v);
    }
    return u;
}

void run(std::size_t nx, std::size_t nt, hip::target_distribution_policy const& policy, bool random_init) {
    hip::heat_solver hs(nx, policy);
    std::vector<double> u0(nx);
    if (random_init) {
        std::mt19937_64 gen(nx * 31 + nt);
        std::normal_distribution<double> dis;
        for (auto& x : u0) x = dis(gen);
        hs.set(u0);
    } else {
        for (std::size_t i = 0; i != nx; ++i) u0[i] = static_cast<double>(i);
    }
    hs.do_work(nt);
    const std::vector<double> got = hs.to_host();
    const std::vector<double> want = serial(u0, nt);
    std::size_t bad = 0;
    for (std::size_t i = 0; i != nx; ++i)
        if (got[i] != want[i]) {
            if (bad < 3)
                std::cout << "    i " << i << " got " << std::hexfloat << got[i] << " want " << want[i] << std::defaultfloat
                          << std::endl;
            ++bad;
        }
    if (!HPX_TEST_EQ(bad, std::size_t(0)))
        std::cout << "  nx " << nx << " nt " << nt << " partitions " << hs.current().get_num_partitions()
                  << (random_init ? " random" : " ramp") << ": " << bad << " points differ" << std::endl;
}

// Wall time per fused pass with many small partitions on one device, where
// the hand-offs between passes, not the kernels, set the pace (r05: marks
// waited for on the device; r04 synchronised every stream between passes).
void pass_timing(std::vector<hip::target> const& targets) {
    for (std::size_t np : {7, 64}) {
        hip::heat_solver hs(np * 4096, hip::target_layout(targets[0], np));
        hs.do_work(16);
        const std::size_t passes = 200;
        const auto t0 = std::chrono::steady_clock::now();
        hs.do_work(16 * passes);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        std::cout << "  pass timing: " << np << " partitions x 4096 points, 16 steps per pass: " << us / passes
                  << " us per pass" << std::endl;
    }
}

int hpx_main(int, char**) {
    const auto targets = hip::get_local_targets();
    for (bool rnd : {false, true})
        for (std::size_t nt : {1, 15, 33, 100}) {
            run(10007, nt, hip::target_layout, rnd);
            run(10007, nt, hip::target_layout(targets, 3), rnd);
            run(1001, nt, hip::target_layout(targets, 7), rnd);
            run(90, nt, hip::target_layout(targets, 9), rnd);  // 10-point partitions: passes of <= 10 steps
        }
    run(1, 5, hip::target_layout, true);  // a ring of one point
    pass_timing(targets);
    // every cross-stream hand-off (carries, halos) was ordered on the device
    HPX_TEST_EQ(hip::detail::stream_order_host_waits().load(), 0ul);
    return hpx::finalize();
}

int main(int argc, char* argv[]) {
    HPX_TEST_EQ(hpx::init(argc, argv), 0);
    int errors = hpx::util::report_errors();
    if (!errors) std::cout << "stencil_partitioned: all tests passed" << std::endl;
    return errors;
}
