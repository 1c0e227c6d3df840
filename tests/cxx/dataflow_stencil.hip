// examples/1d_stencil/1d_stencil_4.cpp on HIP targets, composed the
// reference's way: every partition of every time step is an
// hpx::shared_future<partition_data> (:101), computed by
// hpx::dataflow(hpx::launch::async, unwrapping(heat_part), left, middle,
// right) (:135-170) with a sliding_semaphore bounding the depth of the tree
// (:156-186), the solution collected by hpx::when_all (:192) and waited for by
// hpx::wait_all (:218).  Here a partition lives in device memory and
// heat_part is a hip-executor for_loop_n under par(task) returning
// hpx::future<partition_data>, which dataflow unwraps: a step's future is
// ready when its kernel has run, and the next step's kernel is launched by
// the completion engine once its three inputs are.
//
// Checked bit for bit against the oracle's serial stencil
// (oracle_stencil_heat, 1d_stencil_1.cpp:41-72) for 1-10 partitions, several
// partition sizes, step counts and tree depths, from the reference's ramp
// (U0 = i) and from a random state; partitions are dealt over several
// targets (streams) of device 0.
//
// usage: dataflow_stencil
#pragma clang fp contract(off)  // heat() rounds like the host oracle

#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/include/lcos.hpp>
#include <hpx/util/lightweight_test.hpp>

#include "../../oracle/oracle.h"

#include <chrono>
#include <cstdint>
#include <iostream>
#include <memory>
#include <random>
#include <vector>

namespace hip = hpx::compute::hip;
namespace ex = hpx::parallel::execution;

double k = 0.5;   // heat transfer coefficient
double dt = 1.;   // time step
double dx = 1.;   // grid spacing

// 1d_stencil_4.cpp:39-50
inline std::size_t idx(std::size_t i, int dir, std::size_t size) {
    if (i == 0 && dir == -1) return size - 1;
    if (i == size - 1 && dir == +1) return 0;
    return i + dir;
}

// 1d_stencil_4.cpp:52-85, in device memory: the points of one partition in a
// compute::vector on one target.  Copies share the buffer (the reference's
// partition_data is move-only; a shared_future hands out const references).
struct partition_data {
    using vec = hpx::compute::vector<double, hip::allocator<double>>;
    std::shared_ptr<vec> data_;
    std::shared_ptr<hip::default_executor> exec_;  // the target the partition lives on

    partition_data(std::size_t size, std::shared_ptr<hip::default_executor> exec)
        : data_(std::make_shared<vec>(size, hip::allocator<double>(exec->target()))), exec_(std::move(exec)) {}
    // base_value = initial_value * size; data[i] = base_value + i
    partition_data(std::size_t size, double initial_value, std::shared_ptr<hip::default_executor> exec)
        : partition_data(size, std::move(exec)) {
        std::vector<double> h(size);
        const double base_value = double(initial_value * size);
        for (std::size_t i = 0; i != size; ++i) h[i] = base_value + double(i);
        upload(h);
    }
    partition_data(std::vector<double> const& values, std::shared_ptr<hip::default_executor> exec)
        : partition_data(values.size(), std::move(exec)) {
        upload(values);
    }
    void upload(std::vector<double> const& h) {
        hpx::parallel::copy(ex::par, h.begin(), h.end(), data_->begin());
    }
    std::vector<double> to_host() const {
        std::vector<double> h(size());
        hpx::parallel::copy(ex::par, data_->begin(), data_->end(), h.begin());
        return h;
    }
    std::size_t size() const { return data_->size(); }
    double* ptr() const { return data_->data(); }
};

struct stepper {
    // 1d_stencil_4.cpp:99-101
    typedef hpx::shared_future<partition_data> partition;
    typedef std::vector<partition> space;

    // 1d_stencil_4.cpp:104-107
    HPX_HOST_DEVICE static double heat(double left, double middle, double right, double c) {
        return middle + c * (left - 2 * middle + right);
    }

    // 1d_stencil_4.cpp:111-127 as a hip-executor loop over the partition's
    // points; the result is ready when the kernel has run
    static hpx::future<partition_data> heat_part(partition_data const& left, partition_data const& middle,
                                                 partition_data const& right) {
        const std::size_t size = middle.size();
        partition_data next(size, middle.exec_);
        double const* l = left.ptr();
        double const* m = middle.ptr();
        double const* r = right.ptr();
        double* o = next.ptr();
        const double c = k * dt / (dx * dx);
        hpx::future<void> done = hpx::parallel::for_loop_n(
            ex::par(ex::task).on(*middle.exec_), o, size, [=] HPX_HOST_DEVICE(double* p) {
                const std::size_t i = static_cast<std::size_t>(p - o);
                const double lv = i == 0 ? l[size - 1] : m[i - 1];
                const double rv = i == size - 1 ? r[0] : m[i + 1];
                *p = heat(lv, m[i], rv, c);
            });
        return done.then(hpx::launch::sync, [next](hpx::future<void>&& f) {
            f.get();
            return next;
        });
    }

    std::vector<std::shared_ptr<hip::default_executor>> execs;

    // 1d_stencil_4.cpp:131-193
    hpx::future<space> do_work(std::size_t np, std::size_t nx, std::size_t nt, std::uint64_t nd,
                               std::vector<double> const* init) {
        using hpx::dataflow;
        using hpx::util::unwrapping;

        std::vector<space> U(2);
        for (space& s : U) s.resize(np);

        // initial conditions: f(0, i) = i (or the given state)
        for (std::size_t i = 0; i != np; ++i) {
            auto const& e = execs[i % execs.size()];
            if (init) {
                std::vector<double> part(init->begin() + i * nx, init->begin() + (i + 1) * nx);
                U[0][i] = hpx::make_ready_future(partition_data(part, e));
            } else {
                U[0][i] = hpx::make_ready_future(partition_data(nx, double(i), e));
            }
        }

        // limit depth of dependency tree.  The semaphore outlives do_work
        // (the reference keeps it on do_work's stack, where the continuations
        // of the last nd steps may still signal it after do_work returned)
        auto sem = std::make_shared<hpx::lcos::local::sliding_semaphore>(nd);

        auto Op = unwrapping(&stepper::heat_part);

        for (std::size_t t = 0; t != nt; ++t) {
            space const& current = U[t % 2];
            space& next = U[(t + 1) % 2];
            for (std::size_t i = 0; i != np; ++i) {
                next[i] = dataflow(hpx::launch::async, Op, current[idx(i, -1, np)], current[i],
                                   current[idx(i, +1, np)]);
            }
            // every nd time steps, attach a continuation which triggers the
            // semaphore once computation has reached this point
            if ((t % nd) == 0) {
                next[0].then([sem, t](partition&&) { sem->signal(t); });
            }
            // suspend if the tree has become too deep
            sem->wait(t);
        }
        return hpx::when_all(U[nt % 2]);
    }
};

void run(std::size_t np, std::size_t nx, std::size_t nt, std::uint64_t nd, std::size_t ntargets, bool random_init) {
    stepper step;
    for (std::size_t j = 0; j != ntargets; ++j)
        step.execs.push_back(std::make_shared<hip::default_executor>(hip::target(0)));
    std::vector<double> u(np * nx);
    if (random_init) {
        std::mt19937_64 gen(np * 131 + nx * 7 + nt);
        std::normal_distribution<double> dis;
        for (auto& x : u) x = dis(gen);
    } else {
        for (std::size_t i = 0; i != u.size(); ++i) u[i] = double(i);
    }
    const auto t0 = std::chrono::steady_clock::now();
    hpx::future<stepper::space> result = step.do_work(np, nx, nt, nd, random_init ? &u : nullptr);
    stepper::space solution = result.get();
    hpx::wait_all(solution);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    std::vector<double> got;
    for (auto const& p : solution) {
        HPX_TEST(p.is_ready());
        auto h = p.get().to_host();
        got.insert(got.end(), h.begin(), h.end());
    }
    std::vector<double> want = u;
    HPX_TEST_EQ(oracle_stencil_heat(want.data(), want.size(), nt, k, dt, dx), 0);
    std::size_t bad = 0;
    for (std::size_t i = 0; i != want.size(); ++i)
        if (got[i] != want[i]) {
            if (bad < 3)
                std::cout << "    i " << i << " got " << std::hexfloat << got[i] << " want " << want[i] << std::defaultfloat
                          << std::endl;
            ++bad;
        }
    HPX_TEST_EQ(bad, std::size_t(0));
    std::cout << "  np " << np << " nx " << nx << " nt " << nt << " nd " << nd << " targets " << ntargets
              << (random_init ? " random" : " ramp") << ": " << (bad ? "MISMATCH" : "bit-exact") << ", " << ms
              << " ms (" << ms * 1e3 / double(nt) << " us/step)" << std::endl;
}

int hpx_main(int, char**) {
    // the reference's defaults: np 10, nx 10, nt 45, nd 10 (1d_stencil_4.cpp:242-251)
    run(10, 10, 45, 10, 1, false);
    run(10, 10, 45, 10, 3, true);
    for (std::size_t np = 1; np <= 9; ++np) run(np, 64 + 37 * np, 20 + np, 1 + np % 4, 1 + np % 3, true);
    run(4, 1 << 20, 12, 4, 2, true);
    run(8, 100000, 30, 5, 4, false);
    const int errs = hpx::util::report_errors();
    if (!errs) std::cout << "dataflow_stencil: all tests passed" << std::endl;
    return errs;
}

int main(int argc, char** argv) { return hpx::init(argc, argv); }
