// The error contract of the parallel algorithms: the shape of the
// reference's exception tests (tests/unit/parallel/algorithms/
// foreach_tests.hpp:110-205 and their siblings), with device-side failures
// in place of the throwing host functors:
//
//   * a failure under seq / par / par.on(exec) throws hpx::exception_list
//     holding the original error (handle_exception_impl, parallel/
//     exception_list.hpp:20-61);
//   * under par(task) the algorithm returns, and the future's get() throws
//     hpx::exception_list (handle_exception_task_impl, :63-111);
//   * an allocation failure is std::bad_alloc, never wrapped
//     (handle_local_exceptions.hpp:30-40);
//   * a failure that surfaces only when the queued device work completes
//     (the device error word) follows the same rules.
//
// The failures are injected at the C ABI (hpxhip_debug_inject_error: the next
// algorithm entry returns the given status without enqueuing anything;
// hpxhip_debug_raise_device_error: the device error word is set from the
// stream), or come from real invalid calls (an unsupported conversion, a
// reversed range).  `exception_list unseq` checks that par_unseq terminates
// (run by tests/test_cxx_api.py in its own process, expecting SIGABRT).
#include <hpx/hpx.hpp>
#include <hpx/hpx_init.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <numeric>
#include <string>
#include <vector>

namespace ex = hpx::parallel::execution;
namespace fn = hpx::compute::hip::functional;
using executor_type = hpx::compute::hip::default_executor;
using ivec = hpx::compute::vector<int, hpx::compute::hip::allocator<int>>;

// test_num_exceptions: one exception per failed call here (a device
// algorithm is one launch, not one task per chunk); the element is the
// original kernel_error carrying the injected status.
void check_list(hpx::exception_list const& e, int status) {
    HPX_TEST_EQ(e.size(), std::size_t(1));
    HPX_TEST_EQ(e.status, status);
    for (auto const& p : e) {
        bool inner = false;
        try {
            std::rethrow_exception(p);
        } catch (hpx::kernel_error const& k) {
            inner = (k.status == status);
        } catch (...) {
        }
        HPX_TEST(inner);
    }
}

void inject(int status) { HPX_TEST_EQ(hpxhip_debug_inject_error(status, 1), 0); }

// foreach_tests.hpp:112-139 test_for_each_exception
template <typename P>
void test_exception(P policy, ivec& c, char const* name) {
    inject(HPXHIP_ERROR_INVALID_ARGUMENT);
    bool caught = false;
    try {
        hpx::parallel::for_each(policy, c.begin(), c.end(), fn::add_value<int>{1});
        HPX_TEST_MSG(false, name);
    } catch (hpx::exception_list const& e) {
        caught = true;
        check_list(e, HPXHIP_ERROR_INVALID_ARGUMENT);
    } catch (...) {
        HPX_TEST_MSG(false, name);
    }
    HPX_TEST_MSG(caught, name);
}

// foreach_tests.hpp:141-172 test_for_each_exception_async
template <typename P>
void test_exception_async(P policy, ivec& c, char const* name) {
    inject(HPXHIP_ERROR_INVALID_ARGUMENT);
    bool caught = false, returned = false;
    try {
        auto f = hpx::parallel::for_each(policy, c.begin(), c.end(), fn::add_value<int>{1});
        returned = true;
        HPX_TEST(f.is_ready());
        f.get();
        HPX_TEST_MSG(false, name);
    } catch (hpx::exception_list const& e) {
        caught = true;
        check_list(e, HPXHIP_ERROR_INVALID_ARGUMENT);
    } catch (...) {
        HPX_TEST_MSG(false, name);
    }
    HPX_TEST_MSG(caught, name);
    HPX_TEST_MSG(returned, name);
}

// foreach_tests.hpp:175-205 test_for_each_bad_alloc (+ _async)
template <typename P>
void test_bad_alloc(P policy, ivec& c, char const* name) {
    inject(HPXHIP_ERROR_OUT_OF_MEMORY);
    bool caught = false;
    try {
        (void)hpx::parallel::reduce(policy, c.begin(), c.end(), 0);
        HPX_TEST_MSG(false, name);
    } catch (hpx::exception_list const&) {
        HPX_TEST_MSG(false, name);  // bad_alloc is never wrapped
    } catch (std::bad_alloc const&) {
        caught = true;
    } catch (...) {
        HPX_TEST_MSG(false, name);
    }
    HPX_TEST_MSG(caught, name);
}
template <typename P>
void test_bad_alloc_async(P policy, ivec& c, char const* name) {
    inject(HPXHIP_ERROR_OUT_OF_MEMORY);
    bool caught = false, returned = false;
    try {
        auto f = hpx::parallel::reduce(policy, c.begin(), c.end(), 0);
        returned = true;
        (void)f.get();
        HPX_TEST_MSG(false, name);
    } catch (hpx::exception_list const&) {
        HPX_TEST_MSG(false, name);
    } catch (std::bad_alloc const&) {
        caught = true;
    } catch (...) {
        HPX_TEST_MSG(false, name);
    }
    HPX_TEST_MSG(caught, name);
    HPX_TEST_MSG(returned, name);
}

// The device error word set from the stream: the call itself enqueues fine,
// the failure is seen when the queued work has run.
void test_device_side_failure(executor_type& exec, ivec& c) {
    auto t = exec.target();
    bool caught = false;
    HPX_TEST_EQ(hpxhip_debug_raise_device_error(t.stream(), 7u), 0);
    try {
        (void)hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), 0);
        HPX_TEST(false);
    } catch (hpx::exception_list const& e) {
        caught = true;
        check_list(e, HPXHIP_ERROR_DEVICE_TIMEOUT);
    }
    HPX_TEST(caught);

    caught = false;
    HPX_TEST_EQ(hpxhip_debug_raise_device_error(t.stream(), 9u), 0);
    auto f = hpx::parallel::transform_reduce(ex::par(ex::task).on(exec), c.begin(), c.end(), 0L, std::plus<long>(),
                                             fn::identity{});
    try {
        (void)f.get();
        HPX_TEST(false);
    } catch (hpx::exception_list const& e) {
        caught = true;
        check_list(e, HPXHIP_ERROR_DEVICE_TIMEOUT);
    }
    HPX_TEST(caught);
    // the word is cleared by the report: the next call succeeds
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par.on(exec), c.begin(), c.end(), 0), 10007 * 10006 / 2 + 10007 * 3);
}

// Real invalid calls (no injection): a conversion no reduction kernel was
// built for, and a reversed range.
void test_invalid_calls(ivec& c) {
    hpx::compute::vector<float, hpx::compute::hip::allocator<float>> v(64, 1.0f);
    bool caught = false;
    try {
        (void)hpx::parallel::transform_reduce(ex::par, v.begin(), v.end(), 0.0f, std::plus<float>(), fn::negate{});
    } catch (hpx::exception_list const& e) {
        caught = true;
        check_list(e, HPXHIP_ERROR_UNSUPPORTED);
    }
    HPX_TEST(caught);

    caught = false;
    auto f = hpx::parallel::fill(ex::par(ex::task), c.end(), c.begin(), 1);
    try {
        f.get();
    } catch (hpx::exception_list const& e) {
        caught = true;
        HPX_TEST_EQ(e.size(), std::size_t(1));
        HPX_TEST_EQ(e.status, HPXHIP_ERROR_INVALID_ARGUMENT);
    }
    HPX_TEST(caught);

    // allocation beyond HBM: std::bad_alloc from the allocator
    caught = false;
    try {
        ivec huge(std::size_t(1) << 48);
    } catch (std::bad_alloc const&) {
        caught = true;
    }
    HPX_TEST(caught);
}

// Every algorithm family reports through the same contract (one injected
// failure per call, sync and task).
template <typename P, typename PT>
void test_all_algorithms(P pol, PT task, ivec& c, ivec& d) {
    auto expect = [&](auto&& call, char const* name) {
        inject(HPXHIP_ERROR_INVALID_ARGUMENT);
        bool caught = false;
        try {
            call();
        } catch (hpx::exception_list const& e) {
            caught = e.size() == 1 && e.status == HPXHIP_ERROR_INVALID_ARGUMENT;
        } catch (...) {
        }
        HPX_TEST_MSG(caught, name);
    };
    expect([&] { hpx::parallel::fill(pol, d.begin(), d.end(), 3); }, "fill");
    expect([&] { hpx::parallel::copy(pol, c.begin(), c.end(), d.begin()); }, "copy");
    expect([&] { hpx::parallel::transform(pol, c.begin(), c.end(), d.begin(), fn::add_value<int>{2}); }, "transform");
    expect([&] { hpx::parallel::transform(pol, c.begin(), c.end(), c.begin(), d.begin(), std::plus<int>()); },
           "transform binary");
    expect([&] { (void)hpx::parallel::reduce(pol, c.begin(), c.end(), 0); }, "reduce");
    expect([&] { hpx::parallel::inclusive_scan(pol, c.begin(), c.end(), d.begin()); }, "inclusive_scan");
    expect([&] { hpx::parallel::exclusive_scan(pol, c.begin(), c.end(), d.begin(), 0); }, "exclusive_scan");
    expect([&] { hpx::parallel::copy_if(pol, c.begin(), c.end(), d.begin(), fn::not_less_than<int>{0}); }, "copy_if");
    expect([&] { hpx::parallel::sort(pol, d.begin(), d.end()); }, "sort");
    expect([&] { (void)hpx::parallel::is_sorted(pol, d.begin(), d.end()); }, "is_sorted");
    expect([&] { hpx::parallel::inclusive_scan(task, c.begin(), c.end(), d.begin()).get(); }, "inclusive_scan task");
    expect([&] { hpx::parallel::sort(task, d.begin(), d.end()).get(); }, "sort task");
    expect([&] { (void)hpx::parallel::transform_reduce(task, c.begin(), c.end(), c.begin(), 0).get(); },
           "inner product task");
}

int run_unseq() {
    // par_unseq: an exception calls std::terminate (handle_exception_impl<
    // parallel_unsequenced_policy>, parallel/exception_list.hpp:138-158).  A
    // reversed range over an empty vector fails before any device call.
    ivec v;
    hpx::parallel::fill(ex::par_unseq, v.begin() + 1, v.begin(), 0);
    std::cout << "exception_list unseq: returned (expected std::terminate)" << std::endl;
    return 0;
}

int hpx_main(int argc, char* argv[]) {
    if (argc > 1 && std::strcmp(argv[1], "unseq") == 0) return run_unseq();
    executor_type exec;
    ivec c(10007), d(10007);
    std::vector<int> h(10007);
    std::iota(h.begin(), h.end(), 3);
    hpx::parallel::copy(ex::par, h.begin(), h.end(), c.begin());

    test_exception(ex::seq, c, "seq");
    test_exception(ex::par, c, "par");
    test_exception(ex::par.on(exec), c, "par.on(exec)");
    test_exception_async(ex::seq(ex::task), c, "seq(task)");
    test_exception_async(ex::par(ex::task), c, "par(task)");
    test_exception_async(ex::par(ex::task).on(exec), c, "par(task).on(exec)");
    test_bad_alloc(ex::seq, c, "seq bad_alloc");
    test_bad_alloc(ex::par.on(exec), c, "par bad_alloc");
    test_bad_alloc_async(ex::par(ex::task).on(exec), c, "par(task) bad_alloc");
    test_device_side_failure(exec, c);
    test_invalid_calls(c);
    test_all_algorithms(ex::par.on(exec), ex::par(ex::task).on(exec), c, d);

    // nothing left injected: the data is untouched by the failed calls
    HPX_TEST_EQ(hpxhip_debug_inject_error(0, 0), 0);
    HPX_TEST_EQ(hpx::parallel::reduce(ex::par, c.begin(), c.end(), 0L), 10007L * 10006 / 2 + 10007L * 3);
    int errs = hpx::util::report_errors();
    if (errs == 0) std::cout << "exception_list: all tests passed" << std::endl;
    return errs;
}

int main(int argc, char* argv[]) { return hpx::init(argc, argv); }
