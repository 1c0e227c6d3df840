// Future composition of the HIP backend's C++ layer on host values (no GPU
// needed: nothing here enqueues device work; the completion engine runs the
// continuations).  Restatements of the reference's lcos unit tests:
//
//   tests/unit/lcos/local_dataflow.cpp:69-126   dataflow(unwrapping(f), ...) over
//                                               nested dataflows, vectors of futures
//   tests/unit/lcos/local_dataflow.cpp:134-225  dataflow(f, futures...) receives
//                                               ready futures
//   tests/unit/lcos/local_dataflow.cpp:239-290  plain (non-future) arguments
//   tests/unit/lcos/future_then.cpp             then chains, then on shared_future
//   tests/unit/lcos/when_all.cpp                vector / iterator / variadic forms
//   tests/unit/lcos/shared_future.cpp           copies share one result
//   tests/unit/lcos/sliding_semaphore.cpp       wait/signal across threads
//   tests/unit/util/unwrap.cpp                  unwrapping of void / vector / plain
//
// usage: futures
#include <hpx/hpx_init.hpp>
#include <hpx/include/lcos.hpp>
#include <hpx/util/lightweight_test.hpp>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

using hpx::dataflow;
using hpx::future;
using hpx::make_ready_future;
using hpx::shared_future;
using hpx::util::unwrapping;

// ------------------------------------------------- local_dataflow.cpp:37-126
std::atomic<std::uint32_t> void_f_count{0}, int_f_count{0}, void_f1_count{0}, int_f1_count{0}, int_f2_count{0},
    int_f_vector_count{0};
void void_f() { ++void_f_count; }
int int_f() {
    ++int_f_count;
    return 42;
}
void void_f1(int) { ++void_f1_count; }
int int_f1(int i) {
    ++int_f1_count;
    return i + 42;
}
int int_f2(int l, int r) {
    ++int_f2_count;
    return l + r;
}
int int_f_vector(std::vector<int> const& vf) {
    ++int_f_vector_count;
    int sum = 0;
    for (int f : vf) sum += f;
    return sum;
}

void function_pointers() {
    future<void> f1 = dataflow(unwrapping(&void_f1), hpx::async(&int_f));
    future<int> f2 = dataflow(unwrapping(&int_f1), dataflow(unwrapping(&int_f1), make_ready_future(42)));
    future<int> f3 = dataflow(unwrapping(&int_f2), dataflow(unwrapping(&int_f1), make_ready_future(42)),
                              dataflow(unwrapping(&int_f1), make_ready_future(37)));
    std::vector<future<int>> vf;
    for (std::size_t i = 0; i < 10; ++i) vf.push_back(dataflow(unwrapping(&int_f1), make_ready_future(42)));
    future<int> f4 = dataflow(unwrapping(&int_f_vector), std::move(vf));
    future<int> f5 = dataflow(unwrapping(&int_f1), dataflow(unwrapping(&int_f1), make_ready_future(42)),
                              dataflow(unwrapping(&void_f), make_ready_future()));
    f1.wait();
    HPX_TEST_EQ(f2.get(), 126);
    HPX_TEST_EQ(f3.get(), 163);
    HPX_TEST_EQ(f4.get(), 10 * 84);
    HPX_TEST_EQ(f5.get(), 126);
    HPX_TEST_EQ(void_f_count.load(), 1u);
    HPX_TEST_EQ(int_f_count.load(), 1u);
    HPX_TEST_EQ(void_f1_count.load(), 1u);
    HPX_TEST_EQ(int_f1_count.load(), 16u);
    HPX_TEST_EQ(int_f2_count.load(), 1u);
    HPX_TEST_EQ(int_f_vector_count.load(), 1u);
}

// ------------------------------------------------ local_dataflow.cpp:128-225
std::atomic<std::uint32_t> future_void_f1_count{0}, future_void_f2_count{0}, future_int_f1_count{0},
    future_int_f2_count{0};
void future_void_f1(future<void> f1) {
    HPX_TEST(f1.is_ready());
    ++future_void_f1_count;
}
void future_void_sf1(shared_future<void> f1) {
    HPX_TEST(f1.is_ready());
    ++future_void_f1_count;
}
void future_void_f2(future<void> f1, future<void> f2) {
    HPX_TEST(f1.is_ready());
    HPX_TEST(f2.is_ready());
    ++future_void_f2_count;
}
int future_int_f1(future<void> f1) {
    HPX_TEST(f1.is_ready());
    ++future_int_f1_count;
    return 1;
}
int future_int_f2(future<int> f1, future<int> f2) {
    HPX_TEST(f1.is_ready());
    HPX_TEST(f2.is_ready());
    ++future_int_f2_count;
    return f1.get() + f2.get();
}

void future_function_pointers() {
    future<void> f1 = dataflow(&future_void_f1, hpx::async(&future_void_sf1, shared_future<void>(make_ready_future())));
    f1.wait();
    HPX_TEST_EQ(future_void_f1_count.load(), 2u);
    future_void_f1_count = 0;

    future<void> f2 = dataflow(&future_void_f2, hpx::async(&future_void_sf1, shared_future<void>(make_ready_future())),
                               hpx::async(&future_void_sf1, shared_future<void>(make_ready_future())));
    f2.wait();
    HPX_TEST_EQ(future_void_f1_count.load(), 2u);
    HPX_TEST_EQ(future_void_f2_count.load(), 1u);

    future<int> f3 = dataflow(&future_int_f1, make_ready_future());
    HPX_TEST_EQ(f3.get(), 1);
    future<int> f4 = dataflow(&future_int_f2, dataflow(&future_int_f1, make_ready_future()),
                              dataflow(&future_int_f1, make_ready_future()));
    HPX_TEST_EQ(f4.get(), 2);
    HPX_TEST_EQ(future_int_f1_count.load(), 3u);
    HPX_TEST_EQ(future_int_f2_count.load(), 1u);
}

// ------------------------------------------------ local_dataflow.cpp:239-290
void plain_arguments() {
    std::atomic<int> count{0};
    future<void> f1 = dataflow([&](int i) { count += i; }, 42);
    future<int> f2 = dataflow([&](int i) { return i + 42; }, 42);
    f1.wait();
    HPX_TEST_EQ(count.load(), 42);
    HPX_TEST_EQ(f2.get(), 84);
    // mixed: a plain value and a future
    future<int> f3 = dataflow([](int i, future<int> f) { return i + f.get(); }, 42, make_ready_future(84));
    HPX_TEST_EQ(f3.get(), 126);
    // launch policies
    future<int> f4 = dataflow(hpx::launch::sync, unwrapping([](int a, int b) { return a * b; }), make_ready_future(6),
                              make_ready_future(7));
    HPX_TEST_EQ(f4.get(), 42);
    std::atomic<int> deferred_runs{0};
    future<int> f5 = dataflow(hpx::launch::deferred, [&] { return ++deferred_runs; });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    HPX_TEST_EQ(deferred_runs.load(), 0);  // nothing runs it until it is waited for
    HPX_TEST_EQ(f5.get(), 1);
    HPX_TEST_EQ(deferred_runs.load(), 1);
}

// ------------------------------------------------------------ future_then.cpp
void future_then() {
    future<int> f1 = make_ready_future(1);
    future<int> f2 = f1.then([](future<int>&& f) { return f.get() + 1; });
    future<int> f3 = f2.then(hpx::launch::sync, [](future<int> f) { return f.get() * 10; });
    HPX_TEST_EQ(f3.get(), 20);
    // a continuation returning a future is unwrapped
    future<int> f4 = make_ready_future(5).then([](future<int> f) { return make_ready_future(f.get() * 3); });
    HPX_TEST_EQ(f4.get(), 15);
    // a continuation on a shared_future; every copy reads the same value
    shared_future<int> sf = make_ready_future(7).share();
    future<int> c1 = sf.then([](shared_future<int> f) { return f.get() + 1; });
    future<int> c2 = sf.then([](shared_future<int> const& f) { return f.get() + 2; });
    HPX_TEST_EQ(c1.get(), 8);
    HPX_TEST_EQ(c2.get(), 9);
    HPX_TEST_EQ(sf.get(), 7);
    // a dropped continuation still runs (eager, as HPX's)
    std::atomic<int> ran{0};
    {
        future<int> pending = hpx::async([] {
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
            return 3;
        });
        pending.then([&](future<int> f) { ran = f.get(); });
    }
    for (int i = 0; i < 2000 && ran.load() == 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    HPX_TEST_EQ(ran.load(), 3);
    // a long chain of sync continuations does not grow the stack without bound
    future<int> chain = make_ready_future(0);
    hpx::lcos::local::sliding_semaphore gate(0);
    future<void> start = hpx::async([&] { gate.wait(1); });
    future<int> head = start.then(hpx::launch::sync, [](future<void>) { return 0; });
    for (int i = 0; i < 20000; ++i) head = head.then(hpx::launch::sync, [](future<int> f) { return f.get() + 1; });
    gate.signal(1);
    HPX_TEST_EQ(head.get(), 20000);
}

// ------------------------------------------------------------- when_all.cpp
void when_all_forms() {
    std::vector<future<int>> v;
    for (int i = 0; i < 8; ++i) v.push_back(hpx::async([i] { return i * i; }));
    auto all = hpx::when_all(v);  // lvalue range: the futures are moved in
    std::vector<future<int>> got = all.get();
    int s = 0;
    for (auto& f : got) s += f.get();
    HPX_TEST_EQ(s, 140);

    std::vector<shared_future<int>> sv;
    for (int i = 0; i < 4; ++i) sv.push_back(make_ready_future(i + 1).share());
    auto sall = hpx::when_all(sv);  // shared futures are copied: sv stays valid
    auto sgot = sall.get();
    HPX_TEST_EQ(sgot.size(), std::size_t(4));
    HPX_TEST_EQ(sv[3].get() + sgot[0].get(), 5);

    std::vector<future<int>> it;
    for (int i = 0; i < 3; ++i) it.push_back(make_ready_future(10 * i));
    auto iall = hpx::when_all(it.begin(), it.end()).get();
    HPX_TEST_EQ(iall[2].get(), 20);

    future<int> a = hpx::async([] { return 1; });
    shared_future<double> b = make_ready_future(2.5).share();
    future<void> c = make_ready_future();
    auto t = hpx::when_all(a, b, c).get();  // future<tuple<future<int>, shared_future<double>, future<void>>>
    HPX_TEST_EQ(std::get<0>(t).get(), 1);
    HPX_TEST_EQ(std::get<1>(t).get(), 2.5);
    HPX_TEST(std::get<2>(t).is_ready());
    HPX_TEST(!a.valid());  // moved into the group
    HPX_TEST(b.valid());   // copied

    auto e = hpx::when_all().get();
    HPX_TEST_EQ(std::tuple_size<decltype(e)>::value, std::size_t(0));

    // when_all(...).then(...)
    std::vector<future<int>> w;
    for (int i = 0; i < 5; ++i) w.push_back(hpx::async([i] { return i; }));
    future<int> sum = hpx::when_all(std::move(w)).then([](future<std::vector<future<int>>> f) {
        int r = 0;
        for (auto& x : f.get()) r += x.get();
        return r;
    });
    HPX_TEST_EQ(sum.get(), 10);

    // wait_all over futures, shared futures and ranges
    future<int> x = hpx::async([] { return 4; });
    std::vector<shared_future<int>> xs = {hpx::async([] { return 5; }).share(), make_ready_future(6).share()};
    hpx::wait_all(x, xs);
    HPX_TEST(x.is_ready());
    HPX_TEST(xs[0].is_ready() && xs[1].is_ready());
    hpx::wait_all(xs.begin(), xs.end());
    HPX_TEST_EQ(x.get() + xs[0].get() + xs[1].get(), 15);
}

// -------------------------------------------------------- errors propagate
void errors() {
    future<int> bad = hpx::async([]() -> int { throw std::runtime_error("boom"); });
    future<int> down = dataflow(unwrapping([](int v) { return v + 1; }), std::move(bad));
    bool caught = false;
    try {
        down.get();
    } catch (std::runtime_error const& e) {
        caught = std::string(e.what()) == "boom";
    }
    HPX_TEST(caught);
    future<int> ok = hpx::make_exceptional_future<int>(std::logic_error("x"));
    HPX_TEST(ok.has_exception());
    // a moved-out value cannot be read twice
    future<std::vector<int>> vv = make_ready_future(std::vector<int>{1, 2, 3});
    HPX_TEST_EQ(vv.get().size(), std::size_t(3));
    bool second = false;
    try {
        vv.get();
    } catch (hpx::exception const&) {
        second = true;
    }
    HPX_TEST(second);
}

// -------------------------------------------------- sliding_semaphore.cpp
void sliding_semaphore_test() {
    hpx::lcos::local::sliding_semaphore sem(2);
    std::atomic<std::int64_t> reached{0};
    std::thread waiter([&] {
        for (std::int64_t t = 0; t < 10; ++t) {
            sem.wait(t);
            reached = t;
        }
    });
    for (std::int64_t t = 0; t < 10; ++t) {
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
        HPX_TEST(reached.load() <= t + 2);
        sem.signal(t);
    }
    waiter.join();
    HPX_TEST_EQ(reached.load(), std::int64_t(9));
}

int hpx_main(int, char**) {
    function_pointers();
    future_function_pointers();
    plain_arguments();
    future_then();
    when_all_forms();
    errors();
    sliding_semaphore_test();
    const int errs = hpx::util::report_errors();
    if (!errs) std::cout << "futures: all tests passed" << std::endl;
    return errs;
}

int main(int argc, char** argv) { return hpx::init(argc, argv); }
