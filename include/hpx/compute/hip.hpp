// hpx/compute/hip.hpp -- header-only C++ mirror of HPX 1.4.0's hpx::compute
// CUDA layer for the MI355X backend, on top of the C ABI in <hpxhip.h>.
//
//   hpx::compute::hip::target            <- hpx/compute/cuda/target.hpp:36-200,
//                                           src/compute/cuda/cuda_target.cpp:97-317
//   hpx::compute::hip::get_local_targets <- src/compute/cuda/get_cuda_targets.cpp:30-65
//   hpx::compute::hip::allocator<T>      <- hpx/compute/cuda/allocator.hpp:36-259
//   (executors: <hpx/compute/hip/default_executor.hpp>, concurrent_executor.hpp)
//   hpx::compute::vector<T, Alloc>       <- hpx/compute/vector.hpp:28-372
//   device iterator + value_proxy        <- hpx/compute/detail/iterator.hpp:23-85,
//                                           cuda/value_proxy.hpp:25-124
//   completion of device work -> future  <- src/compute/cuda/cuda_target.cpp:97-142
//                                           (futures: <hpx/lcos/future.hpp>)
//
// Compiles with any C++17 host compiler (g++ is enough) and links against
// hpx_amd/libhpxhip.so; there is no host fallback -- a failing call throws.
#pragma once

#include <hpxhip.h>
#include <hpx/exception.hpp>
#include <hpx/exception_list.hpp>
#include <hpx/lcos/future.hpp>
#include <hpx/lcos/when_all.hpp>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <iterator>
#include <memory>
#include <mutex>
#include <new>
#include <ostream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace hpx {

// Errors (hpx::exception, kernel_error, out_of_memory, exception_list) come
// from <hpx/exception.hpp> / <hpx/exception_list.hpp>; futures, when_all and
// the completion engine from <hpx/lcos/future.hpp> / <hpx/lcos/when_all.hpp>.

namespace compute { namespace hip {

namespace detail {
// Per-device resources shared by every target copy of a process: the pinned
// result slots through which reduce / copy_if / for_loop results travel back,
// and a pool of non-blocking streams.  Both outlive any one target, so a
// future never depends on the lifetime of the (often temporary) policy,
// executor or target that launched its work -- the role the intrusive
// refcount pinned across the stream callback plays in the reference
// (cuda_target.cpp:123-142).  Pools live for the whole process (never freed:
// a completion callback may still run during static destruction).
class device_pool {
public:
    static constexpr unsigned kChunkSlots = 256, kSlotBytes = 64;

    static device_pool& get(int device) {
        static std::mutex m;
        static std::vector<device_pool*>* pools = new std::vector<device_pool*>();
        std::lock_guard<std::mutex> lk(m);
        if (device < 0) throw hpx::exception(HPXHIP_ERROR_INVALID_ARGUMENT, "negative device id");
        if (pools->size() <= static_cast<std::size_t>(device)) pools->resize(device + 1, nullptr);
        if (!(*pools)[device]) (*pools)[device] = new device_pool(device);
        return *(*pools)[device];
    }

    struct slot_ref {
        unsigned id;
        void* dev;
        void* host;
    };

    slot_ref acquire() {
        std::lock_guard<std::mutex> lk(mtx_);
        if (free_.empty()) reap();
        if (free_.empty()) grow();
        unsigned id = free_.back();
        free_.pop_back();
        auto const& c = chunks_[id / kChunkSlots];
        std::size_t off = std::size_t(id % kChunkSlots) * kSlotBytes;
        return {id, static_cast<char*>(c.first) + off, static_cast<char*>(c.second) + off};
    }
    // No HIP call: safe from a stream callback.
    void release(unsigned id) {
        std::lock_guard<std::mutex> lk(mtx_);
        free_.push_back(id);
    }
    // A slot whose future was dropped before its work completed: freed (and
    // its event returned) once the event shows the work done.
    void defer_release(unsigned id, hpxhip_event ev) {
        std::lock_guard<std::mutex> lk(mtx_);
        deferred_.emplace_back(id, ev);
    }

    // Device blocks of 2^cls bytes (cls >= 8) for the small per-call arrays of
    // the segmented algorithms (segment totals and carries), kept per size
    // class for the process lifetime like the slots.
    struct block_ref {
        unsigned cls, idx;
        void* dev;
    };
    block_ref acquire_block(std::size_t bytes) {
        unsigned cls = 8;
        while ((std::size_t(1) << cls) < bytes) ++cls;
        std::lock_guard<std::mutex> lk(mtx_);
        auto& fl = block_free_[cls];
        if (fl.empty()) {
            void* d = nullptr;
            check(hpxhip_malloc(device_, &d, std::size_t(1) << cls), "device block");
            blocks_.push_back(d);
            fl.push_back(static_cast<unsigned>(blocks_.size() - 1));
        }
        const unsigned idx = fl.back();
        fl.pop_back();
        return {cls, idx, blocks_[idx]};
    }
    // No HIP call: safe from a stream callback.
    void release_block(block_ref const& b) {
        std::lock_guard<std::mutex> lk(mtx_);
        block_free_[b.cls].push_back(b.idx);
    }
    // The same for pinned host blocks (staging of stream-ordered H2D copies:
    // the bytes must stay valid until the copy has run, so the block returns
    // to the pool from the stream, not when the caller's frame ends).
    block_ref acquire_host_block(std::size_t bytes) {
        unsigned cls = 8;
        while ((std::size_t(1) << cls) < bytes) ++cls;
        std::lock_guard<std::mutex> lk(mtx_);
        auto& fl = host_free_[cls];
        if (fl.empty()) {
            void* h = nullptr;
            check(hpxhip_malloc_host(&h, std::size_t(1) << cls), "pinned block");
            host_blocks_.push_back(h);
            fl.push_back(static_cast<unsigned>(host_blocks_.size() - 1));
        }
        const unsigned idx = fl.back();
        fl.pop_back();
        return {cls, idx, host_blocks_[idx]};
    }
    void release_host_block(block_ref const& b) {
        std::lock_guard<std::mutex> lk(mtx_);
        host_free_[b.cls].push_back(b.idx);
    }

    // HIP events for the early completion of futures (target::async_result)
    hpxhip_event take_event() {
        {
            std::lock_guard<std::mutex> lk(mtx_);
            if (!events_.empty()) {
                hpxhip_event e = events_.back();
                events_.pop_back();
                return e;
            }
        }
        // created on this pool's device (an event is recorded on streams of
        // the device it was created on), without timestamps
        hpxhip_event e = nullptr;
        if (hpxhip_event_create_on(device_, 0, &e) != HPXHIP_SUCCESS) e = nullptr;
        return e;
    }
    void give_event(hpxhip_event e) {
        std::lock_guard<std::mutex> lk(mtx_);
        events_.push_back(e);
    }

    hpxhip_stream take_stream() {
        {
            std::lock_guard<std::mutex> lk(mtx_);
            if (!streams_.empty()) {
                hpxhip_stream s = streams_.back();
                streams_.pop_back();
                return s;
            }
        }
        hpxhip_stream s = nullptr;
        check(hpxhip_stream_create(device_, &s), "hpxhip_stream_create");
        return s;
    }
    // A stream handed back may still have queued work: whoever takes it next
    // is ordered behind that work, which is at least as strong as the
    // reference's destroy-while-busy (cudaStreamDestroy returns at once).
    // Pooled streams are never destroyed: a completion's event may be queried
    // or waited on long after the stream it was recorded on went back to the
    // pool, and HIP reads that stream's state then (a destroyed one reported
    // "event last recorded in a capturing stream").  The pool holds at most as
    // many streams as targets were ever alive at once.
    void give_stream(hpxhip_stream s) {
        std::lock_guard<std::mutex> lk(mtx_);
        streams_.push_back(s);
    }

private:
    explicit device_pool(int device) : device_(device) {}
    void reap() {  // called with mtx_ held
        for (std::size_t i = 0; i < deferred_.size();) {
            if (hpxhip_event_query(deferred_[i].second) == HPXHIP_SUCCESS) {
                free_.push_back(deferred_[i].first);
                events_.push_back(deferred_[i].second);
                deferred_[i] = deferred_.back();
                deferred_.pop_back();
            } else {
                ++i;
            }
        }
    }
    void grow() {  // called with mtx_ held
        void* d = nullptr;
        void* h = nullptr;
        check(hpxhip_malloc(device_, &d, std::size_t(kChunkSlots) * kSlotBytes), "result slots");
        int rc = hpxhip_malloc_host(&h, std::size_t(kChunkSlots) * kSlotBytes);
        if (rc != HPXHIP_SUCCESS) {
            hpxhip_free(d);
            check(rc, "result slots");
        }
        unsigned base = static_cast<unsigned>(chunks_.size()) * kChunkSlots;
        chunks_.emplace_back(d, h);
        for (unsigned i = kChunkSlots; i-- > 0;) free_.push_back(base + i);
    }

    int device_;
    std::mutex mtx_;
    std::vector<std::pair<void*, void*>> chunks_;  // (device, pinned host) per chunk
    std::vector<unsigned> free_;
    std::vector<hpxhip_stream> streams_;
    std::vector<hpxhip_event> events_;
    std::vector<std::pair<unsigned, hpxhip_event>> deferred_;
    std::vector<void*> blocks_, host_blocks_;
    std::vector<unsigned> block_free_[64], host_free_[64];
};

// Host waits taken by stream ordering because the runtime refused a
// device-side one (tests assert it stays 0).
inline std::atomic<unsigned long>& stream_order_host_waits() {
    static std::atomic<unsigned long> n{0};
    return n;
}

// Run fn (no HIP calls: it runs on the HIP callback thread) once the work
// queued on s so far is done.
inline void on_stream_done(hpxhip_stream s, std::function<void()> fn) {
    auto* p = new std::function<void()>(std::move(fn));
    int rc = hpxhip_stream_add_callback(
        s,
        [](void* u, int) {
            auto* f = static_cast<std::function<void()>*>(u);
            (*f)();
            delete f;
        },
        p);
    if (rc != HPXHIP_SUCCESS) {
        delete p;
        check(rc, "hpxhip_stream_add_callback");
    }
}

// A mark behind the work queued on a stream so far: a pooled event of the
// stream's own device recorded there (an event is recorded on streams of the
// device it was created on; hipStreamWaitEvent accepts an event of another
// device).  wait_on(after) makes `after` wait for it on the device, so a
// cross-device hand-off -- a segmented carry, a stencil halo -- costs the
// host two enqueues, not a wait (segmented_algorithms/reduce.hpp:191-207
// chains the same dependencies through futures).  A wait captures the
// event's state when it is enqueued, so the event may be re-recorded or go
// back to the pool right after.  Only if the runtime refuses the record does
// wait_on() fall back to a host wait for the stream.
class stream_mark {
    hpxhip_stream s_ = nullptr;
    device_pool* pool_ = nullptr;
    hpxhip_event ev_ = nullptr;

public:
    explicit stream_mark(hpxhip_stream s) : s_(s) {
        int dev = 0;
        check(hpxhip_stream_device(s, &dev), "stream ordering");
        pool_ = &device_pool::get(dev);
        ev_ = pool_->take_event();
        if (ev_ && hpxhip_event_record(ev_, s) != HPXHIP_SUCCESS) {
            pool_->give_event(ev_);
            ev_ = nullptr;
        }
    }
    stream_mark(stream_mark&& o) noexcept : s_(o.s_), pool_(o.pool_), ev_(o.ev_) { o.ev_ = nullptr; }
    stream_mark(stream_mark const&) = delete;
    stream_mark& operator=(stream_mark const&) = delete;
    stream_mark& operator=(stream_mark&&) = delete;
    ~stream_mark() {
        if (ev_) pool_->give_event(ev_);
    }
    void wait_on(hpxhip_stream after) const {
        if (after == s_) return;
        if (ev_) {
            check(hpxhip_stream_wait_event(after, ev_), "stream ordering");
            return;
        }
        stream_order_host_waits().fetch_add(1);
        check(hpxhip_stream_synchronize(s_), "stream ordering");
    }
};

// `after` waits (on the device) for the work queued on `before` so far.
inline void stream_after(hpxhip_stream after, hpxhip_stream before) {
    if (after == before) return;
    stream_mark(before).wait_on(after);
}
}  // namespace detail

// One 64-byte (device, pinned host) result slot, returned to its device pool
// when the owner goes away.  Algorithms queue `kernel -> D2H copy into host()`
// and hand the slot to the completion (target::async_result), which copies
// the bytes into the future's shared state before releasing it.
class result_slot {
    detail::device_pool* pool_ = nullptr;
    detail::device_pool::slot_ref ref_{};

public:
    result_slot() = default;
    result_slot(detail::device_pool& p) : pool_(&p), ref_(p.acquire()) {}
    result_slot(result_slot&& o) noexcept : pool_(o.pool_), ref_(o.ref_) { o.pool_ = nullptr; }
    result_slot& operator=(result_slot&& o) noexcept {
        if (this != &o) {
            reset();
            pool_ = o.pool_;
            ref_ = o.ref_;
            o.pool_ = nullptr;
        }
        return *this;
    }
    result_slot(result_slot const&) = delete;
    result_slot& operator=(result_slot const&) = delete;
    ~result_slot() { reset(); }

    explicit operator bool() const { return pool_ != nullptr; }
    void* device() const { return ref_.dev; }
    void const* host() const { return ref_.host; }
    void reset() {
        if (pool_) pool_->release(ref_.id);
        pool_ = nullptr;
    }
    // ownership moves to a completion callback (released there)
    std::pair<detail::device_pool*, detail::device_pool::slot_ref> detach() {
        auto r = std::make_pair(pool_, ref_);
        pool_ = nullptr;
        return r;
    }
};

// ------------------------------------------------------------------ target
class target {
    struct handle {
        int device = 0;
        hpxhip_stream stream = nullptr;
        std::mutex mtx;  // lazy stream creation, cuda_target.cpp:257 spinlock
        ~handle() {
            // the stream goes back to the device pool, queued work and all
            if (stream) detail::device_pool::get(device).give_stream(stream);
        }
    };
    std::shared_ptr<handle> h_;

    // Completion of an async_result future, run once: by a get() that
    // waited on the event recorded behind the work, by is_ready() finding
    // the event complete, or by the completion engine polling the event --
    // registered only when a continuation needs it (arm).  Completion copies the result slot's
    // bytes into the state and returns the slot to its pool (the work is
    // done by then); a future dropped before completion hands its slot and
    // event to the pool, which frees them once the event has fired.
    template <typename S>
    struct completion final : lcos::detail::early_completion, std::enable_shared_from_this<completion<S>> {
        S* st = nullptr;  // kept alive by the future, and by an armed callback's reference
        detail::device_pool* pool = nullptr;
        detail::device_pool::slot_ref slot{};
        std::function<void(unsigned char const*)> on_ready;
        hpxhip_event ev = nullptr;
        hpxhip_stream stream = nullptr;
        int device = 0;
        std::mutex m;
        bool done = false, armed = false;

        void complete(int status) {
            bool first = false;
            {
                std::lock_guard<std::mutex> lk(m);
                if (!done) {
                    done = first = true;
                    if (pool) {
                        std::memcpy(st->raw, slot.host, sizeof(st->raw));
                        pool->release(slot.id);
                        pool = nullptr;
                    }
                    if (status == 0 && on_ready) on_ready(st->raw);
                }
            }
            if (first) st->set_ready(status);
        }
        // A failing event wait (a faulted kernel: sticky HIP error) readies
        // the future with that status, so get() reports it through the
        // algorithm's error mapping (exception_list) and a second get()
        // returns the same error.
        void wait_and_complete() override {
            {
                std::lock_guard<std::mutex> lk(m);
                if (done) return;
            }
            if (!ev) return;  // armed at creation: the callback completes it
            complete(hpxhip_event_synchronize(ev));
        }
        bool try_complete() override {
            {
                std::lock_guard<std::mutex> lk(m);
                if (done) return true;
            }
            if (!ev) return false;
            const int rc = hpxhip_event_query(ev);
            if (rc == HPXHIP_ERROR_NOT_READY) return false;
            complete(rc);
            return true;
        }
        // Complete without a waiter: the completion engine polls the event
        // (its thread may run continuations that call HIP).  Without an event
        // (its creation failed) a stream callback posts the completion to the
        // engine, so no continuation runs on HIP's callback thread.  Both
        // hold the state (keep) and this completion until it has run.
        void arm(std::shared_ptr<void> keep) override {
            {
                std::lock_guard<std::mutex> lk(m);
                if (done || armed) return;
                armed = true;
            }
            auto self = this->shared_from_this();
            if (ev) {
                lcos::detail::engine::get().watch(ev, [self, keep](int rc) { self->complete(rc); });
                return;
            }
            struct box {
                std::shared_ptr<void> keep;
                std::shared_ptr<completion> c;
            };
            auto* b = new box{std::move(keep), self};
            int rc = hpxhip_stream_add_callback(
                stream,
                [](void* p, int status) {
                    auto* bp = static_cast<box*>(p);
                    lcos::detail::engine::get().post([bp, status] {
                        bp->c->complete(status);
                        delete bp;
                    });
                },
                b);
            if (rc != HPXHIP_SUCCESS) {
                delete b;
                complete(rc);
            }
        }
        ~completion() override {
            if (pool) {  // never completed: the work may still write the slot
                if (ev) {
                    pool->defer_release(slot.id, ev);
                    ev = nullptr;
                } else {
                    pool->release(slot.id);  // no event was recorded: the callback path completed or never queued
                }
            }
            if (ev) detail::device_pool::get(device).give_event(ev);
        }
    };

    explicit target(std::shared_ptr<handle> h) noexcept : h_(std::move(h)) {}

public:
    target() : target(0) {}
    explicit target(int device) : h_(std::make_shared<handle>()) { h_->device = device; }
    // a copy gets its own stream (cuda_target.cpp:203-211)
    target(target const& o) : h_(std::make_shared<handle>()) { h_->device = o.h_->device; }
    target& operator=(target const& o) {
        if (this != &o) {
            h_ = std::make_shared<handle>();
            h_->device = o.h_->device;
        }
        return *this;
    }
    // A move shares the handle (same stream) instead of leaving the source
    // without one: a moved-from target stays usable (device(), stream(),
    // synchronize()), and iterators that share the handle stay valid.
    target(target&& o) noexcept : h_(o.h_) {}
    target& operator=(target&& o) noexcept {
        h_ = o.h_;
        return *this;
    }
    // A view of the same handle and stream (not a copy: no new stream).
    // Device iterators hold one, so they do not point into the object that
    // handed them out (a vector moved after begin() was taken).
    static target shared(target const& o) noexcept { return target(o.h_); }

    struct native_handle_type;
    // A non-owning view of a handle: same device and stream, no reference
    // count (an aliasing shared_ptr without a control block), so copying it
    // costs a pointer copy.  Device iterators and value proxies hold one; it
    // stays valid while a target that owns the handle lives (the container's
    // allocator), as the reference's target_ptr does (target_ptr.hpp:63-65).
    static target view(native_handle_type nh);
    static target view(target const& o) noexcept { return target(std::shared_ptr<handle>(std::shared_ptr<handle>(), o.h_.get())); }

    struct native_handle_type {
        handle* h;
        int get_device() const { return h->device; }
        hpxhip_stream get_stream() const {
            std::lock_guard<std::mutex> lk(h->mtx);
            if (!h->stream) h->stream = detail::device_pool::get(h->device).take_stream();
            return h->stream;
        }
        std::size_t processing_units() const {
            hpxhip_device_props p;
            detail::check(hpxhip_device_props_get(h->device, &p), "hpxhip_device_props_get");
            return static_cast<std::size_t>(p.compute_units);
        }
    };
    native_handle_type native_handle() const { return native_handle_type{h_.get()}; }
    int device() const { return h_->device; }
    hpxhip_stream stream() const { return native_handle().get_stream(); }

    void synchronize() const {
        detail::check(hpxhip_stream_synchronize(stream()), "hpxhip_stream_synchronize");
        uint32_t code = 0;
        detail::check(hpxhip_device_error(h_->device, &code), "hpxhip_device_error");
        if (code) throw kernel_error(HPXHIP_ERROR_DEVICE_TIMEOUT, "device kernel error word set");
    }

    // cuda_target.cpp:307-317: a future that becomes ready when all work queued
    // so far on the stream is done; completed from the HIP callback thread.
    future<void> get_future() const {
        return async_result<void>([](unsigned char const*) {});
    }

    // A future completed once all work queued so far is done.  A HIP event
    // is recorded behind the work; get() waits on it and completes the state
    // itself, is_ready() queries it, and only a continuation (then,
    // when_all) registers a host callback (r04: registering one per call and
    // waiting for its hand-off had cost ~20 of the ~31 us of a par(task) +
    // get(), profiles/r03_cxx_call_overhead.log).  Completion copies the
    // result slot's bytes into the shared state, returns the slot, then
    // on_ready(bytes) runs (no HIP calls: it may run on the callback thread;
    // e.g. a for_loop reduction folding its view into the live-out variable,
    // for_loop_reduction.hpp:60-66) and the state becomes ready.
    // value(bytes) runs on the first get(), after the device error word is
    // checked.
    template <typename R>
    future<R> async_result(std::function<R(unsigned char const*)> value, result_slot slot = {},
                           std::function<void(unsigned char const*)> on_ready = {}) const {
        using S = lcos::detail::shared_state<R>;
        auto st = std::make_shared<S>();
        int dev = h_->device;
        S* self = st.get();  // value_fn is owned by the state it reads
        st->value_fn = [dev, self, value = std::move(value)]() -> R {
            uint32_t code = 0;
            detail::check(hpxhip_device_error(dev, &code), "hpxhip_device_error");
            if (code) throw kernel_error(HPXHIP_ERROR_DEVICE_TIMEOUT, "device kernel error word set");
            return value(self->raw);
        };
        hpxhip_stream s = stream();
        auto c = std::make_shared<completion<S>>();
        c->st = st.get();
        c->on_ready = std::move(on_ready);
        c->device = dev;
        c->stream = s;
        if (slot) {
            auto d = slot.detach();
            c->pool = d.first;
            c->slot = d.second;
        }
        c->ev = detail::device_pool::get(dev).take_event();
        if (c->ev && hpxhip_event_record(c->ev, s) != HPXHIP_SUCCESS) {
            detail::device_pool::get(dev).give_event(c->ev);
            c->ev = nullptr;
        }
        if (!c->ev) c->arm(st);  // no event: only the callback can complete it
        st->early = c;
        return future<R>(st);
    }

    // A (device, pinned host) slot from this device's pool; see result_slot.
    result_slot make_result_slot() const { return result_slot(detail::device_pool::get(h_->device)); }

    std::size_t processing_units() const { return native_handle().processing_units(); }

    friend bool operator==(target const& a, target const& b) { return a.h_->device == b.h_->device; }
    friend bool operator!=(target const& a, target const& b) { return !(a == b); }
};
inline target target::view(native_handle_type nh) {
    if (!nh.h) return target(0);  // a default-constructed iterator: device 0
    return target(std::shared_ptr<handle>(std::shared_ptr<handle>(), nh.h));
}
inline std::vector<target> get_local_targets() {
    int n = 0;
    detail::check(hpxhip_get_device_count(&n), "hpxhip_get_device_count");
    std::vector<target> ts;
    for (int i = 0; i < n; ++i) ts.emplace_back(i);
    return ts;
}

template <typename T>
struct dtype_of;
template <> struct dtype_of<int32_t> { static constexpr int value = HPXHIP_I32; };
template <> struct dtype_of<uint32_t> { static constexpr int value = HPXHIP_U32; };
template <> struct dtype_of<int64_t> { static constexpr int value = HPXHIP_I64; };
template <> struct dtype_of<uint64_t> { static constexpr int value = HPXHIP_U64; };
template <> struct dtype_of<float> { static constexpr int value = HPXHIP_F32; };
template <> struct dtype_of<double> { static constexpr int value = HPXHIP_F64; };
#if defined(__LP64__) && !defined(_WIN32)
template <> struct dtype_of<long long> { static constexpr int value = HPXHIP_I64; };
template <> struct dtype_of<unsigned long long> { static constexpr int value = HPXHIP_U64; };
#endif

// --------------------------------------------------------------- allocator
template <typename T>
class allocator {
    hip::target target_;

public:
    using value_type = T;
    using pointer = T*;
    using const_pointer = T const*;
    using size_type = std::size_t;
    using difference_type = std::ptrdiff_t;
    using target_type = hip::target;
    template <typename U>
    struct rebind {
        using other = allocator<U>;
    };

    allocator() = default;
    explicit allocator(hip::target const& t) : target_(t) {}
    template <typename U>
    allocator(allocator<U> const& o) : target_(o.target()) {}

    target_type const& target() const { return target_; }

    pointer allocate(size_type n) {
        void* p = nullptr;
        detail::check(hpxhip_malloc(target_.device(), &p, n * sizeof(T)), "hip::allocator::allocate");
        return static_cast<pointer>(p);
    }
    void deallocate(pointer p, size_type) {
        if (p) hpxhip_free(p);
    }
    size_type max_size() const {
        size_t free_b = 0, total = 0;
        detail::check(hpxhip_mem_info(target_.device(), &free_b, &total), "hip::allocator::max_size");
        return total / sizeof(T);
    }
    // Documented deviation: bulk_construct value-initialises on the device
    // (the reference's host path leaves memory uninitialised, allocator.hpp:173-195).
    void bulk_construct(pointer p, size_type n, T const& v = T()) {
        if (!n) return;
        detail::check(hpxhip_fill(dtype_of<T>::value, &v, p, n, target_.stream()), "hip::allocator::bulk_construct");
        target_.synchronize();
    }
    void bulk_destroy(pointer, size_type) {}  // trivially destructible element types only
};

// --------------------------------------------------------- device iterator
// value_proxy.hpp:25-124: element access from the host, one copy each way.
// Holds a view of the container's target handle (not a pointer into the
// iterator that made it), so a proxy outlives a temporary iterator.
template <typename T>
class value_proxy {
    T* p_;
    hip::target t_;  // non-owning view (target::view)

public:
    value_proxy(T* p, hip::target t) : p_(p), t_(std::move(t)) {}
    operator T() const {
        T v;
        detail::check(hpxhip_memcpy_async(&v, p_, sizeof(T), HPXHIP_D2H, t_.stream()), "value_proxy read");
        t_.synchronize();
        return v;
    }
    value_proxy& operator=(T const& v) {
        detail::check(hpxhip_memcpy_async(p_, &v, sizeof(T), HPXHIP_H2D, t_.stream()), "value_proxy write");
        t_.synchronize();
        return *this;
    }
    friend std::ostream& operator<<(std::ostream& os, value_proxy const& v) { return os << T(v); }
};

// Holds the container's target handle by raw pointer (a native handle), not
// a pointer to the container's target object: iterators stay valid when the
// container is moved, as std::vector's do, while the data lives.  Trivially
// copyable (a copy is two pointers, no reference count, no new stream), so a
// device closure may capture one.
template <typename T>
class device_iterator {
    T* p_ = nullptr;
    hip::target::native_handle_type h_{nullptr};  // null: device 0

public:
    using iterator_category = std::random_access_iterator_tag;
    using value_type = T;
    using difference_type = std::ptrdiff_t;
    using pointer = T*;
    using reference = value_proxy<T>;
    using target_type = hip::target;

    device_iterator() = default;
    device_iterator(T* p, hip::target const& t) : p_(p), h_(t.native_handle()) {}
    T* device_ptr() const { return p_; }
    // a non-owning view of the container's target (same stream)
    hip::target target() const { return hip::target::view(h_); }

    reference operator*() const { return reference(p_, target()); }
    reference operator[](difference_type i) const { return reference(p_ + i, target()); }
    device_iterator& operator++() { ++p_; return *this; }
    device_iterator operator++(int) { auto r = *this; ++p_; return r; }
    device_iterator& operator--() { --p_; return *this; }
    device_iterator& operator+=(difference_type n) { p_ += n; return *this; }
    device_iterator& operator-=(difference_type n) { p_ -= n; return *this; }
    friend device_iterator operator+(device_iterator a, difference_type n) { return a += n; }
    friend device_iterator operator+(difference_type n, device_iterator a) { return a += n; }
    friend device_iterator operator-(device_iterator a, difference_type n) { return a -= n; }
    friend difference_type operator-(device_iterator const& a, device_iterator const& b) { return a.p_ - b.p_; }
    friend bool operator==(device_iterator const& a, device_iterator const& b) { return a.p_ == b.p_; }
    friend bool operator!=(device_iterator const& a, device_iterator const& b) { return a.p_ != b.p_; }
    friend bool operator<(device_iterator const& a, device_iterator const& b) { return a.p_ < b.p_; }
};

template <typename It>
struct is_device_iterator : std::false_type {};
template <typename T>
struct is_device_iterator<device_iterator<T>> : std::true_type {};

}}  // namespace compute::hip

namespace compute {

// ------------------------------------------------------------------ vector
template <typename T, typename Allocator = hip::allocator<T>>
class vector {
    Allocator alloc_;
    std::size_t size_ = 0;
    T* data_ = nullptr;

public:
    using value_type = T;
    using allocator_type = Allocator;
    using size_type = std::size_t;
    using iterator = hip::device_iterator<T>;
    using const_iterator = hip::device_iterator<T>;

    vector() = default;
    explicit vector(size_type n, Allocator const& a = Allocator()) : alloc_(a), size_(n) {
        data_ = alloc_.allocate(n);
        alloc_.bulk_construct(data_, n);
    }
    vector(size_type n, T const& v, Allocator const& a = Allocator()) : alloc_(a), size_(n) {
        data_ = alloc_.allocate(n);
        alloc_.bulk_construct(data_, n, v);
    }
    vector(vector const&) = delete;
    vector& operator=(vector const&) = delete;
    // the allocator (and its target's handle) moves with the data: iterators
    // taken before the move keep the same target and stream
    vector(vector&& o) noexcept : alloc_(std::move(o.alloc_)), size_(o.size_), data_(o.data_) {
        o.data_ = nullptr;
        o.size_ = 0;
    }
    vector& operator=(vector&& o) noexcept {
        if (this != &o) {
            if (data_) alloc_.deallocate(data_, size_);
            alloc_ = std::move(o.alloc_);
            size_ = o.size_;
            data_ = o.data_;
            o.data_ = nullptr;
            o.size_ = 0;
        }
        return *this;
    }
    ~vector() {
        if (data_) alloc_.deallocate(data_, size_);
    }

    size_type size() const { return size_; }
    size_type capacity() const { return size_; }
    bool empty() const { return size_ == 0; }
    T* device_data() const { return data_; }
    T* data() const { return data_; }
    allocator_type const& get_allocator() const { return alloc_; }
    iterator begin() const { return iterator(data_, alloc_.target()); }
    iterator end() const { return iterator(data_ + size_, alloc_.target()); }
    hip::value_proxy<T> operator[](size_type i) const {
        return hip::value_proxy<T>(data_ + i, hip::target::view(alloc_.target()));
    }
};

}  // namespace compute
}  // namespace hpx
