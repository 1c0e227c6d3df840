// internal.hpp -- host-side helpers shared by the C-ABI translation units:
// enum -> type/functor dispatch, launch geometry, the per-stream scratch
// cache and the device error word.
#pragma once

#include <hpxhip/kernels/common.hpp>
#include "../../include/hpxhip.h"

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <type_traits>

namespace hpxhip {

#define HPXHIP_CHECK(expr)                                  \
    do {                                                    \
        hipError_t e_ = (expr);                             \
        if (e_ != hipSuccess) return static_cast<int>(e_);  \
    } while (0)

#define HPXHIP_CHECK_LAUNCH()                               \
    do {                                                    \
        hipError_t e_ = hipGetLastError();                  \
        if (e_ != hipSuccess) return static_cast<int>(e_);  \
    } while (0)

// ------------------------------------------------------------ annotation
// HPX names the work of each algorithm for its tracers (annotate_function,
// hpx/util/annotated_function.hpp:38-115, used per chunk in
// for_each.hpp:173 and transform.hpp:133).  Here each C-ABI algorithm call
// is one roctx range ("hpxhip_scan", ...) on the calling host thread, around
// the enqueue of its kernels -- visible with `rocprofv3 --marker-trace`.
// Off unless HPXHIP_ROCTX=1; the roctx library is then dlopen'ed, so the
// library has no link-time dependency on the profiler.
bool roctx_enabled();
void roctx_push(const char* name);
void roctx_pop();
struct annotate {
    bool on;
    explicit annotate(const char* name) : on(roctx_enabled()) {
        if (on) roctx_push(name);
    }
    ~annotate() {
        if (on) roctx_pop();
    }
    annotate(const annotate&) = delete;
    annotate& operator=(const annotate&) = delete;
};
// Fault injection (hpxhip_debug_inject_error): the injected status, taken by
// the next algorithm entry on this thread.
extern thread_local int g_inject_status;
extern thread_local int g_inject_count;
extern thread_local int g_event_inject_status;  // hpxhip_debug_inject_event_error
extern thread_local int g_event_inject_count;
inline int take_injected_error() {
    if (__builtin_expect(g_inject_count == 0, 1)) return 0;
    --g_inject_count;
    return g_inject_status;
}
// Every C-ABI algorithm entry starts with this: its roctx range, then an
// injected failure if one is pending.
#define HPXHIP_ANNOTATE(name)                              \
    ::hpxhip::annotate hpxhip_annotate_(name);             \
    if (int injected_ = ::hpxhip::take_injected_error())   \
        return injected_

template <typename T>
struct tag {
    using type = T;
};

// ---------------------------------------------------------------- dtypes
template <typename F>
int with_dtype(int dt, F&& f) {
    switch (dt) {
        case HPXHIP_I32: return f(tag<int32_t>{});
        case HPXHIP_U32: return f(tag<uint32_t>{});
        case HPXHIP_I64: return f(tag<int64_t>{});
        case HPXHIP_U64: return f(tag<uint64_t>{});
        case HPXHIP_F32: return f(tag<float>{});
        case HPXHIP_F64: return f(tag<double>{});
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

inline size_t dtype_size(int dt) {
    switch (dt) {
        case HPXHIP_I32:
        case HPXHIP_U32:
        case HPXHIP_F32: return 4;
        case HPXHIP_I64:
        case HPXHIP_U64:
        case HPXHIP_F64: return 8;
        default: return 0;
    }
}

template <typename T>
constexpr int dtype_of() {
    if constexpr (std::is_same_v<T, int32_t>) return HPXHIP_I32;
    else if constexpr (std::is_same_v<T, uint32_t>) return HPXHIP_U32;
    else if constexpr (std::is_same_v<T, int64_t>) return HPXHIP_I64;
    else if constexpr (std::is_same_v<T, uint64_t>) return HPXHIP_U64;
    else if constexpr (std::is_same_v<T, float>) return HPXHIP_F32;
    else return HPXHIP_F64;
}

// Accumulator / compute dtype for a given input dtype: the same type, or a
// widening to int64 (integers) / double (everything).
template <typename TI, typename F>
int with_wide_dtype(int dt, F&& f) {
    if (dt == dtype_of<TI>()) return f(tag<TI>{});
    if constexpr (std::is_integral_v<TI>) {
        if (dt == HPXHIP_I64) return f(tag<int64_t>{});
    }
    if (dt == HPXHIP_F64) return f(tag<double>{});
    return HPXHIP_ERROR_UNSUPPORTED;
}

// ------------------------------------------------------------ operators
template <typename T, typename F>
int with_binop(int op, F&& f) {
    switch (op) {
        case HPXHIP_PLUS: return f(op_plus{});
        case HPXHIP_MULTIPLIES: return f(op_multiplies{});
        case HPXHIP_MIN: return f(op_min{});
        case HPXHIP_MAX: return f(op_max{});
        case HPXHIP_BIT_AND:
        case HPXHIP_BIT_OR:
        case HPXHIP_BIT_XOR:
            if constexpr (std::is_integral_v<T>) {
                if (op == HPXHIP_BIT_AND) return f(op_bit_and{});
                if (op == HPXHIP_BIT_OR) return f(op_bit_or{});
                return f(op_bit_xor{});
            } else {
                return HPXHIP_ERROR_UNSUPPORTED;
            }
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

// Unary element functors (hpxhip_unary).  C is the compute type.
template <int KIND, typename C>
struct unary_fn {
    C s0, s1;
    __host__ __device__ __forceinline__ C operator()(C x) const {
        if constexpr (KIND == HPXHIP_U_IDENTITY) return x;
        else if constexpr (KIND == HPXHIP_U_SCALE) return wrap_mul(x, s0);
        else if constexpr (KIND == HPXHIP_U_ADD_SCALAR) return wrap_add(x, s0);
        else if constexpr (KIND == HPXHIP_U_AFFINE) return wrap_add(wrap_mul(x, s0), s1);
        else if constexpr (KIND == HPXHIP_U_NEGATE) {
            if constexpr (std::is_integral_v<C>) return wrap_mul(x, static_cast<C>(-1));
            else return -x;
        } else if constexpr (KIND == HPXHIP_U_ABS) {
            if constexpr (std::is_unsigned_v<C>) return x;
            else if constexpr (std::is_integral_v<C>) return x < 0 ? wrap_mul(x, static_cast<C>(-1)) : x;
            else return __builtin_fabs(x);
        } else return wrap_mul(x, x);  // SQUARE
    }
};

template <typename C, typename F>
int with_unary(int kind, const void* scalars, F&& f) {
    C s[2] = {C(0), C(0)};
    if (scalars) __builtin_memcpy(s, scalars, 2 * sizeof(C));
    switch (kind) {
        case HPXHIP_U_IDENTITY: return f(unary_fn<HPXHIP_U_IDENTITY, C>{s[0], s[1]});
        case HPXHIP_U_SCALE: return f(unary_fn<HPXHIP_U_SCALE, C>{s[0], s[1]});
        case HPXHIP_U_ADD_SCALAR: return f(unary_fn<HPXHIP_U_ADD_SCALAR, C>{s[0], s[1]});
        case HPXHIP_U_AFFINE: return f(unary_fn<HPXHIP_U_AFFINE, C>{s[0], s[1]});
        case HPXHIP_U_NEGATE: return f(unary_fn<HPXHIP_U_NEGATE, C>{s[0], s[1]});
        case HPXHIP_U_ABS: return f(unary_fn<HPXHIP_U_ABS, C>{s[0], s[1]});
        case HPXHIP_U_SQUARE: return f(unary_fn<HPXHIP_U_SQUARE, C>{s[0], s[1]});
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

// Binary element functors (hpxhip_binary).
template <int KIND, typename C>
struct binary_fn {
    C s0;
    __host__ __device__ __forceinline__ C operator()(C x, C y) const {
        if constexpr (KIND == HPXHIP_B_ADD) return wrap_add(x, y);
        else if constexpr (KIND == HPXHIP_B_TRIAD) return wrap_add(x, wrap_mul(y, s0));
        else if constexpr (KIND == HPXHIP_B_SUB) {
            if constexpr (std::is_integral_v<C>) {
                using U = std::make_unsigned_t<C>;
                return static_cast<C>(static_cast<U>(x) - static_cast<U>(y));
            } else return x - y;
        } else if constexpr (KIND == HPXHIP_B_MUL) return wrap_mul(x, y);
        else if constexpr (KIND == HPXHIP_B_AXPY) return wrap_add(wrap_mul(x, s0), y);
        else if constexpr (KIND == HPXHIP_B_MIN) return (y < x) ? y : x;
        else return (x < y) ? y : x;  // MAX
    }
};

template <typename C, typename F>
int with_binary(int kind, const void* scalars, F&& f) {
    C s = C(0);
    if (scalars) __builtin_memcpy(&s, scalars, sizeof(C));
    switch (kind) {
        case HPXHIP_B_ADD: return f(binary_fn<HPXHIP_B_ADD, C>{s});
        case HPXHIP_B_TRIAD: return f(binary_fn<HPXHIP_B_TRIAD, C>{s});
        case HPXHIP_B_SUB: return f(binary_fn<HPXHIP_B_SUB, C>{s});
        case HPXHIP_B_MUL: return f(binary_fn<HPXHIP_B_MUL, C>{s});
        case HPXHIP_B_AXPY: return f(binary_fn<HPXHIP_B_AXPY, C>{s});
        case HPXHIP_B_MIN: return f(binary_fn<HPXHIP_B_MIN, C>{s});
        case HPXHIP_B_MAX: return f(binary_fn<HPXHIP_B_MAX, C>{s});
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

// Predicates (hpxhip_pred).
template <int KIND, typename T>
struct pred_fn {
    T a;
    __host__ __device__ __forceinline__ bool operator()(T x) const {
        if constexpr (KIND == HPXHIP_P_LT) return x < a;
        else if constexpr (KIND == HPXHIP_P_LE) return x <= a;
        else if constexpr (KIND == HPXHIP_P_GT) return x > a;
        else if constexpr (KIND == HPXHIP_P_GE) return x >= a;
        else if constexpr (KIND == HPXHIP_P_EQ) return x == a;
        else if constexpr (KIND == HPXHIP_P_NE) return x != a;
        else if constexpr (KIND == HPXHIP_P_NOT_LT) return !(x < a);
        else {
            if constexpr (std::is_integral_v<T>) return (x & a) != 0;
            else return false;
        }
    }
};

template <typename T, typename F>
int with_pred(int kind, const void* arg, F&& f) {
    T a = T(0);
    if (arg) __builtin_memcpy(&a, arg, sizeof(T));
    switch (kind) {
        case HPXHIP_P_LT: return f(pred_fn<HPXHIP_P_LT, T>{a});
        case HPXHIP_P_LE: return f(pred_fn<HPXHIP_P_LE, T>{a});
        case HPXHIP_P_GT: return f(pred_fn<HPXHIP_P_GT, T>{a});
        case HPXHIP_P_GE: return f(pred_fn<HPXHIP_P_GE, T>{a});
        case HPXHIP_P_EQ: return f(pred_fn<HPXHIP_P_EQ, T>{a});
        case HPXHIP_P_NE: return f(pred_fn<HPXHIP_P_NE, T>{a});
        case HPXHIP_P_NOT_LT: return f(pred_fn<HPXHIP_P_NOT_LT, T>{a});
        case HPXHIP_P_BITS:
            if constexpr (std::is_integral_v<T>) return f(pred_fn<HPXHIP_P_BITS, T>{a});
            else return HPXHIP_ERROR_UNSUPPORTED;
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

// ------------------------------------------------------------ geometry
struct device_info {
    int cus = 256;
    int device = 0;
};
// Cached per-device properties (compute units etc).
const device_info& current_device_info();
int stream_device(hipStream_t s, int* device);

// Makes the stream's device current for the scope of an entry point (a
// thread may drive several targets, as hpx::compute::cuda::target does via
// scoped_active_target, scoped_active_target.hpp:24-90).
struct device_guard {
    int prev = -1;
    int dev = 0;
    int status = 0;
    explicit device_guard(hipStream_t s) {
        status = stream_device(s, &dev);
        if (status != 0) return;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        if (cur != dev) {
            prev = cur;
            status = static_cast<int>(hipSetDevice(dev));
        }
    }
    ~device_guard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Elements needed to bring `p` to a 16-byte boundary (in units of elem_size).
inline uint64_t head_to_align16(const void* p, size_t elem_size) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uintptr_t mis = a & 15u;
    if (mis == 0) return 0;
    if (mis % elem_size != 0) return UINT64_MAX;  // never aligns
    return (16u - mis) / elem_size;
}

// ------------------------------------------------------------- scratch
// Per-stream cached device scratch; returns a pointer with at least `bytes`
// bytes (grown with hipMalloc -- not graph-capturable).
int scratch_get(hipStream_t s, size_t bytes, void** out);
// Resolve caller scratch or the cache.
inline int resolve_scratch(hipStream_t s, void* scratch, size_t scratch_bytes, size_t need,
                           void** out) {
    if (need == 0) {
        *out = scratch;
        return 0;
    }
    if (scratch) {
        if (scratch_bytes < need) return HPXHIP_ERROR_INVALID_ARGUMENT;
        *out = scratch;
        return 0;
    }
    return scratch_get(s, need, out);
}
// Device error word for the stream's device.
uint32_t* device_error_word(hipStream_t s);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Scratch sizing (defined in the algorithm TUs).
size_t reduce_scratch_bytes(uint64_t n);
size_t scan_scratch_bytes(int dtype, uint64_t n);
size_t copy_if_scratch_bytes(int dtype, uint64_t n);
size_t sort_scratch_bytes(int key_dtype, int value_dtype, uint64_t n);
size_t merge_scratch_bytes(uint64_t n);
size_t merge_runs_scratch_bytes(uint64_t n);

}  // namespace hpxhip
