// elementwise.hip -- fill / copy / for_each / transform (unary, binary).
//
// Replaces the reference's one-thread-per-element closure launch
// (hpx/compute/cuda/default_executor.hpp:87-136 -> detail/launch.hpp:32-137,
// block = 1024, 32-bit index, scalar access) with a gfx950 streaming kernel:
//   * 16-byte vector accesses (global_load_dwordx4 / global_store_dwordx4);
//   * one 16-B vector per thread per array and a grid covering the whole
//     range (measured on MI355X, 2^30 doubles: triad 6.1 TB/s with this flat
//     launch vs 5.1 TB/s for a 2048-block grid-stride loop with 4 vectors
//     in flight per thread -- scripts/ubench/ew.hip); the loop only strides
//     when the range exceeds 2^31-1 blocks.  64-bit indexing throughout;
//   * read+write kernels use 64-thread blocks and nontemporal (`nt`) loads
//     and stores: triad 6.16 -> 6.73 TB/s (scripts/ubench/ew2.hip); the
//     write-only fill keeps plain stores on 256-thread blocks (6.94 TB/s);
//   * a head (to reach 16-B alignment) and a tail handled inside the same
//     launch, so any iterator offset works; ranges whose arrays cannot all
//     be aligned together fall back to the scalar (V = 1) instantiation.
// FP expressions are compiled with -ffp-contract=off so x + y*s0 rounds
// exactly like the host functor in stream.cpp:257 (bit-exact parity).
#include "internal.hpp"

using namespace hpxhip;

namespace {

constexpr int kThreads = 256;     // fill / generate (write-only streams)
constexpr int kRwThreads = 64;    // transform / copy / for_each (read + write streams)

// Geometry: vector part of [0, nvec) processed grid-stride, each thread
// handling vectors i, i+S, ..., i+(U-1)S per iteration (coalesced per
// instruction: a wave touches 64 consecutive 16-B vectors).
struct span3 {
    uint64_t head;  // scalar elements before the vector part
    uint64_t nvec;  // vectors of V elements
    uint64_t tail;  // scalar elements after the vector part
};

inline unsigned grid_for(uint64_t work_items, int threads = kThreads) {
    const uint64_t per_block = static_cast<uint64_t>(threads);
    uint64_t blocks = (work_items + per_block - 1) / per_block;
    const uint64_t cap = 0x7fffffffull;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    return static_cast<unsigned>(blocks);
}

// out[i] = (TO) f((C) in[i])
template <typename TI, typename C, typename TO, typename F, int V>
__global__ __launch_bounds__(kRwThreads) void k_unary(const TI* in, TO* out, span3 sp, F f) {
    using VI = vec<TI, V>;
    using VO = vec<TO, V>;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kRwThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kRwThreads;

    // Head and tail: scalar, first threads of the grid.
    if (tid < sp.head) out[tid] = static_cast<TO>(f(static_cast<C>(in[tid])));
    const uint64_t tail0 = sp.head + sp.nvec * V;
    if (tid < sp.tail) out[tail0 + tid] = static_cast<TO>(f(static_cast<C>(in[tail0 + tid])));

    const VI* vin = reinterpret_cast<const VI*>(in + sp.head);
    VO* vout = reinterpret_cast<VO*>(out + sp.head);
    for (uint64_t i = tid; i < sp.nvec; i += stride) {
        const VI x = ld_stream(&vin[i]);
        VO y;
#pragma unroll
        for (int e = 0; e < V; ++e) y.v[e] = static_cast<TO>(f(static_cast<C>(x.v[e])));
        st_stream(&vout[i], y);
    }
}

// out[i] = (TO) f((C) a[i], (C) b[i])
template <typename TI, typename C, typename TO, typename F, int V>
__global__ __launch_bounds__(kRwThreads) void k_binary(const TI* a, const TI* b, TO* out, span3 sp, F f) {
    using VI = vec<TI, V>;
    using VO = vec<TO, V>;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kRwThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kRwThreads;

    if (tid < sp.head) out[tid] = static_cast<TO>(f(static_cast<C>(a[tid]), static_cast<C>(b[tid])));
    const uint64_t tail0 = sp.head + sp.nvec * V;
    if (tid < sp.tail)
        out[tail0 + tid] = static_cast<TO>(f(static_cast<C>(a[tail0 + tid]), static_cast<C>(b[tail0 + tid])));

    const VI* va = reinterpret_cast<const VI*>(a + sp.head);
    const VI* vb = reinterpret_cast<const VI*>(b + sp.head);
    VO* vout = reinterpret_cast<VO*>(out + sp.head);
    for (uint64_t i = tid; i < sp.nvec; i += stride) {
        const VI x = ld_stream(&va[i]);
        const VI y = ld_stream(&vb[i]);
        VO z;
#pragma unroll
        for (int e = 0; e < V; ++e) z.v[e] = static_cast<TO>(f(static_cast<C>(x.v[e]), static_cast<C>(y.v[e])));
        st_stream(&vout[i], z);
    }
}

// Inputs whose offset inside 16 B differs from the output's (a[i + 1] - a[i]
// style ranges): the head brings the output to a 1-KiB boundary as above; a
// misaligned input is read as the aligned 16-B vectors i and i + 1 and its
// elements shifted by sh (in elements) in registers.  Plain loads: vector
// i + 1 is the next lane's vector i, so the second read hits the cache.  The
// caller moves the last vector to the scalar tail, so i + 1 stays inside the
// range; head >= V keeps vector 0 at or after the range start (ld_shifted:
// common.hpp).  r04: taking vector i + 1 from the next lane over DPP instead
// (shift_from_next_lane, as the scan's shifted input does) measured the same
// or slower here -- triad b+1/c+0/a+0 3.98-3.99 ms both ways, b+0/c+1/a+3
// 4.17 -> 4.26 (profiles/r04_unaligned_probe_dpp_elementwise.log): the
// second load is a cache hit, the shuffles are not free.
template <typename TI, typename C, typename TO, typename F, int V>
__global__ __launch_bounds__(kRwThreads) void k_unary_sh(const TI* in, TO* out, span3 sp, F f, int sh) {
    using VO = vec<TO, V>;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kRwThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kRwThreads;
    if (tid < sp.head) out[tid] = static_cast<TO>(f(static_cast<C>(in[tid])));
    const uint64_t tail0 = sp.head + sp.nvec * V;
    if (tid < sp.tail) out[tail0 + tid] = static_cast<TO>(f(static_cast<C>(in[tail0 + tid])));
    const vec<TI, V>* vin = reinterpret_cast<const vec<TI, V>*>(in + sp.head - sh);
    VO* vout = reinterpret_cast<VO*>(out + sp.head);
    for (uint64_t i = tid; i < sp.nvec; i += stride) {
        const vec<TI, V> x = ld_shifted<TI, V>(vin, i, sh);
        VO y;
#pragma unroll
        for (int e = 0; e < V; ++e) y.v[e] = static_cast<TO>(f(static_cast<C>(x.v[e])));
        st_stream(&vout[i], y);
    }
}

template <typename TI, typename C, typename TO, typename F, int V>
__global__ __launch_bounds__(kRwThreads) void k_binary_sh(const TI* a, const TI* b, TO* out, span3 sp, F f, int sha,
                                                          int shb) {
    using VO = vec<TO, V>;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kRwThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kRwThreads;
    if (tid < sp.head) out[tid] = static_cast<TO>(f(static_cast<C>(a[tid]), static_cast<C>(b[tid])));
    const uint64_t tail0 = sp.head + sp.nvec * V;
    if (tid < sp.tail)
        out[tail0 + tid] = static_cast<TO>(f(static_cast<C>(a[tail0 + tid]), static_cast<C>(b[tail0 + tid])));
    const vec<TI, V>* va = reinterpret_cast<const vec<TI, V>*>(a + sp.head - sha);
    const vec<TI, V>* vb = reinterpret_cast<const vec<TI, V>*>(b + sp.head - shb);
    VO* vout = reinterpret_cast<VO*>(out + sp.head);
    for (uint64_t i = tid; i < sp.nvec; i += stride) {
        const vec<TI, V> x = ld_shifted<TI, V>(va, i, sha);
        const vec<TI, V> y = ld_shifted<TI, V>(vb, i, shb);
        VO z;
#pragma unroll
        for (int e = 0; e < V; ++e) z.v[e] = static_cast<TO>(f(static_cast<C>(x.v[e]), static_cast<C>(y.v[e])));
        st_stream(&vout[i], z);
    }
}

// data[i] = value
template <typename T, int V>
__global__ __launch_bounds__(kThreads) void k_fill(T* out, span3 sp, T value) {
    using VT = vec<T, V>;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    if (tid < sp.head) out[tid] = value;
    const uint64_t tail0 = sp.head + sp.nvec * V;
    if (tid < sp.tail) out[tail0 + tid] = value;
    VT y;
#pragma unroll
    for (int e = 0; e < V; ++e) y.v[e] = value;
    VT* vout = reinterpret_cast<VT*>(out + sp.head);
    for (uint64_t i = tid; i < sp.nvec; i += stride) vout[i] = y;
}

// Split [0, n) into head/vector/tail for the given pointers (all must share
// the same misalignment); returns false if they cannot be vectorised together.
// The head also carries the written array (the last pointer) to a 1-KiB
// boundary, so every wave's 1-KiB store covers whole 128-B lines: a range
// that is 16-B but not line aligned otherwise writes a partial line at both
// ends of every wave's run (triad over arrays offset by one double: 4.59 ms
// vs 3.77 aligned, profiles/r02_unaligned_ranges.log).  The extra head (at
// most 1008 B) is a few scalar threads.
constexpr uintptr_t kStoreAlign = 1024;
template <int V>
bool make_span(uint64_t n, size_t esize, span3* sp, std::initializer_list<const void*> ptrs) {
    uint64_t head = UINT64_MAX;
    bool first = true;
    const void* last = nullptr;
    for (const void* p : ptrs) {
        uint64_t h = head_to_align16(p, esize);
        if (h == UINT64_MAX) return false;
        if (first) {
            head = h;
            first = false;
        } else if (h != head) {
            return false;
        }
        last = p;
    }
    const uintptr_t vstart = reinterpret_cast<uintptr_t>(last) + head * esize;  // 16-B aligned
    head += ((kStoreAlign - vstart % kStoreAlign) % kStoreAlign) / esize;
    if (head > n) head = n;
    sp->head = head;
    sp->nvec = (n - head) / V;
    sp->tail = n - head - sp->nvec * V;
    return true;
}

// Span for inputs that are element aligned but offset from the output inside
// 16 B: the head from the output alone (>= V elements), each input's shift,
// and the last vector moved to the tail.  False if a pointer is not element
// aligned or the range is too short to be worth it.
template <int V>
bool make_span_shifted(uint64_t n, size_t esize, span3* sp, const void* out, std::initializer_list<const void*> ins,
                       int* sh) {
    if (reinterpret_cast<uintptr_t>(out) % esize) return false;
    uint64_t head = head_to_align16(out, esize);
    const uintptr_t vstart = reinterpret_cast<uintptr_t>(out) + head * esize;
    head += ((kStoreAlign - vstart % kStoreAlign) % kStoreAlign) / esize;
    if (head < static_cast<uint64_t>(V)) head += kStoreAlign / esize;
    if (n < head + 4 * kStoreAlign / esize) return false;
    int k = 0;
    for (const void* p : ins) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        if (a % esize) return false;
        sh[k++] = static_cast<int>(((a + head * esize) % 16) / esize);
    }
    sp->head = head;
    sp->nvec = (n - head) / V - 1;  // the last vector joins the tail
    sp->tail = n - head - sp->nvec * V;
    return true;
}

template <typename TI, typename C, typename TO, typename F>
int launch_unary(const TI* in, TO* out, uint64_t n, F f, hipStream_t s) {
    constexpr int VW = 16 / (sizeof(TI) > sizeof(TO) ? sizeof(TI) : sizeof(TO));
    constexpr int V = VW < 1 ? 1 : VW;
    span3 sp;
    int sh[1];
    if ((sizeof(TI) == sizeof(TO)) && make_span<V>(n, sizeof(TI), &sp, {in, out})) {
        hipLaunchKernelGGL((k_unary<TI, C, TO, F, V>), dim3(grid_for(sp.nvec + sp.head + sp.tail, kRwThreads)),
                           dim3(kRwThreads), 0, s, in, out, sp, f);
    } else if (V > 1 && sizeof(TI) == sizeof(TO) && make_span_shifted<V>(n, sizeof(TI), &sp, out, {in}, sh)) {
        hipLaunchKernelGGL((k_unary_sh<TI, C, TO, F, V>), dim3(grid_for(sp.nvec + sp.head + sp.tail, kRwThreads)),
                           dim3(kRwThreads), 0, s, in, out, sp, f, sh[0]);
    } else {
        sp = span3{0, n, 0};
        hipLaunchKernelGGL((k_unary<TI, C, TO, F, 1>), dim3(grid_for(n, kRwThreads)), dim3(kRwThreads), 0, s, in, out,
                           sp, f);
    }
    HPXHIP_CHECK_LAUNCH();
    return 0;
}

template <typename TI, typename C, typename TO, typename F>
int launch_binary(const TI* a, const TI* b, TO* out, uint64_t n, F f, hipStream_t s) {
    constexpr int VW = 16 / (sizeof(TI) > sizeof(TO) ? sizeof(TI) : sizeof(TO));
    constexpr int V = VW < 1 ? 1 : VW;
    span3 sp;
    int sh[2];
    if ((sizeof(TI) == sizeof(TO)) && make_span<V>(n, sizeof(TI), &sp, {a, b, out})) {
        hipLaunchKernelGGL((k_binary<TI, C, TO, F, V>), dim3(grid_for(sp.nvec + sp.head + sp.tail, kRwThreads)),
                           dim3(kRwThreads), 0, s, a, b, out, sp, f);
    } else if (V > 1 && sizeof(TI) == sizeof(TO) && make_span_shifted<V>(n, sizeof(TI), &sp, out, {a, b}, sh)) {
        hipLaunchKernelGGL((k_binary_sh<TI, C, TO, F, V>), dim3(grid_for(sp.nvec + sp.head + sp.tail, kRwThreads)),
                           dim3(kRwThreads), 0, s, a, b, out, sp, f, sh[0], sh[1]);
    } else {
        sp = span3{0, n, 0};
        hipLaunchKernelGGL((k_binary<TI, C, TO, F, 1>), dim3(grid_for(n, kRwThreads)), dim3(kRwThreads), 0, s, a,
                           b, out, sp, f);
    }
    HPXHIP_CHECK_LAUNCH();
    return 0;
}

// Strided pointer inductions: grid-stride loop, one element per thread per
// trip.  Strided accesses cannot be vectorised; at |stride| = 1 the entry
// points below use the contiguous kernels instead.
template <typename TI, typename C, typename TO, typename F>
__global__ __launch_bounds__(kThreads) void k_unary_strided(const TI* in, int64_t si, TO* out, int64_t so, uint64_t n,
                                                            F f) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += step) {
        const int64_t k = static_cast<int64_t>(i);
        out[k * so] = static_cast<TO>(f(static_cast<C>(in[k * si])));
    }
}

template <typename TI, typename C, typename TO, typename F>
__global__ __launch_bounds__(kThreads) void k_binary_strided(const TI* a, int64_t sa, const TI* b, int64_t sb,
                                                             TO* out, int64_t so, uint64_t n, F f) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; i < n; i += step) {
        const int64_t k = static_cast<int64_t>(i);
        out[k * so] = static_cast<TO>(f(static_cast<C>(a[k * sa]), static_cast<C>(b[k * sb])));
    }
}

// (in, compute, out) combinations that are built: compute == in or F64;
// out == in or == compute.
template <typename TI, typename F>
int with_compute_out(int compute_dt, int out_dt, F&& f) {
    return with_wide_dtype<TI>(compute_dt, [&](auto ct) -> int {
        using C = typename decltype(ct)::type;
        if (out_dt == dtype_of<TI>()) return f(ct, tag<TI>{});
        if (out_dt == dtype_of<C>()) return f(ct, tag<C>{});
        return HPXHIP_ERROR_UNSUPPORTED;
    });
}

// Counter-based generator for hpx::parallel::generate with a splitmix64
// functor (x_i = f(splitmix64(seed ^ i))) and iota (x_i = start + i).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void k_generate(T* out, uint64_t n, uint64_t base, int kind, uint64_t seed,
                                                        int64_t lo, uint64_t span) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x; j < n; j += stride) {
        const uint64_t i = base + j;  // global index
        T v;
        if (kind == HPXHIP_GEN_IOTA) {
            v = static_cast<T>(lo + static_cast<int64_t>(i));
        } else {
            const uint64_t z = splitmix64(seed ^ i);
            if (kind == HPXHIP_GEN_BITS) {
                if constexpr (sizeof(T) == 8) __builtin_memcpy(&v, &z, 8);
                else {
                    const uint32_t w = static_cast<uint32_t>(z >> 32);
                    __builtin_memcpy(&v, &w, 4);
                }
            } else if (kind == HPXHIP_GEN_RANGE) {
                const uint64_t r = span ? (z % span) : z;
                v = static_cast<T>(static_cast<int64_t>(static_cast<uint64_t>(lo) + r));
            } else {  // HPXHIP_GEN_UNIT
                if constexpr (sizeof(T) == 8) v = static_cast<T>(static_cast<double>(z >> 11) * 0x1.0p-53);
                else v = static_cast<T>(static_cast<float>(z >> 40) * 0x1.0p-24f);
            }
        }
        out[j] = v;
    }
}

}  // namespace

extern "C" {

int hpxhip_generate_at(int dtype, int kind, uint64_t seed, uint64_t index_base, int64_t lo, int64_t hi, void* data,
                       uint64_t n, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_generate_at");
    if (n == 0) return 0;
    if (!data || kind < HPXHIP_GEN_IOTA || kind > HPXHIP_GEN_UNIT) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    const uint64_t span = static_cast<uint64_t>(hi) - static_cast<uint64_t>(lo) + 1u;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        hipLaunchKernelGGL((k_generate<T>), dim3(grid_for(n / 4 + 1)), dim3(kThreads), 0, s, static_cast<T*>(data), n,
                           index_base, kind, seed, lo, span);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    });
}

int hpxhip_generate(int dtype, int kind, uint64_t seed, int64_t lo, int64_t hi, void* data, uint64_t n,
                    hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_generate");
    return hpxhip_generate_at(dtype, kind, seed, 0, lo, hi, data, n, stream);
}

int hpxhip_fill(int dtype, const void* value, void* data, uint64_t n, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_fill");
    if (n == 0) return 0;
    if (!value || !data) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        constexpr int V = 16 / sizeof(T);
        T v;
        __builtin_memcpy(&v, value, sizeof(T));
        span3 sp;
        if (!make_span<V>(n, sizeof(T), &sp, {data})) {
            sp = span3{0, n, 0};
            hipLaunchKernelGGL((k_fill<T, 1>), dim3(grid_for(n)), dim3(kThreads), 0, s, static_cast<T*>(data), sp, v);
        } else {
            hipLaunchKernelGGL((k_fill<T, V>), dim3(grid_for(sp.nvec + sp.head + sp.tail)), dim3(kThreads), 0, s,
                               static_cast<T*>(data), sp, v);
        }
        HPXHIP_CHECK_LAUNCH();
        return 0;
    });
}

int hpxhip_copy(int dtype, const void* in, void* out, uint64_t n, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_copy");
    if (n == 0) return 0;
    if (!in || !out) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return launch_unary<T, T, T>(static_cast<const T*>(in), static_cast<T*>(out), n,
                                     unary_fn<HPXHIP_U_IDENTITY, T>{T(0), T(0)}, s);
    });
}

int hpxhip_for_each(int dtype, int unary_kind, const void* scalars, void* data, uint64_t n,
                    hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_for_each");
    if (n == 0) return 0;
    if (!data) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return with_unary<T>(unary_kind, scalars, [&](auto f) -> int {
            return launch_unary<T, T, T>(static_cast<const T*>(data), static_cast<T*>(data), n, f, s);
        });
    });
}

int hpxhip_transform(int in_dtype, int compute_dtype, int out_dtype, int unary_kind, const void* scalars,
                     const void* in, void* out, uint64_t n, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_transform");
    if (n == 0) return 0;
    if (!in || !out) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_compute_out<TI>(compute_dtype, out_dtype, [&](auto ct, auto ot) -> int {
            using C = typename decltype(ct)::type;
            using TO = typename decltype(ot)::type;
            return with_unary<C>(unary_kind, scalars, [&](auto f) -> int {
                return launch_unary<TI, C, TO>(static_cast<const TI*>(in), static_cast<TO*>(out), n, f, s);
            });
        });
    });
}

int hpxhip_transform_binary(int in_dtype, int compute_dtype, int out_dtype, int binary_kind,
                            const void* scalars, const void* in1, const void* in2, void* out, uint64_t n,
                            hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_transform_binary");
    if (n == 0) return 0;
    if (!in1 || !in2 || !out) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_compute_out<TI>(compute_dtype, out_dtype, [&](auto ct, auto ot) -> int {
            using C = typename decltype(ct)::type;
            using TO = typename decltype(ot)::type;
            return with_binary<C>(binary_kind, scalars, [&](auto f) -> int {
                return launch_binary<TI, C, TO>(static_cast<const TI*>(in1), static_cast<const TI*>(in2),
                                                static_cast<TO*>(out), n, f, s);
            });
        });
    });
}

// A strided walk must stay inside a 47-bit address span (the GPU's virtual
// address space): any larger |stride| * (n - 1) is a caller error (e.g. an
// unsigned stride wrapped into a huge one), never a valid range.
static bool strided_span_ok(int64_t stride, uint64_t n, size_t elem) {
    if (n < 2) return true;
    const unsigned __int128 mag = static_cast<unsigned __int128>(stride < 0 ? -static_cast<__int128>(stride) : stride);
    return mag * (n - 1) * elem < (static_cast<unsigned __int128>(1) << 47);
}

int hpxhip_transform_strided(int in_dtype, int compute_dtype, int out_dtype, int unary_kind, const void* scalars,
                             const void* in, int64_t in_stride, void* out, int64_t out_stride, uint64_t n,
                             hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_transform_strided");
    if (n == 0) return 0;
    if (!in || !out || (out_stride == 0 && n > 1)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (!strided_span_ok(in_stride, n, dtype_size(in_dtype)) || !strided_span_ok(out_stride, n, dtype_size(out_dtype)))
        return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (in_stride == 1 && out_stride == 1)
        return hpxhip_transform(in_dtype, compute_dtype, out_dtype, unary_kind, scalars, in, out, n, stream);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_compute_out<TI>(compute_dtype, out_dtype, [&](auto ct, auto ot) -> int {
            using C = typename decltype(ct)::type;
            using TO = typename decltype(ot)::type;
            return with_unary<C>(unary_kind, scalars, [&](auto f) -> int {
                hipLaunchKernelGGL((k_unary_strided<TI, C, TO, decltype(f)>), dim3(grid_for(n)), dim3(kThreads), 0, s,
                                   static_cast<const TI*>(in), in_stride, static_cast<TO*>(out), out_stride, n, f);
                HPXHIP_CHECK_LAUNCH();
                return 0;
            });
        });
    });
}

int hpxhip_transform_binary_strided(int in_dtype, int compute_dtype, int out_dtype, int binary_kind,
                                    const void* scalars, const void* in1, int64_t in1_stride, const void* in2,
                                    int64_t in2_stride, void* out, int64_t out_stride, uint64_t n,
                                    hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_transform_binary_strided");
    if (n == 0) return 0;
    if (!in1 || !in2 || !out || (out_stride == 0 && n > 1)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (!strided_span_ok(in1_stride, n, dtype_size(in_dtype)) || !strided_span_ok(in2_stride, n, dtype_size(in_dtype)) ||
        !strided_span_ok(out_stride, n, dtype_size(out_dtype)))
        return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (in1_stride == 1 && in2_stride == 1 && out_stride == 1)
        return hpxhip_transform_binary(in_dtype, compute_dtype, out_dtype, binary_kind, scalars, in1, in2, out, n,
                                       stream);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_compute_out<TI>(compute_dtype, out_dtype, [&](auto ct, auto ot) -> int {
            using C = typename decltype(ct)::type;
            using TO = typename decltype(ot)::type;
            return with_binary<C>(binary_kind, scalars, [&](auto f) -> int {
                hipLaunchKernelGGL((k_binary_strided<TI, C, TO, decltype(f)>), dim3(grid_for(n)), dim3(kThreads), 0,
                                   s, static_cast<const TI*>(in1), in1_stride, static_cast<const TI*>(in2), in2_stride,
                                   static_cast<TO*>(out), out_stride, n, f);
                HPXHIP_CHECK_LAUNCH();
                return 0;
            });
        });
    });
}

}  // extern "C"
