// merge.hip -- hpx::parallel::merge and the sorted-range searches the
// segmented sort uses to cut its partitions.
//
// Reference: merge.hpp:52-80 (sequential_merge: take from the second range
// only when comp(*first2, *first1), so equal keys keep first-range-first
// order) and merge.hpp:161-243 (parallel_merge_helper: recursive halving at
// the upper bound of the larger range's midpoint in the other range).  On the
// GPU the split points are merge-path diagonals instead of a recursion:
//   k_merge_partition  one thread per output tile boundary d: binary search
//                      on the diagonal for the number of first-range
//                      elements among the first d outputs;
//   k_merge            one block per 2048-element output tile: both input
//                      runs of the tile staged in LDS with 16-B loads, a
//                      per-thread diagonal search in LDS, an 8-element serial
//                      merge in registers, and the tile written back through
//                      LDS with 16-B stores.
// Keys are compared through the radix sort's ordered bit patterns
// (sort_kernel.hpp: integers as std::less, floats in IEEE total order), so
// sort + merge agree on every dtype.  Traffic: 16 B/key (u64): each input
// read once, the output written once.
#include "internal.hpp"
#include <hpxhip/kernels/merge_kernel.hpp>

using namespace hpxhip;

namespace {

using namespace hpxhip::merge_detail;

// out[i] = number of sorted[] elements ordered before values[i]
// (lower_bound; upper: also those equal to it).
template <typename U, typename X>
__global__ __launch_bounds__(256) void k_bounds(const U* __restrict__ sorted, uint64_t n, const U* __restrict__ values,
                                                 uint64_t m, int upper, X xf, uint64_t* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= m) return;
    const U v = xf(values[i]);
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const U x = xf(sorted[mid]);
        if (upper ? (x <= v) : (x < v)) lo = mid + 1;
        else hi = mid;
    }
    out[i] = lo;
}

template <typename T, bool DESC>
int run_merge(const void* a, uint64_t na, const void* b, uint64_t nb, void* out, hipStream_t s, void* scratch,
              size_t scratch_bytes) {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    using X = ordered_bits<T, DESC>;
    const uint64_t total = na + nb;
    const uint64_t ntiles = (total + kTile - 1) / kTile;
    void* ws = nullptr;
    int rc = resolve_scratch(s, scratch, scratch_bytes, (ntiles + 1) * 8, &ws);
    if (rc) return rc;
    uint64_t* splits = static_cast<uint64_t*>(ws);
    const U* ua = static_cast<const U*>(a);
    const U* ub = static_cast<const U*>(b);
    using C = key_less<X>;
    hipLaunchKernelGGL((k_merge_partition<U, C>), dim3(static_cast<unsigned>((ntiles + 1 + 255) / 256)), dim3(256), 0,
                       s, ua, na, ub, nb, ntiles, C{}, splits);
    HPXHIP_CHECK_LAUNCH();
    const bool aligned = (reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                          reinterpret_cast<uintptr_t>(out)) % 16 == 0;
    if (aligned)
        hipLaunchKernelGGL((k_merge<U, C, true>), dim3(static_cast<unsigned>(ntiles)), dim3(kThreads), 0, s, ua, na, ub,
                           nb, splits, C{}, static_cast<U*>(out), device_error_word(s));
    else
        hipLaunchKernelGGL((k_merge<U, C, false>), dim3(static_cast<unsigned>(ntiles)), dim3(kThreads), 0, s, ua, na,
                           ub, nb, splits, C{}, static_cast<U*>(out), device_error_word(s));
    HPXHIP_CHECK_LAUNCH();
    return 0;
}

}  // namespace

namespace hpxhip {
size_t merge_scratch_bytes(uint64_t n) { return ((n + kTile - 1) / kTile + 1) * 8; }
}  // namespace hpxhip

// is_sorted.hpp:40-120 counts a pair (i, i+1) as out of order iff
// pred(key[i+1], key[i]) with pred = std::less (std::greater when
// descending), on the VALUES: for floats -0.0 and +0.0 compare equal and a
// NaN is never out of order (every comparison with it is false), unlike the
// radix key order the sort uses.
template <typename T, bool DESC>
struct value_out_of_order {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    __device__ __forceinline__ bool operator()(U cur, U next) const {
        const T a = __builtin_bit_cast(T, cur), b = __builtin_bit_cast(T, next);
        return DESC ? (a < b) : (b < a);
    }
};

// Adjacent pairs out of order; thread t handles the pairs starting in its
// 16-byte vector (the neighbour of the vector's last element is the next
// vector's first, re-read through the cache).
template <typename U, typename X>
__global__ __launch_bounds__(256) void k_unsorted_pairs(const U* __restrict__ keys, uint64_t n, X after,
                                                        unsigned long long* __restrict__ count) {
    constexpr int V = 16 / sizeof(U);
    using VT = vec<U, V>;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    uint64_t c = 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(keys) % 16) == 0;
    if (aligned) {
        const uint64_t nvec = n / V;
        const VT* vk = reinterpret_cast<const VT*>(keys);
        for (uint64_t v = tid; v < nvec; v += stride) {
            const VT x = ld_stream(&vk[v]);
#pragma unroll
            for (int e = 0; e + 1 < V; ++e) c += after(x.v[e], x.v[e + 1]);
            const uint64_t nx = (v + 1) * V;
            if (nx < n) c += after(x.v[V - 1], keys[nx]);
        }
        for (uint64_t i = nvec * V + tid; i + 1 < n; i += stride) c += after(keys[i], keys[i + 1]);
    } else {
        for (uint64_t i = tid; i + 1 < n; i += stride) c += after(keys[i], keys[i + 1]);
    }
    const uint64_t w = wave_reduce(c, op_plus{});
    if (lane_id() == 0 && w) atomicAdd(count, static_cast<unsigned long long>(w));
}

extern "C" {

int hpxhip_merge(int dtype, const void* in1, uint64_t n1, const void* in2, uint64_t n2, void* out, int descending,
                 hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_merge");
    if (n1 + n2 == 0) return 0;
    if ((n1 && !in1) || (n2 && !in2) || !out) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        if (descending) return run_merge<T, true>(in1, n1, in2, n2, out, s, scratch, scratch_bytes);
        return run_merge<T, false>(in1, n1, in2, n2, out, s, scratch, scratch_bytes);
    });
}

int hpxhip_sorted_bounds(int dtype, const void* sorted, uint64_t n, const void* values_dev, uint64_t m, int upper,
                         int descending, uint64_t* out_dev, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_sorted_bounds");
    if (m == 0) return 0;
    if ((n && !sorted) || !values_dev || !out_dev) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
        const dim3 grid(static_cast<unsigned>((m + 255) / 256));
        if (descending)
            hipLaunchKernelGGL((k_bounds<U, ordered_bits<T, true>>), grid, dim3(256), 0, s,
                               static_cast<const U*>(sorted), n, static_cast<const U*>(values_dev), m, upper,
                               ordered_bits<T, true>{}, out_dev);
        else
            hipLaunchKernelGGL((k_bounds<U, ordered_bits<T, false>>), grid, dim3(256), 0, s,
                               static_cast<const U*>(sorted), n, static_cast<const U*>(values_dev), m, upper,
                               ordered_bits<T, false>{}, out_dev);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    });
}

// is_sorted.hpp:40-120 (hpx::parallel::is_sorted / is_sorted_until): the
// number of adjacent pairs out of order (value comparison, see above), counted
// on the device (grid-stride, 16-B loads, wave reduction, one 64-bit atomic
// add per wave); 0 <=> sorted.  *count_dev is overwritten.
int hpxhip_unsorted_pairs(int dtype, const void* keys, uint64_t n, int descending, uint64_t* count_dev,
                          hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_unsorted_pairs");
    if (!count_dev || (n && !keys)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    HPXHIP_CHECK(hipMemsetAsync(count_dev, 0, sizeof(uint64_t), s));
    if (n < 2) return 0;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
        const unsigned grid = static_cast<unsigned>(std::min<uint64_t>((n + 1023) / 1024, 8192));
        if (descending)
            hipLaunchKernelGGL((k_unsorted_pairs<U, value_out_of_order<T, true>>), dim3(grid), dim3(256), 0, s,
                               static_cast<const U*>(keys), n, value_out_of_order<T, true>{},
                               reinterpret_cast<unsigned long long*>(count_dev));
        else
            hipLaunchKernelGGL((k_unsorted_pairs<U, value_out_of_order<T, false>>), dim3(grid), dim3(256), 0, s,
                               static_cast<const U*>(keys), n, value_out_of_order<T, false>{},
                               reinterpret_cast<unsigned long long*>(count_dev));
        HPXHIP_CHECK_LAUNCH();
        return 0;
    });
}

}  // extern "C"
