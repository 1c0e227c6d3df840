// sort.hip -- hpx::parallel::sort / sort_by_key as an LSD onesweep radix sort.
//
// Reference: sort.hpp:78-229 is a host quicksort (median-of-3 pivot, Hoare
// partition, std::sort leaves below 65536 elements, sort_limit_per_task
// sort.hpp:48); sort_by_key.hpp:42-78 sorts a zip of (key, value).  Neither
// has a GPU path.  Radix sorting by the keys' ordered bit patterns yields the
// same sequence for every strict weak order std::less induces on integers
// (and the IEEE total order for floats), so results are bit-exact against
// std::sort for integer keys.
//
// Structure (8-bit digits, 4 passes for 32-bit keys, 8 for 64-bit keys;
// kernels in sort_kernel.hpp):
//   k_hist        one read of the keys -> all passes' 256-bin histograms
//                 (per-block LDS histograms, one global atomic per bin);
//   k_bin_offsets exclusive scan of each pass's histogram;
//   k_onesweep    per pass, per tile: wave-level match ranking (8 ballots
//                 per key, no LDS atomics), per-wave LDS digit counters,
//                 tile-local counting sort into LDS, per-digit decoupled
//                 look-back across tiles (one thread per digit, batched
//                 granule loads, {flag,count} granules written by one sc1
//                 store), and a coalesced write of the LDS-sorted tile.
// A pass whose digit is constant over all keys is skipped (the histogram is
// read back once per sort).  Traffic model: 8 B/key histogram + 16 B/key per
// executed pass (+ values).
#include "internal.hpp"
#include "sort_kernel.hpp"

#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;

namespace {

constexpr int kHistThreads = 256;
constexpr int kHistBlocksPerCU = 4;  // 4 lane copies x 8 KiB per pass histogram: 2.48 -> 1.87 ms (profiles/r01_ubench_sortpass2.log)

// Tile shape per variant (scripts/ubench/sortpass.hip): keys only -> 512
// threads x 16 keys = 8192-key tiles (64 KiB of u64 keys staged in LDS, 2
// blocks/CU); with values -> 256 x 16 (keys and values staged).  Look-back:
// each digit's thread loads 4 predecessors per step (4.88 ms/pass vs 5.00 at
// 8 and 5.48 at 16; rocPRIM's radix_sort_keys takes 50.2 ms for the whole
// 2^30 u64 sort on the same GPU, this one 43.5 ms).
template <bool HAS_VAL>
struct tile_shape {
    static constexpr int threads = HAS_VAL ? 256 : 512;
    static constexpr int items = 16;
    static constexpr int lbb = 4;
    static constexpr int tile = threads * items;
};

struct sort_layout {
    uint64_t ntiles;
    size_t alt_keys, alt_vals, hist, start, counter, lb, lb_bytes, total;
    bool wide;  // 64-bit granules
};

sort_layout make_layout(uint64_t n, size_t ksize, size_t vsize, int tile) {
    sort_layout L;
    L.ntiles = (n + tile - 1) / tile;
    L.wide = n >= (1ull << 31);
    size_t off = 0;
    L.alt_keys = off;
    off = align_up(off + n * ksize, 256);
    L.alt_vals = off;
    off = align_up(off + n * vsize, 256);
    L.hist = off;
    off += 8 * kRadix * 8;
    L.start = off;
    off += 8 * kRadix * 8;
    L.counter = off;  // counter (16 B) immediately followed by lb: one memset
    off += 256;
    L.lb = off;
    L.lb_bytes = L.ntiles * kRadix * (L.wide ? 8 : 4);
    off = align_up(off + L.lb_bytes, 256);
    L.total = off;
    return L;
}

template <typename T, bool DESC, typename VAL, bool HAS_VAL>
int run_sort(void* keys, void* vals, uint64_t n, hipStream_t s, void* scratch, size_t scratch_bytes) {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    using X = ordered_bits<T, DESC>;
    using TS = tile_shape<HAS_VAL>;
    const sort_layout L = make_layout(n, sizeof(U), HAS_VAL ? sizeof(VAL) : 0, TS::tile);
    void* ws = nullptr;
    int rc = resolve_scratch(s, scratch, scratch_bytes, L.total, &ws);
    if (rc) return rc;
    char* base = static_cast<char*>(ws);
    auto* hist = reinterpret_cast<unsigned long long*>(base + L.hist);
    auto* start = reinterpret_cast<unsigned long long*>(base + L.start);
    uint32_t* counter = reinterpret_cast<uint32_t*>(base + L.counter);
    uint32_t* err = device_error_word(s);
    const int passes = static_cast<int>(sizeof(U));

    HPXHIP_CHECK(hipMemsetAsync(hist, 0, 8 * kRadix * 8, s));
    const unsigned hist_grid = static_cast<unsigned>(current_device_info().cus * kHistBlocksPerCU);
    hipLaunchKernelGGL((k_hist<U, X, kHistThreads>), dim3(hist_grid), dim3(kHistThreads), 0, s,
                       static_cast<const U*>(keys), n, passes, X{}, hist);
    HPXHIP_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_bin_offsets, dim3(passes), dim3(256), 0, s, hist, start);
    HPXHIP_CHECK_LAUNCH();

    // Pass skipping needs the histogram on the host.
    std::vector<unsigned long long> h(static_cast<size_t>(passes) * kRadix);
    HPXHIP_CHECK(hipMemcpyAsync(h.data(), hist, h.size() * 8, hipMemcpyDeviceToHost, s));
    HPXHIP_CHECK(hipStreamSynchronize(s));

    U* kc = static_cast<U*>(keys);
    U* ka = reinterpret_cast<U*>(base + L.alt_keys);
    VAL* vc = static_cast<VAL*>(vals);
    VAL* va = reinterpret_cast<VAL*>(base + L.alt_vals);
    int executed = 0;
    for (int p = 0; p < passes; ++p) {
        bool constant = false;
        for (int d = 0; d < kRadix; ++d)
            if (h[p * kRadix + d] == n) constant = true;
        if (constant) continue;
        HPXHIP_CHECK(hipMemsetAsync(counter, 0, 256 + L.lb_bytes, s));
        const dim3 grid(static_cast<unsigned>(L.ntiles)), block(TS::threads);
        if (L.wide)
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, unsigned long long, X, TS::threads, TS::items, TS::lbb>), grid,
                               block, 0, s, kc, ka, vc, va, n, 8 * p, start + p * kRadix,
                               reinterpret_cast<unsigned long long*>(base + L.lb), counter, err, X{});
        else
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, uint32_t, X, TS::threads, TS::items, TS::lbb>), grid, block, 0, s,
                               kc, ka, vc, va, n, 8 * p, start + p * kRadix, reinterpret_cast<uint32_t*>(base + L.lb),
                               counter, err, X{});
        HPXHIP_CHECK_LAUNCH();
        std::swap(kc, ka);
        std::swap(vc, va);
        ++executed;
    }
    if (executed & 1) {
        HPXHIP_CHECK(hipMemcpyAsync(keys, kc, n * sizeof(U), hipMemcpyDeviceToDevice, s));
        if constexpr (HAS_VAL) HPXHIP_CHECK(hipMemcpyAsync(vals, vc, n * sizeof(VAL), hipMemcpyDeviceToDevice, s));
    }
    return 0;
}

template <typename T, typename VAL, bool HAS_VAL>
int dispatch_desc(int descending, void* keys, void* vals, uint64_t n, hipStream_t s, void* scratch, size_t sb) {
    if (descending) return run_sort<T, true, VAL, HAS_VAL>(keys, vals, n, s, scratch, sb);
    return run_sort<T, false, VAL, HAS_VAL>(keys, vals, n, s, scratch, sb);
}

}  // namespace

namespace hpxhip {
size_t sort_scratch_bytes(int key_dtype, int value_dtype, uint64_t n) {
    const bool has_val = value_dtype >= 0;
    return make_layout(n, dtype_size(key_dtype), has_val ? dtype_size(value_dtype) : 0,
                       has_val ? tile_shape<true>::tile : tile_shape<false>::tile)
        .total;
}
}  // namespace hpxhip

extern "C" {

int hpxhip_sort(int dtype, void* keys, uint64_t n, int descending, hpxhip_stream stream, void* scratch,
                size_t scratch_bytes) {
    if (n < 2) return 0;
    if (!keys) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return dispatch_desc<T, uint32_t, false>(descending, keys, nullptr, n, s, scratch, scratch_bytes);
    });
}

int hpxhip_sort_by_key(int key_dtype, int value_dtype, void* keys, void* values, uint64_t n, int descending,
                       hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    if (n < 2) return 0;
    if (!keys || !values) return HPXHIP_ERROR_INVALID_ARGUMENT;
    const size_t vs = dtype_size(value_dtype);
    if (vs == 0) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(key_dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        if (vs == 8) return dispatch_desc<T, uint64_t, true>(descending, keys, values, n, s, scratch, scratch_bytes);
        return dispatch_desc<T, uint32_t, true>(descending, keys, values, n, s, scratch, scratch_bytes);
    });
}

}  // extern "C"
