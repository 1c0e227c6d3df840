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
//                 per key folded with v_bitop3, no LDS atomics), per-wave LDS
//                 digit counters, tile-local counting sort into LDS, per-digit
//                 decoupled look-back across tiles (one thread per digit,
//                 batched granule loads, {flag,count} granules written by one
//                 sc1 store), and a coalesced write of the LDS-sorted tile.
// A pass whose digit is constant over all keys is skipped (the histogram is
// read back once per sort).  Traffic: 8 B/key histogram + 16 B/key per
// executed pass (+ values).
//
// Hybrid tail (64-bit keys only, >= 2^22 of them, >= 3 live digits, bucket
// sizes estimated from the histograms within one workgroup's LDS): onesweep
// passes on the two most significant live digits only (p2, then p1), which
// orders the keys by a 16-bit prefix; k_bucket_bounds finds the 65536 bucket
// starts by binary search; the host packs whole buckets into segments of at
// most 18432 keys; k_bucket_sort sorts each segment completely inside one
// CU's LDS (two stable LDS passes + odd-even rounds, see sort_kernel.hpp).
// 56 B/key instead of 136 for random 2^30 u64 keys (42.3 -> 21.1 ms).
// Buckets larger than a segment are finished by per-bucket LSD; more than
// kMaxBigBuckets of them (skewed keys) by the plain LSD.
#include "internal.hpp"
#include "sort_kernel.hpp"

#include <algorithm>
#include <utility>
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
// 2^30 u64 sort on the same GPU, the plain LSD here 40 ms, the hybrid 21 ms).
template <bool HAS_VAL>
struct tile_shape {
    static constexpr int threads = HAS_VAL ? 256 : 512;
    static constexpr int items = 16;
    static constexpr int lbb = 4;
    static constexpr int tile = threads * items;
};

struct sort_layout {
    uint64_t ntiles;
    size_t alt_keys, alt_vals, hist, bits, start, bounds, segs, counter, lb, lb_bytes, total;
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
    L.bits = off;  // OR / AND of the ordered keys
    off += 256;
    L.start = off;
    off += 8 * kRadix * 8;
    L.bounds = off;  // hybrid: bucket bounds and segment table (65537 u64 each)
    off = align_up(off + 8 * (kBuckets + 1), 256);
    L.segs = off;  // (begin, end) pairs
    off = align_up(off + 16 * kBuckets, 256);
    L.counter = off;  // counter (16 B) immediately followed by lb: one memset
    off += 256;
    L.lb = off;
    L.lb_bytes = L.ntiles * kRadix * (L.wide ? 8 : 4);
    off = align_up(off + L.lb_bytes, 256);
    L.total = off;
    return L;
}

// Hybrid tail (keys-only 64-bit sorts of at least 2^22 keys whose bucket
// sizes, estimated from the two digits' histograms, fit one workgroup's LDS).
constexpr int kBucketThreads = 1024;
constexpr int kBucketItems = 18;
constexpr uint64_t kBucketCap = static_cast<uint64_t>(kBucketThreads) * kBucketItems;
constexpr uint64_t kHybridMin = 1ull << 22;
constexpr size_t kMaxBigBuckets = 64;  // more oversized buckets than this -> finish as plain LSD

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
    const unsigned hist_grid = static_cast<unsigned>(current_device_info().cus * kHistBlocksPerCU);

    auto* bits = reinterpret_cast<unsigned long long*>(base + L.bits);
    // histograms of digits [first, passes) of keys[0, cnt) -> hist, their
    // exclusive bin starts -> start, OR / AND of the keys -> bits
    auto histogram = [&](const U* k, uint64_t cnt, int first) -> int {
        HPXHIP_CHECK(hipMemsetAsync(hist, 0, 8 * kRadix * 8, s));
        HPXHIP_CHECK(hipMemsetAsync(bits, 0, 8, s));
        HPXHIP_CHECK(hipMemsetAsync(bits + 1, 0xff, 8, s));
        hipLaunchKernelGGL((k_hist<U, X, kHistThreads>), dim3(hist_grid), dim3(kHistThreads), 0, s, k, cnt, first, passes,
                           X{}, hist, bits);
        HPXHIP_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_bin_offsets, dim3(passes), dim3(256), 0, s, hist, start);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    };
    // one stable onesweep pass of digit p over cnt keys
    auto pass = [&](const U* kin, U* kout, const VAL* vin, VAL* vout, uint64_t cnt, int p) -> int {
        const uint64_t nt = (cnt + TS::tile - 1) / TS::tile;
        HPXHIP_CHECK(hipMemsetAsync(counter, 0, 256 + nt * kRadix * (L.wide ? 8 : 4), s));
        const dim3 grid(static_cast<unsigned>(nt)), block(TS::threads);
        if (L.wide)
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, unsigned long long, X, TS::threads, TS::items, TS::lbb>), grid,
                               block, 0, s, kin, kout, vin, vout, cnt, 8 * p, start + p * kRadix,
                               reinterpret_cast<unsigned long long*>(base + L.lb), counter, err, X{});
        else
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, uint32_t, X, TS::threads, TS::items, TS::lbb>), grid, block, 0,
                               s, kin, kout, vin, vout, cnt, 8 * p, start + p * kRadix,
                               reinterpret_cast<uint32_t*>(base + L.lb), counter, err, X{});
        HPXHIP_CHECK_LAUNCH();
        return 0;
    };

    // Pass skipping needs the live digits on the host (a digit is live iff
    // OR and AND of the keys differ on it).  A sort that may take the hybrid
    // path counts only the two top digits first (the LDS atomics, not the
    // read, bound k_hist) and counts the rest only when it needs them.
    std::vector<unsigned long long> h(static_cast<size_t>(passes) * kRadix);
    std::vector<int> live;  // non-constant digits, most significant first
    int counted = (!HAS_VAL && sizeof(U) == 8 && n >= kHybridMin) ? passes - 2 : 0;
    auto count_digits = [&](int first) -> int {
        if ((rc = histogram(static_cast<const U*>(keys), n, first))) return rc;
        unsigned long long ob[2];
        HPXHIP_CHECK(hipMemcpyAsync(h.data(), hist, h.size() * 8, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipMemcpyAsync(ob, bits, 16, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));
        live.clear();
        for (int p = passes - 1; p >= 0; --p)
            if (((ob[0] ^ ob[1]) >> (8 * p)) & 0xffu) live.push_back(p);
        counted = first;
        return 0;
    };
    if ((rc = count_digits(counted))) return rc;
    if (counted > 0 && !(live.size() >= 3 && live[0] == passes - 1 && live[1] == passes - 2))
        if ((rc = count_digits(0))) return rc;

    U* kc = static_cast<U*>(keys);
    U* ka = reinterpret_cast<U*>(base + L.alt_keys);
    VAL* vc = static_cast<VAL*>(vals);
    VAL* va = reinterpret_cast<VAL*>(base + L.alt_vals);
    // LSD over live[from..] (least significant first), whole array, result in keys
    auto lsd = [&](size_t from) -> int {
        if (counted > 0 && (rc = histogram(kc, n, 0))) return rc;  // a permutation: same counts
        int executed = 0;
        for (size_t i = live.size(); i-- > from;) {
            if ((rc = pass(kc, ka, vc, va, n, live[i]))) return rc;
            std::swap(kc, ka);
            std::swap(vc, va);
            ++executed;
        }
        if (executed & 1) {
            HPXHIP_CHECK(hipMemcpyAsync(keys, kc, n * sizeof(U), hipMemcpyDeviceToDevice, s));
            if constexpr (HAS_VAL) HPXHIP_CHECK(hipMemcpyAsync(vals, vc, n * sizeof(VAL), hipMemcpyDeviceToDevice, s));
        }
        return 0;
    };

    if constexpr (HAS_VAL || sizeof(U) != 8) {
        return lsd(0);
    } else {
    bool hybrid = n >= kHybridMin && live.size() >= 3;
    if (hybrid) {
        unsigned long long m1 = 0, m2 = 0;
        for (int d = 0; d < kRadix; ++d) {
            m1 = std::max(m1, h[live[0] * kRadix + d]);
            m2 = std::max(m2, h[live[1] * kRadix + d]);
        }
        hybrid = static_cast<double>(m1) * static_cast<double>(m2) / static_cast<double>(n) <= 0.95 * kBucketCap;
    }
    if (!hybrid) return lsd(0);

    // ---- hybrid: prefix passes (p2, then p1: keys -> alt -> keys)
    const int p1 = live[0], p2 = live[1];
    if ((rc = pass(kc, ka, nullptr, nullptr, n, p2))) return rc;
    if ((rc = pass(ka, kc, nullptr, nullptr, n, p1))) return rc;
    auto* bounds = reinterpret_cast<uint64_t*>(base + L.bounds);
    hipLaunchKernelGGL((k_bucket_bounds<U, X>), dim3((kBuckets + 1 + 255) / 256), dim3(256), 0, s, kc, n, 8 * p1,
                       8 * p2, X{}, bounds);
    HPXHIP_CHECK_LAUNCH();
    std::vector<uint64_t> off(kBuckets + 1);
    HPXHIP_CHECK(hipMemcpyAsync(off.data(), bounds, off.size() * 8, hipMemcpyDeviceToHost, s));
    HPXHIP_CHECK(hipStreamSynchronize(s));

    // segments: runs of whole buckets of at most kBucketCap keys; larger
    // buckets are finished separately
    std::vector<uint64_t> segs;
    std::vector<std::pair<uint64_t, uint64_t>> big;
    uint64_t sb = 0, se = 0;
    auto close = [&] {
        if (se > sb) {
            segs.push_back(sb);
            segs.push_back(se);
        }
    };
    for (int v = 0; v < kBuckets; ++v) {
        const uint64_t bs = off[v], be = off[v + 1];
        if (be == bs) continue;
        if (be - bs > kBucketCap) {
            close();
            big.emplace_back(bs, be - bs);
            sb = se = be;
            continue;
        }
        if (be - sb > kBucketCap) {
            close();
            sb = bs;
        }
        se = be;
    }
    close();
    if (big.size() > kMaxBigBuckets) {
        // finish as plain LSD: low digits, then the prefix digits again
        return lsd(0);
    }

    if (!segs.empty()) {
        auto* segd = reinterpret_cast<uint64_t*>(base + L.segs);
        HPXHIP_CHECK(hipMemcpyAsync(segd, segs.data(), segs.size() * 8, hipMemcpyHostToDevice, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));  // `segs` is pageable and local
        hipLaunchKernelGGL((k_bucket_sort<U, X, kBucketThreads, kBucketItems>), dim3(static_cast<unsigned>(segs.size() / 2)),
                           dim3(kBucketThreads), 0, s, kc, segd, 8 * live[2] + 8, X{});
        HPXHIP_CHECK_LAUNCH();
    }
    // oversized buckets: LSD over the low digits of each, with its own histogram
    for (const auto& [bs, len] : big) {
        if ((rc = histogram(kc + bs, len, 0))) return rc;
        U* a = kc + bs;
        U* b = ka + bs;
        for (size_t i = live.size(); i-- > 2;) {
            if ((rc = pass(a, b, nullptr, nullptr, len, live[i]))) return rc;
            std::swap(a, b);
        }
        if (a != kc + bs) HPXHIP_CHECK(hipMemcpyAsync(kc + bs, a, len * sizeof(U), hipMemcpyDeviceToDevice, s));
    }
    return 0;
    }
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
