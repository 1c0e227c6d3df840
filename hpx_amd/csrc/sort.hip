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
// Hybrid tail (keys-only sorts and 64-bit sort_by_key, >= 2^22 keys, >= 3
// live digits, bucket sizes estimated from the histograms within one
// workgroup's LDS): onesweep passes on the most significant live bits only
// (the 9-bit field under the top byte, then the top byte: a 17-bit prefix;
// or the two top live bytes), so every prefix value is a contiguous bucket;
// k_bucket_bounds finds the bucket starts by binary search; k_bucket_sort
// sorts each bucket (or a host-packed run of small buckets) completely inside
// one CU's LDS (two stable LDS passes + odd-even rounds, see sort_kernel.hpp).
// 56 B/key instead of 136 for random 2^30 u64 keys (42.3 -> 19.0 ms); 28
// instead of 36 for u32 keys, whose two LDS passes cover every bit under the
// prefix (15.8 -> 13.7 ms, profiles/r02_sort_u32_hybrid.log).
// Buckets larger than a segment are finished by per-bucket LSD; more than
// kMaxBigBuckets of them (skewed keys) by the plain LSD.  sort_by_key takes
// the 16-bit form with the values moved by the prefix passes and staged in
// LDS beside their keys (9216-pair segments): 2^28 u64/u64 pairs 20.7 ->
// 9.2 ms, 104 instead of 264 B/pair (profiles/r02_sort_by_key_hybrid.log).
#include "internal.hpp"
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdlib>
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
    size_t alt_keys, alt_vals, hist, xhist, bits, start, xstart, bounds, segs, counter, lb, lb_bytes, total;
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
    L.xhist = off;  // the 9-bit prefix field's histogram
    off += kXBins * 8;
    L.bits = off;  // OR / AND of the ordered keys
    off += 256;
    L.start = off;
    off += 8 * kRadix * 8;
    L.xstart = off;
    off += kXBins * 8;
    L.bounds = off;  // hybrid: bucket bounds (up to 2^17 + 1) and segment (begin, end) pairs
    off = align_up(off + 8 * (kMaxBuckets + 1), 256);
    L.segs = off;
    off = align_up(off + 16 * kMaxBuckets, 256);
    L.counter = off;  // counter (16 B) immediately followed by lb: one memset
    off += 256;
    L.lb = off;
    L.lb_bytes = L.ntiles * kXBins * (L.wide ? 8 : 4);  // room for a 9-bit pass
    off = align_up(off + L.lb_bytes, 256);
    L.total = off;
    return L;
}

// Hybrid tail (keys-only sorts of at least 2^22 keys whose bucket
// sizes, estimated from the prefix fields' histograms, fit the LDS):
//   17-bit prefix (top byte + the 9 bits under it): segments of <= 9216 keys
//     sorted by 512-thread workgroups, two per CU, so one workgroup's loads
//     and stores overlap the other's LDS passes (7.2 vs 9.7 ms for the
//     segment sort at 2^30, profiles/r02_ubench_segment_sort.log);
//   16-bit prefix (the two top live bytes): segments of <= 18432 keys, one
//     1024-thread workgroup per CU -- for buckets too large for the first
//     form (more than ~2^30.1 random keys) or top bytes that are constant.
// HPXHIP_SORT_HYBRID=0 / 16 turns the hybrid / its 17-bit form off (tests,
// ablations).
constexpr int kSegThreads16 = 1024, kSegThreads17 = 512, kSegItems = 18;
constexpr uint64_t kCap16 = static_cast<uint64_t>(kSegThreads16) * kSegItems;
constexpr uint64_t kCap17 = static_cast<uint64_t>(kSegThreads17) * kSegItems;
// sort_by_key (64-bit keys): the 16-bit form with the values staged beside
// the keys, segments of <= 1024 x 9 pairs (144 KiB of LDS with 8-B values,
// one workgroup per CU); buckets fit up to about 2^29 random pairs.
constexpr int kSegItemsKV = 9;
constexpr uint64_t kCapKV = static_cast<uint64_t>(kSegThreads16) * kSegItemsKV;
// the 9-bit field under the top byte: bits [47, 56) of a 64-bit key, [15, 24) of a 32-bit one
template <typename U>
constexpr int field17_shift() { return static_cast<int>(8 * sizeof(U)) - 17; }
constexpr uint64_t kHybridMin = 1ull << 22;
constexpr size_t kMaxBigBuckets = 64;  // more oversized buckets than this -> finish as plain LSD

int hybrid_mode() {
    const char* e = std::getenv("HPXHIP_SORT_HYBRID");
    if (!e) return 17;
    return std::atoi(e);
}

// HPXHIP_SORT_DIRECT=<d>: take the per-bucket segment sort when the average
// bucket holds at least 1/d of a segment (default 2; ablations).
double direct_divisor() {
    const char* e = std::getenv("HPXHIP_SORT_DIRECT");
    return e ? std::atof(e) : 2.0;
}

inline int top_bit(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

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
    auto* xhist = reinterpret_cast<unsigned long long*>(base + L.xhist);
    auto* start = reinterpret_cast<unsigned long long*>(base + L.start);
    auto* xstart = reinterpret_cast<unsigned long long*>(base + L.xstart);
    uint32_t* counter = reinterpret_cast<uint32_t*>(base + L.counter);
    uint32_t* err = device_error_word(s);
    const int passes = static_cast<int>(sizeof(U));
    const unsigned hist_grid = static_cast<unsigned>(current_device_info().cus * kHistBlocksPerCU);
    constexpr int kField17Shift = field17_shift<U>();
    // 32-bit keys: the two LDS passes under a 16/17-bit prefix sort a single
    // bucket's whole key (no odd-even rounds)
    int mode = n >= kHybridMin ? hybrid_mode() : 0;
    if (HAS_VAL && mode > 16) mode = 16;  // no 9-bit pass with values

    auto* bits = reinterpret_cast<unsigned long long*>(base + L.bits);
    // histograms of digits [first, passes) of keys[0, cnt) -> hist, their
    // exclusive bin starts -> start, OR / AND of the keys -> bits; with
    // xfield, also the 9-bit field under the top byte -> xhist / xstart
    auto histogram = [&](const U* k, uint64_t cnt, int first, bool xfield) -> int {
        HPXHIP_CHECK(hipMemsetAsync(hist, 0, 8 * kRadix * 8 + kXBins * 8, s));  // hist and xhist
        HPXHIP_CHECK(hipMemsetAsync(bits, 0, 8, s));
        HPXHIP_CHECK(hipMemsetAsync(bits + 1, 0xff, 8, s));
        hipLaunchKernelGGL((k_hist<U, X, kHistThreads>), dim3(hist_grid), dim3(kHistThreads), 0, s, k, cnt, first, passes,
                           X{}, hist, bits, xfield ? kField17Shift : -1, xhist);
        HPXHIP_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_bin_offsets<kRadix>, dim3(passes), dim3(kRadix), 0, s, hist, start);
        HPXHIP_CHECK_LAUNCH();
        if (xfield) {
            hipLaunchKernelGGL(k_bin_offsets<kXBins>, dim3(1), dim3(kXBins), 0, s, xhist, xstart);
            HPXHIP_CHECK_LAUNCH();
        }
        return 0;
    };
    // one stable onesweep pass of the rb-bit digit at `shift` over cnt keys
    auto pass = [&](const U* kin, U* kout, const VAL* vin, VAL* vout, uint64_t cnt, int shift, int rb,
                    const unsigned long long* bstart) -> int {
        const uint64_t nt = (cnt + TS::tile - 1) / TS::tile;
        HPXHIP_CHECK(hipMemsetAsync(counter, 0, 256 + nt * (uint64_t(1) << rb) * (L.wide ? 8 : 4), s));
        const dim3 grid(static_cast<unsigned>(nt)), block(TS::threads);
        auto launch = [&](auto gtag, auto rbtag) {
            using G = decltype(gtag);
            constexpr int RB = decltype(rbtag)::value;
            // Tile ids: blockIdx for 32-bit keys (4 x 8-bit passes 15.9 vs
            // 16.3 ms at 2^30), the atomic counter for 64-bit keys (9-bit
            // pass 5.85 vs 6.23 ms, byte pass 4.93 vs 5.00;
            // profiles/r02_ubench_tile_order_ab.log).
            constexpr bool DYN = sizeof(U) == 8;
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, G, X, TS::threads, TS::items, TS::lbb, RB, true, DYN>),
                               grid, block, 0,
                               s, kin, kout, vin, vout, cnt, shift, bstart, reinterpret_cast<G*>(base + L.lb), counter,
                               err, X{});
        };
        using R8 = std::integral_constant<int, 8>;
        using R9 = std::integral_constant<int, 9>;
        if (rb == 9) {
            if constexpr (!HAS_VAL) {
                if (L.wide) launch((unsigned long long)0, R9{});
                else launch(uint32_t(0), R9{});
            } else {
                return HPXHIP_ERROR_INVALID_ARGUMENT;
            }
        } else {
            if (L.wide) launch((unsigned long long)0, R8{});
            else launch(uint32_t(0), R8{});
        }
        HPXHIP_CHECK_LAUNCH();
        return 0;
    };
    auto pass8 = [&](const U* kin, U* kout, const VAL* vin, VAL* vout, uint64_t cnt, int p) -> int {
        return pass(kin, kout, vin, vout, cnt, 8 * p, 8, start + p * kRadix);
    };

    // Pass skipping needs the live digits on the host (a digit is live iff
    // OR and AND of the keys differ on it).  A sort that may take the hybrid
    // path counts only the two top digits (and the 9-bit field under the top
    // byte) first -- the LDS atomics, not the read, bound k_hist -- and counts
    // the rest only when it needs them.
    std::vector<unsigned long long> h(static_cast<size_t>(passes) * kRadix);
    std::vector<unsigned long long> hx(kXBins);
    std::vector<int> live;  // non-constant digits, most significant first
    uint64_t diff = 0;      // bits in which the keys differ (ordered form)
    // 17-bit form: the top byte and the 9-bit field; 16-bit form: the two top bytes
    int counted = mode ? passes - (mode == 17 ? 1 : 2) : 0;
    auto count_digits = [&](int first) -> int {
        const bool xf17 = mode == 17 && first > 0;
        if ((rc = histogram(static_cast<const U*>(keys), n, first, xf17))) return rc;
        unsigned long long ob[2];
        HPXHIP_CHECK(hipMemcpyAsync(h.data(), hist, h.size() * 8, hipMemcpyDeviceToHost, s));
        if (xf17) HPXHIP_CHECK(hipMemcpyAsync(hx.data(), xhist, hx.size() * 8, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipMemcpyAsync(ob, bits, 16, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));
        diff = ob[0] ^ ob[1];
        live.clear();
        for (int p = passes - 1; p >= 0; --p)
            if ((diff >> (8 * p)) & 0xffu) live.push_back(p);
        counted = first;
        return 0;
    };
    if ((rc = count_digits(counted))) return rc;
    const bool top_two = live.size() >= 3 && live[0] == passes - 1 && live[1] == passes - 2;
    if (counted > 0 && !top_two)
        if ((rc = count_digits(0))) return rc;
    const int counted_first = counted;  // the digits [counted_first, passes) have histograms

    U* kc = static_cast<U*>(keys);
    U* ka = reinterpret_cast<U*>(base + L.alt_keys);
    VAL* vc = static_cast<VAL*>(vals);
    VAL* va = reinterpret_cast<VAL*>(base + L.alt_vals);
    // LSD over live[from..] (least significant first), whole array, result in keys
    auto lsd = [&](size_t from) -> int {
        if (counted > 0 && (rc = histogram(kc, n, 0, false))) return rc;  // a permutation: same counts
        int executed = 0;
        for (size_t i = live.size(); i-- > from;) {
            if ((rc = pass8(kc, ka, vc, va, n, live[i]))) return rc;
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

    if (!mode || live.size() < 3) return lsd(0);
    auto max_of = [](const unsigned long long* c, int bins) {
        unsigned long long m = 0;
        for (int d = 0; d < bins; ++d) m = std::max(m, c[d]);
        return static_cast<double>(m);
    };
    const double dn = static_cast<double>(n);
    const double m_top = max_of(&h[live[0] * kRadix], kRadix);
    int variant = 0;  // 17 or 16 (prefix bits), 0 = plain LSD
    if (mode == 17 && counted_first > 0 && top_two && m_top * max_of(hx.data(), kXBins) / dn <= 0.95 * kCap17) {
        variant = 17;
    } else if (mode >= 16) {
        if (live[1] < counted_first && (rc = count_digits(0))) return rc;  // the second byte was not counted
        if (m_top * max_of(&h[live[1] * kRadix], kRadix) / dn <= 0.95 * (HAS_VAL ? kCapKV : kCap16)) variant = 16;
    }
    if (!variant) return lsd(0);

    // ---- prefix passes (low field, then the top live byte: keys -> alt -> keys)
    const int p1 = live[0];
    const int s2 = variant == 17 ? kField17Shift : 8 * live[1];
    const int b2 = variant == 17 ? 9 : 8;
    if (variant == 17) {
        if ((rc = pass(kc, ka, nullptr, nullptr, n, s2, 9, xstart))) return rc;
    } else {
        if ((rc = pass8(kc, ka, vc, va, n, live[1]))) return rc;
    }
    if ((rc = pass8(ka, kc, va, vc, n, p1))) return rc;
    const uint32_t nb = 256u << b2;
    auto* bounds = reinterpret_cast<uint64_t*>(base + L.bounds);
    hipLaunchKernelGGL((k_bucket_bounds<U, X>), dim3((nb + 1 + 255) / 256), dim3(256), 0, s, kc, n, 8 * p1, s2, b2, nb,
                       X{}, bounds);
    HPXHIP_CHECK_LAUNCH();
    // the highest bit in which keys of one bucket can differ
    const int top_single = top_bit(diff & ((uint64_t(1) << s2) - 1));
    const uint64_t cap = HAS_VAL ? kCapKV : variant == 17 ? kCap17 : kCap16;
    std::vector<uint64_t> off;
    auto read_bounds = [&]() -> int {
        off.resize(nb + 1);
        HPXHIP_CHECK(hipMemcpyAsync(off.data(), bounds, off.size() * 8, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));
        return 0;
    };
    // oversized buckets: LSD over the live bytes under the prefix, with the
    // bucket's own histogram (the byte that holds bit 47 under a 17-bit
    // prefix is included: its prefix bit is constant inside the bucket)
    auto finish_big = [&](const std::vector<std::pair<uint64_t, uint64_t>>& big) -> int {
        for (const auto& [bs, len] : big) {
            if ((rc = histogram(kc + bs, len, 0, false))) return rc;
            U* a = kc + bs;
            U* b = ka + bs;
            VAL* av = HAS_VAL ? vc + bs : nullptr;
            VAL* bv = HAS_VAL ? va + bs : nullptr;
            for (size_t i = live.size(); i-- > 0;) {
                if (8 * live[i] >= s2) continue;
                if ((rc = pass8(a, b, av, bv, len, live[i]))) return rc;
                std::swap(a, b);
                std::swap(av, bv);
            }
            if (a != kc + bs) {
                HPXHIP_CHECK(hipMemcpyAsync(kc + bs, a, len * sizeof(U), hipMemcpyDeviceToDevice, s));
                if constexpr (HAS_VAL)
                    HPXHIP_CHECK(hipMemcpyAsync(vc + bs, av, len * sizeof(VAL), hipMemcpyDeviceToDevice, s));
            }
        }
        return 0;
    };
    // Buckets of at least DIRECT_DIV-th of a segment on average (random keys
    // from about 2^29.2 up with the 17-bit prefix): one workgroup per bucket
    // straight from the bounds, so no read-back and host packing (1.2 ms of
    // idle GPU at 2^30, profiles/r02_sort_direct_buckets.log) sits between
    // the prefix passes and the segment sort; only an oversized bucket brings
    // the bounds to the host.
    const double direct_div = direct_divisor();
    if (top_single > 0 && (HAS_VAL || variant == 17) &&
        direct_div * static_cast<double>(n) >= static_cast<double>(nb) * cap) {
        auto* oversized = reinterpret_cast<uint32_t*>(bits + 2);
        HPXHIP_CHECK(hipMemsetAsync(oversized, 0, 4, s));
        if constexpr (HAS_VAL)
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItemsKV, 16, VAL, true, true>), dim3(nb),
                               dim3(kSegThreads16), 0, s, kc, bounds, top_single, X{}, vc, oversized);
        else
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems, 16, uint32_t, false, true>), dim3(nb),
                               dim3(kSegThreads17), 0, s, kc, bounds, top_single, X{}, nullptr, oversized);
        HPXHIP_CHECK_LAUNCH();
        uint32_t big_flag = 0;
        HPXHIP_CHECK(hipMemcpyAsync(&big_flag, oversized, 4, hipMemcpyDeviceToHost, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));
        if (!big_flag) return 0;
        if ((rc = read_bounds())) return rc;
        std::vector<std::pair<uint64_t, uint64_t>> big;
        for (uint32_t v = 0; v < nb; ++v)
            if (off[v + 1] - off[v] > cap) big.emplace_back(off[v], off[v + 1] - off[v]);
        if (big.size() > kMaxBigBuckets) return lsd(0);
        return finish_big(big);
    }
    if ((rc = read_bounds())) return rc;

    // segments: runs of whole buckets of at most `cap` keys; larger buckets
    // are finished separately
    std::vector<uint64_t> segs;
    std::vector<std::pair<uint64_t, uint64_t>> big;
    uint64_t sb = 0, se = 0;
    auto close = [&] {
        if (se > sb) {
            segs.push_back(sb);
            segs.push_back(se);
        }
    };
    for (uint32_t v = 0; v < nb; ++v) {
        const uint64_t bs = off[v], be = off[v + 1];
        if (be == bs) continue;
        if (be - bs > cap) {
            close();
            big.emplace_back(bs, be - bs);
            sb = se = be;
            continue;
        }
        if (be - sb > cap) {
            close();
            sb = bs;
        }
        se = be;
    }
    close();
    if (big.size() > kMaxBigBuckets) return lsd(0);  // plain LSD from here (the prefix passes are wasted)

    if (!segs.empty() && top_single > 0) {
        auto* segd = reinterpret_cast<uint64_t*>(base + L.segs);
        HPXHIP_CHECK(hipMemcpyAsync(segd, segs.data(), segs.size() * 8, hipMemcpyHostToDevice, s));
        HPXHIP_CHECK(hipStreamSynchronize(s));  // `segs` is pageable and local
        const dim3 grid(static_cast<unsigned>(segs.size() / 2));
        if constexpr (HAS_VAL)
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItemsKV, 16, VAL, true>), grid,
                               dim3(kSegThreads16), 0, s, kc, segd, top_single, X{}, vc);
        else if (variant == 17)
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems>), grid, dim3(kSegThreads17), 0, s, kc,
                               segd, top_single, X{});
        else
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItems>), grid, dim3(kSegThreads16), 0, s, kc,
                               segd, top_single, X{});
        HPXHIP_CHECK_LAUNCH();
    }
    return finish_big(big);
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
    HPXHIP_ANNOTATE("hpxhip_sort");
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
    HPXHIP_ANNOTATE("hpxhip_sort_by_key");
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
