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
#ifndef HPXHIP_KV_THREADS
#define HPXHIP_KV_THREADS 256
#endif
#ifndef HPXHIP_KV_ITEMS
#define HPXHIP_KV_ITEMS 16
#endif
struct tile_shape {
    static constexpr int threads = HAS_VAL ? HPXHIP_KV_THREADS : 512;
    static constexpr int items = HAS_VAL ? HPXHIP_KV_ITEMS : 16;
    static constexpr int lbb = 4;
    static constexpr int tile = threads * items;
};

// tiles per chunk of the per-tile offset scan (k_chunk_sums, k_tile_offsets)
constexpr uint64_t kTileChunk = 256;

struct sort_layout {
    uint64_t ntiles;
    size_t alt_keys, alt_vals, hist, xhist, thist, joint, bits, start, xstart, tstart, bounds, ctl, counter, lb,
        lb_bytes, tcount, csum, nchunks, segs, big, shist, sstart, segs2, bs2, pad, pad_keys, total;
    bool wide;  // 64-bit granules
};

bool takes_pre18(uint64_t n, size_t vsize, int tile);
// r06: sort_by_key may plan 512 x 9 pair segments (k_bucket_sort C_SEGD); 0: A/B builds
#ifndef HPXHIP_SORT_KV512
#define HPXHIP_SORT_KV512 1
#endif
// r06: the padded second pass (k_pad_scatter); 0: the look-back pass (A/B builds)
#ifndef HPXHIP_SORT_PAD
#define HPXHIP_SORT_PAD 1
#endif
// the 18-bit form's segment capacity (kCap18 below), the padded pass's largest slot
constexpr uint64_t kPadSlotMax = 512 * 9;
constexpr uint64_t kHybridMin = 1ull << 22;

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
    L.thist = off;  // the top 9 bits' histogram (18-bit form)
    off += kXBins * 8;
    L.joint = off;  // ... per field region (8 x 512, k_hist_tiles; zeroed with the histograms)
    off += 8 * kXBins * 8;
    L.bits = off;  // OR / AND of the ordered keys
    off += 256;
    L.start = off;
    off += 8 * kRadix * 8;
    L.xstart = off;
    off += kXBins * 8;
    L.tstart = off;
    off += kXBins * 8;
    L.bounds = off;  // hybrid: bucket bounds (up to 2^18 + 1)
    off = align_up(off + 8 * (kMaxBuckets + 1), 256);
    L.ctl = off;  // the device-side plan (ctl words below)
    off += 256;
    L.counter = off;  // counter (16 B) immediately followed by lb: one zero fill per pass
    off += 256;
    L.lb = off;
    // room for a 9-bit pass, and for the tiles of a segmented one (each
    // segment rounds its tiles up)
    L.lb_bytes = (L.ntiles + kMaxBig) * kXBins * (L.wide ? 8 : 4);
    off = align_up(off + L.lb_bytes, 256);
    // 18-bit form, keys only, n < 2^32: per-tile field counts -> offsets of
    // the first prefix pass, and the chunk totals (k_hist_tiles); reserved
    // only when the sort takes that pass (2 KiB per 8192-key tile)
    const bool pre = takes_pre18(n, vsize, tile);
    L.nchunks = pre ? (L.ntiles + kTileChunk - 1) / kTileChunk : 0;
    L.tcount = off;
    off = align_up(off + (pre ? L.ntiles * kXBins * 4 : 0), 256);
    L.csum = off;
    off = align_up(off + L.nchunks * kXBins * 4, 256);
    // hybrid-sized sorts: the segmented LSD's table, the oversized bucket
    // ids, and per segment every digit's histogram and bin starts
    const bool hybrid = n >= kHybridMin;
    L.segs = off;
    off = align_up(off + (hybrid ? sizeof(seg_table) : 0), 256);
    L.big = off;
    off = align_up(off + (hybrid ? 4 * (kMaxBig + 1) : 0), 256);
    L.shist = off;
    off = align_up(off + (hybrid ? 8ull * kMaxBig * 8 * kRadix : 0), 256);
    L.sstart = off;
    off = align_up(off + (hybrid ? 8ull * kMaxBig * 8 * kRadix : 0), 256);
    // 18-bit form: the second prefix pass's 8 field regions and their bin starts
    L.segs2 = off;
    off = align_up(off + (pre ? sizeof(seg_table) : 0), 256);
    L.bs2 = off;
    off = align_up(off + (pre ? 8 * kXBins * 8 : 0), 256);
    // r06: the padded second pass's bucket slots (k_pad_scatter): room for
    // the plan's buckets x slot capacity, at most 2^18 x kCap18 (9.7 GB at
    // 2^30 u64 keys); the slot counters live at the start of lb (free until
    // the look-back pass that replaces a padded pass whose slot overflowed)
    L.pad_keys = pre ? std::min<uint64_t>(n + n / 4 + kPadSlotMax, static_cast<uint64_t>(kMaxBuckets) * kPadSlotMax) : 0;
    L.pad = off;
    off = align_up(off + L.pad_keys * ksize, 256);
    L.total = off;
    return L;
}

// Hybrid tail (keys-only sorts and pairs of at least 2^22 elements whose
// bucket sizes, estimated from the prefix fields' histograms, fit the LDS):
//   17-bit prefix (top byte + the 9 bits under it): segments of <= 9216 keys
//     sorted by 512-thread workgroups, two per CU, so one workgroup's loads
//     and stores overlap the other's LDS passes (7.2 vs 9.7 ms for the
//     segment sort at 2^30, profiles/r02_ubench_segment_sort.log);
//   16-bit prefix (the two top live bytes): the same 512-thread segments, or
//     1024-thread segments of <= 18432 keys (one workgroup per CU) for
//     buckets too large for both -- e.g. top bytes that are constant.
//   18-bit prefix (default, keys): the top 9 bits + the 9 bits under them,
//     ~4096-key buckets in 512 x 9 segments (kCap18 below).
// HPXHIP_SORT_HYBRID=0 / 16 / 17 selects the plain LSD / the 16-bit form /
// the 17-bit form (tests, ablations); a plan whose buckets do not fit its
// form's segments falls back to the 16-bit form, then to the LSD.
constexpr int kSegThreads16 = 1024, kSegThreads17 = 512, kSegItems = 18;
constexpr uint64_t kCap16 = static_cast<uint64_t>(kSegThreads16) * kSegItems;
constexpr uint64_t kCap17 = static_cast<uint64_t>(kSegThreads17) * kSegItems;
// sort_by_key: the 16-bit form with the values staged beside the keys,
// segments of <= 1024 x 9 pairs (144 KiB of LDS with 8-B values, one
// workgroup per CU).
constexpr int kSegItemsKV = 9;
constexpr uint64_t kCapKV = static_cast<uint64_t>(kSegThreads16) * kSegItemsKV;
// r06: pairs in 512 x 9 segments (72 KiB of keys and 8-B values: two
// workgroups per CU, so one's loads and stores overlap the other's LDS
// passes; the 1024 x 9 segment holds 144 KiB and runs alone on its CU),
// planned when the buckets fit -- e.g. 2^28 pairs with 2^16 buckets
constexpr uint64_t kCapKV2 = static_cast<uint64_t>(kSegThreads17) * kSegItemsKV;
// 18-bit form (keys, HPXHIP_SORT_HYBRID=18): two 9-bit prefix passes (the
// field [P-18, P-9), then the top 9 bits) and ~4096-key buckets sorted by
// 512 x 9 workgroups, three per CU (2^30 u64: 5.26 ms against 6.43-6.59 for
// the 8192-key 512 x 18 shape, profiles/r04_ubench_segment_occupancy.log).
constexpr int kSegItems18 = 9;
constexpr uint64_t kCap18 = static_cast<uint64_t>(kSegThreads17) * kSegItems18;
static_assert(kCap18 == kPadSlotMax, "padded slots hold a segment");
// r06: the one-pass segment sort (k_bucket_sort ONEB) bound to three
// workgroups per CU (6 waves per SIMD: <= 80 VGPRs); unbounded it took 119
// r06: the look-back second pass (the padded pass's fallback) as a
// persistent grid; 0: one workgroup per tile (A/B builds)
#ifndef HPXHIP_XREG_PERSIST
#define HPXHIP_XREG_PERSIST 1
#endif
#ifndef HPXHIP_SEG_MINW18
#define HPXHIP_SEG_MINW18 6
#endif
constexpr int kSegMinW18 = HPXHIP_SEG_MINW18;
// the 9-bit field under the top byte: bits [47, 56) of a 64-bit key, [15, 24) of a 32-bit one
template <typename U>
constexpr int field17_shift() { return static_cast<int>(8 * sizeof(U)) - 17; }
// 18-bit form: the field under the top 9 bits, and the top 9 bits
template <typename U>
constexpr int field18_shift() { return static_cast<int>(8 * sizeof(U)) - 18; }
template <typename U>
constexpr int top9_shift() { return static_cast<int>(8 * sizeof(U)) - 9; }

// Default form (r04): the 18-bit form -- 2^30 u64 17.81 vs 18.42 ms for the
// 17-bit form, u32 12.84 vs 13.03, u32 2^28 3.39 vs 3.68
// (profiles/r04_sort_probe_18bit.log): the 4096-key buckets' segment sort
// (5.1-5.4 ms against 6.4-6.6) more than pays for the second pass being
// 9-bit instead of 8-bit (5.3-5.6 against 4.7-4.9).
int hybrid_mode() {
    const char* e = std::getenv("HPXHIP_SORT_HYBRID");
    if (!e) return 18;
    return std::atoi(e);
}

// The 18-bit form's first prefix pass from precomputed tile offsets: keys
// only, n < 2^32 (32-bit offsets), 8192-key tiles, and a hybrid-sized sort
bool takes_pre18(uint64_t n, size_t vsize, int tile) {
    return vsize == 0 && n >= kHybridMin && n < (uint64_t(1) << 32) && tile == 8192 && hybrid_mode() == 18;
}

// ---------------------------------------------------------------- the plan
// The sort is planned ON THE DEVICE: the host enqueues one fixed sequence of
// kernels for (dtype, n, keys / pairs) and every kernel reads its part of
// the plan from these words and returns at once when the plan does not take
// it.  So no histogram, bucket bound or oversized flag travels to the host,
// the call returns as soon as the work is enqueued (sort.hpp:251-276 returns
// a future under task policies), and a sort can be captured in a graph.
enum : int {
    C_A9 = 0,          // shift of the 9-bit prefix pass (17-bit form), -1 = not run
    C_A8 = 1,          // shift of the second-byte prefix pass (16-bit form), -1
    C_B = 2,           // shift of the top-byte prefix pass, -1
    C_LSD = 3,         // [3, 11): LSD pass shifts, least significant first, -1
    C_BOUNDS = 11,     // {on, nb, s1, s2, b2} of k_bucket_bounds
    C_SEGA = 16,       // {on, nb, top_single}: 512-thread segment sort (keys) / the pairs kernel
    C_SEGB = 19,       // {on, nb, top_single}: 1024-thread segment sort (keys, buckets over 9216)
    C_OVERSIZED = 22,  // raised by a segment sort: a bucket over its LDS capacity
    C_HIST_A = 23,     // count digits [0, first) before the prefix passes
    C_HIST_B = 24,     // ... after a hybrid whose oversized buckets send the whole array to the LSD
    C_COPY = 25,       // the LSD ended in the alternate buffer: copy back
    C_PENDING = 26,    // stage 0 needs the second live byte's histogram to decide
    C_NLSD = 27,       // live digits
    C_DIGITS = 28,     // [28, 36): live digits, least significant first
    C_FIRST = 36,      // the first histogram counted digits [first, passes)
    C_B9 = 37,         // shift of the top-9-bit prefix pass (18-bit form), -1
    C_SEGC = 38,       // {on, nb, top_single}: 512 x 9 segment sort (18-bit form)
    C_SEGLSD = 44,     // hybrid-sized sorts: the LSD passes run over the segment table
    C_SEGHIST = 45,    // ... whose histograms are counted first (the oversized-bucket finish)
    C_REDO = 46,       // buckets the one-pass segment sort handed to the two-pass form (ids in the lb scratch)
    C_PAD = 47,        // r06: slot capacity of the padded second pass (k_pad_scatter), 0 = not taken
    C_B9P = 48,        // ... its top-9 shift, -1 = not run
    C_PADOVF = 49,     // ... raised when a slot overflowed (the look-back pass runs instead)
    C_SEGD = 50,       // r06: {on, nb, top_single}: 512 x 9 pairs segment sort (sort_by_key, buckets <= 4608)
    C_WORDS = 53
};
static_assert(C_WORDS * 4 <= 256, "plan words fit their slot");

// A bucket width is planned only if the estimated largest bucket, (largest
// top-byte bin) x (largest field bin) / n, plus five standard deviations of
// a Poisson count of that mean fits the segment's LDS capacity (a bucket
// over the capacity sends the whole sort to the LSD).  2^30 uniform keys:
// 8192 + 453 <= 9216 for 17-bit buckets.
__device__ inline bool fits(double est, double cap) { return est + 5.0 * sqrt(est) <= cap; }

__device__ inline int top_bit_d(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

// Planner, one thread.  stage 0 runs on the first histogram (the top digit
// and the 9-bit field under it for the 17-bit form, the two top digits for
// the 16-bit form; every digit for small sorts); stage 1 (after the gated count of the remaining digits) decides a
// plan stage 0 left pending.
//   17-bit form: the top two digits live, the 9-bit field's histogram known:
//     prefix passes on the 9-bit field then the top byte, buckets = top byte +
//     the top b2 <= 9 bits of the field, b2 the smallest whose estimated
//     largest bucket fits a 512-thread segment (two workgroups per CU);
//   16-bit form (pairs, or keys the 17-bit form does not fit): prefix passes
//     on the two top live bytes, b2 <= 8, a 512-thread (keys) / pairs
//     segment, or the 1024-thread keys segment for b2 = 8 buckets over 9216;
//   otherwise the LSD over the live digits.
// One segment covering the whole array (the segmented LSD as a plain LSD).
__device__ inline void whole_array(seg_table* segs, uint64_t n, int tile) {
    segs->nseg = 1;
    segs->start[0] = 0;
    segs->len[0] = n;
    segs->tile0[0] = 0;
    segs->tile0[1] = (n + tile - 1) / tile;
}

__global__ void k_sort_plan(const unsigned long long* __restrict__ hist, const unsigned long long* __restrict__ xhist,
                            const unsigned long long* __restrict__ thist,
                            const unsigned long long* __restrict__ bits, uint64_t n, int passes, int first, int mode,
                            int has_val, int stage, int32_t* __restrict__ ctl, seg_table* __restrict__ segs = nullptr,
                            uint32_t* __restrict__ big = nullptr, int tile = 0, uint64_t pad_keys = 0,
                            const unsigned long long* __restrict__ joint = nullptr) {
    if (blockIdx.x != 0) return;
    // 18-bit form: the statistics of the two 9-bit histograms, by the 64
    // threads of the launch (r05; one thread reading 9 x 512 bins took ~0.1
    // ms per plan): the largest top-9 bin; per field width b2 the largest
    // group of 2^(9-b2) field bins (all, and those without a hot bin); the
    // hot bins (over twice the mean) of both and their excess keys
    __shared__ double s_mtop, s_mt, s_et, s_ef, s_mg[10], s_mgn[10];
    __shared__ int s_jover[10];
    __shared__ int s_ht, s_hf;
    // r06: the field histogram staged in LDS first -- the group sums below
    // had walked it in global memory, one dependent load after another (the
    // plan took 85-140 us of every 2^30 sort, profiles/r06_sort_kernel_stats_u64_a.csv)
    __shared__ double s_x[kXBins];
    if (mode == 18 && !has_val && stage == 0 && thist) {
        const int t = threadIdx.x;
        for (int i = t; i < kXBins; i += 64) s_x[i] = static_cast<double>(xhist[i]);
        __syncthreads();
        const double mean = static_cast<double>(n) / kXBins;
        double mtop = 0, mt = mean, et = 0, ef = 0;
        int ht = 0, hf = 0;
        for (int i = t; i < kXBins; i += 64) {
            const double a = static_cast<double>(thist[i]), b = s_x[i];
            mtop = a > mtop ? a : mtop;
            if (a > 2 * mean) ++ht, et += a - mean;
            else mt = a > mt ? a : mt;
            if (b > 2 * mean) ++hf, ef += b - mean;
        }
        double mg[10], mgn[10];
        for (int b2 = 1; b2 <= 9; ++b2) {
            const int g = 1 << (9 - b2);
            mg[b2] = 0;
            mgn[b2] = 0;
            for (int i = t * g; i < kXBins; i += 64 * g) {
                double sum = 0;
                bool hot = false;
                for (int k = 0; k < g; ++k) {
                    const double b = s_x[i + k];
                    sum += b;
                    hot = hot || b > 2 * mean;
                }
                mg[b2] = sum > mg[b2] ? sum : mg[b2];
                if (!hot) mgn[b2] = sum > mgn[b2] ? sum : mgn[b2];
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            auto mx = [](double a, double b) { return a > b ? a : b; };
            mtop = mx(mtop, __shfl_xor(mtop, o));
            mt = mx(mt, __shfl_xor(mt, o));
            et += __shfl_xor(et, o);
            ef += __shfl_xor(ef, o);
            ht += __shfl_xor(ht, o);
            hf += __shfl_xor(hf, o);
            for (int b2 = 1; b2 <= 9; ++b2) {
                mg[b2] = mx(mg[b2], __shfl_xor(mg[b2], o));
                mgn[b2] = mx(mgn[b2], __shfl_xor(mgn[b2], o));
            }
        }
        // r06: the joint (field region x top-9) histogram bounds the buckets
        // from below, which the marginals cannot: per field width b2, the
        // cells that must hold a bucket over the segment -- b2 <= 3: a bucket
        // is exactly (top-9 digit, 2^(3 - b2) regions), its size the joint
        // sum; b2 > 3: a region's 2^(b2 - 3) buckets of one top-9 digit
        // share joint[r][t], so one holds at least joint / 2^(b2 - 3).  A
        // field correlated with the top bits (u64corr: every bucket oversized
        // while the marginals are uniform) had run the prefix passes and the
        // segment sorts for nothing before the whole-array LSD.
        int jover[10];
        for (int b2 = 1; b2 <= 9; ++b2) jover[b2] = 0;
        if (joint) {
            // staged in LDS first (as the field histogram): 64 independent
            // loads per thread instead of eight dependent rounds
            __shared__ float s_joint[8 * kXBins];
#pragma unroll 16
            for (int i = t; i < 8 * kXBins; i += 64) s_joint[i] = static_cast<float>(joint[i]);
            __syncthreads();
            for (int tt = t; tt < kXBins; tt += 64) {
                double j[8];
                for (int r = 0; r < 8; ++r) j[r] = static_cast<double>(s_joint[r * kXBins + tt]);
                for (int b2 = 1; b2 <= 9; ++b2) {
                    if (b2 <= 3) {
                        const int g = 1 << (3 - b2);
                        for (int r0 = 0; r0 < 8; r0 += g) {
                            double sum = 0;
                            for (int r = r0; r < r0 + g; ++r) sum += j[r];
                            jover[b2] += sum > static_cast<double>(kCap18);
                        }
                    } else {
                        // (j / 2^k > cap as j > cap * 2^k: exact, and no f64
                        // division -- 384 of them per thread had been most of
                        // the plan's ~50 us)
                        const double lim = static_cast<double>(kCap18) * static_cast<double>(1 << (b2 - 3));
                        for (int r = 0; r < 8; ++r) jover[b2] += j[r] > lim;
                    }
                }
            }
            for (int o = 32; o > 0; o >>= 1)
                for (int b2 = 1; b2 <= 9; ++b2) jover[b2] += __shfl_xor(jover[b2], o);
        }
        if (t == 0) {
            s_mtop = mtop, s_mt = mt, s_et = et, s_ef = ef, s_ht = ht, s_hf = hf;
            for (int b2 = 1; b2 <= 9; ++b2) s_mg[b2] = mg[b2], s_mgn[b2] = mgn[b2], s_jover[b2] = jover[b2];
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    if (stage == 1) {
        if (!ctl[C_PENDING]) return;
        first = 0;  // every digit is counted now
    } else {
        for (int i = 0; i < C_WORDS; ++i) ctl[i] = 0;
        for (int i = 0; i < 11; ++i) ctl[i] = -1;
        ctl[C_B9] = -1;
        ctl[C_B9P] = -1;
        ctl[C_FIRST] = first;
        if (big) big[0] = 0;
    }
    ctl[C_PENDING] = 0;
    const uint64_t diff = bits[0] ^ bits[1];
    int live[8], nl = 0;
    for (int p = passes - 1; p >= 0; --p)
        if ((diff >> (8 * p)) & 0xffu) live[nl++] = p;
    ctl[C_NLSD] = nl;
    for (int i = 0; i < nl; ++i) ctl[C_DIGITS + i] = live[nl - 1 - i];
    auto lsd = [&] {
        for (int i = 0; i < nl; ++i) ctl[C_LSD + i] = 8 * live[nl - 1 - i];
        ctl[C_COPY] = nl & 1;
        if (stage == 0) ctl[C_HIST_A] = first > 0;
        if (segs) {  // a hybrid-sized sort: its LSD runs as a one-segment segmented LSD
            whole_array(segs, n, tile);
            ctl[C_SEGLSD] = 1;
        }
    };
    if (mode == 0 || nl < 3) return lsd();
    const double dn = static_cast<double>(n);
    auto bin_max = [](const unsigned long long* c, int bins, int group) {
        unsigned long long m = 0;
        for (int g = 0; g < bins; g += group) {
            unsigned long long sum = 0;
            for (int j = 0; j < group; ++j) sum += c[g + j];
            m = sum > m ? sum : m;
        }
        return static_cast<double>(m);
    };
    auto plan = [&](int s1, int s2, int b2, int seg, int tbits = 8) {
        const uint32_t nb = (1u << tbits) << b2;
        ctl[C_BOUNDS + 0] = 1;
        ctl[C_BOUNDS + 1] = static_cast<int32_t>(nb);
        ctl[C_BOUNDS + 2] = s1;
        ctl[C_BOUNDS + 3] = s2;
        ctl[C_BOUNDS + 4] = b2;
        ctl[seg + 0] = 1;
        ctl[seg + 1] = static_cast<int32_t>(nb);
        ctl[seg + 2] = top_bit_d(diff & ((uint64_t(1) << s2) - 1));
    };
    const bool top_two = live[0] == passes - 1 && live[1] == passes - 2;
    if (mode == 18 && !has_val && stage == 0 && top_two) {
        // top 9 bits [8P - 9, 8P), field [8P - 18, 8P - 9): b2 <= 9 bits of the field
        const int fs = 8 * passes - 18;
        bool futile = false;
        for (int b2 = 1; b2 <= 9; ++b2) {
            const double est = s_mtop * s_mg[b2] / dn;
            // (r06) more cells over the segment than the bounded finish keeps:
            // a wider field, or no 18-bit plan
            if (fits(est, kCap18) && s_jover[b2] > kMaxBig) {
                futile = true;
                continue;
            }
            if (fits(est, kCap18)) {
                ctl[C_A9] = fs;
                // r06: the padded second pass when its slots -- the estimated
                // largest bucket + 7 sigma, whole 64-key lines -- fit the scratch
                const uint32_t nb = 512u << b2;
                uint32_t cap = (static_cast<uint32_t>(est + 7.0 * sqrt(est) + 1.0) + 63u) & ~63u;
                cap = cap < kCap18 ? cap : static_cast<uint32_t>(kCap18);
                if (pad_keys > 0 && static_cast<uint64_t>(nb) * cap <= pad_keys) {
                    ctl[C_B9P] = 8 * passes - 9;
                    ctl[C_PAD] = static_cast<int32_t>(cap);
                } else {
                    ctl[C_B9] = 8 * passes - 9;
                }
                return plan(8 * passes - 9, fs + 9 - b2, b2, C_SEGC, 9);
            }
        }
        if (futile) return lsd();  // (r06) the marginals fit, the joint histogram does not
        // r05: skew concentrated in a few buckets -- a few hot top-9 bins
        // whose excess keys sit in a few hot field bins (the same keys: the
        // excess masses match) -- is left to the bounded finish of the
        // oversized buckets (at most kMaxBig of them, k_sort_fallback) when
        // every bucket outside the hot bins fits: buckets sized for the keys
        // outside the hot bins (the fewest field bits whose groups without a
        // hot bin fit) are planned instead of the whole-array LSD (VERDICT
        // r04: one hot prefix had cost 2.5x the uniform sort).
        if (s_ht > 0 && s_hf > 0 && s_ht * s_hf <= kMaxBig && s_et <= 1.25 * s_ef && s_ef <= 1.25 * s_et) {
            const double mean = dn / kXBins;
            for (int b2 = 1; b2 <= 9; ++b2) {
                const double g = static_cast<double>(1 << (9 - b2)) * mean;
                if (fits(s_mt * (s_mgn[b2] > g ? s_mgn[b2] : g) / dn, kCap18)) {
                    ctl[C_A9] = fs;
                    ctl[C_B9] = 8 * passes - 9;
                    return plan(8 * passes - 9, fs + 9 - b2, b2, C_SEGC, 9);
                }
            }
        }
    }
    if (mode == 17 && !has_val && first > 0 && top_two) {
        const double m_top = bin_max(hist + live[0] * kRadix, kRadix, 1);
        const int fs = 8 * passes - 17;
        for (int b2 = 1; b2 <= 9; ++b2)
            if (fits(m_top * bin_max(xhist, kXBins, 1 << (9 - b2)) / dn, kCap17)) {
                ctl[C_A9] = fs;
                ctl[C_B] = 8 * live[0];
                return plan(8 * live[0], fs + 9 - b2, b2, C_SEGA);
            }
    }
    if (mode >= 16) {
        if (live[1] < first) {  // the second live byte was not counted: decide after the full count
            ctl[C_PENDING] = 1;
            ctl[C_HIST_A] = 1;
            return;
        }
        const double m_top = bin_max(hist + live[0] * kRadix, kRadix, 1);
        const unsigned long long* h2 = hist + live[1] * kRadix;
        if (has_val && HPXHIP_SORT_KV512)
            for (int b2 = 1; b2 <= 8; ++b2)
                if (fits(m_top * bin_max(h2, kRadix, 1 << (8 - b2)) / dn, kCapKV2)) {
                    ctl[C_A8] = 8 * live[1];
                    ctl[C_B] = 8 * live[0];
                    return plan(8 * live[0], 8 * live[1] + 8 - b2, b2, C_SEGD);
                }
        for (int b2 = 1; b2 <= 8; ++b2)
            if (fits(m_top * bin_max(h2, kRadix, 1 << (8 - b2)) / dn, has_val ? kCapKV : kCap17)) {
                ctl[C_A8] = 8 * live[1];
                ctl[C_B] = 8 * live[0];
                return plan(8 * live[0], 8 * live[1] + 8 - b2, b2, C_SEGA);
            }
        if (!has_val && fits(m_top * bin_max(h2, kRadix, 1) / dn, kCap16)) {
            ctl[C_A8] = 8 * live[1];
            ctl[C_B] = 8 * live[0];
            return plan(8 * live[0], 8 * live[1], 8, C_SEGB);
        }
    }
    lsd();
}

// After the segment sorts: buckets over their LDS capacity (skewed keys)
// were left unsorted.  Up to kMaxBig of them (the whole-array
// LSD for one oversized bucket cost 2.5-2.9x) are finished by a segmented
// LSD over their own ranges and the live digits under the bucket prefix
// (the keys of a bucket agree on every bit at or above s2); more send the
// whole array through the LSD over every live digit (a one-segment table).
// Either way the passes count their segments' histograms first.
__global__ void k_sort_fallback(int32_t* __restrict__ ctl, const uint64_t* __restrict__ bounds,
                                const uint32_t* __restrict__ big, seg_table* __restrict__ segs, uint64_t n,
                                int tile) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || ctl[C_OVERSIZED] == 0) return;
    const int nl = ctl[C_NLSD];
    const uint32_t nbig = big[0];
    int np = 0;
    if (nbig <= static_cast<uint32_t>(kMaxBig)) {
        uint32_t ids[kMaxBig];
        for (uint32_t i = 0; i < nbig; ++i) {  // the recorded buckets, in address order
            uint32_t v = big[1 + i], k = i;
            for (; k > 0 && ids[k - 1] > v; --k) ids[k] = ids[k - 1];
            ids[k] = v;
        }
        segs->nseg = nbig;
        uint64_t t = 0;
        for (uint32_t j = 0; j < nbig; ++j) {
            segs->start[j] = bounds[ids[j]];
            segs->len[j] = bounds[ids[j] + 1] - bounds[ids[j]];
            segs->tile0[j] = t;
            t += (segs->len[j] + tile - 1) / tile;
        }
        segs->tile0[nbig] = t;
        const int s2 = ctl[C_BOUNDS + 3];
        for (int i = 0; i < nl; ++i)
            if (8 * ctl[C_DIGITS + i] < s2) ctl[C_LSD + np++] = 8 * ctl[C_DIGITS + i];
        ctl[C_SEGHIST] = np > 0;  // their histograms: k_seg_hist over just their keys
    } else {
        // the whole array: its histograms from the optimized count (k_hist),
        // of the digits the first count skipped
        whole_array(segs, n, tile);
        for (int i = 0; i < nl; ++i) ctl[C_LSD + np++] = 8 * ctl[C_DIGITS + i];
        ctl[C_HIST_B] = ctl[C_FIRST] > 0 && !ctl[C_HIST_A];
    }
    ctl[C_COPY] = np & 1;
    ctl[C_SEGLSD] = np > 0;
}

// Zero fill of a pass's look-back state, run iff *gate >= 0 (the pass runs).
__global__ __launch_bounds__(256) void k_zero_gated(uint4* __restrict__ p, uint64_t n16, const int32_t* __restrict__ gate) {
    if (*gate < 0) return;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16; i += stride)
        p[i] = make_uint4(0, 0, 0, 0);
}

// After the padded second pass (r06): a slot overflowed -> the look-back
// pass runs from the same input, the bounds come from the binary search and
// the segment sort reads the keys; else the bounds come from the slot counts
// (k_pad_bounds) and the segment sort reads the slots.
__global__ void k_pad_check(int32_t* __restrict__ ctl) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || ctl[C_B9P] < 0) return;
    if (ctl[C_PADOVF]) {
        ctl[C_B9] = ctl[C_B9P];
        ctl[C_PAD] = 0;
    } else {
        ctl[C_BOUNDS] = 0;
    }
}

// dst[0, n) = src[0, n), run iff *gate != 0.
template <typename E>
__global__ __launch_bounds__(256) void k_copy_gated(const E* __restrict__ src, E* __restrict__ dst, uint64_t n,
                                                     const int32_t* __restrict__ gate) {
    if (*gate == 0) return;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

inline unsigned grid_for(uint64_t items, uint64_t cap = 8192) {
    const uint64_t g = (items + 255) / 256;
    return static_cast<unsigned>(g < 1 ? 1 : (g > cap ? cap : g));
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
    auto* xhist = reinterpret_cast<unsigned long long*>(base + L.xhist);
    auto* start = reinterpret_cast<unsigned long long*>(base + L.start);
    auto* xstart = reinterpret_cast<unsigned long long*>(base + L.xstart);
    auto* bits = reinterpret_cast<unsigned long long*>(base + L.bits);
    auto* bounds = reinterpret_cast<uint64_t*>(base + L.bounds);
    auto* ctl = reinterpret_cast<int32_t*>(base + L.ctl);
    uint32_t* counter = reinterpret_cast<uint32_t*>(base + L.counter);
    uint32_t* err = device_error_word(s);
    const int passes = static_cast<int>(sizeof(U));
    const unsigned hist_grid = static_cast<unsigned>(current_device_info().cus * kHistBlocksPerCU);
    constexpr int kField17Shift = field17_shift<U>();
    int mode = n >= kHybridMin ? hybrid_mode() : 0;
    if (HAS_VAL && mode > 16) mode = 16;  // no 9-bit pass with values
    // a sort that may take the hybrid counts only the digits its plan reads
    // first -- the LDS atomics, not the read, bound k_hist -- and the rest
    // only when the plan needs them: the 17-bit form reads the top byte and
    // the 9-bit field under it (r04: the second byte's count, which only the
    // 16-bit form reads, moved to the gated count; one LDS atomic per key
    // fewer), the 16-bit form the two top bytes
    const int first = mode == 18 ? passes : (mode == 17 ? passes - 1 : (mode ? passes - 2 : 0));
    const bool xfield = mode == 17 || mode == 18;
    auto* thist = reinterpret_cast<unsigned long long*>(base + L.thist);
    auto* tstart = reinterpret_cast<unsigned long long*>(base + L.tstart);

    U* kc = static_cast<U*>(keys);
    U* ka = reinterpret_cast<U*>(base + L.alt_keys);
    VAL* vc = static_cast<VAL*>(vals);
    VAL* va = reinterpret_cast<VAL*>(base + L.alt_vals);

    auto offsets = [&]() -> int {
        hipLaunchKernelGGL(k_bin_offsets<kRadix>, dim3(passes), dim3(kRadix), 0, s, hist, start);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    };
    // the remaining digits [0, first), iff *gate
    auto count_rest = [&](const int32_t* gate) -> int {
        hipLaunchKernelGGL((k_hist<U, X, kHistThreads>), dim3(hist_grid), dim3(kHistThreads), 0, s, kc, n, 0, first,
                           X{}, hist, bits, -1, xhist, gate, -1, static_cast<unsigned long long*>(nullptr), 1);
        HPXHIP_CHECK_LAUNCH();
        return offsets();
    };
    // one stable onesweep pass; ctl word: its digit shift or -1 (not run).
    // Launch geometry: passes the plan usually takes get one workgroup per
    // tile (a new workgroup starts as soon as one leaves); passes it usually
    // skips -- the LSD fallback of a hybrid-sized sort, the second-byte pass
    // of the 17-bit form -- a persistent grid of two workgroups per CU
    // claiming tiles (k_onesweep PERSIST), so skipping them costs one gate read
    // per workgroup.  A skipped 2^30-key pass with one workgroup per tile
    // dispatched 131072 workgroups that only read the gate: ~0.1 ms each,
    // ~0.9 ms per sort (19.3 -> 20.2 ms when the plan moved to the device);
    // running every pass persistent instead cost far more (26.3 ms: the
    // segment sort and the prefix passes lose the dispatcher's overlap of a
    // leaving workgroup with a starting one; profiles/r03_sort_probe_persistent.log).
    auto pass = [&](const U* kin, U* kout, const VAL* vin, VAL* vout, int rb, const int32_t* word,
                    bool persist, const unsigned long long* bs9 = nullptr, const uint32_t* pre = nullptr) -> int {
        const unsigned long long* b9 = bs9 ? bs9 : xstart;  // a 9-bit pass's bin starts
        const uint64_t nt = L.ntiles;
        // the look-back state; the PRE pass (no look-back) only claims tiles
        // from the counter (r06: it had zeroed all 268 MB of granules at 2^30)
        const uint64_t zbytes = pre ? 256 : align_up(256 + nt * (uint64_t(1) << rb) * (L.wide ? 8 : 4), 16);
        {  // (the PRE pass too: its tiles are claimed from the counter, which this zeroes)
            hipLaunchKernelGGL(k_zero_gated, dim3(grid_for(zbytes / 16, 2048)), dim3(256), 0, s,
                               reinterpret_cast<uint4*>(counter), zbytes / 16, word);
            HPXHIP_CHECK_LAUNCH();
        }
        const uint64_t cap = 2ull * static_cast<uint64_t>(current_device_info().cus);
        const dim3 grid(static_cast<unsigned>(persist && nt > cap ? cap : nt)), block(TS::threads);
        auto launch = [&](auto gtag, auto rbtag) {
            using G = decltype(gtag);
            constexpr int RB = decltype(rbtag)::value;
            // Tile ids: blockIdx for 32-bit keys (4 x 8-bit passes 15.9 vs
            // 16.3 ms at 2^30), the atomic counter for 64-bit keys (9-bit
            // pass 5.85 vs 6.23 ms, byte pass 4.93 vs 5.00;
            // profiles/r02_ubench_tile_order_ab.log); persistent grids
            // always claim from the counter.
            constexpr bool DYN = sizeof(U) == 8;
            if (persist)
                hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, G, X, TS::threads, TS::items, TS::lbb, RB, true, true,
                                               true>),
                                   grid, block, 0, s, kin, kout, vin, vout, n, 0, RB == 9 ? b9 : start,
                                   reinterpret_cast<G*>(base + L.lb), counter, err, X{}, word, nt);
            else
                hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, G, X, TS::threads, TS::items, TS::lbb, RB, true, DYN>),
                                   grid, block, 0, s, kin, kout, vin, vout, n, 0, RB == 9 ? b9 : start,
                                   reinterpret_cast<G*>(base + L.lb), counter, err, X{}, word);
        };
        using R8 = std::integral_constant<int, 8>;
        using R9 = std::integral_constant<int, 9>;
        if (rb == 9 && pre) {
            // precomputed tile offsets: no look-back.  Tile ids from the
            // counter, as the look-back pass takes them: in blockIdx order
            // the pass ran 8.4 ms against 5.1 (profiles/r04_sort_pre_blockidx.txt)
            // -- the order in which tiles finish decides how the partial
            // lines at the ends of their digit runs meet in the caches
            // r05: tiles in 8 contiguous regions, one per XCD (XREG): 4.75 ->
            // 3.81 ms at 2^30 u64 (profiles/r05_ubench_sortpass5.log)
            if constexpr (!HAS_VAL)
                hipLaunchKernelGGL((k_onesweep<U, VAL, false, uint32_t, X, TS::threads, TS::items, -1, 9, true, false,
                                               false, false, true>),
                                   grid, block, 0, s, kin, kout, vin, vout, n, 0, b9,
                                   reinterpret_cast<uint32_t*>(base + L.lb), counter, err, X{}, word, nt, pre);
        } else if (rb == 9) {
            if constexpr (!HAS_VAL) {
                if (L.wide) launch((unsigned long long)0, R9{});
                else launch(uint32_t(0), R9{});
            }
        } else {
            if (L.wide) launch((unsigned long long)0, R8{});
            else launch(uint32_t(0), R8{});
        }
        HPXHIP_CHECK_LAUNCH();
        return 0;
    };

    // ---- first histogram (+ OR / AND of the keys) and the plan
    HPXHIP_CHECK(hipMemsetAsync(hist, 0, 8 * kRadix * 8 + 10 * kXBins * 8, s));  // hist, xhist, thist, joint
    HPXHIP_CHECK(hipMemsetAsync(bits, 0, 8, s));
    HPXHIP_CHECK(hipMemsetAsync(bits + 1, 0xff, 8, s));
    // 18-bit form, keys, n < 2^32: the first count also leaves the field's
    // per-tile counts for the first prefix pass (k_hist_tiles)
    // (same-box A/B, profiles/r04_sort_ab_pre_offsets.log: 2^30 u64 17.99-18.05
    // -> 17.58-17.68 ms, u32 13.17-13.26 -> 12.55-12.62 against the look-back pass)
    const bool pre18 = takes_pre18(n, HAS_VAL ? sizeof(VAL) : 0, TS::tile);
    auto* tcount = reinterpret_cast<uint32_t*>(base + L.tcount);
    auto* csum = reinterpret_cast<uint32_t*>(base + L.csum);
    // (r05: tiles strided over 2 workgroups per CU; the chunk totals for the
    // offsets come from k_chunk_sums)
    if (pre18)
        hipLaunchKernelGGL((k_hist_tiles<U, X, 8192, kXBins>),
                           dim3(static_cast<unsigned>(std::min<uint64_t>(L.ntiles, 2ull * current_device_info().cus))),
                           dim3(kXBins), 0, s, kc, n, L.ntiles, X{}, field18_shift<U>(), top9_shift<U>(), tcount, xhist,
                           thist, bits, reinterpret_cast<unsigned long long*>(base + L.joint));
    else if (mode == 18)  // the field and the top 9 bits; no byte digit
        hipLaunchKernelGGL((k_hist<U, X, kHistThreads, 4, 2, true>), dim3(hist_grid), dim3(kHistThreads), 0, s, kc, n,
                           first, passes, X{}, hist, bits, field18_shift<U>(), xhist,
                           static_cast<const int32_t*>(nullptr), top9_shift<U>(), thist);
    else
        hipLaunchKernelGGL((k_hist<U, X, kHistThreads>), dim3(hist_grid), dim3(kHistThreads), 0, s, kc, n, first,
                           passes, X{}, hist, bits, xfield ? kField17Shift : -1, xhist,
                           static_cast<const int32_t*>(nullptr));
    HPXHIP_CHECK_LAUNCH();
    if ((rc = offsets())) return rc;
    if (xfield) {
        hipLaunchKernelGGL(k_bin_offsets<kXBins>, dim3(1), dim3(kXBins), 0, s, xhist, xstart);
        HPXHIP_CHECK_LAUNCH();
    }
    if (mode == 18) {
        hipLaunchKernelGGL(k_bin_offsets<kXBins>, dim3(1), dim3(kXBins), 0, s, thist, tstart);
        HPXHIP_CHECK_LAUNCH();
    }
    if (pre18) {  // the second prefix pass's field regions
        hipLaunchKernelGGL(k_region_plan, dim3(1), dim3(kXBins), 0, s, xstart, tstart,
                           reinterpret_cast<const unsigned long long*>(base + L.joint), n, TS::tile,
                           reinterpret_cast<seg_table*>(base + L.segs2),
                           reinterpret_cast<unsigned long long*>(base + L.bs2));
        HPXHIP_CHECK_LAUNCH();
    }
    // hybrid-sized sorts: the LSD runs over the segment table (the whole
    // array, or the oversized buckets the segment sorts leave)
    auto* segs = mode ? reinterpret_cast<seg_table*>(base + L.segs) : nullptr;
    auto* big = mode ? reinterpret_cast<uint32_t*>(base + L.big) : nullptr;
    hipLaunchKernelGGL(k_sort_plan, dim3(1), dim3(64), 0, s, hist, xhist, thist, bits, n, passes, first, mode,
                       HAS_VAL ? 1 : 0, 0, ctl, segs, big, TS::tile, static_cast<uint64_t>(HPXHIP_SORT_PAD ? L.pad_keys : 0),
                       pre18 ? reinterpret_cast<const unsigned long long*>(base + L.joint) : nullptr);
    HPXHIP_CHECK_LAUNCH();
    if (first > 0) {
        if ((rc = count_rest(ctl + C_HIST_A))) return rc;
        hipLaunchKernelGGL(k_sort_plan, dim3(1), dim3(64), 0, s, hist, xhist, thist, bits, n, passes, first, mode,
                           HAS_VAL ? 1 : 0, 1, ctl, segs, big, TS::tile);
        HPXHIP_CHECK_LAUNCH();
    }

    // ---- hybrid: prefix passes (keys -> alt -> keys), bucket bounds, per-bucket LDS sort
    if (mode) {
        if (pre18) {  // the first prefix pass's tile offsets, iff the plan takes it
            hipLaunchKernelGGL(k_chunk_sums, dim3(static_cast<unsigned>(L.nchunks)), dim3(kXBins), 0, s, tcount,
                               L.ntiles, static_cast<uint32_t>(kTileChunk), csum, ctl + C_A9);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_tile_chunk_scan, dim3(1), dim3(kXBins), 0, s, csum, L.nchunks, xstart, ctl + C_A9);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_tile_offsets, dim3(static_cast<unsigned>(L.nchunks)), dim3(kXBins), 0, s, tcount,
                               L.ntiles, static_cast<uint32_t>(kTileChunk), csum, ctl + C_A9);
            HPXHIP_CHECK_LAUNCH();
        }
        if (!HAS_VAL && (mode == 17 || mode == 18) &&
            (rc = pass(kc, ka, nullptr, nullptr, 9, ctl + C_A9, false, nullptr, pre18 ? tcount : nullptr)))
            return rc;
        // the second-byte pass runs in the 16-bit form only (pairs; keys the
        // 17-/18-bit form does not fit); the top-byte pass in the 16- and
        // 17-bit forms, the top-9-bit pass in the 18-bit form
        if ((rc = pass(kc, ka, vc, va, 8, ctl + C_A8, mode >= 17))) return rc;
        if ((rc = pass(ka, kc, va, vc, 8, ctl + C_B, mode == 18))) return rc;
        if constexpr (!HAS_VAL) {
            if (mode == 18 && pre18) {
                // r06: the padded second pass (k_pad_scatter), iff planned:
                // slot counters zeroed (with the tile counter), the pass, and
                // the check that hands a sort whose slots overflowed to the
                // look-back pass below
                const uint64_t nt = L.ntiles + 8;
                auto* pcnt = reinterpret_cast<unsigned long long*>(base + L.lb);
                const uint64_t pz = align_up(256 + 4ull * kMaxBuckets, 16);
                hipLaunchKernelGGL(k_zero_gated, dim3(grid_for(pz / 16, 2048)), dim3(256), 0, s,
                                   reinterpret_cast<uint4*>(counter), pz / 16, ctl + C_B9P);
                HPXHIP_CHECK_LAUNCH();
                hipLaunchKernelGGL((k_pad_scatter<U, X, TS::threads, TS::items>), dim3(static_cast<unsigned>(nt)),
                                   dim3(TS::threads), 0, s, ka, reinterpret_cast<U*>(base + L.pad), ctl + C_B9P,
                                   ctl + C_BOUNDS, ctl + C_PAD, reinterpret_cast<const seg_table*>(base + L.segs2),
                                   counter, pcnt, ctl + C_PADOVF, X{});
                HPXHIP_CHECK_LAUNCH();
                hipLaunchKernelGGL(k_pad_check, dim3(1), dim3(64), 0, s, ctl);
                HPXHIP_CHECK_LAUNCH();
                // r05: the top-9 pass over the field-ordered keys in 8 field
                // regions, one per XCD, each with its own look-back and bin
                // starts (k_region_plan): consecutive tiles' digit runs meet in
                // one L2, as in the first pass (XREG + SEG)
                const uint64_t zbytes = align_up(256 + nt * kXBins * (L.wide ? 8 : 4), 16);
                hipLaunchKernelGGL(k_zero_gated, dim3(grid_for(zbytes / 16, 2048)), dim3(256), 0, s,
                                   reinterpret_cast<uint4*>(counter), zbytes / 16, ctl + C_B9);
                HPXHIP_CHECK_LAUNCH();
                // r06: a persistent grid (two workgroups per CU claiming the
                // regions' tiles in order), since the padded pass leaves this
                // pass to its rare overflow: a skipped launch of one workgroup
                // per tile had dispatched 131080 workgroups that only read the
                // gate (~60 us per 2^30 sort)
                const unsigned gx = static_cast<unsigned>(std::min<uint64_t>(nt, 2ull * current_device_info().cus));
                auto launch = [&](auto gtag) {
                    using G = decltype(gtag);
                    hipLaunchKernelGGL((k_onesweep<U, VAL, false, G, X, TS::threads, TS::items, TS::lbb, 9, true, false,
                                                   HPXHIP_XREG_PERSIST != 0, true, true>),
                                       dim3(HPXHIP_XREG_PERSIST ? gx : static_cast<unsigned>(nt)), dim3(TS::threads), 0, s, ka, kc,
                                       static_cast<const VAL*>(nullptr), static_cast<VAL*>(nullptr), n, 0,
                                       reinterpret_cast<const unsigned long long*>(base + L.bs2),
                                       reinterpret_cast<G*>(base + L.lb), counter, err, X{}, ctl + C_B9, nt,
                                       static_cast<const uint32_t*>(nullptr),
                                       reinterpret_cast<const seg_table*>(base + L.segs2),
                                       static_cast<const unsigned long long*>(xstart));
                };
                if (L.wide) launch((unsigned long long)0);
                else launch(uint32_t(0));
                HPXHIP_CHECK_LAUNCH();
            } else if (mode == 18 && (rc = pass(ka, kc, nullptr, nullptr, 9, ctl + C_B9, false, tstart))) {
                return rc;
            }
        }
        hipLaunchKernelGGL((k_bucket_bounds<U, X>), dim3((kMaxBuckets + 1 + 255) / 256), dim3(256), 0, s, kc, n, 0, 0,
                           0, 0u, X{}, bounds, ctl + C_BOUNDS);
        HPXHIP_CHECK_LAUNCH();
        if (!HAS_VAL && mode == 18 && pre18) {  // the padded pass's bounds: a scan of its slot counts
            const auto* pcnt = reinterpret_cast<const unsigned long long*>(base + L.lb);
            auto* bsum = reinterpret_cast<uint64_t*>(base + L.lb + 4ull * kMaxBuckets);  // lb_bytes > 4 x 2^18 + 2 KiB
            const dim3 grid(kMaxBuckets / 1024);  // blocks past the plan's buckets leave
            hipLaunchKernelGGL(k_pad_sums, grid, dim3(256), 0, s, pcnt, ctl + C_BOUNDS, ctl + C_PAD, bsum);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL(k_pad_bounds, grid, dim3(256), 0, s, pcnt, ctl + C_BOUNDS, ctl + C_PAD,
                               static_cast<const uint64_t*>(bsum), bounds);
            HPXHIP_CHECK_LAUNCH();
        }
        auto* oversized = reinterpret_cast<uint32_t*>(ctl + C_OVERSIZED);
        // The segment sort the plan usually takes: one workgroup per bucket
        // over the buckets a typical plan has (twice n / 8192, at most the
        // 2^17 a plan can have; workgroups past the planned count leave), then
        // a grid striding over any further buckets (k_bucket_sort PERSIST,
        // two workgroups per CU: a skewed plan with more, smaller buckets), so
        // a small sort does not dispatch 2^17 workgroups.  Striding over all
        // buckets instead ran the 2^30 segment sort 7.2 -> 9.7 ms: the loop
        // costs the kernel 19 more spilled VGPRs
        // (profiles/r03_sort_probe_seg_persist.log,
        // r03_sort_kernel_stats_seg_persist.csv).  The 1024-thread keys
        // segment (buckets over 9216, rare) strides over all of them, one
        // workgroup per CU.
        const unsigned cus = static_cast<unsigned>(current_device_info().cus);
        const uint64_t want = 2 * (n / 8192 + 1);
        constexpr uint64_t kMax17 = uint64_t(1) << 17;  // a 16- or 17-bit plan's buckets
        const uint32_t g0 = static_cast<uint32_t>(want > kMax17 ? kMax17 : want);
        if constexpr (HAS_VAL) {
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItemsKV, 16, VAL, true, true>),
                               dim3(g0), dim3(kSegThreads16), 0, s, kc, bounds, 0, X{}, vc, oversized,
                               ctl + C_SEGA, 0u, big);
            HPXHIP_CHECK_LAUNCH();
            if (g0 < kMax17)
                hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItemsKV, 16, VAL, true, true, true>),
                                   dim3(cus), dim3(kSegThreads16), 0, s, kc, bounds, 0, X{}, vc, oversized,
                                   ctl + C_SEGA, g0, big);
            HPXHIP_CHECK_LAUNCH();
            // r06: the 512 x 9 pairs segments (C_SEGD): one workgroup per
            // expected bucket, then a striding grid over the rest
            constexpr uint64_t kMax16 = uint64_t(1) << 16;
            const uint64_t wantd = 2 * (n / 4096 + 1);
            const uint32_t gd = static_cast<uint32_t>(wantd > kMax16 ? kMax16 : wantd);
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItemsKV, 16, VAL, true, true>), dim3(gd),
                               dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, vc, oversized, ctl + C_SEGD, 0u, big);
            HPXHIP_CHECK_LAUNCH();
            if (gd < kMax16)
                hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItemsKV, 16, VAL, true, true, true>),
                                   dim3(2 * cus), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, vc, oversized,
                                   ctl + C_SEGD, gd, big);
        } else if (mode == 18) {
            // the 18-bit form's ~4096-key buckets: one workgroup per expected
            // bucket, then a striding grid; the 512 x 18 segment (a plan that
            // fell back to the 16-bit form) strides over all of them
            const uint64_t want18 = 2 * (n / 4096 + 1);
            const uint32_t g18 = static_cast<uint32_t>(want18 > kMaxBuckets ? kMaxBuckets : want18);
            // r06: the one-pass form (HPXHIP_SEG_ONE bits, k_bucket_sort ONEB);
            // buckets with a bin too large for it are listed (ctl[C_REDO], ids
            // in the look-back scratch, free after the prefix passes) and
            // sorted by the two-pass form in a third, striding launch
            auto* redo_n = reinterpret_cast<uint32_t*>(ctl + C_REDO);
            auto* redo_ids = reinterpret_cast<uint32_t*>(base + L.lb);  // lb_bytes >= 576 x 2 KiB > 4 x 2^18
            // (the padded pass's slot counters there are read by k_pad_bounds, before)
            const U* padp = L.pad_keys ? reinterpret_cast<const U*>(base + L.pad) : nullptr;
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems18, 16, uint32_t, false, true, false,
                                              kSegMinW18, false, HPXHIP_SEG_ONE>),
                               dim3(g18), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr, oversized,
                               ctl + C_SEGC, 0u, big, redo_n, HPXHIP_SEG_ONE > 0 ? redo_ids : nullptr,
                               padp, ctl + C_PAD);
            HPXHIP_CHECK_LAUNCH();
            if (g18 < kMaxBuckets)
                hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems18, 16, uint32_t, false, true, true,
                                                  kSegMinW18, false, HPXHIP_SEG_ONE>),
                                   dim3(3 * cus), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr,
                                   oversized, ctl + C_SEGC, g18, big, redo_n, HPXHIP_SEG_ONE > 0 ? redo_ids : nullptr,
                                   padp, ctl + C_PAD);
            HPXHIP_CHECK_LAUNCH();
            if (HPXHIP_SEG_ONE > 0)
                hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems18, 16, uint32_t, false, true, true>),
                                   dim3(3 * cus), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr,
                                   oversized, ctl + C_SEGC, 0u, big, redo_n, redo_ids, padp, ctl + C_PAD);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems, 16, uint32_t, false, true, true>),
                               dim3(2 * cus), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr,
                               oversized, ctl + C_SEGA, 0u, big);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItems, 16, uint32_t, false, true, true>),
                               dim3(cus), dim3(kSegThreads16), 0, s, kc, bounds, 0, X{}, nullptr,
                               oversized, ctl + C_SEGB, 0u, big);
        } else {
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems, 16, uint32_t, false, true>),
                               dim3(g0), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr, oversized,
                               ctl + C_SEGA, 0u, big);
            HPXHIP_CHECK_LAUNCH();
            if (g0 < kMax17)
                hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads17, kSegItems, 16, uint32_t, false, true, true>),
                                   dim3(2 * cus), dim3(kSegThreads17), 0, s, kc, bounds, 0, X{}, nullptr,
                                   oversized, ctl + C_SEGA, g0, big);
            HPXHIP_CHECK_LAUNCH();
            hipLaunchKernelGGL((k_bucket_sort<U, X, kSegThreads16, kSegItems, 16, uint32_t, false, true, true>),
                               dim3(cus), dim3(kSegThreads16), 0, s, kc, bounds, 0, X{}, nullptr,
                               oversized, ctl + C_SEGB, 0u, big);
        }
        HPXHIP_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_sort_fallback, dim3(1), dim3(64), 0, s, ctl, bounds, big, segs, n, TS::tile);
        HPXHIP_CHECK_LAUNCH();
        if (first > 0 && (rc = count_rest(ctl + C_HIST_B))) return rc;
    }

    if (mode) {
        // ---- a hybrid-sized sort's LSD (usually skipped): the planned LSD of
        // keys the hybrid does not fit (one segment: the whole array, bin
        // starts from the global histogram) or the oversized-bucket finish
        // (the recorded buckets, their histograms counted here).  Persistent
        // grids, every launch gated by the plan.
        auto* shist = reinterpret_cast<unsigned long long*>(base + L.shist);
        auto* sstart = reinterpret_cast<unsigned long long*>(base + L.sstart);
        const unsigned cus = static_cast<unsigned>(current_device_info().cus);
        HPXHIP_CHECK(hipMemsetAsync(shist, 0, 8ull * kMaxBig * 8 * kRadix, s));
        hipLaunchKernelGGL((k_seg_hist<U, X, 256, TS::tile>), dim3(2 * cus), dim3(256), 0, s, kc, segs, X{}, shist,
                           ctl + C_SEGHIST);
        HPXHIP_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_seg_offsets, dim3(kMaxBig * 8), dim3(kRadix), 0, s, shist, segs, sstart, ctl + C_SEGLSD,
                           ctl + C_SEGHIST, static_cast<const unsigned long long*>(hist));
        HPXHIP_CHECK_LAUNCH();
        const uint64_t nt = L.ntiles + kMaxBig;  // the segments' tiles (each segment rounds up)
        const uint64_t zbytes = align_up(256 + nt * kRadix * (L.wide ? 8 : 4), 16);
        for (int i = 0; i < passes; ++i) {
            const bool even = (i & 1) == 0;
            const int32_t* word = ctl + C_LSD + i;
            hipLaunchKernelGGL(k_zero_gated, dim3(grid_for(zbytes / 16, 2048)), dim3(256), 0, s,
                               reinterpret_cast<uint4*>(counter), zbytes / 16, word);
            HPXHIP_CHECK_LAUNCH();
            auto launch = [&](auto gtag) {
                using G = decltype(gtag);
                hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, G, X, TS::threads, TS::items, TS::lbb, 8, true, true,
                                               true, true>),
                                   dim3(2 * cus), dim3(TS::threads), 0, s, even ? kc : ka, even ? ka : kc,
                                   even ? vc : va, even ? va : vc, n, 0, sstart, reinterpret_cast<G*>(base + L.lb),
                                   counter, err, X{}, word, uint64_t(0), static_cast<const uint32_t*>(nullptr),
                                   static_cast<const seg_table*>(segs));
            };
            if (L.wide) launch((unsigned long long)0);
            else launch(uint32_t(0));
            HPXHIP_CHECK_LAUNCH();
        }
        hipLaunchKernelGGL((k_seg_copy<U>), dim3(grid_for(n)), dim3(256), 0, s, ka, kc, segs, ctl + C_COPY);
        HPXHIP_CHECK_LAUNCH();
        if constexpr (HAS_VAL) {
            hipLaunchKernelGGL((k_seg_copy<VAL>), dim3(grid_for(n)), dim3(256), 0, s, va, vc, segs, ctl + C_COPY);
            HPXHIP_CHECK_LAUNCH();
        }
        return 0;
    }

    // ---- LSD over the live digits (keys <-> alt): the plan of a small sort
    for (int i = 0; i < passes; ++i) {
        const bool even = (i & 1) == 0;
        if ((rc = pass(even ? kc : ka, even ? ka : kc, even ? vc : va, even ? va : vc, 8, ctl + C_LSD + i, false)))
            return rc;
    }
    hipLaunchKernelGGL((k_copy_gated<U>), dim3(grid_for(n)), dim3(256), 0, s, ka, kc, n, ctl + C_COPY);
    HPXHIP_CHECK_LAUNCH();
    if constexpr (HAS_VAL) {
        hipLaunchKernelGGL((k_copy_gated<VAL>), dim3(grid_for(n)), dim3(256), 0, s, va, vc, n, ctl + C_COPY);
        HPXHIP_CHECK_LAUNCH();
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
