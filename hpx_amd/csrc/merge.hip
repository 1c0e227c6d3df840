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

// ---------------------------------------------------------- multiway merge
// hpxhip_merge_runs (r05): the p <= 8 sorted runs the segmented sort's
// all-to-all delivers, merged in ONE pass over the keys (16 B/key) instead of
// ceil(log2 p) pairwise rounds (3 x 16 B/key at p = 8).
//   1. k_mw_samples: every S-th key of every run (p sorted sample runs, kept),
//      merged pairwise (run_merge) into one sorted sample of M keys;
//   2. splitters v_k = sample[k q], k = 1 .. K-1 (q = 3p); k_mw_bounds: for
//      every splitter and run the lower and upper bound -- first in the run's
//      own samples (a few MiB, cache resident), then inside the S keys
//      between two of them;
//   3. k_mw_merge, one 256-thread workgroup per task k: the keys equal to
//      v_k are copied straight to their place (any order is sorted), the
//      keys strictly between v_k and v_{k+1} -- at most (q + p) S = CAP of
//      them: run j holds fewer than (c_j + 1) S keys between two of its
//      samples, and at most q samples lie strictly between two splitters --
//      are staged in LDS (as ordered bits) and merged there by ceil(log2 p)
//      merge-path rounds (outputs staged in registers: one LDS buffer,
//      16 KiB, so several workgroups share a CU), then written out.  Task k starts at output
//      position sum_j lower_bound_j(v_k); a repeated splitter leaves its
//      equal keys to the last task holding it.
// Keys only (equal keys are interchangeable), in the sort's key order.
// Measured at 2^30 u64 (profiles/r05_merge_runs_variants.log): p = 4 5.4 ms
// against 6.5 for two pairwise rounds, p = 8 8.4 against 9.8, p = 2 3.8
// against 3.3 -- the LDS rounds, not the bytes, bound it; the segmented sort
// takes it for 4 <= p <= 8.
inline size_t merge_scratch_bytes_for(uint64_t n) { return ((n + kTile - 1) / kTile + 1) * 8; }

// (HPXHIP_MW_THREADS / HPXHIP_MW_MINW: variant builds for the probes only)
#ifndef HPXHIP_MW_THREADS
#define HPXHIP_MW_THREADS 256
#endif
#ifndef HPXHIP_MW_MINW
#define HPXHIP_MW_MINW 8
#endif
#ifndef HPXHIP_MW_ITEMS
#define HPXHIP_MW_ITEMS 8
#endif
// HPXHIP_MW_ROUND: 1 = branch-free merge step (one LDS read per output),
// 0 = the two-sided step; HPXHIP_MW_ABLATE (probes only, wrong output): 1 =
// no LDS rounds
#ifndef HPXHIP_MW_ROUND
#define HPXHIP_MW_ROUND 1
#endif
#ifndef HPXHIP_MW_ABLATE
#define HPXHIP_MW_ABLATE 0
#endif
constexpr int kMwThreads = HPXHIP_MW_THREADS;
constexpr int kMwItems = HPXHIP_MW_ITEMS;
constexpr int kMwCap = kMwThreads * kMwItems;  // keys strictly between two splitters, at most
constexpr int kMwMaxRuns = 8;
constexpr uint32_t kMwQ = 3;  // splitters every kMwQ * p samples

struct mw_runs {
    uint64_t off[kMwMaxRuns + 1];   // run j = in[off[j], off[j + 1])
    uint64_t soff[kMwMaxRuns + 1];  // run j's samples = sample[soff[j], soff[j + 1])
    uint32_t p;
    uint32_t stride;  // S
    uint32_t q;       // samples per splitter
};

template <typename U>
__global__ __launch_bounds__(256) void k_mw_samples(const U* __restrict__ in, mw_runs r, U* __restrict__ sample) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= r.soff[r.p]) return;
    uint32_t j = 0;
    while (j + 1 < r.p && r.soff[j + 1] <= i) ++j;
    sample[i] = in[r.off[j] + (i - r.soff[j]) * r.stride];
}

// first index in [lo, hi) of a[] whose key is not before v (UPPER: after v)
template <bool UPPER, typename U, typename X>
__device__ __forceinline__ uint64_t mw_search(const U* a, uint64_t lo, uint64_t hi, U v, X xf) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const U x = xf(a[mid]);
        if (UPPER ? (x <= v) : (x < v)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// lower (UPPER: upper) bound of v in run j, through the run's samples
template <bool UPPER, typename U, typename X>
__device__ __forceinline__ uint64_t mw_bound(const U* run, uint64_t len, const U* samp, uint64_t ns, uint32_t S, U v,
                                            X xf) {
    // c samples (run[0], run[S], ...) are before v: the bound is in
    // ((c - 1) S, c S]
    const uint64_t c = mw_search<UPPER>(samp, 0, ns, v, xf);
    if (c == 0) return 0;
    const uint64_t lo = (c - 1) * S + 1;
    const uint64_t hi = c * S < len ? c * S : len;
    return mw_search<UPPER>(run, lo, hi, v, xf);
}

// LB / UB [(K + 1) x p]: row k = the lower / upper bounds of splitter v_k in
// every run, relative to the run's start (row 0: 0, row K: the run lengths)
template <typename U, typename X>
__global__ __launch_bounds__(256) void k_mw_bounds(const U* __restrict__ in, mw_runs r, const U* __restrict__ runsamp,
                                                   const U* __restrict__ sorted, uint64_t K, X xf,
                                                   uint64_t* __restrict__ LB, uint64_t* __restrict__ UB) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= (K + 1) * r.p) return;
    const uint64_t k = i / r.p;
    const uint32_t j = static_cast<uint32_t>(i % r.p);
    const uint64_t len = r.off[j + 1] - r.off[j];
    if (k == 0 || k == K) {
        LB[i] = UB[i] = k == 0 ? 0 : len;
        return;
    }
    const U* run = in + r.off[j];
    const U* samp = runsamp + r.soff[j];
    const uint64_t ns = r.soff[j + 1] - r.soff[j];
    const U v = xf(sorted[k * r.q]);
    const uint64_t lb = mw_bound<false>(run, len, samp, ns, r.stride, v, xf);
    LB[i] = lb;
    // distinct keys: the key at the lower bound is already past v
    UB[i] = (lb == len || xf(run[lb]) != v) ? lb : mw_bound<true>(run, len, samp, ns, r.stride, v, xf);
}

// LDS position of staged key i: one pad element every 8, so the lanes of a
// merge round -- 8 outputs apart, 64 B for u64 -- do not pile onto the same
// banks (16 lanes per bank unpadded)
__device__ __forceinline__ constexpr int mw_pad(int i) { return i + (i >> 3); }

// One round inside the LDS: runs (2i, 2i + 1) of s (bounds b[0..nruns])
// merged in place; thread t computes outputs [8t, 8t + 8) into registers,
// then (after the barrier every thread reaches) writes them back.  The pair
// state is set up by a merge-path search at the thread's first output and
// restarted (at the pair's start, no search) when the outputs cross into
// the next pair.  s holds the keys' ordered bits (staged through xf), so the
// rounds compare and move plain unsigned words for every dtype.
template <typename U>
__device__ __forceinline__ void mw_round(U* s, const int* b, int nruns, int total) {
    const int o0 = static_cast<int>(threadIdx.x) * kMwItems;
    U r[kMwItems];
    int a0 = 0, a1 = 0, b1 = 0, ia = 0, ib = 0, la = 0, lb = 0, pi = 0;
    U va{}, vb{};
    auto enter = [&](int i, int dk) {  // pair i, its first dk outputs done
        pi = i;
        a0 = b[2 * i];
        const bool pair = 2 * i + 1 < nruns;
        a1 = pair ? b[2 * i + 1] : b[nruns];
        b1 = pair ? b[2 * i + 2] : a1;
        la = a1 - a0;
        lb = b1 - a1;
        int lo = dk > lb ? dk - lb : 0, hi = dk < la ? dk : la;
        while (lo < hi) {  // a-elements among the pair's first dk outputs (a first on ties)
            const int mid = (lo + hi) >> 1;
            if (!(s[mw_pad(a1 + dk - mid - 1)] < s[mw_pad(a0 + mid)])) lo = mid + 1;
            else hi = mid;
        }
        ia = lo;
        ib = dk - lo;
        va = s[mw_pad(a0 + (ia < la ? ia : 0))];
        vb = s[mw_pad(a1 + (ib < lb ? ib : 0))];
    };
    if (o0 < total) {
        int i = 0;
        while (2 * (i + 1) < nruns && b[2 * (i + 1)] <= o0) ++i;
        enter(i, o0 - b[2 * i]);
    }
#pragma unroll
    for (int q = 0; q < kMwItems; ++q) {
        const int o = o0 + q;
        if (o < total) {
            while (o == b1 && 2 * (pi + 1) < nruns) enter(pi + 1, 0);  // (skipping empty pairs)
#if HPXHIP_MW_ROUND == 1
            // one LDS read per output: the head of the side taken (an
            // exhausted side's index reads the other run's first key or the
            // pad element past the last run, never used)
            const bool takeb = ib < lb && (ia >= la || vb < va);
            r[q] = takeb ? vb : va;
            ia += takeb ? 0 : 1;
            ib += takeb ? 1 : 0;
            const U nv = s[mw_pad(takeb ? a1 + ib : a0 + ia)];
            va = takeb ? va : nv;
            vb = takeb ? nv : vb;
#else
            const bool takeb = ia >= la || (ib < lb && vb < va);
            if (takeb) {
                r[q] = vb;
                ++ib;
                vb = s[mw_pad(a1 + (ib < lb ? ib : 0))];
            } else {
                r[q] = va;
                ++ia;
                va = s[mw_pad(a0 + (ia < la ? ia : 0))];
            }
#endif
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kMwItems; ++q)
        if (o0 + q < total) s[mw_pad(o0 + q)] = r[q];
    __syncthreads();
}

// Keys are staged as ordered bits and turned back at the write-out.  (The
// first version compared xf(a) < xf(b) inside the rounds; builds with other
// register budgets -- __launch_bounds__(256, 8), 512 threads -- then wrote
// some float64 keys in their transformed form, ~bits of the right key
// (scripts/mw_debug.py, profiles/r05_merge_runs_debug.log): the round loop no
// longer holds a key in two forms.)  8 waves per SIMD (40-58 VGPRs, no
// scratch): p = 4 5.4 ms, p = 8 8.4 ms at 2^30 u64, against 5.7 / 8.9 with
// the default bound and 6.2 / 9.5 with 512 threads
// (profiles/r05_merge_runs_variants.log).
template <typename U, typename X, bool VEC>
__global__ __launch_bounds__(kMwThreads, HPXHIP_MW_MINW) void k_mw_merge(const U* __restrict__ in, mw_runs r,
                                                                          const uint64_t* __restrict__ LB,
                                                                          const uint64_t* __restrict__ UB, X xf,
                                                                          U* __restrict__ out,
                                                                          uint32_t* __restrict__ err) {
    __shared__ alignas(16) U s[mw_pad(kMwCap) + 1];  // (+1: a finished run's head reads one past)
    __shared__ int sbnd[kMwMaxRuns + 1];
    // run j: keys == v_k at [eq_j, lo_j), keys strictly between at [lo_j, hi_j)
    // (round 6: the per-run bounds live in LDS, one thread per run loads
    // them -- held in scalar registers they had pushed the kernel to 20-24
    // SGPR spills, the regime in which an earlier form was miscompiled, see
    // DESIGN.md (e); the build refuses SGPR spills here, Makefile)
    __shared__ uint64_t s_eq[kMwMaxRuns], s_lo[kMwMaxRuns], s_hi[kMwMaxRuns], s_go[kMwMaxRuns];
    const uint64_t k = blockIdx.x;
    const uint32_t p = r.p;
    if (threadIdx.x < p) {
        const uint32_t j = threadIdx.x;
        const uint64_t e = LB[k * p + j], l = UB[k * p + j], h = LB[(k + 1) * p + j];
        s_eq[j] = e;
        s_lo[j] = l;
        s_hi[j] = h;
        s_go[j] = r.off[j];
    }
    __syncthreads();
    // v_{k+1} == v_k (a repeated splitter: some run holds keys equal to v_k
    // before lower_bound(v_{k+1})): the last task with this splitter copies
    // its equal keys, this one has nothing to do
    bool dup = false;
    for (uint32_t j = 0; j < p; ++j) dup = dup || s_hi[j] < s_lo[j];
    if (dup) return;
    uint64_t pos = 0;  // sum_j lower_bound_j(v_k): where the task's output starts
    for (uint32_t j = 0; j < p; ++j) pos += s_eq[j];
    // the keys equal to v_k, run after run
    for (uint32_t j = 0; j < p; ++j) {
        const uint64_t ne = s_lo[j] - s_eq[j];
        const U* src = in + s_go[j] + s_eq[j];
        for (uint64_t e = threadIdx.x; e < ne; e += kMwThreads) out[pos + e] = src[e];
        pos += ne;
    }
    uint64_t total = 0;
    for (uint32_t j = 0; j < p; ++j) total += s_hi[j] - s_lo[j];
    if (total > static_cast<uint64_t>(kMwCap)) {  // cannot happen with consistent keys (see above)
        if (threadIdx.x == 0) raise_device_error(err, HPXHIP_DEVERR_RANGE);
        return;
    }
    // stage the runs' middle parts back to back (a loop per run: staging
    // flattened over the runs -- every load issued before the first LDS
    // store -- measured slower, r05 lease ai: p = 2 4.34 vs 3.65 ms, p = 8
    // 7.74 vs 7.75)
    int c = 0;
    for (uint32_t j = 0; j < p; ++j) {
        const int nj = static_cast<int>(s_hi[j] - s_lo[j]);
        if constexpr (VEC) {  // 16-B loads of the aligned vectors covering the part
            constexpr int V = 16 / sizeof(U);
            using VT = vec<U, V>;
            const uint64_t g0 = s_go[j] + s_lo[j], g1 = s_go[j] + s_hi[j];
            const VT* vs = reinterpret_cast<const VT*>(in);
            // whole vectors below g1 only (round 6, ADVICE r05: the vector
            // holding g1 - 1 also holds keys past the last run, which may
            // be past the buffer -- scripts/diag/mw_host caught the read
            // under ASan); the ragged tail by scalar loads
            const uint64_t vend = g1 / V;
            for (uint64_t v = g0 / V + threadIdx.x; v < vend; v += kMwThreads) {
                const VT x = ld_stream(&vs[v]);
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = v * V + e;
                    if (i >= g0) s[mw_pad(c + static_cast<int>(i - g0))] = xf(x.v[e]);
                }
            }
            const uint64_t t0 = vend * V > g0 ? vend * V : g0;
            for (uint64_t i = t0 + threadIdx.x; i < g1; i += kMwThreads)
                s[mw_pad(c + static_cast<int>(i - g0))] = xf(in[i]);
        } else {
            const U* src = in + s_go[j] + s_lo[j];
            for (int e = threadIdx.x; e < nj; e += kMwThreads) s[mw_pad(c + e)] = xf(ld_stream(&src[e]));
        }
        if (threadIdx.x == 0) sbnd[j] = c;
        c += nj;
    }
    if (threadIdx.x == 0) sbnd[p] = c;
    __syncthreads();
    const int n = c;
    int nruns = HPXHIP_MW_ABLATE ? 1 : static_cast<int>(p);
    while (nruns > 1) {
        mw_round(s, sbnd, nruns, n);
        const int nn = (nruns + 1) / 2;
        if (threadIdx.x == 0) {
            for (int i = 1; i < nn; ++i) sbnd[i] = sbnd[2 * i];
            sbnd[nn] = n;
        }
        __syncthreads();
        nruns = nn;
    }
    // write-out: a head up to the output's next 128-B line, 16-B vectors, a
    // tail (out 16-B aligned when VEC); line-aligned vectors keep two waves
    // from writing halves of one line (copy_if_kernel.hpp OUT_ALIGN)
    U* o = out + pos;
    constexpr int V = 16 / sizeof(U);
    using VT = vec<U, V>;
    const int head = VEC ? min(n, static_cast<int>(((128u - (reinterpret_cast<uintptr_t>(o) & 127u)) & 127u) / sizeof(U)))
                         : n;
    const int nvec = (n - head) / V;
    for (int e = threadIdx.x; e < head; e += kMwThreads) o[e] = xf.inverse(s[mw_pad(e)]);
    for (int q = threadIdx.x; q < nvec; q += kMwThreads) {
        VT w;
#pragma unroll
        for (int e = 0; e < V; ++e) w.v[e] = xf.inverse(s[mw_pad(head + q * V + e)]);
        st_stream(reinterpret_cast<VT*>(o + head) + q, w);
    }
    for (int e = head + nvec * V + threadIdx.x; e < n; e += kMwThreads) o[e] = xf.inverse(s[mw_pad(e)]);
}

// sample stride S for p runs: the bound (q + p) S <= kMwCap with q = kMwQ p
inline uint32_t mw_stride(uint32_t p) { return static_cast<uint32_t>(kMwCap / ((kMwQ + 1) * p)); }

struct mw_layout {
    uint64_t M, K;
    size_t runsamp, sa, sb, splits, lb, ub, total;
};

inline mw_layout mw_plan(const uint64_t* len, uint32_t p) {
    mw_layout L{};
    const uint32_t S = mw_stride(p);
    const uint64_t q = kMwQ * p;
    for (uint32_t j = 0; j < p; ++j) L.M += (len[j] + S - 1) / S;
    L.K = (L.M + q - 1) / q;
    if (L.K == 0) L.K = 1;
    size_t off = 0;
    L.runsamp = off;  // the samples in run order (kept for the bound searches)
    off = align_up(off + L.M * 8, 256);
    L.sa = off;  // the merge's ping-pong buffers
    off = align_up(off + L.M * 8, 256);
    L.sb = off;
    off = align_up(off + L.M * 8, 256);
    L.splits = off;
    off = align_up(off + merge_scratch_bytes_for(L.M), 256);
    L.lb = off;
    off = align_up(off + (L.K + 1) * p * 8, 256);
    L.ub = off;
    off = align_up(off + (L.K + 1) * p * 8, 256);
    L.total = off;
    return L;
}

template <typename T, bool DESC>
int run_merge_runs(const void* in, const uint64_t* off, uint32_t p, void* out, hipStream_t s, void* scratch,
                   size_t scratch_bytes) {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    using X = ordered_bits<T, DESC>;
    const U* ui = static_cast<const U*>(in) + off[0];
    mw_runs r{};
    r.p = p;
    r.stride = mw_stride(p);
    r.q = kMwQ * p;
    uint64_t len[kMwMaxRuns];
    for (uint32_t j = 0; j <= p; ++j) r.off[j] = off[j] - off[0];
    for (uint32_t j = 0; j < p; ++j) len[j] = r.off[j + 1] - r.off[j];
    for (uint32_t j = 0; j < p; ++j) r.soff[j + 1] = r.soff[j] + (len[j] + r.stride - 1) / r.stride;
    const mw_layout L = mw_plan(len, p);
    void* ws = nullptr;
    int rc = resolve_scratch(s, scratch, scratch_bytes, L.total, &ws);
    if (rc) return rc;
    char* base = static_cast<char*>(ws);
    U* runsamp = reinterpret_cast<U*>(base + L.runsamp);
    U* sbuf[2] = {reinterpret_cast<U*>(base + L.sa), reinterpret_cast<U*>(base + L.sb)};
    if (L.M) {
        hipLaunchKernelGGL((k_mw_samples<U>), dim3(static_cast<unsigned>((L.M + 255) / 256)), dim3(256), 0, s, ui, r,
                           runsamp);
        HPXHIP_CHECK_LAUNCH();
    }
    // the sample's p sorted runs, merged pairwise (runsamp -> sa -> sb -> sa ...)
    uint64_t sr[kMwMaxRuns + 1];
    uint32_t ns = p;
    for (uint32_t j = 0; j <= p; ++j) sr[j] = r.soff[j];
    const U* src = runsamp;
    int which = 0;
    while (ns > 1) {
        U* dst = sbuf[which];
        uint32_t nn = 0;
        for (uint32_t j = 0; j < ns; j += 2) {
            const uint64_t a0 = sr[j], a1 = sr[j + 1];
            if (j + 1 < ns) {
                const uint64_t b1 = sr[j + 2];
                if (b1 > a0 && (rc = run_merge<T, DESC>(src + a0, a1 - a0, src + a1, b1 - a1, dst + a0, s,
                                                        base + L.splits, merge_scratch_bytes_for(L.M))))
                    return rc;
            } else if (a1 > a0) {
                HPXHIP_CHECK(hipMemcpyAsync(dst + a0, src + a0, (a1 - a0) * sizeof(U), hipMemcpyDeviceToDevice, s));
            }
            sr[nn++] = a0;
        }
        sr[nn] = sr[ns];
        ns = nn;
        src = dst;
        which ^= 1;
    }
    auto* LB = reinterpret_cast<uint64_t*>(base + L.lb);
    auto* UB = reinterpret_cast<uint64_t*>(base + L.ub);
    const uint64_t nb = (L.K + 1) * p;
    hipLaunchKernelGGL((k_mw_bounds<U, X>), dim3(static_cast<unsigned>((nb + 255) / 256)), dim3(256), 0, s, ui, r,
                       runsamp, src, L.K, X{}, LB, UB);
    HPXHIP_CHECK_LAUNCH();
    if ((reinterpret_cast<uintptr_t>(ui) | reinterpret_cast<uintptr_t>(out)) % 16 == 0)
        hipLaunchKernelGGL((k_mw_merge<U, X, true>), dim3(static_cast<unsigned>(L.K)), dim3(kMwThreads), 0, s, ui, r,
                           LB, UB, X{}, static_cast<U*>(out), device_error_word(s));
    else
        hipLaunchKernelGGL((k_mw_merge<U, X, false>), dim3(static_cast<unsigned>(L.K)), dim3(kMwThreads), 0, s, ui, r,
                           LB, UB, X{}, static_cast<U*>(out), device_error_word(s));
    HPXHIP_CHECK_LAUNCH();
    return 0;
}

}  // namespace

namespace hpxhip {
size_t merge_scratch_bytes(uint64_t n) { return ((n + kTile - 1) / kTile + 1) * 8; }
// worst case over the run counts for n keys in total (the sample is largest
// at 8 runs, plus one partial sample block per run)
size_t merge_runs_scratch_bytes(uint64_t n) {
    size_t worst = 0;
    for (uint32_t p = 2; p <= kMwMaxRuns; ++p) {
        uint64_t len[kMwMaxRuns] = {};
        len[0] = n;
        for (uint32_t j = 1; j < p; ++j) len[j] = 1;  // every run adds a partial sample block
        const mw_layout L = mw_plan(len, p);
        worst = std::max(worst, L.total + static_cast<size_t>(p) * 8 * 4 + 4096);
    }
    return worst;
}
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

int hpxhip_merge_runs(int dtype, const void* in, const uint64_t* run_offsets, int nruns, void* out, int descending,
                      hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_merge_runs");
    if (!run_offsets || nruns < 1 || nruns > kMwMaxRuns) return HPXHIP_ERROR_INVALID_ARGUMENT;
    for (int j = 0; j < nruns; ++j)
        if (run_offsets[j + 1] < run_offsets[j]) return HPXHIP_ERROR_INVALID_ARGUMENT;
    const uint64_t n = run_offsets[nruns] - run_offsets[0];
    if (n == 0) return 0;
    if (!in || !out) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        if (nruns == 1) {
            HPXHIP_CHECK(hipMemcpyAsync(out, static_cast<const T*>(in) + run_offsets[0], n * sizeof(T),
                                        hipMemcpyDeviceToDevice, s));
            return 0;
        }
        const uint32_t p = static_cast<uint32_t>(nruns);
        if (descending) return run_merge_runs<T, true>(in, run_offsets, p, out, s, scratch, scratch_bytes);
        return run_merge_runs<T, false>(in, run_offsets, p, out, s, scratch, scratch_bytes);
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
