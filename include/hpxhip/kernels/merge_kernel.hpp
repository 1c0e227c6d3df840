// merge_kernel.hpp -- merge-path merge and the block / pass kernels of a
// comparison merge sort (see hpx_amd/csrc/merge.hip for the merge notes).
// Every kernel orders elements through a strict weak ordering `less(a, b)`:
// the library passes the radix sort's ordered-bits comparison (key_less), the
// C++ layer's device closures a user comparator (sort.hpp:364 with any comp
// and projection; hpx/parallel/detail/device_algorithms.hpp).
//
// Stability (merge.hpp:52-80: take from the second range only when
// comp(*first2, *first1)): equal elements keep first-range-first order in
// every merge, and the block sort's odd-even network swaps only strictly
// ordered neighbours, so the merge sort is stable.
#pragma once

#include <hpxhip/kernels/common.hpp>

namespace hpxhip {
namespace merge_detail {

constexpr int kThreads = 256;
// r04: 16 items per thread (4096-element tiles) ran the 2^28 u64 comparator
// sort 24.7 ms against 18.2 (profiles/r04_closure_timing_sort_items16.log)
constexpr int kItems = 8;
constexpr int kTile = kThreads * kItems;  // output elements per merge block

// a <= b in the ordering: !(b < a)
template <typename T, typename Less>
__device__ __forceinline__ bool not_after(const T& a, const T& b, const Less& less) {
    return !less(b, a);
}

// The radix sort's key order as a comparator (integers as std::less,
// floats in IEEE total order; descending inverts), merge.hip's form.
template <typename X>
struct key_less {
    X xf;
    template <typename U>
    __device__ __forceinline__ bool operator()(U a, U b) const {
        return xf(a) < xf(b);
    }
};

// Number of a-elements among the first d outputs of the stable merge.
template <typename T, typename Less>
__device__ __forceinline__ uint64_t path_split(const T* a, uint64_t na, const T* b, uint64_t nb, uint64_t d,
                                               const Less& less) {
    uint64_t lo = d > nb ? d - nb : 0;
    uint64_t hi = d < na ? d : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (not_after(a[mid], b[d - mid - 1], less)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <typename T, typename Less>
__global__ __launch_bounds__(256) void k_merge_partition(const T* __restrict__ a, uint64_t na, const T* __restrict__ b,
                                                          uint64_t nb, uint64_t ntiles, Less less,
                                                          uint64_t* __restrict__ splits) {
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (t > ntiles) return;
    const uint64_t total = na + nb;
    const uint64_t d = t * kTile < total ? t * kTile : total;
    splits[t] = path_split(a, na, b, nb, d, less);
}

template <typename T>
constexpr int vec_elems() {
    return (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? static_cast<int>(16 / sizeof(T)) : 1;
}

// Stage src[lo, hi) into dst[0, hi - lo); VEC: aligned 16-B loads (src 16-B
// aligned), else element loads.
template <typename T, bool VEC>
__device__ __forceinline__ void stage(const T* __restrict__ src, uint64_t lo, uint64_t hi, T* dst) {
    if (hi <= lo) return;
    if constexpr (VEC && vec_elems<T>() > 1) {
        constexpr int V = vec_elems<T>();
        using VT = vec<T, V>;
        const uint64_t v0 = lo / V, v1 = (hi + V - 1) / V;
        const VT* vs = reinterpret_cast<const VT*>(src);
        for (uint64_t v = v0 + threadIdx.x; v < v1; v += kThreads) {
            const VT x = ld_stream(&vs[v]);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = v * V + e;
                if (i >= lo && i < hi) dst[i - lo] = x.v[e];
            }
        }
    } else {
        for (uint64_t i = lo + threadIdx.x; i < hi; i += kThreads) dst[i - lo] = src[i];
    }
}

// Merge of the tile's two runs staged in s[0, la) and s[la, la + lb):
// thread k's kItems outputs from its diagonal, written back into s.
template <typename T, typename Less>
__device__ __forceinline__ void merge_in_lds(T* s, int la, int lb, const Less& less) {
    const int len = la + lb;
    const int dk = min(static_cast<int>(threadIdx.x) * kItems, len);
    int lo = dk > lb ? dk - lb : 0, hi = dk < la ? dk : la;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (not_after(s[mid], s[la + dk - mid - 1], less)) lo = mid + 1;
        else hi = mid;
    }
    int ia = lo, ib = dk - lo;
    T r[kItems];
    // the heads of both runs stay in registers; branch-free step (r05, as
    // hpxhip_merge_runs' mw_round): one LDS read per output, the head of the
    // side taken (an exhausted side's index reads a key never used)
    T va = s[ia < la ? ia : 0];
    T vb = s[la + ib < len ? la + ib : 0];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        const bool takeb = ib < lb && (ia >= la || less(vb, va));
        r[k] = takeb ? vb : va;
        ia += takeb ? 0 : 1;
        ib += takeb ? 1 : 0;
        const int ni = takeb ? la + ib : ia;
        const T nv = s[ni < len ? ni : 0];
        va = takeb ? va : nv;
        vb = takeb ? nv : vb;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems; ++k)
        if (dk + k < len) s[dk + k] = r[k];
    __syncthreads();
}

// One block per kTile outputs of merge(a[0, na), b[0, nb)) -> out.
// VEC: a, b and out 16-B aligned (16-B loads and stores).
template <typename T, typename Less, bool VEC>
__global__ __launch_bounds__(kThreads) void k_merge(const T* __restrict__ a, uint64_t na, const T* __restrict__ b,
                                                     uint64_t nb, const uint64_t* __restrict__ splits, Less less,
                                                     T* __restrict__ out, uint32_t* __restrict__ err = nullptr) {
    __shared__ T s[kTile];
    const uint64_t t = blockIdx.x;
    const uint64_t total = na + nb;
    const uint64_t d0 = t * kTile;
    const uint64_t d1 = d0 + kTile < total ? d0 + kTile : total;
    // clamped as in k_pass_merge: consistent splits pass unchanged; a clamp
    // that changes one raises the device error word
    const uint64_t s0 = splits[t], s1 = splits[t + 1];
    const uint64_t a1 = min(s1, min(na, d1));
    const uint64_t a0 = min(s0, min(a1, d0));
    const uint64_t b0 = min(d0 - a0, nb), b1 = max(b0, min(d1 - a1, nb));
    if (threadIdx.x == 0 && (a0 != s0 || a1 != s1 || b0 != d0 - a0 || b1 != d1 - a1))
        raise_device_error(err, HPXHIP_DEVERR_RANGE);
    const int la = static_cast<int>(a1 - a0), lb = static_cast<int>(b1 - b0);
    const int len = la + lb;
    stage<T, VEC>(a, a0, a1, s);
    stage<T, VEC>(b, b0, b1, s + la);
    __syncthreads();
    merge_in_lds(s, la, lb, less);
    constexpr int V = vec_elems<T>();
    if (VEC && V > 1 && len == kTile) {
        using VT = vec<T, V>;
        VT* vo = reinterpret_cast<VT*>(out + d0);
        const VT* vsrc = reinterpret_cast<const VT*>(s);
        for (int v = threadIdx.x; v < kTile / V; v += kThreads) st_stream(&vo[v], vsrc[v]);
    } else {
        for (int i = threadIdx.x; i < len; i += kThreads) out[d0 + i] = s[i];
    }
}

// ------------------------------------------------------------ merge sort
// Block sort: one block sorts kTile consecutive elements in LDS -- each
// thread's kItems with an odd-even transposition network in registers, then
// log2(kThreads) rounds of merge-path merges of run pairs in LDS.
template <typename T, typename Less>
__global__ __launch_bounds__(kThreads) void k_block_sort(T* __restrict__ data, uint64_t n, Less less) {
    __shared__ T s[kTile];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    const int len = static_cast<int>(n - base < kTile ? n - base : kTile);
    for (int i = threadIdx.x; i < len; i += kThreads) s[i] = data[base + i];
    __syncthreads();
    // thread-local runs of kItems (the last thread's may be shorter)
    const int t0 = static_cast<int>(threadIdx.x) * kItems;
    const int cnt = len > t0 ? (len - t0 < kItems ? len - t0 : kItems) : 0;
    T r[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) r[k] = k < cnt ? s[t0 + k] : s[0];
#pragma unroll
    for (int round = 0; round < kItems; ++round)
#pragma unroll
        for (int k = round & 1; k + 1 < kItems; k += 2)
            if (k + 1 < cnt && less(r[k + 1], r[k])) {
                const T x = r[k];
                r[k] = r[k + 1];
                r[k + 1] = x;
            }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems; ++k)
        if (k < cnt) s[t0 + k] = r[k];
    __syncthreads();
    // merge runs of w -> 2w inside the block
    for (int w = kItems; w < kTile; w *= 2) {
        const int pair = t0 / (2 * w);                 // run pair of this thread's outputs
        const int p0 = pair * 2 * w;
        const int la = len > p0 ? (len - p0 < w ? len - p0 : w) : 0;
        const int lb = len > p0 + w ? (len - p0 - w < w ? len - p0 - w : w) : 0;
        const int dk = t0 - p0;                        // diagonal inside the pair
        T* sa = s + p0;
        int ia = 0, ib = 0;
        if (dk < la + lb) {
            int lo = dk > lb ? dk - lb : 0, hi = dk < la ? dk : la;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (not_after(sa[mid], sa[la + dk - mid - 1], less)) lo = mid + 1;
                else hi = mid;
            }
            ia = lo;
            ib = dk - lo;
        }
        const int outs = dk < la + lb ? (la + lb - dk < kItems ? la + lb - dk : kItems) : 0;
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            if (k < outs) {
                const bool takeb = ia >= la || (ib < lb && less(sa[la + ib], sa[ia]));
                r[k] = takeb ? sa[la + ib] : sa[ia];
                if (takeb) ++ib;
                else ++ia;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kItems; ++k)
            if (k < outs) s[t0 + k] = r[k];
        __syncthreads();
    }
    for (int i = threadIdx.x; i < len; i += kThreads) data[base + i] = s[i];
}

// One merge pass of the sort: sorted runs of w elements (w a multiple of
// kTile) are merged pairwise, src -> dst.  Split points: one per output
// tile, tiles never straddle a run pair.
template <typename T, typename Less>
__global__ __launch_bounds__(256) void k_pass_partition(const T* __restrict__ src, uint64_t n, uint64_t w,
                                                         uint64_t ntiles, Less less, uint64_t* __restrict__ splits) {
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (t >= ntiles) return;
    const uint64_t o = t * kTile;
    const uint64_t p0 = o / (2 * w) * (2 * w);
    const uint64_t na = n - p0 < w ? n - p0 : w;
    const uint64_t nb = n - p0 - na < w ? n - p0 - na : w;
    splits[t] = path_split(src + p0, na, src + p0 + na, nb, o - p0, less);
}

// VEC (src and dst 16-B aligned): the run slices are staged with aligned
// 16-B loads and a full tile is stored with 16-B nontemporal stores (r04;
// element loads and stores before).
template <typename T, typename Less, bool VEC = false>
__global__ __launch_bounds__(kThreads) void k_pass_merge(const T* __restrict__ src, uint64_t n, uint64_t w,
                                                          const uint64_t* __restrict__ splits, Less less,
                                                          T* __restrict__ dst, uint32_t* __restrict__ err = nullptr) {
    __shared__ T s[kTile];
    const uint64_t t = blockIdx.x;
    const uint64_t d0 = t * kTile;
    const uint64_t p0 = d0 / (2 * w) * (2 * w);
    const uint64_t na = n - p0 < w ? n - p0 : w;
    const uint64_t nb = n - p0 - na < w ? n - p0 - na : w;
    const uint64_t dl0 = d0 - p0;                                   // diagonal in the pair
    const uint64_t dl1 = dl0 + kTile < na + nb ? dl0 + kTile : na + nb;
    // splits come from k_pass_partition over the same data; the clamps keep
    // every access inside the run pair even if the data changed in between
    // (a caller racing the sort: garbage order, but no stray access)
    const uint64_t s1 = dl1 == na + nb ? na : splits[t + 1];  // tile t + 1 is in the same pair
    const uint64_t s0 = splits[t];
    const uint64_t a1 = min(s1, min(na, dl1));
    const uint64_t a0 = min(s0, min(a1, dl0));
    const uint64_t b0 = min(dl0 - a0, nb), b1 = max(b0, min(dl1 - a1, nb));
    if (threadIdx.x == 0 && (a0 != s0 || a1 != s1 || b0 != dl0 - a0 || b1 != dl1 - a1))
        raise_device_error(err, HPXHIP_DEVERR_RANGE);
    const int la = static_cast<int>(a1 - a0), lb = static_cast<int>(b1 - b0);
    const int len = la + lb;
    const T* a = src + p0;
    const T* b = src + p0 + na;  // 16-B aligned whenever lb > 0 (na = w, a multiple of kTile)
    if constexpr (VEC) {
        stage<T, true>(a, a0, a1, s);
        stage<T, true>(b, b0, b1, s + la);
    } else {
        for (int i = threadIdx.x; i < la; i += kThreads) s[i] = a[a0 + i];
        for (int i = threadIdx.x; i < lb; i += kThreads) s[la + i] = b[b0 + i];
    }
    __syncthreads();
    merge_in_lds(s, la, lb, less);
    constexpr int V = vec_elems<T>();
    if (VEC && V > 1 && len == kTile) {
        using VT = vec<T, V>;
        const VT* vsrc = reinterpret_cast<const VT*>(s);
        VT* vo = reinterpret_cast<VT*>(dst + d0);
        for (int v = threadIdx.x; v < kTile / V; v += kThreads) st_stream(&vo[v], vsrc[v]);
    } else {
        for (int i = threadIdx.x; i < len; i += kThreads) dst[d0 + i] = s[i];
    }
}

}  // namespace merge_detail
}  // namespace hpxhip
