// sort_kernel.hpp -- kernels of the LSD onesweep radix sort (see sort.hip
// for the algorithm notes).  Header so that scripts/ubench instantiates the
// shipped kernels with other tile shapes.
#pragma once

#include "common.hpp"

namespace hpxhip {
namespace sort_detail {

constexpr int kRadix = 256;

// ordered_bits (storage bits -> ordered unsigned bits): common.hpp

// Look-back granule (one aligned store, the data is the flag):
//   0 = not yet published; ((c+1) << 1) = tile aggregate c; (v << 1) | 1 = inclusive v.
template <typename G>
__device__ __forceinline__ G enc_agg(uint64_t c) { return static_cast<G>((c + 1) << 1); }
template <typename G>
__device__ __forceinline__ G enc_incl(uint64_t v) { return static_cast<G>((v << 1) | 1u); }

// ---------------------------------------------------------------- histogram
// One read of the keys -> all passes' 256-bin histograms.  Each bin has
// COPIES lane-private LDS counters (lane % COPIES), interleaved so that bin
// b, copy c sits at word b*COPIES + c: lanes of one wave-instruction that hit
// different bins then collide on a bank only when their bins agree mod
// 32/COPIES, instead of mod 32 (the single-copy histogram spent 72 % of its
// LDS cycles in bank conflicts, profiles/r01_pmc_sort.txt).  Keys are read
// with nontemporal 16-B loads.
template <typename U, typename X, int THREADS = 256, int COPIES = 4>
__global__ __launch_bounds__(THREADS) void k_hist(const U* __restrict__ keys, uint64_t n, int passes, X xf,
                                                   unsigned long long* __restrict__ hist) {
    constexpr int P = static_cast<int>(sizeof(U));
    __shared__ uint32_t h[P * kRadix * COPIES];
    for (int i = threadIdx.x; i < P * kRadix * COPIES; i += THREADS) h[i] = 0;
    __syncthreads();
    constexpr int V = 16 / sizeof(U);
    using VT = vec<U, V>;
    const uint32_t copy = threadIdx.x % COPIES;
    const uint64_t nvec = n / V;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * THREADS + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * THREADS;
    const VT* vk = reinterpret_cast<const VT*>(keys);
    auto count = [&](U b) {
#pragma unroll
        for (int p = 0; p < P; ++p)
            if (p < passes) atomicAdd(&h[(p * kRadix + ((b >> (8 * p)) & 0xff)) * COPIES + copy], 1u);
    };
    for (uint64_t i = tid; i < nvec; i += stride * 4) {
        VT x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < nvec) x[u] = ld_stream(&vk[i + u * stride]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < nvec) {
#pragma unroll
                for (int e = 0; e < V; ++e) count(xf(x[u].v[e]));
            }
    }
    if (tid < n - nvec * V) count(xf(keys[nvec * V + tid]));
    __syncthreads();
    for (int i = threadIdx.x; i < passes * kRadix; i += THREADS) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < COPIES; ++k) c += h[i * COPIES + k];
        if (c) atomicAdd(&hist[i], static_cast<unsigned long long>(c));
    }
}

// Exclusive scan of each pass's 256 counts (one 256-thread block per pass).
__global__ __launch_bounds__(256) void k_bin_offsets(const unsigned long long* __restrict__ hist,
                                                      unsigned long long* __restrict__ start) {
    __shared__ uint64_t s_w[4];
    const int p = blockIdx.x;
    const int d = threadIdx.x;
    const uint64_t c = hist[p * kRadix + d];
    const uint64_t incl = wave_inclusive_scan(c, op_plus{});
    const int wave = d / kWave;
    if (lane_id() == kWave - 1) s_w[wave] = incl;
    __syncthreads();
    uint64_t pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_w[w];
    start[p * kRadix + d] = pre + incl - c;
}

// ----------------------------------------------------------------- onesweep
// One 8-bit LSD pass over TILE = THREADS*ITEMS keys per workgroup; the whole
// tile is counting-sorted in LDS and written out coalesced.
//   LBB: granules each digit's thread loads per look-back step (the walk back
//        to the nearest inclusive prefix covers LBB tiles per round trip);
//        0 = no look-back (ablation only: wrong output).
// Measured variants (scripts/ubench/sortpass.hip, profiles/r01_ubench_sort*):
// 512 x 16 keys with LBB = 4 was the fastest pass (4.88 ms at 2^30 u64);
// staging the tile in two LDS phases, a cooperative look-back over all
// threads (64-128 tiles per round trip) and 32 keys per thread were slower.
template <typename U, typename VAL, bool HAS_VAL, typename G, typename X, int THREADS = 512, int ITEMS = 16,
          int LBB = 8>
__global__ __launch_bounds__(THREADS) void k_onesweep(const U* __restrict__ kin, U* __restrict__ kout,
                                                       const VAL* __restrict__ vin, VAL* __restrict__ vout,
                                                       uint64_t n, int shift,
                                                       const unsigned long long* __restrict__ bin_start,
                                                       G* __restrict__ lb, uint32_t* __restrict__ counter,
                                                       uint32_t* __restrict__ err, X xf) {
    static_assert(THREADS >= kRadix && THREADS % kRadix == 0, "one thread per digit for the look-back");
    constexpr int WAVES = THREADS / kWave;
    constexpr int TILE = THREADS * ITEMS;
    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_whist[WAVES][kRadix];
    __shared__ uint32_t s_local[kRadix];
    __shared__ uint32_t s_wsum[kRadix / kWave];
    __shared__ uint64_t s_adj[kRadix];
    __shared__ U s_keys[TILE];
    __shared__ VAL s_vals[HAS_VAL ? TILE : 1];

    const int t = threadIdx.x;
    const int wave = t / kWave;
    const int lane = lane_id();
    if (t == 0) s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = t; i < WAVES * kRadix; i += THREADS) (&s_whist[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t tile_base = tile * TILE;
    const uint64_t wbase = tile_base + static_cast<uint64_t>(wave) * (TILE / WAVES);

    // ---- load: round r, lane l -> tile position wave*(TILE/WAVES) + r*64 + l
    U k[ITEMS];
    VAL v[HAS_VAL ? ITEMS : 1];
    const bool full = tile_base + TILE <= n;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < n) {
            k[r] = kin[i];
            if constexpr (HAS_VAL) v[r] = vin[i];
        } else {
            k[r] = 0;
        }
    }

    // ---- wave-level match ranking (stable: round-major, then lane order)
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        const bool valid = full || i < n;
        const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t below = static_cast<uint32_t>(__builtin_popcountll(peers & lt_mask));
        const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(peers));
        const uint32_t old = s_whist[wave][d];
        rank[r] = old + below;
        if (valid && below == 0) s_whist[wave][d] = old + cnt;
    }
    __syncthreads();

    // ---- per-digit tile count and per-wave offsets (thread t < 256 owns digit t)
    uint32_t tile_count = 0;
    uint32_t count_incl = 0;
    G* my = lb + tile * kRadix;
    if (t < kRadix) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const uint32_t c = s_whist[w][t];
            s_whist[w][t] = tile_count;
            tile_count += c;
        }
        // publish this tile's aggregate for digit t as early as possible
        if (tile != 0 && LBB > 0)
            __hip_atomic_store(&my[t], enc_agg<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        count_incl = wave_inclusive_scan(tile_count, op_plus{});
        if (lane == kWave - 1) s_wsum[wave] = count_incl;
    }
    __syncthreads();
    if (t < kRadix) {
        uint32_t pre = 0;
#pragma unroll
        for (int w = 0; w < kRadix / kWave; ++w)
            if (w < wave) pre += s_wsum[w];
        s_local[t] = pre + count_incl - tile_count;
    }
    __syncthreads();

    // ---- counting sort of the tile into LDS
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < n) {
            const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
            const uint32_t pos = s_local[d] + s_whist[wave][d] + rank[r];
            s_keys[pos] = k[r];
            if constexpr (HAS_VAL) s_vals[pos] = v[r];
        }
    }

    // ---- per-digit look-back across tiles (thread t < 256 owns digit t)
    if (t < kRadix) {
        uint64_t excl = 0;
        if (tile == 0) {
            if (LBB > 0) __hip_atomic_store(&my[t], enc_incl<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if constexpr (LBB > 0) {
            int64_t pred = static_cast<int64_t>(tile) - 1;
            uint32_t spins = 0;
            bool done = false;
            while (!done) {
                G g[LBB];
#pragma unroll
                for (int j = 0; j < LBB; ++j)
                    g[j] = (pred - j >= 0) ? __hip_atomic_load(&lb[static_cast<uint64_t>(pred - j) * kRadix + t],
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : enc_incl<G>(0);
                int used = 0;
#pragma unroll
                for (int j = 0; j < LBB; ++j) {
                    if (done || used != j) continue;  // stop at the first unpublished granule
                    if (g[j] == 0) continue;
                    if (g[j] & 1u) {
                        excl += static_cast<uint64_t>(g[j] >> 1);
                        done = true;
                    } else {
                        excl += static_cast<uint64_t>(g[j] >> 1) - 1;
                    }
                    ++used;
                }
                pred -= used;
                if (!done && used < LBB) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) {
                        if (err)
                            __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __hip_atomic_store(&my[t], enc_incl<G>(excl + tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_adj[t] = static_cast<uint64_t>(bin_start[t]) + excl - s_local[t];
    }
    __syncthreads();

    // ---- coalesced write of the LDS-sorted tile
    const uint32_t nvalid = full ? TILE : static_cast<uint32_t>(n - tile_base);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint32_t i = r * THREADS + t;
        if (i < nvalid) {
            const U key = s_keys[i];
            const uint32_t d = static_cast<uint32_t>(xf(key) >> shift) & 0xffu;
            const uint64_t dst = s_adj[d] + i;
            kout[dst] = key;
            if constexpr (HAS_VAL) vout[dst] = s_vals[i];
        }
    }
}

}  // namespace sort_detail
}  // namespace hpxhip
