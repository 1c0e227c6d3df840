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
// Structure (8-bit digits, 4 passes for 32-bit keys, 8 for 64-bit keys):
//   k_hist        one read of the keys -> all passes' 256-bin histograms
//                 (per-block LDS histograms, one global atomic per bin);
//   k_bin_offsets exclusive scan of each pass's histogram;
//   k_onesweep    per pass, per 4096-key tile: wave-level match ranking
//                 (8 ballots per key, no LDS atomics), per-wave LDS digit
//                 counters, tile-local counting sort into LDS, per-bin
//                 decoupled look-back across tiles (one thread per bin,
//                 32-bit {flag,count} granules written by one sc1 store), and
//                 a coalesced write of the LDS-sorted tile.
// A pass whose digit is constant over all keys is skipped (the histogram is
// read back once per sort).  Traffic model: 8 B/key histogram + 16 B/key per
// executed pass (+ values).
#include "internal.hpp"

#include <vector>

using namespace hpxhip;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;  // 4096 keys
constexpr int kRadix = 256;
constexpr int kHistBlocksPerCU = 2;

// Storage-bits -> ordered unsigned bits (ascending), optionally inverted.
template <typename T, bool DESC>
struct ordered_bits {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    __device__ __forceinline__ U operator()(U raw) const {
        constexpr U sign = U(1) << (sizeof(U) * 8 - 1);
        U u;
        if constexpr (std::is_floating_point_v<T>) u = (raw & sign) ? ~raw : (raw | sign);
        else if constexpr (std::is_signed_v<T>) u = raw ^ sign;
        else u = raw;
        return DESC ? ~u : u;
    }
};

// Look-back granule: 0 = not yet published; ((c+1) << 1) = tile aggregate c;
// (v << 1) | 1 = inclusive prefix v.
template <typename G>
__device__ __forceinline__ G enc_agg(uint64_t c) { return static_cast<G>((c + 1) << 1); }
template <typename G>
__device__ __forceinline__ G enc_incl(uint64_t v) { return static_cast<G>((v << 1) | 1u); }

// ---------------------------------------------------------------- histogram
template <typename U, typename X>
__global__ __launch_bounds__(kThreads) void k_hist(const U* __restrict__ keys, uint64_t n, int passes, X xf,
                                                    unsigned long long* __restrict__ hist) {
    __shared__ uint32_t h[sizeof(U)][kRadix];
    for (int i = threadIdx.x; i < static_cast<int>(sizeof(U)) * kRadix; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    constexpr int V = 16 / sizeof(U);
    using VT = vec<U, V>;
    const uint64_t nvec = n / V;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kThreads;
    const VT* vk = reinterpret_cast<const VT*>(keys);
    for (uint64_t i = tid; i < nvec; i += stride * 4) {
        VT x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < nvec) x[u] = vk[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < nvec) {
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const U b = xf(x[u].v[e]);
#pragma unroll
                    for (int p = 0; p < static_cast<int>(sizeof(U)); ++p)
                        if (p < passes) atomicAdd(&h[p][(b >> (8 * p)) & 0xff], 1u);
                }
            }
    }
    if (tid < n - nvec * V) {
        const U b = xf(keys[nvec * V + tid]);
        for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(b >> (8 * p)) & 0xff], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < passes * kRadix; i += kThreads) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&hist[i], static_cast<unsigned long long>(c));
    }
}

// Exclusive scan of each pass's 256 counts (one block per pass).
__global__ __launch_bounds__(kThreads) void k_bin_offsets(const unsigned long long* __restrict__ hist,
                                                           unsigned long long* __restrict__ start) {
    __shared__ uint64_t s_w[kWaves];
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
template <typename U, typename VAL, bool HAS_VAL, typename G, typename X>
__global__ __launch_bounds__(kThreads) void k_onesweep(const U* __restrict__ kin, U* __restrict__ kout,
                                                        const VAL* __restrict__ vin, VAL* __restrict__ vout,
                                                        uint64_t n, int shift,
                                                        const unsigned long long* __restrict__ bin_start,
                                                        G* __restrict__ lb, uint32_t* __restrict__ counter,
                                                        uint32_t* __restrict__ err, X xf) {
    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_whist[kWaves][kRadix];
    __shared__ uint32_t s_local[kRadix];
    __shared__ uint32_t s_wsum[kWaves];
    __shared__ uint64_t s_adj[kRadix];
    __shared__ U s_keys[kTile];
    __shared__ VAL s_vals[HAS_VAL ? kTile : 1];

    const int t = threadIdx.x;
    const int wave = t / kWave;
    const int lane = lane_id();
    if (t == 0) s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s_whist[w][t] = 0;
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t tile_base = tile * kTile;
    const uint64_t wbase = tile_base + wave * (kTile / kWaves);

    // ---- load: round r, lane l -> tile position wave*1024 + r*64 + l
    U k[kItems];
    VAL v[HAS_VAL ? kItems : 1];
    const bool full = tile_base + kTile <= n;
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < n) {
            k[r] = kin[i];
            if constexpr (HAS_VAL) v[r] = vin[i];
        } else {
            k[r] = 0;
        }
    }

    // ---- wave-level match ranking
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
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
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    __syncthreads();

    // ---- per-bin tile count, wave offsets (thread t == bin t)
    uint32_t tile_count = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t c = s_whist[w][t];
        s_whist[w][t] = tile_count;
        tile_count += c;
    }
    // publish this tile's aggregate for bin t as early as possible
    G* my = lb + tile * kRadix;
    if (tile != 0) __hip_atomic_store(&my[t], enc_agg<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ---- tile-local exclusive offsets over bins
    {
        const uint32_t incl = wave_inclusive_scan(tile_count, op_plus{});
        if (lane == kWave - 1) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w)
            if (w < wave) pre += s_wsum[w];
        s_local[t] = pre + incl - tile_count;
    }
    __syncthreads();

    // ---- counting sort of the tile into LDS
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < n) {
            const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
            const uint32_t pos = s_local[d] + s_whist[wave][d] + rank[r];
            s_keys[pos] = k[r];
            if constexpr (HAS_VAL) s_vals[pos] = v[r];
        }
    }

    // ---- per-bin look-back across tiles
    {
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(&my[t], enc_incl<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int64_t pred = static_cast<int64_t>(tile) - 1;
            uint32_t spins = 0;
            while (pred >= 0) {
                const G g = __hip_atomic_load(&lb[static_cast<uint64_t>(pred) * kRadix + t], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                if (g == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) {
                        if (err)
                            __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    continue;
                }
                if (g & 1u) {
                    excl += static_cast<uint64_t>(g >> 1);
                    break;
                }
                excl += static_cast<uint64_t>(g >> 1) - 1;
                --pred;
            }
            __hip_atomic_store(&my[t], enc_incl<G>(excl + tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_adj[t] = static_cast<uint64_t>(bin_start[t]) + excl - s_local[t];
    }
    __syncthreads();

    // ---- coalesced write of the LDS-sorted tile
    const uint32_t nvalid = full ? kTile : static_cast<uint32_t>(n - tile_base);
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint32_t i = r * kThreads + t;
        if (i < nvalid) {
            const U key = s_keys[i];
            const uint32_t d = static_cast<uint32_t>(xf(key) >> shift) & 0xffu;
            const uint64_t dst = s_adj[d] + i;
            kout[dst] = key;
            if constexpr (HAS_VAL) vout[dst] = s_vals[i];
        }
    }
}

struct sort_layout {
    uint64_t ntiles;
    size_t alt_keys, alt_vals, hist, start, counter, lb, lb_bytes, total;
    bool wide;  // 64-bit granules
};

sort_layout make_layout(uint64_t n, size_t ksize, size_t vsize) {
    sort_layout L;
    L.ntiles = (n + kTile - 1) / kTile;
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
    const sort_layout L = make_layout(n, sizeof(U), HAS_VAL ? sizeof(VAL) : 0);
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
    hipLaunchKernelGGL((k_hist<U, X>), dim3(hist_grid), dim3(kThreads), 0, s, static_cast<const U*>(keys), n, passes,
                       X{}, hist);
    HPXHIP_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_bin_offsets, dim3(passes), dim3(kThreads), 0, s, hist, start);
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
        const dim3 grid(static_cast<unsigned>(L.ntiles)), block(kThreads);
        if (L.wide)
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, unsigned long long, X>), grid, block, 0, s, kc, ka, vc,
                               va, n, 8 * p, start + p * kRadix,
                               reinterpret_cast<unsigned long long*>(base + L.lb), counter, err, X{});
        else
            hipLaunchKernelGGL((k_onesweep<U, VAL, HAS_VAL, uint32_t, X>), grid, block, 0, s, kc, ka, vc, va, n,
                               8 * p, start + p * kRadix, reinterpret_cast<uint32_t*>(base + L.lb), counter, err,
                               X{});
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
    return make_layout(n, dtype_size(key_dtype), value_dtype < 0 ? 0 : dtype_size(value_dtype)).total;
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
