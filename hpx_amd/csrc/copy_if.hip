// copy_if.hip -- stable stream compaction (hpx::parallel::copy_if).
//
// Reference: copy.hpp:401-494 -- phase 1 writes a bool flag per element
// (boost::shared_array<bool>, copy.hpp:416) and counts hits per chunk,
// phase 2 prefixes the counts, phase 3 re-reads input + flags and scatters.
// Here: one pass.  Each wave evaluates the predicate on 64 lanes x 16 B,
// ranks hits with `ballot` + `mbcnt` (no flag array in HBM), the tile's hit
// count goes through the same decoupled look-back as the scan
// (lookback.hpp), and hits are written to out[prefix + rank]: each wave
// round's hits are compacted through LDS and stored by consecutive lanes.
// Input loads are nontemporal.  Traffic: 8 B read + 8 B x selectivity
// written per int64 element.
#include "internal.hpp"
#include "lookback.hpp"

using namespace hpxhip;

namespace {

// 1024 threads x 8 vectors = 128 KiB tiles: the tile-id counter (one agent
// atomic per tile, ~88 per microsecond chip-wide) must not bound the pass,
// see scan_kernel.hpp.
constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;
constexpr int kRounds = 8;

template <typename T>
constexpr uint64_t tile_elems() {
    return static_cast<uint64_t>(kThreads) * kRounds * (16 / sizeof(T));
}

__device__ __forceinline__ uint32_t rank_below(uint64_t mask) {
    // number of set bits of `mask` in lanes below this lane
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
}

template <typename T, typename Pred, bool ALIGNED>
__global__ __launch_bounds__(kThreads) void k_copy_if(const T* in, T* out, uint64_t n, Pred pred,
                                                       uint64_t* count_dev, uint32_t* counter,
                                                       tile_state<uint64_t> st, uint64_t ntiles) {
    constexpr int V = 16 / sizeof(T);
    constexpr uint64_t TILE = tile_elems<T>();
    constexpr uint64_t WAVE_ELEMS = TILE / kWaves;
    using VT = vec<T, V>;

    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_wave_total[kWaves];
    __shared__ uint64_t s_prefix;
    __shared__ T s_stage[kWaves][kWave * V];  // one wave round of hits, compacted

    if (threadIdx.x == 0)
        s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint64_t tile = s_tile;
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();
    const uint64_t tile_base = tile * TILE;
    const uint64_t wbase = tile_base + wave * WAVE_ELEMS;
    const bool full = tile_base + TILE <= n;

    VT x[kRounds];
    uint32_t hit = 0;  // bit (r*V + e)
    if (ALIGNED && full) {
        const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
        for (int r = 0; r < kRounds; ++r) x[r] = ld_stream(&src[r * kWave + lane]);
#pragma unroll
        for (int r = 0; r < kRounds; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) hit |= static_cast<uint32_t>(pred(x[r].v[e])) << (r * V + e);
    } else {
#pragma unroll
        for (int r = 0; r < kRounds; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                const bool ok = i < n;
                x[r].v[e] = ok ? in[i] : T(0);
                hit |= static_cast<uint32_t>(ok && pred(x[r].v[e])) << (r * V + e);
            }
    }

    // Per-element rank within the wave's segment (segment order = round,
    // lane, element).
    uint32_t rank[kRounds][V];
    uint32_t wave_count = 0;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        uint32_t lane_before = 0;  // hits of this lane's earlier elements
        uint32_t round_total = 0;
        uint32_t below = 0;        // hits in lower lanes (all elements)
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const uint64_t m = __ballot((hit >> (r * V + e)) & 1u);
            below += rank_below(m);
            round_total += __builtin_popcountll(m);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            rank[r][e] = wave_count + below + lane_before;
            lane_before += (hit >> (r * V + e)) & 1u;
        }
        wave_count += round_total;
    }
    if (lane == 0) s_wave_total[wave] = wave_count;
    __syncthreads();
    uint32_t wave_prefix = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        if (w < wave) wave_prefix += s_wave_total[w];
        agg += s_wave_total[w];
    }

    if (wave == 0) {
        uint64_t p = 0;
        if (tile == 0) {
            if (lane == 0) st.publish(0, static_cast<uint64_t>(agg), TILE_INCLUSIVE);
        } else {
            if (lane == 0) st.publish(tile, static_cast<uint64_t>(agg), TILE_AGGREGATE);
            p = st.exclusive_prefix(tile, op_plus{});
            if (lane == 0) st.publish(tile, p + agg, TILE_INCLUSIVE);
        }
        if (lane == 0) {
            s_prefix = p;
            if (tile == ntiles - 1) *count_dev = p + agg;
        }
    }
    __syncthreads();
    // Write-out: per wave round, the hits are compacted into LDS at their
    // round-local rank and stored back by consecutive lanes, so each store
    // instruction covers one contiguous run of the output (a direct
    // out[base + rank] scatter leaves holes in every wave store).
    const uint64_t base = s_prefix + wave_prefix;
    T* stage = s_stage[wave];
    uint32_t round_base = 0;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        uint32_t cnt = 0;
#pragma unroll
        for (int e = 0; e < V; ++e) cnt += __builtin_popcountll(__ballot((hit >> (r * V + e)) & 1u));
#pragma unroll
        for (int e = 0; e < V; ++e)
            if ((hit >> (r * V + e)) & 1u) stage[rank[r][e] - round_base] = x[r].v[e];
        // LDS is in order within a wave; the wait + clobber keep the compiler
        // from hoisting the reads above the writes of other lanes.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const uint32_t j = k * kWave + lane;
            if (j < cnt) out[base + round_base + j] = stage[j];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next round's writes
        round_base += cnt;
    }
}

__global__ void k_zero_count(uint64_t* c) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *c = 0;
}

struct cif_layout {
    uint64_t ntiles;
    size_t slots_off, total;  // [counter | tile slots], all zeroed per call
};

cif_layout make_layout(uint64_t n, uint64_t tile) {
    cif_layout L;
    L.ntiles = (n + tile - 1) / tile;
    L.slots_off = 256;
    L.total = align_up(L.slots_off + L.ntiles * tile_state<uint64_t>::bytes_per_tile(), 256);
    return L;
}

}  // namespace

namespace hpxhip {
size_t copy_if_scratch_bytes(int dtype, uint64_t n) {
    return make_layout(n, dtype_size(dtype) == 8 ? tile_elems<uint64_t>() : tile_elems<uint32_t>()).total;
}
}  // namespace hpxhip

extern "C" int hpxhip_copy_if(int dtype, int pred_kind, const void* pred_arg, const void* in, void* out, uint64_t n,
                              uint64_t* count_dev, hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    if (!count_dev || (n && (!in || !out))) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    if (n == 0) {
        hipLaunchKernelGGL(k_zero_count, dim3(1), dim3(64), 0, s, count_dev);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    }
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return with_pred<T>(pred_kind, pred_arg, [&](auto p) -> int {
            using P = decltype(p);
            const cif_layout L = make_layout(n, tile_elems<T>());
            void* ws = nullptr;
            int rc = resolve_scratch(s, scratch, scratch_bytes, L.total, &ws);
            if (rc) return rc;
            char* base = static_cast<char*>(ws);
            HPXHIP_CHECK(hipMemsetAsync(base, 0, L.total, s));
            tile_state<uint64_t> st{reinterpret_cast<uint64_t*>(base + L.slots_off), device_error_word(s)};
            uint32_t* counter = reinterpret_cast<uint32_t*>(base);
            const bool aligned = reinterpret_cast<uintptr_t>(in) % 16 == 0;
            const dim3 grid(static_cast<unsigned>(L.ntiles)), block(kThreads);
            if (aligned)
                hipLaunchKernelGGL((k_copy_if<T, P, true>), grid, block, 0, s, static_cast<const T*>(in),
                                   static_cast<T*>(out), n, p, count_dev, counter, st, L.ntiles);
            else
                hipLaunchKernelGGL((k_copy_if<T, P, false>), grid, block, 0, s, static_cast<const T*>(in),
                                   static_cast<T*>(out), n, p, count_dev, counter, st, L.ntiles);
            HPXHIP_CHECK_LAUNCH();
            return 0;
        });
    });
}
