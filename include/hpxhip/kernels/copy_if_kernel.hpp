// copy_if_kernel.hpp -- the single-pass stream compaction kernel (see
// copy_if.hip for the algorithm notes).  Header so that scripts/ubench
// instantiates exactly the shipped kernel with other tile shapes.
#pragma once

#include <hpxhip/kernels/common.hpp>
#include <hpxhip/kernels/lookback.hpp>

namespace hpxhip {
namespace copy_if_detail {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;

template <typename T, int ROUNDS, int THREADS = kThreads>
constexpr uint64_t tile_elems() {
    return static_cast<uint64_t>(THREADS) * ROUNDS * (16 / sizeof(T));
}

__device__ __forceinline__ uint32_t rank_below(uint64_t mask) {
    // number of set bits of `mask` in lanes below this lane
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mask), 0u));
}

// Hit bits of one lane: bit (r*V + e) for element e of round r.
template <int BITS>
using hit_word = std::conditional_t<(BITS <= 32), uint32_t, uint64_t>;

// MINW: minimum waves per SIMD (8 = two 1024-thread workgroups per CU).
// ABL: ablation bits for scripts/ubench/copyif.hip only (wrong output):
//   1 = no look-back (tile prefix 0), 2 = hits stored straight from
//   registers at their ranks (no LDS compaction), 4 = no write-out at all.
// SV: tile-state value type (uint32_t halves the look-back granules; valid
// while n < 2^32).  WIDE: 8-byte elements stored as 16-B pairs (r04,
// 2.191-2.196 -> 2.183-2.185 ms at 2^30 int64, profiles/r04_ubench_copyif8_wide.log).
// ONEHOP: the one-hop fixed look-back (lookback.hpp).
template <typename T, typename Pred, bool ALIGNED, int ROUNDS, int MINW = 4, int ABL = 0, typename SV = uint64_t,
          bool DYN_ID = HPXHIP_TILE_DYN_ID, bool NT_STORE = false, int RPB = 1, bool FIXED = false,
          int THREADS = kThreads, bool WIDE = false, bool ONEHOP = false>
__global__ __launch_bounds__(THREADS, MINW) void k_copy_if(const T* in, T* out, uint64_t n, Pred pred,
                                                       uint64_t* count_dev, uint32_t* counter,
                                                       tile_state<SV> st, uint64_t ntiles,
                                                       const uint64_t* prefix0 = nullptr) {
    constexpr int V = 16 / sizeof(T);
    constexpr int WAVES = THREADS / kWave;
    constexpr uint64_t TILE = tile_elems<T, ROUNDS, THREADS>();
    constexpr uint64_t WAVE_ELEMS = TILE / WAVES;
    using VT = vec<T, V>;
    using H = hit_word<ROUNDS * V>;
    static_assert(ROUNDS * V <= 64, "hit bits per lane");

    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_wave_total[WAVES];
    __shared__ uint64_t s_prefix;
    static_assert(ROUNDS % RPB == 0, "rounds per write-out batch");
    __shared__ T s_stage[WAVES][kWave * V * RPB];  // RPB wave rounds of hits, compacted

    if constexpr (DYN_ID) {  // ablation: tile ids from the atomic counter
        if (threadIdx.x == 0)
            s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
    const uint64_t tile = DYN_ID ? s_tile : blockIdx.x;  // tile order = dispatch order (lookback.hpp)
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();
    const uint64_t tile_base = tile * TILE;
    const uint64_t wbase = tile_base + wave * WAVE_ELEMS;
    const bool full = tile_base + TILE <= n;

    VT x[ROUNDS];
    H hit = 0;
    if (ALIGNED && full) {
        const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) x[r] = ld_stream(&src[r * kWave + lane]);
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) hit |= static_cast<H>(pred(x[r].v[e])) << (r * V + e);
    } else {
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                const bool ok = i < n;
                x[r].v[e] = ok ? in[i] : T(0);
                hit |= static_cast<H>(ok && pred(x[r].v[e])) << (r * V + e);
            }
    }

    // Hits of the wave's segment (segment order = round, lane, element): the
    // per-element ranks are recomputed in the write-out from the hit bits,
    // so no rank array is held across the look-back.
    const uint32_t wave_count = wave_reduce(static_cast<uint32_t>(__builtin_popcountll(hit)), op_plus{});
    if (lane == 0) s_wave_total[wave] = wave_count;
    __syncthreads();
    uint32_t wave_prefix = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
        if (w < wave) wave_prefix += s_wave_total[w];
        agg += s_wave_total[w];
    }

    if (wave == 0) {
        SV p = 0;
        if (tile == 0) {
            // prefix0: hits of a head the caller compacted first (misaligned input)
            if (prefix0) p = static_cast<SV>(*prefix0);
            if (lane == 0) {
                if constexpr (FIXED) {  // the fixed-association look-back (lookback.hpp)
                    st.publish(0, static_cast<SV>(agg), TILE_AGGREGATE);
                    st.publish(0, p, TILE_INCLUSIVE);
                } else {
                    st.publish(0, static_cast<SV>(p + agg), TILE_INCLUSIVE);
                }
            }
        } else if constexpr ((ABL & 1) == 0) {
            if (lane == 0) st.publish(tile, static_cast<SV>(agg), TILE_AGGREGATE);
            if constexpr (FIXED) {
                // ONEHOP (lookback.hpp): 8-byte elements 2.176-2.184 -> 2.138-2.146
                // ms at 2^30 int64; 4-byte ones spill 35 VGPRs with it (14 without)
                // and slow down, 2.27 -> 2.58 ms at 2^31 int32; the int64 scan
                // measured 2.544 -> 2.576 and keeps the two-hop form
                // (profiles/r04_ubench_lookback_onehop.log)
                p = st.template exclusive_prefix_fixed<ONEHOP>(tile, op_plus{});
            } else {
                p = st.exclusive_prefix(tile, op_plus{});
                if (lane == 0) st.publish(tile, static_cast<SV>(p + agg), TILE_INCLUSIVE);
            }
        }
        if (lane == 0) {
            s_prefix = p;
            if (tile == ntiles - 1) *count_dev = static_cast<uint64_t>(p) + agg;
        }
    }
    __syncthreads();
    // Write-out: per wave round, the hits are compacted into LDS at their
    // round-local rank and stored back by consecutive lanes, so each store
    // instruction covers one contiguous run of the output (a direct
    // out[base + rank] scatter leaves holes in every wave store).
    const uint64_t base = s_prefix + wave_prefix;
    if constexpr ((ABL & 4) != 0) return;
    if constexpr ((ABL & 2) != 0) {
        uint32_t rb = 0;
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
            uint32_t cnt = 0, below = 0;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t m = __ballot((hit >> (r * V + e)) & 1u);
                below += rank_below(m);
                cnt += static_cast<uint32_t>(__builtin_popcountll(m));
            }
            uint32_t lb = 0;
#pragma unroll
            for (int e = 0; e < V; ++e)
                if ((hit >> (r * V + e)) & 1u) out[base + rb + below + lb++] = x[r].v[e];
            rb += cnt;
        }
        return;
    }
    // RPB rounds per batch: the batch's hits are compacted into LDS
    // back to back (one LDS wait per batch instead of one per round) and
    // stored as one contiguous run.
    T* stage = s_stage[wave];
    uint32_t out_base = 0;
#pragma unroll
    for (int b = 0; b < ROUNDS / RPB; ++b) {
        uint32_t bcnt = 0;
#pragma unroll
        for (int rr = 0; rr < RPB; ++rr) {
            const int r = b * RPB + rr;
            uint32_t cnt = 0, below = 0;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t m = __ballot((hit >> (r * V + e)) & 1u);
                below += rank_below(m);
                cnt += static_cast<uint32_t>(__builtin_popcountll(m));
            }
            uint32_t lane_before = 0;
#pragma unroll
            for (int e = 0; e < V; ++e)
                if ((hit >> (r * V + e)) & 1u) stage[bcnt + below + lane_before++] = x[r].v[e];
            bcnt += cnt;
        }
        // LDS is in order within a wave; the wait + clobber keep the compiler
        // from hoisting the reads above the writes of other lanes.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (WIDE && sizeof(T) == 8) {
            // 16-B stores: one element up to the output's next 16-B boundary,
            // then element pairs, then an odd last element
            using V2 = vec<T, 2>;
            T* o = out + base + out_base;
            const uint32_t head = bcnt ? static_cast<uint32_t>((reinterpret_cast<uintptr_t>(o) >> 3) & 1u) : 0u;
            const uint32_t npairs = (bcnt - head) / 2;
            if (lane == 0 && head) st_stream(&o[0], stage[0]);
            if (lane == 0 && ((bcnt - head) & 1u)) st_stream(&o[bcnt - 1], stage[bcnt - 1]);
#pragma unroll
            for (int k = 0; k < (V * RPB + 1) / 2; ++k) {
                const uint32_t q = k * kWave + lane;
                if (q < npairs) {
                    V2 w;
                    w.v[0] = stage[head + 2 * q];
                    w.v[1] = stage[head + 2 * q + 1];
                    st_stream(reinterpret_cast<V2*>(o + head + 2 * q), w);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < V * RPB; ++k) {
                const uint32_t j = k * kWave + lane;
                if (j < bcnt) {
                    if constexpr (NT_STORE) st_stream(&out[base + out_base + j], stage[j]);
                    else out[base + out_base + j] = stage[j];
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next batch's writes
        out_base += bcnt;
    }
}

// Pipelined form (r05, aligned input): a persistent grid of one 1024-thread
// workgroup per CU walks tiles claimed in order from `counter`.  A tile's
// hits are compacted into LDS (the whole tile, 128 KiB), then the next
// tile's loads are issued into the registers the tile just left, and only
// then does the workgroup take the tile's look-back and store its hits from
// LDS -- so a CU's write-out and look-back run under its next tile's reads
// instead of between them (k_copy_if holds the tile in registers until its
// write-out, and two of them per CU fall into step).  Tiles are claimed in
// order, so every look-back waits only on tiles already claimed by running
// workgroups (forward progress without co-residency).  Same tile shape,
// look-back and output as k_copy_if<..., FIXED, ONEHOP>.
// OUT_ALIGN: the write-out starts its vectors at this output alignment
// (the elements before it are stored one by one).  128 (a cache line): each
// wave's 1-KiB store run covers whole lines, so two waves never write halves
// of one line -- 2^30 int64 WRITE_SIZE 1.02 -> 1.0015x the hits, 1.985 ->
// 1.96-1.97 ms (profiles/r05_ubench_copyif9_align128.log, r05_pmc_copy_if.txt).
template <typename T, typename Pred, int ROUNDS, typename SV, int MINW = 4, int OUT_ALIGN = 128>
__global__ __launch_bounds__(kThreads, MINW) void k_copy_if_pipe(const T* in, T* out, uint64_t n, Pred pred,
                                                                 uint64_t* count_dev, uint32_t* counter,
                                                                 tile_state<SV> st, uint64_t ntiles,
                                                                 const uint64_t* prefix0 = nullptr) {
    constexpr int V = 16 / sizeof(T);
    constexpr uint64_t TILE = tile_elems<T, ROUNDS>();
    constexpr uint64_t WAVE_ELEMS = TILE / kWaves;
    using VT = vec<T, V>;
    using H = hit_word<ROUNDS * V>;
    static_assert(ROUNDS * V <= 64, "hit bits per lane");

    __shared__ T s_stage[TILE];
    __shared__ uint32_t s_wave_total[kWaves];
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_prefix;

    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();
    auto claim = [&] {
        if (threadIdx.x == 0)
            s_next = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    VT x[ROUNDS];
    auto load = [&](uint64_t t) {
        const uint64_t wbase = t * TILE + wave * WAVE_ELEMS;
        if (wbase + WAVE_ELEMS <= n) {
            const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) x[r] = ld_stream(&src[r * kWave + lane]);
        } else {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                    x[r].v[e] = i < n ? in[i] : T(0);
                }
        }
    };

    claim();
    __syncthreads();
    uint64_t tile = s_next;
    if (tile >= ntiles) return;
    load(tile);
    while (true) {
        const uint64_t wbase = tile * TILE + wave * WAVE_ELEMS;
        H hit = 0;
        if (wbase + WAVE_ELEMS <= n) {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) hit |= static_cast<H>(pred(x[r].v[e])) << (r * V + e);
        } else {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                    hit |= static_cast<H>(i < n && pred(x[r].v[e])) << (r * V + e);
                }
        }
        const uint32_t wave_count = wave_reduce(static_cast<uint32_t>(__builtin_popcountll(hit)), op_plus{});
        if (lane == 0) s_wave_total[wave] = wave_count;
        claim();
        __syncthreads();  // (A) wave totals, the next tile id
        uint32_t wave_prefix = 0, agg = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            if (w < wave) wave_prefix += s_wave_total[w];
            agg += s_wave_total[w];
        }
        if (tile > 0 && threadIdx.x == 0) st.publish(tile, static_cast<SV>(agg), TILE_AGGREGATE);
        // compaction: the wave's hits in segment order (round, lane, element)
        uint32_t rb = wave_prefix;
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
            uint32_t cnt = 0, below = 0;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t m = __ballot((hit >> (r * V + e)) & 1u);
                below += rank_below(m);
                cnt += static_cast<uint32_t>(__builtin_popcountll(m));
            }
            uint32_t lb = 0;
#pragma unroll
            for (int e = 0; e < V; ++e)
                if ((hit >> (r * V + e)) & 1u) s_stage[rb + below + lb++] = x[r].v[e];
            rb += cnt;
        }
        const uint64_t next = s_next;
        __syncthreads();  // (B) the tile's hits are in LDS; x is free
        if (next < ntiles) load(next);
        if (wave == 0) {
            SV p = 0;
            if (tile == 0) {
                if (prefix0) p = static_cast<SV>(*prefix0);
                if (lane == 0) {
                    st.publish(0, static_cast<SV>(agg), TILE_AGGREGATE);
                    st.publish(0, p, TILE_INCLUSIVE);
                }
            } else {
                p = st.template exclusive_prefix_fixed<true>(tile, op_plus{});
            }
            if (lane == 0) {
                s_prefix = p;
                if (tile == ntiles - 1) *count_dev = static_cast<uint64_t>(p) + agg;
            }
        }
        __syncthreads();  // (C) the tile's output offset
        // write-out: a head up to the output's next OUT_ALIGN boundary,
        // whole 16-B vectors, a tail
        T* o = out + s_prefix;
        constexpr uintptr_t AM = OUT_ALIGN - 1;
        const uint32_t head =
            agg ? min(agg, static_cast<uint32_t>(((OUT_ALIGN - (reinterpret_cast<uintptr_t>(o) & AM)) & AM) / sizeof(T)))
                : 0u;
        const uint32_t nvec = (agg - head) / V;
        const uint32_t tail = agg - head - nvec * V;
        if (threadIdx.x < head) o[threadIdx.x] = s_stage[threadIdx.x];
        else if (threadIdx.x >= 64 && threadIdx.x - 64 < tail) {
            const uint32_t j = head + nvec * V + (threadIdx.x - 64);
            o[j] = s_stage[j];
        }
#pragma unroll
        for (int k = 0; k < static_cast<int>(TILE / V / kThreads); ++k) {
            const uint32_t q = k * kThreads + threadIdx.x;
            if (q < nvec) {
                VT w;
#pragma unroll
                for (int e = 0; e < V; ++e) w.v[e] = s_stage[head + q * V + e];
                st_stream(reinterpret_cast<VT*>(o + head) + q, w);
            }
        }
        if (next >= ntiles) break;
        tile = next;
    }
}

// Head of a misaligned input (fewer than 16 B of elements): compacted by one
// thread into out[0..c), c -> *count; the aligned kernel continues from c.
template <typename T, typename Pred>
__global__ void k_copy_if_head(const T* in, T* out, uint64_t h, Pred pred, uint64_t* count) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t c = 0;
    for (uint64_t i = 0; i < h; ++i)
        if (pred(in[i])) out[c++] = in[i];
    *count = c;
}

__global__ void k_zero_count(uint64_t* c) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *c = 0;
}

}  // namespace copy_if_detail
}  // namespace hpxhip
