// scan_kernel.hpp -- the single-pass scan kernel (see scan.hip for the
// algorithm notes).  Header so that the microbenchmarks under scripts/ubench
// instantiate exactly the shipped kernel with other tile shapes.
#pragma once

#include <hpxhip/kernels/common.hpp>
#include <hpxhip/kernels/lookback.hpp>

namespace hpxhip {
namespace scan_detail {

// Shipped tile shape: 1024 threads x 16 vectors of 16 B = 256 KiB per tile,
// one workgroup per CU (122 VGPRs).  Tile id = blockIdx.x (lookback.hpp; the
// round-1 atomic counter is the DYN_ID ablation: its dequeue round trip in
// front of every tile cost 0.11-0.13 ms at 2^30 int64).  The counter also
// saturates at ~88 increments per microsecond (MI355X guide, row `dequeue`):
// at 32 KiB tiles it, not HBM, bounded the scan (measured 3.3 ms for 2^30
// int64 even with the look-back removed).  Fewer,
// larger tiles also mean fewer look-back hand-offs.  Output stores are `nt`
// (NT_STORE): in blockIdx order 2.70-2.71 vs 2.78 ms for 2^30 int64 and
// 2.82-2.85 vs 2.96 for f64 with plain stores; under the atomic counter `nt`
// stores were slower, which is why round 1 rejected them
// (profiles/r02_ubench_scan_nt_store.log).  At 2^30 int64 the same
// kernel takes 2.99 ms with 128 KiB tiles (two workgroups per CU), 2.85 ms
// with 192 KiB and 2.82 ms with 256 KiB (scripts/ubench/scan.hip,
// profiles/r01_ubench_scan_structure.log).  A variant with a dedicated
// look-back wave (15 loading waves + 1) was slower at every tile size.
constexpr int kThreads = 1024;
constexpr int kRounds = 16;

// Tiles per group of the fixed-association look-back (lookback.hpp).  A
// tile folds up to GROUP - 1 published aggregates, and the groups' first
// tiles form a chain of hand-offs: r04 at 2^30 int64 / f64 (16384-element
// tiles, profiles/r04_ab_lookback_group.log): 64 tiles 2.62 ms, 32 tiles
// 2.55, 16 tiles 3.2 (the chain binds).
#ifndef HPXHIP_SCAN_LB_GROUP
#define HPXHIP_SCAN_LB_GROUP 32
#endif
constexpr int kScanGroup = HPXHIP_SCAN_LB_GROUP;
template <typename X>
using scan_state = tile_state<X, kScanGroup>;

// Rounds per launch variant: 16 for aligned integer and double scans (r03:
// double had spilled at 16 and ran 12 rounds -- 2.83 ms for 2^30 f64 --
// until the deferred round carry (DEFER below) cut its temporaries: 121
// VGPRs at 16 rounds, 2.68-2.69 ms, profiles/r03_ubench_scan7.log); float
// (four values and their lane-local scan per vector) still spills at 16 and
// keeps 12; the element-wise unaligned path uses 8.
constexpr int kRoundsF32 = 12;
template <typename T, bool ALIGNED>
constexpr int rounds_for() {
    if constexpr (!ALIGNED) return 8;
    else if constexpr (std::is_integral_v<T> || sizeof(T) == 8) return kRounds;
    else return kRoundsF32;
}

template <typename T, int ROUNDS = kRounds, int THREADS = kThreads>
constexpr uint64_t tile_elems() {
    return static_cast<uint64_t>(THREADS) * ROUNDS * (16 / sizeof(T));
}

// Wave 0 of a tile: scans the WAVES wave totals in s_wave_total with DPP,
// publishes the tile (aggregate, look-back, inclusive) and leaves in
// s_wave_total[w] the tile prefix (op) the exclusive prefix of wave w.
// FIXED: the fixed-association look-back (lookback.hpp) -- tile 0 publishes
// its aggregate and the initial prefix E(0).  Shipped for every scan (r03):
// floating-point results become reproducible run to run, and it is also the
// faster hand-off (2^30 f64 2.64 -> 2.61 ms, int64 2.64-2.65 -> 2.62-2.63;
// profiles/r03_ubench_scan7_fixed.log): every tile reads 64 aggregates
// published right after their loads plus one group word, instead of walking
// a variable window and publishing an inclusive value of its own.
template <typename T, typename Op, int WAVES, bool LOOKBACK, int LBK = 1, bool FIXED = false, typename ST>
__device__ __forceinline__ void tile_prefix(uint64_t tile, const ST& st, Op op, const T* prefix_dev, T init,
                                            T* s_wave_total) {
    constexpr bool NOID = is_noid_op<Op>::value;
    const int lane = lane_id();
    if constexpr (NOID) {
        // lanes >= WAVES pad with any value: they only feed lanes >= WAVES
        static_assert(FIXED && LOOKBACK, "an operator without identity takes the fixed look-back");
        const T wt = s_wave_total[lane < WAVES ? lane : 0];
        const T wi = wave_inclusive_scan_noid(wt, op);
        const T agg = readlane(wi, WAVES - 1);
        const T wex = dpp<DPP_WAVE_SHR1>(wi, wi);  // lane 0: nothing before wave 0
        T p;
        if (tile == 0) {
            p = prefix_dev ? *prefix_dev : init;
            if (lane == 0) {
                st.publish(0, agg, TILE_AGGREGATE);
                st.publish(0, p, TILE_INCLUSIVE);  // E(0)
            }
        } else {
            if (lane == 0) st.publish(tile, agg, TILE_AGGREGATE);
            p = st.exclusive_prefix_fixed_noid(tile, op);
        }
        if (lane < WAVES) s_wave_total[lane] = lane == 0 ? p : op(p, wex);
        return;
    } else {
    const T id = Op::template identity<T>();
    const T wt = lane < WAVES ? s_wave_total[lane] : id;
    const T wi = wave_inclusive_scan(wt, op);
    const T agg = readlane(wi, WAVES - 1);
    const T wex = wave_shift_right<T, Op>(wi);
    T p;
    if (tile == 0) {
        p = prefix_dev ? *prefix_dev : init;
        if (lane == 0) {
            if constexpr (FIXED) {
                st.publish(0, agg, TILE_AGGREGATE);
                st.publish(0, p, TILE_INCLUSIVE);  // E(0)
            } else {
                st.publish(0, op(p, agg), TILE_INCLUSIVE);
            }
        }
    } else {
        if constexpr (LOOKBACK) {
            if (lane == 0) st.publish(tile, agg, TILE_AGGREGATE);
            if constexpr (FIXED) {
                p = st.exclusive_prefix_fixed(tile, op);
            } else {
                p = st.template exclusive_prefix<Op, LBK>(tile, op);
                if (lane == 0) st.publish(tile, op(p, agg), TILE_INCLUSIVE);
            }
        } else {
            p = id;  // ablation only: measures the pass without the tile hand-off
        }
    }
    if (lane < WAVES) s_wave_total[lane] = op(p, wex);
    }
}

// T: element type of in/out; X: the scanned value type (T for the built-in
// operators; opt<T> for a user operator without an identity, the C++
// layer's device closures): conv maps T -> X, unwrap_value X -> T.
template <typename T, typename Conv, typename Op, bool INCL, bool ALIGNED, int ROUNDS = kRounds,
          int THREADS = kThreads, bool LOOKBACK = true, int MINW = 1, bool EARLY = false, int LBK = 1,
          bool DYN_ID = HPXHIP_TILE_DYN_ID, bool NT_STORE = true, typename X = T, bool DEFER = std::is_floating_point_v<X> && sizeof(X) == 8, bool FIXED = true,
          bool SHIFTED = false>
__global__ __launch_bounds__(THREADS, MINW) void k_scan(const T* in, T* out, uint64_t n, Conv conv, Op op, X init,
                                                   const X* prefix_dev, uint32_t* counter, scan_state<X> st) {
    constexpr int V = 16 / sizeof(T);
    constexpr int WAVES = THREADS / kWave;
    constexpr uint64_t TILE = tile_elems<T, ROUNDS, THREADS>();
    constexpr uint64_t WAVE_ELEMS = TILE / WAVES;
    using VT = vec<T, V>;

    __shared__ uint32_t s_tile;
    __shared__ X s_wave_total[WAVES];

    if constexpr (DYN_ID) {
        if (threadIdx.x == 0)
            s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
    const uint64_t tile = DYN_ID ? s_tile : blockIdx.x;
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();
    // NOID (noid_op, a user operator): no identity -- out-of-range elements
    // hold X{} (they only feed outputs that are not stored), and the one
    // position with nothing before it (lane 0's first element of an
    // exclusive scan: in every round with DEFER, in round 0 without) is
    // handled by index at the store.
    constexpr bool NOID = is_noid_op<Op>::value;
    constexpr bool DEF = DEFER;
    static_assert(!(NOID && EARLY), "EARLY needs an identity");
    const X id = [] {
        if constexpr (NOID) return X{};
        else return Op::template identity<X>();
    }();

    const uint64_t tile_base = tile * TILE;
    const uint64_t wbase = tile_base + wave * WAVE_ELEMS;
    // SHIFTED reads one vector past the wave's block (below)
    const bool full = tile_base + TILE + (SHIFTED ? V : 0) <= n;

    // ---- load (all rounds in flight) and convert
    X x[ROUNDS][V];
    if constexpr (SHIFTED) {
        // (r04) The output is 16-B aligned, the input s elements past a
        // 16-B boundary (ranges whose offsets differ inside 16 B; they took
        // the element-wise kernel before).  Each lane loads the aligned
        // vector A under its output vector; the output vector is A's last
        // V - s elements and the first s of the next aligned vector, which
        // the next lane holds (DPP wave_shl:1), lane 63 takes from the next
        // round's lane 0, and the last round's lane 63 from one extra vector
        // past the wave's block.  One 16-B load per lane per round, as in the
        // aligned kernel.
        if (full) {
            const int sh = static_cast<int>((reinterpret_cast<uintptr_t>(in) % 16) / sizeof(T));
            const VT* src = reinterpret_cast<const VT*>(in + wbase - sh);
            VT raw[ROUNDS];
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) raw[r] = ld_stream(&src[r * kWave + lane]);
            const VT tail = src[ROUNDS * kWave];
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) {
                const VT y = shift_from_next_lane<T, V>(raw[r], r + 1 < ROUNDS ? readlane(raw[r + 1], 0) : tail, sh);
#pragma unroll
                for (int e = 0; e < V; ++e) x[r][e] = conv(y.v[e]);
            }
        }
    }
    if (SHIFTED && full) {
        // loaded above
    } else if (ALIGNED && full) {
        const VT* src = reinterpret_cast<const VT*>(in + wbase);
        VT raw[ROUNDS];
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) raw[r] = ld_stream(&src[r * kWave + lane]);
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) x[r][e] = conv(raw[r].v[e]);
    } else {
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                x[r][e] = i < n ? conv(in[i]) : id;
            }
    }

    // EARLY (ablation, associative integer ops only): the tile aggregate is
    // formed from per-lane folds before the per-round scans, so wave 0
    // publishes it and walks the look-back while the other waves scan their
    // rounds.  Measured slower at every tile shape (2.91-2.95 ms vs 2.82-2.84
    // for 2^30 int64, profiles/r01_ubench_scan_early_agg.log): not shipped.
    if constexpr (EARLY) {
        X lt = id;
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) lt = op(lt, x[r][e]);
        const X wt = wave_reduce(lt, op);
        if (lane == 0) s_wave_total[wave] = wt;
        __syncthreads();
        if (wave == 0) tile_prefix<X, Op, WAVES, LOOKBACK, LBK, FIXED>(tile, st, op, prefix_dev, init, s_wave_total);
    }

    // ---- per-round lane scan + wave scan; x becomes the wave-local result
    // DEFER: x[r] = (lane-exclusive prefix within round r) (op) local and the
    // round totals stay wave-uniform (readlane -> SGPRs); the carry of the
    // rounds before r is folded in only at the store.  Each round's scan then
    // finishes without the serial carry chain, so the compiler keeps 4 B of
    // temporaries per element instead of 6 (it had hoisted every round's wave
    // scan above the chain and held x, run and the shifted scan of each
    // round: f64 at 16 rounds spilled 24 VGPRs).  The regrouping keeps the
    // left-to-right order of the operands (non-commutative user ops).
    // Default for double only: int64 measured the same either way (2.68-2.70
    // ms), float at 12 rounds spills 4 VGPRs with it and none without.
    X carry = id;
    X tr[DEF ? ROUNDS : 1];
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        X local[V];
        if constexpr (NOID) {
            // lane-local scan from the first element; x[r][e] becomes the
            // wave-local value, except (lane 0, e = 0) of an exclusive scan,
            // which has none (its output is the carry alone)
            X run = x[r][0];
            local[0] = x[r][0];
#pragma unroll
            for (int e = 1; e < V; ++e) {
                const X nxt = op(run, x[r][e]);
                local[e] = INCL ? nxt : run;
                run = nxt;
            }
            const X incl = wave_inclusive_scan_noid(run, op);
            const X excl = dpp<DPP_WAVE_SHR1>(incl, incl);  // lane 0: nothing before it in the round
            const X tot = readlane(incl, kWave - 1);
            if (DEF || r == 0) {
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    if (!INCL && e == 0) x[r][e] = excl;  // lane 0: unused (index rule at the store)
                    else x[r][e] = lane == 0 ? local[e] : op(excl, local[e]);
                }
            } else {
                const X pre = lane == 0 ? carry : op(carry, excl);
#pragma unroll
                for (int e = 0; e < V; ++e) x[r][e] = (!INCL && e == 0) ? pre : op(pre, local[e]);
            }
            if constexpr (DEF) tr[r] = tot;
            else carry = r == 0 ? tot : op(carry, tot);
        } else {
            X run = id;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const X nxt = op(run, x[r][e]);
                local[e] = INCL ? nxt : run;
                run = nxt;
            }
            const X incl = wave_inclusive_scan(run, op);
            const X excl = wave_shift_right<X, Op>(incl);
            if constexpr (DEF) {
#pragma unroll
                for (int e = 0; e < V; ++e) x[r][e] = op(excl, local[e]);
                tr[r] = readlane(incl, kWave - 1);
            } else {
                const X pre = op(carry, excl);
#pragma unroll
                for (int e = 0; e < V; ++e) x[r][e] = op(pre, local[e]);
                carry = op(carry, readlane(incl, kWave - 1));
            }
        }
    }
    if constexpr (NOID && DEF) {
        carry = tr[0];
#pragma unroll
        for (int r = 1; r < ROUNDS; ++r) carry = op(carry, tr[r]);
    } else if constexpr (!NOID && DEF) {
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) carry = op(carry, tr[r]);
    }
    if constexpr (!EARLY) {
        if (lane == 0) s_wave_total[wave] = carry;
        __syncthreads();
        if (wave == 0) tile_prefix<X, Op, WAVES, LOOKBACK, LBK, FIXED>(tile, st, op, prefix_dev, init, s_wave_total);
    }
    __syncthreads();
    const X pre = s_wave_total[wave];

    // ---- store (DEFER: round r adds the carry of rounds < r here)
    X rc = pre;
    // NOID: lane 0's first element of an exclusive scan has nothing before it
    // in its round -- its output is the carry
    auto value = [&](const X& c, int r, int e) -> T {
        if constexpr (NOID && !INCL) {
            if (e == 0 && lane == 0 && (DEF || r == 0)) return unwrap_value(c);
        }
        return unwrap_value(op(c, x[r][e]));
    };
    if (ALIGNED && full) {
        VT* dst = reinterpret_cast<VT*>(out + wbase);
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
            VT y;
#pragma unroll
            for (int e = 0; e < V; ++e) y.v[e] = value(DEF ? rc : pre, r, e);
            if constexpr (DEF) rc = op(rc, tr[r]);
            if constexpr (NT_STORE) st_stream(&dst[r * kWave + lane], y);
            else dst[r * kWave + lane] = y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                if (i < n) out[i] = value(DEF ? rc : pre, r, e);
            }
            if constexpr (DEF) rc = op(rc, tr[r]);
        }
    }
}

}  // namespace scan_detail
}  // namespace hpxhip
