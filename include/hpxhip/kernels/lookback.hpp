// lookback.hpp -- single-pass decoupled look-back tile state (scan, copy_if).
//
// HPX's scan_partitioner (util/scan_partitioner.hpp:62-156) runs three
// phases: chunk totals, a left-to-right prefix of totals (dataflow), and a
// fix-up pass -- two passes over the data.  On the GPU the same prefix is
// formed in ONE pass: each tile publishes its aggregate as soon as it has
// loaded its input, then walks back over its predecessors (64 at a time, one
// per lane of the look-back wave) until it meets an inclusive prefix.
//
// Tile id = blockIdx.x (scan; onesweep passes over 32-bit keys) or an atomic
// counter (copy_if; onesweep passes over 64-bit keys), whichever measured
// faster per kernel (profiles/r02_ubench_tile_order_ab.log).
// blockIdx forward progress: the dispatcher hands out a
// kernel's workgroups in increasing id order (round robin over the XCDs,
// each XCD in order), so the lowest unfinished tile is always resident (every
// workgroup dispatched before it on its XCD has a lower id and has finished)
// and all of its predecessors are done -- it completes, and by induction so
// does the grid.  Round 1 took ids from an atomic counter instead, which
// needs no dispatch-order argument but puts one device-scope round trip
// (1-3 us while HBM is saturated) in front of every tile's first load:
// 2.83-2.84 ms vs 2.70 ms for the 2^30 int64 scan, i.e. the scan's tile
// copy floor (scripts/ubench/scan3.hip, profiles/r02_ubench_scan_tile_order.log).
// With the atomic counter a tile only waits on tiles whose workgroups are
// already running, with no dispatch-order argument.  Every wait is bounded
// (kSpinLimit), so a broken ordering assumption raises the device error word
// instead of hanging.
//
// Hand-off form: the data IS the flag (MI355X guide, Guideline 16 recipe R2).
// A value is published as 8-byte granules {status tag : 32, value word : 32},
// each written by one agent-scope relaxed (sc1) 8-byte store; a 64-bit value
// is two granules.  The reader polls the granules themselves with sc1 loads
// and accepts a slot only when every granule carries the slot's tag, so no
// store drain sits between value and flag (the earlier value-then-drain-
// then-flag form put two write-through round trips on every tile's critical
// path).  Aggregate and inclusive values live in separate slots, each written
// once per call, so a reader never mixes the halves of two different values.
// Slots are zeroed (TILE_INVALID) by the per-call memset.  Every wait is
// bounded (kSpinLimit) and raises the device error word.
#pragma once

#include <hpxhip/kernels/common.hpp>

#ifndef HPXHIP_LB_GROUP
#define HPXHIP_LB_GROUP 64
#endif
// Default of the fixed-association look-back's one-hop form (below); the
// kernels choose it per call (copy_if: one-hop, scans: two-hop).
#ifndef HPXHIP_LB_ONEHOP
#define HPXHIP_LB_ONEHOP 0
#endif

namespace hpxhip {

enum : uint32_t { TILE_INVALID = 0, TILE_AGGREGATE = 1, TILE_INCLUSIVE = 2 };

// GROUP: tiles per group of the fixed-association look-back (below).
template <typename T, int GROUP = HPXHIP_LB_GROUP>
struct tile_state {
    static constexpr int G = sizeof(T) / 4;  // granules per value (1 or 2; up to 8 for opt<T> values)
    static_assert(sizeof(T) % 4 == 0 && sizeof(T) <= 32, "tile values of whole 32-bit words");

    uint64_t* slots;  // [ntiles][2 (aggregate, inclusive)][G]
    uint32_t* err;    // device error word (may be null)

    static constexpr size_t bytes_per_tile() { return 2 * G * sizeof(uint64_t); }

    // Lane-uniform call by ONE lane.
    __device__ __forceinline__ void publish(uint64_t tile, T v, uint32_t status) const {
        uint32_t w[G];
        to_words(v, w);
        uint64_t* p = slots + (tile * 2 + (status == TILE_INCLUSIVE ? 1 : 0)) * G;
#pragma unroll
        for (int g = 0; g < G; ++g)
            __hip_atomic_store(&p[g], (static_cast<uint64_t>(status) << 32) | w[g], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }

    // Status and value of tile j's best published slot (TILE_INVALID if none).
    __device__ __forceinline__ uint32_t read(uint64_t j, T* v) const {
        const uint64_t* p = slots + j * 2 * G;
        uint64_t a[G], c[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            c[g] = __hip_atomic_load(&p[G + g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a[g] = __hip_atomic_load(&p[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool inc = true, agg = true;
        uint32_t wc[G], wa[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            inc = inc && static_cast<uint32_t>(c[g] >> 32) == TILE_INCLUSIVE;
            agg = agg && static_cast<uint32_t>(a[g] >> 32) == TILE_AGGREGATE;
            wc[g] = static_cast<uint32_t>(c[g]);
            wa[g] = static_cast<uint32_t>(a[g]);
        }
        if (inc) {
            *v = from_words<T>(wc);
            return TILE_INCLUSIVE;
        }
        if (agg) {
            *v = from_words<T>(wa);
            return TILE_AGGREGATE;
        }
        return TILE_INVALID;
    }

    // Called by ALL 64 lanes of one wave; returns the exclusive prefix of
    // `tile` (op-combination of every predecessor's elements) on every lane.
    // Requires tile > 0 and that tile 0 publishes an inclusive value.
    // Each round reads 64*K predecessors (lane l reads slots pred-l-64k, k <
    // K, all loads in flight together): with ~256 tiles in flight at once
    // (one per CU) a 64-wide window can need several round trips before it
    // meets an inclusive value, each costing a hand-off latency.
    template <typename Op, int K = 1>
    __device__ __forceinline__ T exclusive_prefix(uint64_t tile, Op op) const {
        const T id = Op::template identity<T>();
        const int lane = lane_id();
        T excl = id;
        int64_t pred = static_cast<int64_t>(tile) - 1;
        uint32_t spins = 0;
        while (true) {
            T v[K];
            uint32_t f[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int64_t j = pred - lane - k * kWave;
                v[k] = id;
                f[k] = TILE_INCLUSIVE;  // j < 0: behind tile 0, never reached
                if (j >= 0) f[k] = read(static_cast<uint64_t>(j), &v[k]);
            }
            while (true) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < K; ++k) ok = ok && f[k] != TILE_INVALID;
                if (__all(ok)) break;
                __builtin_amdgcn_s_sleep(HPXHIP_LB_SLEEP);
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (f[k] == TILE_INVALID) f[k] = read(static_cast<uint64_t>(pred - lane - k * kWave), &v[k]);
                if (++spins > kSpinLimit) {
                    if (lane == 0 && err)
                        __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    return excl;
                }
            }
            // Predecessors in order of distance: slot (k, lane) is pred - lane - 64k.
            bool found = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (found) break;  // wave-uniform
                const uint64_t inclusive_lanes = __ballot(f[k] == TILE_INCLUSIVE);
                const int first = inclusive_lanes ? __builtin_ctzll(inclusive_lanes) : kWave;
                // lane l holds tile pred - l - 64k: fold the window oldest
                // first, then put it before the nearer tiles already folded
                T w = lane > first ? id : v[k];
                const T s = wave_reduce(w, flipped_op<Op>{op});
                excl = op(s, excl);
                found = first < kWave;
            }
            if (found) break;
            pred -= K * kWave;
        }
        return excl;
    }

    // ---- fixed-association form (floating-point scans) -------------------
    // exclusive_prefix adds up whichever predecessors have published when the
    // tile looks, so a floating-point scan's association -- and its last bits
    // -- varied from run to run.  Here the association is fixed: tiles form
    // groups of 64; E(64g), the exclusive prefix of a group's first tile, is
    //   E(64g) = E(64(g-1)) (op) fold(aggregate(64(g-1)) .. aggregate(64g-1)),
    // published by tile 64g in its inclusive slot, and tile t of group g
    // takes E(64g) (op) fold(aggregate(64g) .. aggregate(t-1)).  Each fold is
    // one wave reduction over lanes in index order (identity-padded), so the
    // result is a function of the input alone: bitwise reproducible, like
    // HPX's par for a fixed core count (scan_partitioner.hpp:62-156).  The
    // waits are on lower tile ids only (dispatch-order forward progress, as
    // above) and bounded.  Tile 0 publishes its aggregate and E(0) = the
    // scan's initial prefix.
    // Group = kGroup tiles (GROUP; HPXHIP_LB_GROUP sets the default): lane l folds the
    // aggregates of tiles base + l*kGroupK .. base + l*kGroupK + kGroupK - 1
    // (in order; kGroupK = 1 up to 64 tiles), the wave reduction then folds
    // the lanes in order.  The E(first) hand-offs form a chain, one link per
    // group; a tile waits for up to kGroup - 1 aggregates.  r04 A/B at 2^30
    // (profiles/r04_ab_lookback_group.log): 256 tiles (4 per lane) 2.89 vs
    // 2.59 ms int64 scan, 2.87 vs 2.18 copy_if -- the per-tile fold, not the
    // chain, is what the group size trades.
    static constexpr uint64_t kGroup = GROUP;
    static constexpr int kGroupK = kGroup > static_cast<uint64_t>(kWave) ? static_cast<int>(kGroup / kWave) : 1;
    static_assert(kGroup % kGroupK == 0 && (kGroup <= static_cast<uint64_t>(kWave) || kGroup % kWave == 0),
                  "group: up to 64 tiles, or a multiple of 64");

    // Loads the aggregates [base + lane*K, ...) < base + cnt of this lane,
    // all in flight together, re-polling the unpublished ones; v[j] valid for
    // lane*K + j < cnt.  False on timeout.
    __device__ __forceinline__ bool wait_aggregates(uint64_t base, uint64_t cnt, T (&v)[kGroupK],
                                                    uint32_t& spins) const {
        const uint64_t l0 = static_cast<uint64_t>(lane_id()) * kGroupK;
        bool pending[kGroupK];
#pragma unroll
        for (int j = 0; j < kGroupK; ++j) pending[j] = l0 + j < cnt;
        while (true) {
            uint64_t a[kGroupK][G];
#pragma unroll
            for (int j = 0; j < kGroupK; ++j)
                if (pending[j]) {
                    const uint64_t* p = slots + (base + l0 + j) * 2 * G;
#pragma unroll
                    for (int g = 0; g < G; ++g) a[j][g] = __hip_atomic_load(&p[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            bool any = false;
#pragma unroll
            for (int j = 0; j < kGroupK; ++j)
                if (pending[j]) {
                    bool ok = true;
                    uint32_t w[G];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        ok = ok && static_cast<uint32_t>(a[j][g] >> 32) == TILE_AGGREGATE;
                        w[g] = static_cast<uint32_t>(a[j][g]);
                    }
                    if (ok) {
                        v[j] = from_words<T>(w);
                        pending[j] = false;
                    } else {
                        any = true;
                    }
                }
            if (!any) return true;
            __builtin_amdgcn_s_sleep(HPXHIP_LB_SLEEP);
            if (++spins > kSpinLimit) return false;
        }
    }

    // Lane-uniform; waits until slot (j, status) is published.
    __device__ __forceinline__ bool wait_slot(uint64_t j, uint32_t status, T* v, uint32_t& spins) const {
        const uint64_t* p = slots + (j * 2 + (status == TILE_INCLUSIVE ? 1 : 0)) * G;
        while (true) {
            uint64_t a[G];
            bool ok = true;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                a[g] = __hip_atomic_load(&p[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = ok && static_cast<uint32_t>(a[g] >> 32) == status;
            }
            if (ok) {
                uint32_t w[G];
#pragma unroll
                for (int g = 0; g < G; ++g) w[g] = static_cast<uint32_t>(a[g]);
                *v = from_words<T>(w);
                return true;
            }
            __builtin_amdgcn_s_sleep(HPXHIP_LB_SLEEP);
            if (++spins > kSpinLimit) return false;
        }
    }

    // ---- one-hop form (r04) ----------------------------------------------
    // A tile of group g >= 1 that is not the group's first takes
    //   E(g) = E(g-1) (op) fold(aggregate(64(g-1)) .. aggregate(64g-1))
    // itself, from E(g-1) (published a whole group earlier) and the previous
    // group's aggregates, instead of waiting for the group's first tile to
    // publish E(g): the only fresh waits left are on the aggregates of its
    // nearest predecessors, one hand-off instead of two.  The association --
    // and so every bit of a floating-point result -- is the two-hop form's:
    // E(g) is folded the same way by every tile of the group, and the group's
    // first tile still publishes it.  Lane l polls the previous group's
    // aggregate l, its own group's aggregate l (l < pos) and E(g-1), all in
    // flight together.
    __device__ __forceinline__ bool wait_onehop(uint64_t first, uint64_t pos, T* prev_agg, T* own_agg, T* e,
                                                uint32_t& spins) const {
        const uint64_t lane = static_cast<uint64_t>(lane_id());
        const uint64_t* p1 = slots + (first - kGroup + lane) * 2 * G;  // aggregate slot
        const uint64_t* p2 = slots + (first + lane) * 2 * G;           // aggregate slot
        const uint64_t* p3 = slots + ((first - kGroup) * 2 + 1) * G;   // inclusive slot: E(g-1)
        bool w1 = lane < kGroup, w2 = lane < pos, w3 = true;
        while (true) {
            uint64_t a1[G], a2[G], a3[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if (w1) a1[g] = __hip_atomic_load(&p1[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w2) a2[g] = __hip_atomic_load(&p2[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w3) a3[g] = __hip_atomic_load(&p3[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            auto take = [&](bool& w, const uint64_t (&a)[G], uint32_t status, T* v) {
                if (!w) return;
                bool ok = true;
                uint32_t x[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    ok = ok && static_cast<uint32_t>(a[g] >> 32) == status;
                    x[g] = static_cast<uint32_t>(a[g]);
                }
                if (ok) {
                    *v = from_words<T>(x);
                    w = false;
                }
            };
            take(w1, a1, TILE_AGGREGATE, prev_agg);
            take(w2, a2, TILE_AGGREGATE, own_agg);
            take(w3, a3, TILE_INCLUSIVE, e);
            if (!(w1 || w2 || w3)) return true;
            __builtin_amdgcn_s_sleep(HPXHIP_LB_SLEEP);
            if (++spins > kSpinLimit) return false;
        }
    }

    // Called by ALL 64 lanes of one wave, tile > 0.  Returns the exclusive
    // prefix on every lane; a group's first tile also publishes it.
    template <bool ONEHOP = HPXHIP_LB_ONEHOP, typename Op>
    __device__ __forceinline__ T exclusive_prefix_fixed(uint64_t tile, Op op) const {
        const T id = Op::template identity<T>();
        const int lane = lane_id();
        const uint64_t first = tile / kGroup * kGroup;
        if constexpr (ONEHOP && kGroupK == 1) {
            if (first > 0) {
                const uint64_t pos = tile - first;
                uint32_t spins = 0;
                T a1 = id, a2 = id, e = id;
                const bool ok = wait_onehop(first, pos, &a1, &a2, &e, spins);
                if (!__all(ok)) {
                    if (lane == 0 && err)
                        __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    return id;
                }
                const T eg = op(readlane(e, 0), wave_reduce(a1, op));  // E(g)
                if (pos == 0) {
                    if (lane == 0) publish(tile, eg, TILE_INCLUSIVE);
                    return eg;
                }
                return op(eg, wave_reduce(a2, op));
            }
        }
        // the aggregates to fold: the previous group's (a group's first
        // tile) or this group's tiles before this one
        const uint64_t base = tile == first ? first - kGroup : first;
        const uint64_t cnt = tile == first ? kGroup : tile - first;
        uint32_t spins = 0;
        T a = id;
        bool ok = true;
        if constexpr (kGroupK == 1) {
            if (static_cast<uint64_t>(lane) < cnt) ok = wait_slot(base + lane, TILE_AGGREGATE, &a, spins);
        } else {
            T v[kGroupK];
            ok = wait_aggregates(base, cnt, v, spins);
#pragma unroll
            for (int j = 0; j < kGroupK; ++j)
                if (static_cast<uint64_t>(lane) * kGroupK + j < cnt) a = op(a, v[j]);
        }
        T e = id;
        if (ok) ok = wait_slot(base, TILE_INCLUSIVE, &e, spins);  // E(base): base is a group's first tile
        if (!__all(ok)) {
            if (lane == 0 && err)
                __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return id;
        }
        const T excl = op(readlane(e, 0), wave_reduce(a, op));
        if (tile == first && lane == 0) publish(tile, excl, TILE_INCLUSIVE);
        return excl;
    }

    // The same for an operator without identity (noid_op): the cnt >= 1
    // aggregates are folded by an identity-free wave scan read at lane
    // cnt - 1 (lanes past cnt hold any value and are not read).
    template <bool ONEHOP = HPXHIP_LB_ONEHOP, typename Op>
    __device__ __forceinline__ T exclusive_prefix_fixed_noid(uint64_t tile, Op op) const {
        const int lane = lane_id();
        const uint64_t first = tile / kGroup * kGroup;
        if constexpr (ONEHOP && kGroupK == 1) {
            if (first > 0) {
                const uint64_t pos = tile - first;
                uint32_t spins = 0;
                T a1{}, a2{}, e{};
                const bool ok = wait_onehop(first, pos, &a1, &a2, &e, spins);
                if (!__all(ok)) {
                    if (lane == 0 && err)
                        __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    return e;
                }
                // lanes past the counts hold any value and are not read
                const T eg = op(readlane(e, 0), readlane(wave_inclusive_scan_noid(a1, op), static_cast<int>(kGroup - 1)));
                if (pos == 0) {
                    if (lane == 0) publish(tile, eg, TILE_INCLUSIVE);
                    return eg;
                }
                return op(eg, readlane(wave_inclusive_scan_noid(a2, op), static_cast<int>(pos - 1)));
            }
        }
        const uint64_t base = tile == first ? first - kGroup : first;
        const uint64_t cnt = tile == first ? kGroup : tile - first;
        uint32_t spins = 0;
        T a{};
        bool ok = true;
        if constexpr (kGroupK == 1) {
            if (static_cast<uint64_t>(lane) < cnt) ok = wait_slot(base + lane, TILE_AGGREGATE, &a, spins);
        } else {
            T v[kGroupK];
            ok = wait_aggregates(base, cnt, v, spins);
            a = v[0];  // lanes with no aggregate hold any value: not read
#pragma unroll
            for (int j = 1; j < kGroupK; ++j)
                if (static_cast<uint64_t>(lane) * kGroupK + j < cnt) a = op(a, v[j]);
        }
        T e{};
        if (ok) ok = wait_slot(base, TILE_INCLUSIVE, &e, spins);
        if (!__all(ok)) {
            if (lane == 0 && err)
                __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return e;
        }
        const T excl = op(readlane(e, 0), readlane(wave_inclusive_scan_noid(a, op),
                                                   static_cast<int>((cnt - 1) / kGroupK)));
        if (tile == first && lane == 0) publish(tile, excl, TILE_INCLUSIVE);
        return excl;
    }
};

}  // namespace hpxhip
