// lookback.hpp -- single-pass decoupled look-back tile state (scan, copy_if).
//
// HPX's scan_partitioner (util/scan_partitioner.hpp:62-156) runs three
// phases: chunk totals, a left-to-right prefix of totals (dataflow), and a
// fix-up pass -- two passes over the data.  On the GPU the same prefix is
// formed in ONE pass: each tile publishes its aggregate as soon as it has
// loaded its input, then walks back over its predecessors (64 at a time, one
// per lane of the look-back wave) until it meets an inclusive prefix.
//
// Tile ids come from an atomic counter, so a tile only ever waits on tiles
// whose workgroups are already running (forward progress does not depend on
// dispatch order).  Hand-off form (MI355X guide, Guideline 16 table row 1):
// the value is stored with an agent-scope sc1 store, the lane drains
// (`s_waitcnt vmcnt(0)`), then stores the flag; the consumer polls the flag
// with sc1 loads and only after the poll matched loads the value with sc1.
// Every wait is bounded (kSpinLimit) and raises the device error word.
#pragma once

#include "common.hpp"

namespace hpxhip {

enum : uint32_t { TILE_INVALID = 0, TILE_AGGREGATE = 1, TILE_INCLUSIVE = 2 };

template <typename T>
struct tile_state {
    uint32_t* flags;  // [ntiles]
    T* agg;           // [ntiles]
    T* incl;          // [ntiles]
    uint32_t* err;    // device error word (may be null)

    // Lane-uniform call by ONE lane.
    __device__ __forceinline__ void publish(uint64_t tile, T v, uint32_t status) const {
        st_agent(status == TILE_INCLUSIVE ? &incl[tile] : &agg[tile], v);
        drain_stores();
        __hip_atomic_store(&flags[tile], status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // Called by ALL 64 lanes of one wave; returns the exclusive prefix of
    // `tile` (op-combination of every predecessor's elements) on every lane.
    // Requires tile > 0 and that tile 0 publishes an inclusive value.
    template <typename Op>
    __device__ __forceinline__ T exclusive_prefix(uint64_t tile, Op op) const {
        const T id = Op::template identity<T>();
        const int lane = lane_id();
        T excl = id;
        int64_t pred = static_cast<int64_t>(tile) - 1;
        uint32_t spins = 0;
        while (true) {
            const int64_t j = pred - lane;
            uint32_t f = TILE_INCLUSIVE;  // j < 0: behind tile 0, never reached
            if (j >= 0) f = __hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (!__all(f != TILE_INVALID)) {
                __builtin_amdgcn_s_sleep(1);
                if (f == TILE_INVALID)
                    f = __hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (++spins > kSpinLimit) {
                    if (lane == 0 && err)
                        __hip_atomic_store(err, HPXHIP_DEVERR_LOOKBACK_TIMEOUT, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    return excl;
                }
            }
            order_after_poll();
            const uint64_t inclusive_lanes = __ballot(f == TILE_INCLUSIVE);
            const int first = inclusive_lanes ? __builtin_ctzll(inclusive_lanes) : kWave;
            T v = id;
            if (lane < first) v = ld_agent(&agg[j]);
            else if (lane == first && j >= 0) v = ld_agent(&incl[j]);
            const T s = wave_reduce(v, op);
            excl = op(s, excl);
            if (first < kWave) break;
            pred -= kWave;
        }
        return excl;
    }
};

}  // namespace hpxhip
