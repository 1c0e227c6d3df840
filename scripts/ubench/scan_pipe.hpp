// scan_pipe.hpp -- EXPERIMENT (not shipped): persistent, register double-buffered
// single-pass scan with a dedicated control wave.  Measured 3.7-4.2 ms for
// 2^30 int64 against 2.83-2.89 ms for the shipped one-tile-per-workgroup
// kernel (profiles/r02_ubench_scan_pipe.log): every phase waits one tile
// hand-off, and the prefetch of one tile does not cover it.
//
// Why: the one-tile-per-workgroup kernel (scan_kernel.hpp) runs one 1024-thread
// workgroup per CU, so each CU alternates load burst -> local scan -> tile
// hand-off -> store burst with nothing in flight in between, and pays the
// tile-id dequeue (1-3 us under streaming, MI355X guide price list row
// `dequeue`) and the workgroup launch/retire on every tile.  Measured: the
// same tile without any look-back still took 2.73-2.82 ms for 2^30 int64
// against 2.53 ms for a copy of the same bytes.
//
// Here a workgroup stays resident and walks tiles in a two-deep register
// pipeline.  Waves 1..15 move data: while they scan and store tile k from
// buffer X, tile k+1 is already loading into buffer Y, and right after
// storing tile k they start loading tile k+2 into X.  Wave 0 issues no data
// loads at all: it dequeues tile ids and runs the decoupled look-back.  (The
// vector-memory counter retires in order, so a look-back poll issued by a
// wave with a prefetch in flight would first wait for the whole prefetch --
// measured: 4.1 ms for 2^30 int64 when every wave both loaded and polled.)
//
// Tile ids still come from one atomic counter, so a tile only ever waits on
// tiles already claimed by running workgroups: the lowest claimed, unfinished
// tile is always some workgroup's CURRENT tile (a prefetched tile was claimed
// after that workgroup's current one), whose predecessors are all done --
// forward progress needs no dispatch-order or co-residency assumption.
//
// Build the translation unit with -mllvm -amdgpu-atomic-optimizer-strategy=None:
// the atomic optimizer rewrites the single-lane add into a wave-aggregated
// add broadcast by readfirstlane right away (an s_waitcnt vmcnt(0)).
#pragma once

#include "../../hpx_amd/csrc/common.hpp"
#include "../../hpx_amd/csrc/lookback.hpp"
#include "../../hpx_amd/csrc/scan_kernel.hpp"

namespace hpxhip {
namespace scan_detail {

constexpr int kPipeThreads = 1024;  // 16 waves: wave 0 control, 15 data waves

template <typename T, int R, int THREADS = kPipeThreads>
struct pipe_shape {
    static constexpr int V = 16 / sizeof(T);
    static constexpr int DATA_WAVES = THREADS / kWave - 1;
    static constexpr uint64_t WAVE_ELEMS = static_cast<uint64_t>(kWave) * R * V;
    static constexpr uint64_t TILE = WAVE_ELEMS * DATA_WAVES;
};

template <typename T, typename Conv, typename Op, bool INCL, int R, int THREADS>
struct pipe_data {
    using S = pipe_shape<T, R, THREADS>;
    static constexpr int V = S::V;
    using VT = vec<T, V>;

    const T* in;
    T* out;
    uint64_t n;
    Conv conv;
    Op op;

    __device__ __forceinline__ bool full(uint64_t tile) const { return tile * S::TILE + S::TILE <= n; }

    // R 16-byte loads per lane, no divergence (the compiler's counted waits
    // stay exact across the pipeline).  In the partial tail tile, vectors past
    // the last whole vector re-read that vector; scan() masks them and reads
    // the scalar remainder itself.
    __device__ __forceinline__ void load(VT (&x)[R], uint64_t tile, int dwave) const {
        const int lane = lane_id();
        const uint64_t wvec = (tile * S::TILE + dwave * S::WAVE_ELEMS) / V;
        const uint64_t nvec = n / V;  // >= 1: the kernel only runs for n >= TILE
        const VT* src = reinterpret_cast<const VT*>(in);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint64_t iv = wvec + static_cast<uint64_t>(r) * kWave + lane;
            iv = iv < nvec ? iv : nvec - 1;
            x[r] = ld_stream(&src[iv]);
        }
    }

    // Wave-local scan of this wave's part of the tile; returns the wave total.
    __device__ __forceinline__ T scan(VT (&x)[R], uint64_t tile, int dwave) const {
        const int lane = lane_id();
        const T id = Op::template identity<T>();
        if (full(tile)) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) x[r].v[e] = conv(x[r].v[e]);
        } else {
            const uint64_t wbase = tile * S::TILE + dwave * S::WAVE_ELEMS;
            const uint64_t whole = (n / V) * V;
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                    x[r].v[e] = i < whole ? conv(x[r].v[e]) : (i < n ? conv(in[i]) : id);
                }
        }
        T carry = id;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            T local[V];
            T run = id;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const T nxt = op(run, x[r].v[e]);
                local[e] = INCL ? nxt : run;
                run = nxt;
            }
            const T incl = wave_inclusive_scan(run, op);
            const T excl = wave_shift_right<T, Op>(incl);
            const T pre = op(carry, excl);
#pragma unroll
            for (int e = 0; e < V; ++e) x[r].v[e] = op(pre, local[e]);
            carry = op(carry, readlane(incl, kWave - 1));
        }
        return carry;
    }

    // Full-tile forms without any branch on the tile (see k_scan_pipe).
    __device__ __forceinline__ T scan_full(VT (&x)[R]) const {
        const T id = Op::template identity<T>();
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) x[r].v[e] = conv(x[r].v[e]);
        T carry = id;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            T local[V];
            T run = id;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const T nxt = op(run, x[r].v[e]);
                local[e] = INCL ? nxt : run;
                run = nxt;
            }
            const T incl = wave_inclusive_scan(run, op);
            const T excl = wave_shift_right<T, Op>(incl);
            const T pre = op(carry, excl);
#pragma unroll
            for (int e = 0; e < V; ++e) x[r].v[e] = op(pre, local[e]);
            carry = op(carry, readlane(incl, kWave - 1));
        }
        return carry;
    }
    __device__ __forceinline__ void store_full(VT (&x)[R], uint64_t tile, int dwave, T pre) const {
        const int lane = lane_id();
        VT* dst = reinterpret_cast<VT*>(out + tile * S::TILE + dwave * S::WAVE_ELEMS);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            VT y;
#pragma unroll
            for (int e = 0; e < V; ++e) y.v[e] = op(pre, x[r].v[e]);
            dst[r * kWave + lane] = y;
        }
    }

    __device__ __forceinline__ void store(VT (&x)[R], uint64_t tile, int dwave, T pre) const {
        const int lane = lane_id();
        const uint64_t wbase = tile * S::TILE + dwave * S::WAVE_ELEMS;
        if (full(tile)) {
            VT* dst = reinterpret_cast<VT*>(out + wbase);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                VT y;
#pragma unroll
                for (int e = 0; e < V; ++e) y.v[e] = op(pre, x[r].v[e]);
                dst[r * kWave + lane] = y;
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                    if (i < n) out[i] = op(pre, x[r].v[e]);
                }
        }
    }
};

__device__ __forceinline__ uint32_t claim_tile(uint32_t* counter) {
    return __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Requires 16-byte aligned in and out and n >= one tile (the caller routes
// other ranges to k_scan).  Launch about as many workgroups as are resident
// at once (one per CU); more only idle at the end.
template <typename T, typename Conv, typename Op, bool INCL, int R, int THREADS = kPipeThreads>
__global__ __launch_bounds__(THREADS, 1) void k_scan_pipe(const T* in, T* out, uint64_t n, Conv conv, Op op, T init,
                                                          const T* prefix_dev, uint32_t* counter, tile_state<T> st,
                                                          uint64_t ntiles) {
    using D = pipe_data<T, Conv, Op, INCL, R, THREADS>;
    using VT = typename D::VT;
    constexpr int DW = D::S::DATA_WAVES;
    __shared__ T s_total[DW];      // data wave totals -> their exclusive tile prefixes
    __shared__ uint32_t s_ids[2];  // [current, next] at start; then s_ids[0] = the tile after next
    const D d{in, out, n, conv, op};
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();

    // The first two ids are dequeued one round trip apart: two back-to-back
    // adds by one workgroup would take two CONSECUTIVE ids, and the second
    // (processed a phase later) would hold up the next workgroup's first
    // tile, which would hold up the next ... -- a chain across the whole
    // grid (measured 16-30 ms for 2^30 int64).  Dequeued a round trip apart,
    // the first ids of all resident workgroups come before their second ids
    // and the tiles in flight stay contiguous.  (Ordering only: the protocol
    // is correct for any interleaving.)
    if (threadIdx.x == 0) s_ids[0] = claim_tile(counter);
    __syncthreads();
    uint64_t cur = s_ids[0];
    if (threadIdx.x == 0) s_ids[1] = claim_tile(counter);
    __syncthreads();
    uint64_t nxt = s_ids[1];
    if (cur >= ntiles) return;  // uniform over the workgroup

    if (wave == 0) {
        // ---------------------------------------------------- control wave
        uint32_t claim = 0;
        if (lane == 0) claim = claim_tile(counter);
        while (true) {
            __syncthreads();  // barrier 1: data totals of `cur` are in s_total
            tile_prefix<T, Op, DW, true>(cur, st, op, prefix_dev, init, s_total);
            if (lane == 0) s_ids[0] = claim;
            __syncthreads();  // barrier 2: prefixes and the next id published
            if (nxt >= ntiles) break;
            cur = nxt;
            nxt = static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(claim));
            // the data waves read s_ids[0] after barrier 2, before barrier 1 of
            // the next phase; it is rewritten only after that barrier
            if (lane == 0) claim = claim_tile(counter);
        }
    } else {
        // ------------------------------------------------------- data waves
        // No memory access in the loop is conditional, so the compiler's
        // counted waits stay exact: the next tile's loads survive the scan
        // of the current one.  The partial tail tile (always the last one)
        // leaves the loop and is finished below.
        const int dw = wave - 1;
        VT xa[R], xb[R];
        // a tile id past the end re-reads the last tile (never used)
        d.load(xa, cur, dw);
        d.load(xb, nxt < ntiles ? nxt : ntiles - 1, dw);
        auto phase = [&](VT(&X)[R]) -> int {
            if (!d.full(cur)) return 2;
            const T total = d.scan_full(X);
            if (lane == 0) s_total[dw] = total;
            __syncthreads();  // barrier 1
            __syncthreads();  // barrier 2
            const T pre = s_total[dw];
            const uint64_t after = s_ids[0];
            d.store_full(X, cur, dw, pre);
            if (nxt >= ntiles) return 1;
            cur = nxt;
            nxt = after;
            d.load(X, nxt < ntiles ? nxt : ntiles - 1, dw);
            return 0;
        };
        auto tail = [&](VT(&X)[R]) {
            const T total = d.scan(X, cur, dw);
            if (lane == 0) s_total[dw] = total;
            __syncthreads();  // barrier 1
            __syncthreads();  // barrier 2
            d.store(X, cur, dw, s_total[dw]);
        };
        while (true) {
            const int ra = phase(xa);
            if (ra) {
                if (ra == 2) tail(xa);
                break;
            }
            const int rb = phase(xb);
            if (rb) {
                if (rb == 2) tail(xb);
                break;
            }
        }
    }
}

}  // namespace scan_detail
}  // namespace hpxhip
