// sort_kernel.hpp -- kernels of the LSD onesweep radix sort (see sort.hip
// for the algorithm notes).  Header so that scripts/ubench instantiates the
// shipped kernels with other tile shapes.
#pragma once

#include <hpxhip/kernels/common.hpp>

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

// Wave match of 8-bit digits: the lanes among `active` whose digit equals
// this lane's.  Per bit one ballot (v_cmp on the lane's bit as 0/-1) folded
// into both halves of the peer mask with one v_bitop3 each (acc & ~(m ^ x),
// truth table 0x90): 4 VALU per bit where the select/xor/and form took 9
// (scripts/ubench/bucket.hip; the ranking is the VALU-bound part of a pass).
// The ballot stays an inline-asm v_cmp into one SGPR pair.  r04 A/B
// (profiles/r04_sort_ab_ballot.log): the compiler's ballot
// (__builtin_amdgcn_ballot_w64) gives every bit its own SGPRs and interleaves
// neighbouring keys, but the full sort got slower (2^30 u64 18.9-19.0 vs
// 18.3-18.5 ms, u32 14.1 vs 13.5): the extra SGPR pairs spill into VGPR
// lanes in the segment sort and lengthen the onesweep passes.
// HPXHIP_MATCH_ASM=0 builds the builtin form.
#ifndef HPXHIP_MATCH_ASM
#define HPXHIP_MATCH_ASM 1
#endif
// the segment sort's first LDS pass ranked by LDS atomics (k_bucket_sort;
// r05 lease ak, profiles/r05_merge_step_seg_atom1.log: no change, off)
#ifndef HPXHIP_SEG_ATOM1
#define HPXHIP_SEG_ATOM1 0
#endif
// the offset-fed first prefix pass ranked by LDS atomics (k_onesweep; r05
// lease al, profiles/r05_sort_os_atom1.log: 2^30 u32 12.16 -> 11.62 ms, u64
// unchanged at 16.1)
#ifndef HPXHIP_OS_ATOM1
#define HPXHIP_OS_ATOM1 1
#endif
// k_onesweep's tile loads without per-key branches (r05 lease ap,
// profiles/r05_sort_uncond_load.log: first prefix pass ~4.2 -> 3.95 ms, 2^30
// u64 16.48-16.57 -> 15.92-16.06 ms, u32 11.65-11.70 -> 11.41-11.51)
#ifndef HPXHIP_OS_UNCOND_LOAD
#define HPXHIP_OS_UNCOND_LOAD 1
#endif
// ... and k_bucket_sort's segment loads
#ifndef HPXHIP_SEG_UNCOND_LOAD
#define HPXHIP_SEG_UNCOND_LOAD 0
#endif
template <int BITS = 8>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t active) {
    uint32_t lo = static_cast<uint32_t>(active), hi = static_cast<uint32_t>(active >> 32);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const uint32_t x = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(d), b, 1));
        uint64_t m;
#if HPXHIP_MATCH_ASM
        asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(m) : "v"(x));
#else
        m = __builtin_amdgcn_ballot_w64(x != 0);
#endif
        lo = __builtin_amdgcn_bitop3_b32(lo, static_cast<uint32_t>(m), x, 0x90);
        hi = __builtin_amdgcn_bitop3_b32(hi, static_cast<uint32_t>(m >> 32), x, 0x90);
    }
    return (static_cast<uint64_t>(hi) << 32) | lo;
}
// number of set bits of `peers` below this lane
__device__ __forceinline__ uint32_t peers_below(uint64_t peers) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(peers >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(peers), 0u));
}

// ------------------------------------------------ segmented LSD (r05)
// The oversized-bucket finish of the hybrid sort (sort.hip): the LSD passes
// run over a table of segments -- the few buckets a segment sort could not
// hold, or the whole array -- each sorted on its own.  Tile ids are global
// (the look-back state is one array); tile t belongs to segment j with
// tile0[j] <= t < tile0[j + 1], and its keys are start[j] + (t - tile0[j]) *
// TILE onwards.  Written by the planner on the device.
constexpr int kMaxBig = 64;
struct seg_table {
    uint64_t start[kMaxBig];
    uint64_t len[kMaxBig];
    uint64_t tile0[kMaxBig + 1];
    uint32_t nseg;
};

// ---------------------------------------------------------------- histogram
// One read of the keys -> all passes' 256-bin histograms.  Each bin has
// COPIES lane-private LDS counters (lane % COPIES), interleaved so that bin
// b, copy c sits at word b*COPIES + c: lanes of one wave-instruction that hit
// different bins then collide on a bank only when their bins agree mod
// 32/COPIES, instead of mod 32 (the single-copy histogram spent 72 % of its
// LDS cycles in bank conflicts, profiles/r01_pmc_sort.txt).  Keys are read
// with nontemporal 16-B loads.
// Digits [first, passes) are counted; bits[0] / bits[1] receive the OR / AND
// of all ordered keys (a digit is constant iff OR and AND agree on it), so a
// caller may count only the digits it needs first.  xshift >= 0 also counts
// the 9-bit field at bits [xshift, xshift + 9) into xhist (512 bins; the
// hybrid sort's 9-bit prefix pass).
constexpr int kXBins = 512;
// r04 (scripts/ubench/hist3.hip, profiles/r04_ubench_hist_context.log): LDS
// sized for the one or two counted digits with 8-16 lane copies measured the
// same (1.43-1.50 ms back to back, 1.60-1.69 right after the keys were
// written) as this shape; a plain 16-B read of the keys takes 1.22 / 1.29 ms.
// TF (the 18-bit form, sort.hip): also the top 9 bits, [tshift, tshift + 9),
// into thist (512 bins).
template <typename U, typename X, int THREADS = 256, int COPIES = 4, int D = static_cast<int>(sizeof(U)),
          bool TF = false>
__global__ __launch_bounds__(THREADS) void k_hist(const U* __restrict__ keys, uint64_t n, int first, int passes, X xf,
                                                   unsigned long long* __restrict__ hist,
                                                   unsigned long long* __restrict__ bits, int xshift,
                                                   unsigned long long* __restrict__ xhist,
                                                   const int32_t* __restrict__ gate = nullptr, int tshift = -1,
                                                   unsigned long long* __restrict__ thist = nullptr,
                                                   int skip_constant = 0) {
    if (gate && *gate == 0) return;  // device-planned sort: this count is not needed
    constexpr int P = static_cast<int>(sizeof(U));
    // skip_constant (a second count, after the first has left the keys' OR /
    // AND in bits): digits on which every key agrees are not counted -- no
    // plan reads them, and all 64 lanes adding into one bin serialise (r04:
    // keys below 2^16 spent ~1 ms of their 2^30 sort counting six constant
    // bytes)
    uint32_t live = 0xffu;
    if (skip_constant) {
        const unsigned long long diff = bits[0] ^ bits[1];
#pragma unroll
        for (int p = 0; p < P; ++p)
            if (((diff >> (8 * p)) & 0xffu) == 0) live &= ~(1u << p);
    }
    static_assert(D >= 1 && D <= P, "digit slots");
    __shared__ uint32_t h[D * kRadix * COPIES];
    __shared__ uint32_t hx[kXBins * COPIES];
    __shared__ uint32_t ht[TF ? kXBins * COPIES : 1];
    for (int i = threadIdx.x; i < D * kRadix * COPIES; i += THREADS) h[i] = 0;
    for (int i = threadIdx.x; i < kXBins * COPIES; i += THREADS) hx[i] = 0;
    if constexpr (TF)
        for (int i = threadIdx.x; i < kXBins * COPIES; i += THREADS) ht[i] = 0;
    __syncthreads();
    constexpr int V = 16 / sizeof(U);
    using VT = vec<U, V>;
    const uint32_t copy = threadIdx.x % COPIES;
    // a range starting inside a 16-B vector (a bucket of the hybrid sort's
    // oversized-bucket finish starts anywhere): its head is counted by
    // scalar loads and the 16-B loads start at the first aligned key
    const uint64_t mis = (reinterpret_cast<uintptr_t>(keys) % 16) / sizeof(U);
    const uint64_t head = mis ? (n < V - mis ? n : V - mis) : 0;
    const U* akeys = keys + head;
    const uint64_t nvec = (n - head) / V;
    const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * THREADS + threadIdx.x;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * THREADS;
    const VT* vk = reinterpret_cast<const VT*>(akeys);
    U any = 0, all = static_cast<U>(~U(0));
    auto count = [&](U b) {
        any |= b;
        all &= b;
#pragma unroll
        for (int p = 0; p < P; ++p)
            if (p >= first && p < passes && p - first < D && ((live >> p) & 1u))
                atomicAdd(&h[((p - first) * kRadix + ((b >> (8 * p)) & 0xff)) * COPIES + copy], 1u);
        if (xshift >= 0) atomicAdd(&hx[static_cast<uint32_t>((b >> xshift) & (kXBins - 1)) * COPIES + copy], 1u);
        if constexpr (TF) atomicAdd(&ht[static_cast<uint32_t>((b >> tshift) & (kXBins - 1)) * COPIES + copy], 1u);
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
    if (tid < n - head - nvec * V) count(xf(akeys[nvec * V + tid]));
    if (tid < head) count(xf(keys[tid]));
    any = wave_reduce(any, op_bit_or{});
    all = wave_reduce(all, op_bit_and{});
    if (lane_id() == 0) {
        atomicOr(&bits[0], static_cast<unsigned long long>(any));
        atomicAnd(&bits[1], static_cast<unsigned long long>(all) | (sizeof(U) == 8 ? 0ull : ~0ull << 32));
    }
    __syncthreads();
    const int counted = (passes - first < D ? passes - first : D) * kRadix;
    for (int i = threadIdx.x; i < counted; i += THREADS) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < COPIES; ++k) c += h[i * COPIES + k];
        if (c) atomicAdd(&hist[first * kRadix + i], static_cast<unsigned long long>(c));
    }
    if (xshift >= 0)
        for (int i = threadIdx.x; i < kXBins; i += THREADS) {
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < COPIES; ++k) c += hx[i * COPIES + k];
            if (c) atomicAdd(&xhist[i], static_cast<unsigned long long>(c));
        }
    if constexpr (TF)
        for (int i = threadIdx.x; i < kXBins; i += THREADS) {
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < COPIES; ++k) c += ht[i * COPIES + k];
            if (c) atomicAdd(&thist[i], static_cast<unsigned long long>(c));
        }
}

// ------------------------------------------- per-tile counts (r04, 18-bit form)
// The first prefix pass without a look-back.  A 9-bit pass runs 5.54 ms at
// 2^30 keys with its look-back and 3.37 with none at all
// (profiles/r04_ubench_sortpass3_lbb0.log; that ablation's wrong offsets
// also fold its stores into a few lines, so it overstates the saving), and
// the first pass's tiles are the input's own: their digit counts can come out
// of the histogram read that precedes the pass.  Measured: the pass 5.3-5.5
// -> 5.1 ms, the sort 2^30 u64 18.0 -> 17.6 ms, u32 13.2 -> 12.6.  k_hist_tiles reads the keys
// once, in the onesweep's 8192-key tiles (strided over the grid), and writes
//   tcount[t * 512 + d]  tile t's count of field digit d,
// plus the field's and the top 9 bits' histograms and the keys' OR / AND (what
// k_hist<..., TF> gives).  k_chunk_sums (r05) totals the tile counts per
// chunk of kTileChunk tiles, k_tile_chunk_scan turns the chunk totals into
// exclusive prefixes (from the digits' bin starts), k_tile_offsets the tile
// counts into each tile's destination offsets, which the pass reads instead
// of walking back (k_onesweep PRE).  Offsets are 32-bit: n < 2^32.
template <typename U, typename X, int TILE = 8192, int THREADS = 512>
__global__ __launch_bounds__(THREADS) void k_hist_tiles(const U* __restrict__ keys, uint64_t n, uint64_t ntiles,
                                                         X xf, int xshift, int tshift, uint32_t* __restrict__ tcount,
                                                         unsigned long long* __restrict__ xhist,
                                                         unsigned long long* __restrict__ thist,
                                                         unsigned long long* __restrict__ bits,
                                                         unsigned long long* __restrict__ joint) {
    static_assert(THREADS == kXBins, "one thread per field digit");
    constexpr int V = 16 / static_cast<int>(sizeof(U));
    constexpr int VPT = TILE / V / THREADS;  // 16-B vectors per thread per tile
    static_assert(VPT * V * THREADS == TILE, "tile of whole vectors");
    using VT = vec<U, V>;
    __shared__ uint32_t cnt[2 * kXBins];
    // r05: the top 9 bits counted per field region (field >> 6: 8 regions of
    // 64 field digits) -- joint[region][top9], whose sum over the regions is
    // the top-9 histogram; the second prefix pass runs one region per XCD
    // and takes each region's bin starts from it (k_region_plan)
    __shared__ uint32_t hj[8 * kXBins];
    const int d = threadIdx.x;
    cnt[d] = 0;
    cnt[kXBins + d] = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) hj[x * kXBins + d] = 0;
    __syncthreads();
    const bool aligned = reinterpret_cast<uintptr_t>(keys) % 16 == 0;
    U any = 0, all = static_cast<U>(~U(0));
    uint32_t csum_d = 0;
    // A (field, top-9) cell that the first lane still to add shares with at
    // least 4 lanes of its wave is counted once, for all of them, up to three
    // such cells per key; the other lanes add one each (r05: sorted or
    // heavily skewed input -- a hot prefix in the first tiles -- had
    // serialized the lanes of a wave on one or two LDS words: the histogram
    // took 2.9 ms at 2^28 u64hot against 0.42 for uniform keys).  Those
    // shared counts go to a two-entry per-wave cache (scalar registers) and
    // reach LDS only when evicted or at the tile's end: the waves of a
    // workgroup no longer take turns on the same hot words.  Uniform keys pay
    // one readlane + compare + ballot per key (peeling the first two lanes'
    // cells unconditionally had cost them 4x: 1.75 ms at 2^28).
    uint32_t cc0 = ~0u, cc1 = ~0u, cn0 = 0, cn1 = 0;
    auto add_cell = [&](uint32_t c, uint32_t v, uint32_t* ct) {
        atomicAdd(&ct[c >> 12], v);
        atomicAdd(&hj[c & 0xfffu], v);
    };
    auto count = [&](U b, uint32_t* ct) {
        any |= b;
        all &= b;
        const uint32_t f = static_cast<uint32_t>(b >> xshift) & (kXBins - 1);
        const uint32_t j = (f >> 6) * kXBins + (static_cast<uint32_t>(b >> tshift) & (kXBins - 1));
        const uint32_t cell = (f << 12) | j;
        uint64_t rem = __ballot(1);
#pragma unroll
        for (int it = 0; it < 3; ++it) {
            if (rem == 0) break;
            const int lead = __builtin_ctzll(rem);
            const uint32_t c0 = __builtin_amdgcn_readlane(cell, lead);
            const uint64_t grp = __ballot(cell == c0) & rem;
            const uint32_t c = static_cast<uint32_t>(__builtin_popcountll(grp));
            if (c < 4) break;
            if (c0 == cc0) {
                cn0 += c;
            } else if (c0 == cc1) {
                cn1 += c;
            } else {
                if (cn1 && lane_id() == lead) add_cell(cc1, cn1, ct);
                cc1 = cc0;
                cn1 = cn0;
                cc0 = c0;
                cn0 = c;
            }
            rem &= ~grp;
        }
        if ((rem >> lane_id()) & 1u) add_cell(cell, 1u, ct);
    };
    // r05: tiles strided over the grid (workgroup w: tiles w, w + G, ...)
    // instead of a chunk of consecutive tiles each: a hot run of keys (sorted
    // or skewed input) no longer lands on a few workgroups that the whole
    // launch then waits for, and a 2^28-key sort fills the chip (512
    // workgroups against 128 chunks); the chunk totals come from k_chunk_sums
    // r05: the next tile's keys are loaded while this tile's are counted
    // (x / xn; the grid has 2 workgroups per CU, so the registers are there),
    // and the per-tile counts alternate between two LDS arrays, so one
    // barrier per tile separates a tile's counting from its flush
    auto full_tile = [&](uint64_t t) { return aligned && (t + 1) * TILE <= n; };
    auto load = [&](VT (&dst)[VPT], uint64_t t) {
        const VT* vk = reinterpret_cast<const VT*>(keys + t * TILE);
#pragma unroll
        for (int j = 0; j < VPT; ++j) dst[j] = ld_stream(&vk[j * THREADS + d]);
    };
    VT x[VPT];
    uint64_t t = blockIdx.x;
    if (t < ntiles && full_tile(t)) load(x, t);
    int buf = 0;
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * TILE;
        const uint64_t tn = t + gridDim.x;
        const bool pf = tn < ntiles && full_tile(tn);
        VT xn[VPT];
        if (pf) load(xn, tn);
        uint32_t* ct = cnt + buf * kXBins;
        if (full_tile(t)) {
#pragma unroll
            for (int j = 0; j < VPT; ++j)
#pragma unroll
                for (int e = 0; e < V; ++e) count(xf(x[j].v[e]), ct);
        } else {
            const uint64_t m = n - base < TILE ? n - base : TILE;
            for (uint64_t i = d; i < m; i += THREADS) count(xf(keys[base + i]), ct);
        }
        // lane 0 holds the wave's cache: in the ragged loop a lane that drops
        // out never comes back, and lane 0 is the last of its wave to drop out
        if (lane_id() == 0) {
            if (cn0) add_cell(cc0, cn0, ct);
            if (cn1) add_cell(cc1, cn1, ct);
        }
        cc0 = cc1 = ~0u;
        cn0 = cn1 = 0;
        __syncthreads();  // the tile's counts are complete; the other array was flushed a tile ago
        const uint32_t c = ct[d];
        tcount[t * kXBins + d] = c;
        csum_d += c;
        ct[d] = 0;  // counted into again two tiles on, after the next barrier
        buf ^= 1;
        if (pf) {
#pragma unroll
            for (int j = 0; j < VPT; ++j) x[j] = xn[j];
        }
    }
    if (csum_d) atomicAdd(&xhist[d], static_cast<unsigned long long>(csum_d));
    uint32_t tc = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        const uint32_t c = hj[x * kXBins + d];
        tc += c;
        if (c) atomicAdd(&joint[x * kXBins + d], static_cast<unsigned long long>(c));
    }
    if (tc) atomicAdd(&thist[d], static_cast<unsigned long long>(tc));
    any = wave_reduce(any, op_bit_or{});
    all = wave_reduce(all, op_bit_and{});
    if (lane_id() == 0) {
        atomicOr(&bits[0], static_cast<unsigned long long>(any));
        atomicAnd(&bits[1], static_cast<unsigned long long>(all) | (sizeof(U) == 8 ? 0ull : ~0ull << 32));
    }
}

// Chunk totals of the tile counts (workgroup c: chunk c's tiles, thread d:
// digit d); runs iff *gate >= 0.
__global__ __launch_bounds__(kXBins) void k_chunk_sums(const uint32_t* __restrict__ tcount, uint64_t ntiles,
                                                       uint32_t chunk, uint32_t* __restrict__ csum,
                                                       const int32_t* __restrict__ gate) {
    if (*gate < 0) return;
    const int d = threadIdx.x;
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * chunk;
    const uint64_t t1 = t0 + chunk < ntiles ? t0 + chunk : ntiles;
    uint32_t sum = 0;
    uint64_t t = t0;
    for (; t + 8 <= t1; t += 8) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tcount[(t + j) * kXBins + d];
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += v[j];
    }
    for (; t < t1; ++t) sum += tcount[t * kXBins + d];
    csum[static_cast<uint64_t>(blockIdx.x) * kXBins + d] = sum;
}

// Chunk totals -> exclusive prefixes from the field's bin starts (one
// workgroup, thread d walks digit d's column); runs iff *gate >= 0.
__global__ __launch_bounds__(kXBins) void k_tile_chunk_scan(uint32_t* __restrict__ csum, uint64_t nchunks,
                                                            const unsigned long long* __restrict__ xstart,
                                                            const int32_t* __restrict__ gate) {
    if (*gate < 0) return;
    const int d = threadIdx.x;
    uint32_t run = static_cast<uint32_t>(xstart[d]);
    uint64_t c = 0;
    for (; c + 8 <= nchunks; c += 8) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = csum[(c + j) * kXBins + d];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            csum[(c + j) * kXBins + d] = run;
            run += v[j];
        }
    }
    for (; c < nchunks; ++c) {
        const uint32_t v = csum[c * kXBins + d];
        csum[c * kXBins + d] = run;
        run += v;
    }
}

// Tile counts -> tile offsets in place (workgroup c: chunk c's tiles, thread
// d: digit d); runs iff *gate >= 0.
__global__ __launch_bounds__(kXBins) void k_tile_offsets(uint32_t* __restrict__ tcount, uint64_t ntiles,
                                                         uint32_t chunk, const uint32_t* __restrict__ csum,
                                                         const int32_t* __restrict__ gate) {
    if (*gate < 0) return;
    const int d = threadIdx.x;
    uint32_t run = csum[static_cast<uint64_t>(blockIdx.x) * kXBins + d];
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * chunk;
    const uint64_t t1 = t0 + chunk < ntiles ? t0 + chunk : ntiles;
    uint64_t t = t0;
    for (; t + 8 <= t1; t += 8) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tcount[(t + j) * kXBins + d];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            tcount[(t + j) * kXBins + d] = run;
            run += v[j];
        }
    }
    for (; t < t1; ++t) {
        const uint32_t v = tcount[t * kXBins + d];
        tcount[t * kXBins + d] = run;
        run += v;
    }
}

// The second prefix pass of the 18-bit form (r05): its input -- the first
// pass's output, ordered by the field -- cut into 8 regions of 64 field
// digits (contiguous: [xstart[64 x], xstart[64 x + 64])), one per XCD
// (k_onesweep XREG + SEG), each with its own look-back; region x's bin start
// for top-9 digit d is tstart[d] + the keys of digit d in regions < x
// (joint, k_hist_tiles).  One workgroup, thread d owns digit d.
__global__ __launch_bounds__(kXBins) void k_region_plan(const unsigned long long* __restrict__ xstart,
                                                         const unsigned long long* __restrict__ tstart,
                                                         const unsigned long long* __restrict__ joint, uint64_t n,
                                                         int tile, seg_table* __restrict__ segs,
                                                         unsigned long long* __restrict__ bs) {
    const int d = threadIdx.x;
    if (d == 0) {
        segs->nseg = 8;
        uint64_t t = 0;
        for (int x = 0; x < 8; ++x) {
            const uint64_t lo = xstart[64 * x], hi = x < 7 ? xstart[64 * (x + 1)] : n;
            segs->start[x] = lo;
            segs->len[x] = hi - lo;
            segs->tile0[x] = t;
            t += (hi - lo + tile - 1) / tile;
        }
        segs->tile0[8] = t;
    }
    unsigned long long run = tstart[d];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        bs[x * kXBins + d] = run;
        run += joint[x * kXBins + d];
    }
}

// Exclusive scan of each pass's R counts (one R-thread block per pass).
template <int R = kRadix>
__global__ __launch_bounds__(R) void k_bin_offsets(const unsigned long long* __restrict__ hist,
                                                    unsigned long long* __restrict__ start) {
    __shared__ uint64_t s_w[R / kWave];
    const int p = blockIdx.x;
    const int d = threadIdx.x;
    const uint64_t c = hist[p * R + d];
    const uint64_t incl = wave_inclusive_scan(c, op_plus{});
    const int wave = d / kWave;
    if (lane_id() == kWave - 1) s_w[wave] = incl;
    __syncthreads();
    uint64_t pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_w[w];
    start[p * R + d] = pre + incl - c;
}

// Every digit's 256-bin histogram of every segment (hist[j][8][256], the
// segment's pass p at [j][p]); a persistent grid over the segments' TILE-key
// tiles; runs iff *gate.
template <typename U, typename X, int THREADS = 256, int TILE = 8192>
__global__ __launch_bounds__(THREADS) void k_seg_hist(const U* __restrict__ keys, const seg_table* __restrict__ segs,
                                                       X xf, unsigned long long* __restrict__ hist,
                                                       const int32_t* __restrict__ gate) {
    if (*gate == 0) return;
    constexpr int P = static_cast<int>(sizeof(U));
    __shared__ uint32_t s_h[P * kRadix];
    const uint32_t nseg = segs->nseg;
    const uint64_t ntiles = segs->tile0[nseg];
    for (uint64_t tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
        uint32_t j = 0;
        while (j + 1 < nseg && segs->tile0[j + 1] <= tl) ++j;
        const uint64_t lo = segs->start[j] + (tl - segs->tile0[j]) * TILE;
        const uint64_t end = segs->start[j] + segs->len[j];
        const uint64_t hi = lo + TILE < end ? lo + TILE : end;
        for (int i = threadIdx.x; i < P * kRadix; i += THREADS) s_h[i] = 0;
        __syncthreads();
        for (uint64_t i = lo + threadIdx.x; i < hi; i += THREADS) {
            const U u = xf(keys[i]);
#pragma unroll
            for (int q = 0; q < P; ++q) atomicAdd(&s_h[q * kRadix + ((u >> (8 * q)) & 0xffu)], 1u);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < P * kRadix; i += THREADS)
            if (s_h[i]) atomicAdd(&hist[static_cast<uint64_t>(j) * 8 * kRadix + i], static_cast<unsigned long long>(s_h[i]));
        __syncthreads();
    }
}

// Segment j, pass p (block j * 8 + p): bin starts = start[j] + the exclusive
// scan of its histogram; runs iff *gate.  Without *counted (a planned
// whole-array LSD) segment 0's come from the global histogram (ghist).
__global__ __launch_bounds__(kRadix) void k_seg_offsets(const unsigned long long* __restrict__ hist,
                                                         const seg_table* __restrict__ segs,
                                                         unsigned long long* __restrict__ bs,
                                                         const int32_t* __restrict__ gate,
                                                         const int32_t* __restrict__ counted,
                                                         const unsigned long long* __restrict__ ghist) {
    if (*gate == 0) return;
    const uint32_t j = blockIdx.x / 8;
    if (j >= segs->nseg) return;
    __shared__ unsigned long long s_w[kRadix / kWave];
    const uint64_t o = static_cast<uint64_t>(blockIdx.x) * kRadix;
    const int t = threadIdx.x;
    const unsigned long long c = *counted ? hist[o + t] : ghist[o + t];
    const unsigned long long incl = wave_inclusive_scan(c, op_plus{});
    if (lane_id() == kWave - 1) s_w[t / kWave] = incl;
    __syncthreads();
    unsigned long long pre = segs->start[j];
    for (int w = 0; w < t / kWave; ++w) pre += s_w[w];
    bs[o + t] = pre + incl - c;
}

// dst = src over the segments' ranges (the LSD ended in the alternate
// buffer), runs iff *gate.
template <typename E>
__global__ __launch_bounds__(256) void k_seg_copy(const E* __restrict__ src, E* __restrict__ dst,
                                                  const seg_table* __restrict__ segs,
                                                  const int32_t* __restrict__ gate) {
    if (*gate == 0) return;
    for (uint32_t j = 0; j < segs->nseg; ++j) {
        const uint64_t lo = segs->start[j], len = segs->len[j];
        for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; i < len;
             i += static_cast<uint64_t>(gridDim.x) * 256)
            dst[lo + i] = src[lo + i];
    }
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
// RB = 9 (hybrid sort's 9-bit prefix pass): 512 digits, one per thread, with
// 16-bit per-wave counters so two workgroups still fit a CU's LDS.
// STAGE = false (ablation, scripts/ubench/sortpass2.hip): no LDS staging --
// every key is stored from registers straight to its final position.  It
// frees 64 KiB of LDS but the scattered 8-B stores make the pass 3x slower
// (14.3 vs 4.85 ms at 2^30 u64, profiles/r02_ubench_onesweep_direct.log).
// PERSIST (r03, the device-planned sort): a grid of about two workgroups
// per CU claims tiles from the counter until ntiles are done.  The plan
// gates every pass on the device, so passes it skips are still launched; a
// skipped 2^30-key pass had dispatched 131072 workgroups that only read the
// gate and left (~0.1 ms each, ~0.9 ms per sort over the skipped second-byte
// and LSD passes); a persistent grid leaves after one read per workgroup.
// SEG (r05, with PERSIST): the tiles of a seg_table; bin_start holds
// [segment][pass][256] bin starts, and each segment is sorted on its own.
// REGION_ATOM (r06; the 18-bit form's second prefix pass, XREG + SEG over
// the 8 field regions, keys only): a wave whose tile lies inside ONE field
// bin -- no bin of its region starts strictly inside the tile, checked
// against prev_starts, the field's bin starts -- ranks by LDS atomics like
// the offset-fed first pass.  Stability is only owed to the field order of
// the input, and every key of such a tile has the same field; tiles that
// straddle a field bin boundary keep the stable wave match.
#ifndef HPXHIP_REGION_ATOM
#define HPXHIP_REGION_ATOM 1
#endif
template <typename U, typename VAL, bool HAS_VAL, typename G, typename X, int THREADS = 512, int ITEMS = 16,
          int LBB = 8, int RB = 8, bool STAGE = true, bool DYN_ID = HPXHIP_TILE_DYN_ID, bool PERSIST = false,
          bool SEG = false, bool XREG = false>
__global__ __launch_bounds__(THREADS) void k_onesweep(const U* __restrict__ kin, U* __restrict__ kout,
                                                       const VAL* __restrict__ vin, VAL* __restrict__ vout,
                                                       uint64_t n, int shift,
                                                       const unsigned long long* __restrict__ bin_start,
                                                       G* __restrict__ lb, uint32_t* __restrict__ counter,
                                                       uint32_t* __restrict__ err, X xf,
                                                       const int32_t* __restrict__ ctl = nullptr, uint64_t ntiles = 0,
                                                       const uint32_t* __restrict__ pre = nullptr,
                                                       const seg_table* __restrict__ segs = nullptr,
                                                       const unsigned long long* __restrict__ prev_starts = nullptr) {
    static_assert(!PERSIST || STAGE, "the persistent form keeps the LDS-staged write-out");
    static_assert(!SEG || ((PERSIST || XREG) && LBB > 0), "segmented passes: look-back passes, persistent or XREG");
    // XREG + PERSIST (r06, SEG only): workgroups claim tiles from the region
    // counters until every region is done (the claim returns no tile); a
    // claimed tile's predecessors were claimed earlier by running workgroups,
    // so the look-back always finds them published
    static_assert(!XREG || !PERSIST || SEG, "XCD regions, persistent: the segmented (region) pass");
    static_assert(!XREG || SEG || LBB < 0, "XCD regions of equal tile ranges: the offset-fed pass (no look-back)");
    // segment table entries a workgroup loads (XREG: the 8 regions)
    constexpr int NS = XREG ? 8 : kMaxBig;
    // device-planned sort (sort.hip): *ctl = this launch's digit shift, or
    // -1 when the plan does not take this pass (every block returns at once)
    if (ctl) {
        const int32_t sh = *ctl;
        if (sh < 0) return;
        shift = sh;
        if constexpr (RB == 8) bin_start += static_cast<uint32_t>(sh >> 3) * kRadix;
    }
    constexpr int R = 1 << RB;
    constexpr uint32_t DMASK = R - 1;
    using CT = std::conditional_t<(RB > 8), uint16_t, uint32_t>;
    static_assert(THREADS >= R && THREADS % R == 0, "one thread per digit for the look-back");
    constexpr int WAVES = THREADS / kWave;
    constexpr int TILE = THREADS * ITEMS;
    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_seg;
    // SEG: the segment table, loaded once per (persistent) workgroup, so a
    // tile's segment costs LDS reads, not a chain of global loads per tile
    __shared__ uint64_t s_sg[SEG ? 3 * kMaxBig + 2 : 1];
    __shared__ alignas(16) CT s_whist[WAVES][R];
    __shared__ uint32_t s_local[R];
    __shared__ uint32_t s_wsum[R / kWave];
    __shared__ uint64_t s_adj[R];
    __shared__ U s_keys[STAGE ? TILE : 1];
    __shared__ VAL s_vals[(HAS_VAL && STAGE) ? TILE : 1];

    const int t_id = threadIdx.x;
    const int lane_ = lane_id();
    // SEG: s_sg = {start[kMaxBig], len[kMaxBig], tile0[kMaxBig + 1], nseg}
    // (the first NS segments)
    if constexpr (SEG) {
        for (int i = t_id; i <= NS; i += THREADS) {
            if (i < NS) {
                s_sg[i] = segs->start[i];
                s_sg[kMaxBig + i] = segs->len[i];
            }
            s_sg[2 * kMaxBig + i] = segs->tile0[i];
        }
        if (t_id == 0) s_sg[3 * kMaxBig + 1] = segs->nseg;
        __syncthreads();
    }
    // one tile; the persistent form calls it in a loop, the plain form once
    // (a loop around the body in the plain form changes its register
    // allocation)
    auto one = [&]() -> bool {
    int t = t_id, lane = lane_;
    // persistent form: the thread and lane ids are re-derived per tile, so
    // the compiler does not hoist every lane-dependent address of the body
    // out of the tile loop (kept live across it, those had taken the kernel
    // from 94 to 156 VGPRs: one workgroup per CU instead of two)
    if constexpr (PERSIST) asm volatile("" : "+v"(t), "+v"(lane));
    const int wave = t / kWave;
    // tile order = dispatch order (lookback.hpp); DYN_ID / PERSIST: ids from
    // the atomic counter
    if (XREG && t == 0) {
        // XREG: the tiles are cut into 8 contiguous regions, one per XCD
        // (SEG: the table's segments; else equal tile ranges); a workgroup
        // claims the next tile of its own XCD's region (counter 8 words per
        // region), so consecutive tiles -- whose digit runs end and start in
        // the same lines -- are written through one L2 (r05: the first prefix
        // pass 4.75 -> 3.81 ms at 2^30 u64, profiles/r05_ubench_sortpass5.log);
        // a region that is done sends its XCD's workgroups to the next ones
        const uint32_t x = xcc_id();
        uint32_t tl = 0xffffffffu, sg = 0;
        for (uint32_t k = 0; k < 8 && tl == 0xffffffffu; ++k) {
            const uint32_t xr = (x + k) & 7u;
            uint64_t lo, cnt;
            if constexpr (SEG) {
                if (xr >= static_cast<uint32_t>(s_sg[3 * kMaxBig + 1])) continue;
                lo = s_sg[2 * kMaxBig + xr];
                cnt = s_sg[2 * kMaxBig + xr + 1] - lo;
            } else {
                const uint64_t per = (ntiles + 7) / 8;
                lo = xr * per;
                cnt = lo < ntiles ? (ntiles - lo < per ? ntiles - lo : per) : 0;
            }
            if (cnt == 0) continue;
            const uint32_t c = __hip_atomic_fetch_add(counter + 8 * xr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c < cnt) {
                tl = static_cast<uint32_t>(lo + c);
                sg = xr;
            }
        }
        s_tile = tl;
        if constexpr (SEG) s_seg = sg;
    } else if ((DYN_ID || PERSIST) && t == 0) {
        s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (SEG && !XREG) {  // the tile's segment
            const uint32_t nseg = static_cast<uint32_t>(s_sg[3 * kMaxBig + 1]);
            uint32_t j = 0;
            while (j + 1 < nseg && s_sg[2 * kMaxBig + j + 1] <= s_tile) ++j;
            s_seg = j;
        }
    }
    for (int i = t; i < WAVES * R; i += THREADS) (&s_whist[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tile = (DYN_ID || PERSIST || XREG) ? s_tile : blockIdx.x;
    if (XREG && !SEG && tile >= ntiles) return false;
    // SEG: the tile's segment [seg_lo, end), its first tile and bin starts
    uint64_t end = n, seg_lo = 0, first_tile = 0, tile_base = tile * TILE;
    const unsigned long long* bstart = bin_start;
    if constexpr (SEG) {
        const uint32_t nseg = static_cast<uint32_t>(s_sg[3 * kMaxBig + 1]);
        if (tile >= s_sg[2 * kMaxBig + nseg]) return false;
        const uint32_t j = s_seg;
        first_tile = s_sg[2 * kMaxBig + j];
        seg_lo = s_sg[j];
        end = seg_lo + s_sg[kMaxBig + j];
        tile_base = seg_lo + (tile - first_tile) * TILE;
        bstart = bin_start + static_cast<uint64_t>(j) * (RB == 9 ? kXBins : 8 * kRadix);
    } else if (PERSIST && tile >= ntiles) {
        return false;
    }
    // where the outputs may land: the segment itself (a segmented LSD sorts
    // each segment in place), or anywhere (XREG regions are input ranges
    // whose keys go to the whole array)
    const uint64_t out_lo = (SEG && !XREG) ? seg_lo : 0, out_hi = (SEG && !XREG) ? end : n;
    const uint64_t wbase = tile_base + static_cast<uint64_t>(wave) * (TILE / WAVES);

    // ---- load: round r, lane l -> tile position wave*(TILE/WAVES) + r*64 + l
    U k[ITEMS];
    VAL v[HAS_VAL ? ITEMS : 1];
    const bool full = tile_base + TILE <= end;
#if HPXHIP_OS_UNCOND_LOAD
    // unconditional loads (a ragged tile's lanes past `end` load its last
    // element, never ranked or stored): with one load per exec-masked branch
    // the compiler waits for all of them (vmcnt(0)) before the first rank
    {
        const uint64_t last = end - 1;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t i = wbase + r * kWave + lane;
            const uint64_t j = (full || i < end) ? i : last;
            k[r] = kin[j];
            if constexpr (HAS_VAL) v[r] = vin[j];
        }
    }
#else
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < end) {
            k[r] = kin[i];
            if constexpr (HAS_VAL) v[r] = vin[i];
        } else {
            k[r] = 0;
        }
    }
#endif

    // REGION_ATOM: does the tile lie inside one bin of the previous pass's
    // field?  Lane l of every wave checks bin 64 x + l of the tile's region x
    // (its 64 field digits), one L2-resident load issued behind the tile's
    // key loads; the ballot is wave-uniform
    bool atom_rank = false;
    if constexpr (HPXHIP_REGION_ATOM && XREG && SEG && RB == 9 && !HAS_VAL && LBB > 0) {
        if (prev_starts) {
            const uint64_t bs = prev_starts[64u * s_seg + static_cast<uint32_t>(lane)];
            const uint64_t tile_hi = full ? tile_base + TILE : end;
            atom_rank = __ballot(bs > tile_base && bs < tile_hi) == 0;
        }
    }
    // ---- wave-level match ranking (stable: round-major, then lane order)
    uint32_t rank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        const bool valid = full || i < end;
        const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & DMASK;
        if (RB == 9 && atom_rank) {  // (REGION_ATOM, see above)
            if (valid) {
                const uint32_t sh = 16u * (d & 1u);
                const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(&s_whist[wave][0]) + (d >> 1), 1u << sh);
                rank[r] = (old >> sh) & 0xffffu;
            }
            continue;
        }
        if constexpr (HPXHIP_OS_ATOM1 && LBB < 0 && !HAS_VAL) {
            // the offset-fed first prefix pass of a keys-only sort (its order
            // inside a digit is never relied on: the second pass is stable
            // and the segment sort orders every bucket completely) ranks by
            // LDS atomics on the per-wave counters instead of the wave match
            if (valid) {
                if constexpr (sizeof(CT) == 2) {
                    const uint32_t sh = 16u * (d & 1u);
                    const uint32_t old =
                        atomicAdd(reinterpret_cast<uint32_t*>(&s_whist[wave][0]) + (d >> 1), 1u << sh);
                    rank[r] = (old >> sh) & 0xffffu;
                } else {
                    rank[r] = atomicAdd(reinterpret_cast<uint32_t*>(&s_whist[wave][d]), 1u);
                }
            }
            continue;
        }
        const uint64_t peers = match_digit<RB>(d, __ballot(valid));
        const uint32_t below = peers_below(peers);
        const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(peers));
        const uint32_t old = s_whist[wave][d];
        rank[r] = old + below;
        if (valid && below == 0) s_whist[wave][d] = static_cast<CT>(old + cnt);
    }
    __syncthreads();

    // ---- per-digit tile count and per-wave offsets (thread t < R owns digit t)
    uint32_t tile_count = 0;
    uint32_t count_incl = 0;
    G* my = lb + tile * R;
    if (t < R) {
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            const uint32_t c = s_whist[w][t];
            s_whist[w][t] = static_cast<CT>(tile_count);
            tile_count += c;
        }
        // publish this tile's aggregate for digit t as early as possible
        if (tile != first_tile && LBB > 0)
            __hip_atomic_store(&my[t], enc_agg<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        count_incl = wave_inclusive_scan(tile_count, op_plus{});
        if (lane == kWave - 1) s_wsum[wave] = count_incl;
    }
    __syncthreads();
    if (t < R) {
        uint32_t pre = 0;
#pragma unroll
        for (int w = 0; w < R / kWave; ++w)
            if (w < wave) pre += s_wsum[w];
        const uint32_t loc = pre + count_incl - tile_count;
        s_local[t] = loc;
        // the per-wave offsets become tile positions (< TILE fits CT), so
        // the scatter reads one LDS word per key instead of two
        if constexpr (STAGE) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) s_whist[w][t] = static_cast<CT>(s_whist[w][t] + loc);
        }
    }
    __syncthreads();

    // ---- counting sort of the tile into LDS
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (STAGE && (full || i < end)) {
            const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & DMASK;
            const uint32_t pos = s_whist[wave][d] + rank[r];
            s_keys[pos] = k[r];
            if constexpr (HAS_VAL) s_vals[pos] = v[r];
        }
    }

    // ---- per-digit look-back across tiles (thread t < R owns digit t)
    if (t < R) {
        uint64_t excl = 0;
        if (tile == first_tile) {
            if (LBB > 0) __hip_atomic_store(&my[t], enc_incl<G>(tile_count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if constexpr (LBB > 0) {
            int64_t pred = static_cast<int64_t>(tile) - 1;
            uint32_t spins = 0;
            bool done = false;
            while (!done) {
                G g[LBB];
#pragma unroll
                for (int j = 0; j < LBB; ++j)
                    g[j] = (pred - j >= static_cast<int64_t>(first_tile))
                               ? __hip_atomic_load(&lb[static_cast<uint64_t>(pred - j) * R + t],
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
                    __builtin_amdgcn_s_sleep(HPXHIP_LB_SLEEP);
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
        s_adj[t] = static_cast<uint64_t>(bstart[t]) + excl - (STAGE ? s_local[t] : 0u);
        if constexpr (LBB < 0)  // PRE: the tile's destination offsets, precomputed (k_tile_offsets)
            s_adj[t] = static_cast<uint64_t>(pre[tile * R + t]) - (STAGE ? s_local[t] : 0u);
    }
    __syncthreads();
    if constexpr (!STAGE) {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t i = wbase + r * kWave + lane;
            if (full || i < end) {
                const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & DMASK;
                const uint64_t dst = s_adj[d] + s_whist[wave][d] + rank[r];
                if (dst < out_hi && dst >= out_lo) {  // see the write-out below
                    kout[dst] = k[r];
                    if constexpr (HAS_VAL) vout[dst] = v[r];
                } else {
                    raise_device_error(err, HPXHIP_DEVERR_RANGE);
                }
            }
        }
        return false;
    }

    // ---- coalesced write of the LDS-sorted tile
    const uint32_t nvalid = full ? TILE : static_cast<uint32_t>(end - tile_base);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint32_t i = r * THREADS + t;
        if (i < nvalid) {
            const U key = s_keys[i];
            const uint32_t d = static_cast<uint32_t>(xf(key) >> shift) & DMASK;
            const uint64_t dst = s_adj[d] + i;
            // Destinations come from the histogram taken before the pass: they
            // stay below n unless the keys were changed during the sort (a
            // caller racing the sort on another stream).  Then no store leaves
            // the output buffer (it would overwrite the plan words in the
            // scratch that follows it) and the device error word reports it.
            if (dst < out_hi && dst >= out_lo) {
                kout[dst] = key;
                if constexpr (HAS_VAL) vout[dst] = s_vals[i];
            } else {
                raise_device_error(err, HPXHIP_DEVERR_RANGE);
            }
        }
    }
    return true;
    };
    if constexpr (PERSIST) {
        while (one()) __syncthreads();  // the tile's LDS readers are done before the next claim
    } else {
        one();
    }
}

// ------------------------------------------------------- hybrid (MSD) tail
// After two onesweep passes on the most significant live bits (the low
// prefix field of b2 = 8 or 9 bits at s2, then the top live byte at s1) the
// keys are ordered by a (8 + b2)-bit prefix (the 18-bit form: 9 + b2);
// every prefix value is a contiguous bucket.
constexpr int kMaxBuckets = 1 << 18;
// longest run of equal-prefix keys the segment sort orders by insertion
constexpr uint32_t kRunMax = 16;

// tmask: the top digit's mask (0xff, or 0x1ff in the 18-bit form)
template <typename U, typename X>
__device__ __forceinline__ uint32_t bucket_of(U k, int s1, int s2, int b2, X xf, uint32_t tmask = 0xffu) {
    const U u = xf(k);
    return (static_cast<uint32_t>(u >> s1) & tmask) << b2 | (static_cast<uint32_t>(u >> s2) & ((1u << b2) - 1u));
}

#ifndef HPXHIP_PAD_ABL
#define HPXHIP_PAD_ABL 0
#endif
// ---------------------------------------------- padded second pass (r06)
// The 18-bit form's second prefix pass without a look-back.  Its input is
// ordered by the field (the first pass), and what it must produce is every
// bucket -- (top 9 bits, top b2 bits of the field) -- contiguous: the order
// of the keys INSIDE a bucket is never relied on (keys only; the segment sort
// orders each bucket completely).  So each bucket gets a slot of `cap` keys
// in a padded buffer (pad[bucket * cap ...], cap >= the plan's largest
// bucket estimate + 7 sigma), and a tile claims its run of each bucket with
// one global atomic on the bucket's counter (pcnt) instead of walking back
// over its predecessors: no tile waits for another.  The look-back pass took
// 4.9-5.0 ms at 2^30 u64 against 3.8-3.9 for the offset-fed first pass
// (profiles/r06_sort_kernel_stats_u64_c.csv).  The bucket bounds are then the
// exclusive scan of the slot counts (k_pad_bounds), and the segment sort
// reads each bucket from its slot and writes it to its place in the keys.
// Tiles: as the look-back pass (XREG regions of the field, 8192 keys, one
// workgroup per tile claimed from its XCD's region, so consecutive tiles --
// which append to the same slots -- meet in one L2).  A tile's keys span a
// non-decreasing range of field parts fb; local bin = (fb - fb of the tile's
// first key) * 512 + top-9 digit for the first two fb values (block-wide LDS
// atomics, 1024 bins), and keys further on (a tile over three or more field
// parts: small or skewed field bins) claim their slot places one by one.  A
// bucket whose slot overflows raises *ovf: sort.hip then runs the look-back
// pass from the same input (left intact) instead.
// the slot counter word of bucket (top-9 digit t9, field part fb): four
// consecutive digits of one field part per 64-bit word (16-bit fields)
__device__ __forceinline__ uint32_t pad_word(uint32_t t9, uint32_t fb) { return fb * 128u + (t9 >> 2); }
template <typename U, typename X, int THREADS = 512, int ITEMS = 16>
__global__ __launch_bounds__(THREADS, 4) void k_pad_scatter(const U* __restrict__ kin, U* __restrict__ pad,
                                                          const int32_t* __restrict__ g_s1,
                                                          const int32_t* __restrict__ g_bounds,
                                                          const int32_t* __restrict__ g_cap,
                                                          const seg_table* __restrict__ segs,
                                                          uint32_t* __restrict__ counter,
                                                          unsigned long long* __restrict__ pcnt,
                                                          int32_t* __restrict__ ovf, X xf) {
    const int s1 = *g_s1;  // the top-9 digit's shift, -1: the plan does not take this pass
    if (s1 < 0) return;
    const int s2 = g_bounds[3], b2 = g_bounds[4];
    const uint32_t cap = static_cast<uint32_t>(*g_cap);
    const uint32_t bmask = (1u << b2) - 1u;
    constexpr int TILE = THREADS * ITEMS;
    constexpr int WAVES = THREADS / kWave;
    constexpr uint32_t NL = 1024;  // local bins; bin NL: keys placed one by one
    static_assert(THREADS == 512, "one thread per two local bins");
    __shared__ uint32_t s_tile, s_seg;
    __shared__ uint64_t s_sg[3 * kMaxBig + 2];
    __shared__ uint32_t s_cnt[NL + 1];
    __shared__ uint32_t s_adj[NL];
    __shared__ uint32_t s_wsum[WAVES];
    __shared__ U s_keys[TILE];
    const int t = threadIdx.x;
    const int lane = lane_id();
    const int wave = t / kWave;
    for (int i = t; i <= 8; i += THREADS) {
        if (i < 8) {
            s_sg[i] = segs->start[i];
            s_sg[kMaxBig + i] = segs->len[i];
        }
        s_sg[2 * kMaxBig + i] = segs->tile0[i];
    }
    if (t == 0) {
        s_sg[3 * kMaxBig + 1] = segs->nseg;
        // the next tile of this XCD's region (see k_onesweep XREG)
        const uint32_t x = xcc_id();
        uint32_t tl = 0xffffffffu, sg = 0;
        const uint32_t nseg = segs->nseg;
        for (uint32_t k = 0; k < 8 && tl == 0xffffffffu; ++k) {
            const uint32_t xr = (x + k) & 7u;
            if (xr >= nseg) continue;
            const uint64_t lo = segs->tile0[xr], cnt = segs->tile0[xr + 1] - lo;
            if (cnt == 0) continue;
            const uint32_t c = __hip_atomic_fetch_add(counter + 8 * xr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c < cnt) {
                tl = static_cast<uint32_t>(lo + c);
                sg = xr;
            }
        }
        s_tile = tl;
        s_seg = sg;
    }
    for (uint32_t i = t; i <= NL; i += THREADS) s_cnt[i] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile == 0xffffffffu) return;
    const uint32_t j = s_seg;
    const uint64_t seg_lo = s_sg[j], end = seg_lo + s_sg[kMaxBig + j];
    const uint64_t tile_base = seg_lo + (tile - s_sg[2 * kMaxBig + j]) * TILE;
    const bool full = tile_base + TILE <= end;
    const uint64_t wbase = tile_base + static_cast<uint64_t>(wave) * (TILE / WAVES);
    const uint32_t fb0 = static_cast<uint32_t>(xf(kin[tile_base]) >> s2) & bmask;
    auto local_bin = [&](const U& key) {
        const U u = xf(key);
        const uint32_t rel = (static_cast<uint32_t>(u >> s2) & bmask) - fb0;
        return rel < 2u ? rel * 512u + (static_cast<uint32_t>(u >> s1) & 511u) : NL;
    };
    U k[ITEMS];
    {
        const uint64_t last = end - 1;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t i = wbase + r * kWave + lane;
            k[r] = kin[(full || i < end) ? i : last];
        }
    }
    // ranks inside the local bins (LDS atomics: no order is owed inside a bucket)
    uint32_t rank[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < end) rank[r] = atomicAdd(&s_cnt[local_bin(k[r])], 1u);
    }
    __syncthreads();
    // local starts (thread t < 256: bins 4t .. 4t + 3, four top-9 digits of
    // one field part; the one-by-one bin last) and each bin's run of its
    // bucket's slot.  r06: the slot counters are 16-bit fields, four buckets
    // (four top-9 digits of one field part) per 64-bit word, so one atomic
    // claims four runs: 128 atomics per tile instead of 512 (the counters'
    // atomics were 27 % extra write traffic, profiles/r06_pmc_sort_e.txt).  A
    // field can only carry into its neighbour past 65535 keys, long after
    // its slot (<= 4608) overflowed and raised *ovf.
    {
        uint32_t c[4] = {0, 0, 0, 0};
        if (t < 256) {
#pragma unroll
            for (int h = 0; h < 4; ++h) c[h] = s_cnt[4 * t + h];
        }
        const uint32_t sum = c[0] + c[1] + c[2] + c[3];
        const uint32_t incl = wave_inclusive_scan(sum, op_plus{});
        if (lane == kWave - 1) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = incl - sum;
#pragma unroll
        for (int w = 0; w < WAVES; ++w)
            if (w < wave) pre += s_wsum[w];
        if (t < 256) {
            const uint32_t t9 = (4u * t) & 511u, fb = fb0 + ((4u * t) >> 9);
            uint64_t old = 0;
            if (sum) {
                const uint64_t add = static_cast<uint64_t>(c[0]) | static_cast<uint64_t>(c[1]) << 16 |
                                     static_cast<uint64_t>(c[2]) << 32 | static_cast<uint64_t>(c[3]) << 48;
                old = __hip_atomic_fetch_add(&pcnt[pad_word(t9, fb)], add, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            }
            uint32_t ls = pre;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t lb = 4 * t + h;
                if (c[h]) {
                    const uint32_t base = static_cast<uint32_t>(old >> (16 * h)) & 0xffffu;
                    const uint32_t bucket = ((t9 + h) << b2) | fb;
                    if (base + c[h] <= cap) {
                        s_adj[lb] = bucket * cap + base - ls;  // mod 2^32: pad index of local position ls
                    } else {
                        s_adj[lb] = 0xffffffffu;
                        __hip_atomic_store(ovf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                s_cnt[lb] = ls;
                ls += c[h];
            }
            if (t == 255) s_cnt[NL] = ls;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = wbase + r * kWave + lane;
        if (full || i < end) s_keys[s_cnt[local_bin(k[r])] + rank[r]] = k[r];
    }
    __syncthreads();
    const uint32_t nvalid = full ? TILE : static_cast<uint32_t>(end - tile_base);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint32_t i = r * THREADS + t;
        if (i < nvalid) {
            const U key = s_keys[i];
            const uint32_t lb = local_bin(key);
            if (lb < NL) {
                const uint32_t a = s_adj[lb];
                if (a != 0xffffffffu) pad[a + i] = key;
            } else {
                const U u = xf(key);
                const uint32_t bucket = ((static_cast<uint32_t>(u >> s1) & 511u) << b2) |
                                        (static_cast<uint32_t>(u >> s2) & bmask);
                const uint32_t t9 = static_cast<uint32_t>(u >> s1) & 511u;
                const uint64_t old = __hip_atomic_fetch_add(&pcnt[pad_word(t9, static_cast<uint32_t>(u >> s2) & bmask)],
                                                            uint64_t(1) << (16 * (t9 & 3u)), __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t base = static_cast<uint32_t>(old >> (16 * (t9 & 3u))) & 0xffffu;
                if (base < cap) pad[bucket * cap + base] = key;
                else __hip_atomic_store(ovf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// off[v] = sum of the slot counts of buckets < v (v = 0..nb): the bucket
// bounds of the padded pass, in two launches over blocks of 1024 buckets
// (k_pad_sums: each block's total into bsum; k_pad_bounds: each block adds
// the totals before it and scans its own); run iff *g_cap > 0 (the padded
// pass ran and no slot overflowed).  g_bounds = {on, nb, ...}; nb is a power
// of two >= 1024.  (A one-workgroup scan walking 256 buckets per thread took
// 0.21 ms, profiles/r06_sort_kernel_stats_u64_d.csv.)
__device__ __forceinline__ uint32_t pad_count(const unsigned long long* pcnt, uint32_t bucket, int b2) {
    const uint32_t t9 = bucket >> b2, fb = bucket & ((1u << b2) - 1u);
    return static_cast<uint32_t>(pcnt[pad_word(t9, fb)] >> (16 * (t9 & 3u))) & 0xffffu;
}
__global__ __launch_bounds__(256) void k_pad_sums(const unsigned long long* __restrict__ pcnt,
                                                   const int32_t* __restrict__ g_bounds,
                                                   const int32_t* __restrict__ g_cap, uint64_t* __restrict__ bsum) {
    if (*g_cap <= 0) return;
    const uint32_t nb = static_cast<uint32_t>(g_bounds[1]);
    const int b2 = g_bounds[4];
    if (blockIdx.x * 1024u >= nb) return;
    __shared__ uint64_t s_w[4];
    const uint32_t v = blockIdx.x * 1024u + 4u * threadIdx.x;
    uint64_t x = 0;
#pragma unroll
    for (int h = 0; h < 4; ++h) x += pad_count(pcnt, v + h, b2);
    x = wave_reduce(x, op_plus{});
    if (lane_id() == 0) s_w[threadIdx.x / kWave] = x;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}
__global__ __launch_bounds__(256) void k_pad_bounds(const unsigned long long* __restrict__ pcnt,
                                                     const int32_t* __restrict__ g_bounds,
                                                     const int32_t* __restrict__ g_cap,
                                                     const uint64_t* __restrict__ bsum, uint64_t* __restrict__ off) {
    if (*g_cap <= 0) return;
    const uint32_t nb = static_cast<uint32_t>(g_bounds[1]);
    const int b2 = g_bounds[4];
    const uint32_t b = blockIdx.x;
    if (b * 1024u >= nb) return;
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    __shared__ uint64_t s_w[4];
    __shared__ uint64_t s_base;
    if (wave == 0) {  // the totals of the blocks before this one (<= 256: four per lane)
        uint64_t x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t j = static_cast<uint32_t>(lane) * 4u + i;
            if (j < b) x += bsum[j];
        }
        x = wave_reduce(x, op_plus{});
        if (lane == 0) s_base = x;
    }
    const uint32_t v = b * 1024u + 4u * t;
    uint32_t c[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) c[h] = pad_count(pcnt, v + h, b2);
    const uint64_t sum = static_cast<uint64_t>(c[0]) + c[1] + c[2] + c[3];
    const uint64_t incl = wave_inclusive_scan(sum, op_plus{});
    if (lane == kWave - 1) s_w[wave] = incl;
    __syncthreads();
    uint64_t run = s_base + incl - sum;
#pragma unroll
    for (int w = 0; w < 4; ++w)
        if (w < wave) run += s_w[w];
    using V2 = vec<uint64_t, 2>;
    reinterpret_cast<V2*>(off + v)[0] = V2{{run, run + c[0]}};
    reinterpret_cast<V2*>(off + v)[1] = V2{{run + c[0] + c[1], run + c[0] + c[1] + c[2]}};
    if (v + 4 == nb) off[nb] = run + sum;
}

// off[v] = first index whose prefix is >= v (v = 0..nb): a lower_bound per
// bucket over the prefix-ordered keys instead of a pass over all of them.
// ctl (device-planned sort): {on, nb, s1, s2, b2} read on the device.
template <typename U, typename X>
__global__ __launch_bounds__(256) void k_bucket_bounds(const U* __restrict__ keys, uint64_t n, int s1, int s2, int b2,
                                                        uint32_t nb, X xf, uint64_t* __restrict__ off,
                                                        const int32_t* __restrict__ ctl = nullptr) {
    if (ctl) {
        if (!ctl[0]) return;
        nb = static_cast<uint32_t>(ctl[1]);
        s1 = ctl[2];
        s2 = ctl[3];
        b2 = ctl[4];
    }
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v > nb) return;
    // nb = 2^(top digit bits + b2): the top digit is 8 or 9 bits wide
    const uint32_t tmask = (1u << (__builtin_ctz(nb) - b2)) - 1u;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (bucket_of(keys[mid], s1, s2, b2, xf, tmask) < v) lo = mid + 1;
        else hi = mid;
    }
    off[v] = lo;
}

// --------------------------------------------------------- segment sort
// One workgroup sorts one segment (a run of whole buckets, at most
// THREADS*ITEMS keys) completely in LDS and writes it back in place.  The
// segment's keys agree on every bit at or above `top` (the highest bit in
// which its first and last keys differ, or -- one bucket -- the top of the
// next live digit).  Below it:
//   1. two stable LDS passes (the onesweep's wave match ranking, per-wave
//      16-bit counters) on the 16 bits under `top`: the keys are then in
//      order up to runs that agree on all those bits (for 2^30 random keys a
//      16384-key bucket has runs of 1.1 keys on average, rarely over 5);
//   2. (r03) each run of keys equal on those bits is sorted by insertion by
//      the thread that finds its first key (one detection sweep); a segment
//      with a run longer than kRunMax goes on to
//   3. odd-even transposition of neighbours by whole keys until a round
//      swaps nothing -- an inversion can only sit inside one run, so the
//      rounds needed are the longest run's length (round 2 ran these for
//      every segment: 2 x (longest run + 1) LDS sweeps);
//   4. a segment whose runs do not settle within OE_MAX rounds (skewed low
//      bits) is finished by stable LSD passes over every bit under `top`.
// Six 8-bit LDS passes for the 48 bits under a 16-bit prefix took 2.4 ms
// each at 2^30 keys (VALU-bound ranking); this form replaces four of them.
// HAS_VAL (sort_by_key): the values travel with their keys through the same
// LDS passes and swaps (stable: the LDS passes rank in index order and the
// odd-even rounds swap only strictly greater keys), staged in s_vals.
// BOUNDS: `seg` is the bucket-bounds array itself (segment = one bucket,
// [seg[b], seg[b + 1])), as the host uses when buckets average at least half
// a segment: no bounds read-back and no host packing between the prefix
// passes and this kernel.  A bucket too large for the LDS is left alone,
// raises *oversized and records its id in `big` (sort.hip finishes up to
// kMaxBig of them by a segmented LSD over just their ranges).
// PERSIST (device-planned sort, BOUNDS only): a fixed grid strides over the
// planned buckets (bucket b by workgroup b mod gridDim), so a launch the plan
// skips costs one gate read per workgroup instead of one dispatch per bucket.
// ONEB (r06, keys only): the one-pass form.  One ranking pass by LDS atomics
// on 2^ONEB block-wide bins (packed 16-bit counters) of the ONEB bits under
// `top`, one scan of the bins, one scatter; then every key of a bin holding
// more than one key finds its place inside the bin by counting the bin's
// keys below it (ties broken by the scatter position), all keys in parallel,
// and moves there.  For 2^30 random u64 keys (~4096-key buckets, ONEB = 13)
// a key's bin holds 1.5 keys on average.  Replaces the two ranked 8-bit
// passes, whose second (stable, wave-match) pass left the kernel
// compute-bound: with one LDS pass the segment sort had run as fast as a bare
// load + store through LDS (profiles/r05_ubench_seg5_phases.log, ABL2 vs
// ABL4).  The r05 one-pass attempt (seg10) ordered the bins by serial
// insertion, one thread per bin, and lost.  A segment with a bin over
// kOneBinMax keys (low-entropy keys) takes the two-pass path below from the
// same registers.
constexpr uint32_t kOneBinMax = 24;
#ifndef HPXHIP_SEG_ONE
#define HPXHIP_SEG_ONE 13
#endif
template <typename U, typename X, int THREADS = 1024, int ITEMS = 18, int OE_MAX = 16, typename VAL = uint32_t,
          bool HAS_VAL = false, bool BOUNDS = false, bool PERSIST = false, int MINW = 4, bool PRE16 = false,
          int ONEB = 0>
__global__ __launch_bounds__(THREADS, MINW)  // 4 waves per SIMD: one 1024- or two 512-thread blocks per CU
    void k_bucket_sort(U* __restrict__ keys, const uint64_t* __restrict__ seg, int top_single, X xf,
                       VAL* __restrict__ vals = nullptr, uint32_t* __restrict__ oversized = nullptr,
                       const int32_t* __restrict__ ctl = nullptr, uint32_t first_bucket = 0,
                       uint32_t* __restrict__ big = nullptr, uint32_t* __restrict__ redo_n = nullptr,
                       uint32_t* __restrict__ redo_ids = nullptr, const U* __restrict__ pad = nullptr,
                       const int32_t* __restrict__ pad_cap = nullptr) {
    static_assert(!PERSIST || BOUNDS, "the persistent form strides over bucket bounds");
    static_assert(ONEB == 0 || (!HAS_VAL && BOUNDS && ONEB >= 9 && ONEB <= 14), "one-pass form: keys, bucket bounds");
    // device-planned sort: ctl = {on, buckets, top_single}; the grid covers
    // the largest bucket count (or strides over it), blocks past the planned
    // count return
    uint32_t nbk = PERSIST ? first_bucket + gridDim.x : first_bucket + blockIdx.x + 1;
    if (ctl) {
        if (!ctl[0]) return;
        nbk = static_cast<uint32_t>(ctl[1]);
        top_single = ctl[2];
    }
    // the two-pass form over the buckets a one-pass launch handed on
    // (redo_ids[0, *redo_n)); the one-pass form appends to that list
    const bool listed = ONEB == 0 && PERSIST && redo_ids != nullptr;
    if (listed) nbk = *redo_n;
    constexpr int WAVES = THREADS / kWave;
    constexpr int CHUNK = ITEMS * kWave;
    constexpr int BITS = static_cast<int>(sizeof(U) * 8);
    static_assert(THREADS * ITEMS < 65536, "16-bit LDS counters");
    static_assert(THREADS >= kRadix, "one thread per digit in the offset scan");
    __shared__ alignas(16) U s_keys[THREADS * ITEMS];
    __shared__ alignas(16) VAL s_vals[HAS_VAL ? THREADS * ITEMS : 1];
    // the per-wave 16-bit digit counters of the two-pass form; the one-pass
    // form's 2^ONEB bins share their LDS (the larger of the two)
    constexpr int kWhistWords = WAVES * kRadix / 2;
    constexpr int kOneWords = ONEB > 0 ? (1 << (ONEB > 0 ? ONEB - 1 : 0)) : 0;
    constexpr int kAuxWords = kOneWords > kWhistWords ? kOneWords : kWhistWords;
    __shared__ alignas(16) uint32_t s_aux[kAuxWords];
    uint16_t (*s_whist)[kRadix] = reinterpret_cast<uint16_t (*)[kRadix]>(s_aux);
    __shared__ uint32_t s_wsum[(kRadix / kWave) > WAVES ? kRadix / kWave : WAVES];
    __shared__ U s_ends[2];
    // PRE16 (r05): the second LDS pass also leaves each key's 16 sorted bits
    // here, so the run detection reads 8 prefixes per 16-B LDS load instead
    // of three 8-B keys per position
    __shared__ alignas(16) uint16_t s_pre[PRE16 ? THREADS * ITEMS + 16 : 1];

    const int t_id = threadIdx.x;
    const int lane_ = lane_id();
    const int top_planned = top_single;
    // one bucket (segment) bk; the persistent form calls it in a loop, the
    // plain form once -- a loop around the body in the plain form cost the
    // compiler 19 spilled VGPRs
    auto one = [&](uint32_t bk) {
    int t = t_id, lane = lane_;
    // as in k_onesweep: ids re-derived per bucket in the persistent form
    if constexpr (PERSIST) asm volatile("" : "+v"(t), "+v"(lane));
    const int wave = t / kWave;
    uint64_t b, mm;
    if constexpr (BOUNDS) {
        b = seg[bk];
        mm = seg[bk + 1] - b;
        if (mm > static_cast<uint64_t>(THREADS) * ITEMS) {
            if (t == 0) {
                __hip_atomic_store(oversized, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // r05: the bucket's id, for the planner's bounded finish
                // (big[0] counts them; ids past kMaxBig are not kept)
                if (big) {
                    const uint32_t slot = __hip_atomic_fetch_add(big, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (slot < static_cast<uint32_t>(kMaxBig)) big[1 + slot] = bk;
                }
            }
            return;
        }
    } else {
        b = seg[2 * bk];  // (begin, end) pairs
        mm = seg[2 * bk + 1] - b;
    }
    const uint32_t m = static_cast<uint32_t>(mm);
    if (m < 2) return;

    const uint32_t wbase = static_cast<uint32_t>(wave) * CHUNK;
    const uint32_t have = m > wbase ? m - wbase : 0u;
    const int nfull = static_cast<int>(have >= static_cast<uint32_t>(CHUNK) ? ITEMS : have / kWave);
    const uint64_t tail_mask = (have % kWave) ? (~0ull >> (kWave - have % kWave)) : 0ull;
    auto active = [&](int r) -> uint64_t { return r < nfull ? ~0ull : (r == nfull ? tail_mask : 0ull); };
    U* gkeys = keys + b;
    // r06: a bucket of the padded second pass is read from its slot
    // (k_pad_scatter) and written to its place in the keys
    const U* gsrc = gkeys;
    if (!HAS_VAL && BOUNDS && pad) {
        const int32_t pc = *pad_cap;
        if (pc > 0) gsrc = pad + static_cast<uint64_t>(bk) * static_cast<uint32_t>(pc);
    }
    U* lkeys = s_keys + wbase;
    VAL* gvals = HAS_VAL ? vals + b : nullptr;
    VAL* lvals = s_vals + (HAS_VAL ? wbase : 0);

    U k[ITEMS];
    VAL v[HAS_VAL ? ITEMS : 1];
#if HPXHIP_SEG_UNCOND_LOAD
    // unconditional loads, as k_onesweep's (lanes past the segment load its
    // last key; every pass below gates them out by active())
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool on = (active(r) >> lane) & 1u;
        const uint32_t j = on ? wbase + r * kWave + lane : m - 1;
        k[r] = ld_stream(&gsrc[j]);
        if constexpr (HAS_VAL) v[r] = ld_stream(&gvals[j]);
    }
#else
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool on = (active(r) >> lane) & 1u;
        k[r] = on ? ld_stream(&gsrc[wbase + r * kWave + lane]) : U(0);
        if constexpr (HAS_VAL) v[r] = on ? ld_stream(&gvals[wbase + r * kWave + lane]) : VAL(0);
    }
#endif
    // The segment's first and last keys (their highest differing bit is the
    // top of the LDS passes) come from the registers just loaded, through
    // LDS: reading them from global memory first had put one more dependent
    // round trip in front of every segment's loads.
    {
        const uint32_t last = m - 1;
        const uint32_t lw = last / CHUNK, lo = last % CHUNK;
        if (t == 0) s_ends[0] = k[0];
        if (static_cast<uint32_t>(wave) == lw && static_cast<uint32_t>(lane) == lo % kWave) {
            U x = k[0];
#pragma unroll
            for (int r = 1; r < ITEMS; ++r)
                if (static_cast<uint32_t>(r) == lo / kWave) x = k[r];
            s_ends[1] = x;
        }
        __syncthreads();
    }
    const U diff = xf(s_ends[0]) ^ xf(s_ends[1]);
    int top = top_planned;
    if (diff) {
        const int hb = BITS - (sizeof(U) == 8 ? __builtin_clzll(static_cast<uint64_t>(diff))
                                               : __builtin_clz(static_cast<uint32_t>(diff)));
        top = hb > top ? hb : top;
    }
    if (top <= 0) return;  // all keys equal

    // ---- the one-pass form (ONEB, see above)
    if constexpr (ONEB > 0) {
        constexpr uint32_t NB = 1u << ONEB;
        constexpr int WPT = static_cast<int>(NB / 2) / THREADS;  // packed counter words per thread
        static_assert(WPT >= 4 && WPT % 4 == 0 && WPT * THREADS * 2 == static_cast<int>(NB), "bins per thread");
        using W4 = vec<uint32_t, 4>;
        const int sh0 = top > ONEB ? top - ONEB : 0;
        auto digit = [&](const U& x) { return static_cast<uint32_t>(xf(x) >> sh0) & (NB - 1u); };
        auto bin_off = [&](uint32_t d) { return (s_aux[d >> 1] >> (16u * (d & 1u))) & 0xffffu; };
#pragma unroll
        for (int j = 0; j < WPT / 4; ++j) reinterpret_cast<W4*>(s_aux)[j * THREADS + t] = W4{{0u, 0u, 0u, 0u}};
        __syncthreads();
        // ranks inside the bins (LDS atomics; the order inside a bin is
        // settled by the in-bin ranking below), two 16-bit ranks per register
        uint32_t slot[(ITEMS + 1) / 2];
#pragma unroll
        for (int r = 0; r < (ITEMS + 1) / 2; ++r) slot[r] = 0;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = active(r);
            if (act == 0) break;  // uniform
            if ((act >> lane) & 1u) {
                const uint32_t d = digit(k[r]);
                const uint32_t sh = 16u * (d & 1u);
                const uint32_t old = atomicAdd(&s_aux[d >> 1], 1u << sh);
                slot[r / 2] |= ((old >> sh) & 0xffffu) << (16 * (r & 1));
            }
        }
        __syncthreads();
        // exclusive scan of the bins: thread t owns bins [2 WPT t, 2 WPT (t + 1))
        uint32_t w[WPT];
#pragma unroll
        for (int j = 0; j < WPT / 4; ++j) {
            const W4 q = reinterpret_cast<const W4*>(s_aux)[t * (WPT / 4) + j];
#pragma unroll
            for (int i = 0; i < 4; ++i) w[4 * j + i] = q.v[i];
        }
        uint32_t sum = 0, mx = 0;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const uint32_t lo = w[j] & 0xffffu, hi = w[j] >> 16;
            sum += lo + hi;
            mx = lo > mx ? lo : mx;
            mx = hi > mx ? hi : mx;
        }
        const uint32_t incl = wave_inclusive_scan(sum, op_plus{});
        if (lane == kWave - 1) s_wsum[wave] = incl;
        if (__syncthreads_or(mx > kOneBinMax)) {
            // a bin too large for the in-bin ranking: the bucket goes to the
            // two-pass launch that follows (its keys are still in place)
            if (t == 0) redo_ids[atomicAdd(redo_n, 1u)] = bk;
            return;
        }
        {
            uint32_t run = incl - sum;
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww)
                if (ww < wave) run += s_wsum[ww];
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const uint32_t lo = w[j] & 0xffffu, hi = w[j] >> 16;
                w[j] = run | ((run + lo) << 16);  // offsets <= m < 2^16
                run += lo + hi;
            }
#pragma unroll
            for (int j = 0; j < WPT / 4; ++j)
                reinterpret_cast<W4*>(s_aux)[t * (WPT / 4) + j] = W4{{w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]}};
            __syncthreads();
            // scatter into the bins; slot: rank -> position
#pragma unroll
            for (int r = 0; r < ITEMS; ++r) {
                const uint64_t act = active(r);
                if (act == 0) break;
                if ((act >> lane) & 1u) {
                    const uint32_t pos = bin_off(digit(k[r])) + ((slot[r / 2] >> (16 * (r & 1))) & 0xffffu);
                    s_keys[pos] = k[r];
                    slot[r / 2] = (slot[r / 2] & (0xffff0000u >> (16 * (r & 1)))) | (pos << (16 * (r & 1)));
                }
            }
            __syncthreads();
            // a bin's keys agree on every bit at or above sh0; with sh0 = 0
            // they are equal and the scatter is the sorted order
            if (sh0 > 0) {
#pragma unroll
                for (int r = 0; r < ITEMS; ++r) {
                    const uint64_t act = active(r);
                    if (act == 0) break;
                    if ((act >> lane) & 1u) {
                        const uint32_t d = digit(k[r]);
                        const uint32_t s = bin_off(d), e = d + 1 < NB ? bin_off(d + 1) : m;
                        if (e - s > 1) {
                            const uint32_t pos = (slot[r / 2] >> (16 * (r & 1))) & 0xffffu;
                            const U xk = xf(k[r]);
                            uint32_t c = 0;
                            for (uint32_t j = s; j < e; ++j) {
                                const U y = xf(s_keys[j]);
                                c += (y < xk || (y == xk && j < pos)) ? 1u : 0u;
                            }
                            slot[r / 2] = (slot[r / 2] & (0xffff0000u >> (16 * (r & 1)))) | ((s + c) << (16 * (r & 1)));
                        }
                    }
                }
                __syncthreads();  // every bin read before any key moves
#pragma unroll
                for (int r = 0; r < ITEMS; ++r) {
                    const uint64_t act = active(r);
                    if (act == 0) break;
                    if ((act >> lane) & 1u) s_keys[(slot[r / 2] >> (16 * (r & 1))) & 0xffffu] = k[r];
                }
                __syncthreads();
            }
        }
    }

    // one stable pass on the digit at `shift`: registers -> s_keys (ranked).
    // atom (HPXHIP_SEG_ATOM1, keys only): the first pass under `top` ranks by
    // LDS atomics on the packed 16-bit per-wave counters instead of the
    // wave match -- its order inside a digit is arbitrary, which the second
    // (stable) pass and the insertion inside runs never depend on
    auto pass = [&](int shift, bool keep_pre, bool atom) {
        __syncthreads();  // earlier readers of s_keys / s_whist are done
        for (int i = t; i < WAVES * kRadix / 2; i += THREADS) reinterpret_cast<uint32_t*>(&s_whist[0][0])[i] = 0;
        __syncthreads();
        // ranks (< 2^16, static_assert above) packed two per register: the
        // kernel sits at the 128-VGPR bound of two workgroups per CU
        uint32_t rank2[(ITEMS + 1) / 2];
#pragma unroll
        for (int r = 0; r < (ITEMS + 1) / 2; ++r) rank2[r] = 0;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = active(r);
            if (act == 0) break;  // uniform
            const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
            if (HPXHIP_SEG_ATOM1 && !HAS_VAL && atom) {
                if ((act >> lane) & 1u) {
                    const uint32_t sh = 16u * (d & 1u);
                    const uint32_t old =
                        atomicAdd(reinterpret_cast<uint32_t*>(&s_whist[wave][0]) + (d >> 1), 1u << sh);
                    rank2[r / 2] |= ((old >> sh) & 0xffffu) << (16 * (r & 1));
                }
                continue;
            }
            const uint64_t peers = match_digit(d, act);
            const uint32_t below = peers_below(peers);
            const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(peers));
            const uint32_t old = s_whist[wave][d];
            rank2[r / 2] |= (old + below) << (16 * (r & 1));
            if (((act >> lane) & 1u) && below == 0) s_whist[wave][d] = static_cast<uint16_t>(old + cnt);
        }
        __syncthreads();
        uint32_t count = 0, incl = 0;
        if (t < kRadix) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const uint32_t c = s_whist[w][t];
                s_whist[w][t] = static_cast<uint16_t>(count);
                count += c;
            }
            incl = wave_inclusive_scan(count, op_plus{});
            if (lane == kWave - 1) s_wsum[wave] = incl;
        }
        __syncthreads();
        if (t < kRadix) {
            uint32_t pre = 0;
#pragma unroll
            for (int w = 0; w < kRadix / kWave; ++w)
                if (w < wave) pre += s_wsum[w];
            // per-wave offsets -> segment positions (< 2^16): one LDS word
            // per key in the scatter instead of two
            const uint32_t loc = pre + incl - count;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) s_whist[w][t] = static_cast<uint16_t>(s_whist[w][t] + loc);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = active(r);
            if (act == 0) break;
            if ((act >> lane) & 1u) {
                const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
                const uint32_t pos = s_whist[wave][d] + ((rank2[r / 2] >> (16 * (r & 1))) & 0xffffu);
                s_keys[pos] = k[r];
                if constexpr (HAS_VAL) s_vals[pos] = v[r];
                if constexpr (PRE16)
                    if (keep_pre) s_pre[pos] = static_cast<uint16_t>(xf(k[r]) >> (top - 16));
            }
        }
        __syncthreads();
    };
    auto reload = [&] {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const bool on = (active(r) >> lane) & 1u;
            k[r] = on ? lkeys[r * kWave + lane] : U(0);
            if constexpr (HAS_VAL) v[r] = on ? lvals[r * kWave + lane] : VAL(0);
        }
    };

    // pass schedule (one inlined copy of `pass`): the two passes under
    // `top`, then -- only for a segment the odd-even rounds do not settle --
    // the full LSD over every bit under `top`
    bool lsd = false;
    int npass = 2;
    for (int q = 0; ONEB == 0 && q < npass;) {
        const int lo = lsd ? top - 8 * (npass - q) : top - 8 * (2 - q);
        pass(lo > 0 ? lo : 0, !lsd && q == 1 && top > 16, !lsd && q == 0);
        if (++q < npass) {
            reload();
            continue;
        }
        if (lsd || top <= 16 || OE_MAX < 0) break;  // OE_MAX < 0: ablation (two passes only)
        // Runs of keys equal on the passes' bits (and above) are sorted in
        // place by the thread that finds the run's start, by insertion
        // (stable: strictly greater keys move).  One detection sweep and one
        // sort step replace the odd-even rounds' 2 x (longest run + 1)
        // sweeps; a run longer than RUN_MAX sends the segment on to the
        // odd-even rounds below.
        {
            const int fs = top - 16;
            auto pre = [&](const U& x) { return xf(x) >> fs; };
            uint32_t starts = 0;
            constexpr int kGroups = (THREADS * ITEMS / 8 + THREADS - 1) / THREADS;  // PRE16: 8 positions per group
            static_assert(!PRE16 || 8 * kGroups <= 32, "run starts: one bit per position");
            if constexpr (PRE16) {
                using P8 = vec<uint16_t, 8>;
#pragma unroll
                for (int j = 0; j < kGroups; ++j) {
                    const uint32_t g = static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                    const uint32_t base = 8 * g;
                    if (base + 1 >= m) continue;
                    const P8 w = reinterpret_cast<const P8*>(s_pre)[g];
                    const uint16_t before = base > 0 ? s_pre[base - 1] : uint16_t(0);
                    const uint16_t after = s_pre[base + 8];  // read only if base + 8 < m
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t idx = base + i;
                        const uint16_t a = w.v[i];
                        const uint16_t nx = i < 7 ? w.v[i < 7 ? i + 1 : 7] : after;
                        const uint16_t pv = i > 0 ? w.v[i > 0 ? i - 1 : 0] : before;
                        if (idx + 1 < m && a == nx && (idx == 0 || pv != a)) starts |= 1u << (8 * j + i);
                    }
                }
                // no barrier: the insertion below moves keys (s_keys), and
                // the detection reads prefixes only (s_pre, equal along a run)
            } else {
#pragma unroll 3
                for (int j = 0; j < ITEMS; ++j) {
                    const uint32_t i = static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                    if (i + 1 < m) {
                        const U a = pre(s_keys[i]);
                        if (a == pre(s_keys[i + 1]) && (i == 0 || pre(s_keys[i - 1]) != a)) starts |= 1u << j;
                    }
                }
                __syncthreads();  // detection reads done before any run moves
            }
            int long_run = 0;
            while (starts) {
                const int j = __builtin_ctz(starts);
                starts &= starts - 1;
                const uint32_t s = PRE16 ? 8 * (static_cast<uint32_t>(t) + static_cast<uint32_t>(j / 8) * THREADS) + j % 8
                                         : static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                uint32_t e = s + 2;  // the detection saw s + 1 in the run
                if constexpr (PRE16) {
                    const uint16_t p0 = s_pre[s];
                    while (e < m && e - s <= kRunMax && s_pre[e] == p0) ++e;
                } else {
                    const U p0 = pre(s_keys[s]);
                    while (e < m && e - s <= kRunMax && pre(s_keys[e]) == p0) ++e;
                }
                if (e - s > kRunMax) {
                    long_run = 1;
                    continue;
                }
                for (uint32_t p = s + 1; p < e; ++p) {
                    const U x = s_keys[p];
                    uint32_t q = p;
                    while (q > s && xf(s_keys[q - 1]) > xf(x)) --q;
                    if (q == p) continue;
                    VAL y{};
                    if constexpr (HAS_VAL) y = s_vals[p];
                    for (uint32_t r = p; r > q; --r) {
                        s_keys[r] = s_keys[r - 1];
                        if constexpr (HAS_VAL) s_vals[r] = s_vals[r - 1];
                    }
                    s_keys[q] = x;
                    if constexpr (HAS_VAL) s_vals[q] = y;
                }
            }
            if (!__syncthreads_or(long_run)) break;
        }
        bool settled = false;
        for (int it = 0; it < OE_MAX && !settled; ++it) {
            int swapped = 0;
            using V2 = vec<U, 2>;
            for (uint32_t i = t; 2 * i + 1 < m; i += THREADS) {  // pairs (2i, 2i+1): one 16-B LDS access
                V2 p = reinterpret_cast<V2*>(s_keys)[i];
                if (xf(p.v[0]) > xf(p.v[1])) {
                    const U x = p.v[0];
                    p.v[0] = p.v[1];
                    p.v[1] = x;
                    reinterpret_cast<V2*>(s_keys)[i] = p;
                    if constexpr (HAS_VAL) {
                        const VAL y = s_vals[2 * i];
                        s_vals[2 * i] = s_vals[2 * i + 1];
                        s_vals[2 * i + 1] = y;
                    }
                    swapped = 1;
                }
            }
            __syncthreads();
            for (uint32_t i = t; 2 * i + 2 < m; i += THREADS) {  // pairs (2i+1, 2i+2)
                const U a = s_keys[2 * i + 1], c = s_keys[2 * i + 2];
                if (xf(a) > xf(c)) {
                    s_keys[2 * i + 1] = c;
                    s_keys[2 * i + 2] = a;
                    if constexpr (HAS_VAL) {
                        const VAL y = s_vals[2 * i + 1];
                        s_vals[2 * i + 1] = s_vals[2 * i + 2];
                        s_vals[2 * i + 2] = y;
                    }
                    swapped = 1;
                }
            }
            settled = !__syncthreads_or(swapped);
        }
        if (settled) break;
        // stable LSD over every bit under `top`, from the keys as the rounds left them
        lsd = true;
        npass = (top + 7) / 8;
        q = 0;
        __syncthreads();
        reload();
    }
    // Write-back with the lanes aligned to 64-B lines of the output (a
    // bucket starts anywhere): each wave store then covers whole lines, not
    // 9 part-lines per 512 B (WRITE_SIZE 1.067x -> 1.053x the keys).  Same-box
    // A/B (profiles/r02_sort_writeback_ab.log): sort_by_key u64/u64 2^28
    // 8.80 -> 8.56-8.67 ms; keys-only sorts neutral to 0.5 % slower, so they
    // keep the plain loop.
    const uint32_t klead =
        HAS_VAL ? static_cast<uint32_t>(reinterpret_cast<uintptr_t>(gkeys) % 64) / sizeof(U) : 0u;
    for (uint32_t i = t; i < m + klead; i += THREADS)
        if (i >= klead) st_stream(&gkeys[i - klead], s_keys[i - klead]);
    if constexpr (HAS_VAL) {
        const uint32_t vlead = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(gvals) % 64) / sizeof(VAL);
        for (uint32_t i = t; i < m + vlead; i += THREADS)
            if (i >= vlead) st_stream(&gvals[i - vlead], s_vals[i - vlead]);
    }
    };
    // first_bucket: a launch may cover the buckets from there on (a plain
    // launch sized for the typical plan, then a striding one for the rest)
    if constexpr (PERSIST) {
        for (uint32_t bk = first_bucket + blockIdx.x; bk < nbk; bk += gridDim.x) {
            one(listed ? redo_ids[bk] : bk);
            __syncthreads();  // s_keys / s_vals read out before the next bucket's passes
        }
    } else if (first_bucket + blockIdx.x < nbk) {
        one(first_bucket + blockIdx.x);
    }
}

}  // namespace sort_detail
}  // namespace hpxhip
