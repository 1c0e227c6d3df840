// common.hpp -- device-side building blocks shared by every hpx_amd kernel.
//
// MI355X (gfx950, CDNA4) only: wave64, DPP row/wave controls of the GFX9
// family, agent-scope `sc1` hand-offs between workgroups (the XCD L2s are not
// coherent with each other).  Nothing here is a CUDA idiom recompiled: the
// wave primitives are DPP sequences, the inter-workgroup protocol follows
// the write-through (sc1) + drained flag form of the MI355X microarchitecture
// guide (Guideline 16, table row 1).
//
// The binary operators mirror the functors HPX's algorithms accept
// (std::plus, std::multiplies, min/max, bit ops; see e.g.
// hpx/parallel/algorithms/reduce.hpp:200, inclusive_scan.hpp:288) plus the
// identity element every GPU tree/scan needs for inactive lanes.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstring>
#include <limits>
#include <type_traits>

// Ablation builds only (-DHPXHIP_TILE_DYN_ID=true): tile ids of the single-
// pass kernels (scan, copy_if, onesweep sort passes) from an atomic counter
// instead of blockIdx (lookback.hpp).
#ifndef HPXHIP_TILE_DYN_ID
#define HPXHIP_TILE_DYN_ID false
#endif

namespace hpxhip {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Wrapping integer arithmetic (HPX relies on the host's two's-complement
// behaviour; device code must not give the optimiser signed-overflow UB).
template <typename T>
__host__ __device__ __forceinline__ T wrap_add(T a, T b) {
    if constexpr (std::is_integral_v<T>) {
        using U = std::make_unsigned_t<T>;
        return static_cast<T>(static_cast<U>(a) + static_cast<U>(b));
    } else {
        return a + b;
    }
}
template <typename T>
__host__ __device__ __forceinline__ T wrap_mul(T a, T b) {
    if constexpr (std::is_integral_v<T>) {
        using U = std::make_unsigned_t<T>;
        return static_cast<T>(static_cast<U>(a) * static_cast<U>(b));
    } else {
        return a * b;
    }
}

// ---------------------------------------------------------------------------
// Binary operators with identities.  The semantics are the std:: functors'
// (std::min is `(b < a) ? b : a`, std::max is `(a < b) ? b : a`).
struct op_plus {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return wrap_add(a, b); }
    template <typename T> __host__ __device__ static constexpr T identity() { return T(0); }
};
struct op_multiplies {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return wrap_mul(a, b); }
    template <typename T> __host__ __device__ static constexpr T identity() { return T(1); }
};
struct op_min {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return (b < a) ? b : a; }
    template <typename T> __host__ __device__ static constexpr T identity() {
        if constexpr (std::is_floating_point_v<T>) return std::numeric_limits<T>::infinity();
        else return std::numeric_limits<T>::max();
    }
};
struct op_max {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return (a < b) ? b : a; }
    template <typename T> __host__ __device__ static constexpr T identity() {
        if constexpr (std::is_floating_point_v<T>) return -std::numeric_limits<T>::infinity();
        else return std::numeric_limits<T>::lowest();
    }
};
struct op_bit_and {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return a & b; }
    template <typename T> __host__ __device__ static constexpr T identity() { return static_cast<T>(~T(0)); }
};
struct op_bit_or {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return a | b; }
    template <typename T> __host__ __device__ static constexpr T identity() { return T(0); }
};
struct op_bit_xor {
    template <typename T> __host__ __device__ __forceinline__ T operator()(T a, T b) const { return a ^ b; }
    template <typename T> __host__ __device__ static constexpr T identity() { return T(0); }
};

// ---------------------------------------------------------------------------
// opt<T>: a value or "no value".  A user operator (a device closure of the
// C++ layer) has no known identity, but every GPU tree and scan pads
// inactive lanes with one: lifted_op makes "no value" that identity, so the
// kernels run any associative operator unchanged (reduce_kernel.hpp,
// scan_kernel.hpp; hpx/parallel/detail/device_algorithms.hpp).
template <typename T>
struct opt {
    T v;
    uint32_t ok;
};
template <typename T>
__host__ __device__ __forceinline__ T unwrap_value(T x) { return x; }
template <typename T>
__host__ __device__ __forceinline__ T unwrap_value(opt<T> x) { return x.v; }

template <typename F>
struct lifted_op {
    F f;
    template <typename X>
    __device__ __forceinline__ X operator()(X a, X b) const {
        if (!a.ok) return b;
        if (!b.ok) return a;
        return X{f(a.v, b.v), 1u};
    }
    template <typename X>
    __host__ __device__ static constexpr X identity() { return X{}; }
};

// noid_op<F>: a user operator scanned WITHOUT an identity (r04).  The scan
// kernel then keeps plain T values (not opt<T>, whose flag and padding halve
// the rounds that fit the registers: 2^30 int64 3.43 vs 2.66 ms,
// profiles/r04_closure_timing_first.log) and replaces every identity by the
// structure that makes it unnecessary: padded lanes and out-of-range
// elements only ever feed results that are not stored, and the few
// positions with nothing before them (lane 0 of a wave scan, the first
// element of an exclusive lane scan) are known by index.
template <typename F>
struct noid_op {
    F f;
    static constexpr bool kNoIdentity = true;
    template <typename T>
    __device__ __forceinline__ T operator()(T a, T b) const {
        return static_cast<T>(f(a, b));
    }
};
template <typename Op, typename = void>
struct is_noid_op : std::false_type {};
template <typename Op>
struct is_noid_op<Op, std::void_t<decltype(Op::kNoIdentity)>> : std::bool_constant<Op::kNoIdentity> {};

// ---------------------------------------------------------------------------
// 16-byte vector of T (one `global_load_dwordx4` per lane).
template <typename T, int N>
struct alignas(sizeof(T) * N) vec {
    T v[N];
};

template <typename T>
struct vec_width {
    static constexpr int value = 16 / sizeof(T);
};

// ---------------------------------------------------------------------------
// Streaming accesses: `global_load/store ... nt` (nontemporal cache policy).
// Measured on MI355X at 2^30 doubles (scripts/ubench/{rd2,ew2}.hip,
// profiles/r01_ubench_nt.log): read stream 6.36 -> 6.91 TB/s, triad 6.16 ->
// 6.73 TB/s with both loads and stores nt, copy 6.34 -> 6.71 TB/s.  A
// write-only stream (fill) is faster with plain stores (6.94 vs 6.79), so
// the kernels choose per access.  Data touched this way is read once; the
// policy bit changes caching only, never the value or its visibility at the
// next kernel boundary.
template <typename T>
struct nt_word {
    using type = std::conditional_t<
        sizeof(T) == 16, uint32_t __attribute__((ext_vector_type(4))),
        std::conditional_t<sizeof(T) == 8, uint64_t,
                           std::conditional_t<sizeof(T) == 4, uint32_t,
                                              std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>>;
};
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
    using W = typename nt_word<T>::type;
    static_assert(sizeof(W) == sizeof(T), "ld_stream: unsupported width");
    const W w = __builtin_nontemporal_load(reinterpret_cast<const W*>(p));
    T v;
    __builtin_memcpy(&v, &w, sizeof(T));
    return v;
}
template <typename T>
__device__ __forceinline__ void st_stream(T* p, const T& v) {
    using W = typename nt_word<T>::type;
    static_assert(sizeof(W) == sizeof(T), "st_stream: unsupported width");
    W w;
    __builtin_memcpy(&w, &v, sizeof(T));
    __builtin_nontemporal_store(w, reinterpret_cast<W*>(p));
}

// Elements [sh, sh + V) of the aligned vector pair (p[i], p[i + 1]): a
// 16-B-vector read of a range that starts sh elements past a 16-B boundary
// (elementwise and scan kernels for inputs offset from their output).  Plain
// loads: p[i + 1] is the next lane's p[i], a cache hit.
template <typename T, int V>
__device__ __forceinline__ vec<T, V> ld_shifted(const vec<T, V>* p, uint64_t i, int sh) {
    using VT = vec<T, V>;
    if (sh == 0) return ld_stream(&p[i]);
    const VT c = p[i], d = p[i + 1];
    VT r;
#pragma unroll
    for (int e = 0; e < V; ++e) {
        T v = c.v[0];
#pragma unroll
        for (int k = 1; k < 2 * V; ++k)
            if (k == e + sh) v = k < V ? c.v[k] : d.v[k - V];
        r.v[e] = v;
    }
    return r;
}

// ---------------------------------------------------------------------------
// Sort key order (radix sort, merge, sorted-range searches).
// Storage bits -> ordered unsigned bits (ascending), optionally inverted:
// signed integers flip the sign bit, IEEE floats flip all bits of negatives
// and the sign bit of non-negatives (total order), descending inverts.
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
    // ordered bits -> storage bits
    __device__ __forceinline__ U inverse(U o) const {
        constexpr U sign = U(1) << (sizeof(U) * 8 - 1);
        const U u = DESC ? ~o : o;
        if constexpr (std::is_floating_point_v<T>) return (u & sign) ? (u ^ sign) : ~u;
        else if constexpr (std::is_signed_v<T>) return u ^ sign;
        else return u;
    }
};

// ---------------------------------------------------------------------------
// Bit casts between T and 32-bit lanes (DPP moves 32 bits per lane).
template <typename T>
__device__ __forceinline__ void to_words(T x, uint32_t (&w)[(sizeof(T) + 3) / 4]) {
    static_assert(sizeof(T) % 4 == 0 && sizeof(T) <= 32, "whole 32-bit words only");
    __builtin_memcpy(w, &x, sizeof(T));
}
template <typename T>
__device__ __forceinline__ T from_words(const uint32_t (&w)[(sizeof(T) + 3) / 4]) {
    T x;
    __builtin_memcpy(&x, w, sizeof(T));
    return x;
}

// update_dpp on an arbitrary 4/8-byte type; lanes whose source is invalid or
// masked off receive `old`.
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, typename T>
__device__ __forceinline__ T dpp(T old, T src) {
    constexpr int W = (sizeof(T) + 3) / 4;
    uint32_t o[W], s[W], r[W];
    to_words(old, o);
    to_words(src, s);
#pragma unroll
    for (int i = 0; i < W; ++i)
        r[i] = __builtin_amdgcn_update_dpp(o[i], s[i], CTRL, ROW_MASK, BANK_MASK, false);
    return from_words<T>(r);
}

template <typename T>
__device__ __forceinline__ T readlane(T x, int lane) {
    constexpr int W = (sizeof(T) + 3) / 4;
    uint32_t s[W], r[W];
    to_words(x, s);
#pragma unroll
    for (int i = 0; i < W; ++i) r[i] = __builtin_amdgcn_readlane(s[i], lane);
    return from_words<T>(r);
}

template <typename T>
__device__ __forceinline__ T shfl(T x, int src_lane) {
    constexpr int W = (sizeof(T) + 3) / 4;
    uint32_t s[W], r[W];
    to_words(x, s);
#pragma unroll
    for (int i = 0; i < W; ++i) r[i] = __builtin_amdgcn_ds_bpermute(src_lane << 2, s[i]);
    return from_words<T>(r);
}

// DPP controls (GFX9 family, valid on gfx950).
enum : int {
    DPP_ROW_SHR1 = 0x111,
    DPP_ROW_SHR2 = 0x112,
    DPP_ROW_SHR3 = 0x113,
    DPP_ROW_SHR4 = 0x114,
    DPP_ROW_SHR8 = 0x118,
    DPP_WAVE_SHL1 = 0x130,
    DPP_WAVE_SHR1 = 0x138,
    DPP_ROW_BCAST15 = 0x142,
    DPP_ROW_BCAST31 = 0x143,
};

// Elements [sh, sh + V) of the aligned vector pair (mine, the next lane's
// aligned vector): the next lane's vector comes over DPP wave_shl:1, and
// lane 63 (whose source is outside the wave) takes `after`, the aligned
// vector that follows the wave's 64.  A range that starts sh elements past a
// 16-B boundary is then read with one aligned 16-B load per lane (plus one
// wave-uniform vector per wave) instead of two (ld_shifted).  All 64 lanes
// must be active.
template <typename T, int V>
__device__ __forceinline__ vec<T, V> shift_from_next_lane(const vec<T, V>& mine, const vec<T, V>& after, int sh) {
    const vec<T, V> nb = dpp<DPP_WAVE_SHL1>(after, mine);
    vec<T, V> r;
#pragma unroll
    for (int e = 0; e < V; ++e) {
        T v = mine.v[0];
#pragma unroll
        for (int k = 1; k < 2 * V; ++k)
            if (k == e + sh) v = k < V ? mine.v[k] : nb.v[k - V];
        r.v[e] = v;
    }
    return r;
}

// Inclusive wave64 scan: lane l receives x_0 (+) ... (+) x_l, the lower
// lanes always the left operand (a non-commutative associative op -- a user
// operator of the C++ layer -- scans in lane order).
// 7 DPP steps: three row_shr from the original value, row_shr:4/8 inside the
// 16-lane rows, then row_bcast:15/31 across rows.
template <typename T, typename Op>
__device__ __forceinline__ T wave_inclusive_scan(T x, Op op) {
    const T id = Op::template identity<T>();
    T s = op(dpp<DPP_ROW_SHR1>(id, x), x);
    s = op(dpp<DPP_ROW_SHR2>(id, x), s);
    s = op(dpp<DPP_ROW_SHR3>(id, x), s);
    s = op(dpp<DPP_ROW_SHR4, 0xf, 0xe>(id, s), s);
    s = op(dpp<DPP_ROW_SHR8, 0xf, 0xc>(id, s), s);
    s = op(dpp<DPP_ROW_BCAST15, 0xa, 0xf>(id, s), s);
    s = op(dpp<DPP_ROW_BCAST31, 0xc, 0xf>(id, s), s);
    return s;
}

// The same without an identity (noid_op): a lane whose DPP source lies
// outside its row / wave keeps its value instead of combining with an
// identity -- the source-validity masks are those of the DPP controls above.
// Every lane's result is x_0 (+) ... (+) x_l.
template <typename T, typename Op>
__device__ __forceinline__ T wave_inclusive_scan_noid(T x, Op op) {
    const int l = static_cast<int>(__lane_id());
    const int r = l & 15;
    T s = x;
    T t = op(dpp<DPP_ROW_SHR1>(x, x), x);
    s = r >= 1 ? t : s;
    t = op(dpp<DPP_ROW_SHR2>(x, x), s);
    s = r >= 2 ? t : s;
    t = op(dpp<DPP_ROW_SHR3>(x, x), s);
    s = r >= 3 ? t : s;
    t = op(dpp<DPP_ROW_SHR4>(s, s), s);
    s = r >= 4 ? t : s;
    t = op(dpp<DPP_ROW_SHR8>(s, s), s);
    s = r >= 8 ? t : s;
    t = op(dpp<DPP_ROW_BCAST15>(s, s), s);
    s = (l & 16) ? t : s;
    t = op(dpp<DPP_ROW_BCAST31>(s, s), s);
    s = l >= 32 ? t : s;
    return s;
}

// op with its operands swapped (same identity): a fold over lanes that hold
// values in DECREASING index order (the look-back window) in index order.
template <typename Op>
struct flipped_op {
    Op op;
    template <typename T>
    __device__ __forceinline__ T operator()(T a, T b) const {
        return op(b, a);
    }
    template <typename T>
    __host__ __device__ static constexpr T identity() {
        return Op::template identity<T>();
    }
};

// Exclusive companion of an inclusive wave scan (lane 0 gets the identity).
template <typename T, typename Op>
__device__ __forceinline__ T wave_shift_right(T incl) {
    return dpp<DPP_WAVE_SHR1>(Op::template identity<T>(), incl);
}

// Wave64 reduction: every lane receives the total.
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T x, Op op) {
    return readlane(wave_inclusive_scan(x, op), kWave - 1);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// The XCD (0-7) this wave runs on: s_getreg_b32 of HW_REG_XCC_ID (hwreg 20,
// bits [3:0]).  A placement hint for L2 affinity only, never for correctness
// (cdna_hip_programming.md section 1, T1).
__device__ __forceinline__ uint32_t xcc_id() {
    return static_cast<uint32_t>(__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20)) & 7u;
}

// ---------------------------------------------------------------------------
// Inter-workgroup hand-off words (agent scope).  Producer: payload stored
// with sc1 (`relaxed, agent` atomic store), then `s_waitcnt vmcnt(0)`, then
// the flag stored the same way by the same lane.  Consumer: relaxed sc1 poll,
// and only after the poll matched, sc1 loads of the payload.
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
    if constexpr (sizeof(T) == 8) {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        __hip_atomic_store(reinterpret_cast<uint64_t*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        uint32_t u;
        __builtin_memcpy(&u, &v, 4);
        __hip_atomic_store(reinterpret_cast<uint32_t*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
    T v;
    if constexpr (sizeof(T) == 8) {
        uint64_t u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_memcpy(&v, &u, 8);
    } else {
        uint32_t u = __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_memcpy(&v, &u, 4);
    }
    return v;
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Compiler-only ordering: keep payload loads below the poll that licensed them.
__device__ __forceinline__ void order_after_poll() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); }

// Bounded spin: every look-back wait gives up after this many polls and
// raises the device error word instead of hanging the GPU.
constexpr uint32_t kSpinLimit = 1u << 24;
// s_sleep argument between polls (units of 64 clocks)
#ifndef HPXHIP_LB_SLEEP
#define HPXHIP_LB_SLEEP 1
#endif

// Device error word (per library instance); set by a kernel that gave up a
// spin, read back by hpxhip_device_error().
// HPXHIP_DEVERR_RANGE: a scatter destination or merge split outside its
// buffer (inputs changed while the algorithm ran, e.g. a caller racing a sort
// from another stream); the store is dropped and the error raised, so the
// caller gets an error instead of silently wrong output.
enum : uint32_t { HPXHIP_DEVERR_NONE = 0, HPXHIP_DEVERR_LOOKBACK_TIMEOUT = 1, HPXHIP_DEVERR_RANGE = 2 };

__device__ __forceinline__ void raise_device_error(uint32_t* err, uint32_t code) {
    if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace hpxhip
