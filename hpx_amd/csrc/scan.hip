// scan.hip -- inclusive_scan / exclusive_scan / transform_{in,ex}clusive_scan.
//
// Reference: inclusive_scan.hpp:90-173 and exclusive_scan.hpp:100-175 run
// scan_partitioner.hpp:62-156 on the host -- three phases, the data read
// once and written twice plus a re-read (section 3.3 of SURVEY.md).  Here:
// one pass, 16 B/element of HBM traffic (read once, write once).
//
// Tile = 256 threads x 8 vectors of 16 B (4096 int64 / 8192 int32 = 32 KiB).
// Each wave owns a contiguous quarter of the tile and walks it in 8 rounds of
// 64 lanes x 16 B (coalesced 1 KiB per instruction):
//   round r:  lane-serial scan of its V elements -> DPP wave scan of lane
//             totals -> running wave carry (readlane 63);
//   then      wave totals through LDS -> tile aggregate -> decoupled look-back
//             by wave 0 (lookback.hpp) -> every element op'd with the tile
//             prefix and stored with 16-B stores.
// Integer results are exact; FP results follow a tree order that can differ
// from the sequential left fold (tolerance in DESIGN.md).
#include "internal.hpp"
#include "lookback.hpp"

using namespace hpxhip;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kRounds = 8;

template <typename T>
constexpr uint64_t tile_elems() {
    return static_cast<uint64_t>(kThreads) * kRounds * (16 / sizeof(T));
}

template <typename T, typename Conv, typename Op, bool INCL, bool ALIGNED>
__global__ __launch_bounds__(kThreads) void k_scan(const T* in, T* out, uint64_t n, Conv conv, Op op, T init,
                                                    const T* prefix_dev, uint32_t* counter, tile_state<T> st) {
    constexpr int V = 16 / sizeof(T);
    constexpr uint64_t TILE = tile_elems<T>();
    constexpr uint64_t WAVE_ELEMS = TILE / kWaves;
    using VT = vec<T, V>;

    __shared__ uint32_t s_tile;
    __shared__ T s_wave_total[kWaves];
    __shared__ T s_prefix;

    if (threadIdx.x == 0)
        s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint64_t tile = s_tile;
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();
    const T id = Op::template identity<T>();

    const uint64_t tile_base = tile * TILE;
    const uint64_t wbase = tile_base + wave * WAVE_ELEMS;
    const bool full = tile_base + TILE <= n;

    // ---- load (all rounds in flight) and convert
    VT x[kRounds];
    if (ALIGNED && full) {
        const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
        for (int r = 0; r < kRounds; ++r) x[r] = src[r * kWave + lane];
#pragma unroll
        for (int r = 0; r < kRounds; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) x[r].v[e] = conv(x[r].v[e]);
    } else {
#pragma unroll
        for (int r = 0; r < kRounds; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                x[r].v[e] = i < n ? conv(in[i]) : id;
            }
    }

    // ---- per-round lane scan + wave scan; x becomes the wave-local result
    T carry = id;
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
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
    if (lane == 0) s_wave_total[wave] = carry;
    __syncthreads();

    T wave_prefix = id;
    T agg = id;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        if (w < wave) wave_prefix = op(wave_prefix, s_wave_total[w]);
        agg = op(agg, s_wave_total[w]);
    }

    // ---- decoupled look-back (wave 0)
    if (wave == 0) {
        T p;
        if (tile == 0) {
            p = prefix_dev ? *prefix_dev : init;
            if (lane == 0) st.publish(0, op(p, agg), TILE_INCLUSIVE);
        } else {
            if (lane == 0) st.publish(tile, agg, TILE_AGGREGATE);
            p = st.exclusive_prefix(tile, op);
            if (lane == 0) st.publish(tile, op(p, agg), TILE_INCLUSIVE);
        }
        if (lane == 0) s_prefix = p;
    }
    __syncthreads();
    const T pre = op(s_prefix, wave_prefix);

    // ---- store
    if (ALIGNED && full) {
        VT* dst = reinterpret_cast<VT*>(out + wbase);
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            VT y;
#pragma unroll
            for (int e = 0; e < V; ++e) y.v[e] = op(pre, x[r].v[e]);
            dst[r * kWave + lane] = y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < kRounds; ++r)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                if (i < n) out[i] = op(pre, x[r].v[e]);
            }
    }
}

template <typename T>
struct scan_layout {
    uint64_t ntiles;
    size_t flags_off, agg_off, incl_off, total;
    size_t memset_bytes;  // counter + flags, from the allocation start
};

template <typename T>
scan_layout<T> make_layout(uint64_t n) {
    scan_layout<T> L;
    L.ntiles = (n + tile_elems<T>() - 1) / tile_elems<T>();
    L.flags_off = 256;
    L.agg_off = align_up(L.flags_off + L.ntiles * 4, 256);
    L.memset_bytes = L.agg_off;
    L.incl_off = align_up(L.agg_off + L.ntiles * sizeof(T), 256);
    L.total = align_up(L.incl_off + L.ntiles * sizeof(T), 256);
    return L;
}

template <typename T, typename F>
int with_scan_conv(int kind, const void* scalars, F&& f) {
    switch (kind) {
        case HPXHIP_U_IDENTITY:
        case HPXHIP_U_SCALE:
        case HPXHIP_U_SQUARE: break;
        default: return HPXHIP_ERROR_UNSUPPORTED;
    }
    return with_unary<T>(kind, scalars, [&](auto conv) -> int {
        using C = decltype(conv);
        if constexpr (std::is_same_v<C, unary_fn<HPXHIP_U_IDENTITY, T>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SCALE, T>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SQUARE, T>>)
            return f(conv);
        else
            return HPXHIP_ERROR_UNSUPPORTED;
    });
}

}  // namespace

namespace hpxhip {
size_t scan_scratch_bytes(int dtype, uint64_t n) {
    return dtype_size(dtype) == 8 ? make_layout<uint64_t>(n).total : make_layout<uint32_t>(n).total;
}
}  // namespace hpxhip

extern "C" int hpxhip_scan(int dtype, int op, int inclusive, int conv_kind, const void* conv_scalars,
                           const void* init, const void* prefix_dev, const void* in, void* out, uint64_t n,
                           hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    if (n == 0) return 0;
    if (!in || !out || (!init && !prefix_dev)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        T iv = T(0);
        if (init) __builtin_memcpy(&iv, init, sizeof(T));
        return with_binop<T>(op, [&](auto o) -> int {
            using Op = decltype(o);
            return with_scan_conv<T>(conv_kind, conv_scalars, [&](auto conv) -> int {
                using Conv = decltype(conv);
                const scan_layout<T> L = make_layout<T>(n);
                void* ws = nullptr;
                int rc = resolve_scratch(s, scratch, scratch_bytes, L.total, &ws);
                if (rc) return rc;
                char* base = static_cast<char*>(ws);
                HPXHIP_CHECK(hipMemsetAsync(base, 0, L.memset_bytes, s));
                tile_state<T> st{reinterpret_cast<uint32_t*>(base + L.flags_off),
                                 reinterpret_cast<T*>(base + L.agg_off), reinterpret_cast<T*>(base + L.incl_off),
                                 device_error_word(s)};
                uint32_t* counter = reinterpret_cast<uint32_t*>(base);
                const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) &&
                                     (reinterpret_cast<uintptr_t>(out) % 16 == 0);
                const T* pd = static_cast<const T*>(prefix_dev);
                const dim3 grid(static_cast<unsigned>(L.ntiles)), block(kThreads);
                const T* ip = static_cast<const T*>(in);
                T* op_ = static_cast<T*>(out);
                if (inclusive) {
                    if (aligned)
                        hipLaunchKernelGGL((k_scan<T, Conv, Op, true, true>), grid, block, 0, s, ip, op_, n, conv, o,
                                           iv, pd, counter, st);
                    else
                        hipLaunchKernelGGL((k_scan<T, Conv, Op, true, false>), grid, block, 0, s, ip, op_, n, conv, o,
                                           iv, pd, counter, st);
                } else {
                    if (aligned)
                        hipLaunchKernelGGL((k_scan<T, Conv, Op, false, true>), grid, block, 0, s, ip, op_, n, conv, o,
                                           iv, pd, counter, st);
                    else
                        hipLaunchKernelGGL((k_scan<T, Conv, Op, false, false>), grid, block, 0, s, ip, op_, n, conv,
                                           o, iv, pd, counter, st);
                }
                HPXHIP_CHECK_LAUNCH();
                return 0;
            });
        });
    });
}
