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
#include "scan_kernel.hpp"

using namespace hpxhip;

namespace {

using namespace hpxhip::scan_detail;

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
