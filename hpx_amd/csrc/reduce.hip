// reduce.hip -- reduce / transform_reduce / transform_reduce_binary.
//
// The reference has no GPU reduction: reduce.hpp:58-89 and
// transform_reduce.hpp:68-112 need a future<T> per chunk
// (util/partitioner.hpp:44-76), which the CUDA executor cannot return, so
// the host partitioner folds chunk partials `init (+) P0 (+) P1 ...`.
// Here one launch does the whole algorithm:
//   * each 1024-thread block owns a contiguous chunk of 8 x 1024 16-B
//     vectors (128 KiB) and walks it 16 KiB at a time -- the geometry that
//     measured fastest for a read stream on MI355X (6.6 TB/s at 2^30 int64,
//     vs 5.7 TB/s for a 2048-block grid-stride loop; scripts/ubench/rd.hip),
//     all 8 loads in flight before the fold, nontemporal (6.91 TB/s for
//     the bare stream, scripts/ubench/rd2.hip);
//   * per thread a serial fold, DPP wave64 reduction, LDS across waves, one
//     partial per block, written with a plain store as the block retires;
//   * a second one-block launch folds the partials in a fixed order.
//     (The first version folded inside the same launch: the last block to
//     arrive behind agent-scope tickets folded the partials.  The drain +
//     ticket round trip held every 1024-thread block ~2 us past its last
//     load, which at two blocks per CU cost 1.45 ms against 1.24 ms for the
//     bare read stream; the extra launch costs a few microseconds.)
// The reduction tree depends only on n, so FP results are bitwise
// reproducible run to run; integer results are exact.
#include "internal.hpp"
#include <hpxhip/kernels/reduce_kernel.hpp>

using namespace hpxhip;

namespace {

using namespace hpxhip::reduce_detail;

// The precompiled conversion kinds: conv(static_cast<TA>(x)) (unary) or
// conv(TA(x), TA(y)) (binary), the element source of reduce_kernel.hpp.
template <typename TI, typename TA, typename Conv>
struct source {
    const TI* a;
    const TI* b;
    Conv conv;
    __device__ __forceinline__ TA elem(TI x) const { return conv(static_cast<TA>(x)); }
    __device__ __forceinline__ TA elem(TI x, TI y) const { return conv(static_cast<TA>(x), static_cast<TA>(y)); }
};

struct reduce_layout {
    uint64_t blocks;
    size_t total;
};

reduce_layout make_layout(uint64_t n) {
    reduce_layout L;
    L.blocks = max_blocks(n);
    L.total = align_up(L.blocks * 8, 256);
    return L;
}

template <typename TI, typename TA, typename Conv, typename Op, bool BINARY>
int launch_reduce(const TI* a, const TI* b, uint64_t n, Conv conv, Op op, TA init, TA* out, hipStream_t s,
                  void* scratch, size_t scratch_bytes) {
    // a unary range whose pointer is not element-aligned is rejected (the
    // binary form falls back to element loads, reduce_kernel.hpp)
    if (!BINARY && n && head_to_align16(a, sizeof(TI)) == UINT64_MAX) return HPXHIP_ERROR_INVALID_ARGUMENT;
    void* ws = nullptr;
    if (n) {
        int rc = resolve_scratch(s, scratch, scratch_bytes, make_layout(n).total, &ws);
        if (rc) return rc;
    }
    source<TI, TA, Conv> src{a, b, conv};
    return static_cast<int>(reduce_detail::launch<TI, TA, source<TI, TA, Conv>, Op, BINARY>(
        src, n, op, init, out, static_cast<TA*>(ws), s));
}

// Conversion kinds built for reductions: identity (reduce), scale, abs and
// square (norms); binary: multiply (inner product) and add.
template <typename TA, typename F>
int with_reduce_conv(int kind, const void* scalars, F&& f) {
    switch (kind) {
        case HPXHIP_U_IDENTITY:
        case HPXHIP_U_SCALE:
        case HPXHIP_U_ABS:
        case HPXHIP_U_SQUARE: break;
        default: return HPXHIP_ERROR_UNSUPPORTED;
    }
    return with_unary<TA>(kind, scalars, [&](auto conv) -> int {
        using C = decltype(conv);
        if constexpr (std::is_same_v<C, unary_fn<HPXHIP_U_IDENTITY, TA>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SCALE, TA>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_ABS, TA>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SQUARE, TA>>)
            return f(conv);
        else
            return HPXHIP_ERROR_UNSUPPORTED;
    });
}
template <typename TA, typename F>
int with_reduce_binary(int kind, const void* scalars, F&& f) {
    if (kind != HPXHIP_B_MUL && kind != HPXHIP_B_ADD) return HPXHIP_ERROR_UNSUPPORTED;
    return with_binary<TA>(kind, scalars, [&](auto conv) -> int {
        using C = decltype(conv);
        if constexpr (std::is_same_v<C, binary_fn<HPXHIP_B_MUL, TA>> || std::is_same_v<C, binary_fn<HPXHIP_B_ADD, TA>>)
            return f(conv);
        else
            return HPXHIP_ERROR_UNSUPPORTED;
    });
}

}  // namespace

namespace hpxhip {
size_t reduce_scratch_bytes(uint64_t n) { return make_layout(n).total; }
}  // namespace hpxhip

extern "C" {

int hpxhip_transform_reduce(int in_dtype, int acc_dtype, int red_op, int conv_kind, const void* conv_scalars,
                            const void* init, const void* in, uint64_t n, void* out_dev, hpxhip_stream stream,
                            void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_transform_reduce");
    if (!init || !out_dev || (n && !in)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_wide_dtype<TI>(acc_dtype, [&](auto ta) -> int {
            using TA = typename decltype(ta)::type;
            TA iv;
            __builtin_memcpy(&iv, init, sizeof(TA));
            return with_binop<TA>(red_op, [&](auto op) -> int {
                return with_reduce_conv<TA>(conv_kind, conv_scalars, [&](auto conv) -> int {
                    return launch_reduce<TI, TA, decltype(conv), decltype(op), false>(
                        static_cast<const TI*>(in), nullptr, n, conv, op, iv, static_cast<TA*>(out_dev), s, scratch,
                        scratch_bytes);
                });
            });
        });
    });
}

int hpxhip_transform_reduce_binary(int in_dtype, int acc_dtype, int red_op, int binary_kind, const void* bin_scalars,
                                   const void* init, const void* in1, const void* in2, uint64_t n, void* out_dev,
                                   hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_transform_reduce_binary");
    if (!init || !out_dev || (n && (!in1 || !in2))) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(in_dtype, [&](auto ti) -> int {
        using TI = typename decltype(ti)::type;
        return with_wide_dtype<TI>(acc_dtype, [&](auto ta) -> int {
            using TA = typename decltype(ta)::type;
            TA iv;
            __builtin_memcpy(&iv, init, sizeof(TA));
            return with_binop<TA>(red_op, [&](auto op) -> int {
                return with_reduce_binary<TA>(binary_kind, bin_scalars, [&](auto conv) -> int {
                    return launch_reduce<TI, TA, decltype(conv), decltype(op), true>(
                        static_cast<const TI*>(in1), static_cast<const TI*>(in2), n, conv, op, iv,
                        static_cast<TA*>(out_dev), s, scratch, scratch_bytes);
                });
            });
        });
    });
}

}  // extern "C"
