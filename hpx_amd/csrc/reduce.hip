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

using namespace hpxhip;

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;
constexpr int kSteps = 8;  // vectors per thread per block

struct reduce_geom {
    uint64_t head, nvec, tail;
};

// Two-input loader so that one kernel template serves the unary conv
// (transform_reduce) and the binary conv (transform_reduce_binary).
template <typename TI, typename TA, typename Conv, bool BINARY>
struct source {
    const TI* a;
    const TI* b;
    Conv conv;
    __device__ __forceinline__ TA at(uint64_t i) const {
        if constexpr (BINARY) return conv(static_cast<TA>(a[i]), static_cast<TA>(b[i]));
        else return conv(static_cast<TA>(a[i]));
    }
};

// Block-wide reduction of one value per thread (fixed tree).
template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T x, Op op, T* lds) {
    const int wave = threadIdx.x / kWave;
    const T w = wave_reduce(x, op);
    if (lane_id() == 0) lds[wave] = w;
    __syncthreads();
    T r = Op::template identity<T>();
    if (wave == 0) r = wave_reduce(lane_id() < kWaves ? lds[lane_id()] : Op::template identity<T>(), op);
    return r;  // valid in wave 0
}

template <typename TI, typename TA, typename Conv, typename Op, bool BINARY, int V>
__global__ __launch_bounds__(kThreads) void k_reduce(source<TI, TA, Conv, BINARY> src, reduce_geom g, Op op, TA init,
                                                      TA* __restrict__ partials, TA* __restrict__ out) {
    using VI = vec<TI, V>;
    __shared__ TA lds[kWaves];

    const TA id = Op::template identity<TA>();
    const uint64_t tid = threadIdx.x;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kThreads * kSteps + tid;

    TA acc = id;
    if (blockIdx.x == 0) {
        if (tid < g.head) acc = op(acc, src.at(tid));
        const uint64_t tail0 = g.head + g.nvec * V;
        if (tid < g.tail) acc = op(acc, src.at(tail0 + tid));
    }
    const VI* va = reinterpret_cast<const VI*>(src.a + g.head);
    const VI* vb = reinterpret_cast<const VI*>((BINARY ? src.b : src.a) + g.head);
    if (base + static_cast<uint64_t>(kSteps - 1) * kThreads < g.nvec) {
        // full chunk: every load in flight before the first fold
        VI x[kSteps], y[kSteps];
#pragma unroll
        for (int k = 0; k < kSteps; ++k) {
            x[k] = ld_stream(&va[base + static_cast<uint64_t>(k) * kThreads]);
            if constexpr (BINARY) y[k] = ld_stream(&vb[base + static_cast<uint64_t>(k) * kThreads]);
        }
#pragma unroll
        for (int k = 0; k < kSteps; ++k)
#pragma unroll
            for (int e = 0; e < V; ++e) {
                TA c;
                if constexpr (BINARY) c = src.conv(static_cast<TA>(x[k].v[e]), static_cast<TA>(y[k].v[e]));
                else c = src.conv(static_cast<TA>(x[k].v[e]));
                acc = op(acc, c);
            }
    } else {
#pragma unroll 2
    for (int k = 0; k < kSteps; ++k) {
        const uint64_t i = base + static_cast<uint64_t>(k) * kThreads;
        if (i < g.nvec) {
            const VI x = ld_stream(&va[i]);
            VI y;
            if constexpr (BINARY) y = ld_stream(&vb[i]);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                TA c;
                if constexpr (BINARY) c = src.conv(static_cast<TA>(x.v[e]), static_cast<TA>(y.v[e]));
                else c = src.conv(static_cast<TA>(x.v[e]));
                acc = op(acc, c);
            }
        }
    }
    }

    const TA blk = block_reduce(acc, op, lds);
    if (tid == 0) {
        if (gridDim.x == 1) *out = op(init, blk);
        else partials[blockIdx.x] = blk;
    }
}

// Fold of the block partials (one block; the previous launch's stores are
// visible at the kernel boundary).  Thread t folds partials t, t + 1024, ...
// with kBatch loads in flight, then the block tree: a fixed order for a given
// partial count.
template <typename TA, typename Op>
__global__ __launch_bounds__(kThreads) void k_reduce_partials(const TA* __restrict__ partials, uint32_t count, Op op,
                                                              TA init, TA* __restrict__ out) {
    constexpr int kBatch = 16;
    __shared__ TA lds[kWaves];
    const TA id = Op::template identity<TA>();
    TA r = id;
    for (uint32_t i0 = 0; i0 < count; i0 += kThreads * kBatch) {
        TA v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            const uint32_t i = i0 + k * kThreads + threadIdx.x;
            v[k] = i < count ? partials[i] : id;
        }
#pragma unroll
        for (int k = 0; k < kBatch; ++k) r = op(r, v[k]);
    }
    const TA total = block_reduce(r, op, lds);
    if (threadIdx.x == 0) *out = op(init, total);
}

template <typename TA, typename Op>
__global__ void k_write_init(TA init, TA* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = init;
}

struct reduce_layout {
    uint64_t blocks;
    size_t total;
};

reduce_layout make_layout(uint64_t n) {
    // worst case (4-byte elements, V = 4): vectors = n/4 (+ head/tail)
    reduce_layout L;
    const uint64_t per_block = static_cast<uint64_t>(kThreads) * kSteps;
    const uint64_t nvec = n;  // upper bound on vectors for V >= 1
    L.blocks = (nvec + per_block - 1) / per_block;
    if (L.blocks == 0) L.blocks = 1;
    L.total = align_up(L.blocks * 8, 256);
    return L;
}

template <typename TI, typename TA, typename Conv, typename Op, bool BINARY>
int launch_reduce(const TI* a, const TI* b, uint64_t n, Conv conv, Op op, TA init, TA* out, hipStream_t s,
                  void* scratch, size_t scratch_bytes) {
    if (n == 0) {
        hipLaunchKernelGGL((k_write_init<TA, Op>), dim3(1), dim3(64), 0, s, init, out);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    }
    const reduce_layout L = make_layout(n);
    void* ws = nullptr;
    int rc = resolve_scratch(s, scratch, scratch_bytes, L.total, &ws);
    if (rc) return rc;
    TA* partials = static_cast<TA*>(ws);

    constexpr int V = 16 / sizeof(TI);
    source<TI, TA, Conv, BINARY> src{a, b, conv};
    reduce_geom g;
    uint64_t ha = head_to_align16(a, sizeof(TI));
    uint64_t hb = BINARY ? head_to_align16(b, sizeof(TI)) : ha;
    const uint64_t per_block = static_cast<uint64_t>(kThreads) * kSteps;
    uint64_t blocks = 0;
    if (ha != UINT64_MAX && ha == hb) {
        if (ha > n) ha = n;
        g.head = ha;
        g.nvec = (n - ha) / V;
        g.tail = n - ha - g.nvec * V;
        blocks = (g.nvec + per_block - 1) / per_block;
        if (blocks == 0) blocks = 1;
        hipLaunchKernelGGL((k_reduce<TI, TA, Conv, Op, BINARY, V>), dim3(static_cast<unsigned>(blocks)),
                           dim3(kThreads), 0, s, src, g, op, init, partials, out);
    } else if constexpr (BINARY) {
        // Inputs that cannot be aligned together: scalar loads.
        g = reduce_geom{0, n, 0};
        blocks = (n + per_block - 1) / per_block;
        hipLaunchKernelGGL((k_reduce<TI, TA, Conv, Op, BINARY, 1>), dim3(static_cast<unsigned>(blocks)),
                           dim3(kThreads), 0, s, src, g, op, init, partials, out);
    } else {
        return HPXHIP_ERROR_INVALID_ARGUMENT;  // pointer not element-aligned
    }
    HPXHIP_CHECK_LAUNCH();
    if (blocks > 1) {
        hipLaunchKernelGGL((k_reduce_partials<TA, Op>), dim3(1), dim3(kThreads), 0, s, partials,
                           static_cast<uint32_t>(blocks), op, init, out);
        HPXHIP_CHECK_LAUNCH();
    }
    return 0;
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
