// reduce_kernel.hpp -- the reduce / transform_reduce kernels (see
// hpx_amd/csrc/reduce.hip for the algorithm notes and measurements).
// Header so that the library's precompiled operator kinds and the C++
// layer's device closures (hpx/parallel/detail/device_algorithms.hpp, user
// HPX_HOST_DEVICE conv/op under hipcc) instantiate the same kernel bodies.
//
// Src (the element source) provides
//   const TI* a, *b;                            the input range(s)
//   __device__ TA elem(TI x) const;            conv of one element (unary)
//   __device__ TA elem(TI x, TI y) const;      conv of two elements (binary)
// Op provides operator()(TA, TA) and a static identity<TA>() used for
// inactive lanes of the DPP tree (a user op without one is lifted to
// opt<T>, device_algorithms.hpp).
#pragma once

#include <hpxhip/kernels/common.hpp>

namespace hpxhip {
namespace reduce_detail {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;
constexpr int kSteps = 8;  // 16-B vectors per thread per block (128 KiB per block)

struct geom {
    uint64_t head, nvec, tail;  // scalar head (to 16 B), vectors, scalar tail
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

template <typename TI, typename TA, typename Src, typename Op, bool BINARY, int V>
__global__ __launch_bounds__(kThreads) void k_reduce(Src src, geom g, Op op, TA init, TA* __restrict__ partials,
                                                      TA* __restrict__ out) {
    using VI = vec<TI, V>;
    __shared__ TA lds[kWaves];

    const TA id = Op::template identity<TA>();
    const uint64_t tid = threadIdx.x;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kThreads * kSteps + tid;
    auto at = [&](uint64_t i) -> TA {
        if constexpr (BINARY) return src.elem(src.a[i], src.b[i]);
        else return src.elem(src.a[i]);
    };

    TA acc = id;
    if (blockIdx.x == 0) {
        if (tid < g.head) acc = op(acc, at(tid));
        const uint64_t tail0 = g.head + g.nvec * V;
        if (tid < g.tail) acc = op(acc, at(tail0 + tid));
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
                if constexpr (BINARY) acc = op(acc, src.elem(x[k].v[e], y[k].v[e]));
                else acc = op(acc, src.elem(x[k].v[e]));
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
                    if constexpr (BINARY) acc = op(acc, src.elem(x.v[e], y.v[e]));
                    else acc = op(acc, src.elem(x.v[e]));
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

template <typename TA>
__global__ void k_write_init(TA init, TA* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = init;
}

// Blocks of the main launch for n elements (upper bound over V >= 1).
__host__ __device__ inline uint64_t max_blocks(uint64_t n) {
    const uint64_t per_block = static_cast<uint64_t>(kThreads) * kSteps;
    const uint64_t b = (n + per_block - 1) / per_block;
    return b ? b : 1;
}

// Elements before the first 16-B boundary of p (UINT64_MAX: p is not
// element-aligned, so no head makes it 16-B aligned).
__host__ __device__ inline uint64_t head_to_align16(const void* p, size_t elem_size) {
    const uintptr_t mis = reinterpret_cast<uintptr_t>(p) & 15u;
    if (mis == 0) return 0;
    if (mis % elem_size != 0) return UINT64_MAX;
    return (16u - mis) / elem_size;
}

// Queue the reduction of [a, a + n) (and b for BINARY) into *out on s.
// partials: max_blocks(n) TA values of scratch.  Returns a hipError_t.
template <typename TI, typename TA, typename Src, typename Op, bool BINARY>
hipError_t launch(Src src, uint64_t n, Op op, TA init, TA* out, TA* partials, hipStream_t s) {
    if (n == 0) {
        hipLaunchKernelGGL((k_write_init<TA>), dim3(1), dim3(64), 0, s, init, out);
        return hipGetLastError();
    }
    constexpr int V = 16 % sizeof(TI) == 0 ? 16 / sizeof(TI) : 1;
    const uint64_t per_block = static_cast<uint64_t>(kThreads) * kSteps;
    uint64_t ha = V > 1 ? head_to_align16(src.a, sizeof(TI)) : 0;
    uint64_t hb = (BINARY && V > 1) ? head_to_align16(src.b, sizeof(TI)) : ha;
    geom g;
    uint64_t blocks;
    if (ha != UINT64_MAX && ha == hb) {
        if (ha > n) ha = n;
        g.head = ha;
        g.nvec = (n - ha) / V;
        g.tail = n - ha - g.nvec * V;
        blocks = (g.nvec + per_block - 1) / per_block;
        if (blocks == 0) blocks = 1;
        hipLaunchKernelGGL((k_reduce<TI, TA, Src, Op, BINARY, V>), dim3(static_cast<unsigned>(blocks)),
                           dim3(kThreads), 0, s, src, g, op, init, partials, out);
    } else {
        // inputs that cannot be 16-B aligned together: element loads
        g = geom{0, n, 0};
        blocks = (n + per_block - 1) / per_block;
        hipLaunchKernelGGL((k_reduce<TI, TA, Src, Op, BINARY, 1>), dim3(static_cast<unsigned>(blocks)),
                           dim3(kThreads), 0, s, src, g, op, init, partials, out);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || blocks <= 1) return e;
    hipLaunchKernelGGL((k_reduce_partials<TA, Op>), dim3(1), dim3(kThreads), 0, s, partials,
                       static_cast<uint32_t>(blocks), op, init, out);
    return hipGetLastError();
}

}  // namespace reduce_detail
}  // namespace hpxhip
