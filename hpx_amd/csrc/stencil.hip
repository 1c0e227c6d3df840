// stencil.hip -- examples/1d_stencil heat equation step.
//
// Reference operator (1d_stencil_1.cpp:43-46, identical in _4/_4_parallel/_8):
//     heat(l, m, r) = m + (k*dt/(dx*dx)) * (l - 2*m + r)
// evaluated in double with periodic boundaries (1d_stencil_1.cpp:58-70;
// idx() wrap in 1d_stencil_4_parallel.cpp:35-38).  Compiled with
// -ffp-contract=off and the same association, so results are bit-identical
// to the serial reference.
//
// Kernel: each lane loads one 16-B vector (two points); the left/right
// neighbours come from the adjacent lanes (ds_bpermute), the wave's edge
// lanes read one extra point (or the halo at the partition ends).
// Traffic: 16 B/point/step (read cur, write next).  Default cache policy:
// the edge lanes' extra loads then hit the lines the adjacent wave just
// fetched (nontemporal loads cost 12 %); nontemporal stores measured 1 %
// faster in isolation but 4 % slower in the library probe, so they are not
// used; 256-thread blocks beat 64-1024 (scripts/ubench/stencil.hip,
// profiles/r01_ubench_stencil.log).
#include "internal.hpp"

using namespace hpxhip;

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ double heat(double l, double m, double r, double c) {
    return m + c * (l - 2 * m + r);
}

// Vector body: points [0, 2*nvec) as nvec 16-B vectors (cur, next aligned).
__global__ __launch_bounds__(kThreads) void k_heat_vec(const double* __restrict__ cur, double* __restrict__ next,
                                                        uint64_t n, uint64_t nvec, const double* __restrict__ lh,
                                                        const double* __restrict__ rh, double c) {
    using V2 = vec<double, 2>;
    const uint64_t g = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    const int lane = lane_id();
    const bool in = g < nvec;
    V2 x = {{0.0, 0.0}};
    if (in) x = reinterpret_cast<const V2*>(cur)[g];
    const double from_left = shfl(x.v[1], lane == 0 ? 0 : lane - 1);
    const double from_right = shfl(x.v[0], lane == kWave - 1 ? kWave - 1 : lane + 1);
    if (!in) return;
    const uint64_t i0 = 2 * g;
    double l, r;
    if (lane == 0 || g == 0) l = (i0 == 0) ? *lh : cur[i0 - 1];
    else l = from_left;
    if (lane == kWave - 1 || g + 1 == nvec) r = (i0 + 2 >= n) ? *rh : cur[i0 + 2];
    else r = from_right;
    V2 y;
    y.v[0] = heat(l, x.v[0], x.v[1], c);
    y.v[1] = heat(x.v[0], x.v[1], r, c);
    reinterpret_cast<V2*>(next)[g] = y;
}

// Scalar points [first, n).
__global__ __launch_bounds__(kThreads) void k_heat_scalar(const double* __restrict__ cur, double* __restrict__ next,
                                                           uint64_t first, uint64_t n, const double* __restrict__ lh,
                                                           const double* __restrict__ rh, double c) {
    const uint64_t i = first + static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    const double l = (i == 0) ? *lh : cur[i - 1];
    const double r = (i + 1 == n) ? *rh : cur[i + 1];
    next[i] = heat(l, cur[i], r, c);
}

int launch_step(const double* cur, double* next, uint64_t n, const double* lh, const double* rh, double c,
                hipStream_t s) {
    const bool aligned = (reinterpret_cast<uintptr_t>(cur) % 16 == 0) && (reinterpret_cast<uintptr_t>(next) % 16 == 0);
    uint64_t first = 0;
    if (aligned && n >= 2) {
        const uint64_t nvec = n / 2;
        const uint64_t blocks = (nvec + kThreads - 1) / kThreads;
        hipLaunchKernelGGL(k_heat_vec, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0, s, cur, next, n, nvec,
                           lh, rh, c);
        HPXHIP_CHECK_LAUNCH();
        first = 2 * nvec;
    }
    if (first < n) {
        const uint64_t blocks = (n - first + kThreads - 1) / kThreads;
        hipLaunchKernelGGL(k_heat_scalar, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0, s, cur, next,
                           first, n, lh, rh, c);
        HPXHIP_CHECK_LAUNCH();
    }
    return 0;
}

}  // namespace

extern "C" {

int hpxhip_stencil_heat_step(const double* cur, double* next, uint64_t n, const double* left_halo_dev,
                             const double* right_halo_dev, double k, double dt, double dx, hpxhip_stream stream) {
    if (n == 0) return 0;
    if (!cur || !next || !left_halo_dev || !right_halo_dev || cur == next) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if ((n / 2 + kThreads - 1) / kThreads > 0x7fffffffull) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    const double c = k * dt / (dx * dx);
    return launch_step(cur, next, n, left_halo_dev, right_halo_dev, c, s);
}

int hpxhip_stencil_heat_run(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt, double dx,
                            hpxhip_stream stream) {
    if (n == 0 || nt == 0) return 0;
    if (!u0 || !u1 || u0 == u1) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    const double c = k * dt / (dx * dx);
    for (uint64_t t = 0; t < nt; ++t) {
        const double* cur = (t % 2 == 0) ? u0 : u1;
        double* nxt = (t % 2 == 0) ? u1 : u0;
        // periodic: left of point 0 is point n-1, right of point n-1 is point 0
        int rc = launch_step(cur, nxt, n, cur + (n - 1), cur, c, s);
        if (rc) return rc;
    }
    return 0;
}

}  // extern "C"
