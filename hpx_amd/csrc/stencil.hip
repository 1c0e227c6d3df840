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

// ------------------------------------------------------ temporal blocking
// S fused steps per pass (S even, 2..16): each wave owns a window of WIN = 1024
// consecutive points held in registers as ROWS rows x 64 lanes x P points
// (row r, lane l -> window points r*64P + l*P .. +P-1; loads and stores are
// 16-B vectors), steps it S times with the neighbours taken from the
// adjacent lanes by DPP wave shifts (row ends through readlane), and writes
// the WIN - 2S points that are still exact (a point's value after S steps
// depends on the S points each side).  Window w starts at out_lo + w*OUT - S,
// OUT = WIN - 2S, so consecutive windows overlap by 2S points.  P = 4 halves
// the cross-lane moves per point of P = 2.  r06: the pass is bound by each
// wave's serial per-step chain (profiles/r06_heat_valu_pmc_g.txt), so ROWS =
// 4 (independent rows: twice the chains per wave, 1024-point windows) against
// 2: 2^30 points x 100 steps 26.7-27.6 -> 25.5-26.2 ms (ramp), 30.5-31.5 ->
// 29.1-29.8 (random); 2 x 8, 4 x 8 (138 VGPRs) and 1 x 8 were no better
// (profiles/r06_heat_window_ab_r.log).
// HBM traffic per pass: 8 B read x WIN/OUT + 8 B written per point, i.e.
// 16.13 B per point for S = 8 steps (16.26 B for S = 16) instead of 16 B per
// point per step.
// Every point sees exactly the single-step arithmetic (heat() above, same
// association, -ffp-contract=off), so results are bit-identical to S single
// steps.  Points outside [0, n) come from the halos: cur[-j] = lh[S - j],
// cur[n + j] = rh[j] (j < S; for one periodic partition lh = cur + n - S,
// rh = cur).
#ifndef HPXHIP_HEAT_PTS
#define HPXHIP_HEAT_PTS 4
#endif
#ifndef HPXHIP_HEAT_ROWS
#define HPXHIP_HEAT_ROWS 4
#endif
#ifndef HPXHIP_HEAT_LANERUN
#define HPXHIP_HEAT_LANERUN 1
#endif
constexpr int kFusedPts = HPXHIP_HEAT_PTS;                  // points per lane per row
constexpr int kFusedRows = HPXHIP_HEAT_ROWS;
static_assert(kFusedPts % 2 == 0 && kFusedRows * kFusedPts * kWave > 2 * 16, "16-B vectors; a window wider than its halos");
constexpr int kFusedWin = kFusedRows * kFusedPts * kWave;  // 1024 points (hpx_amd/stencil.py FUSED_WINDOW)

template <int S>
__global__ __launch_bounds__(kThreads) void k_heat_fused(const double* __restrict__ cur, double* __restrict__ next,
                                                          uint64_t n, uint64_t out_lo, uint64_t out_hi,
                                                          const double* __restrict__ lh,
                                                          const double* __restrict__ rh, double c, bool aligned) {
    static_assert(S >= 2 && S <= 16 && S % 2 == 0, "even fused step counts");
    constexpr int P = kFusedPts;
    constexpr int ROW = P * kWave;
    using V2 = vec<double, 2>;
    constexpr uint64_t OUT = kFusedWin - 2 * S;
    const uint64_t wave_g = (static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x) / kWave;
    const uint64_t o0 = out_lo + wave_g * OUT;
    if (o0 >= out_hi) return;  // wave-uniform
    const uint64_t o1 = min(o0 + OUT, out_hi);
    const int lane = lane_id();
    const int64_t w0 = static_cast<int64_t>(o0) - S;  // window start (may be < 0)
    const bool inside = aligned && w0 >= 0 && static_cast<uint64_t>(w0) + kFusedWin <= n;

    double x[kFusedRows][P];
    if (inside) {
#pragma unroll
        for (int r = 0; r < kFusedRows; ++r)
#pragma unroll
            for (int h = 0; h < P / 2; ++h) {
                const V2 v = *reinterpret_cast<const V2*>(cur + w0 + r * ROW + lane * P + 2 * h);
                x[r][2 * h] = v.v[0];
                x[r][2 * h + 1] = v.v[1];
            }
    } else {
#pragma unroll
        for (int r = 0; r < kFusedRows; ++r)
#pragma unroll
            for (int e = 0; e < P; ++e) {
                const int64_t i = w0 + r * ROW + lane * P + e;
                double v = 0.0;  // beyond the halos: feeds only points that are not written
                if (i < 0) {
                    if (i >= -S) v = lh[S + i];
                } else if (static_cast<uint64_t>(i) < n) {
                    v = cur[i];
                } else if (static_cast<uint64_t>(i) < n + S) {
                    v = rh[static_cast<uint64_t>(i) - n];
                }
                x[r][e] = v;
            }
    }

#if HPXHIP_HEAT_LANERUN
    // r06, lane runs: the window passes through the wave's own LDS slice once
    // after the loads and once before the stores, so that during the steps
    // lane l holds the Q = ROWS x P consecutive points [lQ, lQ + Q): a step then
    // needs two wave shifts (the run's two ends) instead of per-row shifts,
    // row-crossing readlanes and their moves (124 -> 86 VALU instructions per
    // step at 4 x 4; the kernel is VALU-issue bound).  LDS granules of 16 B
    // are rotated by the run index (two-way bank conflicts at most on the
    // run-wise reads).  2^30 points x 100 steps 25.2-25.6 -> 23.3-23.8 ms
    // (ramp), 28.4-29.0 -> 27.0-27.2 (random), bit-identical; 2 x 4 runs
    // (8 points per lane) 24.8-25.0 (profiles/r06_heat_lanerun_ab_t.log).
    // The 32 KiB of LDS per block hold it to 5 waves per SIMD.
    constexpr int Q = kFusedRows * P;
    constexpr int QG = Q / 2;  // 16-B granules per run
    __shared__ alignas(16) double s_win[kThreads / kWave][kFusedWin];
    double* sw = s_win[threadIdx.x / kWave];
    auto gpos = [](int pnt) {  // LDS slot (in doubles) of window point pnt (even)
        const int run = pnt / Q, g = (pnt % Q) / 2;
        return run * Q + ((g + run) % QG) * 2;
    };
#pragma unroll
    for (int r = 0; r < kFusedRows; ++r)
#pragma unroll
        for (int h = 0; h < P / 2; ++h)
            *reinterpret_cast<V2*>(sw + gpos(r * ROW + lane * P + 2 * h)) = V2{{x[r][2 * h], x[r][2 * h + 1]}};
    __builtin_amdgcn_wave_barrier();
    double y[Q];
#pragma unroll
    for (int g = 0; g < QG; ++g) {
        const V2 v = *reinterpret_cast<const V2*>(sw + lane * Q + ((g + lane) % QG) * 2);
        y[2 * g] = v.v[0];
        y[2 * g + 1] = v.v[1];
    }
#pragma unroll
    for (int t = 0; t < S; ++t) {
        // the window's outer neighbours (lane 0's left, lane 63's right) are
        // 0.0: they feed only the 2S points that are not written
        const double lft = dpp<DPP_WAVE_SHR1>(0.0, y[Q - 1]);
        const double rgt = dpp<DPP_WAVE_SHL1>(0.0, y[0]);
        double prev = lft;
#pragma unroll
        for (int e = 0; e < Q; ++e) {
            const double m = y[e];
            y[e] = heat(prev, m, e + 1 < Q ? y[e + 1] : rgt, c);
            prev = m;
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int g = 0; g < QG; ++g)
        *reinterpret_cast<V2*>(sw + lane * Q + ((g + lane) % QG) * 2) = V2{{y[2 * g], y[2 * g + 1]}};
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < kFusedRows; ++r)
#pragma unroll
        for (int h = 0; h < P / 2; ++h) {
            const V2 v = *reinterpret_cast<const V2*>(sw + gpos(r * ROW + lane * P + 2 * h));
            x[r][2 * h] = v.v[0];
            x[r][2 * h + 1] = v.v[1];
        }
#else
#pragma unroll
    for (int t = 0; t < S; ++t) {
        double L[kFusedRows], R[kFusedRows];
#pragma unroll
        for (int r = 0; r < kFusedRows; ++r) {
            // left of point 0: lane-1's last point; lane 0 takes lane 63's last point of row r-1
            const double lfill = r > 0 ? readlane(x[r - 1][P - 1], kWave - 1) : 0.0;
            L[r] = dpp<DPP_WAVE_SHR1>(lfill, x[r][P - 1]);
            // right of the last point: lane+1's point 0; lane 63 takes lane 0's point 0 of row r+1
            const double rfill = r + 1 < kFusedRows ? readlane(x[r + 1][0], 0) : 0.0;
            R[r] = dpp<DPP_WAVE_SHL1>(rfill, x[r][0]);
        }
#pragma unroll
        for (int r = 0; r < kFusedRows; ++r) {
            double prev = L[r];
#pragma unroll
            for (int e = 0; e < P; ++e) {
                const double m = x[r][e];
                const double right = e + 1 < P ? x[r][e + 1] : R[r];
                x[r][e] = heat(prev, m, right, c);
                prev = m;
            }
        }
    }
#endif

#pragma unroll
    for (int r = 0; r < kFusedRows; ++r)
#pragma unroll
        for (int h = 0; h < P / 2; ++h) {
            const int64_t i = w0 + r * ROW + lane * P + 2 * h;  // even when aligned
            const bool ok0 = i >= static_cast<int64_t>(o0) && i < static_cast<int64_t>(o1);
            const bool ok1 = i + 1 >= static_cast<int64_t>(o0) && i + 1 < static_cast<int64_t>(o1);
            if (aligned && ok0 && ok1) {
                V2 v;
                v.v[0] = x[r][2 * h];
                v.v[1] = x[r][2 * h + 1];
                *reinterpret_cast<V2*>(next + i) = v;
            } else {
                if (ok0) next[i] = x[r][2 * h];
                if (ok1) next[i + 1] = x[r][2 * h + 1];
            }
        }
}

int launch_fused(const double* cur, double* next, uint64_t n, uint64_t out_lo, uint64_t out_hi, const double* lh,
                 const double* rh, int steps, double c, hipStream_t s) {
    if (out_hi <= out_lo) return 0;
    const uint64_t OUT = kFusedWin - 2 * steps;
    const uint64_t waves = (out_hi - out_lo + OUT - 1) / OUT;
    const uint64_t blocks = (waves * kWave + kThreads - 1) / kThreads;
    // 16-B vector path: both buffers 16-B aligned and every window start even
    const bool aligned = (reinterpret_cast<uintptr_t>(cur) % 16 == 0) && (reinterpret_cast<uintptr_t>(next) % 16 == 0) &&
                         out_lo % 2 == 0;
    const dim3 g(static_cast<unsigned>(blocks)), b(kThreads);
    switch (steps) {
        case 2: hipLaunchKernelGGL(k_heat_fused<2>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 4: hipLaunchKernelGGL(k_heat_fused<4>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 6: hipLaunchKernelGGL(k_heat_fused<6>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 8: hipLaunchKernelGGL(k_heat_fused<8>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 10: hipLaunchKernelGGL(k_heat_fused<10>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 12: hipLaunchKernelGGL(k_heat_fused<12>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 14: hipLaunchKernelGGL(k_heat_fused<14>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        case 16: hipLaunchKernelGGL(k_heat_fused<16>, g, b, 0, s, cur, next, n, out_lo, out_hi, lh, rh, c, aligned); break;
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
    HPXHIP_CHECK_LAUNCH();
    return 0;
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

// nt periodic steps ping-ponging u0/u1: passes of up to
// HPXHIP_STENCIL_MAX_FUSED steps (even), a single step for an odd remainder;
// tiny rings step one at a time.  match_parity: give every planned chunk a
// pass count with the parity of its step count (an 8 becomes 6 + 2, or a 2
// becomes 1 + 1), so the result lands in u0 for even nt and in u1 for odd nt
// as hpxhip_stencil_heat_run promises; otherwise the fewest passes, and
// *flips (one per pass) says where the result is.
int run_passes(double* u0, double* u1, uint64_t n, uint64_t nt, double c, bool match_parity, hipStream_t s,
               uint64_t* flips) {
    const bool fuse = n >= 2 * static_cast<uint64_t>(kFusedWin);
    uint64_t done = 0;
    while (done < nt) {
        uint64_t passes[64];
        int np = 0;
        const uint64_t cap = fuse ? 60 * HPXHIP_STENCIL_MAX_FUSED : 64;
        const uint64_t chunk = nt - done < cap ? nt - done : cap;
        uint64_t r = chunk;
        while (fuse && r >= 2) {
            const uint64_t st = r >= HPXHIP_STENCIL_MAX_FUSED ? HPXHIP_STENCIL_MAX_FUSED : (r & ~uint64_t(1));
            passes[np++] = st;
            r -= st;
        }
        while (r > 0) {
            passes[np++] = 1;
            --r;
        }
        if (match_parity && static_cast<uint64_t>(np) % 2 != chunk % 2) {  // then some pass is >= 2
            int i = 0;
            while (passes[i] < 4 && i + 1 < np) ++i;
            const bool split_big = passes[i] >= 4;
            if (!split_big) {
                i = 0;
                while (passes[i] != 2) ++i;
            }
            for (int j = np; j > i + 1; --j) passes[j] = passes[j - 1];
            passes[i] -= split_big ? 2 : 1;
            passes[i + 1] = split_big ? 2 : 1;
            ++np;
        }
        for (int i = 0; i < np; ++i, ++*flips) {
            const double* cur = (*flips % 2 == 0) ? u0 : u1;
            double* nxt = (*flips % 2 == 0) ? u1 : u0;
            const int st = static_cast<int>(passes[i]);
            // periodic: left of point 0 is point n-1 (the last st points for
            // a fused pass), right of point n-1 is point 0
            const int rc = st == 1 ? launch_step(cur, nxt, n, cur + (n - 1), cur, c, s)
                                   : launch_fused(cur, nxt, n, 0, n, cur + (n - st), cur, st, c, s);
            if (rc) return rc;
        }
        done += chunk;
    }
    return 0;
}

}  // namespace

extern "C" {

int hpxhip_stencil_heat_step(const double* cur, double* next, uint64_t n, const double* left_halo_dev,
                             const double* right_halo_dev, double k, double dt, double dx, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_stencil_heat_step");
    if (n == 0) return 0;
    if (!cur || !next || !left_halo_dev || !right_halo_dev || cur == next) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if ((n / 2 + kThreads - 1) / kThreads > 0x7fffffffull) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    const double c = k * dt / (dx * dx);
    return launch_step(cur, next, n, left_halo_dev, right_halo_dev, c, s);
}

int hpxhip_stencil_heat_steps(const double* cur, double* next, uint64_t n, uint64_t out_lo, uint64_t out_hi,
                              const double* left_halo_dev, const double* right_halo_dev, int steps, double k,
                              double dt, double dx, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_stencil_heat_steps");
    if (out_hi > n || out_lo > out_hi) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (out_hi == out_lo) return 0;
    if (!cur || !next || !left_halo_dev || !right_halo_dev || cur == next) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (steps < 1 || steps > HPXHIP_STENCIL_MAX_FUSED || (steps > 1 && steps % 2)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    const double c = k * dt / (dx * dx);
    if (steps == 1) {
        // one step on [out_lo, out_hi): halos are the neighbouring points of cur or the halo arrays
        const double* l = out_lo == 0 ? left_halo_dev : cur + out_lo - 1;
        const double* r = out_hi == n ? right_halo_dev : cur + out_hi;
        return launch_step(cur + out_lo, next + out_lo, out_hi - out_lo, l, r, c, s);
    }
    return launch_fused(cur, next, n, out_lo, out_hi, left_halo_dev, right_halo_dev, steps, c, s);
}

int hpxhip_stencil_heat_run(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt, double dx,
                            hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_stencil_heat_run");
    if (n == 0 || nt == 0) return 0;
    if (!u0 || !u1 || u0 == u1) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    uint64_t flips = 0;
    return run_passes(u0, u1, n, nt, k * dt / (dx * dx), true, s, &flips);
}

int hpxhip_stencil_heat_run_fused(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt, double dx,
                                  int* result_in_u1, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_stencil_heat_run_fused");
    if (!result_in_u1) return HPXHIP_ERROR_INVALID_ARGUMENT;
    *result_in_u1 = 0;
    if (n == 0 || nt == 0) return 0;
    if (!u0 || !u1 || u0 == u1) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    uint64_t flips = 0;
    const int rc = run_passes(u0, u1, n, nt, k * dt / (dx * dx), false, s, &flips);
    *result_in_u1 = static_cast<int>(flips % 2);
    return rc;
}

}  // extern "C"
