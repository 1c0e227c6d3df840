// Microbenchmark (round 2, session 2): what makes a tile-per-workgroup copy
// slower than the flat copy?  2^30 x 8 B copies, 16-B nt loads and stores.
//   flat        one vector per thread, one load then one store
//   wc          wave chunks (the scan layout): wave w of tile t owns R
//               contiguous 1-KiB rounds; all R loads in flight, then R stores
//   wc-thr G    the same, at most G loads of a wave in flight (sliding window)
//   wc-stream   wave chunks, each round stored as soon as it arrives (the
//               layout without holding the tile)
//   wc-persist  wave-chunk tiles walked by a resident grid (tile += grid)
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tile3.hip -o tile3
#include "../../hpx_amd/csrc/common.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using V = vec<uint64_t, 2>;

template <int TH>
__global__ __launch_bounds__(TH) void k_flat(const V* in, V* out, uint64_t nv) {
    const uint64_t i = blockIdx.x * uint64_t(TH) + threadIdx.x;
    if (i < nv) st_stream(&out[i], ld_stream(&in[i]));
}

template <int R, int TH>
__device__ __forceinline__ uint64_t wc_base(uint64_t tile) {
    const int wave = threadIdx.x / 64;
    return tile * uint64_t(R) * TH + uint64_t(wave) * R * 64 + (threadIdx.x % 64);
}

template <int R, int TH>
__global__ __launch_bounds__(TH) void k_wc(const V* in, V* out) {
    const uint64_t b = wc_base<R, TH>(blockIdx.x);
    V a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = ld_stream(&in[b + r * 64]);
#pragma unroll
    for (int r = 0; r < R; ++r) st_stream(&out[b + r * 64], a[r]);
}

// Sliding window: load r+G is issued only after load r has returned (the
// asm barrier on a[r] forces the wait at that point).
template <int R, int TH, int G>
__global__ __launch_bounds__(TH) void k_wc_thr(const V* in, V* out) {
    const uint64_t b = wc_base<R, TH>(blockIdx.x);
    V a[R];
#pragma unroll
    for (int r = 0; r < G; ++r) a[r] = ld_stream(&in[b + r * 64]);
#pragma unroll
    for (int r = G; r < R; ++r) {
        asm volatile("" : "+v"(a[r - G].v[0]));
        a[r] = ld_stream(&in[b + r * 64]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) st_stream(&out[b + r * 64], a[r]);
}

template <int R, int TH>
__global__ __launch_bounds__(TH) void k_wc_stream(const V* in, V* out) {
    const uint64_t b = wc_base<R, TH>(blockIdx.x);
    V a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = ld_stream(&in[b + r * 64]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        asm volatile("" : "+v"(a[r].v[0]));
        st_stream(&out[b + r * 64], a[r]);
    }
}

template <int R, int TH>
__global__ __launch_bounds__(TH) void k_wc_persist(const V* in, V* out, uint64_t ntiles) {
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t b = wc_base<R, TH>(t);
        V a[R];
#pragma unroll
        for (int r = 0; r < R; ++r) a[r] = ld_stream(&in[b + r * 64]);
#pragma unroll
        for (int r = 0; r < R; ++r) st_stream(&out[b + r * 64], a[r]);
    }
}

int main() {
    const uint64_t n = 1ull << 30, nv = n / 2;
    V *in, *out;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&out, n * 8));
    CK(hipMemset(in, 1, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto bench = [&](const char* name, auto f) {
        f();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int r = 0; r < 9; ++r) {
            CK(hipEventRecord(e0));
            f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-40s min %7.3f ms med %7.3f ms  %7.1f GB/s\n", name, ts[0], ts[4], 16.0 * n / ts[0] / 1e6);
        fflush(stdout);
    };
    for (int pass = 0; pass < 2; ++pass) {
        bench("flat 64x1", [&] { hipLaunchKernelGGL(k_flat<64>, dim3(unsigned(nv / 64)), dim3(64), 0, 0, in, out, nv); });
        bench("flat 1024x1", [&] {
            hipLaunchKernelGGL(k_flat<1024>, dim3(unsigned(nv / 1024)), dim3(1024), 0, 0, in, out, nv); });
#define WC(R, TH) bench("wc " #TH "x" #R, [&] { \
        hipLaunchKernelGGL((k_wc<R, TH>), dim3(unsigned(nv / (R * TH))), dim3(TH), 0, 0, in, out); })
#define THR(R, TH, G) bench("wc-thr " #TH "x" #R " G" #G, [&] { \
        hipLaunchKernelGGL((k_wc_thr<R, TH, G>), dim3(unsigned(nv / (R * TH))), dim3(TH), 0, 0, in, out); })
#define STR(R, TH) bench("wc-stream " #TH "x" #R, [&] { \
        hipLaunchKernelGGL((k_wc_stream<R, TH>), dim3(unsigned(nv / (R * TH))), dim3(TH), 0, 0, in, out); })
#define PER(R, TH, K) bench("wc-persist " #TH "x" #R " grid " #K "xCU", [&] { \
        hipLaunchKernelGGL((k_wc_persist<R, TH>), dim3(unsigned(K * cus)), dim3(TH), 0, 0, in, out, nv / (R * TH)); })
        WC(16, 1024); WC(1, 1024); WC(2, 1024); WC(4, 256); WC(1, 64); WC(4, 64); WC(16, 64);
        THR(16, 1024, 1); THR(16, 1024, 2); THR(16, 1024, 4); THR(16, 1024, 8);
        STR(16, 1024); STR(4, 256);
        PER(16, 1024, 1); PER(4, 256, 8); PER(1, 1024, 2);
    }
    return 0;
}
