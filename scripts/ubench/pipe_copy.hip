// Microbenchmark: is the scan's one-tile-per-workgroup memory pattern the
// limit?  Persistent tile copies with the next tile's loads issued before the
// current tile's stores (software pipelined, registers double-buffered)
// against the flat copy, 2^30 x 8 B.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 pipe_copy.hip -o pipe_copy
#include "../../hpx_amd/csrc/common.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using V = vec<uint64_t, 2>;

__global__ __launch_bounds__(64) void k_flat(const V* in, V* out, uint64_t nv) {
    const uint64_t i = blockIdx.x * 64ull + threadIdx.x;
    if (i < nv) st_stream(&out[i], ld_stream(&in[i]));
}

template <int R, int TH>
__device__ __forceinline__ void load_tile(V (&x)[R], const V* in, uint64_t t) {
    const V* src = in + t * (uint64_t(R) * TH);
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_stream(&src[r * TH + threadIdx.x]);
}
template <int R, int TH>
__device__ __forceinline__ void store_tile(V (&x)[R], V* out, uint64_t t) {
    V* dst = out + t * (uint64_t(R) * TH);
#pragma unroll
    for (int r = 0; r < R; ++r) st_stream(&dst[r * TH + threadIdx.x], x[r]);
}

// tiles b, b+G, b+2G, ... per block; loads of the next tile before the stores of this one
template <int R, int TH>
__global__ __launch_bounds__(TH) void k_pipe(const V* in, V* out, uint64_t ntiles) {
    const uint64_t G = gridDim.x;
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    V a[R], b[R];
    load_tile<R, TH>(a, in, t);
    while (true) {
        const bool hb = t + G < ntiles;
        if (hb) load_tile<R, TH>(b, in, t + G);
        store_tile<R, TH>(a, out, t);
        if (!hb) break;
        t += G;
        const bool ha = t + G < ntiles;
        if (ha) load_tile<R, TH>(a, in, t + G);
        store_tile<R, TH>(b, out, t);
        if (!ha) break;
        t += G;
    }
}

// one tile per block (the shipped scan's pattern without the scan)
template <int R, int TH>
__global__ __launch_bounds__(TH) void k_tile(const V* in, V* out) {
    V a[R];
    load_tile<R, TH>(a, in, blockIdx.x);
    store_tile<R, TH>(a, out, blockIdx.x);
}

// one tile per block, wave w of tile t takes the wave-chunk (w + S*t) mod WAVES
// of the tile (rounds contiguous per wave, as the scan's layout)
template <int R, int TH, int S>
__global__ __launch_bounds__(TH) void k_tile_rot(const V* in, V* out) {
    constexpr int WAVES = TH / 64;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int chunk = (wave + S * static_cast<int>(blockIdx.x)) % WAVES;
    const uint64_t base = uint64_t(blockIdx.x) * R * TH + uint64_t(chunk) * R * 64;
    V a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = ld_stream(&in[base + r * 64 + lane]);
#pragma unroll
    for (int r = 0; r < R; ++r) st_stream(&out[base + r * 64 + lane], a[r]);
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
        printf("%-44s min %7.3f ms med %7.3f ms  %7.1f GB/s\n", name, ts[0], ts[4], 16.0 * n / ts[0] / 1e6);
        fflush(stdout);
    };
    bench("flat copy 64x1", [&] { hipLaunchKernelGGL(k_flat, dim3(unsigned(nv / 64)), dim3(64), 0, 0, in, out, nv); });
    bench("tile 1024x16 (scan shape, 1/CU)", [&] {
        hipLaunchKernelGGL((k_tile<16, 1024>), dim3(unsigned(nv / (16 * 1024))), dim3(1024), 0, 0, in, out); });
    bench("tile 512x16 (2/CU)", [&] {
        hipLaunchKernelGGL((k_tile<16, 512>), dim3(unsigned(nv / (16 * 512))), dim3(512), 0, 0, in, out); });
#define ROT0(R, TH) bench("tile " #TH "x" #R " wave-chunks", [&] { \
        hipLaunchKernelGGL((k_tile_rot<R, TH, 0>), dim3(unsigned(nv / (R * TH))), dim3(TH), 0, 0, in, out); })
    ROT0(16, 1024); ROT0(8, 1024); ROT0(4, 1024); ROT0(16, 512); ROT0(8, 512); ROT0(4, 512);
    ROT0(16, 256); ROT0(8, 256); ROT0(4, 256); ROT0(2, 256); ROT0(32, 256); ROT0(12, 1024);
    return 0;
}
