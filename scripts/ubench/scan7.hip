// Microbenchmark (round 3): f64 inclusive plus-scan tile shapes and the deferred round carry
// (DEFER: round totals held wave-uniform, carry folded in at the store),
// and the fixed-association look-back (FIXED, reproducible FP scans); then
// (after FIXED shipped) tile shapes with several workgroups per CU; then
// (after the 512 x 16 shape shipped) 384- and 768-thread shapes.  The shipped
// FP scan runs 1024 threads x 12 rounds (16 spill 24 VGPRs: 4 waves/SIMD cap a
// wave at 128 registers).  Fewer threads per tile raise the register cap:
// 512 threads x 32 rounds (2 waves/SIMD, 256 VGPRs) and 256 x 64 (1 wave/SIMD)
// keep the 256-KiB tile; int64 at the same shapes for comparison.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I../../include scan7.hip -o scan7
#include <hpxhip/kernels/scan_kernel.hpp>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;

template <typename T> struct idc { __device__ T operator()(T x) const { return x; } };

template <typename T>
struct bench {
  using Conv = idc<T>;
  uint64_t N; T *in, *out; char* ws; uint32_t* err; hipEvent_t e0, e1;
  template <typename L> void run(const char* name, L launch, uint64_t check_tile) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 2.0 * sizeof(T) * N;
    bool ok = true;
    const uint64_t idx[5] = {0, check_tile - 1, check_tile, N / 2 + 12345, N - 1};
    for (uint64_t i : idx) { T h; CK(hipMemcpy(&h, out + i, sizeof(T), hipMemcpyDeviceToHost)); ok = ok && h == T(i + 1); }
    printf("%-44s min %7.3f ms med %7.3f ms  %7.1f GB/s (%5.1f%%) %s\n", name, t[0], t[7], B / t[0] / 1e6,
           B / t[0] / 1e6 / 80.0, ok ? "ok" : "MISMATCH");
    fflush(stdout);
  }
  template <int R, int TH, int MINW = 1, bool DEFER = true, bool FIXED = false>
  void shipped(const char* name) {
    const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
    const uint64_t ntiles = (N + tile - 1) / tile;
    const size_t total = 256 + ntiles * tile_state<T>::bytes_per_tile();
    tile_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      scan_detail::k_scan<T, Conv, op_plus, true, true, R, TH, true, MINW, false, 1, false, true, T, DEFER, FIXED><<<ntiles, TH>>>(
            in, out, N, Conv{}, op_plus{}, T(0), static_cast<const T*>(nullptr), reinterpret_cast<uint32_t*>(ws), st);
    }, tile);
  }
};

template <typename T>
__global__ void k_ones(T* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) p[i] = T(1);
}

int main() {
  const uint64_t N = 1ull << 30;
  char* ws; uint32_t* err; void *in, *out;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  bench<int64_t> bi{N, (int64_t*)in, (int64_t*)out, ws, err, e0, e1};
  bench<double> bd{N, (double*)in, (double*)out, ws, err, e0, e1};
  for (int rep = 0; rep < 2; ++rep) {
    k_ones<int64_t><<<8192, 256>>>((int64_t*)in, N); CK(hipDeviceSynchronize());
    bi.shipped<16, 512, 4, false, true>("i64 T512 R16 2/CU fixed (shipped)");
    bi.shipped<12, 384, 5, false, true>("i64 T384 R12 3/CU fixed");
    bi.shipped<16, 384, 4, false, true>("i64 T384 R16 2/CU fixed");
    bi.shipped<12, 512, 4, false, true>("i64 T512 R12 2/CU fixed");
    bi.shipped<20, 512, 3, false, true>("i64 T512 R20 1/CU fixed");
    bi.shipped<8, 768, 4, false, true>("i64 T768 R8 fixed");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
