// Microbenchmark (round 2, session 2): tile ids from the atomic counter (one
// dequeue round trip before a workgroup can address its tile) against
// blockIdx order (workgroups are dispatched in id order, so every resident
// tile's predecessors were dispatched before it), 2^30 int64 / f64 inclusive
// plus-scan with the shipped kernel, plus 2-per-CU shapes in both orders.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include scan6.hip -o scan6
#include "../../hpx_amd/csrc/scan_kernel.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;

template <typename T>
struct bench {
  using Conv = unary_fn<HPXHIP_U_IDENTITY, T>;
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
  template <int R, int TH, bool DYN, int MINW = 1, int LBK = 1, bool NTS = false>
  void shipped(const char* name) {
    const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
    const uint64_t ntiles = (N + tile - 1) / tile;
    const size_t total = align_up(256 + ntiles * tile_state<T>::bytes_per_tile(), 256);
    tile_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      scan_detail::k_scan<T, Conv, op_plus, true, true, R, TH, true, MINW, false, LBK, DYN, NTS><<<ntiles, TH>>>(
            in, out, N, Conv{0, 0}, op_plus{}, T(0), nullptr, reinterpret_cast<uint32_t*>(ws), st);
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
    bi.shipped<16, 1024, false, 1, 1, true>("i64 T1024 R16 (shipped)");
    bi.shipped<16, 512, false, 2, 1, true>("i64 T512 R16 2/CU");
    bi.shipped<8, 512, false, 4, 1, true>("i64 T512 R8 4/CU");
    bi.shipped<16, 256, false, 4, 1, true>("i64 T256 R16 4/CU");
    bi.shipped<8, 1024, false, 2, 1, true>("i64 T1024 R8 2/CU");
    bi.shipped<16, 512, false, 2, 2, true>("i64 T512 R16 2/CU K2");
    bi.shipped<16, 256, false, 4, 4, true>("i64 T256 R16 4/CU K4");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
