// Microbenchmark: the shipped scan kernel (scan_kernel.hpp) at several tile
// shapes, with and without the look-back (ablation), 2^30 int64, all in one
// process so the comparison shares one box.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include scan.hip -o scan
#include "../../hpx_amd/csrc/scan_kernel.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using T = int64_t;
using Conv = unary_fn<HPXHIP_U_IDENTITY, T>;

int main() {
  const uint64_t N = 1ull << 30;
  T *in, *out; char* ws; uint32_t* err;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMemset(in, 1, N * 8)); CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 16.0 * N;
    printf("%-34s min %7.3f ms med %7.3f ms  %7.1f GB/s (med %7.1f)\n", name, t[0], t[7], B / t[0] / 1e6, B / t[7] / 1e6);
    fflush(stdout);
  };
  auto variant = [&](auto rounds_c, auto threads_c, auto lb_c, const char* name, auto minw_c, auto early_c) {
    constexpr bool EA = decltype(early_c)::value;
    constexpr int MW = decltype(minw_c)::value;
    constexpr int R = decltype(rounds_c)::value;
    constexpr int TH = decltype(threads_c)::value;
    constexpr bool LB = decltype(lb_c)::value;
    const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
    const uint64_t ntiles = (N + tile - 1) / tile;
    const size_t total = align_up(256 + ntiles * tile_state<T>::bytes_per_tile(), 256);
    tile_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      scan_detail::k_scan<T, Conv, op_plus, true, true, R, TH, LB, MW, EA><<<ntiles, TH>>>(
            in, out, N, Conv{0, 0}, op_plus{}, T(0), nullptr, reinterpret_cast<uint32_t*>(ws), st);
    });
    {  // spot check: in = 0x0101..01 everywhere, so out[i] = (i + 1) * that
      const uint64_t v = 0x0101010101010101ull, idx[4] = {0, tile - 1, N / 2 + 12345, N - 1};
      bool ok = true;
      for (uint64_t i : idx) { uint64_t h; CK(hipMemcpy(&h, out + i, 8, hipMemcpyDeviceToHost)); ok = ok && h == (i + 1) * v; }
      printf("   %s check %s\n", name, ok ? "ok" : "MISMATCH");
    }
  };
#define V_(R, TH, LB, NAME) variant(std::integral_constant<int, R>{}, std::integral_constant<int, TH>{}, \
    std::integral_constant<bool, LB>{}, NAME, std::integral_constant<int, 1>{}, std::false_type{})
#define VW(R, TH, LB, NAME, MW) variant(std::integral_constant<int, R>{}, std::integral_constant<int, TH>{}, \
    std::integral_constant<bool, LB>{}, NAME, std::integral_constant<int, MW>{}, std::false_type{})
#define VE(R, TH, NAME) variant(std::integral_constant<int, R>{}, std::integral_constant<int, TH>{}, \
    std::true_type{}, NAME, std::integral_constant<int, 1>{}, std::true_type{})
  for (int rep = 0; rep < 3; ++rep) {
    V_(16, 1024, true, "T1024 R16 lookback (shipped)");
    VE(16, 1024, "T1024 R16 lookback early-agg");
    V_(16, 1024, false, "T1024 R16 no-lookback");
    VE(8, 1024, "T1024 R8 lookback early-agg");
    VE(12, 1024, "T1024 R12 lookback early-agg");
    VE(16, 512, "T512 R16 lookback early-agg");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
