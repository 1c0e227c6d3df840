// Microbenchmark: 1d_stencil heat step variants (2^30 points, 16 B/point):
// block size, nontemporal main loads / stores (edge-lane neighbour loads keep
// the default policy so they hit the lines the adjacent wave just fetched).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I../../include stencil.hip -o stencil
#include "../../hpx_amd/csrc/common.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;

__device__ __forceinline__ double heat(double l, double m, double r, double c) { return m + c * (l - 2 * m + r); }

template <int BT, bool NTL, bool NTS>
__global__ __launch_bounds__(BT) void k_heat(const double* __restrict__ cur, double* __restrict__ next, uint64_t n,
                                             uint64_t nvec, const double* __restrict__ lh, const double* __restrict__ rh,
                                             double c) {
  using V2 = vec<double, 2>;
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * BT + threadIdx.x;
  const int lane = lane_id();
  const bool in = g < nvec;
  V2 x = {{0.0, 0.0}};
  if (in) x = NTL ? ld_stream(&reinterpret_cast<const V2*>(cur)[g]) : reinterpret_cast<const V2*>(cur)[g];
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
  if (NTS) st_stream(&reinterpret_cast<V2*>(next)[g], y);
  else reinterpret_cast<V2*>(next)[g] = y;
}

int main() {
  const uint64_t n = 1ull << 30, nvec = n / 2;
  double *a, *b;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
  CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, auto f) {
    f(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    printf("%-28s min %7.3f ms med %7.3f ms  %7.1f GB/s\n", name, t[0], t[7], 16.0 * n / t[0] / 1e6);
    fflush(stdout);
  };
#define V_(BT, L, S) bench("heat BT" #BT " ntload=" #L " ntstore=" #S, [&] { \
    hipLaunchKernelGGL((k_heat<BT, L, S>), dim3(nvec / BT), dim3(BT), 0, 0, a, b, n, nvec, a + n - 1, a, 0.5); })
  for (int rep = 0; rep < 2; ++rep) {
    V_(256, false, false); V_(256, true, false); V_(256, false, true); V_(256, true, true);
    V_(64, false, false); V_(64, true, true); V_(128, true, true); V_(512, true, true); V_(1024, true, true);
  }
  return 0;
}
