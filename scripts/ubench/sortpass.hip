// Microbenchmark: one onesweep pass (shipped kernel, sort_kernel.hpp) over
// 2^30 random uint64 keys at several tile shapes / look-back modes.
#include "../../hpx_amd/csrc/sort_kernel.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using namespace hpxhip::sort_detail;
using U = uint64_t;
using X = ordered_bits<uint64_t, false>;

__global__ void gen(U* k, uint64_t n) {
  uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i < n) { uint64_t z = i + 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; k[i] = z ^ (z >> 31); }
}

int main() {
  const uint64_t N = 1ull << 30;
  U *kin, *kout; unsigned long long *hist, *start; uint32_t *lbws, *err;
  CK(hipMalloc(&kin, N * 8)); CK(hipMalloc(&kout, N * 8)); CK(hipMalloc(&hist, 8 * 256 * 8));
  CK(hipMalloc(&start, 9 * 256 * 8)); CK(hipMalloc(&lbws, 256 + (N / 4096 + 1) * 256 * 4)); CK(hipMalloc(&err, 64));
  CK(hipMemset(err, 0, 64)); CK(hipMemset(hist, 0, 8 * 256 * 8));

  gen<<<N / 256, 256>>>(kin, N);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    printf("%-40s min %7.3f ms med %7.3f ms  %7.1f GB/s\n", name, t[0], t[3], bytes / t[0] / 1e6);
  };
  run("hist (8 passes)", 8.0 * N, [&] { CK(hipMemsetAsync(hist, 0, 8*256*8, 0));
      k_hist<U, X, 256><<<512, 256>>>(kin, N, 0, 8, X{}, hist, start + 8 * 256, -1, nullptr); });
  run("hist (8 passes) 1024 blocks", 8.0 * N, [&] { CK(hipMemsetAsync(hist, 0, 8*256*8, 0));
      k_hist<U, X, 256><<<1024, 256>>>(kin, N, 0, 8, X{}, hist, start + 8 * 256, -1, nullptr); });
  k_bin_offsets<256><<<8, 256>>>(hist, start);
  CK(hipDeviceSynchronize());
  auto pass = [&](auto th_c, auto it_c, auto lb_c, const char* name) {
    constexpr int TH = decltype(th_c)::value, IT = decltype(it_c)::value, LBB = decltype(lb_c)::value;
    const uint64_t tile = TH * IT, ntiles = (N + tile - 1) / tile;
    run(name, 16.0 * N, [&] {
      CK(hipMemsetAsync(lbws, 0, 256 + ntiles * 256 * 4, 0));
      k_onesweep<U, uint32_t, false, uint32_t, X, TH, IT, LBB><<<ntiles, TH>>>(kin, kout, nullptr, nullptr, N, 0, start,
          lbws + 64, lbws, err, X{});
    });
  };
#define P_(TH, IT, LBB, NAME) pass(std::integral_constant<int, TH>{}, std::integral_constant<int, IT>{}, std::integral_constant<int, LBB>{}, NAME)
  for (int rep = 0; rep < 2; ++rep) {
  P_(256, 16, 8, "T256 I16 B8");
  P_(512, 16, 8, "T512 I16 B8");
  P_(512, 16, 4, "T512 I16 B4");
  P_(512, 16, 16, "T512 I16 B16");
  P_(512, 16, 0, "T512 I16 no-lookback");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
