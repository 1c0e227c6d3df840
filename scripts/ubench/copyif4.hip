// Microbenchmark: the shipped copy_if kernel (copy_if_kernel.hpp) at several
// tile shapes, 2^30 int64, predicate !(x < 0) on ~50 % hits, one process.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include copyif4.hip -o copyif4
#include "../../hpx_amd/csrc/copy_if_kernel.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using namespace hpxhip::copy_if_detail;
using T = int64_t;
using P = pred_fn<HPXHIP_P_NOT_LT, T>;

__global__ void k_fill_blocky(T* p, uint64_t n) {  // sign constant over aligned 128-element blocks
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = (i >> 7) * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29;
    p[i] = (z >> 63) ? -(T)(i + 1) : (T)i; }
}
__global__ void k_fill(T* p, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; p[i] = (T)z; }
}

int main() {
  const uint64_t N = 1ull << 30;
  T *in, *out; char* ws; uint32_t* err; uint64_t* cnt;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMalloc(&cnt, 64));
  T* blocky; CK(hipMalloc(&blocky, N * 8));
  hipLaunchKernelGGL(k_fill_blocky, dim3(N / 256), dim3(256), 0, 0, blocky, N);
  hipLaunchKernelGGL(k_fill, dim3(N / 256), dim3(256), 0, 0, in, N);
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    uint64_t c = 0; CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 8.0 * N + 8.0 * c;
    printf("%-30s min %7.3f ms med %7.3f ms  %7.1f GB/s (med %7.1f)  hits %.4f\n", name, t[0], t[7], B / t[0] / 1e6,
           B / t[7] / 1e6, double(c) / N);
    fflush(stdout);
  };
  auto variant = [&](auto rounds_c, auto abl_c, const char* name) {
    constexpr int R = decltype(rounds_c)::value;
    constexpr int A = decltype(abl_c)::value;
    const uint64_t ntiles = (N + tile_elems<T, R>() - 1) / tile_elems<T, R>();
    const size_t total = align_up(256 + ntiles * tile_state<uint64_t>::bytes_per_tile(), 256);
    tile_state<uint64_t> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      k_copy_if<T, P, true, R, 4, A><<<ntiles, kThreads>>>(in, out, N, P{0}, cnt, reinterpret_cast<uint32_t*>(ws), st, ntiles);
    });
  };
  auto v = [&](auto dyn_c, auto nt_c, const char* name, auto abl_c) {
    constexpr int R = 8;
    constexpr int A = decltype(abl_c)::value;
    constexpr bool DYN = decltype(dyn_c)::value;
    constexpr bool NT = decltype(nt_c)::value;
    using SV = uint32_t;
    const uint64_t ntiles = (N + tile_elems<T, R>() - 1) / tile_elems<T, R>();
    const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
    tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      k_copy_if<T, P, true, R, 4, A, SV, DYN, NT><<<ntiles, kThreads>>>(in, out, N, P{0}, cnt, reinterpret_cast<uint32_t*>(ws), st, ntiles);
    });
  };
  using BT = std::true_type;
  using BF = std::false_type;
  using A0 = std::integral_constant<int, 0>;
  using A1 = std::integral_constant<int, 1>;
  using A4 = std::integral_constant<int, 4>;
  using A5 = std::integral_constant<int, 5>;
  for (int rep = 0; rep < 2; ++rep) {
    v(BT{}, BF{}, "shipped (atomic)", A0{});
    v(BT{}, BF{}, "atomic, no look-back", A1{});
    v(BT{}, BF{}, "atomic, no write-out", A4{});
    v(BT{}, BF{}, "atomic, neither", A5{});
    v(BF{}, BF{}, "blockIdx", A0{});
    v(BF{}, BF{}, "blockIdx, no look-back", A1{});
    v(BF{}, BF{}, "blockIdx, no write-out", A4{});
    v(BF{}, BF{}, "blockIdx, neither", A5{});
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
