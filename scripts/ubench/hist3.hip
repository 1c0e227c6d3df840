// Microbenchmark (round 4): the hybrid sort's first histogram in context.
// In the sort (profiles/r04_*) k_hist takes 1.71-1.73 ms right after the
// keys are generated, against 1.34-1.48 ms back to back in hist2.hip.  Here
// each shape is timed back to back and right after a fill of the keys
// (8 GiB written just before), 2^30 random u64, counts checked.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include hist3.hip -o hist3
#include <hpxhip/kernels/sort_kernel.hpp>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using namespace hpxhip::sort_detail;
using X = ordered_bits<uint64_t, false>;

__global__ void k_fill(uint64_t* p, uint64_t n, uint64_t seed) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; p[i] = z; }
}
__global__ void k_read(const vec<uint64_t, 2>* p, uint64_t n16, unsigned long long* out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const vec<uint64_t, 2> v = ld_stream(&p[i]);
    acc += v.v[0] ^ v.v[1];
  }
  if (acc == 0x123456789ull) *out = acc;
}

int main() {
  const uint64_t N = 1ull << 30;
  uint64_t* k; unsigned long long *hist, *bits, *xhist;
  CK(hipMalloc(&k, 8 * N)); CK(hipMalloc(&hist, 8 * 8 * 256)); CK(hipMalloc(&bits, 64)); CK(hipMalloc(&xhist, 8 * 512));
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int after_fill = 0; after_fill < 2; ++after_fill) {
      std::vector<float> t;
      for (int r = 0; r < 6; ++r) {
        CK(hipMemset(hist, 0, 8 * 8 * 256)); CK(hipMemset(xhist, 0, 8 * 512));
        CK(hipMemset(bits, 0, 8)); CK(hipMemset(bits + 1, 0xff, 8));
        if (after_fill) hipLaunchKernelGGL(k_fill, dim3(N / 256), dim3(256), 0, 0, k, N, 7 + r % 2);
        CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("%-44s %-18s min %7.3f ms med %7.3f ms\n", name, after_fill ? "after a fill" : "back to back", t[0], t[3]);
      fflush(stdout);
    }
  };
  hipLaunchKernelGGL(k_fill, dim3(N / 256), dim3(256), 0, 0, k, N, 7);
  for (int rep = 0; rep < 2; ++rep) {
    run("k_hist 256x4 D8 4 blk/CU (digit 7 + field)", [&] {
      hipLaunchKernelGGL((k_hist<uint64_t, X, 256, 4>), dim3(cus * 4), dim3(256), 0, 0, k, N, 7, 8, X{}, hist, bits, 47, xhist);
    });
    run("k_hist 1024x16 D2 2 blk/CU (shipped r04)", [&] {
      hipLaunchKernelGGL((k_hist<uint64_t, X, 1024, 16, 2>), dim3(cus * 2), dim3(1024), 0, 0, k, N, 7, 8, X{}, hist, bits, 47, xhist);
    });
    run("k_hist 512x8 D2 4 blk/CU", [&] {
      hipLaunchKernelGGL((k_hist<uint64_t, X, 512, 8, 2>), dim3(cus * 4), dim3(512), 0, 0, k, N, 7, 8, X{}, hist, bits, 47, xhist);
    });
    run("plain read of the keys (nt 16 B)", [&] {
      hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const vec<uint64_t, 2>*>(k), N / 2, hist);
    });
  }
  return 0;
}
