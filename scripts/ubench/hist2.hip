// Microbenchmark (round 2, session 3): the hybrid sort's first histogram
// (top byte + the 9-bit field under it, 2^30 random u64 keys).  The shipped
// k_hist sizes its LDS for all eight digits (4 lane copies, 4 blocks/CU);
// the variant here holds only the two counted fields, so it can afford more
// copies or more blocks per CU.  Counts are checked against the shipped kernel.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include hist2.hip -o hist2
#include "../../hpx_amd/csrc/sort_kernel.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using namespace hpxhip::sort_detail;
using X = ordered_bits<uint64_t, false>;

template <int THREADS, int COPIES>
__global__ __launch_bounds__(THREADS) void k_hist_top(const uint64_t* __restrict__ keys, uint64_t n, X xf,
                                                       unsigned long long* __restrict__ hist, int xshift,
                                                       unsigned long long* __restrict__ xhist) {
  __shared__ uint32_t h[kRadix * COPIES];
  __shared__ uint32_t hx[kXBins * COPIES];
  for (int i = threadIdx.x; i < kRadix * COPIES; i += THREADS) h[i] = 0;
  for (int i = threadIdx.x; i < kXBins * COPIES; i += THREADS) hx[i] = 0;
  __syncthreads();
  using VT = vec<uint64_t, 2>;
  const uint32_t copy = threadIdx.x % COPIES;
  const uint64_t nvec = n / 2;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * THREADS + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * THREADS;
  const VT* vk = reinterpret_cast<const VT*>(keys);
  for (uint64_t i = tid; i < nvec; i += stride * 4) {
    VT x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < nvec) x[u] = ld_stream(&vk[i + u * stride]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < nvec)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint64_t b = xf(x[u].v[e]);
          atomicAdd(&h[static_cast<uint32_t>(b >> 56) * COPIES + copy], 1u);
          atomicAdd(&hx[static_cast<uint32_t>((b >> xshift) & (kXBins - 1)) * COPIES + copy], 1u);
        }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kRadix; i += THREADS) {
    uint32_t c = 0;
    for (int k = 0; k < COPIES; ++k) c += h[i * COPIES + k];
    if (c) atomicAdd(&hist[7 * kRadix + i], static_cast<unsigned long long>(c));
  }
  for (int i = threadIdx.x; i < kXBins; i += THREADS) {
    uint32_t c = 0;
    for (int k = 0; k < COPIES; ++k) c += hx[i * COPIES + k];
    if (c) atomicAdd(&xhist[i], static_cast<unsigned long long>(c));
  }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = (i + 7) * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; p[i] = z; }
}

int main() {
  const uint64_t N = 1ull << 30;
  uint64_t* k; unsigned long long *hist, *bits, *xhist;
  CK(hipMalloc(&k, 8 * N)); CK(hipMalloc(&hist, 8 * 8 * 256)); CK(hipMalloc(&bits, 64)); CK(hipMalloc(&xhist, 8 * 512));
  hipLaunchKernelGGL(k_fill, dim3(N / 256), dim3(256), 0, 0, k, N);
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<unsigned long long> ref(256 + 512), got(256 + 512);
  auto run = [&](const char* name, auto launch, bool check) {
    std::vector<float> t;
    for (int r = 0; r < 8; ++r) {
      CK(hipMemset(hist, 0, 8 * 8 * 256)); CK(hipMemset(xhist, 0, 8 * 512));
      CK(hipMemset(bits, 0, 8)); CK(hipMemset(bits + 1, 0xff, 8));
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
    }
    CK(hipMemcpy(got.data(), hist + 7 * 256, 256 * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data() + 256, xhist, 512 * 8, hipMemcpyDeviceToHost));
    if (!check) ref = got;
    std::sort(t.begin(), t.end());
    printf("%-40s min %7.3f ms med %7.3f ms %s\n", name, t[0], t[4], check ? (got == ref ? "counts ok" : "COUNT MISMATCH") : "(reference)");
    fflush(stdout);
  };
  run("shipped k_hist 256x4 copies, 4 blk/CU", [&] {
    hipLaunchKernelGGL((k_hist<uint64_t, X, 256, 4>), dim3(cus * 4), dim3(256), 0, 0, k, N, 7, 8, X{}, hist, bits, 47, xhist);
  }, false);
  run("top-only 256x4 copies, 4 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<256, 4>), dim3(cus * 4), dim3(256), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 256x4 copies, 8 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<256, 4>), dim3(cus * 8), dim3(256), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 256x8 copies, 8 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<256, 8>), dim3(cus * 8), dim3(256), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 256x16 copies, 4 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<256, 16>), dim3(cus * 4), dim3(256), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 512x8 copies, 4 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<512, 8>), dim3(cus * 4), dim3(512), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 1024x16 copies, 2 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<1024, 16>), dim3(cus * 2), dim3(1024), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  run("top-only 256x32 copies, 2 blk/CU", [&] { hipLaunchKernelGGL((k_hist_top<256, 32>), dim3(cus * 2), dim3(256), 0, 0, k, N, X{}, hist, 47, xhist); }, true);
  return 0;
}
