// Microbenchmark (round 4): the STREAM triad's "placement lottery".  The
// same triad kernel over 2^30 doubles runs 3.76-3.84 ms on some array sets
// and 4.05-4.14 on others (profiles/r03_*).  (A) one allocation holding b, c,
// a back to back with relative skews between them; (B) separately allocated
// arrays, re-allocated several times (the lottery itself), with their
// addresses.  Kernel: one 16-B vector per thread per array, nt loads/stores
// (the shipped k_binary geometry, 256-thread blocks).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include skew.hip -o skew
#include <hpxhip/kernels/common.hpp>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using VT = vec<double, 2>;

__global__ __launch_bounds__(256) void k_triad(const VT* b, const VT* c, VT* a, uint64_t nv, double s) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nv) return;
  const VT x = ld_stream(&b[i]), y = ld_stream(&c[i]);
  VT z; z.v[0] = x.v[0] + y.v[0] * s; z.v[1] = x.v[1] + y.v[1] * s;
  st_stream(&a[i], z);
}
__global__ void k_init(double* p, uint64_t n, double v) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) p[i] = v;
}

static hipEvent_t e0, e1;
float triad(double* a, double* b, double* c, uint64_t n) {
  const uint64_t nv = n / 2;
  std::vector<float> t;
  for (int r = 0; r < 9; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_triad, dim3(nv / 256), dim3(256), 0, 0, (const VT*)b, (const VT*)c, (VT*)a, nv, 3.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[1];  // second best of 9 (the first call included)
}

int main() {
  const uint64_t n = 1ull << 30, B = n * 8;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  {
    char* base;
    const uint64_t slack = 64ull << 20;
    CK(hipMalloc(&base, 3 * B + 3 * slack));
    printf("(A) one allocation at %p, b at 0, c at 8 GiB + sc, a at 16 GiB + sc + sa\n", (void*)base);
    const uint64_t skews[][2] = {{0, 0}, {256, 512}, {4096, 8192}, {65536, 131072}, {1 << 20, 2 << 20},
                                 {2 << 20, 4 << 20}, {3 << 20, 6 << 20}, {(2 << 20) + 4096, (4 << 20) + 8192},
                                 {16 << 20, 32 << 20}};
    for (auto& sk : skews) {
      double* b = (double*)base;
      double* c = (double*)(base + B + sk[0]);
      double* a = (double*)(base + 2 * B + sk[0] + sk[1]);
      k_init<<<4096, 256>>>(b, n, 1.0); k_init<<<4096, 256>>>(c, n, 2.0); CK(hipDeviceSynchronize());
      const float ms = triad(a, b, c, n);
      printf("  skew c %9llu  a %9llu   %7.3f ms  %7.1f GB/s\n", (unsigned long long)sk[0], (unsigned long long)sk[1], ms,
             24.0 * n / ms / 1e6);
      fflush(stdout);
    }
    CK(hipFree(base));
  }
  printf("(B) separate allocations, re-allocated\n");
  for (int rep = 0; rep < 8; ++rep) {
    double *a, *b, *c, *pad = nullptr;
    if (rep & 1) CK(hipMalloc(&pad, (uint64_t(rep) + 1) << 21));  // shifts the next allocations
    CK(hipMalloc(&a, B)); CK(hipMalloc(&b, B)); CK(hipMalloc(&c, B));
    k_init<<<4096, 256>>>(b, n, 1.0); k_init<<<4096, 256>>>(c, n, 2.0); CK(hipDeviceSynchronize());
    const float ms = triad(a, b, c, n);
    printf("  a %p b %p c %p   %7.3f ms  %7.1f GB/s\n", (void*)a, (void*)b, (void*)c, ms, 24.0 * n / ms / 1e6);
    fflush(stdout);
    CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c)); if (pad) CK(hipFree(pad));
  }
  return 0;
}
