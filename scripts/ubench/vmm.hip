// Microbenchmark (round 5): does physical mapping decide
// the STREAM triad's "placement lottery"?  The same triad kernel over three
// 2^30-double arrays runs 3.76-3.84 ms on some array sets and 4.05-4.14 on
// others (profiles/r02_ubench_triad_placement.log, r04_ubench_triad_skew.log);
// the virtual address pattern does not decide it.  Here the arrays are built
// through HIP's virtual-memory API -- hipMemCreate of physical chunks of G
// bytes, mapped back to back into one reserved range per array -- for G from
// the allocation granularity to 8 GiB, alternated with plain hipMalloc, and
// re-allocated several times per mode.  Run it in several fresh processes:
// a mode that removes the slow outcome shows only 3.7x-3.8x ms rows.
// Kernel: the shipped k_binary geometry (256-thread blocks, one 16-B vector
// per thread per array, nt loads and stores).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include vmm.hip -o vmm
#include <hpxhip/kernels/common.hpp>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
static float triad(double* a, double* b, double* c, uint64_t n) {
  const uint64_t nv = n / 2;
  std::vector<float> t;
  for (int r = 0; r < 9; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_triad, dim3(nv / 256), dim3(256), 0, 0, (const VT*)b, (const VT*)c, (VT*)a, nv, 3.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[1];  // second best of 9
}

struct vmm_array {
  void* va = nullptr;
  uint64_t bytes = 0, chunk = 0;
  std::vector<hipMemGenericAllocationHandle_t> h;
};

static vmm_array vmm_alloc(uint64_t bytes, uint64_t chunk) {
  vmm_array r;
  r.bytes = bytes; r.chunk = chunk;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  CK(hipMemAddressReserve(&r.va, bytes, 0, nullptr, 0));
  for (uint64_t off = 0; off < bytes; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    CK(hipMemCreate(&h, chunk, &prop, 0));
    CK(hipMemMap(static_cast<char*>(r.va) + off, chunk, 0, h, 0));
    r.h.push_back(h);
  }
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(r.va, bytes, &acc, 1));
  return r;
}
static void vmm_free(vmm_array& r) {
  for (uint64_t i = 0; i < r.h.size(); ++i) {
    CK(hipMemUnmap(static_cast<char*>(r.va) + i * r.chunk, r.chunk));
    CK(hipMemRelease(r.h[i]));
  }
  CK(hipMemAddressFree(r.va, r.bytes));
  r.h.clear();
}

int main(int argc, char** argv) {
  const uint64_t n = 1ull << 30, B = n * 8;
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  CK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity min %zu recommended %zu\n", gmin, grec);
  std::vector<uint64_t> chunks = {0 /* hipMalloc */, 2ull << 20, 64ull << 20, 1ull << 30, B};
  for (auto& ch : chunks)
    if (ch && ch < gmin) ch = gmin;
  for (int rep = 0; rep < reps; ++rep) {
    for (uint64_t ch : chunks) {
      double *a, *b, *c;
      vmm_array va, vb, vc;
      if (!ch) {
        CK(hipMalloc(&a, B)); CK(hipMalloc(&b, B)); CK(hipMalloc(&c, B));
      } else {
        va = vmm_alloc(B, ch); vb = vmm_alloc(B, ch); vc = vmm_alloc(B, ch);
        a = (double*)va.va; b = (double*)vb.va; c = (double*)vc.va;
      }
      k_init<<<4096, 256>>>(a, n, 0.0); k_init<<<4096, 256>>>(b, n, 1.0); k_init<<<4096, 256>>>(c, n, 2.0);
      CK(hipDeviceSynchronize());
      const float ms = triad(a, b, c, n);
      printf("rep %d  %-10s chunk %11llu   %7.3f ms  %7.1f GB/s\n", rep, ch ? "vmm" : "hipMalloc",
             (unsigned long long)ch, ms, 24.0 * n / ms / 1e6);
      fflush(stdout);
      if (!ch) {
        CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c));
      } else {
        vmm_free(va); vmm_free(vb); vmm_free(vc);
      }
    }
  }
  return 0;
}
