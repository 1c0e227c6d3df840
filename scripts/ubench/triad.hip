// Microbenchmark: STREAM triad a = b + 3 c over 2^30 doubles, kernel shapes.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off triad.hip -o triad
#include "../../hpx_amd/csrc/common.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using VT = vec<double, 2>;

template <bool NTL, bool NTS>
__device__ __forceinline__ VT ldv(const VT* p) { if constexpr (NTL) return ld_stream(p); else return *p; }
template <bool NTS>
__device__ __forceinline__ void stv(VT* p, VT v) { if constexpr (NTS) st_stream(p, v); else *p = v; }

// U vectors per thread, block-interleaved (coalesced): flat grid covering n.
template <int TH, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void k_flat(const VT* b, const VT* c, VT* a, uint64_t nv, double s) {
  const uint64_t base = uint64_t(blockIdx.x) * TH * U + threadIdx.x;
  VT x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * TH; if (i < nv) { x[u] = ldv<NTL, NTS>(&b[i]); y[u] = ldv<NTL, NTS>(&c[i]); } }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * TH; if (i < nv) { VT z; z.v[0] = x[u].v[0] + y[u].v[0] * s; z.v[1] = x[u].v[1] + y[u].v[1] * s; stv<NTS>(&a[i], z); } }
}
// grid-stride with U vectors in flight per trip
template <int TH, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(TH) void k_gs(const VT* b, const VT* c, VT* a, uint64_t nv, double s) {
  const uint64_t stride = uint64_t(gridDim.x) * TH * U;
  for (uint64_t base = uint64_t(blockIdx.x) * TH * U + threadIdx.x; base < nv; base += stride) {
    VT x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = base + u * TH; if (i < nv) { x[u] = ldv<NTL, NTS>(&b[i]); y[u] = ldv<NTL, NTS>(&c[i]); } }
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = base + u * TH; if (i < nv) { VT z; z.v[0] = x[u].v[0] + y[u].v[0] * s; z.v[1] = x[u].v[1] + y[u].v[1] * s; stv<NTS>(&a[i], z); } }
  }
}
__global__ void k_init(double* p, uint64_t n, double v) { for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) p[i] = v + (i & 7); }

int main() {
  const uint64_t N = 1ull << 30, NV = N / 2;
  double *a, *b, *c; CK(hipMalloc(&a, N * 8)); CK(hipMalloc(&b, N * 8)); CK(hipMalloc(&c, N * 8));
  k_init<<<8192, 256>>>(b, N, 2.0); k_init<<<8192, 256>>>(c, N, 0.5); CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    double h[2]; CK(hipMemcpy(h, a + N - 2, 16, hipMemcpyDeviceToHost));
    bool ok = h[0] == (2.0 + ((N - 2) & 7)) + (0.5 + ((N - 2) & 7)) * 3.0;
    printf("%-36s min %7.3f med %7.3f ms  %7.1f GB/s (%5.1f%%) %s\n", name, t[0], t[7], 24.0 * N / t[0] / 1e6, 24.0 * N / t[0] / 1e6 / 80, ok ? "ok" : "BAD");
    fflush(stdout);
  };
#define FLAT(TH, U, NTL, NTS) run("flat T" #TH " U" #U " ntl" #NTL " nts" #NTS, [&] { k_flat<TH, U, NTL, NTS><<<(NV + TH * U - 1) / (TH * U), TH>>>((VT*)b, (VT*)c, (VT*)a, NV, 3.0); })
#define GS(TH, U, G, NTL, NTS) run("gs T" #TH " U" #U " G" #G " ntl" #NTL " nts" #NTS, [&] { k_gs<TH, U, NTL, NTS><<<G, TH>>>((VT*)b, (VT*)c, (VT*)a, NV, 3.0); })
  for (int rep = 0; rep < 2; ++rep) {
    FLAT(64, 1, 1, 1);   // shipped shape
    FLAT(64, 1, 1, 0);
    FLAT(64, 1, 0, 0);
    FLAT(128, 1, 1, 1);
    FLAT(256, 1, 1, 1);
    FLAT(256, 2, 1, 1);
    FLAT(256, 4, 1, 1);
    FLAT(512, 2, 1, 1);
    FLAT(1024, 1, 1, 1);
    FLAT(1024, 2, 1, 1);
    FLAT(64, 2, 1, 1);
    FLAT(64, 4, 1, 1);
    GS(256, 2, 2048, 1, 1);
    GS(256, 4, 2048, 1, 1);
    GS(512, 2, 2048, 1, 1);
    GS(1024, 2, 1024, 1, 1);
    GS(256, 4, 8192, 1, 1);
    GS(64, 4, 16384, 1, 1);
  }
  return 0;
}
