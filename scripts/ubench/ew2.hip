// Microbenchmark: nontemporal-load variants of the streaming kernels at 2^30
// doubles (triad a = b + 3c, copy, read+write "scan-like" 128 KiB tiles).
// LD/ST template flags: 0 = plain, 1 = __builtin_nontemporal_{load,store}.
// build: hipcc -O3 --offload-arch=gfx950 ew2.hip -o ew2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2 ld(const d2* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2* p, d2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int BT, int U, bool LNT, bool SNT>
__global__ __launch_bounds__(BT) void triad(const d2* __restrict__ b, const d2* __restrict__ c, d2* __restrict__ a, uint64_t nv) {
  const uint64_t base = blockIdx.x * (uint64_t)BT * U + threadIdx.x;
  d2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; if (i < nv) { x[u] = ld<LNT>(b + i); y[u] = ld<LNT>(c + i); } }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; if (i < nv) st<SNT>(a + i, x[u] + y[u] * 3.0); }
}
template <int BT, int U, bool LNT, bool SNT>
__global__ __launch_bounds__(BT) void copy(const d2* __restrict__ b, d2* __restrict__ a, uint64_t nv) {
  const uint64_t base = blockIdx.x * (uint64_t)BT * U + threadIdx.x;
  d2 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; if (i < nv) x[u] = ld<LNT>(b + i); }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; if (i < nv) st<SNT>(a + i, x[u]); }
}
// scan-shaped: 1024 threads, 8 vectors per thread, each wave owns 8*64
// contiguous vectors (the shipped k_scan layout), one barrier in the middle.
template <bool LNT, bool SNT>
__global__ __launch_bounds__(1024) void tilecopy(const d2* __restrict__ b, d2* __restrict__ a, uint64_t nv) {
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t wb = blockIdx.x * 8192ull + wave * 512;
  d2 x[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) x[r] = ld<LNT>(b + wb + r * 64 + lane);
  __shared__ double s[16];
  double t = 0;
#pragma unroll
  for (int r = 0; r < 8; ++r) t += x[r].x;
  if (lane == 0) s[wave] = t;
  __syncthreads();
  const double p = s[(wave + 1) & 15] * 0.0;
#pragma unroll
  for (int r = 0; r < 8; ++r) st<SNT>(a + wb + r * 64 + lane, x[r] + p);
}
template <bool LNT, bool SNT>
__global__ __launch_bounds__(256) void fill(d2* __restrict__ a, uint64_t nv) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i < nv) st<SNT>(a + i, d2{1.0, 2.0});
}

static hipEvent_t e0, e1;
template <typename F>
void bench(const char* name, F f, double bytes) {
  f(); CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 12; ++r) {
    CK(hipEventRecord(e0)); f(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  printf("%-34s min %7.3f ms med %7.3f ms  %7.1f GB/s (med %7.1f)\n", name, t[0], t[6], bytes / t[0] / 1e6, bytes / t[6] / 1e6);
  fflush(stdout);
}

int main() {
  const uint64_t n = 1ull << 30, nv = n / 2;
  d2 *a, *b, *c;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&c, n * 8));
  CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8)); CK(hipMemset(c, 0, n * 8));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
#define TRIAD(BT, U, L, S) bench("triad BT" #BT " U" #U " L" #L " S" #S, [&] { \
    hipLaunchKernelGGL((triad<BT, U, L, S>), dim3((nv + BT * U - 1) / (BT * U)), dim3(BT), 0, 0, b, c, a, nv); }, n * 24.0)
  TRIAD(256, 1, 0, 0); TRIAD(256, 1, 1, 0); TRIAD(256, 1, 0, 1); TRIAD(256, 1, 1, 1);
  TRIAD(256, 2, 1, 0); TRIAD(256, 2, 1, 1); TRIAD(512, 2, 1, 0); TRIAD(1024, 4, 1, 0); TRIAD(64, 1, 1, 0); TRIAD(64, 1, 1, 1);
#define COPY(BT, U, L, S) bench("copy BT" #BT " U" #U " L" #L " S" #S, [&] { \
    hipLaunchKernelGGL((copy<BT, U, L, S>), dim3((nv + BT * U - 1) / (BT * U)), dim3(BT), 0, 0, b, a, nv); }, n * 16.0)
  COPY(256, 1, 0, 0); COPY(256, 1, 1, 0); COPY(256, 1, 1, 1); COPY(256, 2, 1, 0); COPY(256, 4, 1, 0); COPY(1024, 8, 1, 0);
#define TILE(L, S) bench("tilecopy 1024x8 L" #L " S" #S, [&] { \
    hipLaunchKernelGGL((tilecopy<L, S>), dim3(nv / 8192), dim3(1024), 0, 0, b, a, nv); }, n * 16.0)
  TILE(0, 0); TILE(1, 0); TILE(1, 1); TILE(0, 1);
#define FILL(L, S) bench("fill L" #L " S" #S, [&] { \
    hipLaunchKernelGGL((fill<L, S>), dim3(nv / 256), dim3(256), 0, 0, a, nv); }, n * 8.0)
  FILL(0, 0); FILL(0, 1);
  return 0;
}
