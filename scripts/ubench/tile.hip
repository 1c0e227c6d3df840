// Microbenchmark: the data movement of a single-pass scan tile, without the
// look-back, at several tile shapes (2^30 doubles in -> out, 16 B/elem).
// Each wave owns R*64 consecutive 16-B vectors of its block's tile; the
// block scans nothing but does the same barrier between load and store.
//   tilecopy<T, R>        : one tile per block, tile = blockIdx
//   tilecopy_ctr<T, R>    : tile id from one agent atomic counter
//   tilecopy_xcd<T, R>    : tile id from 8 per-XCD counters (id = k*8 + xcc)
//   persist<T, R>         : persistent blocks, next tile's loads issued
//                           before the current tile's stores
// build: hipcc -O3 --offload-arch=gfx950 tile.hip -o tile
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2 ldnt(const d2* p) { return __builtin_nontemporal_load(p); }

template <int T, int R>
__device__ __forceinline__ void body(const d2* b, d2* a, uint64_t tile, double* s) {
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t wb = tile * (uint64_t)(T * R) + wave * (R * 64);
  d2 x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) x[r] = ldnt(b + wb + r * 64 + lane);
  double t = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) t += x[r].x;
  if (lane == 0) s[wave] = t;
  __syncthreads();
  const double p = s[(wave + 1) % (T / 64)] * 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) a[wb + r * 64 + lane] = x[r] + p;
}

template <int T, int R>
__global__ __launch_bounds__(T) void tilecopy(const d2* b, d2* a) {
  __shared__ double s[T / 64];
  body<T, R>(b, a, blockIdx.x, s);
}
template <int T, int R>
__global__ __launch_bounds__(T) void tilecopy_ctr(const d2* b, d2* a, uint32_t* ctr) {
  __shared__ double s[T / 64];
  __shared__ uint32_t st;
  if (threadIdx.x == 0) st = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  body<T, R>(b, a, st, s);
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}
// persistent, per-XCD counters, tiles interleaved k*8+xcc; loops until out of range
template <int T, int R>
__global__ __launch_bounds__(T) void persist_xcd(const d2* b, d2* a, uint32_t* ctr, uint32_t ntiles) {
  __shared__ double s[T / 64];
  __shared__ uint32_t st;
  const uint32_t x = xcc_id();
  while (true) {
    if (threadIdx.x == 0) st = __hip_atomic_fetch_add(&ctr[x * 64], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
    __syncthreads();
    const uint32_t t = st;
    if (t >= ntiles) return;
    body<T, R>(b, a, t, s);
    __syncthreads();
  }
}
// persistent grid-stride with software prefetch of the next tile
template <int T, int R>
__global__ __launch_bounds__(T) void persist_pf(const d2* b, d2* a, uint32_t ntiles) {
  __shared__ double s[2][T / 64];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  uint32_t t = blockIdx.x;
  d2 x[R], y[R];
  if (t >= ntiles) return;
  {
    const uint64_t wb = t * (uint64_t)(T * R) + wave * (R * 64);
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ldnt(b + wb + r * 64 + lane);
  }
  int par = 0;
  while (true) {
    const uint32_t tn = t + gridDim.x;
    if (tn < ntiles) {
      const uint64_t wb = tn * (uint64_t)(T * R) + wave * (R * 64);
#pragma unroll
      for (int r = 0; r < R; ++r) y[r] = ldnt(b + wb + r * 64 + lane);
    }
    double tt = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) tt += x[r].x;
    if (lane == 0) s[par][wave] = tt;
    __syncthreads();
    const double p = s[par][(wave + 1) % (T / 64)] * 0.0;
    const uint64_t wb = t * (uint64_t)(T * R) + wave * (R * 64);
#pragma unroll
    for (int r = 0; r < R; ++r) a[wb + r * 64 + lane] = x[r] + p;
    if (tn >= ntiles) return;
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = y[r];
    t = tn;
    par ^= 1;
  }
}
template <int BT>
__global__ __launch_bounds__(BT) void flatcopy(const d2* b, d2* a) {
  const uint64_t i = blockIdx.x * (uint64_t)BT + threadIdx.x;
  a[i] = ldnt(b + i);
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
  d2 *a, *b;
  uint32_t* ctr;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&ctr, 4096));
  CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double B = n * 16.0;
  bench("flatcopy 64", [&] { hipLaunchKernelGGL((flatcopy<64>), dim3(nv / 64), dim3(64), 0, 0, b, a); }, B);
#define TC(T, R) bench("tile T" #T " R" #R, [&] { hipLaunchKernelGGL((tilecopy<T, R>), dim3(nv / (T * R)), dim3(T), 0, 0, b, a); }, B)
  TC(1024, 8); TC(1024, 4); TC(1024, 2); TC(512, 8); TC(512, 4); TC(256, 16); TC(256, 8); TC(256, 4); TC(256, 2); TC(128, 8); TC(64, 16); TC(64, 8); TC(64, 4);
#define TCC(T, R) bench("tile+ctr T" #T " R" #R, [&] { CK(hipMemsetAsync(ctr, 0, 4096)); \
    hipLaunchKernelGGL((tilecopy_ctr<T, R>), dim3(nv / (T * R)), dim3(T), 0, 0, b, a, ctr); }, B)
  TCC(1024, 8); TCC(256, 8); TCC(256, 16);
#define PX(T, R, G) bench("persist-xcd T" #T " R" #R " G" #G, [&] { CK(hipMemsetAsync(ctr, 0, 4096)); \
    hipLaunchKernelGGL((persist_xcd<T, R>), dim3(G), dim3(T), 0, 0, b, a, ctr, (uint32_t)(nv / (T * R))); }, B)
  PX(256, 8, 2048); PX(256, 8, 4096); PX(256, 4, 4096); PX(1024, 8, 512); PX(512, 8, 1024); PX(256, 16, 2048);
#define PP(T, R, G) bench("persist-pf T" #T " R" #R " G" #G, [&] { \
    hipLaunchKernelGGL((persist_pf<T, R>), dim3(G), dim3(T), 0, 0, b, a, (uint32_t)(nv / (T * R))); }, B)
  PP(256, 8, 2048); PP(256, 4, 4096); PP(512, 8, 1024); PP(1024, 8, 256); PP(1024, 4, 512); PP(256, 8, 1024);
  return 0;
}
