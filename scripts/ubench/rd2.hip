// Microbenchmark: read-stream geometries for the int64 reduce (2^30 elements,
// 8 GiB).  Each variant writes one partial per block (the fold of the
// partials is not timed here; it is <1 % of the bytes).
// build: hipcc -O3 --offload-arch=gfx950 rd2.hip -o rd2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
struct alignas(16) l2 { long long x, y; };

// flat: block owns BT*U consecutive vectors, all U loads issued first
template <int BT, int U, bool NT>
__global__ __launch_bounds__(BT) void rd_flat(const l2* __restrict__ a, uint64_t nv, long long* part) {
  const uint64_t base = blockIdx.x * (uint64_t)BT * U + threadIdx.x;
  l2 x[U];
  if (base + (U - 1) * (uint64_t)BT < nv) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) { x[u].x = __builtin_nontemporal_load(&a[base + u * BT].x); x[u].y = __builtin_nontemporal_load(&a[base + u * BT].y); }
      else x[u] = a[base + u * BT];
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; x[u] = i < nv ? a[i] : l2{0, 0}; }
  }
  long long s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s += x[u].x + x[u].y;
  // wave reduce via shuffles, then LDS
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ long long w[BT / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) { long long t = 0; for (int i = 0; i < BT / 64; ++i) t += w[i]; part[blockIdx.x] = t; }
}

// chunked: block owns BT*U*C vectors; C batches of U loads
template <int BT, int U>
__global__ __launch_bounds__(BT) void rd_chunk(const l2* __restrict__ a, uint64_t nv, long long* part, int C) {
  const uint64_t base = blockIdx.x * (uint64_t)BT * U * C + threadIdx.x;
  long long s = 0;
  for (int c = 0; c < C; ++c) {
    const uint64_t b = base + (uint64_t)c * BT * U;
    l2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = b + u * BT; x[u] = i < nv ? a[i] : l2{0, 0}; }
#pragma unroll
    for (int u = 0; u < U; ++u) s += x[u].x + x[u].y;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ long long w[BT / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) { long long t = 0; for (int i = 0; i < BT / 64; ++i) t += w[i]; part[blockIdx.x] = t; }
}

// persistent grid-stride over blocks of BT*U vectors; G blocks
template <int BT, int U>
__global__ __launch_bounds__(BT) void rd_persist(const l2* __restrict__ a, uint64_t nv, long long* part) {
  long long s = 0;
  const uint64_t tile = (uint64_t)BT * U;
  for (uint64_t t = blockIdx.x; t * tile < nv; t += gridDim.x) {
    const uint64_t b = t * tile + threadIdx.x;
    l2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = b + u * BT; x[u] = i < nv ? a[i] : l2{0, 0}; }
#pragma unroll
    for (int u = 0; u < U; ++u) s += x[u].x + x[u].y;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ long long w[BT / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) { long long t = 0; for (int i = 0; i < BT / 64; ++i) t += w[i]; part[blockIdx.x] = t; }
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
  l2* a; long long* part;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&part, (nv / 64 + 64) * 8));
  CK(hipMemset(a, 1, n * 8));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double B = n * 8.0;
#define FLAT(BT, U, NT) bench("flat BT" #BT " U" #U " NT=" #NT, [&] { \
    hipLaunchKernelGGL((rd_flat<BT, U, NT>), dim3((nv + BT * U - 1) / (BT * U)), dim3(BT), 0, 0, a, nv, part); }, B)
  FLAT(256, 1, false); FLAT(256, 2, false); FLAT(256, 4, false); FLAT(256, 8, false); FLAT(256, 16, false);
  FLAT(512, 2, false); FLAT(512, 4, false); FLAT(512, 8, false);
  FLAT(1024, 2, false); FLAT(1024, 4, false); FLAT(1024, 8, false);
  FLAT(256, 2, true); FLAT(256, 4, true); FLAT(1024, 8, true);
#define CHUNK(BT, U, C) bench("chunk BT" #BT " U" #U " C" #C, [&] { \
    hipLaunchKernelGGL((rd_chunk<BT, U>), dim3((nv + BT * U * C - 1) / (BT * U * C)), dim3(BT), 0, 0, a, nv, part, C); }, B)
  CHUNK(1024, 2, 4); CHUNK(1024, 4, 2); CHUNK(1024, 8, 1); CHUNK(256, 4, 4); CHUNK(256, 8, 4); CHUNK(512, 4, 4);
#define PERS(BT, U, G) bench("persist BT" #BT " U" #U " G" #G, [&] { \
    hipLaunchKernelGGL((rd_persist<BT, U>), dim3(G), dim3(BT), 0, 0, a, nv, part); }, B)
  PERS(256, 4, 2048); PERS(256, 8, 2048); PERS(512, 4, 1024); PERS(1024, 4, 512); PERS(256, 4, 4096); PERS(1024, 4, 1024);
  return 0;
}
