// Microbenchmark: scan-tile data movement, wave-contiguous vs striped layout
// (2^30 doubles in -> out, 16 B/elem, no look-back).
//   wave-contiguous: wave w owns R*64 consecutive 16-B vectors of the tile
//                    (the shipped scan/copy_if layout) -> 16 concurrent
//                    address streams per 1024-thread block;
//   striped:         round r of the whole block covers T consecutive vectors
//                    (vector = tile*T*R + r*T + tid) -> one stream per block.
// Both do a barrier between the loads and the stores, and take tile ids from
// an agent atomic counter like the shipped kernels.
// build: hipcc -O3 --offload-arch=gfx950 tile2.hip -o tile2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2 ldnt(const d2* p) { return __builtin_nontemporal_load(p); }

template <int T, int R, bool STRIPED>
__global__ __launch_bounds__(T) void tile(const d2* b, d2* a, uint32_t* ctr) {
  __shared__ double s[T / 64];
  __shared__ uint32_t st;
  if (threadIdx.x == 0) st = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint64_t t = st;
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t base = t * (uint64_t)(T * R);
  auto idx = [&](int r) -> uint64_t {
    return STRIPED ? base + (uint64_t)r * T + threadIdx.x : base + (uint64_t)wave * (R * 64) + r * 64 + lane;
  };
  d2 x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) x[r] = ldnt(b + idx(r));
  double tt = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) tt += x[r].x;
  if (lane == 0) s[wave] = tt;
  __syncthreads();
  const double p = s[(wave + 1) % (T / 64)] * 0.0;
#pragma unroll
  for (int r = 0; r < R; ++r) a[idx(r)] = x[r] + p;
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
#define TL(T, R, S) bench(S ? "tile T" #T " R" #R " striped" : "tile T" #T " R" #R " wavecontig", [&] { CK(hipMemsetAsync(ctr, 0, 4096)); \
    hipLaunchKernelGGL((tile<T, R, S>), dim3(nv / (T * R)), dim3(T), 0, 0, b, a, ctr); }, B)
  for (int rep = 0; rep < 2; ++rep) {
    bench("flatcopy 64", [&] { hipLaunchKernelGGL((flatcopy<64>), dim3(nv / 64), dim3(64), 0, 0, b, a); }, B);
    bench("flatcopy 256", [&] { hipLaunchKernelGGL((flatcopy<256>), dim3(nv / 256), dim3(256), 0, 0, b, a); }, B);
    TL(1024, 16, false); TL(1024, 16, true);
    TL(1024, 8, false); TL(1024, 8, true);
    TL(512, 16, false); TL(512, 16, true);
    TL(256, 16, false); TL(256, 16, true);
    TL(256, 4, false); TL(256, 4, true);
  }
  return 0;
}
