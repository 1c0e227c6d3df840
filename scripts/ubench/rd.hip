// Microbenchmark: read-stream (reduce-shaped) variants, 2^30 int64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
struct alignas(16) l2 { long long x, y; };
__device__ long long wsum(long long v) { for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o); return v; }
template <int BT>
__device__ void block_out(long long s, long long* part) {
  __shared__ long long w[BT / 64];
  s = wsum(s); if ((threadIdx.x & 63) == 0) w[threadIdx.x / 64] = s; __syncthreads();
  if (threadIdx.x == 0) { long long t = 0; for (int i = 0; i < BT / 64; ++i) t += w[i]; part[blockIdx.x] = t; }
}
// flat: block owns U*BT consecutive vectors, one pass
template <int BT, int U>
__global__ __launch_bounds__(BT) void rd_flat(const l2* a, uint64_t nv, long long* part) {
  uint64_t base = blockIdx.x * (uint64_t)BT * U + threadIdx.x; long long s = 0;
  l2 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * BT; if (i < nv) x[u] = a[i]; else x[u] = {0,0}; }
#pragma unroll
  for (int u = 0; u < U; ++u) s += x[u].x + x[u].y;
  block_out<BT>(s, part);
}
// chunk loop: block owns C*BT consecutive vectors, walks them BT at a time (U in flight)
template <int BT, int U>
__global__ __launch_bounds__(BT) void rd_chunk(const l2* a, uint64_t nv, uint64_t C, long long* part) {
  uint64_t base = blockIdx.x * (uint64_t)BT * C; long long s = 0;
  for (uint64_t k = 0; k < C; k += U) {
    l2 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { uint64_t i = base + (k + u) * BT + threadIdx.x; if (i < nv) x[u] = a[i]; else x[u] = {0,0}; }
#pragma unroll
    for (int u = 0; u < U; ++u) s += x[u].x + x[u].y;
  }
  block_out<BT>(s, part);
}
int main() {
  const uint64_t N = 1ull << 30, nv = N / 2;
  l2* a; long long* part; CK(hipMalloc(&a, N * 8)); CK(hipMalloc(&part, 64 << 20)); CK(hipMemset(a, 1, N * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    printf("%-34s min %7.3f ms med %7.3f ms  %7.1f GB/s (med %7.1f)\n", name, t[0], t[7], bytes / t[0] / 1e6, bytes / t[7] / 1e6);
  };
  double B = 8.0 * N;
  run("flat BT256 U1", B, [&]{ rd_flat<256,1><<<nv/256,256>>>(a,nv,part); });
  run("flat BT256 U2", B, [&]{ rd_flat<256,2><<<nv/512,256>>>(a,nv,part); });
  run("flat BT256 U4", B, [&]{ rd_flat<256,4><<<nv/1024,256>>>(a,nv,part); });
  run("flat BT512 U1", B, [&]{ rd_flat<512,1><<<nv/512,512>>>(a,nv,part); });
  run("flat BT1024 U1", B, [&]{ rd_flat<1024,1><<<nv/1024,1024>>>(a,nv,part); });
  run("flat BT1024 U2", B, [&]{ rd_flat<1024,2><<<nv/2048,1024>>>(a,nv,part); });
  for (uint64_t C : {4ull, 8ull, 16ull, 64ull, 256ull}) {
    char nm[64];
    snprintf(nm, 64, "chunk BT256 U1 C=%llu", (unsigned long long)C); run(nm, B, [&]{ rd_chunk<256,1><<<nv/(256*C),256>>>(a,nv,C,part); });
    snprintf(nm, 64, "chunk BT256 U4 C=%llu", (unsigned long long)C); run(nm, B, [&]{ rd_chunk<256,4><<<nv/(256*C),256>>>(a,nv,C,part); });
    snprintf(nm, 64, "chunk BT1024 U1 C=%llu", (unsigned long long)C); run(nm, B, [&]{ rd_chunk<1024,1><<<nv/(1024*C),1024>>>(a,nv,C,part); });
  }
  return 0;
}
