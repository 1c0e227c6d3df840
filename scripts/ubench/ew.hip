// Microbenchmark: streaming triad variants on gfx950 (a = b + 3c, 2^30 doubles).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
struct alignas(16) d2 { double x, y; };

// A: grid-stride, U vectors per thread per iteration, strided by grid
template <int U, bool NT>
__global__ __launch_bounds__(256) void triad_gs(const d2* b, const d2* c, d2* a, uint64_t nv) {
  uint64_t tid = blockIdx.x * 256ull + threadIdx.x, st = gridDim.x * 256ull;
  for (uint64_t i = tid; i < nv; i += st * U) {
    d2 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + u * st < nv) { x[u] = b[i + u * st]; y[u] = c[i + u * st]; }
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + u * st < nv) {
      d2 r; r.x = x[u].x + y[u].x * 3.0; r.y = x[u].y + y[u].y * 3.0;
      if (NT) { __builtin_nontemporal_store(r.x, &a[i+u*st].x); __builtin_nontemporal_store(r.y, &a[i+u*st].y); }
      else a[i + u * st] = r;
    }
  }
}
// B: flat, each block owns U*256 consecutive vectors (block-contiguous tile)
template <int U, bool NT>
__global__ __launch_bounds__(256) void triad_flat(const d2* b, const d2* c, d2* a, uint64_t nv) {
  uint64_t base = blockIdx.x * 256ull * U + threadIdx.x;
  d2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 256; if (i < nv) { x[u] = b[i]; y[u] = c[i]; } }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 256; if (i < nv) {
      d2 r; r.x = x[u].x + y[u].x * 3.0; r.y = x[u].y + y[u].y * 3.0;
      if (NT) { __builtin_nontemporal_store(r.x, &a[i].x); __builtin_nontemporal_store(r.y, &a[i].y); }
      else a[i] = r; } }
}
// C: flat but 512 threads
template <int U>
__global__ __launch_bounds__(512) void triad_flat512(const d2* b, const d2* c, d2* a, uint64_t nv) {
  uint64_t base = blockIdx.x * 512ull * U + threadIdx.x;
  d2 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 512; if (i < nv) { x[u] = b[i]; y[u] = c[i]; } }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 512; if (i < nv) {
      d2 r; r.x = x[u].x + y[u].x * 3.0; r.y = x[u].y + y[u].y * 3.0; a[i] = r; } }
}
// D: read-only reduce-like stream (sum) to find the read ceiling
template <int U>
__global__ __launch_bounds__(256) void readsum_flat(const d2* b, uint64_t nv, double* out) {
  uint64_t base = blockIdx.x * 256ull * U + threadIdx.x;
  double s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 256; if (i < nv) { d2 x = b[i]; s += x.x + x.y; } }
  if (s == 12345.678) out[0] = s;
}
template <int U>
__global__ __launch_bounds__(256) void copy_flat(const d2* b, d2* a, uint64_t nv) {
  uint64_t base = blockIdx.x * 256ull * U + threadIdx.x;
  d2 x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 256; if (i < nv) x[u] = b[i]; }
#pragma unroll
  for (int u = 0; u < U; ++u) { uint64_t i = base + u * 256; if (i < nv) a[i] = x[u]; }
}

template <int BT>
__global__ __launch_bounds__(BT) void triad_chunk(const d2* b, const d2* c, d2* a, uint64_t nv, uint64_t C) {
  uint64_t base = blockIdx.x * (uint64_t)BT * C + threadIdx.x;
  for (uint64_t k = 0; k < C; ++k) {
    uint64_t i = base + k * BT;
    if (i < nv) { d2 x = b[i], y = c[i]; d2 r; r.x = x.x + y.x * 3.0; r.y = x.y + y.y * 3.0; a[i] = r; }
  }
}
template <int BT>
__global__ __launch_bounds__(BT) void triad_flat_bt(const d2* b, const d2* c, d2* a, uint64_t nv) {
  uint64_t i = blockIdx.x * (uint64_t)BT + threadIdx.x;
  if (i < nv) { d2 x = b[i], y = c[i]; d2 r; r.x = x.x + y.x * 3.0; r.y = x.y + y.y * 3.0; a[i] = r; }
}

int main() {
  const uint64_t N = 1ull << 30, nv = N / 2;
  d2 *a, *b, *c; double* o;
  CK(hipMalloc(&a, N * 8)); CK(hipMalloc(&b, N * 8)); CK(hipMalloc(&c, N * 8)); CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, N * 8)); CK(hipMemset(b, 0, N * 8)); CK(hipMemset(c, 0, N * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double bytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    printf("%-34s min %7.3f ms med %7.3f ms  %7.1f GB/s (med %7.1f)\n", name, t[0], t[7], bytes / t[0] / 1e6, bytes / t[7] / 1e6);
  };
  double tb = 24.0 * N;
  run("flat BT64", tb, [&]{ triad_flat_bt<64><<<nv/64,64>>>(b,c,a,nv); });
  run("flat BT128", tb, [&]{ triad_flat_bt<128><<<nv/128,128>>>(b,c,a,nv); });
  run("flat BT256", tb, [&]{ triad_flat_bt<256><<<nv/256,256>>>(b,c,a,nv); });
  run("flat BT1024", tb, [&]{ triad_flat_bt<1024><<<nv/1024,1024>>>(b,c,a,nv); });
  for (uint64_t C : {2ull, 4ull, 8ull, 32ull}) {
    char nm[64];
    snprintf(nm, 64, "chunk BT256 C=%llu", (unsigned long long)C); run(nm, tb, [&]{ triad_chunk<256><<<nv/(256*C),256>>>(b,c,a,nv,C); });
    snprintf(nm, 64, "chunk BT1024 C=%llu", (unsigned long long)C); run(nm, tb, [&]{ triad_chunk<1024><<<nv/(1024*C),1024>>>(b,c,a,nv,C); });
  }
  for (int bpc : {8}) for (int dummy : {0}) {
    (void)dummy; unsigned g = 256 * bpc; char nm[64];
    snprintf(nm, 64, "gs U4 grid=%u", g); run(nm, tb, [&]{ triad_gs<4,false><<<g,256>>>(b,c,a,nv); });
    snprintf(nm, 64, "gs U2 grid=%u", g); run(nm, tb, [&]{ triad_gs<2,false><<<g,256>>>(b,c,a,nv); });
    snprintf(nm, 64, "gs U8 grid=%u", g); run(nm, tb, [&]{ triad_gs<8,false><<<g,256>>>(b,c,a,nv); });
    snprintf(nm, 64, "gs U4 NT grid=%u", g); run(nm, tb, [&]{ triad_gs<4,true><<<g,256>>>(b,c,a,nv); });
  }
  run("flat U1", tb, [&]{ triad_flat<1,false><<<(nv+255)/256,256>>>(b,c,a,nv); });
  run("flat U2", tb, [&]{ triad_flat<2,false><<<(nv+511)/512,256>>>(b,c,a,nv); });
  run("flat U4", tb, [&]{ triad_flat<4,false><<<(nv+1023)/1024,256>>>(b,c,a,nv); });
  run("flat U8", tb, [&]{ triad_flat<8,false><<<(nv+2047)/2048,256>>>(b,c,a,nv); });
  run("flat U1 NT", tb, [&]{ triad_flat<1,true><<<(nv+255)/256,256>>>(b,c,a,nv); });
  run("flat U4 NT", tb, [&]{ triad_flat<4,true><<<(nv+1023)/1024,256>>>(b,c,a,nv); });
  run("flat512 U1", tb, [&]{ triad_flat512<1><<<(nv+511)/512,512>>>(b,c,a,nv); });
  run("flat512 U2", tb, [&]{ triad_flat512<2><<<(nv+1023)/1024,512>>>(b,c,a,nv); });
  run("copy flat U1", 16.0*N, [&]{ copy_flat<1><<<(nv+255)/256,256>>>(b,a,nv); });
  run("copy flat U4", 16.0*N, [&]{ copy_flat<4><<<(nv+1023)/1024,256>>>(b,a,nv); });
  run("hipMemcpy D2D", 16.0*N, [&]{ CK(hipMemcpyAsync(a, b, N*8, hipMemcpyDeviceToDevice, 0)); });
  run("readsum flat U1", 8.0*N, [&]{ readsum_flat<1><<<(nv+255)/256,256>>>(b,nv,o); });
  run("readsum flat U4", 8.0*N, [&]{ readsum_flat<4><<<(nv+1023)/1024,256>>>(b,nv,o); });
  run("readsum flat U8", 8.0*N, [&]{ readsum_flat<8><<<(nv+2047)/2048,256>>>(b,nv,o); });
  return 0;
}
