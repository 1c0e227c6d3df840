// Microbenchmark (round 4): the look-back poll interval.  Every waiting
// tile polls its predecessors' slots with agent-scope loads and sleeps
// HPXHIP_LB_SLEEP x 64 clocks between polls; with ~512 tiles resident the
// polls compete with the data stream for the fabric.  Built once per
// (HPXHIP_LB_SLEEP, HPXHIP_LB_GROUP) by scripts/r4/k.sh; runs the shipped
// 2^30 int64 inclusive plus-scan (512 x 16, 32-tile groups) and the shipped
// 2^30 int64 copy_if (1024 x 8, ~50 % hits, HPXHIP_LB_GROUP-tile groups).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -DHPXHIP_LB_SLEEP=S -I../../include -I../../hpx_amd/csrc lbsleep.hip
#include <hpxhip/kernels/copy_if_kernel.hpp>
#include <hpxhip/kernels/scan_kernel.hpp>
#include "internal.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;

template <typename T> struct idc { __device__ T operator()(T x) const { return x; } };

__global__ void k_fill(int64_t* p, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; p[i] = (int64_t)(z & 0xffff) - 0x7fff; }
}

template <typename L>
double best(L launch, hipEvent_t e0, hipEvent_t e1, float* med) {
  launch(); CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
  std::sort(t.begin(), t.end());
  *med = t[7];
  return t[0];
}

int main() {
  const uint64_t N = 1ull << 30;
  char* ws; uint32_t* err; int64_t *in, *out; uint64_t* cnt;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMalloc(&cnt, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k_fill<<<(N + 255) / 256, 256>>>(in, N); CK(hipDeviceSynchronize());
  // reference results: host-side checks on a sample
  std::vector<int64_t> h(N);
  CK(hipMemcpy(h.data(), in, N * 8, hipMemcpyDeviceToHost));
  for (int rep = 0; rep < 2; ++rep) {
    {  // scan, shipped shape
      using T = int64_t;
      constexpr int R = 16, TH = 512;
      const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
      const uint64_t ntiles = (N + tile - 1) / tile;
      const size_t total = 256 + ntiles * scan_detail::scan_state<T>::bytes_per_tile();
      scan_detail::scan_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
      float med;
      double t = best([&] {
        CK(hipMemsetAsync(ws, 0, total, 0));
        scan_detail::k_scan<T, idc<T>, op_plus, true, true, R, TH, true, 4, false, 1, false, true, T, false, true><<<ntiles, TH>>>(
            in, out, N, idc<T>{}, op_plus{}, T(0), static_cast<const T*>(nullptr), reinterpret_cast<uint32_t*>(ws), st);
      }, e0, e1, &med);
      int64_t s = 0; bool ok = true; uint64_t i = 0;
      for (uint64_t probe : {uint64_t(0), tile - 1, tile, N / 2 + 12345, N - 1}) {
        for (; i <= probe; ++i) s += h[i];
        int64_t g; CK(hipMemcpy(&g, out + probe, 8, hipMemcpyDeviceToHost)); ok = ok && g == s;
      }
      printf("onehop %d sleep %2d group %3d  scan i64    min %7.3f ms med %7.3f ms  %7.1f GB/s %s\n", HPXHIP_LB_ONEHOP, HPXHIP_LB_SLEEP,
             scan_detail::kScanGroup, t, med, 16.0 * N / t / 1e6, ok ? "ok" : "MISMATCH");
    }
    {  // copy_if, shipped shape
      using T = int64_t; using SV = uint32_t;
      using P = pred_fn<HPXHIP_P_NOT_LT, T>;
      using namespace copy_if_detail;
      constexpr int R = 8;
      const uint64_t ntiles = (N + tile_elems<T, R>() - 1) / tile_elems<T, R>();
      const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
      tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
      float med;
      double t = best([&] {
        CK(hipMemsetAsync(ws, 0, total, 0));
        k_copy_if<T, P, true, R, 8, 0, SV, false, true, 4, true, kThreads, true><<<ntiles, kThreads>>>(in, out, N, P{0}, cnt,
            reinterpret_cast<uint32_t*>(ws), st, ntiles);
      }, e0, e1, &med);
      uint64_t c = 0; CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
      uint64_t hc = 0; for (uint64_t i = 0; i < N; ++i) hc += h[i] >= 0;
      int64_t g[2]; CK(hipMemcpy(g, out + (c - 2), 16, hipMemcpyDeviceToHost));
      int64_t last[2]; int k = 1;
      for (uint64_t i = N; i-- > 0 && k >= 0;) if (h[i] >= 0) last[k--] = h[i];
      const bool ok = c == hc && g[0] == last[0] && g[1] == last[1];
      printf("onehop %d sleep %2d group %3d  copy_if i64 min %7.3f ms med %7.3f ms  %7.1f GB/s %s\n", HPXHIP_LB_ONEHOP, HPXHIP_LB_SLEEP,
             (int)tile_state<SV>::kGroup, t, med, (8.0 * N + 8.0 * c) / t / 1e6, ok ? "ok" : "MISMATCH");
    }
    {  // copy_if int32 at 2^31 (the same bytes): two-hop vs one-hop
      using T = int32_t; using SV = uint32_t;
      using P = pred_fn<HPXHIP_P_NOT_LT, T>;
      using namespace copy_if_detail;
      constexpr int R = 8;
      const uint64_t N32 = 2 * N;
      const T* in32 = reinterpret_cast<const T*>(in);
      T* out32 = reinterpret_cast<T*>(out);
      const uint64_t ntiles = (N32 + tile_elems<T, R>() - 1) / tile_elems<T, R>();
      const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
      tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
      uint64_t c[2];
      for (int oh = 0; oh < 2; ++oh) {
        float med;
        double t = best([&] {
          CK(hipMemsetAsync(ws, 0, total, 0));
          if (oh) k_copy_if<T, P, true, R, 8, 0, SV, false, false, 1, true, kThreads, false, true><<<ntiles, kThreads>>>(in32, out32, N32, P{0}, cnt,
              reinterpret_cast<uint32_t*>(ws), st, ntiles);
          else k_copy_if<T, P, true, R, 8, 0, SV, false, false, 1, true, kThreads, false, false><<<ntiles, kThreads>>>(in32, out32, N32, P{0}, cnt,
              reinterpret_cast<uint32_t*>(ws), st, ntiles);
        }, e0, e1, &med);
        CK(hipMemcpy(&c[oh], cnt, 8, hipMemcpyDeviceToHost));
        printf("onehop %d             int32 copy_if 2^31 min %7.3f ms med %7.3f ms  %7.1f GB/s hits %llu %s\n", oh, t, med,
               (4.0 * N32 + 4.0 * c[oh]) / t / 1e6, (unsigned long long)c[oh], (oh && c[1] != c[0]) ? "COUNT MISMATCH" : "");
      }
    }
    fflush(stdout);
  }
  uint32_t e = 0; CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", e);
  return 0;
}
