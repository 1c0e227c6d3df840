// Microbenchmark (round 2, session 2): copy_if write-out batching.  RPB wave
// rounds of hits are compacted into LDS back to back and stored as one run
// (RPB = 1: one LDS round trip per round, the round-1 form), int64 at 2^30
// and int32 at 2^31 (8 GiB each), predicate !(x < 0) on ~50 % hits, tile
// ids from the counter and from blockIdx.  Each variant's output count is
// checked against the first.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include copyif6.hip -o copyif6
#include "../../hpx_amd/csrc/copy_if_kernel.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;
using namespace hpxhip::copy_if_detail;

template <typename T>
__global__ void k_fill(T* p, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) { uint64_t z = i * 0x9E3779B97F4A7C15ull; z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; p[i] = (T)z; }
}

template <typename T>
struct harness {
  using P = pred_fn<HPXHIP_P_NOT_LT, T>;
  uint64_t N; T *in, *out; char* ws; uint32_t* err; uint64_t* cnt; hipEvent_t e0, e1; uint64_t ref = 0;
  template <int RPB, bool DYN, int MINW = 4>
  void run(const char* name) {
    constexpr int R = 8;
    using SV = uint32_t;
    const uint64_t ntiles = (N + tile_elems<T, R>() - 1) / tile_elems<T, R>();
    const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
    tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    auto launch = [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      k_copy_if<T, P, true, R, MINW, 0, SV, DYN, false, RPB><<<ntiles, kThreads>>>(in, out, N, P{0}, cnt,
          reinterpret_cast<uint32_t*>(ws), st, ntiles);
    };
    launch(); CK(hipDeviceSynchronize());
    uint64_t c = 0; CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
    if (!ref) ref = c;
    std::vector<float> t;
    for (int r = 0; r < 11; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 1.0 * sizeof(T) * N + 1.0 * sizeof(T) * c;
    printf("%-4s %-34s min %7.3f ms med %7.3f ms  %7.1f GB/s  hits %.4f %s\n", sizeof(T) == 8 ? "i64" : "i32", name,
           t[0], t[5], B / t[0] / 1e6, double(c) / N, c == ref ? "" : "COUNT MISMATCH");
    fflush(stdout);
  }
};

int main() {
  char* ws; uint32_t* err; uint64_t* cnt; void *in, *out;
  const uint64_t bytes = 8ull << 30;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMalloc(&cnt, 64)); CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    {
      harness<int64_t> h{bytes / 8, (int64_t*)in, (int64_t*)out, ws, err, cnt, e0, e1};
      hipLaunchKernelGGL(k_fill<int64_t>, dim3(h.N / 256), dim3(256), 0, 0, h.in, h.N);
      h.run<1, true>("RPB1 atomic minw4 (shipped)");
      h.run<1, true, 8>("RPB1 atomic minw8");
    }
    {
      harness<int32_t> h{bytes / 4, (int32_t*)in, (int32_t*)out, ws, err, cnt, e0, e1};
      hipLaunchKernelGGL(k_fill<int32_t>, dim3(h.N / 256), dim3(256), 0, 0, h.in, h.N);
      h.run<1, true>("RPB1 atomic minw4 (shipped, 70 VGPRs)");
      h.run<1, true, 8>("RPB1 atomic minw8 (<= 64 VGPRs)");
      h.run<1, false, 8>("RPB1 blockIdx minw8");
      h.run<2, true, 8>("RPB2 atomic minw8");
    }
  }
  uint32_t hh = 0; CK(hipMemcpy(&hh, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", hh);
  return 0;
}
