// Microbenchmark (round 4, copyif8): phase split of the shipped 2^30 int64
// copy_if (ABL ablations: 1 no look-back, 4 no write-out, 2 direct scatter)
// and nt stores, for the PMC passes of scripts/r4/l.sh; then (after nt stores
// shipped) 16-B output stores (WIDE).
// (copyif7, round 3:) copy_if with the fixed-association look-back
// (FIXED: tiles read their group's published aggregates plus one group
// prefix word, lookback.hpp exclusive_prefix_fixed) against the shipped
// variable-window look-back, tile ids from the counter and from blockIdx
// (int32 also at 6 and 4 rounds: 8 rounds spill 12-14 VGPRs at 64), and
// with the fixed look-back, nt stores and RPB-round write-out batches (int64);
// then (after those shipped) 512- and 256-thread tiles, more workgroups per CU;
// int64 at 2^30 and int32 at 2^31, predicate !(x < 0) on ~50 % hits.  Each
// variant's output is compared element for element with the first run's.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include -I../../hpx_amd/csrc copyif8.hip -o copyif8
#include <hpxhip/kernels/copy_if_kernel.hpp>
#include "internal.hpp"
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
__global__ void k_diff(const T* a, const T* b, uint64_t n, unsigned long long* bad) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n && a[i] != b[i]) atomicAdd(bad, 1ull);
}

template <typename T>
struct harness {
  using P = pred_fn<HPXHIP_P_NOT_LT, T>;
  uint64_t N; T *in, *out, *ref_out; char* ws; uint32_t* err; uint64_t* cnt; unsigned long long* bad;
  hipEvent_t e0, e1; uint64_t ref = 0;
  template <bool DYN, bool FIXED, int R = 8, bool NTS = false, int RPB = 1, int TH = kThreads, int MINW = 8, int ABL = 0, bool WIDE = false>
  void run(const char* name) {
    using SV = uint32_t;
    const uint64_t ntiles = (N + tile_elems<T, R, TH>() - 1) / tile_elems<T, R, TH>();
    const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
    tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    auto launch = [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      k_copy_if<T, P, true, R, MINW, ABL, SV, DYN, NTS, RPB, FIXED, TH, WIDE><<<ntiles, TH>>>(in, out, N, P{0}, cnt,
          reinterpret_cast<uint32_t*>(ws), st, ntiles);
    };
    launch(); CK(hipDeviceSynchronize());
    uint64_t c = 0; CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
    unsigned long long nbad = 0;
    if (!ref) { ref = c; CK(hipMemcpy(ref_out, out, c * sizeof(T), hipMemcpyDeviceToDevice)); }
    else {
      CK(hipMemset(bad, 0, 8));
      k_diff<T><<<(c + 255) / 256, 256>>>(out, ref_out, c, bad);
      CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
    }
    std::vector<float> t;
    for (int r = 0; r < 11; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 1.0 * sizeof(T) * N + 1.0 * sizeof(T) * c;
    printf("%-4s %-34s min %7.3f ms med %7.3f ms  %7.1f GB/s  hits %.4f %s\n", sizeof(T) == 8 ? "i64" : "i32", name,
           t[0], t[5], B / t[0] / 1e6, double(c) / N, (ABL || (c == ref && nbad == 0)) ? "" : "OUTPUT MISMATCH");
    fflush(stdout);
  }
};

int main(int argc, char** argv) {
  char* ws; uint32_t* err; uint64_t* cnt; unsigned long long* bad; void *in, *out, *ref_out;
  const uint64_t bytes = 8ull << 30;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&ref_out, bytes / 2 + (64 << 20)));
  CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64)); CK(hipMalloc(&cnt, 64)); CK(hipMalloc(&bad, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* only = argc > 1 ? argv[1] : "";
  for (int rep = 0; rep < 2; ++rep) {
    harness<int64_t> h{1ull << 30, (int64_t*)in, (int64_t*)out, (int64_t*)ref_out, ws, err, cnt, bad, e0, e1};
    k_fill<int64_t><<<((1ull << 30) + 255) / 256, 256>>>(h.in, h.N); CK(hipDeviceSynchronize());
    h.run<false, true, 8, true, 4>("T1024 R8 RPB4 2/CU nt (shipped r04)");
    if (only[0]) continue;
    h.run<false, true, 8, true, 4, kThreads, 8, 0, true>("16-B stores");
    h.run<false, true, 8, true, 2, kThreads, 8, 0, true>("16-B stores RPB2");
    h.run<false, true, 8, true, 8, kThreads, 8, 0, true>("16-B stores RPB8");
    harness<int64_t> h2{(1ull << 30) - 3, (int64_t*)in, (int64_t*)out + 1, (int64_t*)ref_out, ws, err, cnt, bad, e0, e1};
    h2.run<false, true, 8, true, 4>("out at 8 B mod 16, n - 3: 8-B stores (reference)");
    h2.run<false, true, 8, true, 4, kThreads, 8, 0, true>("out at 8 B mod 16, n - 3: 16-B stores");
  }
  uint32_t e = 0; CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", e);
  return 0;
}
