// Microbenchmark (round 5, copyif9): the pipelined persistent copy_if
// (k_copy_if_pipe: one workgroup per CU, the tile's hits staged in LDS, the
// next tile's loads issued before the look-back and write-out) against the
// shipped one-tile-per-workgroup kernel, int64 at 2^30 and int32 at 2^31,
// predicate !(x < 0) on ~50 % hits; also ragged n and an output at 8 B mod
// 16.  Each variant's output is compared element for element with the
// shipped kernel's.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include -I../../hpx_amd/csrc copyif9.hip -o copyif9
#include <hpxhip/kernels/copy_if_kernel.hpp>
#include "internal.hpp"
#include <algorithm>
#include <cstdio>
#include <cstring>
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

int g_cus = 256;

template <typename T>
struct harness {
  using P = pred_fn<HPXHIP_P_NOT_LT, T>;
  uint64_t N; T *in, *out, *ref_out; char* ws; uint32_t* err; uint64_t* cnt; unsigned long long* bad;
  hipEvent_t e0, e1; uint64_t ref = 0;
  // kind 0: r04's k_copy_if; 1: k_copy_if_pipe with 16-B aligned vectors,
  // `per_cu` workgroups per CU; 2: k_copy_if_pipe with its vectors 128-B
  // aligned in the output (shipped after lease r5/ab)
  template <int KIND, int R = 8, int MINW = 4>
  void run(const char* name, int per_cu = 1) {
    using SV = uint32_t;
    const uint64_t ntiles = (N + tile_elems<T, R>() - 1) / tile_elems<T, R>();
    const size_t total = align_up(256 + ntiles * tile_state<SV>::bytes_per_tile(), 256);
    tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    auto launch = [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      if constexpr (KIND == 0) {
        constexpr bool W = sizeof(T) == 8;
        k_copy_if<T, P, true, R, 8, 0, SV, false, W, W ? 4 : 1, true, kThreads, W, W><<<ntiles, kThreads>>>(
            in, out, N, P{0}, cnt, reinterpret_cast<uint32_t*>(ws), st, ntiles);
      } else if constexpr (KIND == 1) {
        const uint64_t g = std::min<uint64_t>(ntiles, (uint64_t)g_cus * per_cu);
        k_copy_if_pipe<T, P, R, SV, MINW, 16><<<g, kThreads>>>(in, out, N, P{0}, cnt, reinterpret_cast<uint32_t*>(ws),
                                                               st, ntiles);
      } else {
        const uint64_t g = std::min<uint64_t>(ntiles, (uint64_t)g_cus * per_cu);
        k_copy_if_pipe<T, P, R, SV, MINW, 128><<<g, kThreads>>>(in, out, N, P{0}, cnt, reinterpret_cast<uint32_t*>(ws),
                                                                st, ntiles);
      }
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
    printf("%-4s %-40s min %7.3f ms med %7.3f ms  %7.1f GB/s  hits %.4f %s\n", sizeof(T) == 8 ? "i64" : "i32", name,
           t[0], t[5], B / t[0] / 1e6, double(c) / N, (c == ref && nbad == 0) ? "" : "OUTPUT MISMATCH");
    fflush(stdout);
  }
};

int main(int argc, char** argv) {
  char* ws; uint32_t* err; uint64_t* cnt; unsigned long long* bad; void *in, *out, *ref_out;
  const uint64_t bytes = 8ull << 30;
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes + 64)); CK(hipMalloc(&ref_out, bytes / 2 + (64 << 20)));
  CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64)); CK(hipMalloc(&cnt, 64)); CK(hipMalloc(&bad, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const bool quick = argc > 1 && !strcmp(argv[1], "quick");
  for (int rep = 0; rep < 2; ++rep) {
    {
      harness<int64_t> h{1ull << 30, (int64_t*)in, (int64_t*)out, (int64_t*)ref_out, ws, err, cnt, bad, e0, e1};
      k_fill<int64_t><<<((1ull << 30) + 255) / 256, 256>>>(h.in, h.N); CK(hipDeviceSynchronize());
      h.run<0>("T1024 R8 2/CU (shipped r04)");
      h.run<1>("pipe R8 1/CU");
      h.run<2>("pipe R8 1/CU, 128-B aligned vectors");
      if (!quick) {
        h.run<1>("pipe R8 grid 2/CU (LDS-bound to 1)", 2);
        h.run<1, 4, 8>("pipe R4 1/CU", 1);
        h.run<1, 4, 8>("pipe R4 2/CU", 2);
      }
    }
    if (!quick) {
      harness<int64_t> h{(1ull << 30) - 3, (int64_t*)in, (int64_t*)out + 1, (int64_t*)ref_out, ws, err, cnt, bad, e0, e1};
      h.run<0>("n - 3, out 8 B mod 16: shipped");
      h.run<1>("n - 3, out 8 B mod 16: pipe R8");
      h.run<2>("n - 3, out 8 B mod 16: pipe R8 128-B");
      harness<int64_t> hs{100003, (int64_t*)in, (int64_t*)out + 1, (int64_t*)ref_out, ws, err, cnt, bad, e0, e1};
      hs.run<0>("n 100003: shipped");
      hs.run<1>("n 100003: pipe R8");
      harness<int32_t> h4{1ull << 31, (int32_t*)in, (int32_t*)out, (int32_t*)ref_out, ws, err, cnt, bad, e0, e1};
      k_fill<int32_t><<<((1ull << 31) + 255) / 256, 256>>>(h4.in, h4.N); CK(hipDeviceSynchronize());
      h4.run<0>("T1024 R8 2/CU (shipped)");
      h4.run<1>("pipe R8 1/CU");
      h4.run<2>("pipe R8 1/CU, 128-B aligned vectors");
      harness<int32_t> h5{(1ull << 31) - 5, (int32_t*)in, (int32_t*)out + 1, (int32_t*)ref_out, ws, err, cnt, bad, e0, e1};
      h5.run<0>("n - 5, out 4 B mod 16: shipped");
      h5.run<1>("n - 5, out 4 B mod 16: pipe R8");
    }
  }
  uint32_t e = 0; CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", e);
  return 0;
}
