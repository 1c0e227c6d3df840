// Microbenchmark: shipped one-tile-per-workgroup scan (scan_kernel.hpp) vs
// the persistent double-buffered scan (scan_pipe.hpp), 2^30 int64 / f64
// inclusive plus-scan, all variants in one process; each result spot-checked.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None -I../../include scan2.hip -o scan2
#include "../../hpx_amd/csrc/scan_kernel.hpp"
#include "scan_pipe.hpp"
#include "../../hpx_amd/csrc/internal.hpp"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;


// Ablation of the shipped structure (one 256 KiB tile per 1024-thread
// workgroup): ID = 0 atomic counter, 1 blockIdx (measurement only: relies on
// dispatch order); LB = look-back on/off; SCAN = 0 skips the arithmetic (a
// tile-shaped copy).
template <int ID, bool LB, bool SCAN>
__global__ __launch_bounds__(1024, 1) void k_abl(const int64_t* in, int64_t* out, uint64_t n, uint32_t* counter,
                                                 tile_state<int64_t> st) {
  using T = int64_t; constexpr int R = 16, V = 2, WAVES = 16; using VT = vec<T, V>;
  constexpr uint64_t TILE = 1024ull * R * V, WAVE_ELEMS = TILE / WAVES;
  __shared__ uint32_t s_tile; __shared__ T s_wave_total[WAVES];
  if constexpr (ID == 0) { if (threadIdx.x == 0) s_tile = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); __syncthreads(); }
  const uint64_t tile = ID == 0 ? s_tile : blockIdx.x;
  const int wave = threadIdx.x / kWave, lane = lane_id();
  const uint64_t wbase = tile * TILE + wave * WAVE_ELEMS;
  VT x[R]; const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
  for (int r = 0; r < R; ++r) x[r] = ld_stream(&src[r * kWave + lane]);
  T pre = 0;
  if constexpr (SCAN) {
    op_plus op; T carry = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      T l0 = x[r].v[0], l1 = l0 + x[r].v[1];
      const T incl = wave_inclusive_scan(l1, op); const T excl = wave_shift_right<T, op_plus>(incl);
      const T p = carry + excl; x[r].v[0] = p + l0; x[r].v[1] = p + l1; carry += readlane(incl, kWave - 1);
    }
    if (lane == 0) s_wave_total[wave] = carry;
    __syncthreads();
    if (wave == 0) scan_detail::tile_prefix<T, op_plus, WAVES, LB>(tile, st, op, nullptr, T(0), s_wave_total);
    __syncthreads();
    pre = s_wave_total[wave];
  }
  VT* dst = reinterpret_cast<VT*>(out + wbase);
#pragma unroll
  for (int r = 0; r < R; ++r) { VT y; y.v[0] = pre + x[r].v[0]; y.v[1] = pre + x[r].v[1]; dst[r * kWave + lane] = y; }
}

template <typename T>
struct bench {
  using Conv = unary_fn<HPXHIP_U_IDENTITY, T>;
  uint64_t N; T *in, *out; char* ws; uint32_t* err; hipEvent_t e0, e1; int cus;
  template <typename L> void run(const char* name, L launch, uint64_t check_tile) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    const double B = 2.0 * sizeof(T) * N;
    bool ok = true;
    const uint64_t idx[5] = {0, check_tile - 1, check_tile, N / 2 + 12345, N - 1};
    if (check_tile)
      for (uint64_t i : idx) { T h; CK(hipMemcpy(&h, out + i, sizeof(T), hipMemcpyDeviceToHost)); ok = ok && h == T(i + 1); }
    printf("%-44s min %7.3f ms med %7.3f ms  %7.1f GB/s (%5.1f%%) %s\n", name, t[0], t[7], B / t[0] / 1e6,
           B / t[0] / 1e6 / 80.0, ok ? "ok" : "MISMATCH");
    fflush(stdout);
  }
  template <int ID, bool LB, bool SCAN>
  void abl(const char* name) {
    const uint64_t tile = 32768, ntiles = N / tile;
    const size_t total = align_up(256 + ntiles * tile_state<T>::bytes_per_tile(), 256);
    tile_state<int64_t> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      k_abl<ID, LB, SCAN><<<ntiles, 1024>>>((const int64_t*)in, (int64_t*)out, N, reinterpret_cast<uint32_t*>(ws), st);
    }, SCAN ? tile : 0);
  }
  template <int R, int TH, int LBK = 1, int MINW = 1>
  void shipped(const char* name) {
    const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
    const uint64_t ntiles = (N + tile - 1) / tile;
    const size_t total = align_up(256 + ntiles * tile_state<T>::bytes_per_tile(), 256);
    tile_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      scan_detail::k_scan<T, Conv, op_plus, true, true, R, TH, true, MINW, false, LBK><<<ntiles, TH>>>(
            in, out, N, Conv{0, 0}, op_plus{}, T(0), nullptr, reinterpret_cast<uint32_t*>(ws), st);
    }, tile);
  }
  template <int R>
  void pipe(const char* name, int wg_per_cu) {
    const uint64_t tile = scan_detail::pipe_shape<T, R>::TILE;
    const uint64_t ntiles = (N + tile - 1) / tile;
    const size_t total = align_up(256 + ntiles * tile_state<T>::bytes_per_tile(), 256);
    tile_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    const unsigned grid = std::min<uint64_t>(ntiles, uint64_t(cus) * wg_per_cu);
    run(name, [&] {
      CK(hipMemsetAsync(ws, 0, total, 0));
      scan_detail::k_scan_pipe<T, Conv, op_plus, true, R><<<grid, scan_detail::kPipeThreads>>>(
            in, out, N, Conv{0, 0}, op_plus{}, T(0), nullptr, reinterpret_cast<uint32_t*>(ws), st, ntiles);
    }, tile);
  }
};


template <typename T>
__global__ void k_ones(T* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) p[i] = T(1);
}

int main() {
  const uint64_t N = 1ull << 30;
  char* ws; uint32_t* err; void *in, *out;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ws, 64 << 20)); CK(hipMalloc(&err, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  bench<int64_t> bi{N, (int64_t*)in, (int64_t*)out, ws, err, e0, e1, cus};
  bench<double> bd{N, (double*)in, (double*)out, ws, err, e0, e1, cus};
  for (int rep = 0; rep < 2; ++rep) {
    k_ones<int64_t><<<8192, 256>>>((int64_t*)in, N); CK(hipDeviceSynchronize());
    bi.shipped<16, 1024>("i64 shipped T1024 R16 (256 KiB, 1/CU)");
    bi.shipped<16, 512, 1, 2>("i64 T512 R16 MINW2 (128 KiB, 2/CU)");
    bi.shipped<8, 1024, 1, 2>("i64 T1024 R8 MINW2 (128 KiB, 2/CU)");
    bi.shipped<16, 256, 1, 4>("i64 T256 R16 MINW4 (64 KiB, 4/CU)");
    bi.shipped<8, 512, 1, 4>("i64 T512 R8 MINW4 (64 KiB, 4/CU)");
    bi.shipped<8, 512, 4, 4>("i64 T512 R8 MINW4 K4 (64 KiB, 4/CU)");
    bi.shipped<12, 512, 1, 2>("i64 T512 R12 MINW2 (96 KiB, 2/CU)");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
