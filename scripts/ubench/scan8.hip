// Microbenchmark (round 5, scan8): the pipelined persistent scan
// (k_scan_pipe: one 1024-thread workgroup per CU, the tile's wave-local scan
// staged in LDS, the next tile's loads issued before the look-back and the
// stores) against the shipped k_scan shapes, int64 and f64 inclusive plus at
// 2^30; outputs compared bit for bit with the shipped kernel's on random
// inputs (f64: k_scan's DEFER association, which the pipe keeps), plus a
// ragged n and an exclusive scan.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I../../include scan8.hip -o scan8
#include <hpxhip/kernels/scan_kernel.hpp>
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hpxhip;

namespace hpxhip {
namespace scan_detail {
// Pipelined form (r05, measured here and rejected: 3.23-3.38 ms against
// 2.56 for the shipped k_scan at 2^30, profiles/r05_ubench_scan8_pipe.log): the copy_if
// structure (copy_if_kernel.hpp k_copy_if_pipe) for the scan.  A persistent
// grid of one 1024-thread workgroup per CU claims 128-KiB tiles in order; a
// tile's wave-local scan goes to LDS (the whole tile), the next tile's loads
// are issued into the registers it left, and only then does wave 0 take the
// tile's look-back and the workgroup store the tile from LDS with its
// prefixes added -- the stores run under the next tile's reads.  Same values
// as k_scan with DEFER (round r's prefix = the wave prefix folded with the
// totals of rounds < r, left to right; fixed-association look-back), so
// floating-point results are the shipped kernel's bit for bit.
template <typename T, typename Conv, typename Op, bool INCL, int ROUNDS, typename X = T>
__global__ __launch_bounds__(kThreads, 1) void k_scan_pipe(const T* in, T* out, uint64_t n, Conv conv, Op op,
                                                           X init, const X* prefix_dev, uint32_t* counter,
                                                           scan_state<X> st, uint64_t ntiles) {
    constexpr int V = 16 / sizeof(T);
    constexpr int WAVES = kThreads / kWave;
    constexpr uint64_t TILE = tile_elems<T, ROUNDS, kThreads>();
    constexpr uint64_t WAVE_ELEMS = TILE / WAVES;
    constexpr int ROUND_ELEMS = kWave * V;
    using VT = vec<T, V>;
    static_assert(std::is_same_v<X, T>, "built-in operators: the scanned type is the element type");

    __shared__ alignas(16) X s_stage[TILE];
    __shared__ X s_wave_total[WAVES];
    __shared__ X s_tr[WAVES][ROUNDS];  // round totals
    __shared__ X s_rp[WAVES][ROUNDS];  // round prefixes
    __shared__ uint32_t s_next;
    const X id = Op::template identity<X>();
    const int wave = threadIdx.x / kWave;
    const int lane = lane_id();

    auto claim = [&] {
        if (threadIdx.x == 0)
            s_next = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    VT raw[ROUNDS];
    auto load = [&](uint64_t t) {
        const uint64_t wbase = t * TILE + wave * WAVE_ELEMS;
        if (wbase + WAVE_ELEMS <= n) {
            const VT* src = reinterpret_cast<const VT*>(in + wbase);
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) raw[r] = ld_stream(&src[r * kWave + lane]);
        }
    };

    claim();
    __syncthreads();
    uint64_t tile = s_next;
    if (tile >= ntiles) return;
    load(tile);
    while (true) {
        const uint64_t tile_base = tile * TILE;
        const uint64_t wbase = tile_base + wave * WAVE_ELEMS;
        X x[ROUNDS][V];
        if (wbase + WAVE_ELEMS <= n) {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) x[r][e] = conv(raw[r].v[e]);
        } else {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const uint64_t i = wbase + (static_cast<uint64_t>(r) * kWave + lane) * V + e;
                    x[r][e] = i < n ? conv(in[i]) : id;
                }
        }
        // wave-local scan of each round (k_scan's DEFER form)
        X tr[ROUNDS];
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
            X local[V];
            X run = id;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const X nxt = op(run, x[r][e]);
                local[e] = INCL ? nxt : run;
                run = nxt;
            }
            const X incl = wave_inclusive_scan(run, op);
            const X excl = wave_shift_right<X, Op>(incl);
#pragma unroll
            for (int e = 0; e < V; ++e) x[r][e] = op(excl, local[e]);
            tr[r] = readlane(incl, kWave - 1);
        }
        X carry = id;
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) carry = op(carry, tr[r]);
        __syncthreads();  // (A) the previous tile's stores have read the stage
        {
            X* st_w = s_stage + wave * WAVE_ELEMS;
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) {
                VT y;
#pragma unroll
                for (int e = 0; e < V; ++e) y.v[e] = x[r][e];
                *reinterpret_cast<VT*>(st_w + (r * kWave + lane) * V) = y;
            }
            if (lane == 0) {
                s_wave_total[wave] = carry;
#pragma unroll
                for (int r = 0; r < ROUNDS; ++r) s_tr[wave][r] = tr[r];
            }
        }
        claim();
        __syncthreads();  // (B) the stage, the wave totals, the next tile id
        const uint64_t next = s_next;
        if (next < ntiles) load(next);
        if (wave == 0) tile_prefix<X, Op, WAVES, true, 1, true>(tile, st, op, prefix_dev, init, s_wave_total);
        __syncthreads();  // (C) wave prefixes
        if (threadIdx.x < WAVES * ROUNDS) {  // round prefixes: the wave's, then left to right
            const int w = threadIdx.x / ROUNDS, rr = threadIdx.x % ROUNDS;
            X rc = s_wave_total[w];
            for (int q = 0; q < rr; ++q) rc = op(rc, s_tr[w][q]);
            s_rp[w][rr] = rc;
        }
        __syncthreads();  // (D)
        // write-out: tile-local vector v covers elements [v V, v V + V) of
        // wave v V / WAVE_ELEMS, round (v V % WAVE_ELEMS) / ROUND_ELEMS
        const bool full = tile_base + TILE <= n;
#pragma unroll
        for (int k = 0; k < static_cast<int>(TILE / V / kThreads); ++k) {
            const uint32_t v = k * kThreads + threadIdx.x;
            const uint32_t i0 = v * V;
            const X rp = s_rp[i0 / WAVE_ELEMS][(i0 % WAVE_ELEMS) / ROUND_ELEMS];
            const VT y = *reinterpret_cast<const VT*>(s_stage + i0);
            if (full) {
                VT z;
#pragma unroll
                for (int e = 0; e < V; ++e) z.v[e] = unwrap_value(op(rp, y.v[e]));
                st_stream(reinterpret_cast<VT*>(out + tile_base) + v, z);
            } else {
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (tile_base + i0 + e < n) out[tile_base + i0 + e] = unwrap_value(op(rp, y.v[e]));
            }
        }
        if (next >= ntiles) break;
        tile = next;
    }
}

}  // namespace scan_detail
}  // namespace hpxhip

template <typename T> struct idc { __device__ T operator()(T x) const { return x; } };

template <typename T>
__global__ void k_fill(T* p, uint64_t n, int mode) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull; z ^= z >> 29; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 32;
    if (mode == 0) p[i] = T(1);
    else if constexpr (sizeof(T) == 8 && std::is_floating_point_v<T>) p[i] = T((z >> 11) * 0x1.0p-53) - T(0.5);
    else p[i] = T(z & 0xffff) - T(0x8000);
  }
}
template <typename T>
__global__ void k_diff(const T* a, const T* b, uint64_t n, unsigned long long* bad) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    if (__builtin_bit_cast(uint64_t, a[i]) != __builtin_bit_cast(uint64_t, b[i])) atomicAdd(bad, 1ull);
}

int g_cus = 256;

template <typename T>
struct bench {
  using Conv = idc<T>;
  uint64_t N; T *in, *out, *ref; char* ws; uint32_t* err; unsigned long long* bad; hipEvent_t e0, e1;
  template <typename L> float time(L launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 15; ++r) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    return t[0];
  }
  template <bool INCL, int R, int TH, int MINW, bool DEFER>
  void shipped(uint64_t n) {
    const uint64_t tile = scan_detail::tile_elems<T, R, TH>();
    const uint64_t ntiles = (n + tile - 1) / tile;
    const size_t total = 256 + ntiles * scan_detail::scan_state<T>::bytes_per_tile();
    scan_detail::scan_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    CK(hipMemsetAsync(ws, 0, total, 0));
    scan_detail::k_scan<T, Conv, op_plus, INCL, true, R, TH, true, MINW, false, 1, false, true, T, DEFER, true><<<ntiles, TH>>>(
        in, out, n, Conv{}, op_plus{}, T(0), static_cast<const T*>(nullptr), reinterpret_cast<uint32_t*>(ws), st);
  }
  template <bool INCL, int R>
  void pipe(uint64_t n, int per_cu = 1) {
    const uint64_t tile = scan_detail::tile_elems<T, R, 1024>();
    const uint64_t ntiles = (n + tile - 1) / tile;
    const size_t total = 256 + ntiles * scan_detail::scan_state<T>::bytes_per_tile();
    scan_detail::scan_state<T> st{reinterpret_cast<uint64_t*>(ws + 256), err};
    CK(hipMemsetAsync(ws, 0, total, 0));
    const uint64_t grid = std::min<uint64_t>(ntiles, uint64_t(g_cus) * per_cu);
    scan_detail::k_scan_pipe<T, Conv, op_plus, INCL, R><<<grid, 1024>>>(in, out, n, Conv{}, op_plus{}, T(0),
        static_cast<const T*>(nullptr), reinterpret_cast<uint32_t*>(ws), st, ntiles);
  }
  unsigned long long compare(uint64_t n) {
    CK(hipMemset(bad, 0, 8));
    k_diff<T><<<8192, 256>>>(out, ref, n, bad);
    unsigned long long h; CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost)); return h;
  }
};

template <typename T, int RS, int TS, int MS, bool DS>
void suite(bench<T>& b, const char* tn) {
  const uint64_t N = b.N;
  // speed (ones)
  k_fill<T><<<8192, 256>>>(b.in, N, 0); CK(hipDeviceSynchronize());
  const float ts = b.time([&] { b.template shipped<true, RS, TS, MS, DS>(N); });
  const float t8 = b.time([&] { b.template pipe<true, 8>(N); });
  const float t4 = b.time([&] { b.template pipe<true, 4>(N); });
  const float t42 = b.time([&] { b.template pipe<true, 4>(N, 2); });
  const double B = 2.0 * sizeof(T) * N;
  printf("%s incl 2^30: shipped %.3f ms (%.1f GB/s)  pipe R8 %.3f ms (%.1f)  pipe R4 %.3f ms (%.1f)  R4 grid 2/CU %.3f ms (%.1f)\n",
         tn, ts, B / ts / 1e6, t8, B / t8 / 1e6, t4, B / t4 / 1e6, t42, B / t42 / 1e6);
  // bit-exactness on random data: inclusive at N, ragged, exclusive
  k_fill<T><<<8192, 256>>>(b.in, N, 1); CK(hipDeviceSynchronize());
  for (uint64_t n : {N, N - 12345, uint64_t(1000003), uint64_t(777)}) {
    b.template shipped<true, RS, TS, MS, DS>(n); CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.ref, b.out, n * sizeof(T), hipMemcpyDeviceToDevice));
    b.template pipe<true, 8>(n); CK(hipDeviceSynchronize());
    const auto d8 = b.compare(n);
    b.template shipped<false, RS, TS, MS, DS>(n); CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.ref, b.out, n * sizeof(T), hipMemcpyDeviceToDevice));
    b.template pipe<false, 8>(n); CK(hipDeviceSynchronize());
    const auto e8 = b.compare(n);
    printf("%s n %llu: inclusive pipe vs shipped mismatches %llu, exclusive %llu\n", tn, (unsigned long long)n, d8, e8);
  }
  fflush(stdout);
}

int main() {
  const uint64_t N = 1ull << 30;
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  char* ws; uint32_t* err; unsigned long long* bad; void *in, *out, *ref;
  CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8)); CK(hipMalloc(&ref, N * 8)); CK(hipMalloc(&ws, 64 << 20));
  CK(hipMalloc(&err, 64)); CK(hipMalloc(&bad, 64));
  CK(hipMemset(err, 0, 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  bench<int64_t> bi{N, (int64_t*)in, (int64_t*)out, (int64_t*)ref, ws, err, bad, e0, e1};
  bench<double> bd{N, (double*)in, (double*)out, (double*)ref, ws, err, bad, e0, e1};
  for (int rep = 0; rep < 2; ++rep) {
    suite<int64_t, 16, 512, 4, false>(bi, "i64");
    suite<double, 16, 512, 4, true>(bd, "f64");
  }
  uint32_t h = 0; CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost)); printf("deverr %u\n", h);
  return 0;
}
