// Microbenchmark (round 5, seg5): where the segment sort's time goes, and a
// register-side run detection.  The shipped k_bucket_sort (512 x 9, ~4096-key
// segments, three workgroups per CU) against k_segx, the same algorithm for
// keys only with ablations:
//   ABL 1: no run detection / insertion (two LDS passes + write-back),
//   ABL 2: one LDS pass only, ABL 4: no LDS pass (load + write-back),
//   DETREG: runs detected from the reloaded registers (neighbours by lane
//   shuffles) instead of three LDS reads per key.
// 2^30 u64 keys, 4096-key segments with the segment id in the top bits and
// random low bits ((begin, end) pairs); the fill is timed alone and
// subtracted; sortedness checked after each shape (ablations are unsorted).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include seg5.hip -o seg5
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <typename U, typename X, int ABL, bool DETREG, int THREADS = 512, int ITEMS = 9, int MINW = 6>
__global__ __launch_bounds__(THREADS, MINW) void k_segx(U* __restrict__ keys, const uint64_t* __restrict__ seg,
                                                         int top_single, X xf) {
    constexpr int WAVES = THREADS / kWave;
    constexpr int CHUNK = ITEMS * kWave;
    constexpr int BITS = static_cast<int>(sizeof(U) * 8);
    __shared__ alignas(16) U s_keys[THREADS * ITEMS];
    __shared__ uint16_t s_whist[WAVES][kRadix];
    __shared__ uint32_t s_wsum[kRadix / kWave];
    __shared__ U s_ends[2];
    const int t = threadIdx.x, lane = lane_id(), wave = t / kWave;
    const uint64_t b = seg[2 * blockIdx.x];
    const uint32_t m = static_cast<uint32_t>(seg[2 * blockIdx.x + 1] - b);
    if (m < 2) return;
    const uint32_t wbase = static_cast<uint32_t>(wave) * CHUNK;
    const uint32_t have = m > wbase ? m - wbase : 0u;
    const int nfull = static_cast<int>(have >= static_cast<uint32_t>(CHUNK) ? ITEMS : have / kWave);
    const uint64_t tail_mask = (have % kWave) ? (~0ull >> (kWave - have % kWave)) : 0ull;
    auto active = [&](int r) -> uint64_t { return r < nfull ? ~0ull : (r == nfull ? tail_mask : 0ull); };
    U* gkeys = keys + b;
    U* lkeys = s_keys + wbase;
    U k[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool on = (active(r) >> lane) & 1u;
        k[r] = on ? ld_stream(&gkeys[wbase + r * kWave + lane]) : U(0);
    }
    {
        const uint32_t last = m - 1;
        const uint32_t lw = last / CHUNK, lo = last % CHUNK;
        if (t == 0) s_ends[0] = k[0];
        if (static_cast<uint32_t>(wave) == lw && static_cast<uint32_t>(lane) == lo % kWave) {
            U x = k[0];
#pragma unroll
            for (int r = 1; r < ITEMS; ++r)
                if (static_cast<uint32_t>(r) == lo / kWave) x = k[r];
            s_ends[1] = x;
        }
        __syncthreads();
    }
    const U diff = xf(s_ends[0]) ^ xf(s_ends[1]);
    int top = top_single;
    if (diff) {
        const int hb = BITS - (sizeof(U) == 8 ? __builtin_clzll(static_cast<uint64_t>(diff))
                                               : __builtin_clz(static_cast<uint32_t>(diff)));
        top = hb > top ? hb : top;
    }
    if (top <= 0) return;
    auto pass = [&](int shift) {
        __syncthreads();
        for (int i = t; i < WAVES * kRadix / 2; i += THREADS) reinterpret_cast<uint32_t*>(&s_whist[0][0])[i] = 0;
        __syncthreads();
        uint32_t rank2[(ITEMS + 1) / 2];
#pragma unroll
        for (int r = 0; r < (ITEMS + 1) / 2; ++r) rank2[r] = 0;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = active(r);
            if (act == 0) break;
            const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
            const uint64_t peers = match_digit(d, act);
            const uint32_t below = peers_below(peers);
            const uint32_t cnt = static_cast<uint32_t>(__builtin_popcountll(peers));
            const uint32_t old = s_whist[wave][d];
            rank2[r / 2] |= (old + below) << (16 * (r & 1));
            if (((act >> lane) & 1u) && below == 0) s_whist[wave][d] = static_cast<uint16_t>(old + cnt);
        }
        __syncthreads();
        uint32_t count = 0, incl = 0;
        if (t < kRadix) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
                const uint32_t c = s_whist[w][t];
                s_whist[w][t] = static_cast<uint16_t>(count);
                count += c;
            }
            incl = wave_inclusive_scan(count, op_plus{});
            if (lane == kWave - 1) s_wsum[wave] = incl;
        }
        __syncthreads();
        if (t < kRadix) {
            uint32_t pre = 0;
#pragma unroll
            for (int w = 0; w < kRadix / kWave; ++w)
                if (w < wave) pre += s_wsum[w];
            const uint32_t loc = pre + incl - count;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) s_whist[w][t] = static_cast<uint16_t>(s_whist[w][t] + loc);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = active(r);
            if (act == 0) break;
            if ((act >> lane) & 1u) {
                const uint32_t d = static_cast<uint32_t>(xf(k[r]) >> shift) & 0xffu;
                const uint32_t pos = s_whist[wave][d] + ((rank2[r / 2] >> (16 * (r & 1))) & 0xffffu);
                s_keys[pos] = k[r];
            }
        }
        __syncthreads();
    };
    auto reload = [&] {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const bool on = (active(r) >> lane) & 1u;
            k[r] = on ? lkeys[r * kWave + lane] : U(0);
        }
    };
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r)
            if ((active(r) >> lane) & 1u) lkeys[r * kWave + lane] = k[r];
        __syncthreads();
    } else {
        const int lo1 = top - 16;
        pass(lo1 > 0 ? lo1 : 0);
        if constexpr ((ABL & 2) == 0) {
            reload();
            const int lo2 = top - 8;
            pass(lo2 > 0 ? lo2 : 0);
        }
    }
    if constexpr ((ABL & 7) == 0) {
        if (top > 16) {
            const int fs = top - 16;
            auto pre = [&](const U& x) { return xf(x) >> fs; };
            uint32_t starts = 0;
            if constexpr (DETREG) {
                // keys in the wave-chunk layout s_keys[wbase + r*64 + lane]; a
                // key's successor is lane + 1 of its round, or lane 0 of the
                // next round (the next wave's chunk: one LDS read)
                reload();
                const U after = wbase + CHUNK < m ? pre(s_keys[wbase + CHUNK]) : U(0);
                const U before = wave > 0 ? pre(s_keys[wbase - 1]) : U(0);
#pragma unroll
                for (int r = 0; r < ITEMS; ++r) {
                    const U a = pre(k[r]);
                    const U nx0 = __shfl_down(a, 1);
                    const U pv0 = __shfl_up(a, 1);
                    const U nr = r + 1 < ITEMS ? pre(k[r + 1 < ITEMS ? r + 1 : r]) : after;
                    const U pr = r > 0 ? pre(k[r > 0 ? r - 1 : 0]) : before;
                    const U nx = lane == kWave - 1 ? (r + 1 < ITEMS ? __shfl(nr, 0) : after) : nx0;
                    const U pv = lane == 0 ? (r > 0 ? __shfl(pr, kWave - 1) : before) : pv0;
                    const uint32_t i = wbase + r * kWave + lane;
                    if (i + 1 < m && a == nx && (i == 0 || pv != a)) starts |= 1u << r;
                }
            } else {
#pragma unroll 3
                for (int j = 0; j < ITEMS; ++j) {
                    const uint32_t i = static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                    if (i + 1 < m) {
                        const U a = pre(s_keys[i]);
                        if (a == pre(s_keys[i + 1]) && (i == 0 || pre(s_keys[i - 1]) != a)) starts |= 1u << j;
                    }
                }
            }
            __syncthreads();
            int long_run = 0;
            while (starts) {
                const int j = __builtin_ctz(starts);
                starts &= starts - 1;
                const uint32_t s = DETREG ? wbase + j * kWave + lane
                                          : static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                const U p0 = pre(s_keys[s]);
                uint32_t e = s + 2;
                while (e < m && e - s <= kRunMax && pre(s_keys[e]) == p0) ++e;
                if (e - s > kRunMax) {
                    long_run = 1;
                    continue;
                }
                for (uint32_t p = s + 1; p < e; ++p) {
                    const U x = s_keys[p];
                    uint32_t q = p;
                    while (q > s && xf(s_keys[q - 1]) > xf(x)) --q;
                    if (q == p) continue;
                    for (uint32_t r = p; r > q; --r) s_keys[r] = s_keys[r - 1];
                    s_keys[q] = x;
                }
            }
            __syncthreads();
            (void)long_run;
        }
    }
    for (uint32_t i = t; i < m; i += THREADS) st_stream(&gkeys[i], s_keys[i]);
}

__global__ void k_fill(uint64_t* k, uint64_t n, int segbits, int topbit) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = ((i >> segbits) << topbit) | ((z ^ (z >> 31)) & ((1ull << topbit) - 1));
}
__global__ void k_check(const uint64_t* k, uint64_t n, unsigned long long* bad) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i == 0 || i >= n) return;
    if (k[i - 1] > k[i]) atomicAdd(bad, 1ull);
}

static hipEvent_t e0, e1;
template <typename F>
float best(F f) {
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[0];
}

template <typename L>
void run(uint64_t* k, uint64_t n, int segbits, unsigned long long* bad, const char* tag, L launch) {
    const uint64_t S = 1ull << segbits, nseg = n / S;
    const int topbit = 64 - (30 - segbits);
    std::vector<uint64_t> hs(2 * nseg);
    for (uint64_t s = 0; s < nseg; ++s) { hs[2 * s] = s * S; hs[2 * s + 1] = (s + 1) * S; }
    uint64_t* seg;
    CK(hipMalloc(&seg, hs.size() * 8));
    CK(hipMemcpy(seg, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    auto fill = [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, segbits, topbit); };
    const float f = best(fill);
    const float b = best([&] { fill(); launch(seg, nseg, topbit); });
    CK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    printf("%-52s %7.3f ms (fill %.3f subtracted)  unsorted pairs %llu\n", tag, b - f, f, hb);
    fflush(stdout);
    CK(hipFree(seg));
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t* k;
    unsigned long long* bad;
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&bad, 8));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    using X = ordered_bits<uint64_t, false>;
    for (int rep = 0; rep < 2; ++rep) {
        run(k, n, 12, bad, "shipped k_bucket_sort 512 x 9", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 6>), dim3(nseg),
                               dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "k_segx full (LDS detection)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 0, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "k_segx DETREG (register detection)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 0, true>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "ABL1 two passes, no runs (unsorted)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 1, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "ABL2 one pass (unsorted)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 2, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "ABL4 load + LDS + store only", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 4, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
    }
    return 0;
}
