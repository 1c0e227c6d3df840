// Microbenchmark (round 5, seg7 = seg6 with the persistent form's opaque
// thread ids only in k_segp: seg6 had them in every kernel, 5.1 -> 8.7 ms):
// (seg6) the segment sort's run detection from a
// 16-bit prefix array.  seg5 (profiles/r05_ubench_seg5_phases.log) put the
// detection + insertion at ~0.6 of 5.0 ms (three 8-B LDS reads per key).
// PRE16: the second LDS pass also scatters each key's 16 sorted bits into
// s_pre (2 B per key); the detection reads 8 prefixes per thread as one 16-B
// LDS read, and the run walk compares prefixes, not keys.  Against the
// shipped k_bucket_sort and k_segx with the LDS detection.
// 2^30 u64 keys, 4096-key segments with the segment id in the top bits and
// random low bits ((begin, end) pairs); the fill is timed alone and
// subtracted; sortedness checked after each shape (ablations are unsorted).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include seg7.hip -o seg7
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <typename U, typename X, int ABL, bool PRE16, int THREADS = 512, int ITEMS = 9>
struct segx {
    static constexpr int WAVES = THREADS / kWave;
    static constexpr int CHUNK = ITEMS * kWave;
    static constexpr int BITS = static_cast<int>(sizeof(U) * 8);
    struct smem {};
    __device__ static __forceinline__ void load(const U* keys, uint64_t b, uint32_t m, U (&k)[ITEMS]) {
        const int lane = lane_id(), wave = threadIdx.x / kWave;
        const uint32_t wbase = static_cast<uint32_t>(wave) * CHUNK;
        const uint32_t have = m > wbase ? m - wbase : 0u;
        const int nfull = static_cast<int>(have >= static_cast<uint32_t>(CHUNK) ? ITEMS : have / kWave);
        const uint64_t tail_mask = (have % kWave) ? (~0ull >> (kWave - have % kWave)) : 0ull;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t act = r < nfull ? ~0ull : (r == nfull ? tail_mask : 0ull);
            k[r] = ((act >> lane) & 1u) ? ld_stream(&keys[b + wbase + r * kWave + lane]) : U(0);
        }
    }
    template <bool OPAQUE = false>
    __device__ static __forceinline__ void sort(U* __restrict__ keys, uint64_t b, uint32_t m, int top_single, X xf,
                                                U (&k)[ITEMS], smem& sm) {
    // LDS declared here, not passed in: a reference to a workgroup array
    // passed down became a flat pointer (flat loads/stores: 5.1 -> 8.7 ms)
    __shared__ alignas(16) U s_keys[THREADS * ITEMS];
    __shared__ uint16_t s_whist[WAVES][kRadix];
    __shared__ uint32_t s_wsum[kRadix / kWave];
    __shared__ U s_ends[2];
    __shared__ alignas(16) uint16_t s_pre[PRE16 ? THREADS * ITEMS + 16 : 1];
    (void)sm;
    int t = threadIdx.x, lane = lane_id();
    if constexpr (OPAQUE) asm volatile("" : "+v"(t), "+v"(lane));
    const int wave = t / kWave;
    if (m < 2) return;
    const uint32_t wbase = static_cast<uint32_t>(wave) * CHUNK;
    const uint32_t have = m > wbase ? m - wbase : 0u;
    const int nfull = static_cast<int>(have >= static_cast<uint32_t>(CHUNK) ? ITEMS : have / kWave);
    const uint64_t tail_mask = (have % kWave) ? (~0ull >> (kWave - have % kWave)) : 0ull;
    auto active = [&](int r) -> uint64_t { return r < nfull ? ~0ull : (r == nfull ? tail_mask : 0ull); };
    U* gkeys = keys + b;
    U* lkeys = s_keys + wbase;
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
    auto pass = [&](int shift, bool last) {
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
                if constexpr (PRE16)
                    if (last) s_pre[pos] = static_cast<uint16_t>(xf(k[r]) >> (top - 16));
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
        pass(lo1 > 0 ? lo1 : 0, (ABL & 2) != 0 && top > 16);
        if constexpr ((ABL & 2) == 0) {
            reload();
            const int lo2 = top - 8;
            pass(lo2 > 0 ? lo2 : 0, top > 16);
        }
    }
    if constexpr ((ABL & 7) == 0) {
        if (top > 16) {
            const int fs = top - 16;
            auto pre = [&](const U& x) { return xf(x) >> fs; };
            uint32_t starts = 0;
            if constexpr (PRE16) {
                // groups of 8 positions: one 16-B read of their prefixes, and
                // the neighbours on either side
                using P8 = vec<uint16_t, 8>;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t g = static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                    const uint32_t base = 8 * g;
                    if (base + 1 >= m) continue;
                    const P8 v = reinterpret_cast<const P8*>(s_pre)[g];
                    const uint16_t before = base > 0 ? s_pre[base - 1] : uint16_t(0);
                    const uint16_t after = s_pre[base + 8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t idx = base + i;
                        const uint16_t a = v.v[i];
                        const uint16_t nx = i < 7 ? v.v[i < 7 ? i + 1 : 7] : after;
                        const uint16_t pv = i > 0 ? v.v[i > 0 ? i - 1 : 0] : before;
                        if (idx + 1 < m && a == nx && (idx == 0 || pv != a)) starts |= 1u << (8 * j + i);
                    }
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
                __syncthreads();
            }
            int long_run = 0;
            while (starts) {
                const int j = __builtin_ctz(starts);
                starts &= starts - 1;
                const uint32_t s = PRE16 ? 8 * (static_cast<uint32_t>(t) + static_cast<uint32_t>(j / 8) * THREADS) + j % 8
                                         : static_cast<uint32_t>(t) + static_cast<uint32_t>(j) * THREADS;
                uint32_t e = s + 2;
                if constexpr (PRE16) {
                    const uint16_t p0 = s_pre[s];
                    while (e < m && e - s <= kRunMax && s_pre[e] == p0) ++e;
                } else {
                    const U p0 = pre(s_keys[s]);
                    while (e < m && e - s <= kRunMax && pre(s_keys[e]) == p0) ++e;
                }
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
};

template <typename U, typename X, int ABL, bool PRE16, int THREADS = 512, int ITEMS = 9, int MINW = 6>
__global__ __launch_bounds__(THREADS, MINW) void k_segx(U* __restrict__ keys, const uint64_t* __restrict__ seg,
                                                         int top_single, X xf) {
    using S = segx<U, X, ABL, PRE16, THREADS, ITEMS>;
    typename S::smem sm;
    const uint64_t b = seg[2 * blockIdx.x];
    const uint32_t m = static_cast<uint32_t>(seg[2 * blockIdx.x + 1] - b);
    U k[ITEMS];
    S::load(keys, b, m, k);
    S::sort(keys, b, m, top_single, xf, k, sm);
}

// persistent: workgroup w sorts segments w, w + G, ...; the next segment's
// keys are loaded into registers before the current one is sorted
template <typename U, typename X, int ABL, bool PRE16, int THREADS = 512, int ITEMS = 9, int MINW = 4>
__global__ __launch_bounds__(THREADS, MINW) void k_segp(U* __restrict__ keys, const uint64_t* __restrict__ seg,
                                                         uint32_t nseg, int top_single, X xf) {
    using S = segx<U, X, ABL, PRE16, THREADS, ITEMS>;
    typename S::smem sm;
    uint32_t bk = blockIdx.x;
    if (bk >= nseg) return;
    U k[ITEMS], kn[ITEMS];
    uint64_t b = seg[2 * bk];
    uint32_t m = static_cast<uint32_t>(seg[2 * bk + 1] - b);
    S::load(keys, b, m, k);
    while (true) {
        const uint32_t nb = bk + gridDim.x;
        uint64_t nb_b = 0;
        uint32_t nb_m = 0;
        if (nb < nseg) {
            nb_b = seg[2 * nb];
            nb_m = static_cast<uint32_t>(seg[2 * nb + 1] - nb_b);
            S::load(keys, nb_b, nb_m, kn);
        }
        S::template sort<true>(keys, b, m, top_single, xf, k, sm);
        __syncthreads();
        if (nb >= nseg) break;
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) k[r] = kn[r];
        bk = nb;
        b = nb_b;
        m = nb_m;
    }
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
static int g_cus = 256;
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
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    using X = ordered_bits<uint64_t, false>;
    for (int rep = 0; rep < 2; ++rep) {
        run(k, n, 12, bad, "shipped k_bucket_sort 512 x 9", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 6>), dim3(nseg),
                               dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "k_segx full (LDS detection)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 0, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "k_segx PRE16 (prefix-array detection)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 0, true>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "k_segp persistent prefetch, 2/CU", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segp<uint64_t, X, 0, false>), dim3(2 * g_cus), dim3(512), 0, 0, k, seg,
                               (uint32_t)nseg, top, X{});
        });
        run(k, n, 12, bad, "k_segp persistent prefetch PRE16, 2/CU", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segp<uint64_t, X, 0, true>), dim3(2 * g_cus), dim3(512), 0, 0, k, seg,
                               (uint32_t)nseg, top, X{});
        });
        run(k, n, 12, bad, "k_segp persistent prefetch PRE16, grid 3/CU", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segp<uint64_t, X, 0, true>), dim3(3 * g_cus), dim3(512), 0, 0, k, seg,
                               (uint32_t)nseg, top, X{});
        });
        run(k, n, 12, bad, "ABL1 two passes, no runs (unsorted)", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 1, false>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
        run(k, n, 12, bad, "ABL1 PRE16 two passes + prefix scatter", [&](uint64_t* seg, uint64_t nseg, int top) {
            hipLaunchKernelGGL((k_segx<uint64_t, X, 1, true>), dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
        });
    }
    return 0;
}
