// Microbenchmark (round 5, seg10 = seg9's harness): the shipped k_bucket_sort
// (512 x 9: two ranked 8-bit LDS passes + run detection + insertion) against
// the one-pass form (ONE = 12/13/14: one ranking pass by LDS atomics on packed
// 16-bit bin counters, insertion inside the bins).  2^30 u64 keys in 4096-key
// segments (segment id in the top bits, random low bits), plus segments whose
// low bits take only 64 values (long bins: the odd-even / LSD fallback).  The
// fill is timed alone and subtracted; after each variant the keys are checked
// sorted and their sum / xor against the fill's.
// The ONE form lived in sort_kernel.hpp at commit cbbcee4 only (rejected,
// profiles/r05_ubench_seg10_onepass.log); build against that tree.
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include seg10.hip -o seg10
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill(uint64_t* k, uint64_t n, int segbits, int topbit, uint64_t lowmask) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = ((i >> segbits) << topbit) | ((z ^ (z >> 31)) & ((1ull << topbit) - 1) & lowmask);
}
// out[0] = unsorted pairs, out[1] = sum, out[2] = xor
__global__ void k_check(const uint64_t* k, uint64_t n, unsigned long long* out) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    if (i > 0 && k[i - 1] > k[i]) atomicAdd(&out[0], 1ull);
    atomicAdd(&out[1], static_cast<unsigned long long>(k[i]));
    atomicXor(&out[2], static_cast<unsigned long long>(k[i]));
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
void run(uint64_t* k, uint64_t n, int segbits, uint64_t lowmask, unsigned long long* chk, const char* tag, L launch) {
    const uint64_t S = 1ull << segbits, nseg = n / S;
    const int topbit = 64 - (30 - segbits);
    std::vector<uint64_t> hs(2 * nseg);
    for (uint64_t s = 0; s < nseg; ++s) { hs[2 * s] = s * S; hs[2 * s + 1] = (s + 1) * S; }
    uint64_t* seg;
    CK(hipMalloc(&seg, hs.size() * 8));
    CK(hipMemcpy(seg, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
    auto fill = [&] { hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, k, n, segbits, topbit, lowmask); };
    unsigned long long ref[3], got[3];
    fill();
    CK(hipMemset(chk, 0, 24));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, chk);
    CK(hipMemcpy(ref, chk, 24, hipMemcpyDeviceToHost));
    const float f = best(fill);
    const float b = best([&] { fill(); launch(seg, nseg, topbit); });
    CK(hipMemset(chk, 0, 24));
    hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, k, n, chk);
    CK(hipMemcpy(got, chk, 24, hipMemcpyDeviceToHost));
    printf("%-52s %7.3f ms (fill %.3f subtracted)  unsorted pairs %llu  %s\n", tag, b - f, f, got[0],
           (got[1] == ref[1] && got[2] == ref[2]) ? "checksums ok" : "CHECKSUM MISMATCH");
    fflush(stdout);
    CK(hipFree(seg));
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t* k;
    unsigned long long* chk;
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&chk, 24));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    using X = ordered_bits<uint64_t, false>;
    for (int rep = 0; rep < 2; ++rep) {
        for (int lowcase = 0; lowcase < 2; ++lowcase) {
            // lowcase 1: only 6 live low bits under each segment's top (64 values: long bins)
            const uint64_t lm = lowcase ? (0x3Full << 20) : ~0ull;
            const char* sfx = lowcase ? " [64 values/segment]" : "";
            char tag[128];
            snprintf(tag, sizeof tag, "shipped 512 x 9 (two passes)%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 4, false>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            snprintf(tag, sizeof tag, "ONE 13, MINW 4%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 4, false, 13>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            if (lowcase) continue;
            snprintf(tag, sizeof tag, "ONE 13, MINW 6%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 6, false, 13>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            snprintf(tag, sizeof tag, "ONE 12, MINW 4%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 4, false, 12>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            snprintf(tag, sizeof tag, "ONE 14, MINW 4%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 4, false, 14>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            snprintf(tag, sizeof tag, "ONE 12, MINW 6%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 512, 9, 16, uint32_t, false, false, false, 6, false, 12>),
                                   dim3(nseg), dim3(512), 0, 0, k, seg, top, X{});
            });
            snprintf(tag, sizeof tag, "ONE 13, 256 x 18, MINW 4%s", sfx);
            run(k, n, 12, lm, chk, tag, [&](uint64_t* seg, uint64_t nseg, int top) {
                hipLaunchKernelGGL((k_bucket_sort<uint64_t, X, 256, 18, 16, uint32_t, false, false, false, 4, false, 13>),
                                   dim3(nseg), dim3(256), 0, 0, k, seg, top, X{});
            });
        }
    }
    return 0;
}
