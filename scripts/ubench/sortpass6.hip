// Microbenchmark (round 5): the 18-bit sort's SECOND prefix pass (the top 9
// bits of 2^30 random u64 keys, over the first pass's field-ordered output)
// as shipped in r05 -- 8 field regions, one per XCD (k_onesweep XREG + SEG),
// each with its own look-back and bin starts (k_region_plan from the joint
// histogram of k_hist_tiles) -- against look-back widths LBB 1/2/4/8 and
// against the same regions claimed from one global counter (no XCD
// affinity, SEG + PERSIST-free global order: regions back to back).  Output
// checksums compared across variants; best of 7 (HIP events).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include sortpass6.hip -o sortpass6
#include <hpxhip/kernels/sort_kernel.hpp>

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace hpxhip;
using namespace hpxhip::sort_detail;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill_rand(uint64_t* k, uint64_t n) {
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i ^ 0x5EEDull) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    k[i] = z ^ (z >> 31);
}
// position-weighted checksum: equal iff (with overwhelming probability) the arrays are equal
__global__ void k_sum(const uint64_t* k, uint64_t n, unsigned long long* out) {
    unsigned long long acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x)
        acc += k[i] * (2 * i + 1);
    atomicAdd(out, acc);
}

static hipEvent_t e0, e1;
template <typename F>
float bench(F f) {
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

int main() {
    const uint64_t n = 1ull << 30;
    const uint64_t ntiles = n / 8192, chunk = 256, nchunks = (ntiles + chunk - 1) / chunk;
    uint64_t *kin, *kout;
    unsigned long long *xhist, *xstart, *thist, *bits, *sum, *joint;
    uint32_t *tcount, *csum, *err, *cnt;
    int32_t* gate;
    CK(hipMalloc(&kin, n * 8));
    CK(hipMalloc(&kout, n * 8));
    CK(hipMalloc(&xhist, 512 * 8));
    CK(hipMalloc(&xstart, 512 * 8));
    CK(hipMalloc(&thist, 512 * 8));
    CK(hipMalloc(&joint, 8 * 512 * 8));
    CK(hipMemset(joint, 0, 8 * 512 * 8));
    CK(hipMalloc(&bits, 256));
    CK(hipMalloc(&sum, 8));
    CK(hipMalloc(&tcount, ntiles * 512 * 4));
    CK(hipMalloc(&csum, nchunks * 512 * 4));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&cnt, 256));
    CK(hipMalloc(&gate, 4));
    const int32_t shift = 46;
    CK(hipMemcpy(gate, &shift, 4, hipMemcpyHostToDevice));
    CK(hipMemset(err, 0, 64));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill_rand, dim3(n / 256), dim3(256), 0, 0, kin, n);
    using X = ordered_bits<uint64_t, false>;
    CK(hipMemset(xhist, 0, 512 * 8));
    CK(hipMemset(thist, 0, 512 * 8));
    CK(hipMemset(bits, 0, 8));
    CK(hipMemset(bits + 1, 0xff, 8));
    hipLaunchKernelGGL((k_hist_tiles<uint64_t, X, 8192, kXBins>), dim3(512), dim3(kXBins), 0, 0, kin, n, ntiles,
                       X{}, 46, 55, tcount, xhist, thist, bits, joint);
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, xhist, xstart);
    hipLaunchKernelGGL(k_chunk_sums, dim3(nchunks), dim3(kXBins), 0, 0, tcount, ntiles, uint32_t(chunk), csum, gate);
    hipLaunchKernelGGL(k_tile_chunk_scan, dim3(1), dim3(kXBins), 0, 0, csum, nchunks, xstart, gate);
    hipLaunchKernelGGL(k_tile_offsets, dim3(nchunks), dim3(kXBins), 0, 0, tcount, ntiles, uint32_t(chunk), csum, gate);
    CK(hipDeviceSynchronize());
    auto checksum = [&] {
        CK(hipMemset(sum, 0, 8));
        hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, kout, n, sum);
        unsigned long long h;
        CK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
        return h;
    };
    auto counter = [&](auto flag, auto xreg) {
        constexpr bool DYN = decltype(flag)::value;
        constexpr bool XR = decltype(xreg)::value;
        return bench([&] {
            CK(hipMemsetAsync(cnt, 0, 256));
            hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, 16, -1, 9, true, DYN, false,
                                           false, XR>),
                               dim3(ntiles), dim3(512), 0, 0, kin, kout, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                               n, 46, xstart, (uint32_t*)nullptr, cnt, err, X{}, (const int32_t*)nullptr, ntiles,
                               (const uint32_t*)tcount);
        });
    };
    // pass 1 (shipped: XREG) into kout
    (void)counter(std::false_type{}, std::true_type{});
    CK(hipDeviceSynchronize());
    // pass 2: regions and their bin starts
    unsigned long long *thstart, *bs2, *sum2;
    seg_table* segs2;
    uint64_t* kfin;
    void* lb2;
    CK(hipMalloc(&thstart, 512 * 8));
    CK(hipMalloc(&bs2, 8 * 512 * 8));
    CK(hipMalloc(&segs2, sizeof(seg_table)));
    CK(hipMalloc(&kfin, n * 8));
    CK(hipMalloc(&sum2, 8));
    const uint64_t nt2 = ntiles + 8;
    CK(hipMalloc(&lb2, 256 + nt2 * 512 * 4));
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, thist, thstart);
    hipLaunchKernelGGL(k_region_plan, dim3(1), dim3(kXBins), 0, 0, xstart, thstart, joint, n, 8192, segs2, bs2);
    CK(hipDeviceSynchronize());
    uint32_t* cnt2 = static_cast<uint32_t*>(lb2);
    uint32_t* lbg2 = reinterpret_cast<uint32_t*>(static_cast<char*>(lb2) + 256);
    auto check2 = [&] {
        CK(hipMemset(sum2, 0, 8));
        hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, kfin, n, sum2);
        unsigned long long h;
        CK(hipMemcpy(&h, sum2, 8, hipMemcpyDeviceToHost));
        return h;
    };
#define PASS2(LBB)                                                                                              \
    bench([&] {                                                                                                 \
        CK(hipMemsetAsync(lb2, 0, 256 + nt2 * 512 * 4));                                                        \
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, 16, LBB, 9, true, false, false, \
                                       true, true>),                                                            \
                           dim3(nt2), dim3(512), 0, 0, kout, kfin, (const uint32_t*)nullptr, (uint32_t*)nullptr, n, \
                           55, bs2, lbg2, cnt2, err, X{}, (const int32_t*)nullptr, nt2, (const uint32_t*)nullptr,  \
                           segs2);                                                                              \
    })
    for (int rep = 0; rep < 2; ++rep) {
        const float a = PASS2(4);
        const unsigned long long c4 = check2();
        const float b = PASS2(2);
        const unsigned long long c2 = check2();
        const float c = PASS2(8);
        const unsigned long long c8 = check2();
        const float d = PASS2(1);
        const unsigned long long c1 = check2();
        printf("rep %d  top-9 pass, XCD regions: LBB4 %.3f  LBB2 %.3f  LBB8 %.3f  LBB1 %.3f ms  (LBB4 %.0f GB/s)  same: %s\n",
               rep, a, b, c, d, 16.0 * n / a / 1e6, (c4 == c2 && c4 == c8 && c4 == c1) ? "yes" : "NO");
        fflush(stdout);
    }
    uint32_t herr;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("deverr %u\n", herr);
    return 0;
}
