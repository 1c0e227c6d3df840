// Microbenchmark (round 6): both prefix passes of the 18-bit sort at 2^30
// random u64 keys with 8192-key tiles (512 x 16, shipped: two workgroups per
// CU by LDS) against 4096-key tiles (512 x 8: ~45 KiB of LDS, three per CU),
// and the second pass's look-back width (LBB 1 / 4).  Pass 1 = offset-fed
// (k_hist_tiles counts, XCD regions), pass 2 = look-back over 8 field regions
// (XREG + SEG).  Output checksums compared across shapes; best of 7 (HIP events).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include sortpass7.hip -o sortpass7
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
__global__ void k_sum(const uint64_t* k, uint64_t n, unsigned long long* out) {
    unsigned long long acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) acc += k[i] * (2 * i + 1);
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

using X = ordered_bits<uint64_t, false>;
constexpr uint64_t n = 1ull << 30;
uint64_t *kin, *kmid, *kfin;
unsigned long long* sum;

unsigned long long checksum(const uint64_t* k) {
    CK(hipMemset(sum, 0, 8));
    hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, k, n, sum);
    unsigned long long h;
    CK(hipMemcpy(&h, sum, 8, hipMemcpyDeviceToHost));
    return h;
}

template <int ITEMS>
void run() {
    constexpr int TILE = 512 * ITEMS;
    const uint64_t ntiles = n / TILE, chunk = 256, nchunks = (ntiles + chunk - 1) / chunk;
    unsigned long long *xhist, *xstart, *thist, *thstart, *bits, *joint, *bs2;
    uint32_t *tcount, *csum, *err, *cnt;
    int32_t* gate;
    seg_table* segs2;
    void* lb2;
    CK(hipMalloc(&xhist, 512 * 8));
    CK(hipMalloc(&xstart, 512 * 8));
    CK(hipMalloc(&thist, 512 * 8));
    CK(hipMalloc(&thstart, 512 * 8));
    CK(hipMalloc(&joint, 8 * 512 * 8));
    CK(hipMalloc(&bs2, 8 * 512 * 8));
    CK(hipMalloc(&bits, 256));
    CK(hipMalloc(&tcount, ntiles * 512 * 4));
    CK(hipMalloc(&csum, nchunks * 512 * 4));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&cnt, 256));
    CK(hipMalloc(&gate, 4));
    CK(hipMalloc(&segs2, sizeof(seg_table)));
    const uint64_t nt2 = ntiles + 8;
    CK(hipMalloc(&lb2, 256 + nt2 * 512 * 4));
    const int32_t shift = 46;
    CK(hipMemcpy(gate, &shift, 4, hipMemcpyHostToDevice));
    CK(hipMemset(err, 0, 64));
    CK(hipMemset(joint, 0, 8 * 512 * 8));
    CK(hipMemset(xhist, 0, 512 * 8));
    CK(hipMemset(thist, 0, 512 * 8));
    CK(hipMemset(bits, 0, 8));
    CK(hipMemset(bits + 1, 0xff, 8));
    const float th = bench([&] {
        hipLaunchKernelGGL((k_hist_tiles<uint64_t, X, TILE, kXBins>), dim3(512), dim3(kXBins), 0, 0, kin, n, ntiles,
                           X{}, 46, 55, tcount, xhist, thist, bits, joint);
    });
    // (the timed histogram runs 8 times: recount once)
    CK(hipMemset(joint, 0, 8 * 512 * 8));
    CK(hipMemset(xhist, 0, 512 * 8));
    CK(hipMemset(thist, 0, 512 * 8));
    hipLaunchKernelGGL((k_hist_tiles<uint64_t, X, TILE, kXBins>), dim3(512), dim3(kXBins), 0, 0, kin, n, ntiles, X{},
                       46, 55, tcount, xhist, thist, bits, joint);
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, xhist, xstart);
    hipLaunchKernelGGL(k_chunk_sums, dim3(nchunks), dim3(kXBins), 0, 0, tcount, ntiles, uint32_t(chunk), csum, gate);
    hipLaunchKernelGGL(k_tile_chunk_scan, dim3(1), dim3(kXBins), 0, 0, csum, nchunks, xstart, gate);
    hipLaunchKernelGGL(k_tile_offsets, dim3(nchunks), dim3(kXBins), 0, 0, tcount, ntiles, uint32_t(chunk), csum, gate);
    hipLaunchKernelGGL(k_bin_offsets<512>, dim3(1), dim3(512), 0, 0, thist, thstart);
    hipLaunchKernelGGL(k_region_plan, dim3(1), dim3(kXBins), 0, 0, xstart, thstart, joint, n, TILE, segs2, bs2);
    CK(hipDeviceSynchronize());
    const float t1 = bench([&] {
        CK(hipMemsetAsync(cnt, 0, 256));
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, ITEMS, -1, 9, true, false, false,
                                       false, true>),
                           dim3(ntiles), dim3(512), 0, 0, kin, kmid, (const uint32_t*)nullptr, (uint32_t*)nullptr, n,
                           46, xstart, (uint32_t*)nullptr, cnt, err, X{}, (const int32_t*)nullptr, ntiles,
                           (const uint32_t*)tcount);
    });
    const unsigned long long c1 = checksum(kmid);
    uint32_t* cnt2 = static_cast<uint32_t*>(lb2);
    uint32_t* lbg2 = reinterpret_cast<uint32_t*>(static_cast<char*>(lb2) + 256);
#define PASS2(LBB)                                                                                              \
    bench([&] {                                                                                                 \
        CK(hipMemsetAsync(lb2, 0, 256 + nt2 * 512 * 4));                                                        \
        hipLaunchKernelGGL((k_onesweep<uint64_t, uint32_t, false, uint32_t, X, 512, ITEMS, LBB, 9, true, false, false, \
                                       true, true>),                                                            \
                           dim3(nt2), dim3(512), 0, 0, kmid, kfin, (const uint32_t*)nullptr, (uint32_t*)nullptr, n, \
                           55, bs2, lbg2, cnt2, err, X{}, (const int32_t*)nullptr, nt2, (const uint32_t*)nullptr,  \
                           segs2);                                                                              \
    })
    const float t24 = PASS2(4);
    const unsigned long long c24 = checksum(kfin);
    const float t21 = PASS2(1);
    const unsigned long long c21 = checksum(kfin);
    uint32_t herr;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("tile %5d (512 x %2d): hist %.3f  pass1 %.3f  pass2 LBB4 %.3f  LBB1 %.3f ms | sums %016llx %016llx %s deverr %u\n",
           TILE, ITEMS, th, t1, t24, t21, c1, c24, c24 == c21 ? "lbb-same" : "LBB-DIFF", herr);
    fflush(stdout);
    CK(hipFree(xhist)); CK(hipFree(xstart)); CK(hipFree(thist)); CK(hipFree(thstart)); CK(hipFree(joint));
    CK(hipFree(bs2)); CK(hipFree(bits)); CK(hipFree(tcount)); CK(hipFree(csum)); CK(hipFree(err)); CK(hipFree(cnt));
    CK(hipFree(gate)); CK(hipFree(segs2)); CK(hipFree(lb2));
}

int main() {
    CK(hipMalloc(&kin, n * 8));
    CK(hipMalloc(&kmid, n * 8));
    CK(hipMalloc(&kfin, n * 8));
    CK(hipMalloc(&sum, 8));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_fill_rand, dim3(n / 256), dim3(256), 0, 0, kin, n);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        run<16>();
        run<8>();
        run<12>();
    }
    return 0;
}
