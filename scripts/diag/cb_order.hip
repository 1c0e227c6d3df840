// Diagnostic: ordering of hipLaunchHostFunc callbacks, pageable H2D copies and
// stream-ordered allocations relative to kernels on one stream.
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void spin_then_write(int* out, int n, long long cycles, int val) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = val;
}
__global__ void read_shape(const int* shape, int* out, int n, int base) {
    int i = threadIdx.x;
    if (i < n) { int s = shape[i]; if (s - base >= 0 && s - base < n) out[s - base] = s + 7; }
}
std::atomic<int> fired{0};
void cb(void* p) { fired.store(1); }

int main() {
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int* out; CK(hipMalloc(&out, 4096));
    // (a) callback after a ~100 ms kernel: poll the flag, then D2H on s2
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(out, 0xff, 4096, s2)); CK(hipStreamSynchronize(s2));
        fired = 0;
        hipLaunchKernelGGL(spin_then_write, dim3(1), dim3(256), 0, s1, out, 107, 200000000LL, 42 + rep);
        CK(hipLaunchHostFunc(s1, cb, nullptr));
        while (!fired.load()) {}
        std::vector<int> h(107);
        CK(hipMemcpyAsync(h.data(), out, 107 * 4, hipMemcpyDeviceToHost, s2)); CK(hipStreamSynchronize(s2));
        int bad = 0; for (int v : h) bad += (v != 42 + rep);
        printf("(a) rep %d: callback-then-D2H-other-stream: %d of 107 stale\n", rep, bad);
    }
    // (b) malloc_async + pageable H2D + kernel reading it
    for (int rep = 0; rep < 200; ++rep) {
        CK(hipMemsetAsync(out, 0xff, 4096, s2)); CK(hipStreamSynchronize(s2));
        hipStream_t s = (rep & 1) ? s1 : s2;
        auto* host = new std::vector<int>(107);
        for (int i = 0; i < 107; ++i) (*host)[i] = 1000 * rep + i;
        int* dev; CK(hipMallocAsync((void**)&dev, 107 * 4, s));
        CK(hipMemcpyAsync(dev, host->data(), 107 * 4, hipMemcpyHostToDevice, s));
        CK(hipLaunchHostFunc(s, [](void* p) { delete static_cast<std::vector<int>*>(p); }, host));
        hipLaunchKernelGGL(read_shape, dim3(1), dim3(128), 0, s, dev, out, 107, 1000 * rep);
        CK(hipFreeAsync(dev, s));
        fired = 0;
        CK(hipLaunchHostFunc(s, cb, nullptr));
        while (!fired.load()) {}
        std::vector<int> h(107);
        CK(hipMemcpyAsync(h.data(), out, 107 * 4, hipMemcpyDeviceToHost, s2)); CK(hipStreamSynchronize(s2));
        int bad = 0; for (int i = 0; i < 107; ++i) bad += (h[i] != 1000 * rep + i + 7);
        if (bad || rep < 3) printf("(b) rep %d: %d of 107 wrong\n", rep, bad);
    }
    // (c) same with hipStreamSynchronize instead of the callback
    int tot = 0;
    for (int rep = 0; rep < 200; ++rep) {
        CK(hipMemsetAsync(out, 0xff, 4096, s2)); CK(hipStreamSynchronize(s2));
        auto* host = new std::vector<int>(107);
        for (int i = 0; i < 107; ++i) (*host)[i] = 1000 * rep + i;
        int* dev; CK(hipMallocAsync((void**)&dev, 107 * 4, s1));
        CK(hipMemcpyAsync(dev, host->data(), 107 * 4, hipMemcpyHostToDevice, s1));
        CK(hipLaunchHostFunc(s1, [](void* p) { delete static_cast<std::vector<int>*>(p); }, host));
        hipLaunchKernelGGL(read_shape, dim3(1), dim3(128), 0, s1, dev, out, 107, 1000 * rep);
        CK(hipFreeAsync(dev, s1));
        CK(hipStreamSynchronize(s1));
        std::vector<int> h(107);
        CK(hipMemcpy(h.data(), out, 107 * 4, hipMemcpyDeviceToHost));
        for (int i = 0; i < 107; ++i) tot += (h[i] != 1000 * rep + i + 7);
    }
    printf("(c) stream-sync variant: %d wrong in total\n", tot);
    // (d) pinned staging instead of pageable, callback completion
    int* pinned; CK(hipHostMalloc((void**)&pinned, 107 * 4, 0));
    tot = 0;
    for (int rep = 0; rep < 200; ++rep) {
        CK(hipMemsetAsync(out, 0xff, 4096, s2)); CK(hipStreamSynchronize(s2));
        for (int i = 0; i < 107; ++i) pinned[i] = 1000 * rep + i;
        int* dev; CK(hipMallocAsync((void**)&dev, 107 * 4, s1));
        CK(hipMemcpyAsync(dev, pinned, 107 * 4, hipMemcpyHostToDevice, s1));
        hipLaunchKernelGGL(read_shape, dim3(1), dim3(128), 0, s1, dev, out, 107, 1000 * rep);
        CK(hipFreeAsync(dev, s1));
        fired = 0;
        CK(hipLaunchHostFunc(s1, cb, nullptr));
        while (!fired.load()) {}
        std::vector<int> h(107);
        CK(hipMemcpyAsync(h.data(), out, 107 * 4, hipMemcpyDeviceToHost, s2)); CK(hipStreamSynchronize(s2));
        for (int i = 0; i < 107; ++i) tot += (h[i] != 1000 * rep + i + 7);
    }
    printf("(d) pinned + callback variant: %d wrong in total\n", tot);
    return 0;
}
