// runtime.hip -- targets, streams, completion callbacks, memory and the
// per-stream scratch cache of the C ABI.
//
// Reference behaviour mirrored:
//   * device enumeration / properties: src/compute/cuda/get_cuda_targets.cpp:30-65,
//     cuda_target.cpp:145-184 (processing_units = CU count here, not a
//     SMs x cores table);
//   * lazily created non-blocking stream per target: cuda_target.cpp:255-280
//     (the C++ layer creates it lazily; here the call creates one);
//   * completion -> future: cuda_target.cpp:97-142 used cudaStreamAddCallback;
//     here hipLaunchHostFunc, whose function must not call HIP;
//   * allocator: hpx/compute/cuda/allocator.hpp:108-160 (hipErrorOutOfMemory
//     is reported as HPXHIP_ERROR_OUT_OF_MEMORY so the C++ layer can throw
//     hpx::out_of_memory as allocator.hpp:118-124 does).
#include "internal.hpp"

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

using namespace hpxhip;

namespace {

std::mutex g_mutex;

struct scratch_entry {
    void* ptr = nullptr;
    size_t bytes = 0;
    int device = 0;
};
std::unordered_map<hipStream_t, scratch_entry> g_scratch;
std::unordered_map<int, uint32_t*> g_error_words;
std::unordered_map<int, device_info> g_infos;

int map_alloc_error(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return HPXHIP_ERROR_OUT_OF_MEMORY;
    return static_cast<int>(e);
}

struct callback_box {
    hpxhip_callback fn;
    void* user;
};

void host_trampoline(void* p) {
    callback_box* box = static_cast<callback_box*>(p);
    box->fn(box->user, 0);
    delete box;
}

}  // namespace

namespace hpxhip {

const device_info& current_device_info() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_mutex);
    auto it = g_infos.find(dev);
    if (it != g_infos.end()) return it->second;
    device_info info;
    info.device = dev;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
        info.cus = cus;
    return g_infos.emplace(dev, info).first->second;
}

int stream_device(hipStream_t s, int* device) {
    if (s == nullptr) return static_cast<int>(hipGetDevice(device));
    hipDevice_t d;
    hipError_t e = hipStreamGetDevice(s, &d);
    if (e != hipSuccess) return static_cast<int>(e);
    *device = static_cast<int>(d);
    return 0;
}

int scratch_get(hipStream_t s, size_t bytes, void** out) {
    std::lock_guard<std::mutex> lk(g_mutex);
    scratch_entry& e = g_scratch[s];
    if (e.bytes >= bytes && e.ptr) {
        *out = e.ptr;
        return 0;
    }
    if (e.ptr) {
        // Old buffer may still be in use by queued work on this stream.
        hipError_t se = hipStreamSynchronize(s);
        if (se != hipSuccess) return static_cast<int>(se);
        (void)hipFree(e.ptr);
        e.ptr = nullptr;
        e.bytes = 0;
    }
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 8;
    void* p = nullptr;
    hipError_t ae = hipMalloc(&p, want);
    if (ae != hipSuccess) {
        (void)hipGetLastError();
        ae = hipMalloc(&p, bytes);
        if (ae != hipSuccess) {
            (void)hipGetLastError();
            return map_alloc_error(ae);
        }
        want = bytes;
    }
    e.ptr = p;
    e.bytes = want;
    *out = p;
    return 0;
}

namespace {
struct roctx_api {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
};
const roctx_api& roctx() {
    static const roctx_api api = [] {
        roctx_api a;
        const char* e = std::getenv("HPXHIP_ROCTX");
        if (!e || e[0] != '1') return a;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        a.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (!a.push || !a.pop) a = roctx_api{};
        return a;
    }();
    return api;
}
}  // namespace

bool roctx_enabled() { return roctx().push != nullptr; }
void roctx_push(const char* name) { roctx().push(name); }
void roctx_pop() { roctx().pop(); }

uint32_t* device_error_word(hipStream_t s) {
    int dev = 0;
    if (stream_device(s, &dev) != 0) dev = 0;
    std::lock_guard<std::mutex> lk(g_mutex);
    auto it = g_error_words.find(dev);
    if (it != g_error_words.end()) return it->second;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
    uint32_t* w = nullptr;
    if (hipMalloc(&w, 64) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipSetDevice(prev);
        return nullptr;
    }
    (void)hipMemset(w, 0, 64);
    (void)hipSetDevice(prev);
    g_error_words[dev] = w;
    return w;
}

}  // namespace hpxhip

// ---------------------------------------------------------------------------
namespace {
template <typename T, typename Op>
__global__ void k_fold(T init, const T* __restrict__ v, uint64_t count, T* __restrict__ out, Op op) {
    // Segment-order left fold, one lane: count is the number of segments
    // (<= a few dozen); order is exactly init (op) v0 (op) v1 ...
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        T acc = init;
        for (uint64_t i = 0; i < count; ++i) acc = op(acc, v[i]);
        *out = acc;
    }
}
// The carries of a segmented scan (detail/scan.hpp:646-677): out[0] = init,
// out[j + 1] = out[j] (op) v[j] -- the same segment-order left fold as k_fold,
// every prefix kept.
template <typename T, typename Op>
__global__ void k_fold_exclusive(T init, const T* __restrict__ v, uint64_t count, T* __restrict__ out, Op op) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        T acc = init;
        out[0] = acc;
        for (uint64_t i = 0; i < count; ++i) out[i + 1] = acc = op(acc, v[i]);
    }
}
}  // namespace

extern "C" {

int hpxhip_abi_version(void) { return HPXHIP_ABI_VERSION; }

const char* hpxhip_error_string(int status) {
    switch (status) {
        case HPXHIP_SUCCESS: return "success";
        case HPXHIP_ERROR_INVALID_ARGUMENT: return "hpxhip: invalid argument";
        case HPXHIP_ERROR_UNSUPPORTED: return "hpxhip: dtype/operator combination not supported";
        case HPXHIP_ERROR_DEVICE_TIMEOUT: return "hpxhip: kernel gave up a bounded spin (device timeout)";
        case HPXHIP_ERROR_OUT_OF_MEMORY: return "hpxhip: out of device memory";
        case HPXHIP_ERROR_NOT_READY: return "hpxhip: not ready";
        default: return hipGetErrorString(static_cast<hipError_t>(status));
    }
}

int hpxhip_device_error(int device, uint32_t* code) {
    if (!code) return HPXHIP_ERROR_INVALID_ARGUMENT;
    *code = 0;
    uint32_t* w = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mutex);
        auto it = g_error_words.find(device);
        if (it != g_error_words.end()) w = it->second;
    }
    if (!w) return 0;
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    HPXHIP_CHECK(hipDeviceSynchronize());
    uint32_t v = 0;
    HPXHIP_CHECK(hipMemcpy(&v, w, sizeof(v), hipMemcpyDeviceToHost));
    HPXHIP_CHECK(hipMemset(w, 0, sizeof(uint32_t)));
    HPXHIP_CHECK(hipSetDevice(prev));
    *code = v;
    return 0;
}

extern "C++" {
namespace hpxhip {
thread_local int g_inject_status = 0;
thread_local int g_inject_count = 0;
thread_local int g_event_inject_status = 0;
thread_local int g_event_inject_count = 0;
}  // namespace hpxhip
}

int hpxhip_debug_inject_event_error(int status, int count) {
    if (count < 0 || (count > 0 && (status == HPXHIP_SUCCESS || status == HPXHIP_ERROR_NOT_READY)))
        return HPXHIP_ERROR_INVALID_ARGUMENT;
    hpxhip::g_event_inject_status = status;
    hpxhip::g_event_inject_count = count;
    return 0;
}
int hpxhip_debug_inject_error(int status, int count) {
    if (count < 0 || (count > 0 && status == HPXHIP_SUCCESS)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hpxhip::g_inject_status = status;
    hpxhip::g_inject_count = count;
    return 0;
}

int hpxhip_debug_raise_device_error(hpxhip_stream stream, uint32_t code) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t* w = hpxhip::device_error_word(s);
    if (!w) return HPXHIP_ERROR_OUT_OF_MEMORY;
    HPXHIP_CHECK(hipMemsetD32Async(w, code, 1, s));
    return 0;
}

// ------------------------------------------------------------- devices
int hpxhip_get_device_count(int* count) {
    if (!count) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipError_t e = hipGetDeviceCount(count);
    if (e == hipErrorNoDevice) {
        (void)hipGetLastError();
        *count = 0;
        return 0;
    }
    return static_cast<int>(e);
}
int hpxhip_set_device(int device) { return static_cast<int>(hipSetDevice(device)); }
int hpxhip_get_device(int* device) { return static_cast<int>(hipGetDevice(device)); }

int hpxhip_device_props_get(int device, hpxhip_device_props* props) {
    if (!props) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipDeviceProp_t p;
    HPXHIP_CHECK(hipGetDeviceProperties(&p, device));
    std::memset(props, 0, sizeof(*props));
    std::snprintf(props->name, sizeof(props->name), "%s", p.name);
    std::snprintf(props->arch, sizeof(props->arch), "%s", p.gcnArchName);
    props->compute_units = p.multiProcessorCount;
    props->wave_size = p.warpSize;
    props->max_threads_per_block = p.maxThreadsPerBlock;
    props->clock_khz = p.clockRate;
    props->memory_clock_khz = p.memoryClockRate;
    props->memory_bus_width = p.memoryBusWidth;
    props->total_global_mem = p.totalGlobalMem;
    props->lds_per_block = p.sharedMemPerBlock;
    props->pci_bus_id = p.pciBusID;
    props->pci_device_id = p.pciDeviceID;
    return 0;
}

int hpxhip_device_synchronize(int device) {
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    hipError_t e = hipDeviceSynchronize();
    (void)hipSetDevice(prev);
    return static_cast<int>(e);
}

int hpxhip_enable_peer_access(int device, int peer) {
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        e = hipSuccess;
    }
    (void)hipSetDevice(prev);
    return static_cast<int>(e);
}

int hpxhip_can_access_peer(int device, int peer, int* can) {
    if (!can) return HPXHIP_ERROR_INVALID_ARGUMENT;
    return static_cast<int>(hipDeviceCanAccessPeer(can, device, peer));
}

// ------------------------------------------------------------- streams
int hpxhip_stream_create(int device, hpxhip_stream* stream) {
    if (!stream) return HPXHIP_ERROR_INVALID_ARGUMENT;
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return static_cast<int>(e);
    *stream = reinterpret_cast<hpxhip_stream>(s);
    return 0;
}

int hpxhip_stream_destroy(hpxhip_stream stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    {
        std::lock_guard<std::mutex> lk(g_mutex);
        auto it = g_scratch.find(s);
        if (it != g_scratch.end()) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(it->second.ptr);
            g_scratch.erase(it);
        }
    }
    return static_cast<int>(hipStreamDestroy(s));
}

int hpxhip_stream_synchronize(hpxhip_stream stream) {
    return static_cast<int>(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
}

int hpxhip_stream_query(hpxhip_stream stream) {
    hipError_t e = hipStreamQuery(reinterpret_cast<hipStream_t>(stream));
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return HPXHIP_ERROR_NOT_READY;
    }
    return static_cast<int>(e);
}

int hpxhip_stream_add_callback(hpxhip_stream stream, hpxhip_callback fn, void* user) {
    if (!fn) return HPXHIP_ERROR_INVALID_ARGUMENT;
    callback_box* box = new callback_box{fn, user};
    hipError_t e = hipLaunchHostFunc(reinterpret_cast<hipStream_t>(stream), host_trampoline, box);
    if (e != hipSuccess) {
        delete box;
        return static_cast<int>(e);
    }
    return 0;
}

int hpxhip_event_create(hpxhip_event* event) {
    if (!event) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipEvent_t e = nullptr;
    HPXHIP_CHECK(hipEventCreate(&e));
    *event = reinterpret_cast<hpxhip_event>(e);
    return 0;
}
// An event created with `device` current and, unless `timing`, without
// timestamps (an ordering or completion event: hipEventDisableTiming).  A
// HIP event is recorded on streams of the device it was created on; this is
// what lets one process order work across its GPUs without a host wait.
int hpxhip_event_create_on(int device, int timing, hpxhip_event* event) {
    if (!event) return HPXHIP_ERROR_INVALID_ARGUMENT;
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    if (prev != device) HPXHIP_CHECK(hipSetDevice(device));
    hipEvent_t e = nullptr;
    const hipError_t rc = hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming);
    if (prev != device) (void)hipSetDevice(prev);
    if (rc != hipSuccess) {
        (void)hipGetLastError();
        return static_cast<int>(rc);
    }
    *event = reinterpret_cast<hpxhip_event>(e);
    return 0;
}
int hpxhip_stream_device(hpxhip_stream stream, int* device) {
    if (!device) return HPXHIP_ERROR_INVALID_ARGUMENT;
    return stream_device(reinterpret_cast<hipStream_t>(stream), device);
}
int hpxhip_event_destroy(hpxhip_event event) {
    return static_cast<int>(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
}
int hpxhip_event_record(hpxhip_event event, hpxhip_stream stream) {
    const hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(event), reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) (void)hipGetLastError();  // returned, not left for the next launch's check
    return static_cast<int>(e);
}
// The event calls return their status and clear HIP's last error, so a
// failure the caller handles (a completion falling back to its callback) is
// not reported again by the next launch's hipGetLastError().
int hpxhip_event_synchronize(hpxhip_event event) {
    if (hpxhip::g_event_inject_count > 0) {
        --hpxhip::g_event_inject_count;
        return hpxhip::g_event_inject_status;
    }
    hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(event));
    if (e != hipSuccess) (void)hipGetLastError();
    return static_cast<int>(e);
}
int hpxhip_event_query(hpxhip_event event) {
    if (hpxhip::g_event_inject_count > 0) {
        --hpxhip::g_event_inject_count;
        return hpxhip::g_event_inject_status;
    }
    hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(event));
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return HPXHIP_ERROR_NOT_READY;
    }
    if (e != hipSuccess) (void)hipGetLastError();
    return static_cast<int>(e);
}
int hpxhip_event_elapsed_ms(hpxhip_event start, hpxhip_event stop, float* ms) {
    if (!ms) return HPXHIP_ERROR_INVALID_ARGUMENT;
    return static_cast<int>(
        hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
}
int hpxhip_stream_wait_event(hpxhip_stream stream, hpxhip_event event) {
    return static_cast<int>(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream),
                                               reinterpret_cast<hipEvent_t>(event), 0));
}

// -------------------------------------------------------------- memory
int hpxhip_malloc(int device, void** ptr, size_t bytes) {
    if (!ptr) return HPXHIP_ERROR_INVALID_ARGUMENT;
    *ptr = nullptr;
    if (bytes == 0) return 0;
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    hipError_t e = hipMalloc(ptr, bytes);
    if (e != hipSuccess) (void)hipGetLastError();
    (void)hipSetDevice(prev);
    return e == hipSuccess ? 0 : map_alloc_error(e);
}
int hpxhip_free(void* ptr) { return ptr ? static_cast<int>(hipFree(ptr)) : 0; }
int hpxhip_malloc_host(void** ptr, size_t bytes) {
    if (!ptr) return HPXHIP_ERROR_INVALID_ARGUMENT;
    *ptr = nullptr;
    if (bytes == 0) return 0;
    hipError_t e = hipHostMalloc(ptr, bytes, hipHostMallocDefault);
    if (e != hipSuccess) (void)hipGetLastError();
    return e == hipSuccess ? 0 : map_alloc_error(e);
}
int hpxhip_free_host(void* ptr) { return ptr ? static_cast<int>(hipHostFree(ptr)) : 0; }
int hpxhip_mem_info(int device, size_t* free_bytes, size_t* total_bytes) {
    int prev = 0;
    HPXHIP_CHECK(hipGetDevice(&prev));
    HPXHIP_CHECK(hipSetDevice(device));
    hipError_t e = hipMemGetInfo(free_bytes, total_bytes);
    (void)hipSetDevice(prev);
    return static_cast<int>(e);
}
int hpxhip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, hpxhip_stream stream) {
    if (bytes == 0) return 0;
    hipMemcpyKind k;
    switch (kind) {
        case HPXHIP_H2H: k = hipMemcpyHostToHost; break;
        case HPXHIP_H2D: k = hipMemcpyHostToDevice; break;
        case HPXHIP_D2H: k = hipMemcpyDeviceToHost; break;
        case HPXHIP_D2D: k = hipMemcpyDeviceToDevice; break;
        default: k = hipMemcpyDefault; break;
    }
    return static_cast<int>(hipMemcpyAsync(dst, src, bytes, k, reinterpret_cast<hipStream_t>(stream)));
}
int hpxhip_memcpy_peer_async(void* dst, int dst_device, const void* src, int src_device, size_t bytes,
                             hpxhip_stream stream) {
    if (bytes == 0) return 0;
    return static_cast<int>(hipMemcpyPeerAsync(dst, dst_device, src, src_device, bytes,
                                               reinterpret_cast<hipStream_t>(stream)));
}
int hpxhip_memset_async(void* dst, int value, size_t bytes, hpxhip_stream stream) {
    if (bytes == 0) return 0;
    return static_cast<int>(hipMemsetAsync(dst, value, bytes, reinterpret_cast<hipStream_t>(stream)));
}

int hpxhip_stream_scratch(hpxhip_stream stream, size_t bytes, void** ptr) {
    if (!ptr) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return scratch_get(s, bytes ? bytes : 1, ptr);
}

int hpxhip_device_error_word(hpxhip_stream stream, uint32_t** word) {
    if (!word) return HPXHIP_ERROR_INVALID_ARGUMENT;
    *word = device_error_word(reinterpret_cast<hipStream_t>(stream));
    return *word ? 0 : HPXHIP_ERROR_OUT_OF_MEMORY;
}

int hpxhip_scratch_bytes(int algo, int dtype, int aux_dtype, uint64_t n, size_t* bytes) {
    if (!bytes) return HPXHIP_ERROR_INVALID_ARGUMENT;
    if (dtype_size(dtype) == 0) return HPXHIP_ERROR_INVALID_ARGUMENT;
    switch (algo) {
        case HPXHIP_ALGO_REDUCE: *bytes = reduce_scratch_bytes(n); return 0;
        case HPXHIP_ALGO_SCAN: *bytes = scan_scratch_bytes(dtype, n); return 0;
        case HPXHIP_ALGO_COPY_IF: *bytes = copy_if_scratch_bytes(dtype, n); return 0;
        case HPXHIP_ALGO_SORT: *bytes = sort_scratch_bytes(dtype, -1, n); return 0;
        case HPXHIP_ALGO_MERGE: *bytes = merge_scratch_bytes(n); return 0;
        case HPXHIP_ALGO_MERGE_RUNS: *bytes = merge_runs_scratch_bytes(n); return 0;
        case HPXHIP_ALGO_SORT_BY_KEY:
            if (dtype_size(aux_dtype) == 0) return HPXHIP_ERROR_INVALID_ARGUMENT;
            *bytes = sort_scratch_bytes(dtype, aux_dtype, n);
            return 0;
        default: return HPXHIP_ERROR_INVALID_ARGUMENT;
    }
}

int hpxhip_fold(int dtype, int op, const void* init, const void* values_dev, uint64_t count,
                void* out_dev, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_fold");
    if (!init || !out_dev || (count && !values_dev)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return with_binop<T>(op, [&](auto o) -> int {
            T iv;
            std::memcpy(&iv, init, sizeof(T));
            hipLaunchKernelGGL((k_fold<T, decltype(o)>), dim3(1), dim3(64), 0, s, iv,
                               static_cast<const T*>(values_dev), count, static_cast<T*>(out_dev), o);
            HPXHIP_CHECK_LAUNCH();
            return 0;
        });
    });
}

int hpxhip_fold_exclusive(int dtype, int op, const void* init, const void* values_dev, uint64_t count,
                          void* out_dev, hpxhip_stream stream) {
    HPXHIP_ANNOTATE("hpxhip_fold_exclusive");
    if (!init || !out_dev || (count && !values_dev)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return with_binop<T>(op, [&](auto o) -> int {
            T iv;
            std::memcpy(&iv, init, sizeof(T));
            hipLaunchKernelGGL((k_fold_exclusive<T, decltype(o)>), dim3(1), dim3(64), 0, s, iv,
                               static_cast<const T*>(values_dev), count, static_cast<T*>(out_dev), o);
            HPXHIP_CHECK_LAUNCH();
            return 0;
        });
    });
}

}  // extern "C"
