// scan.hip -- inclusive_scan / exclusive_scan / transform_{in,ex}clusive_scan.
//
// Reference: inclusive_scan.hpp:90-173 and exclusive_scan.hpp:100-175 run
// scan_partitioner.hpp:62-156 on the host -- three phases, the data read
// once and written twice plus a re-read (section 3.3 of SURVEY.md).  Here:
// one pass, 16 B/element of HBM traffic (read once, write once).
//
// Tile = 1024 threads x 16 vectors of 16 B (32768 int64 / 65536 int32 =
// 256 KiB, scan_kernel.hpp).  Each wave owns a contiguous sixteenth of the
// tile and walks it in 16 rounds of 64 lanes x 16 B (coalesced 1 KiB per
// instruction):
//   round r:  lane-serial scan of its V elements -> DPP wave scan of lane
//             totals -> running wave carry (readlane 63);
//   then      wave totals through LDS -> tile aggregate -> decoupled look-back
//             by wave 0 (lookback.hpp) -> every element op'd with the tile
//             prefix and stored with 16-B stores.
// Integer results are exact; FP results follow a tree order that can differ
// from the sequential left fold (tolerance in DESIGN.md).
#include "internal.hpp"
#include <hpxhip/kernels/lookback.hpp>
#include <hpxhip/kernels/scan_kernel.hpp>

using namespace hpxhip;

namespace {

using namespace hpxhip::scan_detail;

// Scratch: [counter | tile slots], zeroed per call.  Sized for the variant
// with the smallest tiles (8 rounds), so one size serves every launch.
constexpr size_t kSlotsOff = 256;

template <typename T, int ROUNDS, int THREADS = kThreads>
uint64_t ntiles_for(uint64_t n) {
    return (n + tile_elems<T, ROUNDS, THREADS>() - 1) / tile_elems<T, ROUNDS, THREADS>();
}

// Workgroup size per variant (r03): aligned 8-byte scans run 512-thread
// tiles of 16 rounds (128 KiB), two workgroups per CU -- with the fixed
// look-back one workgroup's loads and stores now overlap the other's scan:
// 2^30 int64 2.635-2.638 -> 2.580-2.581 ms, f64 2.607-2.612 -> 2.591-2.592
// (profiles/r03_ubench_scan7_shapes.log; with the variable-window look-back
// the same shape had been slower, r02_ubench_scan_shapes_blockidx.log).
// The tile has as many elements as a 1024 x 8 one, so the scratch sizing
// below covers it; float (12 rounds) and the element-wise path keep 1024.
template <typename T, bool ALIGNED>
constexpr int threads_for() {
    return (ALIGNED && (std::is_integral_v<T> || sizeof(T) == 8) && rounds_for<T, ALIGNED>() == 16) ? 512 : kThreads;
}

// [counter | tile slots | head carry]: the carry of a split-off head
// (misaligned ranges) sits past the region the per-call memset clears.
template <typename T>
size_t carry_off(uint64_t n) {
    return align_up(kSlotsOff + ntiles_for<T, 8>(n) * tile_state<T>::bytes_per_tile(), 256);
}
template <typename T>
size_t scratch_total(uint64_t n) {
    return carry_off<T>(n) + 256;
}

// SHIFTED (ALIGNED only): the output is 16-B aligned and the input is not
// (scan_kernel.hpp)
template <typename T, bool INCL, bool ALIGNED, bool SHIFTED = false, typename Conv, typename Op>
int launch_scan(const T* in, T* out, uint64_t n, Conv conv, Op op, T init, const T* prefix_dev, char* ws,
                hipStream_t s) {
    static_assert(ALIGNED || !SHIFTED, "a shifted input needs the vector kernel");
    // SHIFTED keeps the aligned shape (512 x 16 for 8-byte values, 4-10
    // spilled VGPRs): 2^30 int64 in+1/out+0 2.56 ms, in+0/out+3 2.61, against
    // 2.76 / 2.86 with 1024 x 8-round tiles (profiles/r04_unaligned_probe.log)
    constexpr int R = rounds_for<T, ALIGNED>();
    constexpr int TH = threads_for<T, ALIGNED>();
    static_assert(tile_elems<T, R, TH>() >= tile_elems<T, 8>(), "scratch is sized for 1024 x 8-round tiles");
    const uint64_t ntiles = ntiles_for<T, R, TH>(n);
    HPXHIP_CHECK(hipMemsetAsync(ws, 0, align_up(kSlotsOff + ntiles * tile_state<T>::bytes_per_tile(), 256), s));
    scan_detail::scan_state<T> st{reinterpret_cast<uint64_t*>(ws + kSlotsOff), device_error_word(s)};
    hipLaunchKernelGGL((k_scan<T, Conv, Op, INCL, ALIGNED, R, TH, true, TH == kThreads ? 1 : 4, false, 1,
                               HPXHIP_TILE_DYN_ID, true, T, std::is_floating_point_v<T> && sizeof(T) == 8, true,
                               SHIFTED>),
                       dim3(static_cast<unsigned>(ntiles)), dim3(TH), 0, s, in, out, n, conv, op, init, prefix_dev,
                       reinterpret_cast<uint32_t*>(ws), st);
    HPXHIP_CHECK_LAUNCH();
    return 0;
}

// Head of a range whose input and output share a misalignment: scanned by one
// thread (left fold from the init / device prefix), its carry left in
// *carry for the vector kernel over the rest.
template <typename T, bool INCL, typename Conv, typename Op>
__global__ void k_scan_head(const T* in, T* out, uint64_t h, Conv conv, Op op, T init, const T* prefix_dev,
                            T* carry) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    T acc = prefix_dev ? *prefix_dev : init;
    for (uint64_t i = 0; i < h; ++i) {
        const T x = conv(in[i]);
        if (INCL) {
            acc = op(acc, x);
            out[i] = acc;
        } else {
            out[i] = acc;
            acc = op(acc, x);
        }
    }
    *carry = acc;
}

// Misaligned input and output: split off a head that brings the output to a
// 1-KiB boundary (whole-line stores for every wave) and scan the rest with
// the vector kernel seeded by the head's carry.  Same offset inside 16 B:
// int64 offset by one element 3.8 -> ~2.7 ms at 2^30
// (profiles/r02_unaligned_ranges.log).  Different offsets (r04): the input
// is read shifted across lanes (k_scan SHIFTED) instead of by the
// element-wise kernel.  Returns -1 when the split does not apply (the
// element-wise kernel takes the range).
template <typename T, bool INCL, typename Conv, typename Op>
int launch_scan_split(const T* in, T* out, uint64_t n, Conv conv, Op op, T init, const T* prefix_dev, char* ws,
                      hipStream_t s) {
    const uintptr_t ia = reinterpret_cast<uintptr_t>(in), oa = reinterpret_cast<uintptr_t>(out);
    if (ia % sizeof(T) != 0 || oa % sizeof(T) != 0) return -1;
    uint64_t h = head_to_align16(out, sizeof(T));
    const uintptr_t v = oa + h * sizeof(T);
    h += ((1024 - v % 1024) % 1024) / sizeof(T);
    if (n <= 4 * h + 1024) return -1;
    T* carry = reinterpret_cast<T*>(ws + carry_off<T>(n));
    hipLaunchKernelGGL((k_scan_head<T, INCL, Conv, Op>), dim3(1), dim3(64), 0, s, in, out, h, conv, op, init,
                       prefix_dev, carry);
    HPXHIP_CHECK_LAUNCH();
    if (ia % 16 == oa % 16) return launch_scan<T, INCL, true>(in + h, out + h, n - h, conv, op, init, carry, ws, s);
    return launch_scan<T, INCL, true, true>(in + h, out + h, n - h, conv, op, init, carry, ws, s);
}

template <typename T, typename F>
int with_scan_conv(int kind, const void* scalars, F&& f) {
    switch (kind) {
        case HPXHIP_U_IDENTITY:
        case HPXHIP_U_SCALE:
        case HPXHIP_U_SQUARE: break;
        default: return HPXHIP_ERROR_UNSUPPORTED;
    }
    return with_unary<T>(kind, scalars, [&](auto conv) -> int {
        using C = decltype(conv);
        if constexpr (std::is_same_v<C, unary_fn<HPXHIP_U_IDENTITY, T>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SCALE, T>> ||
                      std::is_same_v<C, unary_fn<HPXHIP_U_SQUARE, T>>)
            return f(conv);
        else
            return HPXHIP_ERROR_UNSUPPORTED;
    });
}

}  // namespace

namespace hpxhip {
size_t scan_scratch_bytes(int dtype, uint64_t n) {
    return dtype_size(dtype) == 8 ? scratch_total<uint64_t>(n) : scratch_total<uint32_t>(n);
}
}  // namespace hpxhip

extern "C" int hpxhip_scan(int dtype, int op, int inclusive, int conv_kind, const void* conv_scalars,
                           const void* init, const void* prefix_dev, const void* in, void* out, uint64_t n,
                           hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_scan");
    if (n == 0) return 0;
    if (!in || !out || (!init && !prefix_dev)) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        T iv = T(0);
        if (init) __builtin_memcpy(&iv, init, sizeof(T));
        return with_binop<T>(op, [&](auto o) -> int {
            return with_scan_conv<T>(conv_kind, conv_scalars, [&](auto conv) -> int {
                void* ws = nullptr;
                int rc = resolve_scratch(s, scratch, scratch_bytes, scratch_total<T>(n), &ws);
                if (rc) return rc;
                char* base = static_cast<char*>(ws);
                const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) &&
                                     (reinterpret_cast<uintptr_t>(out) % 16 == 0);
                const T* pd = static_cast<const T*>(prefix_dev);
                const T* ip = static_cast<const T*>(in);
                T* op_ = static_cast<T*>(out);
                if (inclusive) {
                    if (aligned) return launch_scan<T, true, true>(ip, op_, n, conv, o, iv, pd, base, s);
                    const int r = launch_scan_split<T, true>(ip, op_, n, conv, o, iv, pd, base, s);
                    return r >= 0 ? r : launch_scan<T, true, false>(ip, op_, n, conv, o, iv, pd, base, s);
                }
                if (aligned) return launch_scan<T, false, true>(ip, op_, n, conv, o, iv, pd, base, s);
                const int r = launch_scan_split<T, false>(ip, op_, n, conv, o, iv, pd, base, s);
                return r >= 0 ? r : launch_scan<T, false, false>(ip, op_, n, conv, o, iv, pd, base, s);
            });
        });
    });
}
