// copy_if.hip -- stable stream compaction (hpx::parallel::copy_if).
//
// Reference: copy.hpp:401-494 -- phase 1 writes a bool flag per element
// (boost::shared_array<bool>, copy.hpp:416) and counts hits per chunk,
// phase 2 prefixes the counts, phase 3 re-reads input + flags and scatters.
// Here: one pass.  Each wave evaluates the predicate on 64 lanes x 16 B,
// ranks hits with `ballot` + `mbcnt` (no flag array in HBM), the tile's hit
// count goes through the same decoupled look-back as the scan
// (lookback.hpp), and hits are written to out[prefix + rank]: each wave
// round's hits are compacted through LDS and stored by consecutive lanes.
// Input loads are nontemporal.  Traffic: 8 B read + 8 B x selectivity
// written per int64 element.  Aligned inputs (r05) run the pipelined form,
// k_copy_if_pipe: one persistent workgroup per CU stages a tile's hits in
// LDS and issues the next tile's loads before its look-back and write-out;
// misaligned ones (element-wise loads) keep one tile per workgroup.
#include <cstdlib>

#include "internal.hpp"
#include <hpxhip/kernels/copy_if_kernel.hpp>

using namespace hpxhip;

namespace {

using namespace hpxhip::copy_if_detail;

// Rounds (16-B vectors per lane) per tile: kRounds for the aligned path, 8
// for the element-wise unaligned path.  Scratch is sized for 8 (the most
// tiles), so one size serves both.
constexpr int kRounds = 8;
template <bool ALIGNED>
constexpr int rounds_for() {
    return ALIGNED ? kRounds : 8;
}

constexpr size_t kSlotsOff = 256;  // [counter | tile slots], zeroed per call

template <typename T, int ROUNDS>
uint64_t ntiles_for(uint64_t n) {
    return (n + tile_elems<T, ROUNDS>() - 1) / tile_elems<T, ROUNDS>();
}

// [counter | tile slots | head count]: the head count (misaligned inputs)
// sits past the region the per-call memset clears.
template <typename T>
size_t head_count_off(uint64_t n) {
    return align_up(kSlotsOff + ntiles_for<T, 8>(n) * tile_state<uint64_t>::bytes_per_tile(), 256);
}
template <typename T>
size_t scratch_total(uint64_t n) {
    return head_count_off<T>(n) + 256;
}

// Look-back values are hit counts, at most n: below 2^32 elements they travel
// as 32-bit values (one granule per slot instead of two).  That is what
// brings the kernel to 64 VGPRs, i.e. two 1024-thread workgroups per CU, so
// one workgroup's look-back and write-out overlap the other's loads: 2^30
// int64 at 50 % hits 2.55 -> 2.32 ms (profiles/r01_ubench_copyif_state.log).
template <typename T, bool ALIGNED, typename SV, typename P>
int launch_copy_if_sv(const T* in, T* out, uint64_t n, P p, uint64_t* count_dev, char* ws, hipStream_t s,
                      const uint64_t* prefix0) {
    constexpr int R = rounds_for<ALIGNED>();
    const uint64_t ntiles = ntiles_for<T, R>(n);
    HPXHIP_CHECK(hipMemsetAsync(ws, 0, align_up(kSlotsOff + ntiles * tile_state<SV>::bytes_per_tile(), 256), s));
    tile_state<SV> st{reinterpret_cast<uint64_t*>(ws + kSlotsOff), device_error_word(s)};
    // r03: the fixed-association look-back (tiles fold their group's
    // published aggregates plus one group word, lookback.hpp) in blockIdx
    // order: 2^30 int64 at 50 % hits 2.34 -> 2.20-2.21 ms, 2^31 int32 2.38 ->
    // 2.30-2.32 (profiles/r03_ubench_copyif7.log).  With the variable-window
    // look-back the atomic counter had been the faster order (2.33 vs 2.36,
    // profiles/r02_ubench_tile_order_ab.log).
    constexpr bool kDynId = false;
    constexpr bool kFixed = true;
    // 8-byte elements: four wave rounds of hits per LDS batch (one wait per
    // batch), 2.176-2.181 -> 2.164-2.168 ms at 2^30 int64
    // (profiles/r03_ubench_copyif7_writeout.log); no gain for 4-byte ones
    // (profiles/r02_ubench_copyif_writeout.log)
    constexpr int kRpb = (sizeof(T) == 8 && ALIGNED) ? 4 : 1;
    // Aligned, with the 32-bit look-back state: at most 64 VGPRs (8 waves per SIMD),
    // so two workgroups share a CU.  4-byte elements compiled to 70 VGPRs
    // at the old bound (4 waves per SIMD) and ran one workgroup per CU:
    // int32 2^31 2.77 -> 2.38 ms (profiles/r02_ubench_copyif_occupancy.log).
    constexpr int kMinWaves = (std::is_same_v<SV, uint32_t> && ALIGNED) ? 8 : 4;
    // r04: nontemporal output stores for 8-byte elements, 2.182-2.199 ->
    // 2.175-2.176 ms at 2^30 int64 (profiles/r04_ubench_copyif8.log; round 2
    // had measured them slower under counter-ordered tiles)
    constexpr bool kNtStore = sizeof(T) == 8 && ALIGNED;
    // r04, 8-byte elements: 16-B output stores and the one-hop look-back
    // (copy_if_kernel.hpp): 2.18-2.20 -> 2.13-2.15 ms at 2^30 int64
    constexpr bool kWide = sizeof(T) == 8 && ALIGNED;
    constexpr bool kOneHop = sizeof(T) == 8;
    if constexpr (ALIGNED) {
        // r05: the pipelined persistent form (copy_if_kernel.hpp), one
        // workgroup per CU: 2^30 int64 at 50 % hits 2.13-2.14 -> 1.96-1.97 ms,
        // 2^31 int32 2.26-2.28 -> 2.15 (profiles/r05_ubench_copyif9.log)
        const uint64_t grid = std::min<uint64_t>(ntiles, static_cast<uint64_t>(current_device_info().cus));
        hipLaunchKernelGGL((k_copy_if_pipe<T, P, R, SV>), dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, s, in,
                           out, n, p, count_dev, reinterpret_cast<uint32_t*>(ws), st, ntiles, prefix0);
        HPXHIP_CHECK_LAUNCH();
    } else {
        hipLaunchKernelGGL((k_copy_if<T, P, ALIGNED, R, kMinWaves, 0, SV, kDynId, kNtStore, kRpb, kFixed, kThreads,
                                      kWide, kOneHop>),
                           dim3(static_cast<unsigned>(ntiles)), dim3(kThreads), 0, s, in, out, n, p, count_dev,
                           reinterpret_cast<uint32_t*>(ws), st, ntiles, prefix0);
        HPXHIP_CHECK_LAUNCH();
    }
    return 0;
}

template <typename T, bool ALIGNED, typename P>
int launch_copy_if(const T* in, T* out, uint64_t n, P p, uint64_t* count_dev, char* ws, hipStream_t s,
                   const uint64_t* prefix0 = nullptr) {
    // HPXHIP_COPY_IF_STATE64=1 forces the 64-bit form at any n (tests; read per call).
    const char* e = getenv("HPXHIP_COPY_IF_STATE64");
    const bool force64 = e && e[0] == '1';
    if (n < (uint64_t{1} << 32) && !force64)
        return launch_copy_if_sv<T, ALIGNED, uint32_t>(in, out, n, p, count_dev, ws, s, prefix0);
    return launch_copy_if_sv<T, ALIGNED, uint64_t>(in, out, n, p, count_dev, ws, s, prefix0);
}

}  // namespace

namespace hpxhip {
size_t copy_if_scratch_bytes(int dtype, uint64_t n) {
    return dtype_size(dtype) == 8 ? scratch_total<uint64_t>(n) : scratch_total<uint32_t>(n);
}
}  // namespace hpxhip

extern "C" int hpxhip_copy_if(int dtype, int pred_kind, const void* pred_arg, const void* in, void* out, uint64_t n,
                              uint64_t* count_dev, hpxhip_stream stream, void* scratch, size_t scratch_bytes) {
    HPXHIP_ANNOTATE("hpxhip_copy_if");
    if (!count_dev || (n && (!in || !out))) return HPXHIP_ERROR_INVALID_ARGUMENT;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    device_guard g(s);
    if (g.status) return g.status;
    if (n == 0) {
        hipLaunchKernelGGL(k_zero_count, dim3(1), dim3(64), 0, s, count_dev);
        HPXHIP_CHECK_LAUNCH();
        return 0;
    }
    return with_dtype(dtype, [&](auto t) -> int {
        using T = typename decltype(t)::type;
        return with_pred<T>(pred_kind, pred_arg, [&](auto p) -> int {
            void* ws = nullptr;
            int rc = resolve_scratch(s, scratch, scratch_bytes, scratch_total<T>(n), &ws);
            if (rc) return rc;
            const T* ip = static_cast<const T*>(in);
            T* op = static_cast<T*>(out);
            char* base = static_cast<char*>(ws);
            const uint64_t h = head_to_align16(in, sizeof(T));
            if (h == 0) return launch_copy_if<T, true>(ip, op, n, p, count_dev, base, s);
            // A misaligned input whose elements are naturally aligned: the
            // head (< 16 B) is compacted first, the rest takes the vector
            // kernel seeded with the head's count (int64 offset by one
            // element: 3.83 -> ~2.4 ms at 2^30, profiles/r02_unaligned_ranges.log).
            if (h != UINT64_MAX && n > 4 * h) {
                auto* hc = reinterpret_cast<uint64_t*>(base + head_count_off<T>(n));
                hipLaunchKernelGGL((k_copy_if_head<T, decltype(p)>), dim3(1), dim3(64), 0, s, ip, op, h, p, hc);
                HPXHIP_CHECK_LAUNCH();
                return launch_copy_if<T, true>(ip + h, op, n - h, p, count_dev, base, s, hc);
            }
            return launch_copy_if<T, false>(ip, op, n, p, count_dev, base, s);
        });
    });
}
