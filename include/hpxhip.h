/*
 * hpxhip.h -- C ABI of the MI355X (gfx950) backend for HPX's data-parallel
 * algorithm layer.
 *
 * Every entry point is extern "C", takes plain pointers/sizes/enums, and
 * returns an int status: 0 on success, a hipError_t value for a HIP runtime
 * failure, or one of the HPXHIP_ERROR_* codes below.  No function frees
 * caller memory.  All algorithm calls are asynchronous on the given stream
 * (stream order = HPX's sequencing of the algorithm's effects); completion is
 * observed with hpxhip_stream_synchronize / hpxhip_stream_add_callback /
 * events, which the C++ and Python layers turn into hpx::future.
 *
 * What each call replaces in the reference (HPX 1.4.0, /root/reference):
 *   - device/stream/completion  -> hpx/compute/cuda/target.hpp:36-200,
 *       src/compute/cuda/cuda_target.cpp:97-142 (stream callback -> future),
 *       :255-317 (lazy non-blocking stream, synchronize),
 *       src/compute/cuda/get_cuda_targets.cpp:30-65 (enumeration)
 *   - memory                    -> hpx/compute/cuda/allocator.hpp:108-160,
 *       hpx/compute/cuda/transfer.hpp:188-348 (H2D/D2H/D2D copies)
 *   - fill/copy/for_each/transform -> the generic launch_function kernel the
 *       CUDA default_executor instantiates per closure
 *       (hpx/compute/cuda/detail/launch.hpp:32-137,
 *        default_executor.hpp:87-136) for fill.hpp:86, copy.hpp:88-114,
 *        for_each.hpp:369-423, transform.hpp:138-182,411-461,643-694
 *   - reduce/transform_reduce   -> host-only partitioner path
 *       hpx/parallel/algorithms/reduce.hpp:40-89,
 *       transform_reduce.hpp:43-113, transform_reduce_binary.hpp:323,432
 *   - inclusive/exclusive_scan  -> inclusive_scan.hpp:90-173,
 *       exclusive_scan.hpp:100-175 + util/scan_partitioner.hpp:62-156
 *   - copy_if                   -> copy.hpp:401-494
 *   - sort / sort_by_key        -> sort.hpp:182-276, sort_by_key.hpp:42-78
 *   - 1d_stencil heat step      -> examples/1d_stencil/1d_stencil_1.cpp:41-72,
 *       1d_stencil_4_parallel.cpp:87-118
 *
 * The reference has no C ABI (its CUDA calls are inline templates); these
 * entry points are what an FFI or the header-only C++ layer binds.
 */
#ifndef HPXHIP_H
#define HPXHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HPXHIP_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
enum hpxhip_status {
    HPXHIP_SUCCESS = 0,
    /* 1..999: hipError_t values passed through unchanged */
    HPXHIP_ERROR_INVALID_ARGUMENT = 10001,
    HPXHIP_ERROR_UNSUPPORTED = 10002,     /* dtype/op combination not built */
    HPXHIP_ERROR_DEVICE_TIMEOUT = 10003,  /* a kernel gave up a bounded spin */
    HPXHIP_ERROR_OUT_OF_MEMORY = 10004,
    HPXHIP_ERROR_NOT_READY = 10005
};

/* ----------------------------------------------------------------- types */
enum hpxhip_dtype {
    HPXHIP_I32 = 0,
    HPXHIP_U32 = 1,
    HPXHIP_I64 = 2,
    HPXHIP_U64 = 3,
    HPXHIP_F32 = 4,
    HPXHIP_F64 = 5
};

/* Binary reduction / scan operators (std::plus, std::multiplies, ...). */
enum hpxhip_binop {
    HPXHIP_PLUS = 0,
    HPXHIP_MULTIPLIES = 1,
    HPXHIP_MIN = 2,
    HPXHIP_MAX = 3,
    HPXHIP_BIT_AND = 4,
    HPXHIP_BIT_OR = 5,
    HPXHIP_BIT_XOR = 6
};

/* Unary element functors y = f(x); s0, s1 are scalars of the compute dtype. */
enum hpxhip_unary {
    HPXHIP_U_IDENTITY = 0,   /* x                      (copy)                  */
    HPXHIP_U_SCALE = 1,      /* x * s0                 (stream.cpp:224 multiply_step) */
    HPXHIP_U_ADD_SCALAR = 2, /* x + s0                 (for_each_compute.cu:40 i += 5) */
    HPXHIP_U_AFFINE = 3,     /* x * s0 + s1                                    */
    HPXHIP_U_NEGATE = 4,     /* -x                                             */
    HPXHIP_U_ABS = 5,        /* |x|                                            */
    HPXHIP_U_SQUARE = 6      /* x * x                                          */
};

/* Binary element functors z = f(x, y). */
enum hpxhip_binary {
    HPXHIP_B_ADD = 0,   /* x + y        (stream.cpp:243 add_step)              */
    HPXHIP_B_TRIAD = 1, /* x + y * s0   (stream.cpp:257 triad_step;
                           transform_compute.cu:36 a + 3.0*b)                  */
    HPXHIP_B_SUB = 2,   /* x - y                                               */
    HPXHIP_B_MUL = 3,   /* x * y        (inner product's conv)                 */
    HPXHIP_B_AXPY = 4,  /* x * s0 + y                                          */
    HPXHIP_B_MIN = 5,   /* (y < x) ? y : x                                     */
    HPXHIP_B_MAX = 6    /* (x < y) ? y : x                                     */
};

/* Predicates for copy_if: pred(x) against scalar a of the element dtype. */
enum hpxhip_pred {
    HPXHIP_P_LT = 0,     /* x < a                                              */
    HPXHIP_P_LE = 1,     /* x <= a                                             */
    HPXHIP_P_GT = 2,     /* x > a                                              */
    HPXHIP_P_GE = 3,     /* x >= a                                             */
    HPXHIP_P_EQ = 4,     /* x == a                                             */
    HPXHIP_P_NE = 5,     /* x != a                                             */
    HPXHIP_P_NOT_LT = 6, /* !(x < a)   (copyif_random.cpp:45 `!(i < 0)`)       */
    HPXHIP_P_BITS = 7    /* (x & a) != 0, integers only                        */
};

enum hpxhip_memcpy_kind {
    HPXHIP_H2H = 0,
    HPXHIP_H2D = 1,
    HPXHIP_D2H = 2,
    HPXHIP_D2D = 3,
    HPXHIP_DEFAULT = 4
};

/* Algorithms whose scratch size can be queried. */
enum hpxhip_algo {
    HPXHIP_ALGO_REDUCE = 0,
    HPXHIP_ALGO_SCAN = 1,
    HPXHIP_ALGO_COPY_IF = 2,
    HPXHIP_ALGO_SORT = 3,
    HPXHIP_ALGO_SORT_BY_KEY = 4,
    HPXHIP_ALGO_MERGE = 5,  /* n = n1 + n2 */
    HPXHIP_ALGO_MERGE_RUNS = 6  /* n = the runs' total (hpxhip_merge_runs, up to 8 runs) */
};

typedef struct hpxhip_stream_opaque* hpxhip_stream; /* == hipStream_t */
typedef struct hpxhip_event_opaque* hpxhip_event;   /* == hipEvent_t  */
typedef void (*hpxhip_callback)(void* user, int status);

typedef struct hpxhip_device_props {
    char name[256];
    char arch[64];            /* "gfx950:sramecc+:xnack-" */
    int compute_units;        /* 256 on MI355X (cuda_target.cpp:145-184 analogue) */
    int wave_size;            /* 64 */
    int max_threads_per_block;
    int clock_khz;
    int memory_clock_khz;
    int memory_bus_width;
    size_t total_global_mem;
    size_t lds_per_block;
    int pci_bus_id;
    int pci_device_id;
} hpxhip_device_props;

/* ------------------------------------------------------ library / errors */
int hpxhip_abi_version(void);
const char* hpxhip_error_string(int status);
/* Reads and clears the device error word of `device` (kernel-side faults
   that must not hang the GPU, e.g. a look-back spin that gave up). */
int hpxhip_device_error(int device, uint32_t* code);
/* Fault injection for the error-path tests -- the role HPX's throw_always /
   throw_bad_alloc test functors play (tests/unit/parallel/algorithms/
   foreach_tests.hpp:120-205).  hpxhip_debug_inject_error: the next `count`
   algorithm entry points called on this host thread return `status` without
   enqueuing anything (count 0 cancels).  hpxhip_debug_raise_device_error:
   enqueues on `stream` a write of `code` into the device error word, as a
   kernel that gave up a bounded spin does, so the failure surfaces only when
   the queued work completes. */
int hpxhip_debug_inject_error(int status, int count);
int hpxhip_debug_raise_device_error(hpxhip_stream stream, uint32_t code);
/* The next `count` event waits or queries (hpxhip_event_synchronize /
   hpxhip_event_query) on this host thread return `status` -- a completion
   whose event wait fails, as after a kernel fault (count 0 cancels). */
int hpxhip_debug_inject_event_error(int status, int count);

/* ------------------------------------------------ devices (targets) */
int hpxhip_get_device_count(int* count);
int hpxhip_set_device(int device);
int hpxhip_get_device(int* device);
int hpxhip_device_props_get(int device, hpxhip_device_props* props);
int hpxhip_device_synchronize(int device);
int hpxhip_enable_peer_access(int device, int peer);
int hpxhip_can_access_peer(int device, int peer, int* can);

/* ------------------------------------------------ streams & completion */
int hpxhip_stream_create(int device, hpxhip_stream* stream);
int hpxhip_stream_destroy(hpxhip_stream stream);
int hpxhip_stream_synchronize(hpxhip_stream stream);
/* 0 if all work is complete, HPXHIP_ERROR_NOT_READY otherwise. */
int hpxhip_stream_query(hpxhip_stream stream);
/* fn(user, status) runs on a HIP runtime thread once all prior work on the
   stream is done; it must not call HIP (mirrors cuda_target.cpp:97-142). */
int hpxhip_stream_add_callback(hpxhip_stream stream, hpxhip_callback fn, void* user);

int hpxhip_event_create(hpxhip_event* event);
int hpxhip_event_destroy(hpxhip_event event);
/* An event created on `device` (timing 0: hipEventDisableTiming), so it can
   be recorded on that device's streams from any host thread -- the ordering
   event of a cross-device dependency in a multi-GPU process (the reference
   chains such dependencies through futures, segmented_algorithms/
   reduce.hpp:191-207; here hpxhip_stream_wait_event on the event). */
int hpxhip_event_create_on(int device, int timing, hpxhip_event* event);
/* The device a stream belongs to (NULL stream: the current device). */
int hpxhip_stream_device(hpxhip_stream stream, int* device);

int hpxhip_event_record(hpxhip_event event, hpxhip_stream stream);
int hpxhip_event_synchronize(hpxhip_event event);
int hpxhip_event_query(hpxhip_event event);
int hpxhip_event_elapsed_ms(hpxhip_event start, hpxhip_event stop, float* ms);
int hpxhip_stream_wait_event(hpxhip_stream stream, hpxhip_event event);

/* ------------------------------------------------------------- memory */
/* hip::allocator::allocate/deallocate (allocator.hpp:108-160): hipMalloc /
   hipFree; hipErrorOutOfMemory -> HPXHIP_ERROR_OUT_OF_MEMORY. */
int hpxhip_malloc(int device, void** ptr, size_t bytes);
int hpxhip_free(void* ptr);
int hpxhip_malloc_host(void** ptr, size_t bytes); /* pinned */
int hpxhip_free_host(void* ptr);
int hpxhip_mem_info(int device, size_t* free_bytes, size_t* total_bytes);

int hpxhip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, hpxhip_stream stream);
int hpxhip_memcpy_peer_async(void* dst, int dst_device, const void* src, int src_device,
                             size_t bytes, hpxhip_stream stream);
int hpxhip_memset_async(void* dst, int value, size_t bytes, hpxhip_stream stream);
/* Bytes of scratch `algo` needs for n elements of dtype (sort_by_key: the
   value dtype is passed in `aux_dtype`, else ignored). */
int hpxhip_scratch_bytes(int algo, int dtype, int aux_dtype, uint64_t n, size_t* bytes);

/* The per-stream scratch cache itself (>= bytes of device memory, reused by
   later calls on the same stream, so valid for stream-ordered work queued
   before the next call that takes scratch on that stream), and the device
   error word the look-back kernels raise a bounded-spin timeout in.  For
   kernels instantiated outside the library -- the C++ layer's device
   closures (hpx/parallel/detail/device_algorithms.hpp), which run the same
   kernel bodies (include/hpxhip/kernels/) with user callables.  No reference
   counterpart: cuda::target's per-target scratch lives in the CUDA runtime. */
int hpxhip_stream_scratch(hpxhip_stream stream, size_t bytes, void** ptr);
int hpxhip_device_error_word(hpxhip_stream stream, uint32_t** word);

/* Scratch convention for every algorithm below: pass (NULL, 0) to let the
   library use a per-stream cached buffer (grown with hipMalloc, so not
   graph-capturable); or pass a caller-owned device buffer of at least
   hpxhip_scratch_bytes() bytes (capturable, no allocation). */

/* ------------------------------------------------ elementwise (for_each) */
/* fill.hpp:86: data[i] = *value (value: host pointer to one dtype element). */
int hpxhip_fill(int dtype, const void* value, void* data, uint64_t n, hpxhip_stream stream);
/* generate.hpp (hpx::parallel::generate / iota-style initialisation of the
   reference tests, e.g. std::iota in transform_reduce.cpp:29):
     GEN_IOTA : data[i] = lo + i
     GEN_BITS : data[i] = bits of splitmix64(seed ^ i) (upper 32 bits for 4-byte types)
     GEN_RANGE: data[i] = lo + splitmix64(seed ^ i) % (hi - lo + 1)   (integers)
     GEN_UNIT : data[i] = (splitmix64(seed ^ i) >> 11) * 2^-53 in [0,1)
                (float: >> 40, * 2^-24)                                  */
enum hpxhip_gen { HPXHIP_GEN_IOTA = 0, HPXHIP_GEN_BITS = 1, HPXHIP_GEN_RANGE = 2, HPXHIP_GEN_UNIT = 3 };
int hpxhip_generate(int dtype, int kind, uint64_t seed, int64_t lo, int64_t hi, void* data, uint64_t n,
                    hpxhip_stream stream);
/* Same with global indices i = index_base + j for data[j] (a partition of a
   partitioned_vector generates exactly its slice of the global sequence). */
int hpxhip_generate_at(int dtype, int kind, uint64_t seed, uint64_t index_base, int64_t lo, int64_t hi,
                       void* data, uint64_t n, hpxhip_stream stream);
/* copy.hpp:88-114: out[i] = in[i]. */
int hpxhip_copy(int dtype, const void* in, void* out, uint64_t n, hpxhip_stream stream);
/* for_each.hpp:369: data[i] = f(data[i]) in place (for_each_compute.cu `i += 5`). */
int hpxhip_for_each(int dtype, int unary_kind, const void* scalars, void* data, uint64_t n,
                    hpxhip_stream stream);
/* transform.hpp:138 (unary): out[i] = (out_t) f((compute_t) in[i]).
   Built combinations: in == out dtype, compute dtype == in dtype or F64. */
int hpxhip_transform(int in_dtype, int compute_dtype, int out_dtype, int unary_kind,
                     const void* scalars, const void* in, void* out, uint64_t n,
                     hpxhip_stream stream);
/* transform.hpp:411/643 (binary): out[i] = (out_t) f((compute_t) in1[i], (compute_t) in2[i]). */
int hpxhip_transform_binary(int in_dtype, int compute_dtype, int out_dtype, int binary_kind,
                            const void* scalars, const void* in1, const void* in2, void* out,
                            uint64_t n, hpxhip_stream stream);
/* for_loop_n with strided pointer inductions (for_loop_induction.hpp:210-219:
 * value at iteration i = base + stride * i):
 *   out[i*out_stride] = (out_t) f((compute_t) in[i*in_stride])              (unary)
 *   out[i*out_stride] = (out_t) f((compute_t) in1[i*s1], (compute_t) in2[i*s2]) (binary)
 * Strides are in elements and may be negative; an input stride may be 0.  An
 * output stride of 0 with n > 1 is HPXHIP_ERROR_INVALID_ARGUMENT (every
 * iteration would write one element), and so is a walk whose span
 * |stride| * (n-1) * size reaches 2^47 bytes.  Like the reference's raw
 * pointer inductions, the ABI does not know the allocations: a walk that
 * leaves its buffer within that span is the caller's error (the Python mirror
 * checks it against the vector; the C++ layer, pointer-based as HPX's
 * iterators are, does not). */
int hpxhip_transform_strided(int in_dtype, int compute_dtype, int out_dtype, int unary_kind,
                             const void* scalars, const void* in, int64_t in_stride, void* out,
                             int64_t out_stride, uint64_t n, hpxhip_stream stream);
int hpxhip_transform_binary_strided(int in_dtype, int compute_dtype, int out_dtype, int binary_kind,
                                    const void* scalars, const void* in1, int64_t in1_stride,
                                    const void* in2, int64_t in2_stride, void* out,
                                    int64_t out_stride, uint64_t n, hpxhip_stream stream);

/* --------------------------------------------------------- reductions */
/* transform_reduce.hpp:254: *out_dev = init (op) conv(in[0]) (op) ... (op) conv(in[n-1]),
   accumulated in acc_dtype (== in dtype, or I64/F64 widening).  reduce.hpp:200
   is conv_kind = HPXHIP_U_IDENTITY.  out_dev is device memory; init is a
   host pointer to one acc_dtype value.  Integer results are exact; FP results
   use a fixed (run-to-run deterministic) tree, see DESIGN.md for tolerance. */
int hpxhip_transform_reduce(int in_dtype, int acc_dtype, int red_op, int conv_kind,
                            const void* conv_scalars, const void* init, const void* in,
                            uint64_t n, void* out_dev, hpxhip_stream stream, void* scratch,
                            size_t scratch_bytes);
/* transform_reduce_binary.hpp:323: init (op) f(in1[0], in2[0]) (op) ...
   (inner product: red_op = PLUS, binary_kind = B_MUL). */
int hpxhip_transform_reduce_binary(int in_dtype, int acc_dtype, int red_op, int binary_kind,
                                   const void* bin_scalars, const void* init, const void* in1,
                                   const void* in2, uint64_t n, void* out_dev,
                                   hpxhip_stream stream, void* scratch, size_t scratch_bytes);
/* Ordered fold of a short device array: *out_dev = init (op) v[0] (op) ... (op) v[count-1].
   Used for the segment-order combine of segmented reduce/scan carries
   (segmented_algorithms/reduce.hpp:191-207, detail/scan.hpp:667-677). */
int hpxhip_fold(int dtype, int op, const void* init, const void* values_dev, uint64_t count,
                void* out_dev, hpxhip_stream stream);
/* Every prefix of the same fold: out_dev[0] = init, out_dev[j + 1] = out_dev[j] (op) v[j]
   (count + 1 values) -- the carries of a segmented scan in segment order
   (segmented_algorithms/detail/scan.hpp:646-677), folded on the device. */
int hpxhip_fold_exclusive(int dtype, int op, const void* init, const void* values_dev, uint64_t count,
                          void* out_dev, hpxhip_stream stream);

/* -------------------------------------------------------------- scans */
/* inclusive_scan.hpp:288 / exclusive_scan.hpp:292 (+ transform_*_scan with
   conv_kind != IDENTITY).  inclusive: out[i] = P (op) conv(in[0]) ... conv(in[i]);
   exclusive: out[0] = P, out[i] = P (op) conv(in[0]) ... conv(in[i-1]).
   P = *prefix_dev if prefix_dev != NULL (device value; segmented carry),
   else *init (host pointer).  in may alias out (in-place, as
   exclusive_scan_validate.cpp tests).  Single pass, decoupled look-back. */
int hpxhip_scan(int dtype, int op, int inclusive, int conv_kind, const void* conv_scalars,
                const void* init, const void* prefix_dev, const void* in, void* out,
                uint64_t n, hpxhip_stream stream, void* scratch, size_t scratch_bytes);

/* ------------------------------------------------------------ copy_if */
/* copy.hpp:585: stable compaction of in[i] with pred(in[i], *pred_arg) into
   out; *count_dev (uint64, device) receives the number copied, so the
   returned dest iterator is out + count.  out must not overlap in. */
int hpxhip_copy_if(int dtype, int pred_kind, const void* pred_arg, const void* in, void* out,
                   uint64_t n, uint64_t* count_dev, hpxhip_stream stream, void* scratch,
                   size_t scratch_bytes);

/* --------------------------------------------------------------- sort */
/* sort.hpp:364: ascending (std::less) or descending (std::greater) sort of
   keys in place; LSD onesweep radix sort.  F32/F64 use the IEEE total order
   (-0.0 before +0.0; NaNs by sign/payload at the ends). */
int hpxhip_sort(int dtype, void* keys, uint64_t n, int descending, hpxhip_stream stream,
                void* scratch, size_t scratch_bytes);
/* sort_by_key.hpp:42: stable sort of keys with values permuted alongside
   (value dtype = any 4/8-byte dtype). */
int hpxhip_sort_by_key(int key_dtype, int value_dtype, void* keys, void* values, uint64_t n,
                       int descending, hpxhip_stream stream, void* scratch, size_t scratch_bytes);

/* -------------------------------------------------------------- merge */
/* merge.hpp:476: stable merge of the sorted ranges in1[0,n1) and in2[0,n2)
   into out[0,n1+n2) (equal keys: in1's first, merge.hpp:52-80), ascending
   (std::less) or descending (std::greater), in the same key order as
   hpxhip_sort.  out must not overlap the inputs. */
int hpxhip_merge(int dtype, const void* in1, uint64_t n1, const void* in2, uint64_t n2, void* out,
                 int descending, hpxhip_stream stream, void* scratch, size_t scratch_bytes);
/* The segmented sort's merge step (no reference counterpart: HPX 1.4 has no
   segmented sort; its local algorithm is sort.hpp:364): the nruns (1..8)
   sorted runs in[run_offsets[j], run_offsets[j+1]) (run_offsets: a HOST
   array of nruns+1 non-decreasing element offsets) merged into
   out[0, run_offsets[nruns] - run_offsets[0]) in one pass, in the key order
   of hpxhip_sort (keys only: equal keys are not told apart).  out must not
   overlap in.  Scratch: HPXHIP_ALGO_MERGE_RUNS with n = the total. */
int hpxhip_merge_runs(int dtype, const void* in, const uint64_t* run_offsets, int nruns, void* out,
                      int descending, hpxhip_stream stream, void* scratch, size_t scratch_bytes);
/* Batched binary search in a sorted range (the partition cut of the
   segmented sort; std::lower_bound / std::upper_bound semantics under the
   sort's key order): out_dev[i] = number of sorted[] elements ordered before
   values_dev[i] (upper != 0: before or equal).  All pointers are device
   memory; out_dev holds m uint64 counts. */
int hpxhip_sorted_bounds(int dtype, const void* sorted, uint64_t n, const void* values_dev, uint64_t m,
                         int upper, int descending, uint64_t* out_dev, hpxhip_stream stream);

/* is_sorted.hpp:40-120: *count_dev (uint64, device; overwritten) = the
   number of adjacent pairs with pred(keys[i+1], keys[i]), pred = std::less
   (std::greater if descending) on the values -- so -0.0/+0.0 are equal and
   NaN is never out of order, as in the reference (0 <=> sorted); full-size
   sort verification without a host copy. */
int hpxhip_unsorted_pairs(int dtype, const void* keys, uint64_t n, int descending, uint64_t* count_dev,
                          hpxhip_stream stream);

/* ---------------------------------------------------------- 1d_stencil */
/* One heat step of examples/1d_stencil: next[i] = heat(cur[i-1], cur[i], cur[i+1])
   with heat(l,m,r) = m + (k*dt/(dx*dx)) * (l - 2*m + r)  (1d_stencil_1.cpp:43-46).
   cur[-1] := *left_halo_dev, cur[n] := *right_halo_dev (device pointers;
   for one periodic partition pass cur+n-1 and cur). */
int hpxhip_stencil_heat_step(const double* cur, double* next, uint64_t n,
                             const double* left_halo_dev, const double* right_halo_dev,
                             double k, double dt, double dx, hpxhip_stream stream);
/* Temporal blocking: `steps` heat steps in one pass over HBM (steps = 1 or
   an even number up to HPXHIP_STENCIL_MAX_FUSED), writing next[out_lo,
   out_hi) from cur[0, n).  Points left of cur[0] are left_halo_dev[0..steps)
   (left_halo_dev[steps-1] = cur[-1]), points right of cur[n-1] are
   right_halo_dev[0..steps) (right_halo_dev[0] = cur[n]); device pointers.
   Bit-identical to `steps` calls of hpxhip_stencil_heat_step.  Replaces the
   per-step partition update of 1d_stencil_8.cpp:482-531 (the halo becomes
   `steps` points wide, exchanged once per pass). */
#define HPXHIP_STENCIL_MAX_FUSED 16
int hpxhip_stencil_heat_steps(const double* cur, double* next, uint64_t n, uint64_t out_lo, uint64_t out_hi,
                              const double* left_halo_dev, const double* right_halo_dev, int steps, double k,
                              double dt, double dx, hpxhip_stream stream);
/* nt periodic steps on one partition, ping-ponging u0/u1; the result is in
   u0 if nt is even, else in u1 (1d_stencil_1.cpp:58-70).  Runs fused passes
   of up to HPXHIP_STENCIL_MAX_FUSED steps for rings of >= 1024 points. */
int hpxhip_stencil_heat_run(double* u0, double* u1, uint64_t n, uint64_t nt, double k,
                            double dt, double dx, hpxhip_stream stream);
/* As hpxhip_stencil_heat_run with the fewest passes (nt = 16q + r -> q
   passes of 16, then r's); *result_in_u1 (set on return, host memory) tells which
   buffer holds the result. */
int hpxhip_stencil_heat_run_fused(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt,
                                  double dx, int* result_in_u1, hpxhip_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* HPXHIP_H */
