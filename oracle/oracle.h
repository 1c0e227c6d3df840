/*
 * oracle.h -- CPU restatement of HPX 1.4.0's seq/par semantics for the
 * data-parallel algorithm path.  TEST INFRASTRUCTURE ONLY: imported by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker / host baseline, never by the product (hpx_amd/).
 *
 * Enum values are those of include/hpxhip.h (dtype, binop, unary, binary,
 * pred) so a test can feed both with the same arguments.
 *
 * Each function cites the reference code it restates.  Pinning: checked
 * against the reference's own known-answer tests (tests/golden/, generated
 * by tests/golden/make_golden.py from the closed forms in the reference's
 * tests) in tests/test_oracle_golden.py.
 */
#ifndef HPX_ORACLE_H
#define HPX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int oracle_version(void);

/* fill.hpp:38-159 / copy.hpp:55-114 */
int oracle_fill(int dtype, const void* value, void* data, uint64_t n);
int oracle_copy(int dtype, const void* in, void* out, uint64_t n);

/* for_each.hpp:186-195 (seq loop), unary transform transform.hpp:146-155,
   binary transform transform.hpp:411-461 / 643-694 */
int oracle_for_each(int dtype, int unary_kind, const void* scalars, void* data, uint64_t n);
int oracle_transform(int in_dtype, int compute_dtype, int out_dtype, int unary_kind,
                     const void* scalars, const void* in, void* out, uint64_t n);
int oracle_transform_binary(int in_dtype, int compute_dtype, int out_dtype, int binary_kind,
                            const void* scalars, const void* in1, const void* in2, void* out,
                            uint64_t n);

/* transform_reduce.hpp:50-66 (seq: std::accumulate(first,last,init, r(res, conv(x))));
   par (cores > 0): transform_reduce.hpp:68-112 with static_chunk_size
   chunking (static_chunk_size.hpp:68, execution_parameters.hpp:121,
   chunk_size.hpp:56-124): chunk partial P_k = conv(x_first) (op) ... ,
   result = init (op) P_0 (op) ... (op) P_{m-1}.  cores == 0 -> seq. */
int oracle_transform_reduce(int in_dtype, int acc_dtype, int red_op, int conv_kind,
                            const void* conv_scalars, const void* init, const void* in,
                            uint64_t n, void* out, int cores);
/* transform_reduce_binary.hpp:323 (seq: std::inner_product-like left fold) */
int oracle_transform_reduce_binary(int in_dtype, int acc_dtype, int red_op, int binary_kind,
                                   const void* bin_scalars, const void* init, const void* in1,
                                   const void* in2, uint64_t n, void* out, int cores);

/* inclusive_scan.hpp:45-69 (sequential_inclusive_scan: init = op(init, conv(x)); *d = init),
   exclusive_scan.hpp:48-74 (sequential_exclusive_scan: *d = init; init = op(init, x)).
   par (cores > 0): scan_partitioner.hpp:62-156 + inclusive_scan.hpp:121-161:
   chunk local scan seeded by its first element, prefix_k = op(prefix_{k-1}, total_k),
   fix-up out = op(prefix_{k-1}, local). */
int oracle_scan(int dtype, int op, int inclusive, int conv_kind, const void* conv_scalars,
                const void* init, const void* in, void* out, uint64_t n, int cores);

/* copy.hpp:367-377 sequential_copy_if; returns count via *count */
int oracle_copy_if(int dtype, int pred_kind, const void* pred_arg, const void* in, void* out,
                   uint64_t n, uint64_t* count);

/* sort.hpp:237-248 (std::sort with std::less / std::greater).  For F32/F64
   the comparison is the IEEE total order on bit patterns (so -0.0 < +0.0),
   the order the radix sort produces; on data without signed zeros or NaNs
   it equals std::less. */
int oracle_sort(int dtype, void* keys, uint64_t n, int descending);
/* merge.hpp:52-80 sequential_merge (stable, first range first on ties). */
int oracle_merge(int dtype, const void* in1, uint64_t n1, const void* in2, uint64_t n2, void* out, int descending);
/* sort_by_key.hpp:42-78, stable variant (ties keep input order). */
int oracle_sort_by_key(int key_dtype, int value_dtype, void* keys, void* values, uint64_t n,
                       int descending);

/* 1d_stencil_1.cpp:41-72: nt periodic heat steps, serial; result in u (n doubles). */
int oracle_stencil_heat(double* u, uint64_t n, uint64_t nt, double k, double dt, double dx);
/* One step with explicit halos (1d_stencil_4_parallel.cpp:87-118 heat_part). */
int oracle_stencil_heat_step(const double* cur, double* next, uint64_t n, double left,
                             double right, double k, double dt, double dx);

/* stream.cpp:82-133: closed-form expected a,b,c after `iterations` STREAM loops. */
int oracle_stream_expected(uint64_t iterations, double scalar, double* aj, double* bj, double* cj);

/* segmented reduce (segmented_algorithms/reduce.hpp:112-209, detail/reduce.hpp:31-62):
   n split in `parts` partitions of ceil(n/parts) (partitioned_vector_impl.hpp:325),
   S_k seeded by the partition's first element, result init (op) S_0 (op) ... */
int oracle_segmented_reduce(int dtype, int op, const void* init, const void* in, uint64_t n,
                            int parts, void* out);
/* segmented scan (segmented_algorithms/detail/scan.hpp:527-696): carries in
   segment order, per-segment seq scan with init = carry. */
int oracle_segmented_scan(int dtype, int op, int inclusive, const void* init, const void* in,
                          void* out, uint64_t n, int parts);

/* ---- host `par` baseline (bench.py cpu_baseline; HPX par restated with
   std::thread: 4*threads chunks of ceil(N/(4*threads)), first-touch) ---- */
/* Allocate n doubles/int64 with first-touch by the same chunk->thread map. */
void* oracle_par_alloc(uint64_t bytes, int threads);
void oracle_par_free(void* p, uint64_t bytes);
/* a[i] = b[i] + s*c[i] over `threads` threads; returns seconds. */
double oracle_par_triad(double* a, const double* b, const double* c, uint64_t n, double s,
                        int threads);
/* stream.cpp:294-375 (copy, scale, add, triad; `iterations` rounds, the
   first skipped): best/avg seconds per kernel, abc = a[0], b[0], c[0]. */
int oracle_par_stream(uint64_t n, double s, int iterations, int threads, double* best, double* avg,
                      double* abc);
/* sum of int64 with init; returns seconds, result in *out. */
double oracle_par_reduce_i64(const int64_t* in, uint64_t n, int64_t init, int64_t* out,
                             int threads);
/* inclusive scan int64 (3-phase), returns seconds. */
double oracle_par_scan_i64(const int64_t* in, int64_t* out, uint64_t n, int threads);
/* parallel sort uint64 (HPX sort.hpp quicksort restatement, std::sort leaves); seconds */
double oracle_par_sort_u64(uint64_t* keys, uint64_t n, int threads);
double oracle_par_stencil(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt, double dx,
                          int threads);
/* copy_if int64 x >= 0 (3-phase), returns seconds, count in *count */
double oracle_par_copy_if_i64(const int64_t* in, int64_t* out, uint64_t n, uint64_t* count,
                              int threads);

#ifdef __cplusplus
}
#endif
#endif
