// oracle.cpp -- CPU restatement of HPX 1.4.0 seq/par semantics (see oracle.h).
//
// TEST INFRASTRUCTURE: never linked into or called by the product path.
// Compiled with g++ -ffp-contract=off so floating-point expressions round
// exactly as the reference's host functors do.
#include "oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <thread>
#include <type_traits>
#include <vector>

namespace {

enum { I32 = 0, U32, I64, U64, F32, F64 };
enum { PLUS = 0, MULTIPLIES, MIN, MAX, BIT_AND, BIT_OR, BIT_XOR };
enum { U_IDENTITY = 0, U_SCALE, U_ADD_SCALAR, U_AFFINE, U_NEGATE, U_ABS, U_SQUARE };
enum { B_ADD = 0, B_TRIAD, B_SUB, B_MUL, B_AXPY, B_MIN, B_MAX };
enum { P_LT = 0, P_LE, P_GT, P_GE, P_EQ, P_NE, P_NOT_LT, P_BITS };
constexpr int E_INVALID = 10001, E_UNSUPPORTED = 10002;

template <typename T> struct tag { using type = T; };

template <typename F>
int with_dtype(int dt, F&& f) {
    switch (dt) {
        case I32: return f(tag<int32_t>{});
        case U32: return f(tag<uint32_t>{});
        case I64: return f(tag<int64_t>{});
        case U64: return f(tag<uint64_t>{});
        case F32: return f(tag<float>{});
        case F64: return f(tag<double>{});
        default: return E_INVALID;
    }
}
template <typename T> constexpr int dtype_of() {
    if constexpr (std::is_same_v<T, int32_t>) return I32;
    else if constexpr (std::is_same_v<T, uint32_t>) return U32;
    else if constexpr (std::is_same_v<T, int64_t>) return I64;
    else if constexpr (std::is_same_v<T, uint64_t>) return U64;
    else if constexpr (std::is_same_v<T, float>) return F32;
    else return F64;
}
template <typename TI, typename F>
int with_wide(int dt, F&& f) {
    if (dt == dtype_of<TI>()) return f(tag<TI>{});
    if constexpr (std::is_integral_v<TI>) {
        if (dt == I64) return f(tag<int64_t>{});
    }
    if (dt == F64) return f(tag<double>{});
    return E_UNSUPPORTED;
}

// Two's-complement wrapping (what the reference's host build does in
// practice for signed overflow).
template <typename T> T wadd(T a, T b) {
    if constexpr (std::is_integral_v<T>) { using U = std::make_unsigned_t<T>; return T(U(a) + U(b)); }
    else return a + b;
}
template <typename T> T wmul(T a, T b) {
    if constexpr (std::is_integral_v<T>) { using U = std::make_unsigned_t<T>; return T(U(a) * U(b)); }
    else return a * b;
}
template <typename T> T wsub(T a, T b) {
    if constexpr (std::is_integral_v<T>) { using U = std::make_unsigned_t<T>; return T(U(a) - U(b)); }
    else return a - b;
}

// std::plus / std::multiplies / std::min / std::max / bit ops
template <typename T>
std::function<T(T, T)> binop(int op, bool* ok) {
    *ok = true;
    switch (op) {
        case PLUS: return [](T a, T b) { return wadd(a, b); };
        case MULTIPLIES: return [](T a, T b) { return wmul(a, b); };
        case MIN: return [](T a, T b) { return (b < a) ? b : a; };
        case MAX: return [](T a, T b) { return (a < b) ? b : a; };
        default: break;
    }
    if constexpr (std::is_integral_v<T>) {
        if (op == BIT_AND) return [](T a, T b) { return T(a & b); };
        if (op == BIT_OR) return [](T a, T b) { return T(a | b); };
        if (op == BIT_XOR) return [](T a, T b) { return T(a ^ b); };
    }
    *ok = false;
    return nullptr;
}

template <typename C>
std::function<C(C)> unary(int kind, const void* sc, bool* ok) {
    C s[2] = {C(0), C(0)};
    if (sc) std::memcpy(s, sc, sizeof(s));
    const C s0 = s[0], s1 = s[1];
    *ok = true;
    switch (kind) {
        case U_IDENTITY: return [](C x) { return x; };
        case U_SCALE: return [s0](C x) { return wmul(x, s0); };          // stream.cpp:235 val * factor_
        case U_ADD_SCALAR: return [s0](C x) { return wadd(x, s0); };     // for_each_compute.cu:44 i += 5
        case U_AFFINE: return [s0, s1](C x) { return wadd(wmul(x, s0), s1); };
        case U_NEGATE: return [](C x) {
            if constexpr (std::is_integral_v<C>) return wmul(x, C(-1)); else return -x; };
        case U_ABS: return [](C x) {
            if constexpr (std::is_unsigned_v<C>) return x;
            else if constexpr (std::is_integral_v<C>) return x < 0 ? wmul(x, C(-1)) : x;
            else return std::fabs(x); };
        case U_SQUARE: return [](C x) { return wmul(x, x); };
        default: *ok = false; return nullptr;
    }
}

template <typename C>
std::function<C(C, C)> binary(int kind, const void* sc, bool* ok) {
    C s0 = C(0);
    if (sc) std::memcpy(&s0, sc, sizeof(C));
    *ok = true;
    switch (kind) {
        case B_ADD: return [](C x, C y) { return wadd(x, y); };                 // stream.cpp:248
        case B_TRIAD: return [s0](C x, C y) { return wadd(x, wmul(y, s0)); };   // stream.cpp:262
        case B_SUB: return [](C x, C y) { return wsub(x, y); };
        case B_MUL: return [](C x, C y) { return wmul(x, y); };
        case B_AXPY: return [s0](C x, C y) { return wadd(wmul(x, s0), y); };
        case B_MIN: return [](C x, C y) { return (y < x) ? y : x; };
        case B_MAX: return [](C x, C y) { return (x < y) ? y : x; };
        default: *ok = false; return nullptr;
    }
}

template <typename T>
std::function<bool(T)> predicate(int kind, const void* arg, bool* ok) {
    T a = T(0);
    if (arg) std::memcpy(&a, arg, sizeof(T));
    *ok = true;
    switch (kind) {
        case P_LT: return [a](T x) { return x < a; };
        case P_LE: return [a](T x) { return x <= a; };
        case P_GT: return [a](T x) { return x > a; };
        case P_GE: return [a](T x) { return x >= a; };
        case P_EQ: return [a](T x) { return x == a; };
        case P_NE: return [a](T x) { return x != a; };
        case P_NOT_LT: return [a](T x) { return !(x < a); };  // copyif_random.cpp `!(i < 0)`
        case P_BITS:
            if constexpr (std::is_integral_v<T>) return [a](T x) { return (x & a) != 0; };
            break;
        default: break;
    }
    *ok = false;
    return nullptr;
}

// static_chunk_size chunking of [0, count) for `cores` cores:
//   chunk = ceil(count / (4 cores))          static_chunk_size.hpp:68
//   max_chunks = min(4 cores, count)          execution_parameters.hpp:121, chunk_size.hpp:104
//   chunk = max(chunk, ceil(count / max_chunks))  chunk_size.hpp:108-109
std::vector<std::pair<uint64_t, uint64_t>> par_chunks(uint64_t count, int cores) {
    std::vector<std::pair<uint64_t, uint64_t>> out;
    if (count == 0) return out;
    const uint64_t c4 = 4ull * static_cast<uint64_t>(cores);
    uint64_t chunk = (count + c4 - 1) / c4;
    const uint64_t max_chunks = std::min<uint64_t>(c4, count);
    chunk = std::max<uint64_t>(chunk, (count + max_chunks - 1) / max_chunks);
    for (uint64_t b = 0; b < count; b += chunk) out.emplace_back(b, std::min(chunk, count - b));
    return out;
}

// ordered-bit key for the IEEE total order / signed integers
template <typename T>
auto ordered(T x) {
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, uint32_t>;
    U u;
    std::memcpy(&u, &x, sizeof(T));
    constexpr U sign = U(1) << (sizeof(U) * 8 - 1);
    if constexpr (std::is_floating_point_v<T>) return (u & sign) ? U(~u) : U(u | sign);
    else if constexpr (std::is_signed_v<T>) return U(u ^ sign);
    else return u;
}

template <typename T>
void heat_steps(std::vector<double>&, T) {}

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// run f(chunk_index, begin, len) for the par chunks over `threads` threads
template <typename F>
void run_par(uint64_t n, int threads, F&& f) {
    auto chunks = par_chunks(n, threads);
    std::vector<std::thread> pool;
    const int nt = threads;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (size_t k = t; k < chunks.size(); k += nt) f(k, chunks[k].first, chunks[k].second);
        });
    for (auto& th : pool) th.join();
}

template <typename TI, typename TA, typename Conv, typename Op>
TA reduce_impl(const TI* a, uint64_t n, TA init, Conv conv, Op op, int cores) {
    if (cores <= 0 || n == 0) {
        // std::accumulate(first, last, init, r(res, conv(x)))  transform_reduce.hpp:59
        TA acc = init;
        for (uint64_t i = 0; i < n; ++i) acc = op(acc, conv(a[i]));
        return acc;
    }
    // transform_reduce.hpp:84-111: per chunk val = conv(*first), fold rest;
    // then accumulate_n(results, init, r)
    auto chunks = par_chunks(n, cores);
    TA acc = init;
    for (auto& c : chunks) {
        TA val = conv(a[c.first]);
        for (uint64_t i = c.first + 1; i < c.first + c.second; ++i) val = op(val, conv(a[i]));
        acc = op(acc, val);
    }
    return acc;
}

}  // namespace

extern "C" {

int oracle_version(void) { return 1; }

int oracle_fill(int dtype, const void* value, void* data, uint64_t n) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        T v;
        std::memcpy(&v, value, sizeof(T));
        std::fill_n(static_cast<T*>(data), n, v);
        return 0;
    });
}

int oracle_copy(int dtype, const void* in, void* out, uint64_t n) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        std::copy_n(static_cast<const T*>(in), n, static_cast<T*>(out));
        return 0;
    });
}

int oracle_for_each(int dtype, int kind, const void* scalars, void* data, uint64_t n) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        bool ok;
        auto f = unary<T>(kind, scalars, &ok);
        if (!ok) return E_INVALID;
        T* d = static_cast<T*>(data);
        for (uint64_t i = 0; i < n; ++i) d[i] = f(d[i]);
        return 0;
    });
}

int oracle_transform(int in_dt, int c_dt, int out_dt, int kind, const void* sc, const void* in, void* out,
                     uint64_t n) {
    return with_dtype(in_dt, [&](auto ti) {
        using TI = typename decltype(ti)::type;
        return with_wide<TI>(c_dt, [&](auto tc) {
            using C = typename decltype(tc)::type;
            return with_dtype(out_dt, [&](auto to) {
                using TO = typename decltype(to)::type;
                bool ok;
                auto f = unary<C>(kind, sc, &ok);
                if (!ok) return E_INVALID;
                const TI* a = static_cast<const TI*>(in);
                TO* o = static_cast<TO*>(out);
                for (uint64_t i = 0; i < n; ++i) o[i] = static_cast<TO>(f(static_cast<C>(a[i])));
                return 0;
            });
        });
    });
}

int oracle_transform_binary(int in_dt, int c_dt, int out_dt, int kind, const void* sc, const void* in1,
                            const void* in2, void* out, uint64_t n) {
    return with_dtype(in_dt, [&](auto ti) {
        using TI = typename decltype(ti)::type;
        return with_wide<TI>(c_dt, [&](auto tc) {
            using C = typename decltype(tc)::type;
            return with_dtype(out_dt, [&](auto to) {
                using TO = typename decltype(to)::type;
                bool ok;
                auto f = binary<C>(kind, sc, &ok);
                if (!ok) return E_INVALID;
                const TI* a = static_cast<const TI*>(in1);
                const TI* b = static_cast<const TI*>(in2);
                TO* o = static_cast<TO*>(out);
                for (uint64_t i = 0; i < n; ++i)
                    o[i] = static_cast<TO>(f(static_cast<C>(a[i]), static_cast<C>(b[i])));
                return 0;
            });
        });
    });
}

int oracle_transform_reduce(int in_dt, int acc_dt, int red_op, int conv_kind, const void* sc, const void* init,
                            const void* in, uint64_t n, void* out, int cores) {
    return with_dtype(in_dt, [&](auto ti) {
        using TI = typename decltype(ti)::type;
        return with_wide<TI>(acc_dt, [&](auto ta) {
            using TA = typename decltype(ta)::type;
            bool ok1, ok2;
            auto op = binop<TA>(red_op, &ok1);
            auto f = unary<TA>(conv_kind, sc, &ok2);
            if (!ok1 || !ok2) return E_UNSUPPORTED;
            TA iv;
            std::memcpy(&iv, init, sizeof(TA));
            auto conv = [&](TI x) { return f(static_cast<TA>(x)); };
            TA r = reduce_impl<TI, TA>(static_cast<const TI*>(in), n, iv, conv, op, cores);
            std::memcpy(out, &r, sizeof(TA));
            return 0;
        });
    });
}

int oracle_transform_reduce_binary(int in_dt, int acc_dt, int red_op, int bin_kind, const void* sc,
                                   const void* init, const void* in1, const void* in2, uint64_t n, void* out,
                                   int cores) {
    return with_dtype(in_dt, [&](auto ti) {
        using TI = typename decltype(ti)::type;
        return with_wide<TI>(acc_dt, [&](auto ta) {
            using TA = typename decltype(ta)::type;
            bool ok1, ok2;
            auto op = binop<TA>(red_op, &ok1);
            auto f = binary<TA>(bin_kind, sc, &ok2);
            if (!ok1 || !ok2) return E_UNSUPPORTED;
            TA iv;
            std::memcpy(&iv, init, sizeof(TA));
            const TI* a = static_cast<const TI*>(in1);
            const TI* b = static_cast<const TI*>(in2);
            TA acc = iv;
            if (cores <= 0) {
                for (uint64_t i = 0; i < n; ++i) acc = op(acc, f(static_cast<TA>(a[i]), static_cast<TA>(b[i])));
            } else {
                for (auto& c : par_chunks(n, cores)) {
                    TA val = f(static_cast<TA>(a[c.first]), static_cast<TA>(b[c.first]));
                    for (uint64_t i = c.first + 1; i < c.first + c.second; ++i)
                        val = op(val, f(static_cast<TA>(a[i]), static_cast<TA>(b[i])));
                    acc = op(acc, val);
                }
            }
            std::memcpy(out, &acc, sizeof(TA));
            return 0;
        });
    });
}

int oracle_scan(int dtype, int op_kind, int inclusive, int conv_kind, const void* sc, const void* init,
                const void* in, void* out, uint64_t n, int cores) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        bool ok1, ok2;
        auto op = binop<T>(op_kind, &ok1);
        auto conv = unary<T>(conv_kind, sc, &ok2);
        if (!ok1 || !ok2) return E_UNSUPPORTED;
        T iv;
        std::memcpy(&iv, init, sizeof(T));
        const T* a = static_cast<const T*>(in);
        T* o = static_cast<T*>(out);
        if (n == 0) return 0;
        // Work on a copy of the input so in-place calls see the original values.
        std::vector<T> x(a, a + n);
        if (cores <= 0) {
            T acc = iv;
            for (uint64_t i = 0; i < n; ++i) {
                const T nxt = op(acc, conv(x[i]));   // inclusive_scan.hpp:51 / exclusive_scan.hpp:54
                o[i] = inclusive ? nxt : acc;
                acc = nxt;
            }
            return 0;
        }
        // 3-phase (scan_partitioner.hpp:62-156)
        auto chunks = par_chunks(n, cores);
        std::vector<T> totals(chunks.size());
        for (size_t k = 0; k < chunks.size(); ++k) {  // step 1: local scan seeded by first element
            const uint64_t b = chunks[k].first, len = chunks[k].second;
            T run = conv(x[b]);
            if (inclusive) {
                o[b] = run;
                for (uint64_t i = b + 1; i < b + len; ++i) { run = op(run, conv(x[i])); o[i] = run; }
            } else {
                for (uint64_t i = b + 1; i < b + len; ++i) { o[i] = run; run = op(run, conv(x[i])); }
            }
            totals[k] = run;
        }
        T prefix = iv;  // step 2 + step 3
        for (size_t k = 0; k < chunks.size(); ++k) {
            const uint64_t b = chunks[k].first, len = chunks[k].second;
            if (inclusive) {
                for (uint64_t i = b; i < b + len; ++i) o[i] = op(prefix, o[i]);
            } else {
                o[b] = prefix;
                for (uint64_t i = b + 1; i < b + len; ++i) o[i] = op(prefix, o[i]);
            }
            prefix = op(prefix, totals[k]);
        }
        return 0;
    });
}

int oracle_copy_if(int dtype, int pred_kind, const void* arg, const void* in, void* out, uint64_t n,
                   uint64_t* count) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        bool ok;
        auto p = predicate<T>(pred_kind, arg, &ok);
        if (!ok) return E_UNSUPPORTED;
        const T* a = static_cast<const T*>(in);
        T* o = static_cast<T*>(out);
        uint64_t k = 0;
        for (uint64_t i = 0; i < n; ++i)
            if (p(a[i])) o[k++] = a[i];
        *count = k;
        return 0;
    });
}

int oracle_sort(int dtype, void* keys, uint64_t n, int descending) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        T* k = static_cast<T*>(keys);
        if (descending) std::sort(k, k + n, [](T a, T b) { return ordered(b) < ordered(a); });
        else std::sort(k, k + n, [](T a, T b) { return ordered(a) < ordered(b); });
        return 0;
    });
}

int oracle_sort_by_key(int key_dt, int val_dt, void* keys, void* values, uint64_t n, int descending) {
    return with_dtype(key_dt, [&](auto t) {
        using K = typename decltype(t)::type;
        return with_dtype(val_dt, [&](auto tv) {
            using V = typename decltype(tv)::type;
            K* k = static_cast<K*>(keys);
            V* v = static_cast<V*>(values);
            std::vector<uint64_t> idx(n);
            std::iota(idx.begin(), idx.end(), 0);
            if (descending)
                std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return ordered(k[b]) < ordered(k[a]); });
            else
                std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return ordered(k[a]) < ordered(k[b]); });
            std::vector<K> k2(n);
            std::vector<V> v2(n);
            for (uint64_t i = 0; i < n; ++i) { k2[i] = k[idx[i]]; v2[i] = v[idx[i]]; }
            std::copy(k2.begin(), k2.end(), k);
            std::copy(v2.begin(), v2.end(), v);
            return 0;
        });
    });
}

// merge.hpp:52-80 (sequential_merge): take from the second range only when
// comp(*first2, *first1); then copy the rest of both.  comp is std::less /
// std::greater over the sort's key order (ordered()).
int oracle_merge(int dtype, const void* in1, uint64_t n1, const void* in2, uint64_t n2, void* out, int descending) {
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        const T* a = static_cast<const T*>(in1);
        const T* b = static_cast<const T*>(in2);
        T* d = static_cast<T*>(out);
        auto comp = [&](T x, T y) { return descending ? ordered(y) < ordered(x) : ordered(x) < ordered(y); };
        uint64_t i = 0, j = 0;
        if (n1 && n2) {
            while (true) {
                if (comp(b[j], a[i])) {
                    *d++ = b[j++];
                    if (j == n2) break;
                } else {
                    *d++ = a[i++];
                    if (i == n1) break;
                }
            }
        }
        while (i < n1) *d++ = a[i++];
        while (j < n2) *d++ = b[j++];
        return 0;
    });
}

static inline double heat(double left, double middle, double right, double k, double dt, double dx) {
    return middle + (k * dt / (dx * dx)) * (left - 2 * middle + right);  // 1d_stencil_1.cpp:45
}

int oracle_stencil_heat(double* u, uint64_t nx, uint64_t nt, double k, double dt, double dx) {
    if (nx == 0) return 0;
    std::vector<double> next(nx);
    std::vector<double> cur(u, u + nx);
    for (uint64_t t = 0; t < nt; ++t) {  // 1d_stencil_1.cpp:58-70
        if (nx == 1) {
            next[0] = heat(cur[0], cur[0], cur[0], k, dt, dx);
        } else {
            next[0] = heat(cur[nx - 1], cur[0], cur[1], k, dt, dx);
            for (uint64_t i = 1; i + 1 < nx; ++i) next[i] = heat(cur[i - 1], cur[i], cur[i + 1], k, dt, dx);
            next[nx - 1] = heat(cur[nx - 2], cur[nx - 1], cur[0], k, dt, dx);
        }
        cur.swap(next);
    }
    std::copy(cur.begin(), cur.end(), u);
    return 0;
}

int oracle_stencil_heat_step(const double* cur, double* next, uint64_t n, double left, double right, double k,
                             double dt, double dx) {
    for (uint64_t i = 0; i < n; ++i) {
        const double l = i == 0 ? left : cur[i - 1];
        const double r = i + 1 == n ? right : cur[i + 1];
        next[i] = heat(l, cur[i], r, k, dt, dx);
    }
    return 0;
}

int oracle_stream_expected(uint64_t iterations, double scalar, double* aj_, double* bj_, double* cj_) {
    // stream.cpp:100-116
    double aj = 1.0, bj = 2.0, cj = 0.0;
    aj = 2.0E0 * aj;
    for (uint64_t k = 0; k < iterations; k++) {
        cj = aj;
        bj = scalar * cj;
        cj = aj + bj;
        aj = bj + scalar * cj;
    }
    *aj_ = aj;
    *bj_ = bj;
    *cj_ = cj;
    return 0;
}

int oracle_segmented_reduce(int dtype, int op_kind, const void* init, const void* in, uint64_t n, int parts,
                            void* out) {
    if (parts <= 0) return E_INVALID;
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        bool ok;
        auto op = binop<T>(op_kind, &ok);
        if (!ok) return E_UNSUPPORTED;
        T acc;
        std::memcpy(&acc, init, sizeof(T));
        const T* a = static_cast<const T*>(in);
        const uint64_t part = (n + parts - 1) / parts;  // partitioned_vector_impl.hpp:325
        for (int p = 0; p < parts; ++p) {
            const uint64_t b = std::min<uint64_t>(n, p * part), e = std::min<uint64_t>(n, b + part);
            if (b == e) continue;
            T s = a[b];  // detail/reduce.hpp:43-62: no init, first element seeds
            for (uint64_t i = b + 1; i < e; ++i) s = op(s, a[i]);
            acc = op(acc, s);  // segmented_algorithms/reduce.hpp:201-206
        }
        std::memcpy(out, &acc, sizeof(T));
        return 0;
    });
}

int oracle_segmented_scan(int dtype, int op_kind, int inclusive, const void* init, const void* in, void* out,
                          uint64_t n, int parts) {
    if (parts <= 0) return E_INVALID;
    return with_dtype(dtype, [&](auto t) {
        using T = typename decltype(t)::type;
        bool ok;
        auto op = binop<T>(op_kind, &ok);
        if (!ok) return E_UNSUPPORTED;
        T carry;
        std::memcpy(&carry, init, sizeof(T));
        const T* a = static_cast<const T*>(in);
        T* o = static_cast<T*>(out);
        std::vector<T> x(a, a + n);
        const uint64_t part = (n + parts - 1) / parts;
        for (int p = 0; p < parts; ++p) {
            const uint64_t b = std::min<uint64_t>(n, p * part), e = std::min<uint64_t>(n, b + part);
            if (b == e) continue;  // empty segments are skipped (detail/scan.hpp:602-624)
            // step 1: the segment total, seeded by its first element
            // (sequential_segmented_scan_T, detail/scan.hpp:46-59)
            T total = x[b];
            for (uint64_t i = b + 1; i < e; ++i) total = op(total, x[i]);
            // step 2: the segment scanned from its carry (detail/scan.hpp:646-665)
            T acc = carry;
            for (uint64_t i = b; i < e; ++i) {
                const T nxt = op(acc, x[i]);
                o[i] = inclusive ? nxt : acc;
                acc = nxt;
            }
            // step 3: next carry = carry (op) total (detail/scan.hpp:667-677;
            // the sequential form, :409-429, applies op(total, carry), the
            // same value for the commutative operators built here)
            carry = op(carry, total);
        }
        return 0;
    });
}

// ------------------------------------------------------------- par baseline
void* oracle_par_alloc(uint64_t bytes, int threads) {
    char* p = static_cast<char*>(::operator new(bytes));
    // first touch by the thread that will process the chunk
    // (host::block_allocator, block_allocator.hpp:157-200)
    const uint64_t pages = (bytes + 4095) / 4096;
    run_par(pages, threads, [&](size_t, uint64_t b, uint64_t len) {
        std::memset(p + b * 4096, 0, std::min<uint64_t>(len * 4096, bytes - b * 4096));
    });
    return p;
}

void oracle_par_free(void* p, uint64_t) { ::operator delete(p); }

// stream.cpp:294-375 on the host `par` policy: fill a = 1, b = 2, c = 0,
// a = 2a, then `iterations` rounds of copy (c = a), scale (b = s c), add
// (c = a + b) and triad (a = b + s c), each timed; best[k] / avg[k] = min /
// mean seconds over iterations 1.. (the first is skipped, :485-495);
// abc[0..2] = a[0], b[0], c[0] for check_results (:82-133).  Arrays are
// first-touched by the thread that processes them (block_allocator.hpp).
int oracle_par_stream(uint64_t n, double s, int iterations, int threads, double* best, double* avg, double* abc) {
    if (iterations < 2 || n == 0) return 1;
    double* a = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    double* b = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    double* c = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    auto loop = [&](auto&& f) {
        const double t0 = now();
        run_par(n, threads, [&](size_t, uint64_t beg, uint64_t len) {
            for (uint64_t i = beg; i < beg + len; ++i) f(i);
        });
        return now() - t0;
    };
    loop([&](uint64_t i) { a[i] = 1.0; b[i] = 2.0; c[i] = 0.0; });
    loop([&](uint64_t i) { a[i] = a[i] * 2.0; });  // multiply_step(2.0), stream.cpp:303-305
    for (int k = 0; k < 4; ++k) best[k] = 1e300, avg[k] = 0.0;
    for (int it = 0; it < iterations; ++it) {
        double t[4];
        t[0] = loop([&](uint64_t i) { c[i] = a[i]; });
        t[1] = loop([&](uint64_t i) { b[i] = c[i] * s; });  // multiply_step: val * factor_ (:234-237)
        t[2] = loop([&](uint64_t i) { c[i] = a[i] + b[i]; });
        t[3] = loop([&](uint64_t i) { a[i] = b[i] + c[i] * s; });  // triad_step: val1 + val2 * factor_ (:266-269)
        if (it == 0) continue;
        for (int k = 0; k < 4; ++k) {
            best[k] = std::min(best[k], t[k]);
            avg[k] += t[k] / (iterations - 1);
        }
    }
    abc[0] = a[0], abc[1] = b[0], abc[2] = c[0];
    oracle_par_free(a, n * 8);
    oracle_par_free(b, n * 8);
    oracle_par_free(c, n * 8);
    return 0;
}

double oracle_par_triad(double* a, const double* b, const double* c, uint64_t n, double s, int threads) {
    const double t0 = now();
    run_par(n, threads, [&](size_t, uint64_t beg, uint64_t len) {
        for (uint64_t i = beg; i < beg + len; ++i) a[i] = b[i] + c[i] * s;
    });
    return now() - t0;
}

double oracle_par_reduce_i64(const int64_t* in, uint64_t n, int64_t init, int64_t* out, int threads) {
    const double t0 = now();
    auto chunks = par_chunks(n, threads);
    std::vector<int64_t> part(chunks.size());
    run_par(n, threads, [&](size_t k, uint64_t beg, uint64_t len) {
        int64_t v = in[beg];
        for (uint64_t i = beg + 1; i < beg + len; ++i) v = wadd(v, in[i]);
        part[k] = v;
    });
    int64_t acc = init;
    for (auto v : part) acc = wadd(acc, v);
    *out = acc;
    return now() - t0;
}

double oracle_par_scan_i64(const int64_t* in, int64_t* out, uint64_t n, int threads) {
    const double t0 = now();
    auto chunks = par_chunks(n, threads);
    std::vector<int64_t> tot(chunks.size());
    run_par(n, threads, [&](size_t k, uint64_t beg, uint64_t len) {
        int64_t run = in[beg];
        out[beg] = run;
        for (uint64_t i = beg + 1; i < beg + len; ++i) { run = wadd(run, in[i]); out[i] = run; }
        tot[k] = run;
    });
    std::vector<int64_t> pre(chunks.size());
    int64_t p = 0;
    for (size_t k = 0; k < chunks.size(); ++k) { pre[k] = p; p = wadd(p, tot[k]); }
    run_par(n, threads, [&](size_t k, uint64_t beg, uint64_t len) {
        const int64_t v = pre[k];
        for (uint64_t i = beg; i < beg + len; ++i) out[i] = wadd(v, out[i]);
    });
    return now() - t0;
}

double oracle_par_copy_if_i64(const int64_t* in, int64_t* out, uint64_t n, uint64_t* count, int threads) {
    const double t0 = now();
    auto chunks = par_chunks(n, threads);
    std::vector<uint64_t> cnt(chunks.size());
    std::vector<unsigned char> flags(n);
    run_par(n, threads, [&](size_t k, uint64_t beg, uint64_t len) {
        uint64_t c = 0;
        for (uint64_t i = beg; i < beg + len; ++i) { flags[i] = in[i] >= 0; c += flags[i]; }
        cnt[k] = c;
    });
    std::vector<uint64_t> pre(chunks.size());
    uint64_t p = 0;
    for (size_t k = 0; k < chunks.size(); ++k) { pre[k] = p; p += cnt[k]; }
    run_par(n, threads, [&](size_t k, uint64_t beg, uint64_t len) {
        uint64_t o = pre[k];
        for (uint64_t i = beg; i < beg + len; ++i) if (flags[i]) out[o++] = in[i];
    });
    *count = p;
    return now() - t0;
}

// examples/1d_stencil/1d_stencil_4_parallel.cpp:87-156 restated on
// std::threads: per step, the points are split into HPX par chunks, each
// computed from the current buffer (periodic neighbours, idx() :35-38), then
// the buffers swap (the next step depends on all chunks: a join per step).
// Same arithmetic as oracle_stencil_heat, so the result is identical.
double oracle_par_stencil(double* u0, double* u1, uint64_t n, uint64_t nt, double k, double dt, double dx,
                          int threads) {
    const double t0 = now();
    double* cur = u0;
    double* nxt = u1;
    for (uint64_t t = 0; t < nt && n >= 2; ++t) {
        run_par(n, threads, [&](size_t, uint64_t beg, uint64_t len) {
            for (uint64_t i = beg; i < beg + len; ++i) {
                const double l = cur[i == 0 ? n - 1 : i - 1];
                const double r = cur[i + 1 == n ? 0 : i + 1];
                nxt[i] = heat(l, cur[i], r, k, dt, dx);
            }
        });
        std::swap(cur, nxt);
    }
    return now() - t0;
}

// HPX sort.hpp:78-229 restated: median-of-3 pivot, partition, recurse in
// parallel above the chunk limit, std::sort leaves.
static void par_sort_rec(uint64_t* first, uint64_t* last, uint64_t limit, int depth) {
    const uint64_t n = static_cast<uint64_t>(last - first);
    if (n <= limit || depth <= 0) {
        std::sort(first, last);
        return;
    }
    uint64_t* mid = first + n / 2;
    uint64_t a = *first, b = *mid, c = *(last - 1);
    uint64_t pivot = std::max(std::min(a, b), std::min(std::max(a, b), c));
    uint64_t* m1 = std::partition(first, last, [pivot](uint64_t x) { return x < pivot; });
    uint64_t* m2 = std::partition(m1, last, [pivot](uint64_t x) { return !(pivot < x); });
    std::thread th(par_sort_rec, first, m1, limit, depth - 1);
    par_sort_rec(m2, last, limit, depth - 1);
    th.join();
}

double oracle_par_sort_u64(uint64_t* keys, uint64_t n, int threads) {
    const double t0 = now();
    // chunk = max(ceil(N/(4 cores)), 65536)  sort.hpp:48, 190-196
    uint64_t limit = std::max<uint64_t>((n + 4ull * threads - 1) / (4ull * threads), 65536);
    int depth = 1;
    while ((1 << depth) < 4 * threads) ++depth;
    par_sort_rec(keys, keys + n, limit, depth + 2);
    return now() - t0;
}

}  // extern "C"
