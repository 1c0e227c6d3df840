// oracle_sanitize.cpp -- the CPU oracle under AddressSanitizer and
// UndefinedBehaviorSanitizer ("ASan/UBSan on the CPU
// oracle"; the reference builds with HPX_WITH_SANITIZERS,
// CMakeLists.txt:844,1732-1733).  Host code only: g++ compiles this file with
// oracle/oracle.cpp under -fsanitize=address,undefined
// -fno-sanitize-recover=all (Makefile target oracle-sanitize), so any
// out-of-bounds access, leak, signed overflow or misaligned access in the
// checker aborts the run.  Every exported oracle function is driven over
// small and ragged sizes (0, 1, 2, 7, 63, 64, 65, 1000, 4099), and the
// results are cross-checked the way the golden tests do: seq == par for
// integer work at several core counts, seq == segmented at several partition
// counts, sort output ordered and a permutation, inclusive - exclusive ==
// input, copy_if count == predicate count, stencil step == serial step.
#include "../../include/hpxhip.h"
#include "../../oracle/oracle.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                        \
        }                                                                    \
    } while (0)

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static std::vector<int64_t> ints(uint64_t n, uint64_t seed) {
    std::vector<int64_t> v(n);
    for (auto& x : v) x = static_cast<int64_t>(splitmix(seed) % 2001) - 1000;
    return v;
}

static void elementwise(uint64_t n) {
    std::vector<double> a(n), b(n), c(n), d(n);
    for (uint64_t i = 0; i < n; ++i) b[i] = 0.5 * double(i), c[i] = 2.0 + double(i % 7);
    const double two = 2.0, s3 = 3.0;
    CHECK(oracle_fill(HPXHIP_F64, &two, a.data(), n) == 0);
    for (uint64_t i = 0; i < n; ++i) CHECK(a[i] == 2.0);
    CHECK(oracle_copy(HPXHIP_F64, b.data(), a.data(), n) == 0);
    CHECK(std::equal(a.begin(), a.end(), b.begin()));
    const double sc[2] = {3.0, 0.0};
    CHECK(oracle_for_each(HPXHIP_F64, HPXHIP_U_SCALE, sc, a.data(), n) == 0);
    CHECK(oracle_transform(HPXHIP_F64, HPXHIP_F64, HPXHIP_F64, HPXHIP_U_SCALE, sc, b.data(), d.data(), n) == 0);
    CHECK(std::equal(a.begin(), a.end(), d.begin()));
    CHECK(oracle_transform_binary(HPXHIP_F64, HPXHIP_F64, HPXHIP_F64, HPXHIP_B_TRIAD, &s3, b.data(), c.data(),
                                  a.data(), n) == 0);
    for (uint64_t i = 0; i < n; ++i) CHECK(a[i] == b[i] + c[i] * 3.0);
    // int(a + 3.0*b) into int (transform_compute.cu)
    std::vector<int32_t> o(n);
    CHECK(oracle_transform_binary(HPXHIP_F64, HPXHIP_F64, HPXHIP_I32, HPXHIP_B_TRIAD, &s3, b.data(), c.data(),
                                  o.data(), n) == 0);
    for (uint64_t i = 0; i < n; ++i) CHECK(o[i] == int32_t(b[i] + c[i] * 3.0));
}

static void reductions(uint64_t n) {
    const auto x = ints(n, 7 + n);
    const int64_t init = 5;
    const int ops[] = {HPXHIP_PLUS, HPXHIP_MULTIPLIES, HPXHIP_MIN, HPXHIP_MAX, HPXHIP_BIT_AND, HPXHIP_BIT_OR,
                       HPXHIP_BIT_XOR};
    for (int op : ops) {
        int64_t seq = 0;
        CHECK(oracle_transform_reduce(HPXHIP_I64, HPXHIP_I64, op, HPXHIP_U_IDENTITY, nullptr, &init, x.data(), n,
                                      &seq, 0) == 0);
        for (int cores : {1, 3, 8}) {
            int64_t par = 0;
            CHECK(oracle_transform_reduce(HPXHIP_I64, HPXHIP_I64, op, HPXHIP_U_IDENTITY, nullptr, &init, x.data(),
                                          n, &par, cores) == 0);
            CHECK(par == seq);
        }
        for (int parts : {1, 2, 3, 8}) {
            int64_t sg = 0;
            CHECK(oracle_segmented_reduce(HPXHIP_I64, op, &init, x.data(), n, parts, &sg) == 0);
            if (n > 0) CHECK(sg == seq);
        }
    }
    int64_t ip = 0, ip1 = 0;
    CHECK(oracle_transform_reduce_binary(HPXHIP_I64, HPXHIP_I64, HPXHIP_PLUS, HPXHIP_B_MUL, nullptr, &init, x.data(),
                                         x.data(), n, &ip, 0) == 0);
    CHECK(oracle_transform_reduce_binary(HPXHIP_I64, HPXHIP_I64, HPXHIP_PLUS, HPXHIP_B_MUL, nullptr, &init, x.data(),
                                         x.data(), n, &ip1, 4) == 0);
    CHECK(ip == ip1);
}

static void scans(uint64_t n) {
    const auto x = ints(n, 11 + n);
    const int64_t init = -3;
    std::vector<int64_t> inc(n), exc(n), par(n), seg(n);
    CHECK(oracle_scan(HPXHIP_I64, HPXHIP_PLUS, 1, HPXHIP_U_IDENTITY, nullptr, &init, x.data(), inc.data(), n, 0) == 0);
    CHECK(oracle_scan(HPXHIP_I64, HPXHIP_PLUS, 0, HPXHIP_U_IDENTITY, nullptr, &init, x.data(), exc.data(), n, 0) == 0);
    for (uint64_t i = 0; i < n; ++i) CHECK(inc[i] - exc[i] == x[i]);
    for (int cores : {1, 3, 8}) {
        CHECK(oracle_scan(HPXHIP_I64, HPXHIP_PLUS, 1, HPXHIP_U_IDENTITY, nullptr, &init, x.data(), par.data(), n,
                          cores) == 0);
        CHECK(par == inc);
    }
    for (int parts : {1, 2, 3, 8}) {
        CHECK(oracle_segmented_scan(HPXHIP_I64, HPXHIP_PLUS, 0, &init, x.data(), seg.data(), n, parts) == 0);
        CHECK(seg == exc);
    }
    // in place (exclusive_scan_validate.cpp runs both forms)
    std::vector<int64_t> y = x;
    CHECK(oracle_scan(HPXHIP_I64, HPXHIP_PLUS, 1, HPXHIP_U_IDENTITY, nullptr, &init, y.data(), y.data(), n, 0) == 0);
    CHECK(y == inc);
}

static void compaction_and_order(uint64_t n) {
    const auto x = ints(n, 13 + n);
    std::vector<int64_t> out(n + 1);
    uint64_t cnt = 0;
    const int64_t zero = 0;
    CHECK(oracle_copy_if(HPXHIP_I64, HPXHIP_P_NOT_LT, &zero, x.data(), out.data(), n, &cnt) == 0);
    CHECK(cnt == uint64_t(std::count_if(x.begin(), x.end(), [](int64_t v) { return !(v < 0); })));
    for (uint64_t i = 0; i < cnt; ++i) CHECK(out[i] >= 0);

    std::vector<int64_t> k = x;
    CHECK(oracle_sort(HPXHIP_I64, k.data(), n, 0) == 0);
    CHECK(std::is_sorted(k.begin(), k.end()));
    std::vector<int64_t> ref = x;
    std::sort(ref.begin(), ref.end());
    CHECK(k == ref);
    CHECK(oracle_sort(HPXHIP_I64, k.data(), n, 1) == 0);
    CHECK(std::is_sorted(k.rbegin(), k.rend()));

    std::vector<uint64_t> keys(n), vals(n);
    uint64_t s = 17 + n;
    for (uint64_t i = 0; i < n; ++i) keys[i] = splitmix(s) % 16, vals[i] = i;
    CHECK(oracle_sort_by_key(HPXHIP_U64, HPXHIP_U64, keys.data(), vals.data(), n, 0) == 0);
    for (uint64_t i = 1; i < n; ++i) {
        CHECK(keys[i - 1] <= keys[i]);
        if (keys[i - 1] == keys[i]) CHECK(vals[i - 1] < vals[i]);  // stable
    }

    const uint64_t n1 = n / 2, n2 = n - n1;
    std::vector<int64_t> a(ref.begin(), ref.begin() + n1), b(ref.begin() + n1, ref.end()), m(n);
    CHECK(oracle_merge(HPXHIP_I64, b.data(), n2, a.data(), n1, m.data(), 0) == 0);
    CHECK(m == ref);
}

static void stencil(uint64_t n) {
    if (n < 3) return;
    std::vector<double> u(n), cur(n), next(n);
    uint64_t s = 23 + n;
    for (uint64_t i = 0; i < n; ++i) u[i] = cur[i] = double(splitmix(s) % 1000) / 7.0;
    CHECK(oracle_stencil_heat(u.data(), n, 1, 0.5, 1.0, 1.0) == 0);
    CHECK(oracle_stencil_heat_step(cur.data(), next.data(), n, cur[n - 1], cur[0], 0.5, 1.0, 1.0) == 0);
    CHECK(std::memcmp(u.data(), next.data(), n * sizeof(double)) == 0);
    double aj = 0, bj = 0, cj = 0;
    CHECK(oracle_stream_expected(10, 3.0, &aj, &bj, &cj) == 0);
}

static void host_baseline() {
    const uint64_t n = 1 << 16;
    const int threads = 3;
    auto* a = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    auto* b = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    auto* c = static_cast<double*>(oracle_par_alloc(n * 8, threads));
    for (uint64_t i = 0; i < n; ++i) b[i] = 1.0, c[i] = 2.0;
    CHECK(oracle_par_triad(a, b, c, n, 3.0, threads) >= 0.0);
    for (uint64_t i = 0; i < n; ++i) CHECK(a[i] == 7.0);
    const auto x = ints(n, 29);
    std::vector<int64_t> y(n);
    int64_t r = 0, seq = 0;
    const int64_t init = 0;
    CHECK(oracle_par_reduce_i64(x.data(), n, 0, &r, threads) >= 0.0);
    CHECK(oracle_transform_reduce(HPXHIP_I64, HPXHIP_I64, HPXHIP_PLUS, HPXHIP_U_IDENTITY, nullptr, &init, x.data(), n,
                                  &seq, 0) == 0);
    CHECK(r == seq);
    CHECK(oracle_par_scan_i64(x.data(), y.data(), n, threads) >= 0.0);
    CHECK(y[n - 1] == seq);
    uint64_t cnt = 0;
    CHECK(oracle_par_copy_if_i64(x.data(), y.data(), n, &cnt, threads) >= 0.0);
    std::vector<uint64_t> keys(n);
    uint64_t s = 31;
    for (auto& k : keys) k = splitmix(s);
    CHECK(oracle_par_sort_u64(keys.data(), n, threads) >= 0.0);
    CHECK(std::is_sorted(keys.begin(), keys.end()));
    std::vector<double> u0(4099), u1(4099);
    for (uint64_t i = 0; i < u0.size(); ++i) u0[i] = double(i);
    CHECK(oracle_par_stencil(u0.data(), u1.data(), u0.size(), 5, 0.5, 1.0, 1.0, threads) >= 0.0);
    oracle_par_free(a, n * 8);
    oracle_par_free(b, n * 8);
    oracle_par_free(c, n * 8);
}

int main() {
    CHECK(oracle_version() > 0);
    for (uint64_t n : {0ull, 1ull, 2ull, 7ull, 63ull, 64ull, 65ull, 1000ull, 4099ull}) {
        elementwise(n);
        reductions(n);
        scans(n);
        compaction_and_order(n);
        stencil(n);
    }
    host_baseline();
    if (g_fail) {
        std::fprintf(stderr, "oracle_sanitize: %d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("oracle_sanitize: all checks passed\n");
    return 0;
}
