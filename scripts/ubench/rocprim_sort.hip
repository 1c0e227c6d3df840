// Calibration only (not shipped): rocPRIM's radix sort on the same 2^30
// uint64 keys, to know what a tuned library reaches on this GPU.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
__global__ void gen(uint64_t* k, uint64_t n, uint64_t seed) {
  uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i < n) { uint64_t z = (i ^ seed) + 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; k[i] = z ^ (z >> 31); }
}
int main() {
  const size_t N = 1ull << 30;
  uint64_t *in, *out; CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8));
  size_t tmp_bytes = 0; void* tmp = nullptr;
  CK(rocprim::radix_sort_keys(tmp, tmp_bytes, in, out, N));
  CK(hipMalloc(&tmp, tmp_bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < 4; ++r) {
    gen<<<N / 256, 256>>>(in, N, r);
    CK(hipEventRecord(e0));
    CK(rocprim::radix_sort_keys(tmp, tmp_bytes, in, out, N));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  printf("rocprim radix_sort_keys u64 2^30: min %.3f ms  -> %.2f Gkeys/s (tmp %zu MB)\n", t[0], N / t[0] / 1e6, tmp_bytes >> 20);
  // rocprim radix_sort_keys with double buffer
  rocprim::double_buffer<uint64_t> db(in, out);
  size_t tb2 = 0; CK(rocprim::radix_sort_keys(nullptr, tb2, db, N)); void* tmp2; CK(hipMalloc(&tmp2, tb2));
  t.clear();
  for (int r = 0; r < 4; ++r) {
    gen<<<N / 256, 256>>>(db.current(), N, r);
    CK(hipEventRecord(e0));
    CK(rocprim::radix_sort_keys(tmp2, tb2, db, N));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  printf("rocprim radix_sort_keys double_buffer u64 2^30: min %.3f ms -> %.2f Gkeys/s\n", t[0], N / t[0] / 1e6);
  return 0;
}
