// cpu_sort.cpp — TEST / BASELINE INFRASTRUCTURE ONLY (never called by the product path).
//
// Host std::sort / std::stable_sort wrappers: the reference's "host std::sort" plumbing
// path (BASELINE.json configs[0]: 64K uniform u32 keys) and the CPU baseline that bench.py
// times beside the GPU.  __gnu_parallel::sort runs on `threads` OpenMP
// threads when threads > 1.
#include <parallel/algorithm>
#include <omp.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <numeric>
#include <thread>
#include <vector>

extern "C" {

// std::thread::hardware_concurrency() of this host (recorded beside the parallel baseline)
int cpu_hardware_concurrency(void) { return static_cast<int>(std::thread::hardware_concurrency()); }

void cpu_sort_u32(uint32_t* keys, size_t n, int threads) {
  if (threads > 1) {
    omp_set_num_threads(threads);
    __gnu_parallel::sort(keys, keys + n);
  } else {
    std::sort(keys, keys + n);
  }
}

void cpu_sort_u64(uint64_t* keys, size_t n, int threads) {
  if (threads > 1) {
    omp_set_num_threads(threads);
    __gnu_parallel::sort(keys, keys + n);
  } else {
    std::sort(keys, keys + n);
  }
}

// Stable (key, u32 payload) sort: payload follows its key, ties keep input order.
void cpu_stable_sort_pairs_u32(uint32_t* keys, uint32_t* vals, size_t n, int threads) {
  std::vector<uint64_t> kv(n);
  for (size_t i = 0; i < n; ++i) kv[i] = (uint64_t(keys[i]) << 32) | uint64_t(uint32_t(i));
  // (key, input index) is unique, so an unstable sort of the packed word is the stable sort
  if (threads > 1) {
    omp_set_num_threads(threads);
    __gnu_parallel::sort(kv.begin(), kv.end());
  } else {
    std::sort(kv.begin(), kv.end());
  }
  std::vector<uint32_t> v(vals, vals + n);
  for (size_t i = 0; i < n; ++i) {
    keys[i] = uint32_t(kv[i] >> 32);
    vals[i] = v[uint32_t(kv[i])];
  }
}

}  // extern "C"
