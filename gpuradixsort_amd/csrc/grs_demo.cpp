// grs_demo.cpp — the reference's call pattern (main.cpp:117-160) on the C++ facade:
// OriginalDataSsbo(N) <- shuffled 0..N-1; ParallelSort(ssbo); Sort() twice; verify.
//
// usage: grs_demo [N] [seed]    (prints one line; exit 0 iff the output is exactly 0..N-1)
// The reference's std::random_shuffle (main.cpp:125) is replaced by a seeded Fisher-Yates
// over splitmix64 so the run is reproducible; verification strengthens the reference's
// adjacent-order check (ParallelSort.cpp:336-352) to "output == 0..N-1".
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

#include "../../include/grs_parallel_sort.hpp"

static uint64_t splitmix64(uint64_t& s) {
  uint64_t x = (s += 0x9E3779B97F4A7C15ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

int main(int argc, char** argv) {
  const unsigned n = argc > 1 ? static_cast<unsigned>(std::strtoul(argv[1], nullptr, 10)) : 1000000u;
  uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
  try {
    auto originalData = std::make_shared<OriginalDataSsbo>(n);     // main.cpp:117
    std::vector<OriginalData> demoData(n);                          // main.cpp:120-124
    for (unsigned i = 0; i < n; ++i) demoData[i]._value = i;
    for (unsigned i = n; i > 1; --i) std::swap(demoData[i - 1], demoData[splitmix64(seed) % i]);
    originalData->Upload(demoData);                                 // main.cpp:146-149

    ParallelSort parallelSort(originalData);                        // main.cpp:152
    parallelSort.SetProfiling(true);
    parallelSort.Sort();                                            // main.cpp:159-160
    parallelSort.Sort();
    grs::check_hip(hipDeviceSynchronize(), "sync");
    grs_timing t{};
    if (n > 0) t = parallelSort.LastTiming();   // N = 0 is a no-op: nothing was timed

    const std::vector<OriginalData> out = originalData->Download();
    unsigned bad = 0;
    for (unsigned i = 0; i < n; ++i) bad += out[i]._value != i;
    std::printf("grs_demo n=%u sorted=%s mismatches=%u gpu_ms=%.4f passes=%d Gkeys/s=%.2f\n", n,
                bad ? "NO" : "yes", bad, t.total_ms, t.passes,
                t.total_ms > 0 ? n / (t.total_ms * 1e-3) / 1e9 : 0.0);
    return bad ? 1 : 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "grs_demo: %s\n", e.what());
    return 2;
  }
}
