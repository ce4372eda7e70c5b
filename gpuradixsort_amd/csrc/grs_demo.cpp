// grs_demo.cpp — the reference's call pattern (main.cpp:117-160) on the C++ facade:
// OriginalDataSsbo(N) <- shuffled 0..N-1; ParallelSort(ssbo); Sort() twice; verify.
//
// usage: grs_demo [N] [seed]    (prints one line; exit 0 iff the output is exactly 0..N-1)
//        grs_demo particles [N] [seed]
//        the reference's stated purpose (ParallelSort.h:13-31): N Particle structs sorted by the
//        Morton code of their position through ParallelSort(RecordSsbo<Particle>, MortonKey);
//        verified against a host std::stable_sort by the same code
//        grs_demo distance [N] [seed]
//        a user-defined key functor (ParallelSortBy<Particle, DistanceKey>): particles by their
//        float distance from a point, through grs::OrderedBits, verified the same way
//        grs_demo fault [N] [seed]
//        the main call pattern with the look-back fault hook set (GRS_OPT_FAULT_TILE = 0):
//        Sort() must throw grs::Error(GRS_ETIMEOUT); the demo prints it and exits 2
// The reference's std::random_shuffle (main.cpp:125) is replaced by a seeded Fisher-Yates
// over splitmix64 so the run is reproducible; verification strengthens the reference's
// adjacent-order check (ParallelSort.cpp:336-352) to "output == 0..N-1".
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>
#include <vector>

#include "../../include/grs_parallel_sort.hpp"

static uint64_t splitmix64(uint64_t& s) {
  uint64_t x = (s += 0x9E3779B97F4A7C15ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Particle {          // 28 bytes: position, velocity, id (= original index)
  float pos[3];
  float vel[3];
  unsigned int id;
};

static uint32_t spread10(uint32_t v) {
  v &= 0x3FFu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  return (v | (v << 2)) & 0x09249249u;
}
static uint32_t cell10(float v, float lo, float hi) {
  const float t = (v - lo) / (hi - lo);
  if (!(t > 0.0f)) return 0u;
  if (t >= 1.0f) return 1023u;
  const uint32_t q = static_cast<uint32_t>(t * 1024.0f);
  return q < 1024u ? q : 1023u;
}

static int particles(unsigned n, uint64_t seed) {
  const float lo[3] = {-1.0f, -1.0f, -1.0f}, hi[3] = {1.0f, 1.0f, 1.0f};
  std::vector<Particle> host(n);
  for (unsigned i = 0; i < n; ++i) {
    for (int a = 0; a < 3; ++a) {
      host[i].pos[a] = static_cast<float>(splitmix64(seed) >> 40) / 16777216.0f * 2.2f - 1.1f;
      host[i].vel[a] = static_cast<float>(a);
    }
    host[i].id = i;
  }
  auto buf = std::make_shared<RecordSsbo<Particle>>(n);
  buf->Upload(host);
  ParallelSort ps(buf, grs::MortonKey(offsetof(Particle, pos), lo, hi));
  ps.Sort();
  const std::vector<Particle> out = buf->Download();
  std::vector<uint32_t> code(n);
  for (unsigned i = 0; i < n; ++i) {
    const Particle& p = host[i];
    code[i] = (spread10(cell10(p.pos[0], lo[0], hi[0])) << 2) |
              (spread10(cell10(p.pos[1], lo[1], hi[1])) << 1) | spread10(cell10(p.pos[2], lo[2], hi[2]));
  }
  std::vector<unsigned> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::stable_sort(perm.begin(), perm.end(), [&](unsigned a, unsigned b) { return code[a] < code[b]; });
  unsigned bad = 0;
  for (unsigned i = 0; i < n; ++i)
    bad += std::memcmp(&out[i], &host[perm[i]], sizeof(Particle)) != 0;
  std::printf("grs_demo particles n=%u sorted=%s mismatches=%u\n", n, bad ? "NO" : "yes", bad);
  return bad ? 1 : 0;
}

// A user key functor: squared distance of the particle from a point, as order-preserving bits
// (ties are common: positions are quantised to 1/64, so stability is exercised).
struct DistanceKey {
  float c[3];
  __host__ __device__ uint32_t operator()(const Particle& p) const {
    float d = 0.0f;
    for (int a = 0; a < 3; ++a) {
      const float x = p.pos[a] - c[a];
      d = __builtin_fmaf(x, x, d);
    }
    return grs::OrderedBits(d);
  }
};

static int distance(unsigned n, uint64_t seed) {
  std::vector<Particle> host(n);
  for (unsigned i = 0; i < n; ++i) {
    for (int a = 0; a < 3; ++a) {
      host[i].pos[a] = static_cast<float>(static_cast<int>(splitmix64(seed) % 129) - 64) / 64.0f;
      host[i].vel[a] = -static_cast<float>(a);
    }
    host[i].id = i;
  }
  auto buf = std::make_shared<RecordSsbo<Particle>>(n);
  buf->Upload(host);
  const DistanceKey key{{0.25f, -0.5f, 0.125f}};
  ParallelSortBy<Particle, DistanceKey> ps(buf, key);
  ps.Sort();
  ps.Sort();   // sorting sorted records again must not move them (stability)
  const std::vector<Particle> out = buf->Download();
  std::vector<uint32_t> code(n);
  for (unsigned i = 0; i < n; ++i) code[i] = key(host[i]);   // the same functor on the host
  std::vector<unsigned> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::stable_sort(perm.begin(), perm.end(), [&](unsigned a, unsigned b) { return code[a] < code[b]; });
  unsigned bad = 0;
  for (unsigned i = 0; i < n; ++i)
    bad += std::memcmp(&out[i], &host[perm[i]], sizeof(Particle)) != 0;
  std::printf("grs_demo distance n=%u sorted=%s mismatches=%u\n", n, bad ? "NO" : "yes", bad);
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "distance") == 0) {
    const unsigned n = argc > 2 ? static_cast<unsigned>(std::strtoul(argv[2], nullptr, 10)) : 100000u;
    const uint64_t seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
    try {
      return distance(n, seed);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "grs_demo: %s\n", e.what());
      return 2;
    }
  }
  if (argc > 1 && std::strcmp(argv[1], "particles") == 0) {
    const unsigned n = argc > 2 ? static_cast<unsigned>(std::strtoul(argv[2], nullptr, 10)) : 100000u;
    const uint64_t seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
    try {
      return particles(n, seed);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "grs_demo: %s\n", e.what());
      return 2;
    }
  }
  const bool fault = argc > 1 && std::strcmp(argv[1], "fault") == 0;
  if (fault) {
    --argc;
    ++argv;
  }
  const unsigned n = argc > 1 ? static_cast<unsigned>(std::strtoul(argv[1], nullptr, 10)) : 1000000u;
  uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
  try {
    auto originalData = std::make_shared<OriginalDataSsbo>(n);     // main.cpp:117
    std::vector<OriginalData> demoData(n);                          // main.cpp:120-124
    for (unsigned i = 0; i < n; ++i) demoData[i]._value = i;
    for (unsigned i = n; i > 1; --i) std::swap(demoData[i - 1], demoData[splitmix64(seed) % i]);
    originalData->Upload(demoData);                                 // main.cpp:146-149

    ParallelSort parallelSort(originalData);                        // main.cpp:152
    if (fault) parallelSort.SetOption(GRS_OPT_FAULT_TILE, 0);
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
