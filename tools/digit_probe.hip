// Lab probe (not part of libgrs): the VALU cost of the partition's splitter digit.  The same
// bucket histogram as grs_digit_hist (per-lane LDS copies, 16-B loads, one resident round of
// workgroups) over 2^27 u32 keys and 7 splitters, with the bucket computed three ways:
//   mode 0  (s_j, th_j) <= (k, i) as one 64-bit compare per splitter (grs::SplitterIdxDigit)
//   mode 1  the same order through a 32-bit subtract / subtract-with-borrow per splitter
//           (b = N - sum of the borrows of (k, i) - (s_j, th_j))
//   mode 2  keys only, thresholds all zero: sum of (s_j <= k), clamped to the real count
// Each mode's histogram is checked against mode 0's by the driver (tools/digit_probe.py).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int NS = 7;
constexpr int BLOCK = 256;
constexpr int NB = NS + 1;

struct Split {
  uint32_t s[NS];
  uint32_t th[NS];
  uint32_t count;
};

template <int MODE>
__device__ __forceinline__ uint32_t bucket(const Split& sp, uint32_t k, uint32_t i) {
  uint32_t b = 0;
  if constexpr (MODE == 0) {
    const uint64_t e = (static_cast<uint64_t>(k) << 32) | i;
#pragma unroll
    for (int j = 0; j < NS; ++j) b += ((static_cast<uint64_t>(sp.s[j]) << 32) | sp.th[j]) <= e;
  } else if constexpr (MODE == 1) {
    uint32_t borrows = 0;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      uint32_t lo_borrow, hi_borrow;
      const uint32_t lo = __builtin_subc(i, sp.th[j], 0u, &lo_borrow);
      (void)lo;
      const uint32_t hi = __builtin_subc(k, sp.s[j], lo_borrow, &hi_borrow);
      (void)hi;
      borrows += hi_borrow;
    }
    b = NS - borrows;
  } else {
#pragma unroll
    for (int j = 0; j < NS; ++j) b += sp.s[j] <= k;
    b = min(b, sp.count);
  }
  return b;
}

template <int MODE>
__global__ __launch_bounds__(BLOCK) void digit_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                    const Split sp, uint32_t* __restrict__ g_hist) {
  __shared__ uint32_t s_hist[NB * 64];
  const uint32_t t = threadIdx.x, lane = t & 63;
  for (uint32_t i = t; i < NB * 64; i += BLOCK) s_hist[i] = 0;
  __syncthreads();
  const uint32_t nvec = n / 4, stride = gridDim.x * BLOCK;
  const uint4* kv = reinterpret_cast<const uint4*>(keys);
  constexpr int U = 4;
  uint32_t v = blockIdx.x * BLOCK + t;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = kv[v + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t* kk = reinterpret_cast<const uint32_t*>(&x[u]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        atomicAdd(&s_hist[bucket<MODE>(sp, kk[e], (v + u * stride) * 4 + e) * 64 + lane], 1u);
    }
  }
  for (; v < nvec; v += stride) {
    const uint4 x = kv[v];
    const uint32_t* kk = reinterpret_cast<const uint32_t*>(&x);
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(&s_hist[bucket<MODE>(sp, kk[e], v * 4 + e) * 64 + lane], 1u);
  }
  for (uint32_t i = nvec * 4 + blockIdx.x * BLOCK + t; i < n; i += stride)
    atomicAdd(&s_hist[bucket<MODE>(sp, keys[i], i) * 64 + lane], 1u);
  __syncthreads();
  if (t < NB) {
    uint32_t c = 0;
    for (int l = 0; l < 64; ++l) c += s_hist[t * 64 + ((l + t) & 63)];
    if (c) atomicAdd(&g_hist[t], c);
  }
}

template <int MODE>
int launch(const uint32_t* keys, uint32_t n, const Split& sp, uint32_t* hist, int cus) {
  static const int per_cu = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, digit_hist<MODE>, BLOCK, 0) != hipSuccess || b < 1)
      b = 4;
    return b;
  }();
  const int grid = per_cu * cus;
  hipLaunchKernelGGL(digit_hist<MODE>, dim3(grid), dim3(BLOCK), 0, 0, keys, n, sp, hist);
  return hipGetLastError() == hipSuccess ? per_cu : -1;
}

}  // namespace

// splitters / thresholds: NS values each; returns blocks per CU (or -1)
extern "C" int digit_probe_run(int mode, const uint32_t* keys, uint32_t n, const uint32_t* splitters,
                               const uint32_t* thresholds, uint32_t count, uint32_t* hist, int cus) {
  Split sp{};
  for (int j = 0; j < NS; ++j) {
    sp.s[j] = splitters[j];
    sp.th[j] = thresholds[j];
  }
  sp.count = count;
  if (mode == 0) return launch<0>(keys, n, sp, hist, cus);
  if (mode == 1) return launch<1>(keys, n, sp, hist, cus);
  if (mode == 2) return launch<2>(keys, n, sp, hist, cus);
  return -1;
}
