// grs_kernels.hpp — shared device helpers and the non-pass kernels of libgrs (gfx950).
//
// The reference sorts with 32 one-bit passes, each pass being four GLSL dispatches
// (Shaders/ParallelSort/GetBitForPrefixScan.comp:25-68, ParallelPrefixScan.comp:41-196,
// SortIntermediateData.comp:32-67; driven by Source/ComputeControllers/ParallelSort.cpp:236-298).
// That is 130 dispatches and ~40 B of HBM traffic per key per bit.  libgrs re-derives the
// same stable LSD sort for MI355X as:
//
//   grs_upfront_hist2  (here) one read of the keys; LDS-privatised digit histograms of EVERY
//                      pass (replaces K2 + K3a + K3b's role of counting digits)
//   grs_onesweep_v4    (grs_pass.hpp) one launch per digit: rank, publish, look-back, reorder,
//                      scatter (replaces K4's stable split and the scans feeding it)
//
// plus the boundary helpers (K1 iota, K5 record gather, key transforms, verification), the
// stand-alone scan and the segmented-sort helpers.
//
// Stability (equal keys keep input order) is what makes the multi-bit LSD produce exactly
// the reference's order: each reference pass is a stable 1-bit split
// (SortIntermediateData.comp:58-66), so the composite result is the stable sort by key.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "grs_config.h"

namespace grs {

// ----------------------------------------------------------------------------------------
// small device helpers
// ----------------------------------------------------------------------------------------

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K key, int shift, uint32_t mask) {
  return static_cast<uint32_t>(key >> shift) & mask;
}

// Digit of an LSD pass: key bits [shift, shift + bits).
template <typename K>
struct RadixDigit {
  static constexpr bool kIndexed = false;  // digit of the key alone
  int shift;
  uint32_t mask;
  __device__ __forceinline__ uint32_t operator()(K k) const { return digit_of(k, shift, mask); }
  // digit of the all-ones padding key (the largest digit this functor can return)
  __device__ __forceinline__ uint32_t max_digit() const { return mask; }
};

// Bucket of a key-range partition (multi-GPU exchange, gpuradixsort_amd/sharded.py):
// number of splitters <= key, monotone in the key; `count` <= GRS_MAX_SPLITTERS.
template <typename K>
struct SplitterDigit {
  static constexpr bool kIndexed = false;
  uint32_t count;
  K s[GRS_MAX_SPLITTERS];
  __device__ __forceinline__ uint32_t operator()(K k) const {
    uint32_t b = 0;
#pragma unroll 1
    for (uint32_t i = 0; i < count; ++i) b += s[i] <= k;
    return b;
  }
  __device__ __forceinline__ uint32_t max_digit() const { return count; }
};

// The same bucket function with the splitter count fixed at compile time (N = G - 1 for
// G = 2, 4, 8, 16 ranks): fully unrolled, no predicate, the splitters stay in SGPRs.
template <typename K, int N>
struct SplitterDigitN {
  static constexpr bool kIndexed = false;
  uint32_t count;   // == N (kept for layout compatibility with SplitterDigit)
  K s[GRS_MAX_SPLITTERS];
  __device__ __forceinline__ uint32_t operator()(K k) const {
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) b += s[i] <= k;
    return b;
  }
  __device__ __forceinline__ uint32_t max_digit() const { return N; }
};

// Bucket of a key-range partition whose splitters break ties by position: splitter b is the
// element (key kb[b], global index gb[b]) of the global input, and element (k, g) lands in
// bucket #{b : (kb[b], gb[b]) <= (k, g)} (lexicographic).  Every element is distinct in that
// order, so a run of equal keys is split across buckets like any other range (balance for
// all-equal or few-distinct inputs) while buckets stay ranges of the stable global order.
// For the shard starting at global index o, the index part becomes a shard-local threshold
// th[b] = clamp(gb[b] - o, 0, 2^32-1): (k, o + i) >= (kb, gb) <=> k > kb || (k == kb && i >= th).
// N = number of splitters (compile time; G - 1 for G ranks).  kIndexed: the pass calls
// dig(key, shard-local index).
template <typename K, int N>
struct SplitterIdxDigit {
  static constexpr bool kIndexed = true;
  uint32_t count;                 // == N
  K s[GRS_MAX_SPLITTERS];         // splitter keys, non-decreasing
  uint32_t th[GRS_MAX_SPLITTERS]; // shard-local index thresholds
  __device__ __forceinline__ uint32_t operator()(K k, uint32_t i) const {
    uint32_t b = 0;
    if constexpr (sizeof(K) == 4) {
      const uint64_t e = (static_cast<uint64_t>(k) << 32) | i;
#pragma unroll
      for (int j = 0; j < N; ++j) b += ((static_cast<uint64_t>(s[j]) << 32) | th[j]) <= e;
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) b += (s[j] < k) | ((s[j] == k) & (th[j] <= i));
    }
    return b;
  }
  __device__ __forceinline__ uint32_t max_digit() const { return N; }
};

// Number of set bits of `m` in lanes strictly below this lane.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

__device__ __forceinline__ uint32_t lane_id() { return mbcnt64(~0ull); }

// Mask of the lanes of this wave whose digit equals this lane's digit (all 64 lanes active).
// Per digit bit b: sel = splat(bit b of d) (v_bfe_i32), one ballot of it (v_cmp -> SGPR
// pair), then m &= ~(ballot ^ sel) as ONE v_bitop3_b32 per 32-bit half (LUT 0x90 over
// (m, ballot, sel)): 4 VALU per digit bit.  The empty asm pins `sel` in a VGPR so the
// compiler derives the ballot from it instead of re-shifting the digit.
template <int RB>
__device__ __forceinline__ uint64_t match_digit(uint32_t d) {
  uint32_t lo = ~0u, hi = ~0u;
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    uint32_t sel = static_cast<uint32_t>(static_cast<int32_t>(d << (31 - b)) >> 31);
    asm volatile("" : "+v"(sel));
    const uint64_t bb = __builtin_amdgcn_ballot_w64(sel != 0);
    lo = __builtin_amdgcn_bitop3_b32(lo, static_cast<uint32_t>(bb), sel, 0x90);
    hi = __builtin_amdgcn_bitop3_b32(hi, static_cast<uint32_t>(bb >> 32), sel, 0x90);
  }
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint32_t ld_status(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Inclusive wave64 scan of a u32 by DPP (row_shr 1/2/4/8, row_bcast 15/31): 6 VALU, no LDS.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// Workgroup barrier that drains LDS only: __syncthreads() also waits for every outstanding
// global load (vmcnt(0)), which would drain prefetches that are meant to stay in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Inclusive scan of one 64-bit value per lane across a wave.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < GRS_WAVE; o <<= 1) {
    const uint64_t n = __shfl_up(v, o, GRS_WAVE);
    if (lane >= static_cast<uint32_t>(o)) v += n;
  }
  return v;
}

// ----------------------------------------------------------------------------------------
// upfront histogram: counts of every digit of every pass in one read of the keys
// ----------------------------------------------------------------------------------------
//
// keys:       n keys (the unsorted input)
// g_hist:     [passes][RADIX] uint32 counters, zeroed by the caller (control-block memset)
// clear/cw:   status buffer of pass 0, zeroed here (grid-stride) so no separate memset
//             launch is needed; clear2: a second region (the MSD sort's counters).
//
// Counting always happens on 8-bit "super digits"; 4-bit passes (BASELINE C2) read their
// counts off them: pass 2q's digit is the low nibble of super digit q, pass 2q+1's the high
// nibble, so hist4[2q][d] = sum_h cnt8[q][16h + d] and hist4[2q+1][d] = sum_l cnt8[q][16d + l]
// (half the LDS atomics of counting 4-bit digits directly).
// Round 1's layout chose the 16-bit half of a counter word by the digit's low bit: 6 VALU per
// key digit and a scalar branch per digit position, and at 2^30 keys that issue, not HBM, set
// its 0.91 ms.  Here the 16-bit half is chosen by the POSITION's parity instead: super digits 2p and 2p+1 share the word
// of (pair p, digit value d), so the add value is a compile-time 1 or 0x10000 and a digit
// costs v_bfe_u32 + v_lshl_add_u32 (+ the ds_add_u32, whose pair offset is an immediate).
// Copy c of each counter sits in bank c (COPIES = 32: every 32-lane LDS group conflict-free).
// u32 keys: 64 KB per 512-thread block, 2 blocks per CU; u64 keys: 128 KB per 1024-thread
// block, 1 per CU.  A copy counts at most (BLOCK / COPIES) * VEC * ceil(n / VEC / (grid *
// BLOCK)) keys per counter, which the launch keeps below 2^16 (grid > n >> kHist2GridShift).
// FULL: the bit range is the whole key (begin_bit 0, every super digit 8 bits wide), so the
// field offsets are immediates; otherwise they are SGPR operands (one 64-bit shift more for
// u64 keys).  Super digits past the range are counted into digit 0 of their position and
// never read.  A used position shares its word with an unused one only as the low half
// (supers odd); the unused high half's overflow carries out of bit 31, so it cannot corrupt
// the used count.
// u64 keys (round 4): 32 copies too, so no 2-way bank conflicts, in 128 KB of LDS for one
// 1024-thread block per CU (was 16 copies in 64 KB, two 512-thread blocks).
template <typename K>
struct Hist2Layout {
  static constexpr int MAXQ = static_cast<int>(sizeof(K));   // super digits per key
  static constexpr int PAIRS = MAXQ / 2;
  static constexpr int COPIES = 32;
  static constexpr int WORDS = PAIRS * 256 * COPIES;           // u32 64 KB, u64 128 KB
  static constexpr int BLOCK = sizeof(K) == 4 ? 512 : 1024;    // 32 threads per copy
  static constexpr int PER_CU = sizeof(K) == 4 ? 2 : 1;        // resident blocks per CU
};
template <typename K>
constexpr int kHist2GridShift = sizeof(K) == 4 ? 20 : 19;

// QN: super digits counted (MAXQ: every pass's; fewer only in lab measurements).  Pass p's
// counts go to g_hist[p * GRS_HIST_PASS_STRIDE + d].
template <typename K, int RB, bool FULL, int QN = Hist2Layout<K>::MAXQ>
__global__ __launch_bounds__(Hist2Layout<K>::BLOCK) void grs_upfront_hist2(
    const K* __restrict__ keys, uint32_t n, int begin_bit, int end_bit, int passes,
    uint32_t* __restrict__ g_hist, uint32_t* __restrict__ clear, uint32_t clear_words,
    uint32_t* __restrict__ clear_ctrl = nullptr, uint32_t* __restrict__ clear2 = nullptr,
    uint32_t clear2_words = 0) {
  static_assert(RB == 4 || RB == 8, "4- or 8-bit digits");
  using HL = Hist2Layout<K>;
  constexpr int MAXQ = HL::MAXQ;
  static_assert(QN >= 1 && QN <= MAXQ, "super digits counted");
  constexpr int COPIES = HL::COPIES;
  constexpr uint32_t HB = HL::BLOCK;
  __shared__ __attribute__((aligned(16))) uint32_t s_hist[HL::WORDS];

  const uint32_t t = threadIdx.x;
  {
    uint4* z = reinterpret_cast<uint4*>(s_hist);
    for (uint32_t i = t; i < HL::WORDS / 4; i += HB) z[i] = make_uint4(0, 0, 0, 0);
  }
  for (uint32_t i = blockIdx.x * HB + t; i < clear_words; i += gridDim.x * HB) clear[i] = 0;
  // (the MSD sort: its byte-2 histogram and big-segment counters, grs_msd.hpp)
  for (uint32_t i = blockIdx.x * HB + t; i < clear2_words; i += gridDim.x * HB) clear2[i] = 0;
  // the next sort's control block: its histograms (every row) and its tickets
  if (clear_ctrl != nullptr) {
    constexpr uint32_t H = GRS_CTRL_HIST_WORDS, TK = GRS_MAX_PASSES * GRS_XCDS;
    for (uint32_t i = blockIdx.x * HB + t; i < H + TK; i += gridDim.x * HB) clear_ctrl[i] = 0;
  }
  __syncthreads();

  const int supers = (end_bit - begin_bit + 7) / 8;
  int shifts[MAXQ], widths[MAXQ];
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    const int s = begin_bit + q * 8;
    shifts[q] = s;
    const int w = end_bit - s;
    widths[q] = q < supers ? (w < 8 ? w : 8) : 0;
  }
  uint32_t* const base = s_hist + (t & (COPIES - 1));
  auto count = [&](K k) {
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      uint32_t d;
      if constexpr (FULL) {
        if constexpr (sizeof(K) == 4) d = __builtin_amdgcn_ubfe(static_cast<uint32_t>(k), 8 * q, 8);
        else d = __builtin_amdgcn_ubfe(static_cast<uint32_t>(k >> (q < 4 ? 0 : 32)), 8 * (q & 3), 8);
      } else {
        if constexpr (sizeof(K) == 4) d = __builtin_amdgcn_ubfe(static_cast<uint32_t>(k), shifts[q], widths[q]);
        else d = __builtin_amdgcn_ubfe(static_cast<uint32_t>(k >> shifts[q]), 0, widths[q]);
      }
      atomicAdd(base + ((q / 2) * 256 + d) * COPIES, (q & 1) ? 0x10000u : 1u);
    }
  };

  constexpr int VEC = 16 / sizeof(K);
  using V = uint4;
  const uint32_t cnt_n = n, first = blockIdx.x, nblk = gridDim.x;
  const uint32_t nvec = (reinterpret_cast<uintptr_t>(keys) & 15u) ? 0u : cnt_n / VEC;
  const V* kv = reinterpret_cast<const V*>(keys);
  const uint32_t stride = nblk * HB;
  uint32_t v = first * HB + t;
  constexpr int U = 4;   // 16-B loads in flight per thread, plus the next group's while counting
  if (v + (U - 1) * stride < nvec) {
    V cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = kv[v + u * stride];
    for (;;) {
      const uint32_t nv = v + U * stride;
      const bool more = nv + (U - 1) * stride < nvec;
      V nxt[U];
      if (more) {
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = kv[nv + u * stride];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const K* kk = reinterpret_cast<const K*>(&cur[u]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) count(kk[e]);
      }
      v = nv;
      if (!more) break;
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
  }
  for (; v < nvec; v += stride) {
    const V x = kv[v];
    const K* kk = reinterpret_cast<const K*>(&x);
#pragma unroll
    for (int e = 0; e < VEC; ++e) count(kk[e]);
  }
  for (uint64_t i = static_cast<uint64_t>(nvec) * VEC + first * HB + t; i < cnt_n; i += stride)
    count(keys[i]);   // 64-bit index: i + stride can pass 2^32 near GRS_MAX_N
  __syncthreads();

  // reduce the copies: count of super digit value d at position q (rotated start: the 32
  // lanes of a group read 32 different banks)
  auto total8 = [&](uint32_t q, uint32_t d) {
    const uint32_t* row = &s_hist[((q / 2) * 256 + d) * COPIES];
    const uint32_t sh = (q & 1u) * 16u;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < COPIES; ++k) c += (row[(k + t) & (COPIES - 1)] >> sh) & 0xFFFFu;
    return c;
  };
  if constexpr (RB == 8) {
    const uint32_t counted = static_cast<uint32_t>(min(passes, QN));
    for (uint32_t i = t; i < counted * 256; i += HB) {
      const uint32_t c = total8(i / 256, i % 256);
      if (c) atomicAdd(&g_hist[(i / 256) * GRS_HIST_PASS_STRIDE + i % 256], c);
    }
  } else {
    // 4-bit passes read their counts off the 8-bit super digits (see above)
    constexpr int R = (MAXQ * 256 + HB - 1) / HB;
    uint32_t tot[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = t + r * HB;
      tot[r] = i < static_cast<uint32_t>(supers * 256) ? total8(i / 256, i % 256) : 0u;
    }
    __syncthreads();
    uint32_t* s_red = s_hist;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = t + r * HB;
      if (i < static_cast<uint32_t>(supers * 256)) s_red[i] = tot[r];
    }
    __syncthreads();
    static_assert(RB == 8 || QN == MAXQ, "4-bit passes: every super digit counted up front");
    for (uint32_t i = t; i < static_cast<uint32_t>(passes * 16); i += HB) {
      const uint32_t p = i / 16, d = i % 16, q = p / 2;
      const uint32_t* r8 = &s_red[q * 256];
      uint32_t c = 0;
#pragma unroll
      for (int h = 0; h < 16; ++h) c += (p & 1u) ? r8[d * 16 + h] : r8[h * 16 + d];
      if (c) atomicAdd(&g_hist[p * GRS_HIST_PASS_STRIDE + d], c);
    }
  }
}

// Per-digit totals of a finished pass from its look-back status: every tile added its count to
// its group's accumulator ((arrivals << 24) | sum), so a digit's total is the sum over groups.
// One block of 256 threads: digit d (radix <= 16: the partition's buckets) summed by 16 threads
// over every 16th group, then added up in LDS.
__global__ __launch_bounds__(256) void grs_lb_totals(const uint32_t* __restrict__ gacc, uint32_t groups,
                                                     uint32_t radix, uint32_t count,
                                                     uint32_t* __restrict__ totals) {
  __shared__ uint32_t part[256];
  const uint32_t d = threadIdx.x & 15u, q = threadIdx.x >> 4;
  uint32_t sum = 0;
  if (d < count)
    for (uint32_t g = q; g < groups; g += 16) sum += gacc[static_cast<size_t>(g) * radix + d] & 0xFFFFFFu;
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x < count) {
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) tot += part[k * 16 + threadIdx.x];
    totals[threadIdx.x] = tot;
  }
}

// The LSD sort's pass plan (one wave, after the upfront histogram): pass p is TRIVIAL when one
// digit holds all n keys -- its stable scatter is the identity (the reference's own input,
// 0..N-1 shuffled, has log2 N varying bits: at N = 2^24 the 4-bit passes 6 and 7 see one
// digit).  plan[p] = 0 run the pass, 1 copy the keys through unchanged, 2 skip it: a maximal run
// of trivial passes of even length is skipped (every pass flips the buffers, so the data ends
// where it would have), one of odd length copies once and skips the rest.  The number of
// buffer flips keeps its parity, so the host's copy-back decision stands.
enum PassPlan : uint32_t { kPassRun = 0, kPassCopy = 1, kPassSkip = 2 };
__global__ __launch_bounds__(64) void grs_pass_plan(const uint32_t* __restrict__ hist, uint32_t radix,
                                                    int passes, uint32_t n, uint32_t* __restrict__ plan) {
  const uint32_t lane = threadIdx.x;
  uint32_t trivial = 0;   // bit p: pass p sees one digit
  for (int p = 0; p < passes; ++p) {
    bool one = false;
    for (uint32_t d = lane; d < radix; d += 64) one |= hist[p * GRS_HIST_PASS_STRIDE + d] == n;
    if (__ballot(one) != 0ull) trivial |= 1u << p;
  }
  if (lane == 0) {
    for (int p = 0; p < passes;) {
      if (!((trivial >> p) & 1u)) {
        plan[p++] = kPassRun;
        continue;
      }
      int e = p;
      while (e < passes && ((trivial >> e) & 1u)) ++e;
      for (int q = p; q < e; ++q) plan[q] = ((e - p) & 1) && q == p ? kPassCopy : kPassSkip;
      p = e;
    }
  }
}

// Control block and look-back status of a region-mode partition pass, in one launch instead of
// three memsets: ctrl[0, ctrl_words) = 0 (digit counts, tickets), then the count + 1 digit
// "counts" = region (the pass's digit-start scan yields b * region), status[0, words) = 0.
__global__ __launch_bounds__(256) void grs_part_init(uint32_t* __restrict__ ctrl, uint32_t ctrl_words,
                                                     uint32_t region, uint32_t count,
                                                     uint32_t* __restrict__ status, uint32_t words) {
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < ctrl_words; i += stride)
    ctrl[i] = i < count ? region : 0u;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < words; i += stride) status[i] = 0;
}

// Digit of key k at shard-local index i, for plain and indexed digit functors.
template <typename DigitF, typename K>
__device__ __forceinline__ uint32_t digit_call(const DigitF& dig, K k, uint32_t i) {
  if constexpr (DigitF::kIndexed) return dig(k, i);
  else return dig(k);
}

// Histogram of one digit functor (the bucket sizes of a key-range partition).  At most 16
// buckets, so one counter per bucket would take 64 same-address lanes per wave-instruction
// (serialised): lane l adds into its own copy, s_hist[bucket][l] — bank (64·bucket + l) mod
// 32 differs across each 32-lane group, so every add is conflict-free.  dig_dev: when not
// null, the functor is read from device memory (splitters computed on the device).
template <typename K, typename DigitF>
__global__ __launch_bounds__(GRS_HIST_BLOCK) void grs_digit_hist(
    const K* __restrict__ keys, uint32_t n, const DigitF dig, const DigitF* __restrict__ dig_dev,
    uint32_t* __restrict__ g_hist, uint32_t* __restrict__ clear, uint32_t clear_words) {
  constexpr int NB = GRS_MAX_SPLITTERS + 1;
  __shared__ uint32_t s_hist[NB * GRS_WAVE];
  const DigitF dg = dig_dev != nullptr ? *dig_dev : dig;
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  for (uint32_t i = t; i < static_cast<uint32_t>(NB * GRS_WAVE); i += GRS_HIST_BLOCK) s_hist[i] = 0;
  for (uint32_t i = blockIdx.x * GRS_HIST_BLOCK + t; i < clear_words; i += gridDim.x * GRS_HIST_BLOCK)
    clear[i] = 0;
  __syncthreads();
  auto count = [&](K k, uint32_t i) { atomicAdd(&s_hist[digit_call(dg, k, i) * GRS_WAVE + lane], 1u); };
  // 16-B loads, U in flight per thread (a scalar 4-B load per key left the partition's
  // histogram latency-bound); the ragged tail and unaligned bases take scalar loads
  constexpr int VEC = 16 / sizeof(K);
  constexpr int U = 4;
  const uint32_t nvec = (reinterpret_cast<uintptr_t>(keys) & 15u) ? 0u : n / VEC;
  const uint4* kv = reinterpret_cast<const uint4*>(keys);
  const uint32_t stride = gridDim.x * GRS_HIST_BLOCK;
  uint32_t v = blockIdx.x * GRS_HIST_BLOCK + t;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = kv[v + u * stride];
    // all U issued before the first count (the scheduler otherwise pairs each load with its wait)
#pragma unroll
    for (int u = 0; u < U; ++u) asm volatile("" ::"v"(x[u].x), "v"(x[u].y), "v"(x[u].z), "v"(x[u].w));
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const K* kk = reinterpret_cast<const K*>(&x[u]);
#pragma unroll
      for (int e = 0; e < VEC; ++e) count(kk[e], (v + u * stride) * VEC + e);
    }
  }
  for (; v < nvec; v += stride) {
    const uint4 x = kv[v];
    const K* kk = reinterpret_cast<const K*>(&x);
#pragma unroll
    for (int e = 0; e < VEC; ++e) count(kk[e], v * VEC + e);
  }
  for (uint64_t i = static_cast<uint64_t>(nvec) * VEC + blockIdx.x * GRS_HIST_BLOCK + t; i < n;
       i += stride)
    count(keys[i], static_cast<uint32_t>(i));   // 64-bit index: no wrap near GRS_MAX_N
  __syncthreads();
  if (t < static_cast<uint32_t>(NB)) {
    uint32_t c = 0;
    for (int l = 0; l < GRS_WAVE; ++l) c += s_hist[t * GRS_WAVE + ((l + t) & (GRS_WAVE - 1))];
    if (c) atomicAdd(&g_hist[t], c);
  }
}

// ----------------------------------------------------------------------------------------
// auxiliary kernels (boundary helpers; not on the timed hot path)
// ----------------------------------------------------------------------------------------

// splitmix64 (Steele, Lea, Flood 2014) — the synthetic key generator of SURVEY §8(d):
// key[i] = splitmix64(seed ^ (first_index + i)), truncated to the key width.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <typename K>
__global__ void grs_fill_splitmix(K* __restrict__ out, uint64_t n, uint64_t seed, uint64_t first) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = static_cast<K>(splitmix64(seed ^ (first + i)));
}

// The reference's own input: 0..N-1 shuffled (main.cpp:119-125).  pi = a seeded bijection of
// [0, total): four rounds of x -> ((x * a_r + c_r) mod 2^b) ^ (that >> (b/2 + 1)) on b-bit
// values (a_r odd: each step is invertible mod 2^b), walked along its cycle until the value is
// below total (cycle walking keeps it a bijection of [0, total)).
struct PermParams {
  uint64_t a[4], c[4], mask;
  int half;
};
__host__ __device__ __forceinline__ uint64_t perm_b(uint64_t x, const PermParams& p) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    x = (x * p.a[r] + p.c[r]) & p.mask;
    x ^= x >> p.half;
  }
  return x;
}
template <typename K>
__global__ void grs_fill_permutation(K* __restrict__ out, uint64_t n, uint64_t total, uint64_t first,
                                     PermParams p) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint64_t x = perm_b(first + i, p);
    while (x >= total) x = perm_b(x, p);
    out[i] = static_cast<K>(x);
  }
}

__global__ void grs_iota_u32(uint32_t* __restrict__ out, uint64_t n, uint32_t start) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = start + static_cast<uint32_t>(i);
}

// Contiguous copy with the pass's access width (one dword per lane per instruction, 256 B per
// wave-instruction): the known-byte calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for
// bench.py's traffic figure.
__global__ void grs_copy_u32(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                             uint64_t n) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

// K5 generalised (SortOriginalData.comp:27-51): dst[i] = src[min(idx[i], idx_max)] for records
// of `rb` bytes.  Records that are a multiple of 4 bytes move as dwords.  idx_max: the records
// sort passes n - 1, so indices left unwritten by a sort that timed out never read past the
// records; the public gather passes 0xFFFFFFFF (the caller's indices, unchecked).
__global__ void grs_gather_records(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                   const uint32_t* __restrict__ idx, uint64_t n, uint32_t rb,
                                   uint32_t idx_max) {
  const uint64_t total = n * rb;
  if ((rb & 3u) == 0) {
    const uint32_t wpr = rb >> 2;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < n * wpr;
         e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
      const uint64_t r = e / wpr, c = e - r * wpr;
      d[e] = s[static_cast<uint64_t>(min(idx[r], idx_max)) * wpr + c];
    }
  } else {
    for (uint64_t e = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; e < total;
         e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
      const uint64_t r = e / rb, c = e - r * rb;
      dst[e] = src[static_cast<uint64_t>(min(idx[r], idx_max)) * rb + c];
    }
  }
}

// Order-preserving key transforms (the reference supports unsigned keys
// only, ReadMeRadixSort.txt:71-80).  kind 1 = two's-complement signed: flip the sign bit;
// kind 2 = IEEE-754 float: negative values flip every bit, others only the sign bit, so
// -NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN as unsigned integers.  `inverse` undoes it.
template <typename K>
__global__ void grs_key_transform(K* __restrict__ keys, uint64_t n, int kind, int inverse) {
  constexpr K SIGN = static_cast<K>(1) << (8 * sizeof(K) - 1);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const K x = keys[i];
    K y;
    if (kind == 1) {
      y = x ^ SIGN;
    } else if (!inverse) {
      y = (x & SIGN) ? static_cast<K>(~x) : static_cast<K>(x | SIGN);
    } else {
      y = (x & SIGN) ? static_cast<K>(x & ~SIGN) : static_cast<K>(~x);
    }
    keys[i] = y;
  }
}

// Key-extraction pre-pass of grs_sort_records (the reference's K1,
// OriginalDataToIntermediateData.comp:24-52, generalised): key[i] from record i, idx[i] = i.
// Spreads the low 10 (u32) / 21 (u64) bits of v to every third bit.
template <typename K>
__host__ __device__ __forceinline__ K morton_spread(K v) {
  if constexpr (sizeof(K) == 4) {
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
  } else {
    v &= 0x1FFFFFull;
    v = (v | (v << 32)) & 0x001F00000000FFFFull;
    v = (v | (v << 16)) & 0x001F0000FF0000FFull;
    v = (v | (v << 8)) & 0x100F00F00F00F00Full;
    v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
    v = (v | (v << 2)) & 0x1249249249249249ull;
  }
  return v;
}

// Axis value -> cell in [0, 2^B): floor((v - lo) / (hi - lo) * 2^B), clamped; NaN -> 0.
template <int B>
__host__ __device__ __forceinline__ uint32_t morton_cell(float v, float lo, float hi) {
  const float t = (v - lo) / (hi - lo);
  if (!(t > 0.0f)) return 0u;                       // also NaN and hi <= lo
  if (t >= 1.0f) return (1u << B) - 1u;
  const uint32_t q = static_cast<uint32_t>(t * static_cast<float>(1u << B));
  return q < (1u << B) ? q : (1u << B) - 1u;
}

struct KeyExtract {   // device copy of grs_key_extract
  int kind;
  uint32_t offset;
  int transform;
  float lo[3], hi[3];
};

template <typename T>
__device__ __forceinline__ T load_unaligned(const uint8_t* p) {
  T v;
  __builtin_memcpy(&v, p, sizeof(T));
  return v;
}

template <typename K>
__global__ void grs_extract_keys(const uint8_t* __restrict__ rec, uint64_t n, uint32_t rb,
                                 const KeyExtract kx, K* __restrict__ keys,
                                 uint32_t* __restrict__ idx) {
  constexpr int B = sizeof(K) == 4 ? 10 : 21;
  constexpr K SIGN = static_cast<K>(1) << (8 * sizeof(K) - 1);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint8_t* p = rec + i * rb + kx.offset;
    K k;
    if (kx.kind == 0) {
      k = load_unaligned<K>(p);
      if (kx.transform == 1) k ^= SIGN;
      else if (kx.transform == 2) k = (k & SIGN) ? static_cast<K>(~k) : static_cast<K>(k | SIGN);
    } else {
      const K x = morton_cell<B>(load_unaligned<float>(p), kx.lo[0], kx.hi[0]);
      const K y = morton_cell<B>(load_unaligned<float>(p + 4), kx.lo[1], kx.hi[1]);
      const K z = morton_cell<B>(load_unaligned<float>(p + 8), kx.lo[2], kx.hi[2]);
      k = (morton_spread<K>(x) << 2) | (morton_spread<K>(y) << 1) | morton_spread<K>(z);
    }
    keys[i] = k;
    idx[i] = static_cast<uint32_t>(i);
  }
}

// ----------------------------------------------------------------------------------------
// stand-alone device-wide exclusive scan of uint32 (the reference's K3a + K3b,
// ParallelPrefixScan.comp:41-196).  The reference scans 1024-item groups with a Blelloch tree
// in shared memory (K3a), then the <= 1024 group totals in one work group (K3b); sums wrap
// mod 2^32.  Here: one launch.
// ----------------------------------------------------------------------------------------
//
// Single-pass scan (decoupled look-back): one read and one write of the items, 8 B/item.
// A workgroup takes a ticket (tiles start in id order: a tile only waits on started tiles);
// each wave scans its own contiguous 4K items row by row (a row = 64 lanes x 4 consecutive
// items, one 16-byte load per lane: 1 KB per wave-instruction), a DPP wave scan per row plus the
// running row carry, and keeps the prefixes in registers.  The tile's sum is published as
// (AGG, sum) in one 64-bit status word, wave 0 looks back (scan_lookback), publishes
// (INC, prefix + sum), and every wave adds its offset and stores.  Flag and value travel in one
// word, so no ordering between two stores is needed.  Sums wrap mod 2^32.  In place (in == out)
// is allowed: a tile writes only its own range, after reading it.  Scratch (ctl): [0] error
// word, [1] ticket, [2..3] pad, then one 64-bit status word per tile, all zero at the call.
// Measured at 2^28 (tools/ab_scan.py): 0.445 ms with 32 rows per wave (32K-item tiles), 0.48
// with 16; an LDS-transposed variant 0.513; the previous reduce-then-scan (three launches, 12 B
// of traffic per item) 0.61.
__device__ __forceinline__ unsigned long long ld_status64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define GRS_SCAN_OP_BLOCK 256

// One wave's look-back over 64 predecessors per round (lane l reads tile j - l): the nearest
// published inclusive prefix plus every sum after it, or 64 sums and the next 64.  Returns the
// exclusive prefix of `tile` (underestimated after a timeout, which sets ctl[0]).  (A window
// of 4 x 64 per round measured 0.74 against 0.48 ms at 2^28: the steady state finds an
// inclusive prefix a few tiles back, and the wider rounds only add latency; tools/ab_scan.py.)
__device__ __forceinline__ uint32_t scan_lookback(const unsigned long long* status, uint32_t tile,
                                                  uint32_t lane, uint32_t* ctl, uint32_t* err2) {
  constexpr unsigned long long INC = 2ull << 32;
  int32_t j = static_cast<int32_t>(tile) - 1;   // newest predecessor not yet summed
  uint32_t excl = 0, spins = 0;
  for (;;) {
    const int32_t idx = j - static_cast<int32_t>(lane);
    const unsigned long long sw = idx >= 0 ? ld_status64(status + idx) : INC;   // before tile 0: 0
    const uint32_t flag = static_cast<uint32_t>(sw >> 32), val = static_cast<uint32_t>(sw);
    const uint64_t incm = __builtin_amdgcn_ballot_w64(flag == 2u);
    const uint64_t zm = __builtin_amdgcn_ballot_w64(flag == 0u);
    // lanes 0..first (nearest inclusive, or the whole window) must all be published
    const uint32_t first = incm ? static_cast<uint32_t>(__builtin_ctzll(incm)) : GRS_WAVE - 1;
    const uint64_t upto = first == GRS_WAVE - 1 ? ~0ull : (2ull << first) - 1ull;
    if ((zm & upto) == 0) {
      uint32_t v = lane <= first ? val : 0u;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, GRS_WAVE);
      excl += v;
      if (incm) return excl;
      j -= GRS_WAVE;
      continue;
    }
    if (++spins > static_cast<uint32_t>(GRS_SPIN_LIMIT)) {   // prefix underestimated
      if (lane == 0) {
        atomicOr(ctl, 1u);
        if (err2 != nullptr) atomicOr(err2, 1u);   // an internal caller's sorter error word
      }
      return excl;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

template <int R>
__global__ __launch_bounds__(GRS_SCAN_OP_BLOCK) void grs_scan_onepass(
    const uint32_t* in, uint32_t* out, uint32_t n,   // may alias (in place)
    uint32_t* __restrict__ ctl, uint32_t* __restrict__ total, uint32_t* __restrict__ err2) {
  constexpr int B = GRS_SCAN_OP_BLOCK, W = B / GRS_WAVE;
  constexpr uint32_t ROW = 4 * GRS_WAVE, CHUNK = R * ROW, TILE = W * CHUNK;
  constexpr unsigned long long AGG = 1ull << 32, INC = 2ull << 32;
  __shared__ uint32_t s_wsum[W];
  __shared__ uint32_t s_tk, s_prefix;
  unsigned long long* const status = reinterpret_cast<unsigned long long*>(ctl + 4);
  const uint32_t t = threadIdx.x, lane = t & (GRS_WAVE - 1), w = t >> 6;
  if (t == 0) s_tk = atomicAdd(ctl + 1, 1u);
  __syncthreads();
  const uint32_t tile = __builtin_amdgcn_readfirstlane(s_tk);
  // (n + TILE - 1) / TILE would wrap for n > 2^32 - TILE, and GRS_SCAN_MAX_N is above that
  const uint32_t tiles = n / TILE + (n % TILE != 0u ? 1u : 0u);
  const uint32_t base = tile * TILE;
  const uint32_t valid = n - base;   // tile-local bound (base + TILE may pass 2^32)
  const uint32_t wbase = w * CHUNK;  // this wave's first item, tile-local
  uint4 q[R];
  if (valid >= TILE) {
    const uint4* v = reinterpret_cast<const uint4*>(in + base + wbase);
#pragma unroll
    for (int r = 0; r < R; ++r) q[r] = v[r * GRS_WAVE + lane];
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = wbase + r * ROW + 4 * lane;
      const uint32_t* p = in + base + i;
      q[r].x = i < valid ? p[0] : 0u;
      q[r].y = i + 1 < valid ? p[1] : 0u;
      q[r].z = i + 2 < valid ? p[2] : 0u;
      q[r].w = i + 3 < valid ? p[3] : 0u;
    }
  }
  // rows -> exclusive prefixes within the wave's chunk, in place
  uint32_t carry = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t a = q[r].x, b = a + q[r].y, c = b + q[r].z, d = c + q[r].w;
    const uint32_t incl = wave_scan_dpp(d);
    const uint32_t e = carry + incl - d;
    q[r] = make_uint4(e, e + a, e + b, e + c);
    carry += __builtin_amdgcn_readlane(incl, GRS_WAVE - 1);
  }
  if (lane == 0) s_wsum[w] = carry;
  __syncthreads();
  uint32_t agg = 0, wpre = 0;
#pragma unroll
  for (int ww = 0; ww < W; ++ww) {
    const uint32_t ws = s_wsum[ww];
    wpre += static_cast<uint32_t>(ww) < w ? ws : 0u;
    agg += ws;
  }
  if (w == 0) {
    uint32_t excl = 0;
    if (tile == 0) {
      if (lane == 0) st_status64(status, INC | agg);
    } else {
      if (lane == 0) st_status64(status + tile, AGG | agg);
      excl = scan_lookback(status, tile, lane, ctl, err2);
      if (lane == 0) st_status64(status + tile, INC | static_cast<unsigned long long>(excl + agg));
    }
    if (lane == 0) {
      s_prefix = excl;
      if (tile == tiles - 1 && total != nullptr) *total = excl + agg;
    }
  }
  __syncthreads();
  const uint32_t off = s_prefix + wpre;
  if (valid >= TILE) {
    uint4* v = reinterpret_cast<uint4*>(out + base + wbase);
#pragma unroll
    for (int r = 0; r < R; ++r)
      v[r * GRS_WAVE + lane] = make_uint4(q[r].x + off, q[r].y + off, q[r].z + off, q[r].w + off);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = wbase + r * ROW + 4 * lane;
      uint32_t* p = out + base + i;
      if (i < valid) p[0] = q[r].x + off;
      if (i + 1 < valid) p[1] = q[r].y + off;
      if (i + 2 < valid) p[2] = q[r].z + off;
      if (i + 3 < valid) p[3] = q[r].w + off;
    }
  }
}

// Segmented sort of short segments: one workgroup per segment sorts it
// in LDS -- one read and one write of the keys (and payload) instead of the two radix sorts
// and the gather of the general path.  A bitonic network over (key, position in the segment),
// so equal keys keep their input order; the payload follows through the position.  Segments
// of at most GRS_SEG_SMALL_MAX items (the host checks the longest first).
#define GRS_SEG_SMALL_MAX 4096
#define GRS_SEG_SMALL_BLOCK 256

// The longest segment's length -> *out (atomicMax; *out zeroed by the caller).
__global__ void grs_segment_maxlen(const uint32_t* __restrict__ offsets, uint32_t nseg,
                                   uint32_t* __restrict__ out) {
  uint32_t m = 0;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x)
    m = max(m, offsets[s + 1] - offsets[s]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(m, o, GRS_WAVE)));
  if ((threadIdx.x & (GRS_WAVE - 1)) == 0 && m != 0) atomicMax(out, m);
}

// SMAX: a power of two >= the longest segment, chosen by the host (shorter bounds leave room
// for more workgroups per CU).  Thread t holds positions t*E .. t*E + E - 1 (E = SMAX / 256) in
// registers; a compare-exchange at distance j runs in registers (j < E), across the wave by
// lane shuffles (j < 64 E), and through LDS with one barrier only beyond that (3 of 55 stages
// at 1024 items).  Padding positions hold the largest (key, position) and sort last.
template <typename K, uint32_t SMAX>
__global__ __launch_bounds__(GRS_SEG_SMALL_BLOCK) void grs_segment_bitonic(
    K* __restrict__ keys, uint32_t* __restrict__ vals, const uint32_t* __restrict__ offsets) {
  constexpr uint32_t B = GRS_SEG_SMALL_BLOCK;
  static_assert(SMAX <= GRS_SEG_SMALL_MAX && SMAX >= 2 * B && (SMAX & (SMAX - 1)) == 0,
                "power-of-two bound of at least two items per thread");
  constexpr uint32_t E = SMAX / B;
  constexpr bool U64 = sizeof(K) == 8;
  __shared__ uint64_t xk[2][SMAX];                       // cross-wave exchange, double-buffered
  __shared__ uint32_t xi[U64 ? 2 : 1][U64 ? SMAX : 1];   // u64 keys: their positions
  __shared__ uint32_t sv[SMAX];                          // the payload, by input position
  const uint32_t t = threadIdx.x;
  const uint32_t lo = offsets[blockIdx.x];
  const uint32_t len = offsets[blockIdx.x + 1] - lo;
  if (len <= 1 || len > SMAX) return;   // (longer segments never reach this kernel)
  uint32_t p = 2;
  while (p < len) p <<= 1;
  // u32 keys: x = (key << 32) | position (one 64-bit order); u64 keys: x = key, ix = position
  uint64_t x[E];
  uint32_t ix[E];
#pragma unroll
  for (uint32_t e = 0; e < E; ++e) {
    const uint32_t a = t * E + e;
    if (a < len) {
      const K kk = keys[lo + a];
      x[e] = U64 ? static_cast<uint64_t>(kk) : (static_cast<uint64_t>(kk) << 32) | a;
      ix[e] = a;
      if (vals != nullptr) sv[a] = vals[lo + a];
    } else {
      x[e] = ~0ull;
      ix[e] = ~0u;
    }
  }
  // (x, ix) > (y, iy) in the sort order
  auto greater = [](uint64_t xa, uint32_t ia, uint64_t xb, uint32_t ib) {
    if constexpr (U64) return xa > xb || (xa == xb && ia > ib);
    else return xa > xb;
  };
  uint32_t buf = 0;
  for (uint32_t k = 2; k <= p; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j < E) {   // both positions in this thread's registers
#pragma unroll
        for (uint32_t e = 0; e < E; ++e) {
          const uint32_t f = e | j;
          if ((e & j) == 0 && f < E) {
            const bool up = ((t * E + e) & k) == 0;
            if (greater(x[e], ix[e], x[f], ix[f]) == up) {
              const uint64_t tx = x[e];
              x[e] = x[f];
              x[f] = tx;
              const uint32_t ti = ix[e];
              ix[e] = ix[f];
              ix[f] = ti;
            }
          }
        }
      } else {
        uint64_t y[E];
        uint32_t iy[E];
        if (j < GRS_WAVE * E) {   // the partner is lane (lane ^ j / E) of this wave
          const int m = static_cast<int>(j / E);
#pragma unroll
          for (uint32_t e = 0; e < E; ++e) {
            const uint32_t ylo = __shfl_xor(static_cast<uint32_t>(x[e]), m, GRS_WAVE);
            const uint32_t yhi = __shfl_xor(static_cast<uint32_t>(x[e] >> 32), m, GRS_WAVE);
            y[e] = (static_cast<uint64_t>(yhi) << 32) | ylo;
            iy[e] = U64 ? static_cast<uint32_t>(__shfl_xor(ix[e], m, GRS_WAVE)) : 0u;
          }
        } else {   // another wave's: through LDS
#pragma unroll
          for (uint32_t e = 0; e < E; ++e) {
            xk[buf][t * E + e] = x[e];
            if constexpr (U64) xi[buf][t * E + e] = ix[e];
          }
          __syncthreads();
#pragma unroll
          for (uint32_t e = 0; e < E; ++e) {
            y[e] = xk[buf][(t * E + e) ^ j];
            if constexpr (U64) iy[e] = xi[buf][(t * E + e) ^ j];
            else iy[e] = 0u;
          }
          buf ^= 1u;   // the next LDS stage writes the other buffer (a barrier lies between)
        }
#pragma unroll
        for (uint32_t e = 0; e < E; ++e) {
          const uint32_t a = t * E + e;
          const bool up = (a & k) == 0, lower = (a & j) == 0;
          // the lower position of an ascending pair keeps the smaller item, and so on
          if (greater(x[e], ix[e], y[e], iy[e]) == (lower == up)) {
            x[e] = y[e];
            ix[e] = iy[e];
          }
        }
      }
    }
  }
  __syncthreads();   // the payload rows (sv) are read across threads below
#pragma unroll
  for (uint32_t e = 0; e < E; ++e) {
    const uint32_t a = t * E + e;
    if (a < len) {
      if constexpr (U64) {
        keys[lo + a] = static_cast<K>(x[e]);
        if (vals != nullptr) vals[lo + a] = sv[ix[e]];
      } else {
        keys[lo + a] = static_cast<K>(x[e] >> 32);
        if (vals != nullptr) vals[lo + a] = sv[static_cast<uint32_t>(x[e])];
      }
    }
  }
}

// The same short segments by a block LSD radix sort in LDS (the default; the bitonic kernel
// above is the fallback when the device probe of the lane-ordered LDS atomics fails, §6.3):
// 8-bit digits, sizeof(K) passes.  Items are held wave-striped (item j of lane l of wave w is
// segment position w * 64 * I + j * 64 + l, I = SMAX / BLOCK), so the returning LDS add on the
// wave's digit counter ranks them stably, as the sort pass does; per pass one add, one scan of
// the W x 256 counters and one scatter of keys (and payload) through LDS.  BLOCK 256 up to
// 4096 items, 1024 threads beyond (u32 keys to 16384, u64 keys to 8192: the LDS holds the
// keys, the payload and 16 x 256 counters).
#define GRS_SEG_RADIX_MAX32 16384
#define GRS_SEG_RADIX_MAX64 8192
template <typename K, uint32_t SMAX, uint32_t BLOCK>
__global__ __launch_bounds__(BLOCK) void grs_segment_radix(
    K* __restrict__ keys, uint32_t* __restrict__ vals, const uint32_t* __restrict__ offsets) {
  constexpr uint32_t W = BLOCK / GRS_WAVE, I = SMAX / BLOCK;
  static_assert((BLOCK == 256 || BLOCK == 1024) && I >= 2 && (SMAX & (SMAX - 1)) == 0,
                "256 or 1024 threads, a power-of-two bound of at least two items per thread");
  static_assert(SMAX <= (sizeof(K) == 4 ? GRS_SEG_RADIX_MAX32 : GRS_SEG_RADIX_MAX64), "LDS");
  __shared__ K sk[SMAX];
  __shared__ uint32_t sv[SMAX];
  __shared__ uint32_t cnt[W * 256];
  __shared__ uint32_t wtot[4];
  const uint32_t t = threadIdx.x, lane = t & (GRS_WAVE - 1), w = t >> 6;
  const uint32_t lo = offsets[blockIdx.x];
  const uint32_t len = offsets[blockIdx.x + 1] - lo;
  if (len <= 1 || len > SMAX) return;   // (longer segments never reach this kernel)
  const bool pay = vals != nullptr;
  K k[I];
  uint32_t v[I];
#pragma unroll
  for (uint32_t j = 0; j < I; ++j) {
    const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
    k[j] = i < len ? keys[lo + i] : K(0);
    v[j] = pay && i < len ? vals[lo + i] : 0u;
  }
  for (int pass = 0; pass < static_cast<int>(sizeof(K)); ++pass) {
    const int shift = 8 * pass;
    for (uint32_t c = t; c < W * 256; c += BLOCK) cnt[c] = 0;
    __syncthreads();
    uint32_t r[I];
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
      const uint32_t d = static_cast<uint32_t>(k[j] >> shift) & 255u;
      r[j] = i < len ? atomicAdd(&cnt[w * 256 + d], 1u) : 0u;
    }
    __syncthreads();
    // threads 0..255, one per digit: wave offsets, then the digit's start over all digits
    uint32_t c[W], tot = 0, incl = 0;
    if (t < 256) {
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        c[ww] = cnt[ww * 256 + t];
        tot += c[ww];
      }
      incl = wave_scan_dpp(tot);
      if (lane == GRS_WAVE - 1) wtot[w] = incl;
    }
    __syncthreads();
    if (t < 256) {
      uint32_t base = incl - tot;
#pragma unroll
      for (uint32_t ww = 0; ww < 4; ++ww) base += ww < w ? wtot[ww] : 0u;
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        cnt[ww * 256 + t] = base;
        base += c[ww];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
      if (i < len) {
        const uint32_t d = static_cast<uint32_t>(k[j] >> shift) & 255u;
        const uint32_t dst = cnt[w * 256 + d] + r[j];
        sk[dst] = k[j];
        if (pay) sv[dst] = v[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
      if (i < len) {
        k[j] = sk[i];
        if (pay) v[j] = sv[i];
      }
    }
    // (the next pass's counter reset and scatter are behind its first barrier)
  }
#pragma unroll
  for (uint32_t j = 0; j < I; ++j) {
    const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
    if (i < len) {
      keys[lo + i] = k[j];
      if (pay) vals[lo + i] = v[j];
    }
  }
}

// Segmented sort helpers.  After a stable sort of the keys carrying
// their input index perm[j], segk[j] = the segment of input element perm[j]: the largest s
// in [0, nseg) with offsets[s] <= perm[j] (offsets: nseg + 1 non-decreasing device words,
// offsets[0] = 0, offsets[nseg] = n).
template <typename K>
__global__ void grs_segment_ids(const uint32_t* __restrict__ perm,
                                const uint32_t* __restrict__ offsets, uint32_t nseg,
                                K* __restrict__ segk, uint64_t n) {
  for (uint64_t j = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; j < n;
       j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t x = perm[j];
    uint32_t lo = 0, hi = nseg;   // invariant: offsets[lo] <= x (offsets[0] = 0), answer < hi
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (offsets[mid] <= x) lo = mid; else hi = mid;
    }
    segk[j] = static_cast<K>(lo);
  }
}

// out_keys[j] = keys[pos[j]]; out_vals[j] = vals[perm[pos[j]]] (vals may be null).  Both
// indices are clamped to n - 1: after a sort that timed out they may be stale words.
template <typename K>
__global__ void grs_segment_gather(const K* __restrict__ keys, K* __restrict__ out_keys,
                                   const uint32_t* __restrict__ pos,
                                   const uint32_t* __restrict__ perm,
                                   const uint32_t* __restrict__ vals,
                                   uint32_t* __restrict__ out_vals, uint64_t n) {
  for (uint64_t j = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; j < n;
       j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t last = static_cast<uint32_t>(n - 1);
    const uint32_t p = min(pos[j], last);
    out_keys[j] = keys[p];
    if (vals) out_vals[j] = vals[min(perm[p], last)];
  }
}

// Segmented sort of u32 keys without gathers: segment ids in input order by marking each
// segment start (atomic: empty segments stack on one position) and a scan, then one u64 key
// (segment << 32 | key) per item, sorted once and split back.
__global__ void grs_segment_marks(const uint32_t* __restrict__ offsets, uint32_t nseg, uint32_t n,
                                  uint32_t* __restrict__ marks) {
  for (uint32_t s = 1 + blockIdx.x * blockDim.x + threadIdx.x; s < nseg;
       s += gridDim.x * blockDim.x) {
    const uint32_t o = offsets[s];
    if (o < n) atomicAdd(&marks[o], 1u);
  }
}

__global__ void grs_segment_compose(const uint32_t* __restrict__ keys,
                                    const uint32_t* __restrict__ marks,
                                    const uint32_t* __restrict__ marks_excl,
                                    uint64_t* __restrict__ comp, uint64_t n) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    comp[i] = (static_cast<uint64_t>(marks_excl[i] + marks[i]) << 32) | keys[i];
}

__global__ void grs_segment_split(const uint64_t* __restrict__ comp, uint32_t* __restrict__ keys,
                                  uint64_t n) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    keys[i] = static_cast<uint32_t>(comp[i]);
}

// *dst |= *src, then *src = 0: an inner sorter's sticky error word (a look-back timeout) moved
// into the calling sorter's, which its checks read (grs_check_error, grs_stream_check_error).
__global__ void grs_fold_error(uint32_t* __restrict__ src, uint32_t* __restrict__ dst) {
  if (threadIdx.x == 0) {
    const uint32_t e = *src;
    if (e != 0u) {
      atomicOr(dst, e);
      *src = 0u;
    }
  }
}

// Adjacent-order check of the reference (ParallelSort.cpp:336-352), strengthened: counts
// every i with key[i] < key[i-1] (the reference skips 0xffffffff padding; we have none).
template <typename K>
__global__ void grs_count_inversions(const K* __restrict__ keys, uint64_t n,
                                     unsigned long long* __restrict__ out) {
  unsigned long long c = 0;
  for (uint64_t i = 1 + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    c += keys[i] < keys[i - 1];
  if (c) atomicAdd(out, c);
}

}  // namespace grs
