// r1_kernels.hpp — round-1 pass kernels, kept for the lab only (tools/lab.hip): the
// ballot-match pass, the register-prefetch / LDS-DMA persistent passes, the atomic-rank pass
// with its look-back variants (LB1/LB2/LB3 with 30-bit status values) and the v3 persistent
// pass.  libgrs no longer compiles them: its pass is grs_onesweep_v4 (grs_pass.hpp).
// DESIGN.md §3 and the round-1 profiles cite their measurements.
#pragma once

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

// round-1 status word: [31:30] flag, [29:0] count (so at most 2^30-1 items per call)
#define GRS_FLAG_SHIFT 30u
#define GRS_FLAG_NOT_READY 0u
#define GRS_FLAG_AGGREGATE 1u
#define GRS_FLAG_INCLUSIVE 2u
#define GRS_VALUE_MASK 0x3FFFFFFFu

namespace grs {

// ----------------------------------------------------------------------------------------
// one LSD pass: count + publish + rank + look-back + scatter of one RB-bit digit
// ----------------------------------------------------------------------------------------
//
// Tile layout: tile T covers keys [T*TILE, (T+1)*TILE); wave w of the tile owns the
// contiguous sub-range [w*64*ITEMS, (w+1)*64*ITEMS) and loads it "wave-striped": item j of
// lane l is key (w*64*ITEMS + j*64 + l).  Every global load instruction is 64 consecutive
// keys (256 B for u32) and ranking items j = 0..ITEMS-1 in order, lanes in order, visits
// keys in input order, which is what makes the rank stable.
//
// Order of work inside a tile (the look-back latency hides behind the ranking):
//   1. ticket -> tile id; load the tile into registers
//   2. tile digit counts by LDS atomics; publish them (AGGREGATE, or INCLUSIVE for tile 0)
//   3. stable rank: per item, a ballot match mask; one leader lane per distinct digit does
//      a returning LDS atomic on the wave's counter (in program order, so items stay in
//      order without a read->write chain per item); peers read the leader's old count
//   4. look-back over predecessor tiles -> global offset of each digit; publish INCLUSIVE
//   5. reorder the tile in LDS by (digit, input order); store runs to their global slots
//
// status:      [num_tiles][RADIX] look-back words of this pass (zeroed before the launch)
// status_next: the other status buffer: this tile zeroes its own slice for the next pass
// tickets:     per-pass atomic counter; ticket order = tile order, so a tile only ever
//              waits on tiles that already started (no forward-progress assumption)
// DBG (timing ablations in tools/, never set by the library): bit 0 = no look-back (uniform-
// data estimate of the prefix instead), bit 1 = contiguous stores instead of the scatter,
// bit 2 = publish late (after ranking) instead of early.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS>
struct OnesweepSmem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  uint32_t cnt[WAVES * RADIX];  // per-wave digit counters -> local offsets
  uint32_t hist[RADIX];         // tile digit counts (early publish)
  uint32_t base[RADIX];         // global dst of tile-local index 0 of digit d
  uint64_t wsum[WAVES];         // block-scan carries
  uint32_t ticket[2];
  K keys[TILE];
  uint32_t vals[PAIRS ? TILE : 1];
};

// Exclusive prefix of digit d over tiles [0, tile): windowed decoupled look-back.  Polls
// GRS_LB_WIN predecessors at once (independent loads in flight), consumes AGGREGATEs
// nearest-first up to the first INCLUSIVE, restarts the window at the first NOT_READY.
// Tile 0 is always INCLUSIVE, so the walk ends; spins are bounded (error word).
template <int RADIX, bool STATS = false>
__device__ __forceinline__ uint32_t lookback(const uint32_t* status, uint32_t tile, uint32_t d,
                                             uint32_t* error_word) {
  uint32_t prefix = 0;
  int32_t pt = static_cast<int32_t>(tile) - 1;
  uint32_t spins = 0;
  uint32_t rounds = 0, walked = 0;
  const uint64_t t0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
  uint32_t first_rt = 0;
  while (true) {
    ++rounds;
    uint32_t v[GRS_LB_WIN];
#pragma unroll
    for (int k = 0; k < GRS_LB_WIN; ++k)
      v[k] = (pt - k >= 0) ? ld_status(status + static_cast<size_t>(pt - k) * RADIX + d)
                           : (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT);
    int consumed = 0;
    bool done = false;
    bool blocked = false;
#pragma unroll
    for (int k = 0; k < GRS_LB_WIN; ++k) {
      if (!done && !blocked) {
        const uint32_t f = v[k] >> GRS_FLAG_SHIFT;
        if (f == GRS_FLAG_NOT_READY) {
          blocked = true;
        } else {
          prefix += v[k] & GRS_VALUE_MASK;
          ++consumed;
          done = f == GRS_FLAG_INCLUSIVE;
        }
      }
    }
    if constexpr (STATS) {
      if (rounds == 1) first_rt = static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t0);
      walked += consumed;
    }
    if (done) break;
    pt -= consumed;
    if (consumed == 0) {
      if (++spins > GRS_SPIN_LIMIT) {
        atomicOr(error_word, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if constexpr (STATS) {   // lab only: per tile max rounds / spins / walk over digits, RT of digit 0
    uint32_t* st = error_word + 64 + static_cast<size_t>(tile) * 8;
    atomicMax(st + 0, rounds);
    atomicMax(st + 1, spins);
    atomicMax(st + 2, walked);
    if (d == 0) st[3] = first_rt;
  }
  return prefix;
}

// Two-level look-back.  With hundreds of tiles in flight and a poll round trip of 1-2 us
// under full HBM streaming, the INCLUSIVE frontier of a plain decoupled look-back lags
// ~100+ tiles behind the newest tile, and every tile walks that whole distance (measured:
// 115-140 predecessor words per digit, 15-30 poll rounds, half of a tile's lifetime).  So
// tiles are also grouped: group g = tiles [g*G, (g+1)*G).  Every tile adds
// (1 << 24) | its digit count into the group's accumulator word gacc[g][d] (one no-return
// atomic per digit); a word whose top byte reads G holds the complete group aggregate
// (sum < 2^24).  The walk then covers the own group tile by tile (< G words), and earlier
// groups one word each: the group's last tile if it is already INCLUSIVE, else the group
// accumulator; only a group whose accumulator is still incomplete is walked tile by tile.
// Tile words and group words are each single 32-bit values written atomically, so no
// release/acquire ordering is needed anywhere (a poll that reads an old state just polls
// again).
template <int RADIX>
__device__ __forceinline__ bool walk_tiles(const uint32_t* status, int32_t& pt, int32_t bottom,
                                           uint32_t d, uint32_t& prefix, uint32_t& spins,
                                           uint32_t* error_word, uint32_t& rounds) {
  // walks tiles pt, pt-1, ... >= bottom; true = an INCLUSIVE word ended the walk
  while (pt >= bottom) {
    ++rounds;
    uint32_t v[GRS_LB_WIN];
#pragma unroll
    for (int k = 0; k < GRS_LB_WIN; ++k)
      v[k] = (pt - k >= bottom) ? ld_status(status + static_cast<size_t>(pt - k) * RADIX + d) : 0u;
    int consumed = 0;
    bool done = false, blocked = false;
#pragma unroll
    for (int k = 0; k < GRS_LB_WIN; ++k) {
      if (!done && !blocked && pt - k >= bottom) {
        const uint32_t f = v[k] >> GRS_FLAG_SHIFT;
        if (f == GRS_FLAG_NOT_READY) {
          blocked = true;
        } else {
          prefix += v[k] & GRS_VALUE_MASK;
          ++consumed;
          done = f == GRS_FLAG_INCLUSIVE;
        }
      }
    }
    if (done) return true;
    pt -= consumed;
    if (consumed == 0) {
      if (++spins > GRS_SPIN_LIMIT) {
        atomicOr(error_word, 1u);
        return true;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return false;
}

template <int RADIX, int G, bool STATS = false>
__device__ __forceinline__ uint32_t lookback2(const uint32_t* status, const uint32_t* gacc,
                                              uint32_t tile, uint32_t d, uint32_t* error_word) {
  uint32_t prefix = 0, spins = 0, trounds = 0, grounds = 0, fallbacks = 0;
  const int32_t g = static_cast<int32_t>(tile / G);
  int32_t pt = static_cast<int32_t>(tile) - 1;
  bool fin = walk_tiles<RADIX>(status, pt, g * G, d, prefix, spins, error_word, trounds);
  int32_t ph = g - 1;  // groups below g are full (only the last group can be ragged)
  while (!fin && ph >= 0) {
    ++grounds;
    uint32_t sl[GRS_LB_GWIN], ga[GRS_LB_GWIN];
#pragma unroll
    for (int k = 0; k < GRS_LB_GWIN; ++k) {
      const int32_t h = ph - k;
      sl[k] = h >= 0 ? ld_status(status + static_cast<size_t>(h * G + G - 1) * RADIX + d) : 0u;
      ga[k] = h >= 0 ? ld_status(gacc + static_cast<size_t>(h) * RADIX + d) : 0u;
    }
    int consumed = 0;
    bool done = false, blocked = false;
#pragma unroll
    for (int k = 0; k < GRS_LB_GWIN; ++k) {
      if (!done && !blocked && ph - k >= 0) {
        if ((sl[k] >> GRS_FLAG_SHIFT) == GRS_FLAG_INCLUSIVE) {
          prefix += sl[k] & GRS_VALUE_MASK;
          done = true;
        } else if ((ga[k] >> 24) == static_cast<uint32_t>(G)) {
          prefix += ga[k] & 0xFFFFFFu;
          ++consumed;
        } else {
          blocked = true;
        }
      }
    }
    if (done) break;
    ph -= consumed;
    if (blocked && ph >= 0) {
      // group ph is not complete yet: walk its tiles (ends on an INCLUSIVE or at its start)
      ++fallbacks;
      int32_t p2 = ph * G + G - 1;
      if (walk_tiles<RADIX>(status, p2, ph * G, d, prefix, spins, error_word, trounds)) break;
      --ph;
    }
  }
  if constexpr (STATS) {   // lab only: per tile max over digits of tile rounds / group rounds / fallbacks / spins
    uint32_t* st = error_word + 64 + static_cast<size_t>(tile) * 8;
    atomicMax(st + 0, trounds);
    atomicMax(st + 1, spins);
    atomicMax(st + 2, grounds);
    atomicMax(st + 3, fallbacks);
  }
  return prefix;
}

// Three-word look-back (LB3): tiles publish AGGREGATE words only; the group accumulator
// gacc[g][d] gathers (1 << 24) | count of every tile of group g by RETURNING atomics, and the
// tile whose add completes it (old arrivals == tiles in the group - 1) publishes the group's
// INCLUSIVE prefix ginc[g][d].  A tile's exclusive prefix = (aggregates of its own group's
// earlier tiles, < G words) + (prefix of its group: ginc of an earlier group plus the complete
// accumulators in between).  The group-level frontier advances by a whole window of groups
// per poll round trip, and nobody waits on another tile's look-back except the group
// completers (one per group and digit).
template <int RADIX, int G, bool STATS = false>
__device__ __forceinline__ uint32_t lookback3(const uint32_t* status, const uint32_t* gacc,
                                              uint32_t* ginc, uint32_t tile, uint32_t tiles,
                                              uint32_t d, uint32_t old, uint32_t publish,
                                              uint32_t* error_word) {
  uint32_t own = 0, spins = 0, trounds = 0, grounds = 0;
  const int32_t g = static_cast<int32_t>(tile / G);
  int32_t pt = static_cast<int32_t>(tile) - 1;
  walk_tiles<RADIX>(status, pt, g * G, d, own, spins, error_word, trounds);  // no INCLUSIVE words
  uint32_t gp = 0;
  int32_t ph = g - 1;
  while (ph >= 0) {
    ++grounds;
    uint32_t gi[GRS_LB_GWIN], ga[GRS_LB_GWIN];
#pragma unroll
    for (int k = 0; k < GRS_LB_GWIN; ++k) {
      const int32_t h = ph - k;
      gi[k] = h >= 0 ? ld_status(ginc + static_cast<size_t>(h) * RADIX + d) : 0u;
      ga[k] = h >= 0 ? ld_status(gacc + static_cast<size_t>(h) * RADIX + d) : 0u;
    }
    int consumed = 0;
    bool done = false, blocked = false;
#pragma unroll
    for (int k = 0; k < GRS_LB_GWIN; ++k) {
      if (!done && !blocked && ph - k >= 0) {
        if ((gi[k] >> GRS_FLAG_SHIFT) == GRS_FLAG_INCLUSIVE) {
          gp += gi[k] & GRS_VALUE_MASK;
          done = true;
        } else if ((ga[k] >> 24) == static_cast<uint32_t>(G)) {
          gp += ga[k] & 0xFFFFFFu;
          ++consumed;
        } else {
          blocked = true;
        }
      }
    }
    if (done) break;
    ph -= consumed;
    if (consumed == 0) {
      if (++spins > GRS_SPIN_LIMIT) {
        atomicOr(error_word, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  const uint32_t in_group = min(static_cast<uint32_t>(G), tiles - static_cast<uint32_t>(g) * G);
  if ((old >> 24) == in_group - 1)   // this tile completed the group's accumulator
    st_status(ginc + static_cast<size_t>(g) * RADIX + d,
              (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((gp + (old & 0xFFFFFFu) + publish) & GRS_VALUE_MASK));
  if constexpr (STATS) {
    uint32_t* st = error_word + 64 + static_cast<size_t>(tile) * 8;
    atomicMax(st + 0, trounds);
    atomicMax(st + 1, spins);
    atomicMax(st + 2, grounds);
  }
  return gp + own;
}

// Diagnostic build only (DBG bit 3, tools/lab): thread 0 records s_memtime at phase
// boundaries into dbg[64 + tile * 8 + k] (cycles since the workgroup started).
#define GRS_STAMP(k)                                                                       \
  do {                                                                                     \
    if constexpr ((DBG & 8) != 0) {                                                        \
      if (threadIdx.x == 0)                                                                \
        error_word[64 + static_cast<size_t>(tile) * 8 + (k)] =                             \
            static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t_begin);                 \
    }                                                                                      \
  } while (0)

// Load tile `tile` wave-striped into registers; padding slots get the all-ones key.
template <typename K, bool PAIRS, int BLOCK, int ITEMS>
__device__ __forceinline__ void load_tile(const K* __restrict__ keys_in,
                                          const uint32_t* __restrict__ vals_in, uint32_t n,
                                          uint32_t tile, K (&key)[ITEMS], uint32_t (&val)[ITEMS]) {
  constexpr int TILE = BLOCK * ITEMS;
  const uint32_t lane = threadIdx.x & (GRS_WAVE - 1);
  const uint32_t w = threadIdx.x >> 6;
  const uint32_t tile_base = tile * TILE;
  const uint32_t wbase = tile_base + w * (GRS_WAVE * ITEMS);
  if (n - tile_base >= static_cast<uint32_t>(TILE)) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = keys_in[wbase + j * GRS_WAVE + lane];
    if constexpr (PAIRS) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) val[j] = vals_in[wbase + j * GRS_WAVE + lane];
    }
  } else {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * GRS_WAVE + lane;
      // padding sorts after every valid key of its digit: all-ones digit, highest index
      key[j] = i < n ? keys_in[i] : static_cast<K>(~static_cast<K>(0));
      if constexpr (PAIRS) val[j] = i < n ? vals_in[i] : 0u;
    }
  }
}

// Steps 2-5 for one tile whose keys are in registers.  Precondition: every thread of the
// block has passed a barrier since the previous tile's last LDS access.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG, typename DigitF>
__device__ __forceinline__ void process_tile(
    OnesweepSmem<K, PAIRS, RB, BLOCK, ITEMS>& sm, const K (&key)[ITEMS],
    const uint32_t (&val)[ITEMS], uint32_t tile, K* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF& dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ status,
    uint32_t* __restrict__ status_next, uint32_t* __restrict__ error_word,
    uint64_t t_begin = 0) {
  constexpr int RADIX = 1 << RB;
  constexpr int WAVES = BLOCK / GRS_WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr bool EARLY = (DBG & 4) == 0;
  GRS_STAMP(0);
  static_assert(RADIX <= BLOCK, "one look-back thread per digit");

  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();  // digit of the padding key
  const uint32_t tile_base = tile * TILE;
  const uint32_t valid = (n - tile_base) < static_cast<uint32_t>(TILE) ? (n - tile_base) : TILE;
  const uint32_t pad = TILE - valid;
  uint32_t* my_status = status + static_cast<size_t>(tile) * RADIX + t;

  for (uint32_t i = t; i < WAVES * RADIX; i += BLOCK) sm.cnt[i] = 0;
  if (EARLY && t < RADIX) sm.hist[t] = 0;
  if (t < RADIX) status_next[static_cast<size_t>(tile) * RADIX + t] = 0;
  // digits once per item: rank[j] = digit << 16 | (tile-local rank, filled in step 3)
  uint32_t rank[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) rank[j] = dig(key[j]) << 16;
  __syncthreads();

  // ---- 2. tile digit counts, published before the (long) ranking ----
  if constexpr (EARLY) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) atomicAdd(&sm.hist[rank[j] >> 16], 1u);
    __syncthreads();
    GRS_STAMP(1);
    if constexpr ((DBG & 1) == 0) {
      if (t < RADIX) {
        const uint32_t c = sm.hist[t] - ((t == dmask) ? pad : 0u);
        st_status(my_status, ((tile == 0 ? GRS_FLAG_INCLUSIVE : GRS_FLAG_AGGREGATE) << GRS_FLAG_SHIFT) | c);
      }
    }
  }

  // ---- 3. stable rank inside the wave ----
  // Item by item: every lane reads its digit's running wave count, then ONE leader lane per
  // distinct digit adds the item's count for that digit (no-return LDS atomic).  LDS
  // executes a wave's instructions in order, so item j's read sees items < j and no
  // read -> write dependency stalls the loop.  rank[j] = (local rank) | digit << 16.
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    const uint64_t m = match_digit<RB>(d);
    const uint32_t below = mbcnt64(m);
    uint32_t* c = &sm.cnt[w * RADIX + d];
    const uint32_t old = *c;
    if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
    rank[j] |= old + below;
  }
  __syncthreads();
  GRS_STAMP(2);

  // ---- 4. per digit: exclusive over waves, block scans, look-back ----
  uint32_t tile_cnt = 0;
  if (t < RADIX) {
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      const uint32_t c = sm.cnt[ww * RADIX + t];
      sm.cnt[ww * RADIX + t] = tile_cnt;
      tile_cnt += c;
    }
  }
  // exclusive scans over digits of (pass histogram, tile count), packed in one u64:
  // hi 32 bits -> global start of digit d, lo 32 bits -> tile-local start of digit d
  uint64_t packed = 0;
  if (t < RADIX) packed = (static_cast<uint64_t>(pass_hist[t]) << 32) | tile_cnt;
  const uint64_t incl = wave_incl_scan(packed, lane);
  if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
  __syncthreads();
  GRS_STAMP(3);
  uint64_t carry = 0;
  for (uint32_t ww = 0; ww < w; ++ww) carry += sm.wsum[ww];
  const uint64_t excl = carry + incl - packed;

  if (t < RADIX) {
    const uint32_t global_start = static_cast<uint32_t>(excl >> 32);
    const uint32_t local_start = static_cast<uint32_t>(excl);
    // padding keys (last tile only) are ranked but never published or stored
    const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
    uint32_t prefix = 0;
    if constexpr (DBG & 1) {
      prefix = static_cast<uint32_t>((static_cast<uint64_t>(pass_hist[t]) * tile) /
                                     ((n + TILE - 1) / TILE));
    } else if (tile == 0) {
      if (!EARLY) st_status(my_status, (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | publish);
    } else {
      if (!EARLY) st_status(my_status, (GRS_FLAG_AGGREGATE << GRS_FLAG_SHIFT) | publish);
      prefix = lookback<RADIX>(status, tile, t, error_word);
      st_status(my_status, (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((prefix + publish) & GRS_VALUE_MASK));
    }
    sm.base[t] = global_start + prefix - local_start;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) sm.cnt[ww * RADIX + t] += local_start;
  }
  __syncthreads();
  GRS_STAMP(4);

  // ---- 5. reorder the tile in LDS by (digit, input order), then store the runs ----
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    const uint32_t pos = sm.cnt[w * RADIX + d] + (rank[j] & 0xFFFFu);
    sm.keys[pos] = key[j];
    if constexpr (PAIRS) sm.vals[pos] = val[j];
  }
  __syncthreads();
  GRS_STAMP(5);

  // consecutive threads write consecutive slots of each digit run
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + t;
    if (i < valid) {
      const K kk = sm.keys[i];
      uint32_t dst = (DBG & 2) ? tile_base + i : sm.base[dig(kk)] + i;
      if constexpr ((DBG & 1) != 0) dst = dst < n ? dst : n - 1;  // estimated prefix may overrun
      keys_out[dst] = kk;
      if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
    }
  }
  if constexpr ((DBG & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GRS_STAMP(6);
  }
}

// Default tile body: resolves the look-back BEFORE ranking (process_tile, DBG bit 5, ranks
// first and is kept for ablations): the
// tile's INCLUSIVE words are published as soon as its counts and its predecessors' prefixes
// are known, so the chain of inclusive prefixes is not gated by ranking time.
// `after_lookback()` runs on every thread once its look-back part is done (the persistent
// kernel issues the next tile's loads there, so they never sit in front of a look-back wait).
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG, typename DigitF,
          typename Hook = NoHook>
__device__ __forceinline__ void process_tile_lbfirst(
    OnesweepSmem<K, PAIRS, RB, BLOCK, ITEMS>& sm, const K (&key)[ITEMS],
    const uint32_t (&val)[ITEMS], uint32_t tile, K* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF& dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ status,
    uint32_t* __restrict__ status_next, uint32_t* __restrict__ error_word,
    uint64_t t_begin = 0, const Hook& after_lookback = Hook()) {
  constexpr int RADIX = 1 << RB;
  constexpr int WAVES = BLOCK / GRS_WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  static_assert(RADIX <= BLOCK, "one look-back thread per digit");
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();
  const uint32_t tile_base = tile * TILE;
  const uint32_t valid = (n - tile_base) < static_cast<uint32_t>(TILE) ? (n - tile_base) : TILE;
  const uint32_t pad = TILE - valid;
  uint32_t* my_status = status + static_cast<size_t>(tile) * RADIX + t;
  GRS_STAMP(0);

  for (uint32_t i = t; i < WAVES * RADIX; i += BLOCK) sm.cnt[i] = 0;
  if (t < RADIX) sm.hist[t] = 0;
  if (t < RADIX) status_next[static_cast<size_t>(tile) * RADIX + t] = 0;
  uint32_t rank[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) rank[j] = dig(key[j]) << 16;
  __syncthreads();
  if constexpr ((DBG & 64) == 0) {   // lab ablation: DBG bit 6 skips the tile histogram
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) atomicAdd(&sm.hist[rank[j] >> 16], 1u);
  }
  __syncthreads();
  GRS_STAMP(1);

  // tile counts -> (global start, tile-local start) per digit, then the look-back
  const uint32_t tile_cnt = t < RADIX ? sm.hist[t] : 0u;
  const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
  if (t < RADIX) {
    st_status(my_status, ((tile == 0 ? GRS_FLAG_INCLUSIVE : GRS_FLAG_AGGREGATE) << GRS_FLAG_SHIFT) | publish);
  }
  uint64_t packed = 0;
  if (t < RADIX) packed = (static_cast<uint64_t>(pass_hist[t]) << 32) | tile_cnt;
  const uint64_t incl = wave_incl_scan(packed, lane);
  if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
  __syncthreads();
  uint64_t carry = 0;
  for (uint32_t ww = 0; ww < w; ++ww) carry += sm.wsum[ww];
  const uint64_t excl = carry + incl - packed;
  GRS_STAMP(2);
  if (t < RADIX) {
    uint32_t prefix = 0;
    if (tile != 0) {
      prefix = lookback<RADIX>(status, tile, t, error_word);
      st_status(my_status, (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((prefix + publish) & GRS_VALUE_MASK));
    }
    sm.base[t] = static_cast<uint32_t>(excl >> 32) + prefix - static_cast<uint32_t>(excl);
    sm.hist[t] = static_cast<uint32_t>(excl);  // tile-local start of digit t
  }
  GRS_STAMP(3);
  after_lookback();

  // stable rank inside the wave (as process_tile step 3)
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    const uint64_t m = match_digit<RB>(d);
    const uint32_t below = mbcnt64(m);
    uint32_t* c = &sm.cnt[w * RADIX + d];
    const uint32_t old = *c;
    if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
    rank[j] |= old + below;
  }
  __syncthreads();
  GRS_STAMP(4);
  if (t < RADIX) {
    uint32_t run = sm.hist[t];
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      const uint32_t c = sm.cnt[ww * RADIX + t];
      sm.cnt[ww * RADIX + t] = run;
      run += c;
    }
  }
  __syncthreads();

#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    // lab ablation: DBG bit 12 drops the offset lookup (positions become wrong)
    const uint32_t pos = ((DBG & 4096) ? 0u : sm.cnt[w * RADIX + d]) + (rank[j] & 0xFFFFu);
    const uint32_t p2 = (DBG & 4096) ? pos % TILE : pos;
    sm.keys[p2] = key[j];
    if constexpr (PAIRS) sm.vals[p2] = val[j];
  }
  __syncthreads();
  GRS_STAMP(5);
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + t;
    if (i < valid) {
      const K kk = sm.keys[i];
      // lab ablation: DBG bit 7 reads one uniform base instead of the digit's
      uint32_t dst = ((DBG & 128) ? sm.base[0] : sm.base[dig(kk)]) + i;
      if constexpr ((DBG & (1 | 128)) != 0) dst = dst < n ? dst : n - 1;
      keys_out[dst] = kk;
      if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
    }
  }
  if constexpr ((DBG & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GRS_STAMP(6);
  }
}

// One tile per workgroup (grid = number of tiles).
// DBG bits 8-11 (lab only): minimum waves per SIMD for __launch_bounds__ (0 = no bound).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, ((DBG >> 8) & 15) ? ((DBG >> 8) & 15) : 1) void grs_onesweep_pass(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  __shared__ OnesweepSmem<K, PAIRS, RB, BLOCK, ITEMS> sm;
  const uint64_t t_begin = (DBG & 8) ? __builtin_amdgcn_s_memtime() : 0;
  if (threadIdx.x == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tile = sm.ticket[0];
  K key[ITEMS];
  uint32_t val[ITEMS];
  load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, tile, key, val);
  if constexpr ((DBG & 32) == 0)   // default: look-back before ranking
    process_tile_lbfirst<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, key, val, tile, keys_out, vals_out,
                                                          n, dig, pass_hist, status, status_next,
                                                          error_word, t_begin);
  else
    process_tile<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, key, val, tile, keys_out, vals_out, n, dig,
                                                  pass_hist, status, status_next, error_word,
                                                  t_begin);
  if constexpr ((DBG & 8) != 0) {
    if (threadIdx.x == 0) {
      error_word[64 + static_cast<size_t>(tile) * 8 + 7] = static_cast<uint32_t>(t_begin >> 8);
    }
  }
}

// Persistent variant: a fixed grid of workgroups loops over tickets.  The next tile's keys
// are loaded into a second register set right after the current tile's look-back (so no
// look-back wait drains them) and stay in flight through ranking, reorder and stores.  A
// workgroup processes its tickets in increasing order, so it never waits on a tile it holds
// itself (no deadlock whatever the residency).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, ((DBG >> 8) & 15) ? ((DBG >> 8) & 15) : 1) void grs_onesweep_persistent(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  __shared__ OnesweepSmem<K, PAIRS, RB, BLOCK, ITEMS> sm;
  constexpr uint32_t TILE = BLOCK * ITEMS;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  K ka[ITEMS], kb[ITEMS];
  uint32_t va[ITEMS], vb[ITEMS];
  if (threadIdx.x == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
  __syncthreads();
  uint32_t cur = sm.ticket[0];
  if (cur < tiles) load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, cur, ka, va);
  uint32_t nxt = tiles;
  while (cur < tiles) {
    // next ticket; visible to all threads after process_tile's first barrier
    if (threadIdx.x == 0) sm.ticket[1] = atomicAdd(ticket, 1u);
    process_tile_lbfirst<K, PAIRS, RB, BLOCK, ITEMS, DBG>(
        sm, ka, va, cur, keys_out, vals_out, n, dig, pass_hist, status, status_next, error_word,
        0, [&]() {
          nxt = sm.ticket[1];
          if (nxt < tiles) load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, nxt, kb, vb);
        });
    if (nxt >= tiles) break;
    __syncthreads();   // every read of ticket[0] (long done) and of the LDS tile is finished
    if (threadIdx.x == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
    process_tile_lbfirst<K, PAIRS, RB, BLOCK, ITEMS, DBG>(
        sm, kb, vb, nxt, keys_out, vals_out, n, dig, pass_hist, status, status_next, error_word,
        0, [&]() {
          cur = sm.ticket[0];
          if (cur < tiles) load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, cur, ka, va);
        });
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------------------
// streaming onesweep pass: persistent workgroups, LDS-DMA double-buffered tile prefetch
// ----------------------------------------------------------------------------------------
//
// A fixed grid loops over tile tickets.  Tile i+1 is fetched HBM -> LDS with
// global_load_lds_dwordx4 (no VGPRs) as soon as tile i's look-back is resolved, and stays in
// flight through tile i's ranking, reorder and stores and the top of iteration i+1, so every
// workgroup keeps a tile's worth of reads outstanding almost all the time.  Barriers after
// the DMA issue are raw s_barrier + lgkmcnt(0) (a __syncthreads() would drain the DMA); the
// DMA is retired by a counted vmcnt that skips exactly the tile's own scatter stores, which
// are issued after it.  Tickets run two tiles ahead (fetched during a look-back, whose wait
// absorbs the atomic's latency).  A workgroup processes its tickets in increasing order, so
// it never waits on a tile it holds (no deadlock whatever the residency).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS>
struct StreamSmem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  uint32_t cnt[WAVES * RADIX];
  uint32_t hist[RADIX];
  uint32_t base[RADIX];
  uint64_t wsum[WAVES];
  uint32_t ticket[4];
  alignas(16) K kbuf[2][TILE];
  alignas(16) uint32_t vbuf[PAIRS ? 2 : 1][PAIRS ? TILE : 4];
};


// One global_load_lds_dwordx4: 16 bytes per lane from `gsrc` (per lane) into LDS at
// `lds` + 16 * lane (lds wave-uniform).  Written as inline asm on purpose: the compiler
// does not track the DMA, so it inserts no vmcnt(0) in front of unrelated LDS reads (which
// would drain the prefetch); the kernel retires it with its own counted s_waitcnt.
template <bool NT = false>
__device__ __forceinline__ void lds_dma16(const void* gsrc, void* lds) {
  // M0 is compiler-reserved: set and restore it inside the statement that uses it
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lds)));
  uint32_t keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(dst)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(dst)
        : "memory");
}

// HBM -> LDS copy of one full tile (keys, and payload), 1 KiB per wave instruction.
template <typename K, bool PAIRS, int BLOCK, int ITEMS, bool NT = false>
__device__ __forceinline__ void dma_tile(const K* __restrict__ keys_in,
                                         const uint32_t* __restrict__ vals_in, uint32_t tile,
                                         K* kdst, uint32_t* vdst) {
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WAVES = BLOCK / GRS_WAVE;
  constexpr int KCH = TILE * static_cast<int>(sizeof(K)) / 1024;
  constexpr int VCH = TILE * 4 / 1024;
  static_assert(KCH % WAVES == 0 && VCH % WAVES == 0, "whole 1 KiB chunks per wave");
  const uint32_t lane = threadIdx.x & (GRS_WAVE - 1);
  const uint32_t w = threadIdx.x >> 6;
  const char* ks = reinterpret_cast<const char*>(keys_in + static_cast<size_t>(tile) * TILE);
#pragma unroll
  for (int c = 0; c < KCH / WAVES; ++c) {
    const int ch = c * WAVES + w;
    lds_dma16<NT>(ks + ch * 1024 + lane * 16, reinterpret_cast<char*>(kdst) + ch * 1024);
  }
  if constexpr (PAIRS) {
    const char* vs = reinterpret_cast<const char*>(vals_in + static_cast<size_t>(tile) * TILE);
#pragma unroll
    for (int c = 0; c < VCH / WAVES; ++c) {
      const int ch = c * WAVES + w;
      lds_dma16<NT>(vs + ch * 1024 + lane * 16, reinterpret_cast<char*>(vdst) + ch * 1024);
    }
  }
}

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK) void grs_onesweep_stream(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  using SM = StreamSmem<K, PAIRS, RB, BLOCK, ITEMS>;
  constexpr int RADIX = SM::RADIX;
  constexpr int WAVES = SM::WAVES;
  constexpr int TILE = SM::TILE;
  constexpr int WAVE_TILE = GRS_WAVE * ITEMS;
  // scatter stores a wave issues after the DMA of the next tile (full tiles)
  constexpr int NST = ITEMS * (PAIRS ? 2 : 1);
  static_assert(NST <= 63, "vmcnt field");
  static_assert(RADIX <= BLOCK, "one look-back thread per digit");
  __shared__ SM sm;

  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const uint32_t full_tiles = n / TILE;

  // tickets run ahead: at the top of an iteration on tile T_i, T_{i+1} is prefetched into
  // LDS, thread 0 holds T_{i+2} in a register (publishes it to LDS now) and fetches
  // T_{i+3} during the look-back
  constexpr uint32_t TK_THREAD = BLOCK - GRS_WAVE;   // lane 0 of the last wave
  uint32_t tk_reg = 0;
  if (t == TK_THREAD) {
    sm.ticket[0] = atomicAdd(ticket, 1u);
    sm.ticket[1] = atomicAdd(ticket, 1u);
    tk_reg = atomicAdd(ticket, 1u);
  }
  __syncthreads();
  uint32_t cur = sm.ticket[0];
  uint32_t nxt = sm.ticket[1];
  if (cur < full_tiles) dma_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, cur, sm.kbuf[0], sm.vbuf[0]);
  bool prev_full_stores = false;  // previous iteration issued NST scatter stores after its DMA
  int b = 0;
  const uint32_t my_hist = t < RADIX ? pass_hist[t] : 0u;  // this pass's count of digit t

  while (cur < tiles) {
    // ---- retire the DMA of `cur` (older than the previous tile's NST scatter stores) ----
    if (prev_full_stores)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();

    if (t == TK_THREAD) sm.ticket[2 + b] = tk_reg;   // T_{i+2}, read at the end of this iteration
    const uint32_t tile_base = cur * TILE;
    const bool full = cur < full_tiles;
    const uint32_t valid = full ? TILE : n - tile_base;
    const uint32_t pad = TILE - valid;
    if (!full) {
      // the ragged last tile was not prefetched: stage it through LDS in the same layout
      // (padding = all-ones keys), so the common path below reads LDS only
      for (uint32_t i = t; i < static_cast<uint32_t>(TILE); i += BLOCK) {
        sm.kbuf[b][i] = i < valid ? keys_in[tile_base + i] : static_cast<K>(~static_cast<K>(0));
        if constexpr (PAIRS) sm.vbuf[b][i] = i < valid ? vals_in[tile_base + i] : 0u;
      }
      lds_barrier();
    }
    K key[ITEMS];
    uint32_t val[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = sm.kbuf[b][w * WAVE_TILE + j * GRS_WAVE + lane];
    if constexpr (PAIRS) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) val[j] = sm.vbuf[b][w * WAVE_TILE + j * GRS_WAVE + lane];
    }

    uint32_t* my_status = status + static_cast<size_t>(cur) * RADIX + t;
    for (uint32_t i = t; i < WAVES * RADIX; i += BLOCK) sm.cnt[i] = 0;
    if (t < RADIX) sm.hist[t] = 0;
    if (t < RADIX) status_next[static_cast<size_t>(cur) * RADIX + t] = 0;
    uint32_t rank[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) rank[j] = dig(key[j]) << 16;
    lds_barrier();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) atomicAdd(&sm.hist[rank[j] >> 16], 1u);
    lds_barrier();

    const uint32_t tile_cnt = t < RADIX ? sm.hist[t] : 0u;
    const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
    if (t < RADIX)
      st_status(my_status, ((cur == 0 ? GRS_FLAG_INCLUSIVE : GRS_FLAG_AGGREGATE) << GRS_FLAG_SHIFT) | publish);
    uint64_t packed = 0;
    if (t < RADIX) packed = (static_cast<uint64_t>(my_hist) << 32) | tile_cnt;
    const uint64_t incl = wave_incl_scan(packed, lane);
    if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
    lds_barrier();
    uint64_t carry = 0;
    for (uint32_t ww = 0; ww < w; ++ww) carry += sm.wsum[ww];
    const uint64_t excl = carry + incl - packed;
    // T_{i+3}, used one iteration later; fetched by the last wave, which does no look-back
    // (RADIX <= BLOCK - 64) or looks back last, so the atomic's wait costs nobody time
    if (t == TK_THREAD) tk_reg = atomicAdd(ticket, 1u);
    if (t < RADIX) {
      uint32_t prefix = 0;
      if (cur != 0) {
        prefix = lookback<RADIX>(status, cur, t, error_word);
        st_status(my_status, (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((prefix + publish) & GRS_VALUE_MASK));
      }
      sm.base[t] = static_cast<uint32_t>(excl >> 32) + prefix - static_cast<uint32_t>(excl);
      sm.hist[t] = static_cast<uint32_t>(excl);  // tile-local start of digit t
    }
    // ---- prefetch the next tile into the other buffer ----
    const bool nxt_full = nxt < full_tiles;
    if (nxt_full) dma_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, nxt, sm.kbuf[b ^ 1], sm.vbuf[PAIRS ? (b ^ 1) : 0]);

    // ---- stable rank inside the wave ----
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t d = rank[j] >> 16;
      const uint64_t m = match_digit<RB>(d);
      const uint32_t below = mbcnt64(m);
      uint32_t* c = &sm.cnt[w * RADIX + d];
      const uint32_t old = *c;
      if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
      rank[j] |= old + below;
    }
    lds_barrier();
    if (t < RADIX) {
      uint32_t run = sm.hist[t];
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        const uint32_t c = sm.cnt[ww * RADIX + t];
        sm.cnt[ww * RADIX + t] = run;
        run += c;
      }
    }
    lds_barrier();
    // reorder into the current tile's buffer (its keys are in registers now)
    K* kr = sm.kbuf[b];
    uint32_t* vr = sm.vbuf[PAIRS ? b : 0];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t d = rank[j] >> 16;
      const uint32_t pos = sm.cnt[w * RADIX + d] + (rank[j] & 0xFFFFu);
      kr[pos] = key[j];
      if constexpr (PAIRS) vr[pos] = val[j];
    }
    lds_barrier();
    if (full) {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        const K kk = kr[i];
        uint32_t dst = sm.base[dig(kk)] + i;
        keys_out[dst] = kk;
        if constexpr (PAIRS) vals_out[dst] = vr[i];
      }
    } else {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        if (i < valid) {
          const K kk = kr[i];
          const uint32_t dst = sm.base[dig(kk)] + i;
          keys_out[dst] = kk;
          if constexpr (PAIRS) vals_out[dst] = vr[i];
        }
      }
    }
    prev_full_stores = full && nxt_full;
    // ---- advance: next = prefetched tile; the ticket after it was stored two slots on ----
    lds_barrier();   // every read of kr / base / ticket of this iteration is done
    cur = nxt;
    nxt = sm.ticket[2 + b];
    b ^= 1;
  }
}

// ----------------------------------------------------------------------------------------
// atomic-rank onesweep pass (the library default: every key type, tiles as large as LDS allows)
// ----------------------------------------------------------------------------------------
//
// Ranking by ONE returning LDS atomic per key: lane l of wave w adds 1 to the wave's counter
// of its digit with ds_add_rtn_u32 and gets back the count of that digit over the wave's
// earlier items plus the LOWER lanes of this item.  That holds because the LDS serialises the
// lanes of one atomic wave-instruction that hit one address in ascending lane order (gfx950
// property, probed by tools/ldsorder.hip and checked at sorter creation by grs_probe_lds_order;
// the library falls back to the ballot-match pass above if the probe fails).  It replaces
// the 8-ballot match (≈40 VALU per item) with one LDS instruction per item, and the tile
// histogram falls out of the per-wave counters (no separate atomics).
//
// Per tile: rank -> B1 -> per-digit wave prefix + tile count, publish AGGREGATE, block scan
// -> B2 -> look-back (waves holding digits) -> B3 -> reorder into LDS by (digit, input order)
// -> B4 -> zero counters for the next tile; store each digit run to its global slot.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS>
struct ArSmem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  uint32_t cnt[WAVES * RADIX];  // per-wave digit counters -> wave start of each digit in the tile
  uint32_t base[RADIX];         // global destination of tile position 0 of digit d
  uint64_t wsum[WAVES];
  uint32_t ticket[2];
  K keys[TILE];
  uint32_t vals[PAIRS ? TILE : 1];
};

// Steps of one tile whose keys are in registers.  Precondition: sm.cnt is zero and every
// thread passed a barrier after that zeroing and after the previous tile's last LDS read.
// Leaves sm.cnt zero again (zeroed after B4).  `early_hook` runs on waves without a digit to
// look back (right after B1); `late_hook` on the look-back waves once their look-back is
// done: the persistent kernel issues the next tile's loads there, so no look-back poll ever
// waits behind them.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG, typename DigitF,
          typename Hook>
__device__ __forceinline__ void ar_tile(ArSmem<K, PAIRS, RB, BLOCK, ITEMS>& sm,
                                        const K (&key)[ITEMS], const uint32_t (&val)[ITEMS],
                                        uint32_t tile, K* __restrict__ keys_out,
                                        uint32_t* __restrict__ vals_out, uint32_t n,
                                        const DigitF& dig, uint32_t my_hist,
                                        uint32_t* __restrict__ status,
                                        uint32_t* __restrict__ status_next,
                                        uint32_t* __restrict__ error_word, const Hook& hook,
                                        uint64_t t_begin = 0) {
  constexpr int RADIX = 1 << RB;
  constexpr int WAVES = BLOCK / GRS_WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int LB_WAVES = (RADIX + GRS_WAVE - 1) / GRS_WAVE;
  static_assert(RADIX <= BLOCK, "one look-back thread per digit");
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();
  const uint32_t tile_base = tile * TILE;
  const uint32_t valid = (n - tile_base) < static_cast<uint32_t>(TILE) ? (n - tile_base) : TILE;
  const uint32_t pad = TILE - valid;
  // look-back: LB3 (group accumulators + group INCLUSIVE words published by the tile that
  // completes a group) by default; lab ablations: DBG & 32 = two-level with tile INCLUSIVE
  // chain (LB2), DBG & 2048 = the plain windowed look-back
  constexpr bool LB3 = (DBG & (32 | 2048)) == 0;
  constexpr bool LB2 = (DBG & 32) != 0 || LB3;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const uint32_t groups = (tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP;
  uint32_t* gacc = status + static_cast<size_t>(tiles) * RADIX;  // [groups][RADIX] after the tile words
  uint32_t* ginc = gacc + static_cast<size_t>(groups) * RADIX;   // LB3: [groups][RADIX] group inclusives

  GRS_STAMP(0);
  // ---- rank: one returning LDS atomic per item (lane-ordered, see above) ----
  uint32_t rank[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = dig(key[j]);
    rank[j] = (d << 16) | atomicAdd(&sm.cnt[w * RADIX + d], 1u);
  }
  if (t < RADIX) {
    status_next[static_cast<size_t>(tile) * RADIX + t] = 0;
    if (LB2 && tile % GRS_LB_GROUP == 0)
      status_next[static_cast<size_t>(tiles) * RADIX + (tile / GRS_LB_GROUP) * RADIX + t] = 0;
    if (LB3 && tile % GRS_LB_GROUP == 0)
      status_next[static_cast<size_t>(tiles + groups) * RADIX + (tile / GRS_LB_GROUP) * RADIX + t] = 0;
  }
  lds_barrier();  // B1
  GRS_STAMP(1);
  if (w >= LB_WAVES) hook();

  // ---- per digit: wave starts, tile count, early publish, block scan over digits ----
  uint32_t tile_cnt = 0, gold = 0;
  uint32_t* my_status = status + static_cast<size_t>(tile) * RADIX + t;
  if (t < RADIX) {
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      const uint32_t c = sm.cnt[ww * RADIX + t];
      sm.cnt[ww * RADIX + t] = tile_cnt;
      tile_cnt += c;
    }
    const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
    st_status(my_status, ((tile == 0 && !LB3 ? GRS_FLAG_INCLUSIVE : GRS_FLAG_AGGREGATE) << GRS_FLAG_SHIFT) | publish);
    if constexpr (LB3)
      gold = __hip_atomic_fetch_add(gacc + static_cast<size_t>(tile / GRS_LB_GROUP) * RADIX + t,
                                    (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr (LB2)
      __hip_atomic_fetch_add(gacc + static_cast<size_t>(tile / GRS_LB_GROUP) * RADIX + t,
                             (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // hi 32 bits -> global start of digit d over the pass, lo 32 bits -> start in the tile
  const uint64_t packed = t < RADIX ? (static_cast<uint64_t>(my_hist) << 32) | tile_cnt : 0ull;
  uint64_t excl = 0;
  if (w < LB_WAVES) {
    const uint64_t incl = wave_incl_scan(packed, lane);
    if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
    excl = incl - packed;
  }
  lds_barrier();  // B2
  GRS_STAMP(2);
  if (t < RADIX) {
    for (uint32_t ww = 0; ww < w; ++ww) excl += sm.wsum[ww];
    const uint32_t local_start = static_cast<uint32_t>(excl);
    uint32_t prefix = 0;
    if constexpr (LB3) {
      const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
      prefix = lookback3<RADIX, GRS_LB_GROUP, (DBG & 16) != 0>(status, gacc, ginc, tile, tiles, t,
                                                               gold, publish, error_word);
    } else if (tile != 0) {
      const uint32_t publish = (t == dmask) ? tile_cnt - pad : tile_cnt;
      if constexpr (LB2)
        prefix = lookback2<RADIX, GRS_LB_GROUP, (DBG & 16) != 0>(status, gacc, tile, t, error_word);
      else
        prefix = lookback<RADIX, (DBG & 16) != 0>(status, tile, t, error_word);
      st_status(my_status, (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((prefix + publish) & GRS_VALUE_MASK));
    }
    sm.base[t] = static_cast<uint32_t>(excl >> 32) + prefix - local_start;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) sm.cnt[ww * RADIX + t] += local_start;
  }
  if (w < LB_WAVES) hook();
  lds_barrier();  // B3
  GRS_STAMP(3);

  // ---- reorder the tile in LDS by (digit, input order) ----
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    const uint32_t pos = sm.cnt[w * RADIX + d] + (rank[j] & 0xFFFFu);
    sm.keys[pos] = key[j];
    if constexpr (PAIRS) sm.vals[pos] = val[j];
  }
  lds_barrier();  // B4
  GRS_STAMP(4);
  for (uint32_t i = t; i < static_cast<uint32_t>(WAVES * RADIX); i += BLOCK) sm.cnt[i] = 0;

  // ---- store: consecutive threads write consecutive slots of each digit run ----
  if (valid == static_cast<uint32_t>(TILE)) {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const uint32_t i = k * BLOCK + t;
      const K kk = sm.keys[i];
      const uint32_t dst = sm.base[dig(kk)] + i;
      keys_out[dst] = kk;
      if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
    }
  } else {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const uint32_t i = k * BLOCK + t;
      if (i < valid) {
        const K kk = sm.keys[i];
        const uint32_t dst = sm.base[dig(kk)] + i;
        keys_out[dst] = kk;
        if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
      }
    }
  }
  if constexpr ((DBG & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GRS_STAMP(5);
  }
}

// One tile per workgroup (grid = number of tiles).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK) void grs_onesweep_ar(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  using SM = ArSmem<K, PAIRS, RB, BLOCK, ITEMS>;
  __shared__ SM sm;
  const uint64_t t_begin = (DBG & 8) ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t t = threadIdx.x;
  if (t == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < static_cast<uint32_t>(SM::WAVES * SM::RADIX); i += BLOCK) sm.cnt[i] = 0;
  const uint32_t my_hist = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  __syncthreads();
  const uint32_t tile = (DBG & 8192) ? blockIdx.x : sm.ticket[0];  // lab: DBG 8192 = no ticket
  K key[ITEMS];
  uint32_t val[ITEMS];
  load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, tile, key, val);
  if constexpr ((DBG & 8) != 0) {   // stamp 6 = load issue done, 7 = start time
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (t == 0) {
      error_word[64 + static_cast<size_t>(tile) * 8 + 6] = static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t_begin);
      error_word[64 + static_cast<size_t>(tile) * 8 + 7] = static_cast<uint32_t>(t_begin >> 8);
    }
  }
  ar_tile<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, key, val, tile, keys_out, vals_out, n, dig, my_hist,
                                           status, status_next, error_word, NoHook(), t_begin);
}

// Persistent variant: a fixed grid loops over tickets.  The next tile's keys are loaded into
// a second register set as soon as a wave has nothing left to poll (ar_tile's hooks), so they
// are in flight through the current tile's look-back, reorder and stores.  A workgroup
// processes its tickets in increasing order and so never waits on a tile it holds itself.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK) void grs_onesweep_ar_persist(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  using SM = ArSmem<K, PAIRS, RB, BLOCK, ITEMS>;
  __shared__ SM sm;
  constexpr uint32_t TILE = BLOCK * ITEMS;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const uint32_t t = threadIdx.x;
  K ka[ITEMS], kb[ITEMS];
  uint32_t va[ITEMS], vb[ITEMS];
  if (t == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < static_cast<uint32_t>(SM::WAVES * SM::RADIX); i += BLOCK) sm.cnt[i] = 0;
  const uint32_t my_hist = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  __syncthreads();
  uint32_t cur = sm.ticket[0];
  if (cur < tiles) load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, cur, ka, va);
  while (cur < tiles) {
    // next ticket: written before ar_tile's B1, read by the hooks after it
    if (t == 0) sm.ticket[1] = atomicAdd(ticket, 1u);
    uint32_t nxt = tiles;
    ar_tile<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, ka, va, cur, keys_out, vals_out, n, dig, my_hist,
                                             status, status_next, error_word, [&]() {
                                               nxt = sm.ticket[1];
                                               if (nxt < tiles)
                                                 load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, nxt, kb, vb);
                                             });
    lds_barrier();  // counters zeroed, every LDS read of this tile done
    if (nxt >= tiles) break;
    if (t == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
    cur = tiles;
    ar_tile<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, kb, vb, nxt, keys_out, vals_out, n, dig, my_hist,
                                             status, status_next, error_word, [&]() {
                                               cur = sm.ticket[0];
                                               if (cur < tiles)
                                                 load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, cur, ka, va);
                                             });
    lds_barrier();
  }
}

// ----------------------------------------------------------------------------------------
// atomic-rank onesweep pass, one-wave vectorised two-level look-back (ar2)
// ----------------------------------------------------------------------------------------
//
// As ar_tile, but everything between ranking and reordering is done by wave 0 alone, DPL
// digits per lane (4 for 8-bit digits): column prefixes over the per-wave counters (b128 LDS
// rows), tile counts, the AGGREGATE publish (one 16-B sc1 store per lane = 1 KB per tile in
// one instruction), the group accumulators, the tile-local digit starts (one wave scan) and the
// two-level look-back with 16-B sc1 polls (one load instruction per predecessor tile for all
// 256 digits, 4x fewer than one dword per digit).  Wave 0 issues its first poll window, then
// takes part in the reorder (which needs only tile-local offsets), then finishes the look-back;
// the global base of each digit is needed only by the stores after the next barrier.
template <int RADIX>
struct LbCfg {
  static constexpr int DPL = RADIX >= 64 ? RADIX / 64 : 1;  // digits per look-back lane
  static constexpr int LANES = RADIX / DPL;                 // active look-back lanes
  static_assert(DPL == 1 || DPL == 4, "look-back vector width");
};

using lb_rsrc = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ lb_rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// agent-coherent (sc1) vector load / store of DPL consecutive status words
template <int DPL>
__device__ __forceinline__ void lb_ld(lb_rsrc r, uint32_t word, uint32_t (&o)[DPL]) {
  if constexpr (DPL == 4) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, word * 4u, 0, 16);
    o[0] = x[0]; o[1] = x[1]; o[2] = x[2]; o[3] = x[3];
  } else {
    o[0] = __builtin_amdgcn_raw_buffer_load_b32(r, word * 4u, 0, 16);
  }
}
template <int DPL>
__device__ __forceinline__ void lb_st(lb_rsrc r, uint32_t word, const uint32_t (&v)[DPL]) {
  if constexpr (DPL == 4) {
    using v4 = __attribute__((ext_vector_type(4))) uint32_t;
    const v4 x = {v[0], v[1], v[2], v[3]};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, word * 4u, 0, 16);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(v[0], r, word * 4u, 0, 16);
  }
}

// Look-back state of one lane (DPL digits).  Phase 1 walks the tiles of the own group, phase 2
// whole groups (see lookback2).  `issue` loads the first window; `finish` completes the walk.
template <int RADIX, int DPL>
struct Lb2 {
  static constexpr int W = GRS_LB_WIN;
  static constexpr int GW = GRS_LB_GWIN;
  static constexpr int G = GRS_LB_GROUP;
  static constexpr uint32_t ALL = (1u << DPL) - 1u;
  uint32_t prefix[DPL];
  uint32_t done;       // bit k: digit k complete
  int32_t pt;          // next tile to consume (phase 1)
  int32_t bottom;      // first tile of the own group
  uint32_t v[W][DPL];  // window of tile words pt, pt-1, ...

  __device__ __forceinline__ void issue(lb_rsrc st, uint32_t tile, uint32_t lane) {
#pragma unroll
    for (int k = 0; k < DPL; ++k) prefix[k] = 0;
    done = 0;
    pt = static_cast<int32_t>(tile) - 1;
    bottom = static_cast<int32_t>(tile / G) * G;
    load_window(st, lane);
  }
  __device__ __forceinline__ void load_window(lb_rsrc st, uint32_t lane) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      if (pt - k >= bottom) {
        lb_ld<DPL>(st, static_cast<uint32_t>(pt - k) * RADIX + lane * DPL, v[k]);
      } else {
#pragma unroll
        for (int e = 0; e < DPL; ++e) v[k][e] = 0;
      }
    }
  }
  // consume one tile's words for the not-done digits; false = some digit NOT_READY
  __device__ __forceinline__ bool take(const uint32_t (&x)[DPL]) {
    bool ready = true;
#pragma unroll
    for (int e = 0; e < DPL; ++e)
      if (!(done >> e & 1u) && (x[e] >> GRS_FLAG_SHIFT) == GRS_FLAG_NOT_READY) ready = false;
    if (!ready) return false;
#pragma unroll
    for (int e = 0; e < DPL; ++e) {
      if (!(done >> e & 1u)) {
        prefix[e] += x[e] & GRS_VALUE_MASK;
        if ((x[e] >> GRS_FLAG_SHIFT) == GRS_FLAG_INCLUSIVE) done |= 1u << e;
      }
    }
    return true;
  }
  // walk tiles [bottom, pt] starting from the loaded window; true = all digits done
  __device__ __forceinline__ bool walk(lb_rsrc st, uint32_t lane, uint32_t& spins,
                                       uint32_t* error_word) {
    while (true) {
      int consumed = 0;
      bool blocked = false;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        if (!blocked && done != ALL && pt - k >= bottom) {
          if (take(v[k])) ++consumed; else blocked = true;
        }
      }
      pt -= consumed;
      if (done == ALL) return true;
      if (pt < bottom) return false;
      if (consumed == 0) {
        if (++spins > GRS_SPIN_LIMIT) {
          atomicOr(error_word, 1u);
          done = ALL;
          return true;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      load_window(st, lane);
    }
  }
  __device__ __forceinline__ void finish(lb_rsrc st, lb_rsrc ga, uint32_t lane,
                                         uint32_t* error_word) {
    uint32_t spins = 0;
    if (walk(st, lane, spins, error_word)) return;
    int32_t ph = bottom / G - 1;  // groups below the own group are full
    while (ph >= 0 && done != ALL) {
      uint32_t sl[GW][DPL], gv[GW][DPL];
#pragma unroll
      for (int k = 0; k < GW; ++k) {
        if (ph - k >= 0) {
          lb_ld<DPL>(st, static_cast<uint32_t>((ph - k) * G + G - 1) * RADIX + lane * DPL, sl[k]);
          lb_ld<DPL>(ga, static_cast<uint32_t>(ph - k) * RADIX + lane * DPL, gv[k]);
        }
      }
      int consumed = 0;
      bool blocked = false;
#pragma unroll
      for (int k = 0; k < GW; ++k) {
        if (!blocked && done != ALL && ph - k >= 0) {
          bool ok = true;
#pragma unroll
          for (int e = 0; e < DPL; ++e)
            if (!(done >> e & 1u) && (sl[k][e] >> GRS_FLAG_SHIFT) != GRS_FLAG_INCLUSIVE &&
                (gv[k][e] >> 24) != static_cast<uint32_t>(G))
              ok = false;
          if (!ok) {
            blocked = true;
          } else {
#pragma unroll
            for (int e = 0; e < DPL; ++e) {
              if (!(done >> e & 1u)) {
                if ((sl[k][e] >> GRS_FLAG_SHIFT) == GRS_FLAG_INCLUSIVE) {
                  prefix[e] += sl[k][e] & GRS_VALUE_MASK;
                  done |= 1u << e;
                } else {
                  prefix[e] += gv[k][e] & 0xFFFFFFu;
                }
              }
            }
            ++consumed;
          }
        }
      }
      ph -= consumed;
      if (blocked && ph >= 0 && done != ALL) {
        // group ph incomplete: walk its tiles (ends on INCLUSIVE words or at its first tile)
        pt = ph * G + G - 1;
        bottom = ph * G;
        load_window(st, lane);
        if (walk(st, lane, spins, error_word)) return;
        --ph;
      }
    }
  }
};

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS>
struct Ar2Smem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  alignas(16) uint32_t cnt[WAVES * RADIX];  // per-wave digit counters -> tile positions
  alignas(16) uint32_t base[RADIX];         // global destination of tile position 0 of digit d
  uint32_t ticket[2];
  K keys[TILE];
  uint32_t vals[PAIRS ? TILE : 1];
};

// Tile body.  Precondition: sm.cnt is zero and every thread passed a barrier after that and
// after the previous tile's last LDS read.  Leaves sm.cnt zero.  gstart[e] (wave 0, lanes <
// LANES): global start of digit lane*DPL+e in this pass (exclusive scan of the pass histogram).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG, typename DigitF,
          typename Hook>
__device__ __forceinline__ void ar2_tile(Ar2Smem<K, PAIRS, RB, BLOCK, ITEMS>& sm,
                                         const K (&key)[ITEMS], const uint32_t (&val)[ITEMS],
                                         uint32_t tile, K* __restrict__ keys_out,
                                         uint32_t* __restrict__ vals_out, uint32_t n,
                                         const DigitF& dig,
                                         const uint32_t (&gstart)[LbCfg<1 << RB>::DPL],
                                         lb_rsrc st_r, lb_rsrc ga_r, uint32_t* __restrict__ gacc,
                                         uint32_t* __restrict__ status_next,
                                         uint32_t tiles, uint32_t* __restrict__ error_word,
                                         const Hook& hook, uint64_t t_begin = 0) {
  constexpr int RADIX = 1 << RB;
  constexpr int WAVES = BLOCK / GRS_WAVE;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int DPL = LbCfg<RADIX>::DPL;
  constexpr int LANES = LbCfg<RADIX>::LANES;
  constexpr int G = GRS_LB_GROUP;
  static_assert(G <= 255 && static_cast<long>(G) * TILE < (1l << 24), "group accumulator fields");
  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();
  const uint32_t tile_base = tile * TILE;
  const uint32_t valid = (n - tile_base) < static_cast<uint32_t>(TILE) ? (n - tile_base) : TILE;
  const uint32_t pad = TILE - valid;

  GRS_STAMP(0);
  // ---- rank: one returning LDS atomic per item (lane-ordered) ----
  uint32_t rank[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = dig(key[j]);
    rank[j] = (d << 16) | atomicAdd(&sm.cnt[w * RADIX + d], 1u);
  }
  // zero this tile's words of the next pass's status buffer (and its group's accumulators)
  for (uint32_t i = t; i < static_cast<uint32_t>(RADIX); i += BLOCK) {
    status_next[static_cast<size_t>(tile) * RADIX + i] = 0;
    if (tile % G == 0) status_next[static_cast<size_t>(tiles) * RADIX + (tile / G) * RADIX + i] = 0;
  }
  lds_barrier();  // B1
  GRS_STAMP(1);
  if (w != 0) hook();

  uint32_t lstart[DPL], publish[DPL];
  if (w == 0) {
    uint32_t c[WAVES][DPL];
    uint32_t tc[DPL];
#pragma unroll
    for (int e = 0; e < DPL; ++e) tc[e] = 0;
    if (lane < static_cast<uint32_t>(LANES)) {
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        if constexpr (DPL == 4) {
          const uint4 x = *reinterpret_cast<const uint4*>(&sm.cnt[ww * RADIX + lane * 4]);
          c[ww][0] = x.x; c[ww][1] = x.y; c[ww][2] = x.z; c[ww][3] = x.w;
        } else {
          c[ww][0] = sm.cnt[ww * RADIX + lane];
        }
#pragma unroll
        for (int e = 0; e < DPL; ++e) tc[e] += c[ww][e];
      }
    }
    uint32_t lsum = 0;
#pragma unroll
    for (int e = 0; e < DPL; ++e) {
      publish[e] = (lane * DPL + e == dmask) ? tc[e] - pad : tc[e];
      lsum += tc[e];
    }
    if (lane < static_cast<uint32_t>(LANES)) {
      uint32_t pv[DPL];
#pragma unroll
      for (int e = 0; e < DPL; ++e)
        pv[e] = ((tile == 0 ? GRS_FLAG_INCLUSIVE : GRS_FLAG_AGGREGATE) << GRS_FLAG_SHIFT) | publish[e];
      lb_st<DPL>(st_r, tile * RADIX + lane * DPL, pv);
      // group accumulators: (1 << 24) | count, one no-return atomic per digit
#pragma unroll
      for (int e = 0; e < DPL; ++e)
        __hip_atomic_fetch_add(gacc + (tile / G) * RADIX + lane * DPL + e, (1u << 24) | publish[e],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // exclusive wave scan of the lane sums -> tile-local start of each digit
    uint32_t incl = lsum;
#pragma unroll
    for (int o = 1; o < GRS_WAVE; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, GRS_WAVE);
      if (lane >= static_cast<uint32_t>(o)) incl += y;
    }
    uint32_t run = incl - lsum;
#pragma unroll
    for (int e = 0; e < DPL; ++e) {
      lstart[e] = run;
      run += tc[e];
    }
    if (lane < static_cast<uint32_t>(LANES)) {
      uint32_t colrun[DPL];
#pragma unroll
      for (int e = 0; e < DPL; ++e) colrun[e] = lstart[e];
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        if constexpr (DPL == 4) {
          *reinterpret_cast<uint4*>(&sm.cnt[ww * RADIX + lane * 4]) =
              make_uint4(colrun[0], colrun[1], colrun[2], colrun[3]);
        } else {
          sm.cnt[ww * RADIX + lane] = colrun[0];
        }
#pragma unroll
        for (int e = 0; e < DPL; ++e) colrun[e] += c[ww][e];
      }
    }
  }
  lds_barrier();  // B2
  GRS_STAMP(2);

  Lb2<RADIX, DPL> lb;
  if (w == 0 && tile != 0 && lane < static_cast<uint32_t>(LANES)) lb.issue(st_r, tile, lane);

  // ---- reorder the tile in LDS by (digit, input order) ----
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = rank[j] >> 16;
    const uint32_t pos = sm.cnt[w * RADIX + d] + (rank[j] & 0xFFFFu);
    sm.keys[pos] = key[j];
    if constexpr (PAIRS) sm.vals[pos] = val[j];
  }

  if (w == 0 && lane < static_cast<uint32_t>(LANES)) {
    uint32_t prefix[DPL];
#pragma unroll
    for (int e = 0; e < DPL; ++e) prefix[e] = 0;
    if (tile != 0) {
      lb.finish(st_r, ga_r, lane, error_word);
      uint32_t iv[DPL];
#pragma unroll
      for (int e = 0; e < DPL; ++e) {
        prefix[e] = lb.prefix[e];
        iv[e] = (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) | ((prefix[e] + publish[e]) & GRS_VALUE_MASK);
      }
      lb_st<DPL>(st_r, tile * RADIX + lane * DPL, iv);
    }
#pragma unroll
    for (int e = 0; e < DPL; ++e) sm.base[lane * DPL + e] = gstart[e] + prefix[e] - lstart[e];
  }
  if (w == 0) hook();
  lds_barrier();  // B3
  GRS_STAMP(3);
  for (uint32_t i = t; i < static_cast<uint32_t>(WAVES * RADIX); i += BLOCK) sm.cnt[i] = 0;

  // ---- store: consecutive threads write consecutive slots of each digit run ----
  if (valid == static_cast<uint32_t>(TILE)) {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const uint32_t i = k * BLOCK + t;
      const K kk = sm.keys[i];
      const uint32_t dst = sm.base[dig(kk)] + i;
      keys_out[dst] = kk;
      if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
    }
  } else {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
      const uint32_t i = k * BLOCK + t;
      if (i < valid) {
        const K kk = sm.keys[i];
        const uint32_t dst = sm.base[dig(kk)] + i;
        keys_out[dst] = kk;
        if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
      }
    }
  }
  if constexpr ((DBG & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GRS_STAMP(5);
  }
}

// gstart for the look-back lanes of wave 0: exclusive scan of the pass histogram
template <int RADIX>
__device__ __forceinline__ void pass_starts(const uint32_t* __restrict__ pass_hist, uint32_t lane,
                                            uint32_t (&gs)[LbCfg<RADIX>::DPL]) {
  constexpr int DPL = LbCfg<RADIX>::DPL;
  uint32_t h[DPL], s = 0;
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    h[e] = lane * DPL + e < static_cast<uint32_t>(RADIX) ? pass_hist[lane * DPL + e] : 0u;
    s += h[e];
  }
  uint32_t incl = s;
#pragma unroll
  for (int o = 1; o < GRS_WAVE; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, GRS_WAVE);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  uint32_t run = incl - s;
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    gs[e] = run;
    run += h[e];
  }
}

// One tile per workgroup (grid = number of tiles).  Status buffer layout per pass:
// [tiles][RADIX] tile words, then [ceil(tiles / G)][RADIX] group accumulators.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK) void grs_onesweep_ar2(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  using SM = Ar2Smem<K, PAIRS, RB, BLOCK, ITEMS>;
  constexpr int RADIX = SM::RADIX;
  constexpr int DPL = LbCfg<RADIX>::DPL;
  __shared__ SM sm;
  const uint64_t t_begin = (DBG & 8) ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t t = threadIdx.x;
  const uint32_t tiles = (n + SM::TILE - 1) / SM::TILE;
  const uint32_t groups = (tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP;
  if (t == 0) sm.ticket[0] = atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < static_cast<uint32_t>(SM::WAVES * RADIX); i += BLOCK) sm.cnt[i] = 0;
  uint32_t gs[DPL];
  if (t < GRS_WAVE) pass_starts<RADIX>(pass_hist, t, gs);
  const lb_rsrc st_r = make_rsrc(status, (tiles + groups) * RADIX * 4u);
  const lb_rsrc ga_r = make_rsrc(status + static_cast<size_t>(tiles) * RADIX, groups * RADIX * 4u);
  __syncthreads();
  const uint32_t tile = sm.ticket[0];
  K key[ITEMS];
  uint32_t val[ITEMS];
  load_tile<K, PAIRS, BLOCK, ITEMS>(keys_in, vals_in, n, tile, key, val);
  ar2_tile<K, PAIRS, RB, BLOCK, ITEMS, DBG>(sm, key, val, tile, keys_out, vals_out, n, dig, gs,
                                            st_r, ga_r, status + static_cast<size_t>(tiles) * RADIX,
                                            status_next, tiles, error_word, NoHook(), t_begin);
}

// ----------------------------------------------------------------------------------------
// v3 onesweep pass (u32 keys below 12 tiles of 36K keys per CU, or GRS_U32_PASS=v3): persistent workgroups, LDS-DMA double-buffered
// tiles, ranking by lane-ordered LDS atomics, hierarchical look-back overlapped with the
// LDS reorder
// ----------------------------------------------------------------------------------------
//
// Why (tools/lab.py on MI355X, 2^27 uniform u32 keys):
//  * ballot-match ranking costs ~40 VALU per item.  ONE returning LDS atomic per item on the
//    wave's digit counter replaces it: the LDS serialises the lanes of one wave-instruction
//    that hit one address in ascending lane order, so the returned count IS the stable rank
//    (probed by tools/ldsorder.hip, and at sorter creation by grs_capi.hip, which falls back
//    to the ballot-match pass above if the probe fails);
//  * a tile's keys arrive ~3 us after they are requested under full streaming: the next tile
//    is DMA'd (global_load_lds) into the second LDS buffer while the current one is processed;
//  * a plain decoupled look-back walked 100+ predecessor words per digit: a poll round trip
//    is 1-3 us under streaming (it queues behind the CU's own traffic) while hundreds of tiles
//    start per round trip, so the inclusive frontier lags far behind.  HierLookback below
//    reads < 2G + 2SW words per digit in one round.
//
// Status buffer of one pass (uint32 words, all zero at pass start):
//   [tiles][R] tile AGGREGATE words, [groups][R] group accumulators,
//   [supers][R] supergroup accumulators, [supers][R] supergroup INCLUSIVE words
// A pass zeroes its tiles' and groups' words of the OTHER buffer for the next pass; the
// histogram kernel zeroes the first pass's buffer.

// bounded spin step: sleeps and returns true, or raises the error word and returns false
__device__ __forceinline__ bool spin_ok(uint32_t& spins, uint32_t* error_word) {
  if (++spins > GRS_SPIN_LIMIT) {
    atomicOr(error_word, 1u);
    return false;
  }
  __builtin_amdgcn_s_sleep(1);
  return true;
}

// Words of one status buffer: tile words + group + 2 x supergroup words (per digit).
__host__ __device__ constexpr size_t hier_status_words(size_t tiles, size_t radix) {
  return (tiles + (tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP +
          2 * ((tiles + GRS_LB_GROUP * GRS_LB_GROUP - 1) / (GRS_LB_GROUP * GRS_LB_GROUP))) *
         radix;
}

// Hierarchical look-back of one digit.  Levels: tile -> group (G tiles) -> supergroup (G*G
// tiles).  Every tile publishes its AGGREGATE word and adds (1 << 24) | count into its
// group's and its supergroup's accumulator (a word whose top byte reads the level's size is
// complete; sums stay < 2^24); the add that completes a supergroup (its returned arrival
// count = tiles in it - 1) publishes the supergroup's INCLUSIVE prefix.  The exclusive prefix
// of tile T = (supergroups before T's: the newest published INCLUSIVE plus the complete
// accumulators after it) + (groups of T's supergroup before T's group) + (tiles of T's
// group before T).  Every word is one 32-bit value written atomically, so no release /
// acquire is needed: a poll that reads an old state polls again.  `issue` sends every load of
// the first round at once; `finish` consumes them (re-polling what is not ready yet).
template <int RADIX>
struct HierLookback {
  static constexpr int G = GRS_LB_GROUP;
  static constexpr int S = G * G;         // tiles per supergroup
  static constexpr int SW = GRS_LB_GWIN;  // supergroups per poll window
  // All polls are agent-coherent (sc1) buffer loads of one status buffer addressed by 32-bit
  // word offsets: base words of each level are wave-uniform, so no 64-bit address per load
  // stays live across the reorder that runs between `issue` and `finish`.
  uint32_t tw[G - 1];                     // own group's earlier tile words, nearest first
  uint32_t gw[G - 1];                     // own supergroup's earlier group accumulators
  uint32_t si[SW], sa[SW];                // supergroup INCLUSIVE words / accumulators
  int32_t ph;                             // next supergroup to consume
  uint32_t ntw, ngw;

  static __device__ __forceinline__ uint32_t ld(lb_rsrc r, uint32_t word) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, word * 4u, 0, 16);
  }
  // word offsets of the levels inside the status buffer (uniform)
  struct Layout {
    uint32_t gacc, sacc, sinc;
  };
  __device__ __forceinline__ void load_supers(lb_rsrc r, const Layout& L, uint32_t d) {
#pragma unroll
    for (int k = 0; k < SW; ++k) {
      const int32_t h = ph - k;
      si[k] = h >= 0 ? ld(r, L.sinc + static_cast<uint32_t>(h) * RADIX + d) : 0u;
      sa[k] = h >= 0 ? ld(r, L.sacc + static_cast<uint32_t>(h) * RADIX + d) : 0u;
    }
  }
  __device__ __forceinline__ void issue(lb_rsrc r, const Layout& L, uint32_t tile, uint32_t d) {
    const uint32_t g = tile / G, s = tile / S;
    ntw = tile - g * G;
    ngw = g - s * G;
#pragma unroll
    for (int k = 0; k < G - 1; ++k) {
      tw[k] = static_cast<uint32_t>(k) < ntw ? ld(r, (tile - 1 - k) * RADIX + d) : 0u;
      gw[k] = static_cast<uint32_t>(k) < ngw ? ld(r, L.gacc + (g - 1 - k) * RADIX + d) : 0u;
    }
    ph = static_cast<int32_t>(s) - 1;
    load_supers(r, L, d);
  }
  // Exclusive prefix of digit d over tiles [0, tile).  sold: the value this tile's returning
  // add to its supergroup accumulator saw; publish: this tile's count of digit d.
  __device__ __forceinline__ uint32_t finish(lb_rsrc r, const Layout& L, uint32_t* sinc,
                                             uint32_t tile, uint32_t tiles, uint32_t d,
                                             uint32_t sold, uint32_t publish,
                                             uint32_t* error_word, uint32_t* stats = nullptr) {
    uint32_t spins = 0, low = 0, rounds = 1;
    const uint32_t g = tile / G;
#pragma unroll
    for (int k = 0; k < G - 1; ++k) {
      if (static_cast<uint32_t>(k) < ntw) {
        uint32_t v = tw[k];
        while ((v >> GRS_FLAG_SHIFT) == GRS_FLAG_NOT_READY && spin_ok(spins, error_word))
          v = ld(r, (tile - 1 - k) * RADIX + d);
        low += v & GRS_VALUE_MASK;
      }
      if (static_cast<uint32_t>(k) < ngw) {
        uint32_t v = gw[k];
        while ((v >> 24) != static_cast<uint32_t>(G) && spin_ok(spins, error_word))
          v = ld(r, L.gacc + (g - 1 - k) * RADIX + d);
        low += v & 0xFFFFFFu;
      }
    }
    uint32_t hi = 0;
    while (ph >= 0) {
      int consumed = 0;
      bool done = false, blocked = false;
#pragma unroll
      for (int k = 0; k < SW; ++k) {
        if (!done && !blocked && ph - k >= 0) {
          if ((si[k] >> GRS_FLAG_SHIFT) == GRS_FLAG_INCLUSIVE) {
            hi += si[k] & GRS_VALUE_MASK;
            done = true;
          } else if ((sa[k] >> 24) == static_cast<uint32_t>(S)) {
            hi += sa[k] & 0xFFFFFFu;
            ++consumed;
          } else {
            blocked = true;
          }
        }
      }
      if (done) break;
      ph -= consumed;
      if (ph < 0) break;
      if (consumed == 0 && !spin_ok(spins, error_word)) break;
      ++rounds;
      load_supers(r, L, d);
    }
    const uint32_t s = tile / S;
    const uint32_t in_super = min(static_cast<uint32_t>(S), tiles - s * S);
    if ((sold >> 24) == in_super - 1)
      st_status(sinc + static_cast<size_t>(s) * RADIX + d,
                (GRS_FLAG_INCLUSIVE << GRS_FLAG_SHIFT) |
                    ((hi + (sold & 0xFFFFFFu) + publish) & GRS_VALUE_MASK));
    if (stats) {  // lab only: per tile max over digits of poll rounds / spins
      atomicMax(stats + 0, rounds);
      atomicMax(stats + 1, spins);
    }
    return hi + low;
  }
};

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS>
struct V3Smem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  uint32_t cnt[WAVES * RADIX];  // per-wave digit counters -> tile positions
  uint32_t base[RADIX];         // global destination of tile position 0 of digit d
  uint32_t wsum[WAVES];
  uint32_t ticket[2];
  alignas(16) K kbuf[2][TILE];
  alignas(16) uint32_t vbuf[PAIRS ? 2 : 1][PAIRS ? TILE : 4];
};

// Persistent grid (one or two workgroups per CU).  Per iteration on tile `cur` (LDS buffer b):
// Tile DMA cache policy: nontemporal unless DBG & 128.  nt made the pass alone 1-3 % faster
// (tools/lab.py) but the sort slower (the next histogram launch absorbs more dirty lines:
// tools/ab_v3_dma.sh), so the library launches the DBG = 128 instance unless GRS_V3_DMA=nt.
// The scatter stores keep the default policy: partial lines of neighbouring digit runs merge
// in L2 (nt stores measured 1.8x slower).
//   L0   wait for this wave's DMA of `cur` (a counted vmcnt that skips the previous tile's
//        stores), barrier; keys -> registers, wave-striped: item j of lane l of wave w is key
//        w*64*ITEMS + j*64 + l, so ranking items in (j, lane) order is input order
//   rank one returning ds_add per key on the wave's digit counter; take the next ticket
//   B1   digit threads: wave starts + tile count, AGGREGATE word, group / supergroup adds,
//        scan over digits
//   B2   digit threads: fold the tile-local starts into the counters, issue the first
//        look-back round; the ticket of the next tile lands
//   B2.5 waves without a digit start the DMA of `nxt` into buffer b^1; all waves reorder the
//        tile into buffer b by (digit, input order); digit threads finish the look-back and
//        write the digit bases, then their waves start their part of the DMA
//   B3   stores: consecutive threads write consecutive slots of each digit run
// A workgroup takes tickets in increasing order and only ever waits on smaller tiles, and
// every tile publishes its counts before waiting on anything, so the grid always progresses.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int DBG = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, 4) void grs_onesweep_v3(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word) {
  using SM = V3Smem<K, PAIRS, RB, BLOCK, ITEMS>;
  constexpr int RADIX = SM::RADIX;
  constexpr int WAVES = SM::WAVES;
  constexpr int TILE = SM::TILE;
  constexpr int WAVE_TILE = GRS_WAVE * ITEMS;
  constexpr int LB_WAVES = (RADIX + GRS_WAVE - 1) / GRS_WAVE;
  constexpr int G = GRS_LB_GROUP;
  constexpr int S = G * G;
  constexpr int NST = ITEMS * (PAIRS ? 2 : 1);  // global stores a wave issues after its DMA
  static_assert(NST <= 63, "vmcnt field");
  static_assert(RADIX <= BLOCK && LB_WAVES < WAVES, "digit waves plus a ticket wave");
  static_assert(S <= 255 && static_cast<long>(S) * TILE < (1l << 24), "accumulator fields");
  __shared__ SM sm;

  const uint32_t t = threadIdx.x;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t dmask = dig.max_digit();
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const uint32_t full_tiles = n / TILE;
  const uint32_t groups = (tiles + G - 1) / G;
  const uint32_t supers = (tiles + S - 1) / S;
  uint32_t* gacc = status + static_cast<size_t>(tiles) * RADIX;
  uint32_t* sacc = gacc + static_cast<size_t>(groups) * RADIX;
  uint32_t* sinc = sacc + static_cast<size_t>(supers) * RADIX;
  uint32_t* gacc_next = status_next + static_cast<size_t>(tiles) * RADIX;
  uint32_t* sacc_next = gacc_next + static_cast<size_t>(groups) * RADIX;
  uint32_t* sinc_next = sacc_next + static_cast<size_t>(supers) * RADIX;
  const lb_rsrc st_r = make_rsrc(status, (tiles + groups + 2 * supers) * RADIX * 4u);
  const typename HierLookback<RADIX>::Layout lay{tiles * RADIX, (tiles + groups) * RADIX,
                                                 (tiles + groups + supers) * RADIX};
  constexpr uint32_t TK_THREAD = BLOCK - GRS_WAVE;  // lane 0 of the last wave (no digit)

  uint32_t tk = 0;  // TK_THREAD: ticket of the next tile (taken after ranking, lands at B2)
  // lab: DBG & 512 = static XCD-chunked order (needs DBG & 1): block b of label x = b % 8
  // walks tiles x * tpc + b / 8, + gridDim / 8, ... so consecutive tiles share an XCD
  const uint32_t tpc = (((n + TILE - 1) / TILE) + 7) / 8;
  const uint32_t chunk_end = min((blockIdx.x % 8 + 1) * tpc, (n + TILE - 1) / TILE);
  if (t == TK_THREAD)
    sm.ticket[0] = (DBG & 512) ? (blockIdx.x % 8) * tpc + blockIdx.x / 8
                   : (DBG & 64) ? blockIdx.x : atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < static_cast<uint32_t>(WAVES * RADIX); i += BLOCK) sm.cnt[i] = 0;
  // global start of digit t in this pass: exclusive scan of the pass histogram
  uint32_t gstart = 0;
  {
    const uint32_t h = t < static_cast<uint32_t>(RADIX) ? pass_hist[t] : 0u;
    uint32_t incl = h;
#pragma unroll
    for (int o = 1; o < GRS_WAVE; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, GRS_WAVE);
      if (lane >= static_cast<uint32_t>(o)) incl += y;
    }
    if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
    __syncthreads();
    gstart = incl - h;
    for (uint32_t ww = 0; ww < w; ++ww) gstart += sm.wsum[ww];
  }
  __syncthreads();
  uint32_t cur = sm.ticket[0];
  if (cur < full_tiles) dma_tile<K, PAIRS, BLOCK, ITEMS, (DBG & 128) == 0>(keys_in, vals_in, cur, sm.kbuf[0], sm.vbuf[0]);
  bool prev_full_stores = false;  // previous iteration issued NST stores after its DMA
  int b = 0;

#define V3_STAMP(k)                                                                        \
  do {                                                                                     \
    if constexpr ((DBG & 8) != 0) {                                                        \
      if (t == 0)                                                                          \
        error_word[64 + static_cast<size_t>(cur) * 8 + (k)] =                              \
            static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t_it);                    \
    }                                                                                      \
  } while (0)
  while (cur < tiles) {
    const uint64_t t_it = (DBG & 8) ? __builtin_amdgcn_s_memtime() : 0;
    // ---- L0 ----
    if (prev_full_stores)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    V3_STAMP(0);
    const uint32_t tile_base = cur * TILE;
    const bool full = cur < full_tiles;
    const uint32_t valid = full ? TILE : n - tile_base;
    const uint32_t pad = TILE - valid;
    K* kr = sm.kbuf[b];
    uint32_t* vr = sm.vbuf[PAIRS ? b : 0];
    if (!full) {  // the ragged last tile: staged with plain loads, padding = all-ones keys
      for (uint32_t i = t; i < static_cast<uint32_t>(TILE); i += BLOCK) {
        kr[i] = i < valid ? keys_in[tile_base + i] : static_cast<K>(~static_cast<K>(0));
        if constexpr (PAIRS) vr[i] = i < valid ? vals_in[tile_base + i] : 0u;
      }
      lds_barrier();
    }
    K key[ITEMS];
    uint32_t val[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = kr[w * WAVE_TILE + j * GRS_WAVE + lane];
    if constexpr (PAIRS) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) val[j] = vr[w * WAVE_TILE + j * GRS_WAVE + lane];
    }

    // ---- rank: one returning LDS atomic per item (lane-ordered) ----
    uint32_t rank[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t d = dig(key[j]);
      rank[j] = (d << 16) | atomicAdd(&sm.cnt[w * RADIX + d], 1u);
    }
    // zero this tile's (and its group's / supergroup's) words for the next pass
    for (uint32_t i = t; i < static_cast<uint32_t>(RADIX); i += BLOCK) {
      status_next[static_cast<size_t>(cur) * RADIX + i] = 0;
      if (cur % G == 0) gacc_next[static_cast<size_t>(cur / G) * RADIX + i] = 0;
      if (cur % S == 0) {
        sacc_next[static_cast<size_t>(cur / S) * RADIX + i] = 0;
        sinc_next[static_cast<size_t>(cur / S) * RADIX + i] = 0;
      }
    }
    // The next tile's ticket is taken only now, one iteration before that tile is counted: a
    // tile whose ticket is held but whose counts are not published yet stalls every later
    // tile's look-back, so tickets are never taken further ahead.
    if (t == TK_THREAD)
      tk = (DBG & 512)  ? (cur + gridDim.x / 8 < chunk_end ? cur + gridDim.x / 8 : tiles)
           : (DBG & 64) ? cur + gridDim.x : atomicAdd(ticket, 1u);
    lds_barrier();  // B1
    V3_STAMP(1);

    // ---- digit threads: wave starts, tile count, publish, scan over digits ----
    uint32_t tile_cnt = 0, publish = 0, sold = 0, excl = 0;
    if (t < static_cast<uint32_t>(RADIX)) {
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        const uint32_t c = sm.cnt[ww * RADIX + t];
        sm.cnt[ww * RADIX + t] = tile_cnt;
        tile_cnt += c;
      }
      publish = (t == dmask) ? tile_cnt - pad : tile_cnt;  // padding is ranked, never counted
      st_status(status + static_cast<size_t>(cur) * RADIX + t,
                (GRS_FLAG_AGGREGATE << GRS_FLAG_SHIFT) | publish);
      __hip_atomic_fetch_add(gacc + static_cast<size_t>(cur / G) * RADIX + t, (1u << 24) | publish,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sold = __hip_atomic_fetch_add(sacc + static_cast<size_t>(cur / S) * RADIX + t,
                                    (1u << 24) | publish, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
    }
    if (w < static_cast<uint32_t>(LB_WAVES)) {
      uint32_t incl = tile_cnt;
#pragma unroll
      for (int o = 1; o < GRS_WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, GRS_WAVE);
        if (lane >= static_cast<uint32_t>(o)) incl += y;
      }
      if (lane == GRS_WAVE - 1) sm.wsum[w] = incl;
      excl = incl - tile_cnt;
    }
    lds_barrier();  // B2
    V3_STAMP(2);

    HierLookback<RADIX> lb;
    uint32_t local_start = 0;
    if (t < static_cast<uint32_t>(RADIX)) {
      for (uint32_t ww = 0; ww < w; ++ww) excl += sm.wsum[ww];
      local_start = excl;
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) sm.cnt[ww * RADIX + t] += local_start;
      if constexpr ((DBG & 32) != 0) lb.issue(st_r, lay, cur, t);  // lab: in flight during the reorder
    }
    if (t == TK_THREAD) sm.ticket[1] = tk;  // before this wave's DMA (vmcnt accounting)
    lds_barrier();  // B2.5
    V3_STAMP(3);

    const uint32_t nxt = sm.ticket[1];
    const bool nxt_full = nxt < full_tiles;
    if (w >= static_cast<uint32_t>(LB_WAVES) && nxt_full)
      dma_tile<K, PAIRS, BLOCK, ITEMS, (DBG & 128) == 0>(keys_in, vals_in, nxt, sm.kbuf[b ^ 1], sm.vbuf[PAIRS ? (b ^ 1) : 0]);
    // ---- reorder into the current buffer (its keys are in registers) ----
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t d = rank[j] >> 16;
      const uint32_t pos = sm.cnt[w * RADIX + d] + (rank[j] & 0xFFFFu);
      kr[pos] = key[j];
      if constexpr (PAIRS) vr[pos] = val[j];
    }
    if (t < static_cast<uint32_t>(RADIX)) {
      // issued after the reorder: overlapping it (DBG & 32) keeps 30 more VGPRs live through
      // the reorder and spills at 4 waves per SIMD
      uint32_t prefix;
      if constexpr ((DBG & 1) != 0) {  // lab: no look-back (uniform-data estimate)
        prefix = cur * static_cast<uint32_t>(TILE / RADIX);
      } else {
        if constexpr ((DBG & 32) == 0) lb.issue(st_r, lay, cur, t);
        uint32_t* stats = (DBG & 16) ? error_word + 64 + static_cast<size_t>(cur) * 8 : nullptr;
        prefix = lb.finish(st_r, lay, sinc, cur, tiles, t, sold, publish, error_word, stats);
      }
      sm.base[t] = gstart + prefix - local_start;
    }
    if (w < static_cast<uint32_t>(LB_WAVES) && nxt_full)
      dma_tile<K, PAIRS, BLOCK, ITEMS, (DBG & 128) == 0>(keys_in, vals_in, nxt, sm.kbuf[b ^ 1], sm.vbuf[PAIRS ? (b ^ 1) : 0]);
    lds_barrier();  // B3
    V3_STAMP(4);
    for (uint32_t i = t; i < static_cast<uint32_t>(WAVES * RADIX); i += BLOCK) sm.cnt[i] = 0;

    // ---- store ----
    if (full) {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        const K kk = kr[i];
        uint32_t dst = sm.base[dig(kk)] + i;
        if constexpr ((DBG & 1) != 0) dst = min(dst, n - 1);   // lab: estimated bases
        if constexpr ((DBG & 2) != 0) dst = tile_base + i;     // lab: contiguous stores
        if constexpr ((DBG & 256) != 0) {                       // lab: nontemporal stores
          __builtin_nontemporal_store(kk, &keys_out[dst]);
        } else {
          keys_out[dst] = kk;
        }
        if constexpr (PAIRS) vals_out[dst] = vr[i];
      }
    } else {
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        if (i < valid) {
          const K kk = kr[i];
          const uint32_t dst = sm.base[dig(kk)] + i;
          keys_out[dst] = kk;
          if constexpr (PAIRS) vals_out[dst] = vr[i];
        }
      }
    }
    if constexpr ((DBG & 8) != 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      V3_STAMP(5);
    }
    prev_full_stores = full && nxt_full;
    cur = nxt;
    b ^= 1;
  }
#undef V3_STAMP
}


}  // namespace grs
