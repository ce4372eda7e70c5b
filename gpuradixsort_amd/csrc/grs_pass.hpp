// grs_pass.hpp — the LSD pass kernel of libgrs (one launch per digit), gfx950.
//
// Replaces one bit-iteration of the reference's pass loop (ParallelSort.cpp:236-298): K2
// (GetBitForPrefixScan.comp:25-68) + K3a/K3b (ParallelPrefixScan.comp:41-196) + K4
// (SortIntermediateData.comp:32-67), i.e. "extract the digit, scan it within the group and
// over the groups, scatter stably", for a whole RB-bit digit in ONE launch:
//
//   ticket   tile id from an atomic counter: tiles start in id order, so a tile only ever
//            waits on tiles that already started (no forward-progress assumption)
//   load     the tile, wave-striped into registers (item j of lane l of wave w is tile key
//            w*64*ITEMS + j*64 + l): ranking items in (j, lane) order visits input order
//   rank     ONE returning LDS add per key on its wave's digit counter: the LDS serialises the
//            lanes of one wave-instruction that hit one address in ascending lane order, so
//            the returned count is the key's stable rank among its wave's keys of that digit
//            (probed at sorter creation; the ballot-match fallback is OPT 512 below)
//   B1       digit threads: wave starts (column scan), tile count, publish the count, add it
//            into the group accumulator; wave scans over digits (tile and pass starts)
//   B2       tile-local digit starts folded into the wave counters; look-back polls ISSUED
//   B3       all waves reorder the tile in LDS by (digit, input order); the digit threads
//            then FINISH the look-back (its round trip overlapped the reorder) and write the
//            global base of each digit
//   B4       stores: consecutive threads write consecutive slots of each digit run
//
// The variants measured and rejected in rounds 2-3 (XCD ranges, wide look-back, aligned or
// nontemporal stores, ticketless tiles, other persistent schedules, phase stamps) live in
// the round 2-4 lab fork (git show 729d494:tools/lab_pass.hpp, removed in round 5); this file holds
// what libgrs launches.
#pragma once

#include <type_traits>

#include "grs_kernels.hpp"

namespace grs {

// Look-back status of one pass (uint32 words, all zero at pass start):
//   tile words   [tiles][R]   count + 1 of the tile's digit (0 = not published yet)
//   group accs   [groups][R]  (arrivals << 24) | sum of the group's tile counts
//   group incl   [groups][R]  inclusive prefix of the group + 1 (0 = not published yet),
//                             written by the tile whose add completes the accumulator
// Values are stored +1 so that no flag bits are needed: prefixes reach n (< 2^32).
__host__ __device__ constexpr size_t lb3_status_words(size_t tiles, size_t radix) {
  return (tiles + 2 * ((tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP)) * radix;
}

// Debug words after the sticky error word (grs_set_option(GRS_OPT_FAULT_TILE), tests only):
//   error_word[1]  tile + 1 whose tile words are never published (0 = none): every later tile
//                  of its look-back group spins on them until the bound
//   error_word[2]  the spin bound (0 = GRS_SPIN_LIMIT)
struct PassDebug {
  uint32_t fault_tile1;
  uint32_t spin_limit;
  __device__ __forceinline__ static PassDebug read(const uint32_t* error_word) {
    const uint32_t lim = error_word[2];
    return PassDebug{error_word[1], lim != 0u ? lim : static_cast<uint32_t>(GRS_SPIN_LIMIT)};
  }
};

// Exclusive prefix of digit d over tiles [0, tile): own group's earlier tiles (< G words)
// plus the group-level prefix (newest published group INCLUSIVE + complete accumulators
// after it).  issue() sends the first round of loads, finish() consumes them.
// GW: groups polled per round.  The two-round (XL) tiles use 4: the window's registers are
// live across the reorder there, beside the tile's keys and positions.
template <int RADIX, int GW = GRS_LB_GWIN>
struct Lb3 {
  static constexpr int G = GRS_LB_GROUP;
  uint32_t tw[G - 1];
  uint32_t gi[GW], ga[GW];
  int32_t ph;

  int32_t g0;   // first group of the tile's segment (0 for an ordinary pass): the chain stops there

  __device__ __forceinline__ void load_groups(const uint32_t* gacc, const uint32_t* ginc,
                                              uint32_t d) {
#pragma unroll
    for (int k = 0; k < GW; ++k) {
      const int32_t h = ph - k;
      gi[k] = h >= g0 ? ld_status(ginc + static_cast<size_t>(h) * RADIX + d) : 0u;
      ga[k] = h >= g0 ? ld_status(gacc + static_cast<size_t>(h) * RADIX + d) : 0u;
    }
  }
  // tile: the tile's word row; jg: its place in its look-back group (the group's earlier tiles
  // are rows tile - jg .. tile - 1); group: its group; group0: the first group of its segment
  // (0 for an ordinary pass), where the chain stops.  Segmented passes start every segment on
  // a new group, so a group never holds tiles of two segments.
  __device__ __forceinline__ void issue(const uint32_t* status, const uint32_t* gacc,
                                        const uint32_t* ginc, uint32_t tile, uint32_t d,
                                        uint32_t jg, uint32_t group, uint32_t group0) {
    const uint32_t first = tile - jg;
#pragma unroll
    for (int k = 0; k < G - 1; ++k)
      tw[k] = static_cast<uint32_t>(k) < jg ? ld_status(status + static_cast<size_t>(first + k) * RADIX + d) : 1u;
    ph = static_cast<int32_t>(group) - 1;
    g0 = static_cast<int32_t>(group0);
    load_groups(gacc, ginc, d);
  }
  // gold: the value this tile's add to its group accumulator returned; publish: its count;
  // in_group: the tiles of its group (G but in a segment's last group).
  // A spin that exceeds `limit` polls sets the error word and counts the word as 0: prefixes
  // can then only come out SMALLER than the true ones (onesweep_tile clamps the runs to
  // [0, n) for the passes after such a one).
  __device__ __forceinline__ uint32_t finish(const uint32_t* status, const uint32_t* gacc,
                                             uint32_t* ginc, uint32_t tile, uint32_t jg,
                                             uint32_t group, uint32_t in_group,
                                             uint32_t d, uint32_t gold, uint32_t publish,
                                             uint32_t* error_word, uint32_t limit) {
    const uint32_t first = tile - jg;
    uint32_t spins = 0, own = 0;
#pragma unroll
    for (int k = 0; k < G - 1; ++k) {
      uint32_t v = tw[k];
      while (v == 0u) {
        if (++spins > limit) {
          atomicOr(error_word, 1u);
          v = 1u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = ld_status(status + static_cast<size_t>(first + k) * RADIX + d);
      }
      own += v - 1u;
    }
    uint32_t gp = 0;
    while (ph >= g0) {
      int consumed = 0;
      bool done = false, blocked = false;
#pragma unroll
      for (int k = 0; k < GW; ++k) {
        if (!done && !blocked && ph - k >= g0) {
          if (gi[k] != 0u) {
            gp += gi[k] - 1u;
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
      if (ph < g0) break;
      if (consumed == 0) {
        if (++spins > limit) {
          atomicOr(error_word, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      load_groups(gacc, ginc, d);
    }
    if ((gold >> 24) == in_group - 1u)   // this tile's add completed the group
      st_status(ginc + static_cast<size_t>(group) * RADIX + d, gp + (gold & 0xFFFFFFu) + publish + 1u);
    return gp + own;
  }
};

// Where one tile of a pass lies, and its place in the look-back status layout
// [tiles][R] tile words, [groups][R] group accumulators, [groups][R] group inclusives.
// Ordinary pass: tile = ticket, the pass is one segment [0, n), groups of G consecutive tiles.
// Segmented pass (grs_onesweep_seg): tiles never straddle a segment and every segment starts a
// new group, so its chain restarts at its first group and its digit runs start at the
// segment's own base.
#ifdef GRS_DIAG
// Diagnostic builds only (tools/diag): bounds the host sets before a launch (0 = unchecked) --
// [0] output elements, [1] input elements, [2] status words -- and what broke them: [0] bad
// stores, [1] the largest bad store index, [2] bad loads, [3] the largest bad load index, [4]
// tiles whose status layout passes the bound, [5] 1 + the first such tile row.
__device__ uint32_t diag_lim[4];
__device__ uint32_t diag_hit[24];   // [8..] the first digit run past the bound: see onesweep_tile
#endif

struct TileSpan {
  uint32_t tile;       // tile word row (the ticket)
  uint32_t tiles;      // tile rows of the layout
  uint32_t group;      // the tile's look-back group
  uint32_t groups;     // groups of the layout
  uint32_t jg;         // place of the tile in its group
  uint32_t in_group;   // tiles of its group
  uint32_t g0;         // first group of the tile's segment
  uint32_t base;       // index of the tile's first key
  uint32_t valid;      // keys in the tile (<= TILE)
  uint32_t seg_start;  // first index of the tile's segment
  uint32_t seg_len;    // keys in the segment (region passes: the room its runs may take)
  bool solo;           // segmented pass: the segment's only tile -- no status words, no
                       // look-back, its own counts are the segment's
  bool last;           // the segment's last tile (region passes write the digit totals)
  __device__ __forceinline__ static TileSpan whole(uint32_t tile, uint32_t n, uint32_t TILE) {
    constexpr uint32_t G = GRS_LB_GROUP;
    const uint32_t tiles = n / TILE + (n % TILE != 0u ? 1u : 0u);
    const uint32_t b = tile * TILE;
    const uint32_t g = tile / G;
    return TileSpan{tile, tiles, g, (tiles + G - 1) / G, tile % G, min(G, tiles - g * G), 0u,
                    b, (n - b) < TILE ? (n - b) : TILE, 0u, n, false, tile + 1u == tiles};
  }
};

// One tile of a segmented pass, as the planner (grs_seg_plan, grs_msd.hpp) lays it out.
struct SegTile {
  uint32_t row;        // tile word row of the status layout (solo tiles: none)
  uint32_t group;      // look-back group of the tile
  uint32_t flags;      // place in the group (bits 0-3) | tiles of the group (4-7) | solo (8)
                       // | the group's place in its segment (9-30) | last tile of its
                       // segment (31)
  uint32_t base;       // first key of the tile
  uint32_t valid;      // keys in the tile
  uint32_t seg_start;  // first key of the segment
  uint32_t seg_len;    // keys in the segment
  uint32_t seg;        // histogram row of the segment
};

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, bool CNT16 = false,
          bool IDX = false, int ROUNDS = 1>
struct V4Smem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE;
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr int LTILE = TILE / ROUNDS;   // reordered positions held at once
  // per-wave digit counters -> tile position of (wave, digit); CNT16: 16-bit, two per word
  uint32_t cnt[WAVES * RADIX / (CNT16 ? 2 : 1)];
  uint32_t base[RADIX];         // global destination of tile position 0 of digit d
  uint32_t wsum[2 * WAVES];     // wave totals of the digit scans
  uint32_t ticket;
  uint32_t next;                // persistent kernel: the next tile's ticket
  uint32_t span[4];             // OPT 262144: OR of the tile's keys (lo, hi), OR of their complements
  alignas(16) K keys[LTILE];
  uint32_t vals[PAIRS ? LTILE : 1];
  // indexed digits (partition): tile-local start of every digit, from which the store phase
  // reads off the digit of a reordered position (the key alone does not determine it), and per
  // 64-position chunk the digits of its first and last position (first | last << 8)
  uint32_t lstart[IDX ? RADIX + 1 : 1];
  uint16_t cdig[IDX ? TILE / GRS_WAVE : 1];
};
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int OPT, typename DigitF>
using V4SmemFor = V4Smem<K, PAIRS, RB, BLOCK, ITEMS, (OPT & 256) != 0, DigitF::kIndexed,
                         (OPT & 1024) != 0 ? 2 : 1>;

// OPT bits of the shipped pass (grs_capi.hip picks them per shape; 131072 = region pass, set by
// grs_onesweep_region only):
//   16   look-back issued after the reorder (default: before it, overlapped with nothing)
//   256  16-bit wave counters (two digits per LDS word: half the counter LDS)
//   512  ballot-match ranking instead of lane-ordered LDS atomics (the fallback when the
//        device probe of the lane order fails, grs_capi.hip)
//   1024 two-round reorder: the keys stay in registers and LDS holds half the tile at a
//        time (positions [0, TILE/2) are reordered and stored, then [TILE/2, TILE)), so a
//        tile can be twice what LDS holds: longer digit runs per tile, fewer partial lines
//   4096 u32 pairs READ as 8-byte (key, value) records from keys_in (vals_in unused)
//   8192 u32 pairs WRITTEN as 8-byte records to keys_out: one digit run of 8-byte records
//        instead of two of 4-byte words, twice as long (fewer partial lines)
//   16384 / 32768: the records read / written are SPLIT over two buffers: records [0, n/2)
//        in keys_in / keys_out and [n/2, n) in vals_in / vals_out (n even; the caller's two
//        4n-byte arrays hold n records that way)
//   262144 span: the ranking also ORs the tile's valid keys and their complements into sm.span
//        (zeroed by the kernel; the MSD sort's first scatter learns the keys' exact bit span)

// Load tile `tile` wave-striped: item j of lane l of wave w is tile key w*64*ITEMS + j*64 + l.
// Keys past n (last tile) are all-ones padding, which sorts after every valid key of its digit.
// The same for the tile whose first key is index `tile_base`, `valid` keys of it in range
// (valid >= TILE: a full tile).
template <typename K, bool PAIRS, int BLOCK, int ITEMS, int OPT>
__device__ __forceinline__ void tile_load_at(K (&key)[ITEMS], uint32_t (&val)[ITEMS],
                                             const K* __restrict__ keys_in,
                                             const uint32_t* __restrict__ vals_in, uint32_t n,
                                             uint32_t tile_base, uint32_t valid, uint32_t t) {
  constexpr uint32_t TILE = BLOCK * ITEMS;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t wbase = tile_base + w * (GRS_WAVE * ITEMS) + lane;
  constexpr bool IN_REC = (OPT & 4096) != 0;
  static_assert(!IN_REC || (PAIRS && sizeof(K) == 4), "records: u32 key + u32 value");
  // tile-local bounds (compare offsets, never global indices: tile_base + TILE can pass 2^32
  // when n is near GRS_MAX_N, and a wrapped index would read as in range)
  const uint32_t lbase = w * (GRS_WAVE * ITEMS) + lane;
  if constexpr (IN_REC) {
    const uint2* rec = reinterpret_cast<const uint2*>(keys_in);
    const uint2* rec_hi = reinterpret_cast<const uint2*>(vals_in);   // split: records [n/2, n)
    const uint32_t half = n / 2;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const bool in = valid >= TILE || lbase + j * GRS_WAVE < valid;
      const uint32_t idx = wbase + j * GRS_WAVE;
      const bool hi = (OPT & 16384) != 0 && idx >= half;
#ifdef GRS_DIAG
      if (in && diag_lim[1] != 0u && idx >= diag_lim[1]) {
        atomicAdd(&diag_hit[2], 1u);
        atomicMax(&diag_hit[3], idx);
        key[j] = static_cast<K>(~0u);
        val[j] = 0u;
        continue;
      }
#endif
      const uint2 x = !in ? make_uint2(~0u, 0u) : hi ? rec_hi[idx - half] : rec[idx];
      key[j] = static_cast<K>(x.x);
      val[j] = x.y;
    }
  } else if (valid >= TILE) {
#ifdef GRS_DIAG
    if (diag_lim[1] != 0u && wbase + (ITEMS - 1) * GRS_WAVE >= diag_lim[1]) {
      atomicAdd(&diag_hit[2], 1u);
      atomicMax(&diag_hit[3], wbase + (ITEMS - 1) * GRS_WAVE);
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        key[j] = static_cast<K>(~static_cast<K>(0));
        val[j] = 0u;
      }
      return;
    }
#endif
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = keys_in[wbase + j * GRS_WAVE];
    if constexpr (PAIRS) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) val[j] = vals_in[wbase + j * GRS_WAVE];
    }
  } else {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const bool in = lbase + j * GRS_WAVE < valid;
      key[j] = in ? keys_in[wbase + j * GRS_WAVE] : static_cast<K>(~static_cast<K>(0));
      if constexpr (PAIRS) val[j] = in ? vals_in[wbase + j * GRS_WAVE] : 0u;
    }
  }
}

template <typename K, bool PAIRS, int BLOCK, int ITEMS, int OPT>
__device__ __forceinline__ void tile_load(K (&key)[ITEMS], uint32_t (&val)[ITEMS],
                                          const K* __restrict__ keys_in,
                                          const uint32_t* __restrict__ vals_in, uint32_t n,
                                          uint32_t tile, uint32_t t) {
  constexpr uint32_t TILE = BLOCK * ITEMS;
  tile_load_at<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile * TILE,
                                            n - tile * TILE, t);
}

// One tile, from its loaded (or in-flight) keys to its stores.  Precondition: sm.cnt is zero
// and every thread passed a barrier since it was written and since the previous tile's last
// LDS access.  Leaves sm.cnt dirty.
// PF (persistent workgroups, grs_onesweep_v6): thread 0 draws the next ticket during the
// ranking; after the reorder has moved this tile into LDS (two-round tiles: once the last
// round sits in LDS), the next tile's loads are issued into key/val — their latency hides
// behind the look-back and the stores.  Returns the next tile (>= tiles: none); without PF
// returns tiles.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int OPT, bool PF = false,
          bool SEG = false, typename DigitF>
__device__ __forceinline__ uint32_t onesweep_tile(
    V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>& sm, const TileSpan sp, K (&key)[ITEMS],
    uint32_t (&val)[ITEMS], const K* __restrict__ keys_in,
    K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF& dig, uint32_t gh,
    uint32_t* __restrict__ ticket, uint32_t* __restrict__ status,
    uint32_t* __restrict__ status_next, uint32_t* __restrict__ error_word, PassDebug dbg,
    uint32_t* __restrict__ digit_starts = nullptr, uint32_t* __restrict__ region_totals = nullptr,
    uint32_t* __restrict__ spill_flag = nullptr) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  constexpr bool C16 = (OPT & 256) != 0;
  constexpr bool MATCH = (OPT & 512) != 0;
  constexpr bool LATE_LB = (OPT & 16) != 0 || PF;
  constexpr int RADIX = SM::RADIX;
  constexpr int WAVES = SM::WAVES;
  constexpr int TILE = SM::TILE;
  constexpr int ROUNDS = TILE / SM::LTILE;
  constexpr int LTILE = SM::LTILE;
  constexpr int LITEMS = ITEMS / ROUNDS;   // store-loop items per round
  static_assert(LITEMS * ROUNDS == ITEMS, "ITEMS divisible by the rounds");
  static_assert(!C16 || TILE < 65536, "16-bit tile positions");
  static_assert(ROUNDS == 1 || TILE <= 65536, "two-round reorder keeps 16-bit positions");
  uint16_t* const c16 = reinterpret_cast<uint16_t*>(sm.cnt);
  constexpr bool IDX = DigitF::kIndexed;
  auto cnt_ld = [&](uint32_t i) -> uint32_t { if constexpr (C16) return c16[i]; else return sm.cnt[i]; };
  auto cnt_st = [&](uint32_t i, uint32_t v) { if constexpr (C16) c16[i] = static_cast<uint16_t>(v); else sm.cnt[i] = v; };
  constexpr int DW = (RADIX + GRS_WAVE - 1) / GRS_WAVE;  // waves holding digit threads
  constexpr int G = GRS_LB_GROUP;
  static_assert(RADIX <= BLOCK, "one digit thread per digit");
  static_assert(static_cast<long>(G) * TILE < (1l << 24), "group accumulator field");
  // opaque per call: keeps the compiler from hoisting ITEMS per-thread addresses out of a
  // persistent loop (they would stay live across the whole tile and spill)
  uint32_t t = threadIdx.x;
  asm volatile("" : "+v"(t));
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t tile = sp.tile;
  const uint32_t tiles = sp.tiles;
  const uint32_t groups = sp.groups;
  const uint32_t tile_base = sp.base;
  const uint32_t valid = sp.valid;
  const uint32_t pad = TILE - valid;
  const uint32_t dmask = dig.max_digit();
  uint32_t* gacc = status + static_cast<size_t>(tiles) * RADIX;
  uint32_t* ginc = gacc + static_cast<size_t>(groups) * RADIX;
#ifdef GRS_DIAG
  if (t == 0 && diag_lim[2] != 0u &&
      (static_cast<size_t>(tiles + 2 * groups) * RADIX > diag_lim[2] || tile >= tiles || sp.group >= groups)) {
    atomicAdd(&diag_hit[4], 1u);
    atomicCAS(&diag_hit[5], 0u, tile + 1u);
  }
#endif

  // digit of item j (indexed digits: of (key, shard-local index); padding: the largest)
  auto dig_of = [&](int j) -> uint32_t {
    if constexpr (IDX) {
      const uint32_t local = w * (GRS_WAVE * ITEMS) + j * GRS_WAVE + lane;
      return local < valid ? dig(key[j], tile_base + local) : dmask;
    } else {
      return dig(key[j]);
    }
  };

  // ---- rank ----  (two 16-bit ranks per register: a wave ranks at most 64 * ITEMS keys).
  // Indexed digits cost tens of VALU each (the splitter compares), so theirs is computed once
  // and kept in the rank field's top 4 bits for the reorder (ranks < 2^12, digits < 16).
  static_assert(GRS_WAVE * ITEMS < 65536, "16-bit ranks");
  static_assert(!IDX || (GRS_WAVE * ITEMS <= 4096 && RADIX <= 16 && ROUNDS == 1 && !C16),
                "indexed digits ride in the rank field, with 32-bit wave counters");
  static_assert(!MATCH || !C16, "match ranking uses 32-bit counters");
  uint32_t rank[(ITEMS + 1) / 2];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = dig_of(j);
    uint32_t r;
    if constexpr (MATCH) {
      // peers of this lane's digit in this item: the lowest one adds their count; LDS runs a
      // wave's instructions in order, so the plain read sees items < j exactly
      const uint64_t m = match_digit<RB>(d);
      const uint32_t below = mbcnt64(m);
      uint32_t* c = &sm.cnt[w * RADIX + d];
      const uint32_t old = *c;
      if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
      r = old + below;
    } else if constexpr (C16) {
      const uint32_t sh = (d & 1u) << 4;
      r = (atomicAdd(&sm.cnt[(w * RADIX + d) >> 1], 1u << sh) >> sh) & 0xFFFFu;
    } else {
      r = atomicAdd(&sm.cnt[w * RADIX + d], 1u);
    }
    if constexpr (IDX) r |= d << 12;
    if (j & 1)
      rank[j / 2] |= r << 16;
    else
      rank[j / 2] = r;
  }
  if constexpr (PF) {
    if (t == 0) sm.next = atomicAdd(ticket, 1u);  // read after the reorder
  }
  // a solo tile (segmented passes) has no status words and waits on nobody
  const bool solo = SEG && sp.solo;
  // this tile's (and its group's) words of the next pass's status buffer
  if (t < static_cast<uint32_t>(RADIX) && !solo) {
    status_next[static_cast<size_t>(tile) * RADIX + t] = 0;
    if (sp.jg == 0) {
      status_next[static_cast<size_t>(tiles + sp.group) * RADIX + t] = 0;
      status_next[static_cast<size_t>(tiles + groups + sp.group) * RADIX + t] = 0;
    }
  }
  lds_barrier();  // B1

  uint32_t tile_cnt = 0, publish = 0, gold = 0, lstart = 0, gstart = 0;
  if (t < static_cast<uint32_t>(RADIX)) {
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) {
      const uint32_t c = cnt_ld(ww * RADIX + t);
      cnt_st(ww * RADIX + t, tile_cnt);
      tile_cnt += c;
    }
    publish = (t == dmask) ? tile_cnt - pad : tile_cnt;  // padding is ranked, never counted
    if (solo) {
      gh = publish;   // the segment's counts: its digit starts are the tile's own
    } else {
      if (tile + 1u != dbg.fault_tile1)
        st_status(status + static_cast<size_t>(tile) * RADIX + t, publish + 1u);
      gold = __hip_atomic_fetch_add(gacc + static_cast<size_t>(sp.group) * RADIX + t,
                                    (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (w < static_cast<uint32_t>(DW)) {
    const uint32_t li = wave_scan_dpp(tile_cnt);
    const uint32_t gi = wave_scan_dpp(gh);
    if (lane == GRS_WAVE - 1) {
      sm.wsum[w] = li;
      sm.wsum[WAVES + w] = gi;
    }
    lstart = li - tile_cnt;
    gstart = gi - gh;
  }
  lds_barrier();  // B2

  Lb3<RADIX, (ROUNDS > 1 ? GRS_LB_GWIN_XL : GRS_LB_GWIN)> lb;
  if (t < static_cast<uint32_t>(RADIX)) {
    for (uint32_t ww = 0; ww < w; ++ww) {
      lstart += sm.wsum[ww];
      gstart += sm.wsum[WAVES + ww];
    }
    // segmented pass, a segment's first tile: where each digit's run of the segment starts
    // (the next level's segment table, grs_msd_local)
    if (digit_starts != nullptr) digit_starts[t] = sp.seg_start + gstart;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) cnt_st(ww * RADIX + t, cnt_ld(ww * RADIX + t) + lstart);
    if constexpr (IDX) {
      sm.lstart[t] = lstart;
      if (t == static_cast<uint32_t>(RADIX - 1)) sm.lstart[RADIX] = TILE;
    }
    if constexpr (!LATE_LB) {
      if (!solo) lb.issue(status, gacc, ginc, tile, t, sp.jg, sp.group, sp.g0);
    }
  }
  lds_barrier();  // B3

  if constexpr (IDX) {   // the chunk digits (read in the store phase, after B4)
    for (uint32_t c = t; c < static_cast<uint32_t>(TILE / GRS_WAVE); c += BLOCK) {
      uint32_t d0 = 0, d1 = 0;
#pragma unroll
      for (int b = 1; b < RADIX; ++b) {
        const uint32_t ls = sm.lstart[b];
        d0 += ls <= c * GRS_WAVE;
        d1 += ls <= c * GRS_WAVE + GRS_WAVE - 1;
      }
      sm.cdig[c] = static_cast<uint16_t>(d0 | (d1 << 8));
    }
  }
  // ---- reorder the tile in LDS by (digit, input order) ----
  // the digits are recomputed from the keys (1 VALU each) instead of being kept live since
  // the ranking: the empty asm hides the earlier values from common-subexpression elimination
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) asm volatile("" : "+v"(key[j]));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    uint32_t r = (j & 1) ? rank[j / 2] >> 16 : rank[j / 2] & 0xFFFFu;
    uint32_t d;
    if constexpr (IDX) {
      d = r >> 12;
      r &= 0xFFFu;
    } else {
      d = dig_of(j);
    }
    const uint32_t pos = cnt_ld(w * RADIX + d) + r;
    if (ROUNDS == 1 || pos < static_cast<uint32_t>(LTILE)) {
      sm.keys[pos] = key[j];
      if constexpr (PAIRS) sm.vals[pos] = val[j];
    }
    if constexpr (ROUNDS > 1) {   // the rank register now holds the tile position
      if (j & 1)
        rank[j / 2] = (rank[j / 2] & 0xFFFFu) | (pos << 16);
      else
        rank[j / 2] = (rank[j / 2] & 0xFFFF0000u) | pos;
    }
  }
  if constexpr (LATE_LB) {
    if (t < static_cast<uint32_t>(RADIX) && !solo) lb.issue(status, gacc, ginc, tile, t, sp.jg, sp.group, sp.g0);
  }
  uint32_t next = tiles;
  if constexpr (PF && ROUNDS == 1) {   // two rounds: after round 2 sits in LDS
    next = __builtin_amdgcn_readfirstlane(sm.next);
    if (next < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
  }
  if (t < static_cast<uint32_t>(RADIX)) {
    const uint32_t prefix =
        solo ? 0u
             : lb.finish(status, gacc, ginc, tile, sp.jg, sp.group, sp.in_group, t, gold, publish,
                         error_word, dbg.spin_limit);
    if constexpr ((OPT & 131072) != 0) {
      // region pass (grs_onesweep_region; grs_onesweep_seg<REGION>): gh is digit t's region,
      // not its count; the segment's last tile's look-back covers every other tile of it, so it
      // knows each digit's total and whether a run outgrew its region (a solo tile: its own
      // counts, never past its region)
      if (sp.last) {
        const uint32_t tot = prefix + publish;
        region_totals[t] = tot;
        if (tot > gh) atomicOr(spill_flag != nullptr ? spill_flag : &region_totals[RADIX], 1u);
      }
    }
    uint32_t start = gstart + prefix;
    if constexpr (!IDX) {
      // A timed-out look-back only underestimates this pass's prefixes, but the next pass of
      // the same sort then reads keys whose digits no longer match the upfront histogram, and
      // a run could pass n.  Keep every run inside its segment, [0, n) for an ordinary pass (a
      // no-op on consistent counts).
      // In 64 bits: the 32-bit form (gstart > room ? room : gstart + min(prefix, room - gstart))
      // came out of this ROCm 7.2 compiler without its first arm (the device IR computes
      // gstart + min(prefix, room - gstart) unconditionally), so a region run past its room was
      // not held back -- P2's sampled regions write past the region buffer then (found by the
      // bounds-checked build, tools/diag).
      const uint64_t last = sp.seg_len >= publish ? static_cast<uint64_t>(sp.seg_len - publish) : 0u;
      const uint64_t want = static_cast<uint64_t>(gstart) + static_cast<uint64_t>(prefix);
#ifndef GRS_TEST_NO_CLAMP
      start = sp.seg_start + static_cast<uint32_t>(want < last ? want : last);
#else
      // scratch builds only (tools/diag/canary_no_clamp.py): the clamp removed, so that a region
      // run past its room writes past the region buffer and the guard bands must show it
      (void)last;
      start = sp.seg_start + static_cast<uint32_t>(want);
#endif
    }
#ifdef GRS_DIAG
    if (diag_lim[0] != 0u && publish != 0u && start + publish > diag_lim[0] &&
        atomicCAS(&diag_hit[8], 0u, 1u) == 0u) {
      diag_hit[9] = tile;
      diag_hit[10] = t;
      diag_hit[11] = start;
      diag_hit[12] = gstart;
      diag_hit[13] = prefix;
      diag_hit[14] = sp.seg_start;
      diag_hit[15] = sp.seg_len;
      diag_hit[16] = publish;
      diag_hit[17] = gh;
      diag_hit[18] = sp.base;
      diag_hit[19] = sp.valid;
      diag_hit[20] = lstart;
    }
#endif
    // (indexed digits, the partition pass: its one pass per call reads the input as given, so
    // a timed-out look-back there only underestimates its own runs' starts; they stay >= 0 and
    // end before n -- no clamp needed)
    sm.base[t] = start - lstart;
  }
  lds_barrier();  // B4

  // ---- store: consecutive threads write consecutive slots of each digit run ----
  // (SPAN: the stored keys, which are the tile's valid keys, ORed on the way)
  constexpr bool SPAN = (OPT & 262144) != 0;
  K s_or = 0, s_nor = 0;
  // digit of reordered position i.  Indexed digits: a thread visits increasing positions, so
  // its digit only moves forward through the tile-local digit starts (at most RADIX - 1 steps
  // per tile, over empty digits too).
  auto put = [&](uint32_t dst, K kk, uint32_t i) {
#ifdef GRS_DIAG
    if (diag_lim[0] != 0u && dst >= diag_lim[0]) {
      atomicAdd(&diag_hit[0], 1u);
      atomicMax(&diag_hit[1], dst);
      return;
    }
#endif
    if constexpr ((OPT & 8192) != 0) {
      static_assert(PAIRS && sizeof(K) == 4, "records: u32 key + u32 value");
      const uint2 r = make_uint2(static_cast<uint32_t>(kk), sm.vals[i]);
      const unsigned long long x = (static_cast<unsigned long long>(r.y) << 32) | r.x;
      if constexpr ((OPT & 32768) != 0) {   // split records: [n/2, n) in vals_out
        if (dst >= n / 2) reinterpret_cast<unsigned long long*>(vals_out)[dst - n / 2] = x;
        else reinterpret_cast<unsigned long long*>(keys_out)[dst] = x;
      } else {
        reinterpret_cast<unsigned long long*>(keys_out)[dst] = x;
      }
    } else {
      keys_out[dst] = kk;
      if constexpr (PAIRS) vals_out[dst] = sm.vals[i];
    }
  };
  auto dig_at = [&](uint32_t i, K kk) -> uint32_t {
    if constexpr (IDX) {
      // the digits at the ends of i's 64-position chunk (one wave-instruction's positions: a
      // broadcast read); a walk over the digit starts only where a run starts inside the chunk
      const uint32_t c = sm.cdig[i >> 6];
      uint32_t d = c & 255u;
      if (d != (c >> 8))
        while (i >= sm.lstart[d + 1]) ++d;
      return d;
    } else {
      return dig(kk);
    }
  };
#pragma unroll
  for (int rr = 0; rr < ROUNDS; ++rr) {
    if (rr > 0) {
      // round rr: every thread has read the previous round's positions; write this round's
      lds_barrier();
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint32_t pos = (j & 1) ? rank[j / 2] >> 16 : rank[j / 2] & 0xFFFFu;
        const uint32_t lp = pos - static_cast<uint32_t>(rr * LTILE);
        if (lp < static_cast<uint32_t>(LTILE)) {
          sm.keys[lp] = key[j];
          if constexpr (PAIRS) sm.vals[lp] = val[j];
        }
      }
      lds_barrier();
      if constexpr (PF) {
        // the last round's keys are in LDS: the registers take the next tile's loads, which
        // fly behind this round's stores
        if (rr == ROUNDS - 1) {
          next = __builtin_amdgcn_readfirstlane(sm.next);
          if (next < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
        }
      }
    }
    const uint32_t roff = static_cast<uint32_t>(rr * LTILE);
    if (valid == static_cast<uint32_t>(TILE)) {
#pragma unroll
      for (int k = 0; k < LITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        const K kk = sm.keys[i];
        const uint32_t d = dig_at(roff + i, kk);
        put(sm.base[d] + roff + i, kk, i);
        if constexpr (SPAN) {
          s_or |= kk;
          s_nor |= static_cast<K>(~kk);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < LITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        if (roff + i < valid) {
          const K kk = sm.keys[i];
          const uint32_t d = dig_at(roff + i, kk);
          put(sm.base[d] + roff + i, kk, i);
          if constexpr (SPAN) {
            s_or |= kk;
            s_nor |= static_cast<K>(~kk);
          }
        }
      }
    }
  }
  if constexpr (SPAN) {   // wave OR, then one LDS OR per wave (read by the kernel after a barrier)
    uint32_t v[4] = {static_cast<uint32_t>(s_or), static_cast<uint32_t>(static_cast<uint64_t>(s_or) >> 32),
                     static_cast<uint32_t>(s_nor), static_cast<uint32_t>(static_cast<uint64_t>(s_nor) >> 32)};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (sizeof(K) == 4 && (q & 1)) continue;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[q] |= __shfl_xor(v[q], o);
      if (lane == 0 && v[q] != 0u) atomicOr(&sm.span[q], v[q]);
    }
  }
  return next;
}

// A tile of a pass the LSD plan elides (grs_pass_plan: the pass's digit is the same for every
// key, so its stable scatter is the identity): the tile's words of the next pass's status
// zeroed as onesweep_tile would (the next pass's look-back reads them), and for kPassCopy its
// keys (and payload) copied to the same indices.
template <typename K, bool PAIRS, int RADIX, int BLOCK>
__device__ __forceinline__ void elided_tile(uint32_t mode, const TileSpan& sp, const K* __restrict__ keys_in,
                                            K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
                                            uint32_t* __restrict__ vals_out, uint32_t* __restrict__ status_next) {
  const uint32_t t = threadIdx.x;
  if (t < static_cast<uint32_t>(RADIX)) {
    status_next[static_cast<size_t>(sp.tile) * RADIX + t] = 0;
    if (sp.jg == 0) {
      status_next[static_cast<size_t>(sp.tiles + sp.group) * RADIX + t] = 0;
      status_next[static_cast<size_t>(sp.tiles + sp.groups + sp.group) * RADIX + t] = 0;
    }
  }
  if (mode == kPassCopy) {
    for (uint32_t i = t; i < sp.valid; i += BLOCK) {
      keys_out[sp.base + i] = keys_in[sp.base + i];
      if constexpr (PAIRS) vals_out[sp.base + i] = vals_in[sp.base + i];
    }
  }
}

// One tile per workgroup (grid = tiles), tile ids from a ticket counter.  dig_dev: when not
// null, the digit functor is read from device memory instead of the `dig` argument.  plan
// (nullable): this pass's word of grs_pass_plan -- an elided pass only zeroes (and copies).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_v4(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word, const DigitF* __restrict__ dig_dev,
    const uint32_t* __restrict__ plan = nullptr) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  __shared__ SM sm;
  const uint32_t t = threadIdx.x;
  uint32_t tt = t;
  asm volatile("" : "+v"(tt));
  K key[ITEMS];
  uint32_t val[ITEMS];
  const uint32_t mode = plan != nullptr ? __builtin_amdgcn_readfirstlane(*plan) : 0u;
  if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
  // digit functor computed on the device (multi-GPU splitters): uniform scalar loads
  const DigitF dg = dig_dev != nullptr ? *dig_dev : dig;
  __syncthreads();
  const uint32_t tile = __builtin_amdgcn_readfirstlane(sm.ticket);
  if (mode != 0u) {
    elided_tile<K, PAIRS, SM::RADIX, BLOCK>(mode, TileSpan::whole(tile, n, SM::TILE), keys_in, keys_out, vals_in,
                                            vals_out, status_next);
    return;
  }
  tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, tt);
  const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT>(sm, TileSpan::whole(tile, n, SM::TILE), key, val,
                                                 keys_in, keys_out, vals_in,
                                                 vals_out, n, dg, gh, ticket, status, status_next,
                                                 error_word, PassDebug::read(error_word));
}

// The MSD sort's first scatter without an upfront histogram (grs_msd.hpp): digit d's run goes
// to a REGION of R_d = (sample[d] * mult >> 20) + pad keys -- the sampled share of the top byte,
// with slack -- instead of its exact place, so the keys need no counting read before the pass.
// region_len = sum of the regions (the clamp bound).  The last ticket writes the digit totals
// to totals[0..RADIX) and sets totals[RADIX] when a run outgrew its region.
// span (the MSD sort's span words, grs_msd.hpp GRS_MSD_SPAN): the digit's shift is span[4] (the
// sample's guess of the keys' top varying byte), and every tile ORs its keys into span[0..1] and
// their complements into span[2..3], so that grs_msd_span learns the exact span and plans the
// redo (a run past its region, or a varying bit above the guessed digit).
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_region(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const RadixDigit<K> dig,
    const uint32_t* __restrict__ sample, unsigned long long mult, uint32_t pad,
    uint32_t region_len, uint32_t* __restrict__ ticket, uint32_t* __restrict__ status,
    uint32_t* __restrict__ status_next, uint32_t* __restrict__ error_word,
    uint32_t* __restrict__ totals, uint32_t* __restrict__ span) {
  constexpr int ROPT = OPT | 131072 | 262144;
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, ROPT, RadixDigit<K>>;
  __shared__ SM sm;
  const uint32_t t = threadIdx.x;
  uint32_t tt = t;
  asm volatile("" : "+v"(tt));
  K key[ITEMS];
  uint32_t val[ITEMS];
  if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
  if (t < 4) sm.span[t] = 0;
  for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
  RadixDigit<K> dg = dig;
  dg.shift = static_cast<int>(__builtin_amdgcn_readfirstlane(span[4]));
  __syncthreads();
  const uint32_t tile = __builtin_amdgcn_readfirstlane(sm.ticket);
  tile_load<K, PAIRS, BLOCK, ITEMS, ROPT>(key, val, keys_in, vals_in, n, tile, tt);
  const uint32_t gh =
      t < static_cast<uint32_t>(SM::RADIX)
          ? static_cast<uint32_t>((static_cast<unsigned long long>(sample[t]) * mult) >> 20) + pad
          : 0u;
  TileSpan sp = TileSpan::whole(tile, n, SM::TILE);
  sp.seg_len = region_len;
  onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, ROPT>(sm, sp, key, val, keys_in, keys_out, vals_in,
                                                  vals_out, n, dg, gh, ticket, status, status_next,
                                                  error_word, PassDebug::read(error_word), nullptr,
                                                  totals);
  lds_barrier();   // every wave's OR in sm.span
  if (t < 4 && (sizeof(K) == 8 || (t & 1u) == 0u)) {
    // one global OR per word, and only when it adds bits (all but the first tiles skip it)
    const uint32_t mine = sm.span[t];
    const uint32_t cur = __hip_atomic_load(&span[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur | mine) != cur) atomicOr(&span[t], mine);
  }
}

// ---------------------------------------------------------------------------------------
// persistent pass with next-tile prefetch
// ---------------------------------------------------------------------------------------
// grs_onesweep_v4 runs one tile per workgroup, and with one 36K-key tile per CU (LDS) the
// CU's HBM traffic stops between the last store of one tile and the first key of the next:
// the workgroup exits, the next is dispatched, and its loads pay the full HBM latency before
// ranking can start.  Here grid = resident workgroups; each loops over tickets and issues
// tile T+1's loads as soon as tile T sits in LDS, so they fly during T's look-back and
// stores.  Tickets are drawn in increasing order by running workgroups only, and a workgroup
// finishes T before it starts T+1, so the lowest unfinished tile never waits on an unstarted
// one (no residency assumption).  Every workgroup leaves once it draws a ticket >= tiles.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_v6(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word, const DigitF* __restrict__ dig_dev,
    const uint32_t* __restrict__ plan = nullptr) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  __shared__ SM sm;
  const uint32_t t = threadIdx.x;
  const uint32_t mode = plan != nullptr ? __builtin_amdgcn_readfirstlane(*plan) : 0u;
  if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
  const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  const PassDebug dbg = PassDebug::read(error_word);
  const DigitF dg = dig_dev != nullptr ? *dig_dev : dig;
  __syncthreads();
  const uint32_t tiles = (n + SM::TILE - 1) / SM::TILE;
  uint32_t tile = __builtin_amdgcn_readfirstlane(sm.ticket);
  if (mode != 0u) {   // an elided pass (grs_pass_plan): the same ticket loop, zeroing / copying
    while (tile < tiles) {
      elided_tile<K, PAIRS, SM::RADIX, BLOCK>(mode, TileSpan::whole(tile, n, SM::TILE), keys_in, keys_out,
                                              vals_in, vals_out, status_next);
      __syncthreads();   // every thread has read sm.ticket
      if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
      __syncthreads();
      tile = __builtin_amdgcn_readfirstlane(sm.ticket);
    }
    return;
  }
  K key[ITEMS];
  uint32_t val[ITEMS];
  if (tile < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, t);
  while (tile < tiles) {
    tile = onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT, true>(
        sm, TileSpan::whole(tile, n, SM::TILE), key, val, keys_in, keys_out, vals_in, vals_out, n,
        dg, gh, ticket, status,
        status_next, error_word, dbg);
    // every LDS read of the finished tile is done before the counters are reset
    lds_barrier();
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    lds_barrier();
  }
}

// ---------------------------------------------------------------------------------------
// every pass of a sort in one launch
// ---------------------------------------------------------------------------------------
// Grid barrier of a launch whose workgroups are all resident: every wave waits for its stores
// (the workgroup barrier alone does not: one CU's waves share its L1), then the workgroup adds 1
// to *bar with release semantics at agent scope (its XCD's L2 written back: the next pass reads
// on other XCDs) and waits until `target` have arrived (acquire: L1 / L2 invalidated).  The wait
// is bounded like a look-back spin: past it the error word is set and the workgroup goes on.
// Measured (tools/barrier_probe.py, 256 workgroups storing 16 MB a round): 27 us a round against
// 5 us for a kernel boundary (11 us with no fences at all) -- hence not the default.
__device__ __forceinline__ void grid_barrier(uint32_t* bar, uint32_t target, uint32_t* error_word,
                                             uint32_t limit) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    while (ld_status(bar) < target) {
      if (++spins > limit) {
        atomicOr(error_word, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// The P passes of an LSD sort (digit p = bits [shift0 + RB p, + RB)) in ONE launch (option
// GRS_OPT_PASS = 8; measured slower than one launch per pass): grid = the
// resident workgroups (the host checks the occupancy: the barrier needs every one running),
// each running grs_onesweep_v6's ticket loop over pass p's tiles, then a grid barrier before
// pass p + 1 reads what pass p wrote.  Pass p reads (keys_a, vals_a) when p is even and
// (keys_b, vals_b) when odd and writes the other pair; status buffers alternate as in separate
// launches (pass p zeroes its tiles' words of pass p + 1's buffer).  bar: zero at launch.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_fused(
    K* keys_a, K* keys_b, uint32_t* vals_a, uint32_t* vals_b, uint32_t n, int shift0, int passes,
    const uint32_t* __restrict__ hist, uint32_t* __restrict__ tickets, uint32_t* __restrict__ bar,
    uint32_t* status0, uint32_t* status1, uint32_t* __restrict__ error_word) {
  using Dig = RadixDigit<K>;
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, Dig>;
  __shared__ SM sm;
  const uint32_t t = threadIdx.x;
  const PassDebug dbg = PassDebug::read(error_word);
  const uint32_t tiles = (n + SM::TILE - 1) / SM::TILE;
  for (int p = 0; p < passes; ++p) {
    const bool odd = (p & 1) != 0;
    K* const kin = odd ? keys_b : keys_a;
    K* const kout = odd ? keys_a : keys_b;
    uint32_t* const vin = odd ? vals_b : vals_a;
    uint32_t* const vout = odd ? vals_a : vals_b;
    uint32_t* const ticket = tickets + p * GRS_XCDS;
    if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) ? hist[p * GRS_HIST_PASS_STRIDE + t] : 0u;
    __syncthreads();
    const Dig dig{shift0 + RB * p, (1u << RB) - 1u};
    uint32_t tile = __builtin_amdgcn_readfirstlane(sm.ticket);
    K key[ITEMS];
    uint32_t val[ITEMS];
    if (tile < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, kin, vin, n, tile, t);
    while (tile < tiles) {
      tile = onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT, true>(
          sm, TileSpan::whole(tile, n, SM::TILE), key, val, kin, kout, vin, vout, n, dig, gh, ticket,
          odd ? status1 : status0, odd ? status0 : status1, error_word, dbg);
      lds_barrier();
      for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
      lds_barrier();
    }
    if (p + 1 < passes) grid_barrier(bar, static_cast<uint32_t>(p + 1) * gridDim.x, error_word, dbg.spin_limit);
  }
}

// ---------------------------------------------------------------------------------------
// segmented pass: every segment of a table sorted by one digit on its own
// ---------------------------------------------------------------------------------------
// MSD sort and segmented sorts (grs_capi.hip): the same tile code as grs_onesweep_v4, over the
// tiles of a segment table -- tiles never straddle a segment, each segment's look-back chain
// restarts at its first tile, and its digit runs start at the segment's own first key, from
// the segment's own digit counts (hist row `seg`; a segment of one tile ranks, scans and stores
// it with no status words and no look-back).  hdr[0] = tiles (tickets), hdr[1] = look-back
// groups, hdr[2] = tile word rows of the status layout.  PERSIST: grid = resident workgroups looping over tickets (tables whose
// size is known only on the device); otherwise grid >= hdr[0], one tile per workgroup.
// digit_starts (nullable): a segment's first tile writes the start of each digit run of the
// segment to digit_starts[seg * RADIX + d].
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT, bool PERSIST>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_seg(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, const RadixDigit<K> dig, const SegTile* __restrict__ rec,
    const uint32_t* __restrict__ hdr, const uint32_t* __restrict__ hist, uint32_t hist_stride,
    uint32_t* __restrict__ ticket, uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word, uint32_t* __restrict__ digit_starts,
    uint32_t* __restrict__ totals = nullptr, uint32_t* __restrict__ spill = nullptr,
    const uint32_t* __restrict__ gate = nullptr, const uint32_t* __restrict__ shift_dev = nullptr) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, RadixDigit<K>>;
  static_assert((OPT & (16384 | 32768)) == 0, "segmented passes: records in one buffer (n unknown)");
  __shared__ SM sm;
  const uint32_t t = threadIdx.x;
  // gate (nullable): run only when *gate != 0 (a redo that is usually not needed)
  if (gate != nullptr && __builtin_amdgcn_readfirstlane(*gate) == 0u) return;
  const PassDebug dbg = PassDebug::read(error_word);
  // shift_dev (nullable, the MSD sort's digit shift found on the device): the digit's shift is
  // *shift_dev + dig.shift
  RadixDigit<K> dg = dig;
  if (shift_dev != nullptr) dg.shift += static_cast<int>(__builtin_amdgcn_readfirstlane(*shift_dev));
  for (;;) {
    if (t == 0) sm.ticket = atomicAdd(ticket, 1u);
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    __syncthreads();
    const uint32_t tk = __builtin_amdgcn_readfirstlane(sm.ticket);
    if (tk >= hdr[0]) return;   // every workgroup leaves once it draws a ticket past the table
    const SegTile r = rec[tk];
    const bool solo = (r.flags >> 8) & 1u;
    const uint32_t q = (r.flags >> 9) & 0x3FFFFFu;   // the group's place in its segment
    const TileSpan sp{r.row, hdr[2], r.group, hdr[1], r.flags & 15u, (r.flags >> 4) & 15u,
                      r.group - q, r.base, r.valid, r.seg_start, r.seg_len, solo, (r.flags >> 31) != 0u};
    K key[ITEMS];
    uint32_t val[ITEMS];
    uint32_t tt = t;
    asm volatile("" : "+v"(tt));
    tile_load_at<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, 0u, sp.base, sp.valid, tt);
    const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) && !solo
                            ? hist[static_cast<size_t>(r.seg) * hist_stride + t] : 0u;
    // the segment's first tile (place 0 of group 0; its keys may be read from elsewhere than
    // its runs go, so base == seg_start does not tell)
    const bool first = (r.flags & 15u) == 0u && q == 0u;
    uint32_t* ds = digit_starts != nullptr && first
                       ? digit_starts + static_cast<size_t>(r.seg) * SM::RADIX : nullptr;
    // region pass (OPT 131072): hist holds each digit's region, not its count; the segment's last
    // tile writes the digit totals to totals[seg * RADIX + d] and sets *spill if one outgrew
    uint32_t* const tot = (OPT & 131072) != 0 ? totals + static_cast<size_t>(r.seg) * SM::RADIX : nullptr;
    onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT, false, true>(sm, sp, key, val, keys_in, keys_out, vals_in,
                                                   vals_out, 0u, dg, gh, ticket, status,
                                                   status_next, error_word, dbg, ds, tot, spill);
    if constexpr (!PERSIST) return;
    lds_barrier();   // every LDS read of the finished tile before the next ticket's reset
  }
}

}  // namespace grs
