// lab_pass.hpp — the round-3 pass kernel with every lab ablation (tools/lab2.hip only; not
// part of libgrs).  The shipped kernel is gpuradixsort_amd/csrc/grs_pass.hpp: this copy keeps
// the rejected variants (OPT bits below: XCD ranges, wide look-back, destination-aligned
// stores, speculative / ticketless tiles, persistent variants, store policies, 16-lane
// counter sets, accumulator read-back, phase stamps) so that their measurements in DESIGN.md
// §6.0 stay reproducible.  Namespace grs_lab, so it can sit beside the shipped kernel.
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
//            (probed at sorter creation; the ballot-match fallback is RANK_MATCH below)
//   B1       digit threads: wave starts (column scan), tile count, publish the count, add it
//            into the group accumulator; wave scans over digits (tile and pass starts)
//   B2       tile-local digit starts folded into the wave counters; look-back polls ISSUED
//   B3       all waves reorder the tile in LDS by (digit, input order); the digit threads
//            then FINISH the look-back (its round trip overlapped the reorder) and write the
//            global base of each digit
//   B4       stores: consecutive threads write consecutive slots of each digit run
//
// MINW workgroups per CU (launch bounds + LDS sized for it): while one workgroup waits on a
// ticket, a look-back or its loads, another ranks or reorders — the phases of one tile are a
// serial chain, so overlap comes from co-resident tiles.
#pragma once

#include <type_traits>

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

namespace grs_lab {
using namespace grs;

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

// Look-back status of one pass (uint32 words, all zero at pass start):
//   tile words   [tiles][R]   count + 1 of the tile's digit (0 = not published yet)
//   group accs   [groups][R]  (arrivals << 24) | sum of the group's tile counts
//   group incl   [groups][R]  inclusive prefix of the group + 1 (0 = not published yet),
//                             written by the tile whose add completes the accumulator
// Values are stored +1 so that no flag bits are needed: prefixes reach n (< 2^32).
__host__ __device__ constexpr size_t lb3_status_words(size_t tiles, size_t radix) {
  return (tiles + 2 * ((tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP)) * radix;
}

// Exclusive prefix of digit d over tiles [0, tile): own group's earlier tiles (< G words)
// plus the group-level prefix (newest published group INCLUSIVE + complete accumulators
// after it).  issue() sends the first round of loads, finish() consumes them.
// GW: groups polled per round.  The two-round (XL) tiles use 4: the window's registers are
// live across the reorder there, beside the tile's keys and positions.
// OPT 4: one wave's 64 status words (a uniform 64-word row) into its lanes through scalar
// loads with glc (coherent across XCDs, tools/smem_probe.hip): a re-poll that does not queue
// behind the wave's outstanding vector loads (vmcnt retires in order)
typedef uint32_t lab_u32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ uint32_t smem_row_lane(const uint32_t* row) {
  lab_u32x16 v[4];
  asm volatile(
      "s_load_dwordx16 %0, %4, 0x0 glc\n\t"
      "s_load_dwordx16 %1, %4, 0x40 glc\n\t"
      "s_load_dwordx16 %2, %4, 0x80 glc\n\t"
      "s_load_dwordx16 %3, %4, 0xc0 glc\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=s"(v[0]), "=s"(v[1]), "=s"(v[2]), "=s"(v[3]) : "s"(row) : "memory");
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(out) : "s"(v[q][i]), "i"(16 * q + i));
  return out;
}

template <int RADIX, int GW = GRS_LB_GWIN, bool OWNACC = false, bool SC = false>
struct Lb3 {
  static constexpr int G = GRS_LB_GROUP;
  uint32_t tw[G - 1];
  uint32_t gi[GW], ga[GW];
  int32_t ph;
  int32_t g0;   // first group of this tile's chain (XCD ranges: the range's first group)
  uint32_t gown;   // OWNACC: this tile's group accumulator, read with the first round

  __device__ __forceinline__ void load_groups(const uint32_t* gacc, const uint32_t* ginc,
                                              uint32_t d) {
#pragma unroll
    for (int k = 0; k < GW; ++k) {
      const int32_t h = ph - k;
      gi[k] = h >= g0 ? ld_status(ginc + static_cast<size_t>(h) * RADIX + d) : 0u;
      ga[k] = h >= g0 ? ld_status(gacc + static_cast<size_t>(h) * RADIX + d) : 0u;
    }
  }
  __device__ __forceinline__ void issue(const uint32_t* status, const uint32_t* gacc,
                                        const uint32_t* ginc, uint32_t tile, uint32_t d,
                                        int32_t first_group = 0) {
    g0 = first_group;
    const uint32_t first = (tile / G) * G;
#pragma unroll
    for (int k = 0; k < G - 1; ++k)
      tw[k] = first + k < tile ? ld_status(status + static_cast<size_t>(first + k) * RADIX + d) : 1u;
    ph = static_cast<int32_t>(tile / G) - 1;
    load_groups(gacc, ginc, d);
    if constexpr (OWNACC) gown = ld_status(gacc + static_cast<size_t>(tile / G) * RADIX + d);
  }
  // gold: the value this tile's add to its group accumulator returned; publish: its count
  // (OWNACC: the add returned nothing; the group's last tile publishes the inclusive when the
  // accumulator it read back is complete)
  __device__ __forceinline__ uint32_t finish(const uint32_t* status, const uint32_t* gacc,
                                             uint32_t* ginc, uint32_t tile, uint32_t tiles,
                                             uint32_t d, uint32_t gold, uint32_t publish,
                                             uint32_t* error_word) {
    const uint32_t g = tile / G;
    const uint32_t first = g * G;
    uint32_t spins = 0, own = 0;
#pragma unroll
    for (int k = 0; k < G - 1; ++k) {
      uint32_t v = tw[k];
      if constexpr (SC) {   // the whole wave re-polls its row until every lane's word is in
        const uint32_t* row = status + static_cast<size_t>(first + k) * RADIX +
                              (__builtin_amdgcn_readfirstlane(d) & ~63u);
        while (__builtin_amdgcn_ballot_w64(v == 0u) != 0) {
          if (++spins > GRS_SPIN_LIMIT) {
            if (v == 0u) atomicOr(error_word, 1u);
            v = v == 0u ? 1u : v;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          v = smem_row_lane(row);
        }
      } else {
        while (v == 0u) {
          if (++spins > GRS_SPIN_LIMIT) {
            atomicOr(error_word, 1u);
            v = 1u;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          v = ld_status(status + static_cast<size_t>(first + k) * RADIX + d);
        }
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
        if (++spins > GRS_SPIN_LIMIT) {
          atomicOr(error_word, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      load_groups(gacc, ginc, d);
    }
    const uint32_t in_group = min(static_cast<uint32_t>(G), tiles - g * G);
    if constexpr (OWNACC) {
      // only the group's last tile publishes (one writer per line); if it read the accumulator
      // before an earlier tile's add landed, no inclusive appears and the successors sum the
      // complete accumulator instead (a longer walk, the same prefix)
      if (tile - g * G == in_group - 1u && (gown >> 24) == in_group)
        st_status(ginc + static_cast<size_t>(g) * RADIX + d, gp + (gown & 0xFFFFFFu) + 1u);
    } else if ((gold >> 24) == in_group - 1u) {  // this tile's add completed the group
      st_status(ginc + static_cast<size_t>(g) * RADIX + d, gp + (gold & 0xFFFFFFu) + publish + 1u);
    }
    return gp + own;
  }
};

// Wide look-back: the prefix of digit d is resolved by a group of L lanes (lane j of group d is
// thread d * L + j; L a power of two, L lanes of one wave) instead of one digit thread: each
// round reads L groups' inclusive + accumulator words at once (one load each per lane) and
// finds, by two ballots, the newest published inclusive and the newest incomplete accumulator
// among them.  At 4-bit digits L = 64 (one wave per digit): a round covers 64 groups = 512
// tiles, so the look-back of a 2^24-key pass is one round trip instead of up to eight.
template <int RADIX, int L>
struct LbWide {
  static constexpr int G = GRS_LB_GROUP;
  static_assert((L & (L - 1)) == 0 && L >= 2 && L <= GRS_WAVE, "lane groups of 2..64 lanes");
  static constexpr int NOWN = (G - 1 + L - 1) / L;   // own-group tile words per lane
  static constexpr int W = L >= 16 ? 1 : 16 / L;      // groups per lane per round (>= 16 a round)
  uint32_t tw[NOWN];  // own group: tile words j + k * L (first read)
  uint32_t gi[W], ga[W];   // groups ph - (k * L + j)
  int32_t ph, g0;
  uint32_t gp_out;    // the group-level part of the last finish() (groups before the tile's)

  __device__ __forceinline__ static uint32_t gsum(uint32_t v) {
#pragma unroll
    for (int o = 1; o < L; o <<= 1) v += __shfl_xor(v, o, GRS_WAVE);
    return v;
  }
  __device__ __forceinline__ static uint64_t gmask(bool pred, uint32_t lane) {
    const uint64_t b = __builtin_amdgcn_ballot_w64(pred);
    if constexpr (L == GRS_WAVE) return b;
    else return (b >> (lane & ~static_cast<uint32_t>(L - 1))) & ((1ull << L) - 1ull);
  }
  __device__ __forceinline__ void load_groups(const uint32_t* gacc, const uint32_t* ginc,
                                              uint32_t d, uint32_t j) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const int32_t h = ph - static_cast<int32_t>(k * L + j);
      gi[k] = h >= g0 ? ld_status(ginc + static_cast<size_t>(h) * RADIX + d) : 0u;
      ga[k] = h >= g0 ? ld_status(gacc + static_cast<size_t>(h) * RADIX + d) : 0u;
    }
  }
  __device__ __forceinline__ void issue(const uint32_t* status, const uint32_t* gacc,
                                        const uint32_t* ginc, uint32_t tile, uint32_t d,
                                        uint32_t j, int32_t first_group) {
    g0 = first_group;
    const uint32_t first = (tile / G) * G;
#pragma unroll
    for (int k = 0; k < NOWN; ++k) {
      const uint32_t i = first + j + k * L;
      tw[k] = i < tile ? ld_status(status + static_cast<size_t>(i) * RADIX + d) : 1u;
    }
    ph = static_cast<int32_t>(tile / G) - 1;
    load_groups(gacc, ginc, d, j);
  }
  // the exclusive prefix of digit d over tiles [g0 * G, tile), in every lane of the group
  __device__ __forceinline__ uint32_t finish(const uint32_t* status, const uint32_t* gacc,
                                             const uint32_t* ginc, uint32_t tile, uint32_t d,
                                             uint32_t j, uint32_t lane, uint32_t* error_word) {
    const uint32_t first = (tile / G) * G;
    uint32_t spins = 0, own = 0;
#pragma unroll
    for (int k = 0; k < NOWN; ++k) {
      uint32_t v = tw[k];
      while (v == 0u) {
        if (++spins > GRS_SPIN_LIMIT) {
          atomicOr(error_word, 1u);
          v = 1u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = ld_status(status + static_cast<size_t>(first + j + k * L) * RADIX + d);
      }
      own += v - 1u;
    }
    own = gsum(own);
    uint32_t gp = 0;
    while (ph >= g0) {
      // offsets o = k * L + j, newest first: the first published inclusive and the first
      // incomplete accumulator among this round's L * W groups
      uint32_t oinc = L * W, oblk = L * W;
#pragma unroll
      for (int k = W - 1; k >= 0; --k) {
        const int32_t h = ph - static_cast<int32_t>(k * L + j);
        const bool valid = h >= g0;
        const bool inc = valid && gi[k] != 0u;
        const bool cmpl = valid && !inc && (ga[k] >> 24) == static_cast<uint32_t>(G);
        const uint64_t mi = gmask(inc, lane), mb = gmask(valid && !inc && !cmpl, lane);
        if (mi) oinc = k * L + static_cast<uint32_t>(__builtin_ctzll(mi));
        if (mb) oblk = k * L + static_cast<uint32_t>(__builtin_ctzll(mb));
      }
      uint32_t part = 0;
      if (oinc < oblk) {   // a published inclusive before any incomplete group
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const uint32_t o = k * L + j;
          part += o < oinc ? (ga[k] & 0xFFFFFFu) : (o == oinc ? gi[k] - 1u : 0u);
        }
        gp += gsum(part);
        break;
      }
      const uint32_t nvalid = static_cast<uint32_t>(min(ph - g0 + 1, L * W));
      const uint32_t c = min(oblk, nvalid);   // complete groups before the first blocked one
#pragma unroll
      for (int k = 0; k < W; ++k) part += (k * L + j) < c ? (ga[k] & 0xFFFFFFu) : 0u;
      gp += gsum(part);
      ph -= static_cast<int32_t>(c);
      if (ph < g0) break;
      if (c == 0) {
        if (++spins > GRS_SPIN_LIMIT) {
          atomicOr(error_word, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      load_groups(gacc, ginc, d, j);
    }
    gp_out = gp;
    return gp + own;
  }
};

template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, bool CNT16 = false,
          bool IDX = false, int ROUNDS = 1, bool ALIGN = false, bool WIDE = false,
          bool RUNS = false, int VG = 1>
struct V4Smem {
  static constexpr int RADIX = 1 << RB;
  static constexpr int WAVES = BLOCK / GRS_WAVE * VG;   // counter sets: VG per wave
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr int LTILE = TILE / ROUNDS;   // reordered positions held at once
  // per-wave digit counters -> tile position of (wave, digit); CNT16: 16-bit, two per word
  uint32_t cnt[WAVES * RADIX / (CNT16 ? 2 : 1)];
  uint32_t base[RADIX];         // global destination of tile position 0 of digit d
  uint32_t wsum[3 * WAVES];     // wave totals of the digit scans
  uint32_t ticket;
  uint32_t next;                // persistent kernel: the next tile's ticket
  alignas(16) K keys[LTILE];
  uint32_t vals[PAIRS ? LTILE : 1];
  // indexed digits (partition): tile-local start of every digit, from which the store phase
  // reads off the digit of a reordered position (the key alone does not determine it)
  uint32_t lstart[IDX ? RADIX + 1 : 1];
  // destination-aligned stores (OPT 65536): per digit the first store chunk, tile-local run
  // start and run length; jsplit: the first chunk of the second round (two-round tiles)
  uint32_t cstart[ALIGN ? RADIX + 1 : 1];
  uint32_t lst[ALIGN ? RADIX : 1];
  uint32_t rlen[ALIGN ? RADIX : 1];
  uint32_t jsplit;
  // wide look-back (OPT 2097152): per digit the group-accumulator add's old value, the
  // published count and the base without the prefix, handed from the digit threads to the
  // lane group that resolves the digit's prefix
  uint32_t lbv[WIDE ? 3 * RADIX : 1];
  // run-line store policy (OPT 33554432): global [begin, end) of each digit's run of this tile
  uint32_t rbeg[RUNS ? RADIX : 1];
  uint32_t rend[RUNS ? RADIX : 1];
  // G16: tile count and tile-local start of each digit (wave d scans digit d's counter sets)
  uint32_t tcnt[VG > 1 ? RADIX : 1];
  uint32_t lst16[VG > 1 ? RADIX : 1];
};
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int OPT, typename DigitF>
using V4SmemFor = V4Smem<K, PAIRS, RB, BLOCK, ITEMS, (OPT & 256) != 0, DigitF::kIndexed,
                         (OPT & 1024) != 0 ? 2 : 1, (OPT & 65536) != 0 && !DigitF::kIndexed,
                         (OPT & 2097152) != 0, (OPT & 33554432) != 0,
                         (OPT & 67108864) != 0 ? 4 : 1>;

// OPT bits (lab ablations; the library uses OPT = 0):
//   4  the look-back's re-polls of its own group's tile words through scalar loads
//      (smem_row_lane; the digit threads are whole waves at 8-bit digits)
//   8  stamps: s_memtime at phase ends into error_word[64 + tile*8 + k]
//   16 look-back issued after the reorder (no overlap)
//   32 contiguous stores (dst = tile position; wrong output)      64 no look-back (estimate)
//   128 nontemporal key loads
//   256 16-bit wave counters (two digits per LDS word: half the counter LDS)
//   512 ballot-match ranking instead of lane-ordered LDS atomics (the fallback when the
//       device probe of the lane order fails, grs_capi.hip)
//   1024 two-round reorder: the keys stay in registers and LDS holds half the tile at a
//       time (positions [0, TILE/2) are reordered and stored, then [TILE/2, TILE)), so a
//       tile can be twice what LDS holds: longer digit runs per tile, fewer partial lines
//   4096 u32 pairs READ as 8-byte (key, value) records from keys_in (vals_in unused)
//   8192 u32 pairs WRITTEN as 8-byte records to keys_out: one digit run of 8-byte records
//       instead of two of 4-byte words, twice as long (fewer partial lines)
//   16384 / 32768: the records read / written are SPLIT over two buffers: records [0, n/2)
//       in keys_in / keys_out and [n/2, n) in vals_in / vals_out (n even; the caller's two
//       4n-byte arrays hold n records that way)
//   65536 destination-aligned stores: each wave-instruction writes one 64-item chunk of ONE
//       digit run, aligned in the destination (item dst of a run goes to lane dst % 64), so a
//       run of L items costs ceil(((D % 64) + L) / 64) instructions that touch only its own
//       lines, instead of 64-item slices of the tile that start anywhere in a line and cut
//       across runs (every slice then half-writes a line at each end)
//   262144 persistent pass: the next tile's loads are issued after this tile's stores (not
//       after its reorder)
//   524288 persistent pass: the digit-thread waves issue their part of the next tile's loads
//       after their look-back (see PF_SPLIT)
//   1048576 XCD ranges (see draw_ticket_xr): tickets, look-back chains and digit offsets per
//       range of neighbouring tiles on one XCD
//   131072 speculative tile load (grs_onesweep_v4): tile blockIdx.x is loaded while the ticket
//       is in flight; a ticket that differs reloads
//   4194304 tile = blockIdx.x, no ticket (grs_onesweep_v4)
//   8388608 persistent pass without prefetch (grs_onesweep_v6)
//   16777216 every store of the pass nontemporal
//   33554432 nontemporal stores for the 128-B lines wholly inside the tile's digit run, default
//       stores for the run's head and tail lines
//   67108864 16-lane counter sets (4-bit digits): each 16-lane group ranks its own 16 * ITEMS
//       consecutive keys
//   268435456 with 8388608: the tile's stores drained (vmcnt(0)) before the next tile's loads
//   536870912 the group-accumulator add issued at the look-back's finish (not at B1)
//   1073741824 the group-accumulator add at B1 returns nothing; the look-back reads the
//       accumulator back and the group's last tile publishes the inclusive if it is complete

// XCD ranges (OPT 1048576): the tiles form GRS_XCDS contiguous ranges of range_tiles tiles
// (a multiple of the look-back group), one per XCD, each with its own ticket counter and its
// own look-back chain; a tile's digit offsets add the digit counts of the ranges before it
// (per-range histograms of the upfront histogram kernel).  Neighbouring tiles then run on
// one XCD, so the 128-B lines their digit runs share are completed in that XCD's L2 instead
// of reaching HBM as two partial writes.  A workgroup draws from its own XCD's counter and,
// once that range is used up, from the next ones: every range's tiles start in order (the
// look-back's forward progress) whatever the workgroup placement, and the grid's workgroups
// take exactly the grid's tiles.
__device__ __forceinline__ uint32_t xcc_id() {
  // HW_REG_XCC_ID (hwreg 20 on gfx940+), bits [3:0]
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & (GRS_XCDS - 1);
}
__device__ __forceinline__ uint32_t draw_ticket_xr(uint32_t* ticket, uint32_t tiles,
                                                   uint32_t range_tiles) {
  const uint32_t x = xcc_id();
  for (uint32_t k = 0; k < GRS_XCDS; ++k) {
    const uint32_t c = (x + k) & (GRS_XCDS - 1);
    const uint32_t lo = c * range_tiles;
    if (lo >= tiles) continue;
    const uint32_t rc = min(range_tiles, tiles - lo);
    const uint32_t v = atomicAdd(ticket + c, 1u);
    if (v < rc) return lo + v;
  }
  return 0xFFFFFFFFu;   // unreachable: as many workgroups as tiles
}

// Per-XCD ticket heads (OPT 134217728): tile ids = 8 j + c are handed out by counter c in
// increasing j; a workgroup draws from its own XCD's counter and, once that is exhausted, from
// the others in turn.  One head per XCD instead of one for the chip (the dequeue row of the
// microarchitecture guide: 2.8-3.0 us vs 1.1-1.3 us for 256 pullers under streaming).
__device__ __forceinline__ uint32_t draw_ticket_x8(uint32_t* ticket, uint32_t tiles) {
  const uint32_t x = xcc_id();
  for (uint32_t k = 0; k < GRS_XCDS; ++k) {
    const uint32_t c = (x + k) & (GRS_XCDS - 1);
    if (c >= tiles) continue;
    const uint32_t cnt = (tiles - c + GRS_XCDS - 1) / GRS_XCDS;   // tiles with id = c mod 8
    const uint32_t v = atomicAdd(ticket + c, 1u);
    if (v < cnt) return v * GRS_XCDS + c;
  }
  return 0xFFFFFFFFu;   // every tile drawn
}

// Load tile `tile` wave-striped: item j of lane l of wave w is tile key w*64*ITEMS + j*64 + l.
// Keys past n (last tile) are all-ones padding, which sorts after every valid key of its digit.
template <typename K, bool PAIRS, int BLOCK, int ITEMS, int OPT>
__device__ __forceinline__ void tile_load(K (&key)[ITEMS], uint32_t (&val)[ITEMS],
                                          const K* __restrict__ keys_in,
                                          const uint32_t* __restrict__ vals_in, uint32_t n,
                                          uint32_t tile, uint32_t t) {
  constexpr uint32_t TILE = BLOCK * ITEMS;
  const uint32_t lane = t & (GRS_WAVE - 1);
  const uint32_t w = t >> 6;
  const uint32_t tile_base = tile * TILE;
  // G16 (OPT 67108864): each 16-lane group of a wave holds its own 16 * ITEMS consecutive keys
  // (item j of lane l: group offset (l / 16) * 16 * ITEMS + j * 16 + l % 16)
  constexpr bool G16 = (OPT & 67108864) != 0;
  constexpr uint32_t JS = G16 ? 16u : static_cast<uint32_t>(GRS_WAVE);   // item stride
  const uint32_t loff = G16 ? (lane >> 4) * (16u * ITEMS) + (lane & 15u) : lane;
  const uint32_t wbase = tile_base + w * (GRS_WAVE * ITEMS) + loff;
  auto ld = [&](const auto* p, uint32_t i) {
    if constexpr ((OPT & 128) != 0) return __builtin_nontemporal_load(p + i);
    else return p[i];
  };
  constexpr bool IN_REC = (OPT & 4096) != 0;
  static_assert(!IN_REC || (PAIRS && sizeof(K) == 4), "records: u32 key + u32 value");
  static_assert(!IN_REC || !G16, "record loads: wave-striped layout");
  if constexpr (IN_REC) {
    const uint2* rec = reinterpret_cast<const uint2*>(keys_in);
    const uint2* rec_hi = reinterpret_cast<const uint2*>(vals_in);   // split: records [n/2, n)
    const uint32_t half = n / 2;
    const uint32_t valid = n - tile_base;   // tile-local bounds (see below)
    const uint32_t lbase = w * (GRS_WAVE * ITEMS) + lane;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const bool in = valid >= TILE || lbase + j * GRS_WAVE < valid;
      const uint32_t idx = wbase + j * GRS_WAVE;
      const bool hi = (OPT & 16384) != 0 && idx >= half;
      const uint2 x = !in ? make_uint2(~0u, 0u) : hi ? rec_hi[idx - half] : rec[idx];
      key[j] = static_cast<K>(x.x);
      val[j] = x.y;
    }
  } else if (n - tile_base >= TILE) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = ld(keys_in, wbase + j * JS);
    if constexpr (PAIRS) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) val[j] = ld(vals_in, wbase + j * JS);
    }
  } else {
    // the last tile: compare tile-local offsets, never global indices (tile_base + TILE can
    // pass 2^32 when n is near GRS_MAX_N, and a wrapped index would read as in range)
    const uint32_t valid = n - tile_base;
    const uint32_t lbase = w * (GRS_WAVE * ITEMS) + loff;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const bool in = lbase + j * JS < valid;
      key[j] = in ? keys_in[wbase + j * JS] : static_cast<K>(~static_cast<K>(0));
      if constexpr (PAIRS) val[j] = in ? vals_in[wbase + j * JS] : 0u;
    }
  }
}

// One tile, from its loaded (or in-flight) keys to its stores.  Precondition: sm.cnt is zero
// and every thread passed a barrier since it was written and since the previous tile's last
// LDS access.  Leaves sm.cnt dirty.
// PF (persistent workgroups, grs_onesweep_v6): thread 0 draws the next ticket during the
// ranking; after the reorder has moved this tile into LDS (two-round tiles: once the last
// round sits in LDS), the next tile's loads are issued into key/val — their latency hides
// behind the look-back and the stores.  Returns the next
// tile (>= tiles: none); without PF returns tiles.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int OPT, bool PF = false,
          typename DigitF>
__device__ __forceinline__ uint32_t onesweep_tile(
    V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>& sm, uint32_t tile, K (&key)[ITEMS],
    uint32_t (&val)[ITEMS], const K* __restrict__ keys_in,
    K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF& dig, uint32_t gh,
    uint32_t* __restrict__ ticket, uint32_t* __restrict__ status,
    uint32_t* __restrict__ status_next, uint32_t* __restrict__ error_word, uint64_t t_begin,
    const uint32_t* __restrict__ pass_hist = nullptr, uint32_t hist_stride = 0,
    uint32_t range_tiles = 0) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  constexpr bool C16 = (OPT & 256) != 0;
  constexpr int RADIX = SM::RADIX;
  constexpr int WAVES = SM::WAVES;   // counter sets (hardware waves x 4 with G16)
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
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const uint32_t groups = (tiles + G - 1) / G;
  const uint32_t tile_base = tile * TILE;
  const uint32_t valid = (n - tile_base) < static_cast<uint32_t>(TILE) ? (n - tile_base) : TILE;
  const uint32_t pad = TILE - valid;
  const uint32_t dmask = dig.max_digit();
  uint32_t* gacc = status + static_cast<size_t>(tiles) * RADIX;
  uint32_t* ginc = gacc + static_cast<size_t>(groups) * RADIX;
  constexpr bool XR = (OPT & 1048576) != 0;
  // XCD ranges: the pass totals and the counts of the ranges before this tile's (issued here,
  // used at B2 / B4, after the tile's own loads)
  uint32_t roff = 0;
  int32_t g0 = 0;
  if constexpr (XR) {
    const uint32_t x = tile / range_tiles;
    g0 = static_cast<int32_t>((x * range_tiles) / G);
    if (t < static_cast<uint32_t>(RADIX)) {
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t c = 0; c < GRS_XCDS; ++c) {
        const uint32_t v = pass_hist[c * hist_stride + t];
        tot += v;
        roff += c < x ? v : 0u;
      }
      gh = tot;
    }
  }

#define V4_STAMP(k)                                                                        \
  do {                                                                                     \
    if constexpr ((OPT & 8) != 0) {                                                        \
      if (t == 0)                                                                          \
        error_word[64 + static_cast<size_t>(tile) * 12 + (k)] =                             \
            static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t_begin);                 \
    }                                                                                      \
  } while (0)

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
  constexpr bool G16 = (OPT & 67108864) != 0;
  static_assert(!G16 || (!IDX && !C16 && (OPT & 512) == 0 && (OPT & 4096) == 0 &&
                         (OPT & 65536) == 0),
                "16-lane counter sets: plain atomic ranking of loaded keys");
  // counter set of this lane: its wave's, or (G16) its 16-lane group's
  const uint32_t vw = G16 ? w * 4 + (lane >> 4) : w;
  static_assert(!IDX || (GRS_WAVE * ITEMS <= 4096 && RADIX <= 16 && ROUNDS == 1 && !C16),
                "indexed digits ride in the rank field, with 32-bit wave counters");
  uint32_t rank[(ITEMS + 1) / 2];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    uint32_t r;
    if constexpr (IDX) {
      const uint32_t d = dig_of(j);
      if constexpr ((OPT & 512) != 0) {
        const uint64_t m = match_digit<RB>(d);
        const uint32_t below = mbcnt64(m);
        uint32_t* c = &sm.cnt[w * RADIX + d];
        const uint32_t old = *c;
        if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
        r = old + below;
      } else {
        r = atomicAdd(&sm.cnt[w * RADIX + d], 1u);
      }
      r |= d << 12;
    } else if constexpr ((OPT & 512) != 0) {
      // peers of this lane's digit in this item: the lowest one adds their count; LDS runs a
      // wave's instructions in order, so the plain read sees items < j exactly
      static_assert(!C16, "match ranking uses 32-bit counters");
      const uint32_t d = dig_of(j);
      const uint64_t m = match_digit<RB>(d);
      const uint32_t below = mbcnt64(m);
      uint32_t* c = &sm.cnt[w * RADIX + d];
      const uint32_t old = *c;
      if (below == 0) atomicAdd(c, static_cast<uint32_t>(__popcll(m)));
      r = old + below;
    } else if constexpr (C16) {
      const uint32_t d = dig_of(j);
      const uint32_t sh = (d & 1u) << 4;
      r = (atomicAdd(&sm.cnt[(w * RADIX + d) >> 1], 1u << sh) >> sh) & 0xFFFFu;
    } else {
      r = atomicAdd(&sm.cnt[vw * RADIX + dig_of(j)], 1u);
    }
    if (j & 1)
      rank[j / 2] |= r << 16;
    else
      rank[j / 2] = r;
  }
  V4_STAMP(0);
  if constexpr (PF) {
    if (t == 0)
      sm.next = (OPT & 2) != 0 ? tile + gridDim.x
              : XR ? draw_ticket_xr(ticket, tiles, range_tiles)
              : (OPT & 134217728) != 0 ? draw_ticket_x8(ticket, tiles) : atomicAdd(ticket, 1u);  // read after B2
  }
  // this tile's (and its group's) words of the next pass's status buffer
  if (t < static_cast<uint32_t>(RADIX)) {
    status_next[static_cast<size_t>(tile) * RADIX + t] = 0;
    if (tile % G == 0) {
      status_next[static_cast<size_t>(tiles) * RADIX + (tile / G) * RADIX + t] = 0;
      status_next[static_cast<size_t>(tiles + groups) * RADIX + (tile / G) * RADIX + t] = 0;
    }
  }
  lds_barrier();  // B1
  V4_STAMP(1);
  if constexpr (G16) {
    // wave d, lane v: the start of counter set v within digit d's part of the tile (a DPP
    // scan per wave, instead of a digit thread walking 64 sets)
    static_assert(RADIX * GRS_WAVE == BLOCK, "G16: one wave per digit, one lane per counter set");
    const uint32_t c = sm.cnt[lane * RADIX + w];
    const uint32_t incl = wave_scan_dpp(c);
    sm.cnt[lane * RADIX + w] = incl - c;
    if (lane == GRS_WAVE - 1) sm.tcnt[w] = incl;
    lds_barrier();
  }

  constexpr bool ALIGN = (OPT & 65536) != 0 && !IDX;
  constexpr bool WIDE = (OPT & 2097152) != 0;
  // lanes per digit of the wide look-back: the largest power of two <= BLOCK / RADIX, <= 64
  constexpr int LW = (BLOCK / RADIX) >= 64 ? 64 : (BLOCK / RADIX) >= 32 ? 32 : (BLOCK / RADIX) >= 16 ? 16
                   : (BLOCK / RADIX) >= 8 ? 8 : (BLOCK / RADIX) >= 4 ? 4 : 2;
  static_assert(!WIDE || (BLOCK / RADIX >= 2 && !ALIGN && (OPT & 64) == 0),
                "wide look-back: >= 2 lanes per digit, no aligned stores / estimated bases");
  uint32_t tile_cnt = 0, publish = 0, gold = 0, lstart = 0, gstart = 0, cstart = 0, cbound = 0;
  if (t < static_cast<uint32_t>(RADIX)) {
    if constexpr (G16) {
      tile_cnt = sm.tcnt[t];
    } else {
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) {
        const uint32_t c = cnt_ld(ww * RADIX + t);
        cnt_st(ww * RADIX + t, tile_cnt);
        tile_cnt += c;
      }
    }
    publish = (t == dmask) ? tile_cnt - pad : tile_cnt;  // padding is ranked, never counted
    st_status(status + static_cast<size_t>(tile) * RADIX + t, publish + 1u);
    // OPT 536870912: the group-accumulator add is issued just before the look-back's finish
    // (its return is used only there): a value returned here stays live across the reorder,
    // and at 1024 threads (128 VGPRs) it gets spilled, i.e. waited for, right here
    // OPT 1073741824: the add returns nothing (no value to keep live, or to spill and so wait
    // for, across the reorder); the look-back reads the group's accumulator back instead
    if constexpr ((OPT & 1073741824) != 0)
      __hip_atomic_fetch_add(gacc + static_cast<size_t>(tile / G) * RADIX + t,
                             (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if constexpr ((OPT & 536870912) == 0)
      gold = __hip_atomic_fetch_add(gacc + static_cast<size_t>(tile / G) * RADIX + t,
                                    (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (w < static_cast<uint32_t>(DW)) {
    const uint32_t li = wave_scan_dpp(tile_cnt);
    const uint32_t gi = wave_scan_dpp(gh);
    uint32_t ci = 0;
    if constexpr (ALIGN) {
      // store chunks of this digit's run, bounded before its destination alignment is known
      // (the look-back): ceil((63 + L) / 64) >= ceil((D % 64 + L) / 64) for any D
      cbound = publish ? (publish + 126u) >> 6 : 0u;
      ci = wave_scan_dpp(cbound);
    }
    if (lane == GRS_WAVE - 1) {
      sm.wsum[w] = li;
      sm.wsum[WAVES + w] = gi;
      if constexpr (ALIGN) sm.wsum[2 * WAVES + w] = ci;
    }
    lstart = li - tile_cnt;
    gstart = gi - gh;
    cstart = ci - cbound;
    if constexpr (G16) {   // one digit wave (RADIX <= 64): lstart is final here
      if (t < static_cast<uint32_t>(RADIX)) sm.lst16[t] = lstart;
    }
  }
  lds_barrier();  // B2
  V4_STAMP(2);

  static_assert((OPT & 1073741824) == 0 || ((OPT & 2097152) == 0 && (OPT & 536870912) == 0),
                "accumulator read-back: the one-thread-per-digit look-back, add at B1");
  Lb3<RADIX, (ROUNDS > 1 ? GRS_LB_GWIN_XL : GRS_LB_GWIN), (OPT & 1073741824) != 0, (OPT & 4) != 0> lb;
  LbWide<RADIX, WIDE ? LW : 2> lbw;
  const uint32_t wd = t / LW, wj = t & (LW - 1);   // wide look-back: digit and lane in its group
  if (t < static_cast<uint32_t>(RADIX)) {
    for (uint32_t ww = 0; ww < w; ++ww) {
      lstart += sm.wsum[ww];
      gstart += sm.wsum[WAVES + ww];
      if constexpr (ALIGN) cstart += sm.wsum[2 * WAVES + ww];
    }
    if constexpr (ALIGN) {
      sm.cstart[t] = cstart;
      if (t == static_cast<uint32_t>(RADIX - 1)) sm.cstart[RADIX] = cstart + cbound;
      sm.lst[t] = lstart;
      sm.rlen[t] = publish;
    }
    if constexpr (!G16) {
#pragma unroll
      for (int ww = 0; ww < WAVES; ++ww) cnt_st(ww * RADIX + t, cnt_ld(ww * RADIX + t) + lstart);
    }
    if constexpr (IDX) {
      sm.lstart[t] = lstart;
      if (t == static_cast<uint32_t>(RADIX - 1)) sm.lstart[RADIX] = TILE;
    }
    if constexpr (WIDE) {
      sm.lbv[t] = gold;
      sm.lbv[RADIX + t] = publish;
      sm.lbv[2 * RADIX + t] = gstart + roff - lstart;
    } else if constexpr ((OPT & (16 | 64)) == 0 && !PF) {
      lb.issue(status, gacc, ginc, tile, t, g0);
    }
  }
  if constexpr (WIDE && (OPT & 16) == 0 && !PF) {
    if (wd < static_cast<uint32_t>(RADIX)) lbw.issue(status, gacc, ginc, tile, wd, wj, g0);
  }
  if constexpr (G16) sm.cnt[lane * RADIX + w] += sm.lst16[w];   // the fold, one counter a thread
  lds_barrier();  // B3
  V4_STAMP(3);

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
    const uint32_t pos = cnt_ld(vw * RADIX + d) + r;
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
  V4_STAMP(8);   // this wave's reorder issued (stamped by thread 0's wave)
  if constexpr ((OPT & 16) != 0 || PF) {
    if constexpr (WIDE) {
      if (wd < static_cast<uint32_t>(RADIX)) lbw.issue(status, gacc, ginc, tile, wd, wj, g0);
    } else {
      if (t < static_cast<uint32_t>(RADIX)) lb.issue(status, gacc, ginc, tile, t, g0);
    }
  }
  uint32_t next = tiles;
  constexpr bool PF_LATE = (OPT & 262144) != 0;
  // PF_SPLIT: the waves holding digit threads issue their share of the next tile's loads only
  // after their look-back has finished: vmcnt retires loads in issue order, so a look-back poll
  // issued behind the prefetch would wait for all of it
  constexpr bool PF_SPLIT = (OPT & 524288) != 0;
  // NOPF (OPT 8388608): persistent workgroups without prefetch: the next ticket is drawn during
  // the ranking, its tile loaded by the caller's loop once this tile is stored
  constexpr bool NOPF = (OPT & 8388608) != 0;
  if constexpr (PF && ROUNDS == 1 && !PF_LATE && !NOPF) {   // two rounds: after round 2 sits in LDS
    next = __builtin_amdgcn_readfirstlane(sm.next);
    if (next < tiles && (!PF_SPLIT || w >= static_cast<uint32_t>(DW)))
      tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
  }
  if constexpr (WIDE) {
    if (wd < static_cast<uint32_t>(RADIX)) {
      const uint32_t prefix = lbw.finish(status, gacc, ginc, tile, wd, wj, lane, error_word);
      if (wj == 0) {
        const uint32_t wgold = sm.lbv[wd], wpub = sm.lbv[RADIX + wd];
        sm.base[wd] = sm.lbv[2 * RADIX + wd] + prefix;
        const uint32_t g = tile / G;
        const uint32_t in_group = min(static_cast<uint32_t>(G), tiles - g * G);
        if ((wgold >> 24) == in_group - 1u)   // this tile's add completed the group
          st_status(ginc + static_cast<size_t>(g) * RADIX + wd,
                    lbw.gp_out + (wgold & 0xFFFFFFu) + wpub + 1u);
      }
    }
  } else if (t < static_cast<uint32_t>(RADIX)) {
    uint32_t prefix;
    if constexpr ((OPT & 64) != 0) {
      prefix = static_cast<uint32_t>((static_cast<uint64_t>(gh) * tile) / tiles) - roff;
    } else {
      if constexpr ((OPT & 536870912) != 0)
        gold = __hip_atomic_fetch_add(gacc + static_cast<size_t>(tile / G) * RADIX + t,
                                      (1u << 24) | publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prefix = lb.finish(status, gacc, ginc, tile, tiles, t, gold, publish, error_word);
    }
    sm.base[t] = gstart + roff + prefix - lstart;
    V4_STAMP(9);   // thread 0's look-back finished
    if constexpr ((OPT & 33554432) != 0) {
      sm.rbeg[t] = gstart + roff + prefix;
      sm.rend[t] = gstart + roff + prefix + publish;
    }
    if constexpr (ALIGN && ROUNDS > 1) {
      // the run holding tile position LTILE (the round boundary) names the first chunk of
      // round 2: the chunk of that position (it is stored partly in each round)
      if (t == 0) sm.jsplit = 0xFFFFFFFFu;
      const uint32_t D = gstart + roff + prefix;
      if (lstart <= static_cast<uint32_t>(LTILE) && static_cast<uint32_t>(LTILE) < lstart + publish)
        sm.jsplit = cstart + ((D + (LTILE - lstart)) - (D & ~63u)) / 64u;
    }
  }
  // OPT 2048 (with PF_SPLIT): the digit waves' share of the prefetch goes behind their stores
  // instead, so B4 does not wait for its issue
  if constexpr (PF && ROUNDS == 1 && !PF_LATE && PF_SPLIT && !NOPF && (OPT & 2048) == 0) {
    if (next < tiles && w < static_cast<uint32_t>(DW))
      tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
  }
  lds_barrier();  // B4
  V4_STAMP(4);

  // ---- store: consecutive threads write consecutive slots of each digit run ----
  // digit of reordered position i.  Indexed digits: a thread visits increasing positions, so
  // its digit only moves forward through the tile-local digit starts (at most RADIX - 1 steps
  // per tile, over empty digits too).
  uint32_t dcur = 0;
  // store policy (lab): OPT 16777216 every store nontemporal; OPT 33554432 nontemporal for the
  // 128-B lines wholly inside this tile's run of the digit, default for the run's head / tail
  // lines (the ones the neighbouring tiles' runs share)
  auto stv = [&](auto* p, auto v, bool nt) {
    if constexpr (sizeof(v) == 8 && !std::is_integral_v<decltype(v)>) {   // uint2 record
      auto* q = reinterpret_cast<unsigned long long*>(p);
      const unsigned long long x = (static_cast<unsigned long long>(v.y) << 32) | v.x;
      if (nt) __builtin_nontemporal_store(x, q);
      else *q = x;
    } else {
      if (nt) __builtin_nontemporal_store(v, p);
      else *p = v;
    }
  };
  auto put = [&](uint32_t dst, K kk, uint32_t i, bool nt = (OPT & 16777216) != 0) {
    if constexpr ((OPT & 8192) != 0) {
      static_assert(PAIRS && sizeof(K) == 4, "records: u32 key + u32 value");
      const uint2 r = make_uint2(static_cast<uint32_t>(kk), sm.vals[i]);
      if constexpr ((OPT & 32768) != 0) {   // split records: [n/2, n) in vals_out
        if (dst >= n / 2) stv(reinterpret_cast<uint2*>(vals_out) + (dst - n / 2), r, nt);
        else stv(reinterpret_cast<uint2*>(keys_out) + dst, r, nt);
      } else {
        stv(reinterpret_cast<uint2*>(keys_out) + dst, r, nt);
      }
    } else {
      stv(keys_out + dst, kk, nt);
      if constexpr (PAIRS) stv(vals_out + dst, sm.vals[i], nt);
    }
  };
  auto line_in_run = [&](uint32_t dst, uint32_t d) -> bool {
    if constexpr ((OPT & 33554432) != 0) {
      constexpr uint32_t LE = 128 / ((OPT & 8192) != 0 ? 8 : sizeof(K));   // elements per line
      const uint32_t ls = dst & ~(LE - 1);
      return ls >= sm.rbeg[d] && ls + LE <= sm.rend[d];
    } else {
      return (OPT & 16777216) != 0;
    }
  };
  auto dig_at = [&](uint32_t i, K kk) -> uint32_t {
    if constexpr (IDX) {
      while (i >= sm.lstart[dcur + 1]) ++dcur;
      return dcur;
    } else {
      return dig(kk);
    }
  };
  // destination-aligned chunks: wave w takes a contiguous range of chunk indices of this round
  // and walks the digits forward through cstart (wave-uniform values)
  auto store_chunks = [&](uint32_t jbeg, uint32_t jend, uint32_t r0, uint32_t r1) {
    const uint32_t per = (jend - jbeg + WAVES - 1) / WAVES;
    uint32_t j = jbeg + w * per;
    const uint32_t je = min(jend, j + per);
    if (j >= je) return;
    // largest d with cstart[d] <= j (empty digits share the next digit's start)
    uint32_t lo = 0, hi = RADIX;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sm.cstart[mid] <= j) lo = mid; else hi = mid;
    }
    uint32_t d = __builtin_amdgcn_readfirstlane(lo);
    uint32_t cs = __builtin_amdgcn_readfirstlane(sm.cstart[d]);
    uint32_t cn = __builtin_amdgcn_readfirstlane(sm.cstart[d + 1]);
    uint32_t ls = __builtin_amdgcn_readfirstlane(sm.lst[d]);
    uint32_t ln = __builtin_amdgcn_readfirstlane(sm.rlen[d]);
    uint32_t D = __builtin_amdgcn_readfirstlane(sm.base[d]) + ls;
    for (; j < je; ++j) {
      while (j >= cn) {
        ++d;
        cs = cn;
        cn = __builtin_amdgcn_readfirstlane(sm.cstart[d + 1]);
        ls = __builtin_amdgcn_readfirstlane(sm.lst[d]);
        ln = __builtin_amdgcn_readfirstlane(sm.rlen[d]);
        D = __builtin_amdgcn_readfirstlane(sm.base[d]) + ls;
      }
      const uint32_t A = (D & ~63u) + 64u * (j - cs);
      if (A >= D + ln) continue;   // past the run (the chunk bound over-counts by up to one)
      const uint32_t dst = A + lane;
      const uint32_t off = dst - D;   // wraps below D: out of the run
      const uint32_t pos = ls + off;
      if (off < ln && pos >= r0 && pos < r1) {
        const uint32_t i = pos - r0;
        put(dst, sm.keys[i], i);
      }
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
      if constexpr (PF && !NOPF) {
        // the last round's keys are in LDS: the registers take the next tile's loads, which
        // fly behind this round's stores
        if (rr == ROUNDS - 1) {
          next = __builtin_amdgcn_readfirstlane(sm.next);
          if (next < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
        }
      }
    }
    const uint32_t roff = static_cast<uint32_t>(rr * LTILE);
    if constexpr (ALIGN) {
      const uint32_t total = sm.cstart[RADIX];
      const uint32_t js = ROUNDS > 1 ? min(sm.jsplit, total) : total;
      if (rr == 0) store_chunks(0, ROUNDS > 1 ? min(js + 1, total) : total, 0, LTILE);
      else store_chunks(js, total, roff, roff + LTILE);
      continue;
    }
    if (valid == static_cast<uint32_t>(TILE)) {
#pragma unroll
      for (int k = 0; k < LITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        const K kk = sm.keys[i];
        const uint32_t d = dig_at(roff + i, kk);
        uint32_t dst = sm.base[d] + roff + i;
        if constexpr ((OPT & 64) != 0) dst = min(dst, n - 1);
        if constexpr ((OPT & 32) != 0) dst = tile_base + roff + i;
        put(dst, kk, i, line_in_run(dst, d));
      }
    } else {
#pragma unroll
      for (int k = 0; k < LITEMS; ++k) {
        const uint32_t i = k * BLOCK + t;
        if (roff + i < valid) {
          const K kk = sm.keys[i];
          const uint32_t d = dig_at(roff + i, kk);
          const uint32_t dst = sm.base[d] + roff + i;
          put(dst, kk, i, line_in_run(dst, d));
        }
      }
    }
  }
  if constexpr (PF && ROUNDS == 1 && !PF_LATE && PF_SPLIT && !NOPF && (OPT & 2048) != 0) {
    if (next < tiles && w < static_cast<uint32_t>(DW))
      tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
  }
  if constexpr (PF && NOPF) next = __builtin_amdgcn_readfirstlane(sm.next);
  if constexpr (PF && ROUNDS == 1 && PF_LATE && !NOPF) {   // the next tile's loads behind the stores
    next = __builtin_amdgcn_readfirstlane(sm.next);
    if (next < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, next, t);
  }
  if constexpr ((OPT & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    V4_STAMP(5);
    if (t == 0) error_word[64 + static_cast<size_t>(tile) * 12 + 7] = static_cast<uint32_t>(t_begin >> 8);
    // slot 10: every wave's stores drained (absolute, >> 8); slot 11: the CU (XCC, SE, SH, CU)
    asm volatile("s_barrier" ::: "memory");
    if (t == 0) {
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      error_word[64 + static_cast<size_t>(tile) * 12 + 10] =
          static_cast<uint32_t>(__builtin_amdgcn_s_memtime() >> 8);
      error_word[64 + static_cast<size_t>(tile) * 12 + 11] = ((xcc & 0xFu) << 16) | ((hw >> 8) & 0xFFu);
    }
  }
#undef V4_STAMP
  return next;
}

// One tile per workgroup (grid = tiles), tile ids from a ticket counter.  dig_dev: when not
// null, the digit functor is read from device memory instead of the `dig` argument.
template <typename K, bool PAIRS, int RB, int BLOCK, int ITEMS, int MINW, int OPT = 0,
          typename DigitF = RadixDigit<K>>
__global__ __launch_bounds__(BLOCK, MINW) void grs_onesweep_v4(
    const K* __restrict__ keys_in, K* __restrict__ keys_out, const uint32_t* __restrict__ vals_in,
    uint32_t* __restrict__ vals_out, uint32_t n, const DigitF dig,
    const uint32_t* __restrict__ pass_hist, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ status, uint32_t* __restrict__ status_next,
    uint32_t* __restrict__ error_word, const DigitF* __restrict__ dig_dev,
    uint32_t hist_stride = 0, uint32_t range_tiles = 0) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  __shared__ SM sm;
  constexpr bool XR = (OPT & 1048576) != 0;
  const uint64_t t_begin = (OPT & 8) ? __builtin_amdgcn_s_memtime() : 0;
  const uint32_t t = threadIdx.x;
  uint32_t tt = t;
  asm volatile("" : "+v"(tt));
  K key[ITEMS];
  uint32_t val[ITEMS];
  uint32_t tile;
  if constexpr ((OPT & 131072) != 0) {
    // speculative load: with in-order dispatch the ticket mostly equals blockIdx.x, so the
    // tile's loads go out before the ticket's round trip; a different ticket reloads (the
    // ticket alone decides which tile this workgroup sorts)
    const uint32_t guess = blockIdx.x;
    uint32_t tk = 0;
    if (t == 0) tk = atomicAdd(ticket, 1u);
    tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, guess, tt);
    // the ticket goes to LDS after the loads are issued (its wait is then vmcnt(loads))
    if (t == 0) sm.ticket = tk;
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    lds_barrier();
    tile = __builtin_amdgcn_readfirstlane(sm.ticket);
    if (tile != guess) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, tt);
  } else if constexpr ((OPT & 4194304) != 0) {
    // tile = blockIdx.x: no ticket round trip before the loads (see DISPATCH_ORDER below)
    tile = blockIdx.x;
    tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, tt);
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    lds_barrier();
  } else {
    if (t == 0)
      sm.ticket = XR ? draw_ticket_xr(ticket, (n + SM::TILE - 1) / SM::TILE, range_tiles)
                : (OPT & 134217728) != 0 ? draw_ticket_x8(ticket, (n + SM::TILE - 1) / SM::TILE)
                                         : atomicAdd(ticket, 1u);
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    __syncthreads();
    tile = __builtin_amdgcn_readfirstlane(sm.ticket);
    if ((XR || (OPT & 134217728) != 0) && tile >= (n + SM::TILE - 1) / SM::TILE) {   // unreachable (see draw_ticket_xr)
      if (t == 0) atomicOr(error_word, 1u);
      return;
    }
    tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, tt);
  }
  if constexpr ((OPT & 8) != 0) {
    if (t == 0)
      error_word[64 + static_cast<size_t>(tile) * 12 + 6] =
          static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - t_begin);
  }
  const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  // digit functor computed on the device (multi-GPU splitters): uniform scalar loads
  const DigitF dg = dig_dev != nullptr ? *dig_dev : dig;
  onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT>(sm, tile, key, val, keys_in, keys_out, vals_in,
                                                 vals_out, n, dg, gh, ticket, status, status_next,
                                                 error_word, t_begin, pass_hist, hist_stride,
                                                 range_tiles);
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
    uint32_t hist_stride = 0, uint32_t range_tiles = 0) {
  using SM = V4SmemFor<K, PAIRS, RB, BLOCK, ITEMS, OPT, DigitF>;
  __shared__ SM sm;
  constexpr bool XR = (OPT & 1048576) != 0;
  const uint32_t t = threadIdx.x;
  const uint64_t t_entry = (OPT & 8) ? __builtin_amdgcn_s_memtime() : 0;
  // OPT 2: static tiles (blockIdx.x, then + gridDim.x): no ticket round trip, valid only with
  // every workgroup resident (a cooperative launch)
  if (t == 0)
    sm.ticket = (OPT & 2) != 0 ? blockIdx.x
              : XR ? draw_ticket_xr(ticket, (n + SM::TILE - 1) / SM::TILE, range_tiles)
              : (OPT & 134217728) != 0 ? draw_ticket_x8(ticket, (n + SM::TILE - 1) / SM::TILE)
                                       : atomicAdd(ticket, 1u);
  for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
  const uint32_t gh = t < static_cast<uint32_t>(SM::RADIX) ? pass_hist[t] : 0u;
  __syncthreads();
  const DigitF dg = dig_dev != nullptr ? *dig_dev : dig;
  const uint32_t tiles = (n + SM::TILE - 1) / SM::TILE;
  uint32_t tile = __builtin_amdgcn_readfirstlane(sm.ticket);
  K key[ITEMS];
  uint32_t val[ITEMS];
  if (tile < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, t);
  while (tile < tiles) {
    const uint64_t t_begin = (OPT & 8) ? __builtin_amdgcn_s_memtime() : 0;
    tile = onesweep_tile<K, PAIRS, RB, BLOCK, ITEMS, OPT, true>(
        sm, tile, key, val, keys_in, keys_out, vals_in, vals_out, n, dg, gh, ticket, status,
        status_next, error_word, t_begin, pass_hist, hist_stride, range_tiles);
    // every LDS read of the finished tile is done before the counters are reset
    lds_barrier();
    for (uint32_t i = t; i < sizeof(sm.cnt) / 4; i += BLOCK) sm.cnt[i] = 0;
    if constexpr ((OPT & 8388608) != 0) {
      // OPT 268435456: the tile's stores drained before the next tile's loads go out
      if constexpr ((OPT & 268435456) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tile < tiles) tile_load<K, PAIRS, BLOCK, ITEMS, OPT>(key, val, keys_in, vals_in, n, tile, t);
    }
    lds_barrier();
  }
  // stamps: this workgroup's entry and exit (absolute, >> 8) after the tiles' 12 words each
  if constexpr ((OPT & 8) != 0) {
    if (t == 0) {
      uint32_t* wg = error_word + 64 + static_cast<size_t>(tiles) * 12 + 2 * blockIdx.x;
      wg[0] = static_cast<uint32_t>(t_entry >> 8);
      wg[1] = static_cast<uint32_t>(__builtin_amdgcn_s_memtime() >> 8);
    }
  }
}

}  // namespace grs_lab
