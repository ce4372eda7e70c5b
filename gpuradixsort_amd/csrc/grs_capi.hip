// grs_capi.hip — C-ABI of libgrs (include/grs.h): sorter lifecycle, pass driver, helpers.
//
// The pass driver replaces ParallelSort::Sort (Source/ComputeControllers/ParallelSort.cpp:168-298):
// where the reference issues 1 + 32 x 4 GLSL dispatches with a glMemoryBarrier after each,
// one grs_sort call issues
//     grs_upfront_hist2  -> P x grs_onesweep_v4 / v6
// on one stream (no memset: the histogram kernel zeroes the other of two control blocks for
// the next call, see grs_sorter::cb_i) (P = ceil((end_bit - begin_bit) / radix_bits); 4 launches for u32 at 8-bit
// digits), plus one D2D copy when P is odd so the result lands back in the caller's buffer
// (the reference's glCopyBufferSubData, ParallelSort.cpp:312-318).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/grs.h"
#include "grs_config.h"
#include "grs_kernels.hpp"
#include "grs_pass.hpp"
#include "grs_msd.hpp"
#include "grs_shard.hpp"
#include "grs_codec.hpp"

#include <rccl/rccl.h>

namespace {

thread_local std::string g_last_error;

grs_status set_err(grs_status s, const std::string& msg) {
  g_last_error = msg;
  return s;
}

#define GRS_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      return set_err(GRS_EHIP, std::string(#call) + " (grs_capi.hip:" +                \
                                   std::to_string(__LINE__) + "): " + hipGetErrorString(e_)); \
  } while (0)

// Tile shapes of the pass (grs_onesweep_v4, grs_pass.hpp).  Measured on MI355X inside the
// sort (tools/ab_r2.sh, ab_r2b.sh; C4 = 2^30 u32 keys, same box, Gkeys/s): 16 waves per
// workgroup, 16-bit wave counters (half the counter LDS, so the tile grows to what LDS then
// holds: 36K u32 keys) and the look-back issued after the reorder: 126.5 vs 120.7 (32K tiles,
// 32-bit counters, early look-back), 125.2 (512 x 72), 107.7 (nontemporal tile loads); C3
// 59.9 vs 59.2, C5 33.4 vs 32.8.  Big: one 1024-thread workgroup per CU.  Small (grids of
// less than one big tile per CU): 256-thread workgroups of 1.5K-4K keys, four per CU.
// u64 pairs: a tile twice what LDS holds, reordered in two rounds (the keys and payloads stay
// in VGPRs, LDS takes half the tile at a time; 32-bit wave counters): 22K-pair tiles, same
// process (tools/lab2.py, 2^28 pairs, ms per pass) 1.37 vs 1.48 and 1.45 vs 1.72 on two boxes
// against one-round 11K tiles.  u32 pairs (26K tiles) and u64 keys (28K-32K) measured no gain.
template <typename K, bool PAIRS>
struct BigTile {
  static constexpr int BLOCK = 1024, MINW = 1;
  static constexpr bool TWO_ROUNDS = sizeof(K) == 8 && PAIRS;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 17 : 36) : (PAIRS ? 22 : 17);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr uint32_t OPT = TWO_ROUNDS ? (1024u | 16u) : (256u | 16u);
};
// u32 keys at 8-bit digits, large grids: 48K-key tiles of 768 threads x 64 keys reordered in
// two rounds (LDS takes half the tile; 168 VGPRs at 3 waves per SIMD).  Longer digit runs per
// tile: the pass alone (tools/lab2.py, 2^30 keys, same box) 1.90 vs 2.03 ms for the 36K tile,
// 2^29 0.947 vs 0.974; slower at 2^27 (0.278 vs 0.259) and, inside the sort, at 2^28 (118 vs
// 121.5 Gkeys/s; C4 2^30: 129-130 vs 122-124, tools/ab_xl.sh).  Used from 32 XL tiles per CU.
// The same for u32 pairs (768 x 40: 2^28 pairs 1.01 vs 1.06 ms per pass) and u64 keys
// (768 x 44: 0.93 vs 0.96), tools/lab2.py.
template <typename K, bool PAIRS>
struct XLTile {
  static constexpr int BLOCK = 768, MINW = 1;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 40 : 64) : (PAIRS ? 28 : 44);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr bool TWO_ROUNDS = true;
  static constexpr uint32_t OPT = 1024u | 16u;
};
// 4-bit digits (BASELINE C2): 32-bit wave counters (16-bit ones put 64 lanes on 8 words) and
// the look-back before the reorder (tools/lab2.py at 2^24 keys: 1024 x 32 0.042 ms per pass).
template <typename K, bool PAIRS>
struct BigTile4 {
  static constexpr int BLOCK = 1024, MINW = 1;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 16 : 32) : (PAIRS ? 10 : 16);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr bool TWO_ROUNDS = false;
};
template <typename K, bool PAIRS>
struct SmallTile {
  static constexpr int BLOCK = 256, MINW = 4;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 8 : 16) : (PAIRS ? 6 : 8);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr bool TWO_ROUNDS = false;
};
// Ballot-match fallback (32-bit wave counters): the round's first 16-wave shapes.
template <typename K, bool PAIRS>
struct MatchTile {
  static constexpr int BLOCK = 1024, MINW = 1;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 16 : 32) : (PAIRS ? 10 : 16);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr bool TWO_ROUNDS = false;
};
// Partition pass (key-range buckets for the multi-GPU exchange): big tiles (its digit needs
// the element index, so the store phase reads a position's digit off the tile-local digit
// starts instead of the key).  u32 keys: 1024 x 32, not x 36 -- the composite splitter compares
// push the 36-key tile to 128 VGPRs and scratch spills (tools/lab6.py, 2^27 keys into 8
// buckets: 0.304-0.311 vs 0.341 ms a pass; a 12-bit bucket table in LDS instead of the compares
// 0.329-0.360, 32-bit compares with a branch for keys equal to a splitter 0.331).
template <typename K, bool PAIRS>
struct PartTile {
  static constexpr int BLOCK = 1024, MINW = 1;
  static constexpr int ITEMS = sizeof(K) == 4 ? (PAIRS ? 17 : 32) : (PAIRS ? 11 : 17);
  static constexpr int TILE = BLOCK * ITEMS;
  static constexpr bool TWO_ROUNDS = false;
};
// Pass options (grs_pass.hpp OPT bits): big tiles 16-bit wave counters + look-back after the
// reorder; small tiles the look-back after the reorder.  Default-policy tile loads:
// nontemporal loads made the pass alone faster in tools/lab2.py but the sort slower (C4 2^30
// keys, same box: 107.5 vs 122.4 Gkeys/s), the pass reading what the previous pass just wrote.
constexpr uint32_t kBig4Opt = 0;
constexpr uint32_t kSmallOpt = 16;
constexpr uint32_t kMatchOpt = 512 | 16;               // ballot-match ranking (fallback)
// (XCD ranges were a lab option, git show 729d494:tools/lab_pass.hpp: they need the digit counts of every
// range for every pass, and a range of pass p > 0 holds the keys pass p - 1 scattered there,
// which no upfront histogram of the input positions gives)

// Status words of one look-back buffer for `tiles` tiles of radix `radix`.
size_t status_words_for(size_t tiles, size_t radix) { return grs::lb3_status_words(tiles, radix); }

// Probe of the property the atomic-rank passes rely on: the lanes of ONE returning ds_add
// wave-instruction that hit one LDS address get their old values in ascending lane order
// (tools/ldsorder.hip checks it at scale).  out[0] += number of mismatching lanes.
__global__ void grs_probe_lds_order(uint32_t* out) {
  __shared__ uint32_t cnt[256];
  const uint32_t lane = threadIdx.x;  // one wave
  uint32_t bad = 0;
  for (int pattern = 0; pattern < 6; ++pattern) {
    for (uint32_t i = lane; i < 256; i += 64) cnt[i] = 0;
    __syncthreads();
    for (uint32_t round = 0; round < 4; ++round) {
      uint32_t d;
      switch (pattern) {
        case 0: d = 7; break;                                   // all lanes, one address
        case 1: d = lane % 3; break;
        case 2: d = (lane * 37u + round * 11u) & 255u; break;
        case 3: d = (lane & 1) ? 5u : 37u; break;                // two addresses, one bank
        case 4: d = (grs::splitmix64(lane * 131u + round) >> 7) & 15u; break;
        default: d = 255u - lane / 4; break;
      }
      const uint32_t before = cnt[d];
      __syncthreads();
      uint32_t below = 0;
      for (uint32_t l2 = 0; l2 < 64; ++l2) {
        const uint32_t d2 = __shfl(d, l2, 64);
        below += (l2 < lane && d2 == d) ? 1u : 0u;
      }
      const uint32_t old = atomicAdd(&cnt[d], 1u);
      bad += old != before + below;
      __syncthreads();
    }
  }
  if (bad) atomicAdd(out, bad);
}

// At-scale lane-order check (grs_lds_order_check): every wave of 8 ranks `items` digits per
// lane with returning atomics on its own counters and checks each returned value against
// ref[d] + (lower lanes of this item with digit d), from a ballot match and a wave-ordered
// plain LDS count (the LDS runs one wave's instructions in order).
template <int RB, int PACK>
__global__ __launch_bounds__(512) void grs_lds_order_scale(uint32_t pattern, uint32_t items,
                                                           unsigned long long* bad) {
  constexpr int RADIX = 1 << RB;
  __shared__ uint32_t cnt[8][RADIX / PACK];
  __shared__ uint32_t ref[8][RADIX];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t i = threadIdx.x; i < 8u * RADIX / PACK; i += 512) (&cnt[0][0])[i] = 0;
  for (uint32_t i = threadIdx.x; i < 8u * RADIX; i += 512) (&ref[0][0])[i] = 0;
  __syncthreads();
  unsigned long long nbad = 0;
  const uint64_t seed = (static_cast<uint64_t>(blockIdx.x) * 8 + w) * 0x9E3779B97F4A7C15ull + pattern;
  for (uint32_t j = 0; j < items; ++j) {
    const uint64_t r = grs::splitmix64(seed ^ (static_cast<uint64_t>(j) * 64 + lane));
    uint32_t d;
    switch (pattern) {
      case 0: d = static_cast<uint32_t>(r) & (RADIX - 1); break;                 // uniform
      case 1: d = 7u & (RADIX - 1); break;                                        // all equal
      case 2: d = (static_cast<uint32_t>(r) & 3u) * (RADIX / 4); break;           // 4 values, one bank
      case 3: d = lane < 32 ? 3u : static_cast<uint32_t>(r) & (RADIX - 1); break; // half the lanes
      default: d = ((static_cast<uint32_t>(r) & 15u) * 32u) & (RADIX - 1); break; // 16 values, one bank
    }
    const uint64_t m = grs::match_digit<RB>(d);
    const uint32_t below = grs::mbcnt64(m);
    const uint32_t expect = ref[w][d] + below;
    uint32_t got;
    if constexpr (PACK == 2) {
      const uint32_t sh = (d & 1u) << 4;
      got = (atomicAdd(&cnt[w][d >> 1], 1u << sh) >> sh) & 0xFFFFu;
    } else {
      got = atomicAdd(&cnt[w][d], 1u);
    }
    nbad += got != expect;
    if (below == 0) ref[w][d] += static_cast<uint32_t>(__popcll(m));
  }
  if (nbad) atomicAdd(bad, nbad);
}

// Rank mode per device: 0 = atomic ranking (probe passed), 1 = ballot-match fallback.
// grs_set_option(GRS_OPT_RANK, 1) forces the fallback on one sorter (tests cover both paths).
int device_rank_mode(int device) {
  static std::mutex mu;
  static int mode[64];
  static bool known[64];
  std::lock_guard<std::mutex> lock(mu);
  if (device >= 0 && device < 64 && known[device]) return mode[device];
  int m = 1;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 4) == hipSuccess) {
    uint32_t h = 1;
    if (hipMemset(d, 0, 4) == hipSuccess) {
      hipLaunchKernelGGL(grs_probe_lds_order, dim3(1), dim3(64), 0, 0, d);
      if (hipGetLastError() == hipSuccess && hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost) == hipSuccess)
        m = h == 0 ? 0 : 1;
    }
    (void)hipFree(d);
  }
  (void)hipGetLastError();
  if (device >= 0 && device < 64) {
    mode[device] = m;
    known[device] = true;
  }
  return m;
}

}  // namespace

struct grs_sorter {
  int device = 0;
  grs_key_type key_type = GRS_KEY_U32;
  int pairs = 0;
  int radix_bits = 8;
  int rank_mode = 0;               // 0: lane-ordered LDS atomics, 1: ballot-match fallback
  int cus = 0;                     // compute units of the device
  size_t capacity = 0;
  void* alt_keys = nullptr;
  uint32_t* alt_vals = nullptr;
  bool alt_joint = false;          // u32 pairs: alt_vals lies inside alt_keys' allocation (8n bytes)
  int rec_mode = 2;                // GRS_OPT_RECORDS: 0 two arrays, 1 records in the scratch
                                   // only, 2 also split over the caller's arrays
  uint32_t* status = nullptr;      // 2 look-back status buffers: [status_words] | band | [status_words]
  size_t status_words = 0;         // per buffer
  size_t status_stride = 0;        // words from the first buffer to the second
  uint32_t* ctrl = nullptr;        // GRS_CTRL_WORDS
  // run_sort's histogram + ticket block alternates between ctrl and ctrl2: cb[cb_i] is zero at
  // the start of the next call (each call's histogram kernel zeroes the other one for the
  // call after it), so a sort launches no memset; cb_dirty: the partition pass used ctrl
  uint32_t* ctrl2 = nullptr;       // GRS_CTRL_ERROR words (no error word)
  int cb_i = 0;
  bool cb_dirty = false;
  uint32_t* h_err = nullptr;       // pinned host word: the error word read back by checked calls
  size_t scratch_bytes = 0;
  // Profiling ring: the last `ring` calls keep their per-phase hipEvents.
  static constexpr int EV_PER_CALL = GRS_MAX_PASSES + 3;
  int ring = 0;
  long long calls = 0;             // profiled calls recorded so far
  hipEvent_t* ev = nullptr;        // ring * EV_PER_CALL events
  struct CallInfo { int ev_used; int passes; bool copy; int kind = 0; };   // kind 1: MSD
  CallInfo* info = nullptr;        // ring entries
  // grs_sort_segmented scratch (allocated on first use, grown on demand)
  void* seg_buf = nullptr;
  size_t seg_bytes = 0;
  grs_sorter* seg64 = nullptr;     // u64 pair sorter of (segment << 32 | key), u32 keys only
  void* host_stage = nullptr;      // grs_sort_host device staging (keys | payload), on first use
  size_t host_stage_bytes = 0;
  // grs_sort_sharded scratch (first use): samples, gathered samples, count matrix, digit
  void* shard_buf = nullptr;
  size_t shard_bytes = 0;
  void* rec_buf = nullptr;         // record sorts: per-call keys | index | record copy
  size_t rec_bytes = 0;
  void* rec_kbuf = nullptr;        // grs_records_key_buffers: keys | index for the capacity
  uint32_t* shard_host = nullptr;  // pinned: the G x G count matrix read back once per call
  void* xbuf = nullptr;            // grs_sort_sharded send buffer: G regions of n_local items
  size_t xbuf_bytes = 0;
  void* xrbuf = nullptr;           // presorted exchange: the received (encoded) words
  size_t xrbuf_bytes = 0;
  void* codec_buf = nullptr;       // presorted exchange: plan, block sizes / offsets, scan, co-ranks
  size_t codec_bytes = 0;
  // options (grs_set_option; defaults pick by size; nothing is read from the environment)
  int sharded_exchange = 0;        // GRS_OPT_EXCHANGE: 0 auto, 1 partition-first, 2 presorted,
                                   // 3 chunked partition-first (keys only)
  int x_chunks = 0;                // GRS_OPT_X_CHUNKS: chunks of the chunked exchange (0: 4)
  // the chunked exchange's second stream (RCCL calls) and events, created on first use
  hipStream_t xstream = nullptr;
  hipEvent_t xcev[17] = {};        // [c]: chunk c partitioned; [16]: the exchange done
  hipEvent_t xhev = nullptr;       // a chunk's count rows landed on the host
  uint32_t* xchunk_host = nullptr; // pinned: one chunk's count rows (G rows of G + 3 words)
  int merge_mode = 0;              // GRS_OPT_MERGE: 0 ceil(log2 k) 2-way rounds, 1 one k-way pass
  // last grs_sort_sharded call, with profiling on: events at call start / exchange start /
  // exchange end / call end, and the bytes that crossed the links (self part excluded)
  hipEvent_t xev[4] = {};
  bool xev_recorded = false;
  uint64_t x_sent = 0, x_recv = 0;
  int x_presorted = 0;
  uint64_t x_region_redo = 0;      // sharded partitions redone into contiguous buckets (spills)
  int tile_mode = -1;              // GRS_OPT_TILE: -1 by size, 0 small, 1 big
  int pass_mode = 0;               // GRS_OPT_PASS: 0 auto, 4 = grs_onesweep_v4, 6 = grs_onesweep_v6,
                                   // 8 = grs_onesweep_fused
  bool sharded_general = false;    // GRS_OPT_SHARDED_PATH: one rank takes the G-rank path too
  int sharded_send = 0;            // GRS_OPT_SHARDED_SEND: 0 regions, 1 histogram + contiguous
                                   // buckets, 2 test: regions of n / (2G) (full buckets spill)
  int xl_mode = 0;                 // GRS_OPT_XL: 0 by size, 1 wherever big tiles run, 2 never
  int probe_rank_mode = 0;         // the device probe's ranking (GRS_OPT_RANK 0 restores it)
  int fault_tile = -1;             // GRS_OPT_FAULT_TILE (test hook; ctrl debug words)
  uint32_t h2_chunk = 0;           // GRS_OPT_H2_CHUNK: 0 by size, else H2's chunk (keys per block)
  uint32_t h2_piece = 0;           // GRS_OPT_H2_PIECE: 0 default, else H2's sample piece (keys)
  int p3_mode = 0;                 // GRS_OPT_P3: 0 a workgroup per segment, 1 persistent with
                                   // prefetch (u32 keys / pairs; measured slower, round 6), 2 as 0
                                   // without the low-halves kernel for C4's size
  int seg_route = 0;               // GRS_OPT_SEG_ROUTE: 0 by shape, 1 segmented passes, 2 one
                                   // composite-key sort (grs_sort_segmented's longer segments)
  int msd_mode = -1;               // GRS_OPT_MSD: -1 by size, 0 never, 1 whenever it applies,
                                   // 2 = 1 with P2's regions refused (test hook: the exact redo)
  // The MSD sort's scratch (msd_scratch): allocated at grs_create from kMsdMinN items of capacity,
  // by grs_set_option(GRS_OPT_MSD, 1 | 2) below it; released by GRS_OPT_MSD = 0
  void* msd_buf = nullptr;         // the MSD sort's tables (u32 keys without payload, 8-bit)
  void* alt2_keys = nullptr;       // the MSD sort's P2 regions (keys | guard band | payload)
  uint32_t* alt2_vals = nullptr;
  size_t msd_bytes = 0;
  size_t alt_words = 0;            // elements per array of the second buffer (alt)
  // Every device scratch allocation ends in a guard band of kGuardBytes (and allocations that
  // hold several arrays have bands between them), filled with a pattern when allocated and
  // checked by grs_debug_check_guards: a kernel that writes past a scratch array shows there.
  struct ScratchBuf {
    void** owner;                  // the sorter field holding the allocation
    size_t bytes;                  // allocated bytes (bands included)
    std::vector<size_t> bands;     // byte offsets of its guard bands
  };
  std::vector<ScratchBuf> bufs;
  int last_msd_cb = -1;            // the control block of the last sort when it ran the MSD
                                   // schedule, else -1 (grs_debug_msd_flags)
  uint32_t* last_msd_spill2 = nullptr;
  size_t alt_inner_band = 0;       // u32 pairs: the band between alt's keys and payload, which
  bool alt_band_dirty = false;     // the LSD record passes write records across (restored by
                                   // the next MSD sort or guard check)
};

namespace {

// ---- scratch allocations with guard bands (grs_debug_check_guards) ----
constexpr size_t kGuardBytes = 16384;
constexpr uint32_t kGuardWord = 0x6A7DBA5Eu;

hipError_t fill_band(void* at) {
  static const std::vector<uint32_t> pattern(kGuardBytes / 4, kGuardWord);
  return hipMemcpy(at, pattern.data(), kGuardBytes, hipMemcpyHostToDevice);
}

// Frees *p (if any) and forgets its guard bands.
void sbuf_free(grs_sorter* s, void** p) {
  for (size_t i = 0; i < s->bufs.size(); ++i)
    if (s->bufs[i].owner == p) {
      s->scratch_bytes -= s->bufs[i].bytes;
      s->bufs.erase(s->bufs.begin() + static_cast<long>(i));
      break;
    }
  if (*p) (void)hipFree(*p);
  *p = nullptr;
}

// *p = a new allocation (the old one freed first) of `bytes` for the caller followed by a guard
// band; inner = byte offsets in [0, bytes) of further kGuardBytes bands the caller laid out
// between its arrays.  On the current device.
grs_status sbuf_alloc(grs_sorter* s, void** p, size_t bytes, const char* what,
                      std::vector<size_t> inner = {}) {
  sbuf_free(s, p);
  void* d = nullptr;
  if (hipMalloc(&d, bytes + kGuardBytes) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(GRS_ENOMEM, std::string(what) + ": hipMalloc of " + std::to_string(bytes + kGuardBytes) +
                                   " bytes failed");
  }
  inner.push_back(bytes);
  for (size_t o : inner)
    if (fill_band(static_cast<char*>(d) + o) != hipSuccess) {
      (void)hipFree(d);
      return set_err(GRS_EHIP, std::string(what) + ": guard band fill failed");
    }
  *p = d;
  s->bufs.push_back({p, bytes + kGuardBytes, inner});
  s->scratch_bytes += bytes + kGuardBytes;
  return GRS_OK;
}

// Device buffer grown on demand (contents are not kept).
grs_status grow_buf(grs_sorter* s, void** p, size_t* have, size_t need, const char* what) {
  if (*have >= need && *p) return GRS_OK;
  *have = 0;
  const grs_status r = sbuf_alloc(s, p, need, what);
  if (r == GRS_OK) *have = need;
  return r;
}

}  // namespace

extern "C" {

int grs_version(void) { return GRS_VERSION; }

const char* grs_status_string(grs_status s) {
  switch (s) {
    case GRS_OK: return "GRS_OK";
    case GRS_EINVAL: return "GRS_EINVAL";
    case GRS_ENOMEM: return "GRS_ENOMEM";
    case GRS_EHIP: return "GRS_EHIP";
    case GRS_ECAPACITY: return "GRS_ECAPACITY";
    case GRS_ENODEV: return "GRS_ENODEV";
    case GRS_ETIMEOUT: return "GRS_ETIMEOUT";
    case GRS_ERCCL: return "GRS_ERCCL";
  }
  return "GRS_UNKNOWN";
}

const char* grs_last_error(void) { return g_last_error.c_str(); }

void grs_destroy(grs_sorter* s) {
  if (!s) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(s->device);
  // every device scratch allocation (alt, alt2, status, control blocks, tables, the grown
  // buffers) is registered with its guard bands
  for (grs_sorter::ScratchBuf& b : s->bufs)
    if (*b.owner) {
      (void)hipFree(*b.owner);
      *b.owner = nullptr;
    }
  s->bufs.clear();
  if (s->h_err) (void)hipHostFree(s->h_err);
  if (s->seg64) grs_destroy(s->seg64);
  if (s->shard_host) (void)hipHostFree(s->shard_host);
  for (int i = 0; s->ev && i < s->ring * grs_sorter::EV_PER_CALL; ++i)
    if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
  for (hipEvent_t e : s->xev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : s->xcev)
    if (e) (void)hipEventDestroy(e);
  if (s->xhev) (void)hipEventDestroy(s->xhev);
  if (s->xstream) (void)hipStreamDestroy(s->xstream);
  if (s->xchunk_host) (void)hipHostFree(s->xchunk_host);
  delete[] s->ev;
  delete[] s->info;
  (void)hipSetDevice(prev);
  delete s;
}

}  // extern "C"

namespace {

// Tiles of the pass a sort of n items launches, and which shape (true = big).
bool use_big_tiles(const grs_sorter* s, size_t n, size_t big_tile) {
  if (s->tile_mode >= 0) return s->tile_mode == 1;
  // big tiles from one tile per CU up (tools/lab2.py, C2's 2^24 keys at 4-bit digits: 32K-key
  // tiles 0.042 ms per pass, two per CU, against 0.070 for 4K-key tiles, 4 workgroups per CU)
  return (n + big_tile - 1) / big_tile >= static_cast<size_t>(std::max(1, s->cus));
}

// Big-tile pass kernel: the persistent one (grs_onesweep_v6: the next tile's loads fly behind
// the current tile's look-back and stores) where a CU sees only a few tiles, so the exposed
// load of each tile dominates; one tile per workgroup (grs_onesweep_v4) otherwise.  Same box,
// tools/ab_pass.sh, Gkeys/s v6 vs v4: C2 49.8 vs 45.3; C4 119.3 vs 124.2, C3 56.5 vs 61.1,
// C5 32.5 vs 34.3.
bool use_persistent(const grs_sorter* s, size_t tiles, int rb) {
  if (s->pass_mode != 0) return s->pass_mode == 6 || s->pass_mode == 8;
  return rb == 4 || tiles <= 4u * static_cast<size_t>(std::max(1, s->cus));
}

// XL tiles (8-bit digits, big tiles, atomic ranking): forced, or from 32 per CU.
bool use_xl(const grs_sorter* s, size_t n, size_t xl_tile) {
  if (s->rank_mode != 0 || s->xl_mode == 2) return false;
  return s->xl_mode == 1 ||
         (n + xl_tile - 1) / xl_tile >= 32u * static_cast<size_t>(std::max(1, s->cus));
}

// ---- MSD sort (grs_msd.hpp): tables and their layout in the sorter's msd_buf ----
// u32 keys, u32 keys + u32 payload, u64 keys (8-bit digits).
// P3 shapes: one workgroup sorts a 16-bit segment of up to BLOCK * I elements in LDS.
template <int B, int I_, bool C> struct MsdLocal {
  static constexpr int BLOCK = B, I = I_;
  static constexpr bool C16 = C;
  static constexpr uint32_t SMAX = B * I_;
};
using MsdLocalS = MsdLocal<256, 8, false>;    // small sorts: the unrolled item loop costs what
using MsdLocalM = MsdLocal<256, 12, false>;   // the shape holds, not what the segment holds
using MsdLocalA = MsdLocal<256, 20, false>;   // any element (40 KB of LDS at 8 B)
using MsdLocalB = MsdLocal<512, 20, false>;
using MsdLocalW = MsdLocal<1024, 5, false>;   // u64 keys in A's place: 5120 keys, sixteen waves (the
                                              // two rounds + run finish, 1.40 ms at 2^28 against 1.74
                                              // for 256 x 20, tools/lab8.py round 6)
using MsdLocalC2 = MsdLocal<768, 23, true>;   // 4-byte elements, C4's 2^30 keys: C less one item a
                                              // thread (7 % empty slots instead of 11 %: P3 1.95 vs
                                              // 2.04 ms at 2^30, tools/lab8.py round 6)
using MsdLocalC = MsdLocal<768, 24, true>;    // 4-byte elements: two 72-KB workgroups per CU
using MsdLocalD = MsdLocal<1024, 36, true>;   // 4-byte elements past 1.13G keys: one 152-KB workgroup
                                              // per CU (the MSD sort to ~2.3G keys)
constexpr uint32_t kMsdSmaxMin = MsdLocalS::SMAX;
// fallback and redo passes (persistent): the big tile of the key type; 17408 keys is the
// smallest of them (u32 pairs, u64 keys), which sizes the tables
constexpr uint32_t kMsdTileMin = 17408;
static_assert(BigTile<uint32_t, true>::TILE == kMsdTileMin && BigTile<uint64_t, false>::TILE == kMsdTileMin &&
              BigTile<uint32_t, false>::TILE > kMsdTileMin, "MSD table sizing");

struct MsdLayout {   // word offsets into msd_buf
  size_t h2, h2x, h2s, big, spill2, mid, clear, dstart, reg, room, len2, in2, out2, tab, hdr2, rec2, hdr2r, rec2r,
      hdrf, recf, bin, bstart, blen, brow, rows, spill, words;
  size_t r2, rf, bl, mr;   // capacities: P2 records, fallback records, big list, histogram rows
  std::vector<size_t> bands;   // byte offsets of the guard bands between the tables
  // nd: digits of the fallback (2 for u32 keys, 6 for u64)
  static MsdLayout of(size_t cap, size_t nd) {
    MsdLayout L{};
    cap = std::max<size_t>(cap, 1);
    L.r2 = cap / kMsdTileMin + 257;
    L.bl = std::min<size_t>(65536, cap / (kMsdSmaxMin + 1) + 2);
    L.mr = cap / (kMsdTileMin + 1) + 2;
    L.rf = cap / kMsdTileMin + L.bl + 1;
    size_t o = 0;
    // every table followed by a guard band (the last one's is sbuf_alloc's own)
    auto take = [&](size_t w) {
      if (o != 0) {
        L.bands.push_back(o * 4);
        o += kGuardBytes / 4;
      }
      const size_t at = o;
      o += (w + 63) & ~static_cast<size_t>(63);
      return at;
    };
    // h2 (P2's digit totals) | h2x (exact counts, after a P2 spill) | h2s (sampled counts) |
    // big counters, P2's spill flag | mid list: the first `clear` words zeroed by the sample kernel
    L.h2 = take(3 * 65536 + 64 + 2 + 3 * 65536);
    L.h2x = L.h2 + 65536;
    L.h2s = L.h2 + 2 * 65536;
    L.big = L.h2 + 3 * 65536;
    L.spill2 = L.big + 8;
    L.mid = L.big + 64;
    L.clear = 3 * 65536 + 64 + 2;
    L.dstart = take(65536);
    L.reg = take(65536);
    L.room = take(256);
    L.len2 = take(65536);
    L.in2 = take(65536);
    L.out2 = take(65536);
    L.tab = take(4 * 257);
    L.hdr2 = take(4);
    L.rec2 = take(L.r2 * 8);
    L.hdr2r = take(4);
    L.rec2r = take(L.r2 * 8);
    L.hdrf = take(4);
    L.recf = take(L.rf * 8);
    L.bin = take(L.bl);
    L.bstart = take(L.bl);
    L.blen = take(L.bl);
    L.brow = take(L.bl);
    L.rows = take(L.mr * nd * 256);
    L.spill = take(6 * (L.bl + 1));
    L.words = o;
    return L;
  }
  // status words of P2 (256 buckets) and of the fallback passes
  static size_t status_words(size_t cap) {
    cap = std::max<size_t>(cap, 1);
    const size_t t2 = cap / kMsdTileMin + 257;
    const size_t w2 = (t2 + 2 * (t2 / GRS_LB_GROUP + 257)) * 256;
    const size_t tf = 2 * (cap / kMsdTileMin) + 2;            // tiles of multi-tile segments
    const size_t gf = tf / GRS_LB_GROUP + cap / (kMsdTileMin + 1) + 2;
    return std::max(w2, (tf + 2 * gf) * 256);
  }
};

// Elements of the sorter's second buffer (per array) for an MSD sorter: P1 writes its runs
// into sampled regions (n + n/8 + 256 x 4096 + 256 elements at most, grs_msd.hpp).
size_t msd_alt_words(size_t cap) { return std::max<size_t>(cap, 1) + cap / 8 + 256 * 4096 + 1024; }
// Elements of the third buffer (per array): P2 writes its runs into regions sized from a sample
// of P1's output (grs_msd_plan3: at most this many, else the exact path runs).
size_t msd_alt2_words(size_t cap) { return std::max<size_t>(cap, 1) + cap / 10 * 3 + 65536 * 64 + 1024; }

bool msd_type(const grs_sorter* s) {
  return s->radix_bits == 8 && !(s->key_type == GRS_KEY_U64 && s->pairs);
}
// From this many keys the MSD sort is the default (GRS_OPT_MSD = -1), and a sorter of this
// capacity allocates its scratch at grs_create.
constexpr size_t kMsdMinN = size_t(3) << 24;   // MSD vs LSD, same box (r5 s12-13): 2^25 84 vs 88, 2^26 106 vs 96 Gkeys/s
size_t msd_digits(const grs_sorter* s) { return s->key_type == GRS_KEY_U64 ? 6 : 2; }

// Status words one pass of a sort of up to `cap` items can need (largest over the shapes).
template <typename K, bool PAIRS>
size_t max_status_words(const grs_sorter* s, size_t cap, size_t radix) {
  const size_t big = std::min(BigTile<K, PAIRS>::TILE, BigTile4<K, PAIRS>::TILE);
  const size_t small = SmallTile<K, PAIRS>::TILE;
  size_t w0 = 0;
  // small tiles are used below one big tile per CU (or everywhere when forced): below the
  // LARGER of the two big tiles per CU (use_big_tiles asks with the sort's own big tile; sized
  // with the smaller one, u32 pairs and u64 sorts of 4.19M-4.46M items were refused)
  const size_t big_max = std::max(BigTile<K, PAIRS>::TILE, BigTile4<K, PAIRS>::TILE);
  const size_t small_cap = s->tile_mode == 0 ? cap : std::min(cap, big_max * std::max(1, s->cus));
  const size_t match = MatchTile<K, PAIRS>::TILE;
  w0 = status_words_for((cap + match - 1) / match, radix);
  size_t w = std::max(std::max(w0, status_words_for((cap + big - 1) / big, radix)),
                      status_words_for((small_cap + small - 1) / small, radix));
  // the partition pass (16 buckets)
  const size_t part = PartTile<K, PAIRS>::TILE;
  return std::max(w, status_words_for((cap + part - 1) / part, 16));
}

// Status words per look-back buffer for the sorter's capacity and current options.
size_t needed_status_words(const grs_sorter* s) {
  const size_t cap = std::max<size_t>(s->capacity, 1);
  const size_t radix = std::max<size_t>(size_t(1) << s->radix_bits, 16);
  size_t w;
  if (s->key_type == GRS_KEY_U32)
    w = s->pairs ? max_status_words<uint32_t, true>(s, cap, radix)
                 : max_status_words<uint32_t, false>(s, cap, radix);
  else
    w = s->pairs ? max_status_words<uint64_t, true>(s, cap, radix)
                 : max_status_words<uint64_t, false>(s, cap, radix);
  return msd_type(s) ? std::max(w, MsdLayout::status_words(cap)) : w;
}

// The two look-back status buffers, `words` each, a guard band between them.
grs_status alloc_status(grs_sorter* s, size_t words) {
  const size_t stride = words + kGuardBytes / 4;
  const grs_status r = sbuf_alloc(s, reinterpret_cast<void**>(&s->status), (stride + words) * 4,
                                  "look-back status buffers", {words * 4});
  if (r != GRS_OK) return r;
  s->status_words = words;
  s->status_stride = stride;
  return GRS_OK;
}

// The second buffer: `words` elements per array.  u32 pairs: ONE allocation, keys | guard band |
// payload (the LSD record passes write n 8-byte records from its start, across the band:
// alt_band_dirty); otherwise keys, and the payload in an allocation of its own.
grs_status alloc_alt(grs_sorter* s, size_t words) {
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  grs_status r;
  if (s->pairs && s->key_type == GRS_KEY_U32) {
    r = sbuf_alloc(s, &s->alt_keys, (2 * words) * 4 + kGuardBytes, "second buffer", {words * 4});
    if (r != GRS_OK) return r;
    s->alt_vals = reinterpret_cast<uint32_t*>(static_cast<char*>(s->alt_keys) + words * 4 + kGuardBytes);
    s->alt_joint = true;
    s->alt_inner_band = words * 4;
    s->alt_band_dirty = false;
  } else {
    r = sbuf_alloc(s, &s->alt_keys, words * kb, "second buffer");
    if (r == GRS_OK && s->pairs) r = sbuf_alloc(s, reinterpret_cast<void**>(&s->alt_vals), words * 4, "second buffer");
    if (r != GRS_OK) return r;
  }
  s->alt_words = words;
  return GRS_OK;
}

// The MSD sort's scratch on (alt grown to msd_alt_words(capacity) elements per array, the region
// buffer alt2 and the tables msd_buf) or off (released, alt back to capacity elements).
// Synchronises the device when it changes anything.
grs_status msd_scratch(grs_sorter* s, bool on) {
  const size_t cap = std::max<size_t>(s->capacity, 1);
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  const size_t altw = on ? msd_alt_words(cap) : cap;
  const bool change = (s->msd_buf != nullptr) != on || s->alt_words != altw;
  if (!change) return GRS_OK;
  (void)hipDeviceSynchronize();   // in-flight sorts may still use the buffers replaced here
  if (!on) {
    sbuf_free(s, &s->msd_buf);
    sbuf_free(s, &s->alt2_keys);
    s->alt2_vals = nullptr;
    s->msd_bytes = 0;
    return s->alt_words == cap && s->alt_keys ? GRS_OK : alloc_alt(s, cap);
  }
  grs_status r = alloc_alt(s, altw);
  if (r != GRS_OK) return r;
  const MsdLayout L = MsdLayout::of(cap, msd_digits(s));
  s->msd_bytes = L.words * 4;
  r = sbuf_alloc(s, &s->msd_buf, s->msd_bytes, "MSD tables", L.bands);
  if (r != GRS_OK) return r;
  const size_t w2 = msd_alt2_words(cap);
  r = sbuf_alloc(s, &s->alt2_keys, w2 * kb + kGuardBytes + (s->pairs ? w2 * 4 : 0), "MSD region buffer",
                 {w2 * kb});
  if (r != GRS_OK) return r;
  if (s->pairs) s->alt2_vals = reinterpret_cast<uint32_t*>(static_cast<char*>(s->alt2_keys) + w2 * kb + kGuardBytes);
  return GRS_OK;
}

}  // namespace

extern "C" {

grs_status grs_set_option(grs_sorter* s, grs_option opt, int value) {
  if (!s) return set_err(GRS_EINVAL, "grs_set_option: NULL sorter");
  auto bad = [&]() { return set_err(GRS_EINVAL, "grs_set_option: value out of range for option " +
                                                    std::to_string(static_cast<int>(opt))); };
  switch (opt) {
    case GRS_OPT_TILE:
      if (value < -1 || value > 1) return bad();
      s->tile_mode = value;
      break;
    case GRS_OPT_XL:
      if (value < -1 || value > 1) return bad();
      s->xl_mode = value == -1 ? 0 : value == 1 ? 1 : 2;
      break;
    case GRS_OPT_PASS:
      if (value != 0 && value != 4 && value != 6 && value != 8) return bad();
      s->pass_mode = value;
      break;
    case GRS_OPT_RECORDS:
      if (value < 0 || value > 2) return bad();
      s->rec_mode = value;
      break;
    case GRS_OPT_RANK:
      if (value < 0 || value > 1) return bad();
      s->rank_mode = value == 1 ? 1 : s->probe_rank_mode;
      break;
    case GRS_OPT_SHARDED_PATH:
      if (value < 0 || value > 1) return bad();
      s->sharded_general = value == 1;
      break;
    case GRS_OPT_SHARDED_SEND:
      if (value < 0 || value > 2) return bad();
      s->sharded_send = value;
      break;
    case GRS_OPT_EXCHANGE:
      if (value < 0 || value > 3) return bad();
      s->sharded_exchange = value;
      break;
    case GRS_OPT_X_CHUNKS:
      if (value < 0 || value > 16) return bad();
      s->x_chunks = value;
      break;
    case GRS_OPT_FAULT_TILE: {
      if (value < -1) return bad();
      // the pass's debug words after the error word (grs_pass.hpp PassDebug): fault tile + 1,
      // spin bound
      const uint32_t w[2] = {static_cast<uint32_t>(value + 1), value >= 0 ? (1u << 12) : 0u};
      int prev = 0;
      GRS_HIP(hipGetDevice(&prev));
      GRS_HIP(hipSetDevice(s->device));
      const hipError_t e = hipMemcpy(s->ctrl + GRS_CTRL_ERROR + 1, w, sizeof(w), hipMemcpyHostToDevice);
      (void)hipSetDevice(prev);
      if (e != hipSuccess) return set_err(GRS_EHIP, "grs_set_option: hipMemcpy failed");
      s->fault_tile = value;
      break;
    }
    case GRS_OPT_MERGE:
      if (value < 0 || value > 1) return bad();
      s->merge_mode = value;
      break;
    case GRS_OPT_MSD:
      if (value < -1 || value > 2) return bad();
      s->msd_mode = value;
      break;
    case GRS_OPT_SEG_ROUTE:
      if (value < 0 || value > 2) return bad();
      s->seg_route = value;
      break;
    case GRS_OPT_H2_CHUNK:
      if (value != 0 && (value < 4096 || value > (1 << 20) || (value & (value - 1)) != 0)) return bad();
      s->h2_chunk = static_cast<uint32_t>(value);
      break;
    case GRS_OPT_H2_PIECE:
      if (value != 0 && (value < 64 || value > 4096 || (value & (value - 1)) != 0)) return bad();
      s->h2_piece = static_cast<uint32_t>(value);
      break;
    case GRS_OPT_P3:
      if (value < 0 || value > 2) return bad();
      s->p3_mode = value;
      break;

    default:
      return set_err(GRS_EINVAL, "grs_set_option: unknown option");
  }
  // a pinned tile shape can need more look-back status words than the defaults sized
  const size_t words = needed_status_words(s);
  if (words > s->status_words) {
    int prev = 0;
    GRS_HIP(hipGetDevice(&prev));
    GRS_HIP(hipSetDevice(s->device));
    (void)hipDeviceSynchronize();   // earlier sorts may still use the old buffers
    const grs_status r = alloc_status(s, words);
    (void)hipSetDevice(prev);
    if (r != GRS_OK) return r;
  }
  if (opt == GRS_OPT_MSD) {   // allocate or release the MSD sort's scratch
    int prev = 0;
    GRS_HIP(hipGetDevice(&prev));
    GRS_HIP(hipSetDevice(s->device));
    const grs_status r = msd_scratch(s, value != 0 && msd_type(s) && (value != -1 || s->capacity >= kMsdMinN));
    (void)hipSetDevice(prev);
    if (r != GRS_OK) return r;
  }
  return GRS_OK;
}

grs_status grs_get_option(const grs_sorter* s, grs_option opt, int* value) {
  if (!s || !value) return set_err(GRS_EINVAL, "grs_get_option: NULL argument");
  switch (opt) {
    case GRS_OPT_TILE: *value = s->tile_mode; break;
    case GRS_OPT_XL: *value = s->xl_mode == 0 ? -1 : s->xl_mode == 1 ? 1 : 0; break;
    case GRS_OPT_PASS: *value = s->pass_mode; break;
    case GRS_OPT_RECORDS: *value = s->rec_mode; break;
    case GRS_OPT_RANK: *value = s->rank_mode; break;
    case GRS_OPT_SHARDED_PATH: *value = s->sharded_general ? 1 : 0; break;
    case GRS_OPT_SHARDED_SEND: *value = s->sharded_send; break;
    case GRS_OPT_EXCHANGE: *value = s->sharded_exchange; break;
    case GRS_OPT_X_CHUNKS: *value = s->x_chunks; break;
    case GRS_OPT_MERGE: *value = s->merge_mode; break;
    case GRS_OPT_FAULT_TILE: *value = s->fault_tile; break;
    case GRS_OPT_MSD: *value = s->msd_mode; break;
    case GRS_OPT_SEG_ROUTE: *value = s->seg_route; break;
    case GRS_OPT_H2_CHUNK: *value = static_cast<int>(s->h2_chunk); break;
    case GRS_OPT_H2_PIECE: *value = static_cast<int>(s->h2_piece); break;
    case GRS_OPT_P3: *value = s->p3_mode; break;
    default: return set_err(GRS_EINVAL, "grs_get_option: unknown option");
  }
  return GRS_OK;
}

grs_status grs_create(grs_sorter** out, size_t capacity, grs_key_type key_type,
                      int with_u32_payload, int radix_bits, int device) {
  if (!out) return set_err(GRS_EINVAL, "grs_create: out is NULL");
  *out = nullptr;
  if (key_type != GRS_KEY_U32 && key_type != GRS_KEY_U64)
    return set_err(GRS_EINVAL, "grs_create: bad key type");
  if (radix_bits == 0) radix_bits = 8;
  if (radix_bits != 4 && radix_bits != 8)
    return set_err(GRS_EINVAL, "grs_create: radix_bits must be 4, 8 or 0");
  if (capacity > GRS_MAX_N)
    return set_err(GRS_ECAPACITY, "grs_create: capacity exceeds GRS_MAX_N (2^32 - 2^16) items per device call");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_err(GRS_ENODEV, "grs_create: no HIP device");
  if (device < 0 || device >= ndev) return set_err(GRS_ENODEV, "grs_create: bad device ordinal");

  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  GRS_HIP(hipSetDevice(device));
  grs_sorter* s = new grs_sorter();
  s->device = device;
  s->key_type = key_type;
  s->pairs = with_u32_payload ? 1 : 0;
  s->radix_bits = radix_bits;
  s->capacity = capacity;
  s->rank_mode = s->probe_rank_mode = device_rank_mode(device);
  (void)hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, device);
  const size_t kb = key_type == GRS_KEY_U64 ? 8 : 4;
  const size_t cap = std::max<size_t>(capacity, 1);
  (void)kb;
  grs_status st = alloc_status(s, needed_status_words(s));
  if (st == GRS_OK) st = sbuf_alloc(s, reinterpret_cast<void**>(&s->ctrl), GRS_CTRL_WORDS * 4, "grs_create: control block");
  if (st == GRS_OK) st = sbuf_alloc(s, reinterpret_cast<void**>(&s->ctrl2), GRS_CTRL_ERROR * 4, "grs_create: control block");
  if (st == GRS_OK && (hipMemset(s->ctrl, 0, GRS_CTRL_WORDS * 4) != hipSuccess ||
                       hipMemset(s->ctrl2, 0, GRS_CTRL_ERROR * 4) != hipSuccess))
    st = set_err(GRS_EHIP, "grs_create: hipMemset failed");
  // the second buffer and, from kMsdMinN items of capacity (where the MSD sort is the default),
  // the MSD sort's scratch; if that does not fit, the sorter runs the LSD passes (no MSD
  // scratch: 1 n of elements instead of ~2.4 n)
  if (st == GRS_OK) {
    if (msd_type(s) && cap >= kMsdMinN && msd_scratch(s, true) != GRS_OK) (void)msd_scratch(s, false);
    if (!s->alt_keys) st = alloc_alt(s, cap);
  }
  if (st == GRS_OK && hipHostMalloc(reinterpret_cast<void**>(&s->h_err), 4, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    st = set_err(GRS_ENOMEM, "grs_create: hipHostMalloc failed");
  }
  (void)hipSetDevice(prev);
  if (st != GRS_OK) {
    grs_destroy(s);
    return st;
  }
  *out = s;
  return GRS_OK;
}

size_t grs_scratch_bytes(const grs_sorter* s) { return s ? s->scratch_bytes : 0; }

grs_status grs_debug_check_guards(grs_sorter* s, uint64_t* bad_words) {
  if (!s || !bad_words) return set_err(GRS_EINVAL, "grs_debug_check_guards: NULL argument");
  *bad_words = 0;
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  GRS_HIP(hipSetDevice(s->device));
  grs_status r = GRS_OK;
  if (hipDeviceSynchronize() != hipSuccess) r = set_err(GRS_EHIP, "grs_debug_check_guards: synchronise");
  std::vector<uint32_t> h(kGuardBytes / 4);
  uint64_t bad = 0;
  for (const grs_sorter::ScratchBuf& b : s->bufs) {
    if (r != GRS_OK || !*b.owner) continue;
    for (size_t o : b.bands) {
      char* at = static_cast<char*>(*b.owner) + o;
      // alt's inner band after an LSD record sort holds records, legitimately: restored, not counted
      const bool records = b.owner == &s->alt_keys && o == s->alt_inner_band && s->alt_band_dirty;
      if (hipMemcpy(h.data(), at, kGuardBytes, hipMemcpyDeviceToHost) != hipSuccess) {
        r = set_err(GRS_EHIP, "grs_debug_check_guards: read-back");
        break;
      }
      uint64_t c = 0;
      for (uint32_t w : h) c += w != kGuardWord;
      if (!records) bad += c;
      if (c != 0 && fill_band(at) != hipSuccess) r = set_err(GRS_EHIP, "grs_debug_check_guards: restore");
    }
  }
  if (r == GRS_OK) s->alt_band_dirty = false;
  *bad_words = bad;
  (void)hipSetDevice(prev);
  return r;
}

grs_status grs_debug_msd_flags(grs_sorter* s, uint32_t* flags) {
  if (!s || !flags) return set_err(GRS_EINVAL, "grs_debug_msd_flags: NULL argument");
  if (s->last_msd_cb < 0) return set_err(GRS_EINVAL, "grs_debug_msd_flags: the last sort did not run the MSD schedule");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  GRS_HIP(hipSetDevice(s->device));
  grs_status r = GRS_OK;
  const uint32_t* hist = s->last_msd_cb == 0 ? s->ctrl : s->ctrl2;
  uint32_t w[3] = {};
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&w[0], hist + 512 + 256, 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&w[1], s->last_msd_spill2, 4, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&w[2], hist + GRS_MSD_SPAN + 4, 4, hipMemcpyDeviceToHost) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_debug_msd_flags: read-back");
  flags[0] = w[0] != 0u;
  flags[1] = w[1] != 0u;
  flags[2] = w[2];
  (void)hipSetDevice(prev);
  return r;
}

int grs_rank_mode(const grs_sorter* s) { return s ? s->rank_mode : -1; }

grs_status grs_set_profiling(grs_sorter* s, int ring) {
  if (!s) return set_err(GRS_EINVAL, "grs_set_profiling: NULL sorter");
  if (ring < 0 || ring > 4096) return set_err(GRS_EINVAL, "grs_set_profiling: ring out of range");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  GRS_HIP(hipSetDevice(s->device));
  for (int i = 0; s->ev && i < s->ring * grs_sorter::EV_PER_CALL; ++i)
    if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
  delete[] s->ev;
  delete[] s->info;
  s->ev = nullptr;
  s->info = nullptr;
  s->ring = 0;
  s->calls = 0;
  grs_status st = GRS_OK;
  if (ring > 0) {
    s->ev = new hipEvent_t[ring * grs_sorter::EV_PER_CALL]();
    s->info = new grs_sorter::CallInfo[ring]();
    s->ring = ring;
    for (int i = 0; i < ring * grs_sorter::EV_PER_CALL && st == GRS_OK; ++i)
      if (hipEventCreate(&s->ev[i]) != hipSuccess)
        st = set_err(GRS_EHIP, "grs_set_profiling: hipEventCreate failed");
    for (hipEvent_t& e : s->xev)
      if (st == GRS_OK && !e && hipEventCreate(&e) != hipSuccess)
        st = set_err(GRS_EHIP, "grs_set_profiling: hipEventCreate failed");
  }
  s->xev_recorded = false;
  (void)hipSetDevice(prev);
  return st;
}

}  // extern "C"

namespace {

// One pass launch (grs_pass.hpp): grs_onesweep_v4, grid = tiles, one tile per workgroup; or
// PERSIST: grs_onesweep_v6, grid = resident workgroups looping over tickets with prefetch.
template <typename K, bool PAIRS, int RB, typename Tile, uint32_t OPT, bool PERSIST = false,
          typename DigitF>
grs_status launch_pass(grs_sorter* s, const K* src, K* dst, const uint32_t* vsrc, uint32_t* vdst,
                       uint32_t n, const DigitF& dig, const DigitF* dig_dev, const uint32_t* hist,
                       uint32_t* ticket, uint32_t* st_cur, uint32_t* st_nxt, hipStream_t stream,
                       uint32_t expect_tile = 0, const uint32_t* plan = nullptr) {
  const uint32_t tiles = (n + Tile::TILE - 1) / Tile::TILE;
  if (status_words_for(tiles, 1u << RB) > s->status_words)
    return set_err(GRS_ECAPACITY, "status buffer too small (pass: " + std::to_string(tiles) + " tiles, have " +
                                      std::to_string(s->status_words) + " words)");
  if (expect_tile != 0 && expect_tile != static_cast<uint32_t>(Tile::TILE))
    return set_err(GRS_EINVAL, "internal: pass tile differs from the zeroed status layout");
  if constexpr (PERSIST) {
    const uint32_t grid = std::min<uint32_t>(tiles, static_cast<uint32_t>(s->cus * Tile::MINW));
    hipLaunchKernelGGL((grs::grs_onesweep_v6<K, PAIRS, RB, Tile::BLOCK, Tile::ITEMS, Tile::MINW,
                                             OPT, DigitF>),
                       dim3(grid), dim3(Tile::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig, hist,
                       ticket, st_cur, st_nxt, s->ctrl + GRS_CTRL_ERROR, dig_dev, plan);
  } else {
    hipLaunchKernelGGL((grs::grs_onesweep_v4<K, PAIRS, RB, Tile::BLOCK, Tile::ITEMS, Tile::MINW,
                                             OPT, DigitF>),
                       dim3(tiles), dim3(Tile::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig, hist,
                       ticket, st_cur, st_nxt, s->ctrl + GRS_CTRL_ERROR, dig_dev, plan);
  }
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

// One pass with the record flags of kind (run_sort's rec_kind): 0 two arrays, 1 write
// records, 2 read records, 3 read split records + write records, 4 read records + write split.
template <typename K, bool PAIRS, int RB, typename Tile, uint32_t OPT, bool PERSIST>
grs_status launch_rec(int kind, grs_sorter* s, const K* src, K* dst, const uint32_t* vsrc,
                      uint32_t* vdst, uint32_t n, const grs::RadixDigit<K>& dig,
                      const uint32_t* hist, uint32_t* ticket, uint32_t* st_cur, uint32_t* st_nxt,
                      hipStream_t stream, uint32_t expect_tile, const uint32_t* plan = nullptr) {
  using Dig = grs::RadixDigit<K>;
  constexpr bool R = sizeof(K) == 4 && PAIRS && RB == 8;
  constexpr uint32_t W = R ? 8192u : 0u, Rd = R ? 4096u : 0u, RS = R ? 16384u : 0u, WS = R ? 32768u : 0u;
  switch (R ? kind : 0) {
    case 1: return launch_pass<K, PAIRS, RB, Tile, OPT | W, PERSIST>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, hist, ticket, st_cur, st_nxt, stream, expect_tile);
    case 2: return launch_pass<K, PAIRS, RB, Tile, OPT | Rd, PERSIST>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, hist, ticket, st_cur, st_nxt, stream, expect_tile);
    case 3: return launch_pass<K, PAIRS, RB, Tile, OPT | Rd | RS | W, PERSIST>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, hist, ticket, st_cur, st_nxt, stream, expect_tile);
    case 4: return launch_pass<K, PAIRS, RB, Tile, OPT | Rd | W | WS, PERSIST>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, hist, ticket, st_cur, st_nxt, stream, expect_tile);
    default: return launch_pass<K, PAIRS, RB, Tile, OPT, PERSIST>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, hist, ticket, st_cur, st_nxt, stream, expect_tile, plan);
  }
}

// src_in (out-of-place, the presorted exchange): pass 0 reads src_in / vsrc_in instead of
// keys / vals, and the passes alternate so that the last one writes keys / vals (no copy-back).
template <typename K, bool PAIRS, int RB>
grs_status run_sort(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, int begin_bit,
                    int end_bit, hipStream_t stream, const K* src_in = nullptr,
                    const uint32_t* vsrc_in = nullptr) {
  using Big = std::conditional_t<RB == 8, BigTile<K, PAIRS>, BigTile4<K, PAIRS>>;
  using Small = SmallTile<K, PAIRS>;
  constexpr uint32_t kBig = RB == 8 ? BigTile<K, PAIRS>::OPT : kBig4Opt;
  constexpr int RADIX = 1 << RB;
  const bool big = use_big_tiles(s, n, Big::TILE);
  const int passes = (end_bit - begin_bit + RB - 1) / RB;
  // the tile size the passes below launch with: it sets the status layout (tile words, then
  // group words) that the histogram kernel zeroes for pass 0 and every pass for the next one
  uint32_t tile = big ? Big::TILE : Small::TILE;
  if (s->rank_mode != 0 && big) tile = MatchTile<K, PAIRS>::TILE;
  using XL = XLTile<K, PAIRS>;
  constexpr bool kXlType = RB == 8 && !(sizeof(K) == 8 && PAIRS);   // u64 pairs: BigTile is already two-round
  const bool xl = kXlType && big && use_xl(s, n, XL::TILE);
  if (xl) tile = XL::TILE;
  const uint32_t tiles = (n + tile - 1) / tile;
  // the persistent pass prefetches into the registers a two-round reorder still needs
  const bool persist = !xl && !Big::TWO_ROUNDS && use_persistent(s, tiles, RB);
  const size_t words = status_words_for(tiles, RADIX);
  if (words > s->status_words)
    return set_err(GRS_ECAPACITY, "status buffer too small (LSD: n " + std::to_string(n) + ", " +
                                      std::to_string(words) + " words, have " + std::to_string(s->status_words) + ")");
  uint32_t* st0 = s->status;
  uint32_t* st1 = s->status + s->status_stride;
  uint32_t* const cb[2] = {s->ctrl, s->ctrl2};
  uint32_t* hist = cb[s->cb_i];
  uint32_t* tickets = hist + GRS_CTRL_TICKETS;
  uint32_t* hist_next = cb[s->cb_i ^ 1];   // zeroed by this call's histogram kernel
  int ev = 0;
  hipEvent_t* evs = s->ring ? s->ev + (s->calls % s->ring) * grs_sorter::EV_PER_CALL : nullptr;
  auto mark = [&]() -> grs_status {
    if (evs) GRS_HIP(hipEventRecord(evs[ev++], stream));
    return GRS_OK;
  };

  grs_status r;
  if ((r = mark()) != GRS_OK) return r;
  // histograms + tickets are zero (the previous call's histogram kernel cleared them) unless
  // the partition pass used the block since (the error word is sticky: only the checks clear it)
  if (s->cb_dirty && s->cb_i == 0) GRS_HIP(hipMemsetAsync(hist, 0, GRS_CTRL_ERROR * 4, stream));
  s->cb_dirty = false;
  {
    // grs_upfront_hist2: 2 blocks of 512 per CU (u64 keys: 1 of 1024); a multiple of the
    // resident slots so the grid-stride loop ends evenly, and > n >> kHist2GridShift blocks
    // (16-bit counters)
    const int slots = grs::Hist2Layout<K>::PER_CU * s->cus;
    const int need = static_cast<int>(n >> grs::kHist2GridShift<K>) + 1;
    // (one block per CU up to 2^25 keys: two measured slower at C2, 24.8 vs 21.5 us)
    int grid = n <= (1u << 25) ? s->cus : slots;
    if (grid < need) grid = (need + slots - 1) / slots * slots;
    const bool full = begin_bit == 0 && end_bit == static_cast<int>(8 * sizeof(K));
    auto kern = full ? grs::grs_upfront_hist2<K, RB, true> : grs::grs_upfront_hist2<K, RB, false>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(grs::Hist2Layout<K>::BLOCK), 0, stream,
                       src_in ? src_in : keys, n, begin_bit, end_bit, passes, hist, st0,
                       static_cast<uint32_t>(words), hist_next, (uint32_t*)nullptr, 0u);
    GRS_HIP(hipGetLastError());
  }
  s->cb_i ^= 1;   // the next call's block (zero once this call's histogram kernel has run)
  if ((r = mark()) != GRS_OK) return r;

  K* src = keys;
  K* dst = static_cast<K*>(s->alt_keys);
  uint32_t* vsrc = vals;
  uint32_t* vdst = s->alt_vals;
  if (src_in) {   // out of place: the last pass writes keys
    src = const_cast<K*>(src_in);
    vsrc = const_cast<uint32_t*>(vsrc_in);
    if ((passes & 1) != 0) {
      dst = keys;
      vdst = vals;
    }
  }
  // u32 pairs on big / XL tiles, 8-bit digits, even pass count, in place: the passes that write
  // the scratch write it as 8-byte (key, value) records and the next pass reads them back
  // (longer digit runs; the caller's buffers stay two arrays)
  constexpr bool kRecType = sizeof(K) == 4 && PAIRS && RB == 8;
  const bool rec = kRecType && big && !src_in && (passes & 1) == 0 && s->alt_joint &&
                   s->rec_mode != 0 && s->rank_mode == 0;
  if (rec) s->alt_band_dirty = true;   // records run across alt's inner guard band
  // even n, 4+ passes: the middle passes also write records, split over the caller's two
  // arrays (records [0, n/2) in keys, [n/2, n) in vals), so every pass but the last writes
  // records.  Pass p's record flags: 0 = none, 1 = write, 2 = read, 3 = read split + write,
  // 4 = read + write split
  // (not on the persistent pass: at 2^24 pairs it measured slower there)
  // The split records are 8-byte loads and stores on the caller's arrays: both must be 8-byte
  // aligned (a torch view at an odd storage offset, or an offset C pointer, is only 4-byte
  // aligned); otherwise the middle passes keep two arrays.
  const bool caller_aligned =
      ((reinterpret_cast<uintptr_t>(keys) | reinterpret_cast<uintptr_t>(vals)) & 7u) == 0;
  const bool rec_split = rec && (n & 1u) == 0 && passes >= 4 && s->rec_mode == 2 && !persist &&
                         caller_aligned;
  auto rec_kind = [&](int p) -> int {
    if (!rec) return 0;
    if ((p & 1) == 0) return p > 0 && rec_split ? 3 : 1;
    return p < passes - 1 && rec_split ? 4 : 2;
  };
  using Dig = grs::RadixDigit<K>;
  // every pass in one launch (grs_onesweep_fused, GRS_OPT_PASS = 8): the persistent big-tile
  // pass, full-width digits, in place.  Not the default: its grid barrier costs more than a
  // kernel boundary (C2 0.47 vs 0.29 ms a sort, tools/barrier_probe.py)
  const bool fused = persist && big && !rec && !src_in && s->rank_mode == 0 && (end_bit - begin_bit) % RB == 0 &&
                     s->pass_mode == 8;
  if constexpr (!Big::TWO_ROUNDS) {
    if (fused) {
      auto kern = grs::grs_onesweep_fused<K, PAIRS, RB, Big::BLOCK, Big::ITEMS, Big::MINW, kBig>;
      static const int per_cu = [&] {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, Big::BLOCK, 0) != hipSuccess) b = 0;
        return b;
      }();
      if (per_cu < 1) return set_err(GRS_EHIP, "internal: fused pass kernel does not fit a CU");
      const uint32_t grid = std::min<uint32_t>(tiles, static_cast<uint32_t>(per_cu * std::max(1, s->cus)));
      K* const alt = static_cast<K*>(s->alt_keys);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(Big::BLOCK), 0, stream, keys, alt, vals, s->alt_vals, n, begin_bit,
                         passes, hist, tickets, tickets + 1, st0, st1, s->ctrl + GRS_CTRL_ERROR);
      GRS_HIP(hipGetLastError());
      if ((r = mark()) != GRS_OK) return r;
      if ((passes & 1) != 0) {   // odd: the result sits in the scratch
        GRS_HIP(hipMemcpyAsync(keys, alt, static_cast<size_t>(n) * sizeof(K), hipMemcpyDeviceToDevice, stream));
        if (PAIRS) GRS_HIP(hipMemcpyAsync(vals, s->alt_vals, static_cast<size_t>(n) * 4, hipMemcpyDeviceToDevice, stream));
        if ((r = mark()) != GRS_OK) return r;
      }
      if (evs) {
        s->info[s->calls % s->ring] = {ev, 1, (passes & 1) != 0, 2};
        ++s->calls;
      }
      return GRS_OK;
    }
  }
  // the pass plan (grs_pass_plan): passes whose digit is the same for every key are skipped or
  // become one copy (record passes and out-of-place sorts keep every pass)
  const uint32_t* plan = nullptr;
  if (!rec && !src_in && passes >= 2) {
    uint32_t* const pw = s->ctrl + GRS_CTRL_PLAN;
    hipLaunchKernelGGL(grs::grs_pass_plan, dim3(1), dim3(64), 0, stream, hist, static_cast<uint32_t>(RADIX), passes, n, pw);
    GRS_HIP(hipGetLastError());
    plan = pw;
  }
  for (int p = 0; p < passes; ++p) {
    const int shift = begin_bit + p * RB;
    const int bits = std::min(RB, end_bit - shift);
    uint32_t* st_cur = (p & 1) ? st1 : st0;
    const uint32_t* pp = plan ? plan + p : nullptr;
    uint32_t* st_nxt = (p & 1) ? st0 : st1;
    const Dig dig{shift, (1u << bits) - 1u};
    const uint32_t* ph = hist + p * GRS_HIST_PASS_STRIDE;
    uint32_t* tk = tickets + p * GRS_XCDS;
    if (s->rank_mode != 0) {
      r = big ? launch_pass<K, PAIRS, RB, MatchTile<K, PAIRS>, kMatchOpt>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, ph, tk, st_cur, st_nxt, stream, tile, pp)
              : launch_pass<K, PAIRS, RB, Small, kMatchOpt>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, ph, tk, st_cur, st_nxt, stream, tile, pp);
    } else if (xl) {
      if constexpr (kXlType)
        r = launch_rec<K, PAIRS, RB, XL, XL::OPT, false>(rec_kind(p), s, src, dst, vsrc, vdst, n, dig, ph, tk, st_cur, st_nxt, stream, tile, pp);
    } else if (persist && big) {
      if constexpr (!Big::TWO_ROUNDS)
        r = launch_rec<K, PAIRS, RB, Big, kBig, true>(rec_kind(p), s, src, dst, vsrc, vdst, n, dig, ph, tk, st_cur, st_nxt, stream, tile, pp);
    } else if (big && rec) {
      r = launch_rec<K, PAIRS, RB, Big, kBig, false>(rec_kind(p), s, src, dst, vsrc, vdst, n, dig, ph, tk, st_cur, st_nxt, stream, tile);
    } else {
      r = big ? launch_pass<K, PAIRS, RB, Big, kBig>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, ph, tk, st_cur, st_nxt, stream, tile, pp)
              : launch_pass<K, PAIRS, RB, Small, kSmallOpt>(s, src, dst, vsrc, vdst, n, dig, (const Dig*)nullptr, ph, tk, st_cur, st_nxt, stream, tile, pp);
    }
    if (r != GRS_OK) return r;
    if ((r = mark()) != GRS_OK) return r;
    if (src_in && p == 0) {   // pass 1 on: ping-pong between keys and the sorter's scratch
      src = dst;
      vsrc = vdst;
      dst = src == keys ? static_cast<K*>(s->alt_keys) : keys;
      vdst = src == keys ? s->alt_vals : vals;
      continue;
    }
    std::swap(src, dst);
    std::swap(vsrc, vdst);
  }
  const bool copy = !src_in && (passes & 1) != 0;
  if (copy) {  // result sits in scratch: copy back (ParallelSort.cpp:312-318)
    GRS_HIP(hipMemcpyAsync(keys, src, static_cast<size_t>(n) * sizeof(K), hipMemcpyDeviceToDevice,
                           stream));
    if (PAIRS)
      GRS_HIP(hipMemcpyAsync(vals, vsrc, static_cast<size_t>(n) * 4, hipMemcpyDeviceToDevice,
                             stream));
    if ((r = mark()) != GRS_OK) return r;
  }
  if (evs) {
    s->info[s->calls % s->ring] = {ev, passes, copy, 0};
    ++s->calls;
  }
  return GRS_OK;
}

// ---- MSD-first sort (grs_msd.hpp) ----
// The P3 shape for n elements of E bytes: a uniform 16-bit segment holds m = n / 65536, +-
// sqrt(m); the shape must take m + 8 sqrt(m) + 64 (longer segments take the segmented
// fallback).  0: none fits (the LSD sort).
double msd_segment_need(size_t n) {
  const double m = static_cast<double>(n) / 65536.0;
  return m + 8.0 * std::sqrt(m) + 64.0;
}

int msd_local_shape(size_t n, size_t elem) {
  const double need = msd_segment_need(n);
  if (need <= MsdLocalS::SMAX) return 4;
  if (need <= MsdLocalM::SMAX) return 5;
  if (need <= MsdLocalA::SMAX) return 1;
  if (need <= MsdLocalB::SMAX) return 2;
  if (elem == 4 && need <= MsdLocalC2::SMAX) return 7;
  if (elem == 4 && need <= MsdLocalC::SMAX) return 3;
  if (elem == 4 && need <= MsdLocalD::SMAX) return 6;
  return 0;
}

bool use_msd(const grs_sorter* s, size_t n, int begin_bit, int end_bit) {
  if (!msd_type(s) || s->msd_mode == 0 || s->msd_buf == nullptr || s->rank_mode != 0) return false;
  const int kbits = s->key_type == GRS_KEY_U64 ? 64 : 32;
  const size_t elem = kbits / 8 + (s->pairs ? 4 : 0);
  if (begin_bit != 0 || end_bit != kbits || msd_local_shape(n, elem) == 0) return false;
  return s->msd_mode >= 1 || n >= kMsdMinN;
}

// sample -> P1 (regions) -> [redo] -> P2's plan -> H2 -> P2 -> P3 -> fallback (plan,
// histograms, a segmented LSD over the bits below the prefix for the segments P3 left;
// persistent grids that leave at once when there are none).  src_in / vsrc_in (out of place):
// the sample and P1 read them; the result lands in keys / vals either way.  u32 pairs move as
// two arrays throughout: 8-byte (key, value) records between the passes measured no faster
// (DESIGN.md §6.R5).
template <typename K, bool PAIRS, typename P3C>
grs_status run_msd(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, hipStream_t stream,
                   const K* src_in, const uint32_t* vsrc_in) {
  using Big = BigTile<K, PAIRS>;
  using XL = XLTile<K, PAIRS>;
  using Small = SmallTile<K, PAIRS>;
  using FT = BigTile<K, PAIRS>;   // the redo's and the fallback's persistent passes
  using Dig = grs::RadixDigit<K>;
  constexpr int KB = 8 * static_cast<int>(sizeof(K));
  constexpr int ND = (KB - 16) / 8;
  static_assert(!Big::TWO_ROUNDS, "u64 pairs take the LSD sort");
  constexpr uint32_t G = GRS_LB_GROUP;
  const bool big = use_big_tiles(s, n, Big::TILE);
  const bool xl = big && use_xl(s, n, XL::TILE);
  const uint32_t tile1 = xl ? XL::TILE : big ? Big::TILE : Small::TILE;
  const size_t words1 = status_words_for((n + tile1 - 1) / tile1, 256);
  const uint32_t tile2 = xl ? XL::TILE : Big::TILE;
  const size_t t2 = n / tile2 + 257;
  const size_t words2 = (t2 + 2 * (t2 / G + 257)) * 256;
  if (words1 > s->status_words || words2 > s->status_words)
    return set_err(GRS_ECAPACITY, "status buffer too small (MSD: n " + std::to_string(n) + ", P1 " +
                                      std::to_string(words1) + " / P2 " + std::to_string(words2) + " words, have " +
                                      std::to_string(s->status_words) + ")");
  const MsdLayout L = MsdLayout::of(s->capacity, ND);
  if (t2 > L.r2) return set_err(GRS_ECAPACITY, "internal: MSD plan capacity");
  uint32_t* const mb = static_cast<uint32_t*>(s->msd_buf);
  uint32_t* const h2 = mb + L.h2;
  uint32_t* const bigc = mb + L.big;
  uint32_t* const dstart = mb + L.dstart;
  uint32_t* const hdr2 = mb + L.hdr2;
  auto* const rec2 = reinterpret_cast<grs::SegTile*>(mb + L.rec2);
  uint32_t* const hdrf = mb + L.hdrf;
  auto* const recf = reinterpret_cast<grs::SegTile*>(mb + L.recf);
  uint32_t* const rows = mb + L.rows;
  uint32_t* const st[2] = {s->status, s->status + s->status_stride};
  uint32_t* const err = s->ctrl + GRS_CTRL_ERROR;
  uint32_t* const cb[2] = {s->ctrl, s->ctrl2};
  uint32_t* const hist = cb[s->cb_i];
  uint32_t* const tickets = hist + GRS_CTRL_TICKETS;
  uint32_t* const hist_next = cb[s->cb_i ^ 1];
  const K* src = src_in ? src_in : keys;
  const uint32_t* vsrc = src_in ? vsrc_in : vals;
  K* const alt = static_cast<K*>(s->alt_keys);
  uint32_t* const valt = PAIRS ? s->alt_vals : nullptr;
  int ev = 0;
  hipEvent_t* evs = s->ring ? s->ev + (s->calls % s->ring) * grs_sorter::EV_PER_CALL : nullptr;
  auto mark = [&]() -> grs_status {
    if (evs) GRS_HIP(hipEventRecord(evs[ev++], stream));
    return GRS_OK;
  };
  // rows of this call's control block (zeroed by the previous call): the sample's top-byte
  // counts, the redo's exact counts, P1's digit totals + spill flag
  uint32_t* const samp = hist;
  uint32_t* const exact = hist + 256;
  uint32_t* const totals = hist + 512;
  // the keys' span and the top digit's shift (grs_msd.hpp GRS_MSD_SPAN): every digit below reads
  // its shift from span[4] (P1 and its redo: the top digit; H2, P2 and its redo: the byte below
  // it; P3: the rounds below the 16-bit prefix)
  uint32_t* const span = hist + GRS_MSD_SPAN;
  const uint32_t* const top = span + 4;
  // P1's regions: R_d = sample_d * n * 9/8 / sampled + pad (the sample reads every key up to
  // 2^20 keys: exact counts, no pad needed)
  const uint64_t sampled = std::min<uint64_t>(n, uint64_t(GRS_MSD_SAMPLE_CHUNKS) * GRS_WAVE);
  const unsigned long long mult =
      static_cast<unsigned long long>((static_cast<uint64_t>(n) * 9 * (uint64_t(1) << 20) + 8 * sampled - 1) /
                                      (8 * sampled));
  const uint32_t pad = n > sampled ? 4096u : 0u;
  const uint64_t region_len = static_cast<uint64_t>(n) + n / 8 + 256u * pad + 256u;
  if (region_len > msd_alt_words(s->capacity)) return set_err(GRS_ECAPACITY, "internal: MSD regions");
  grs_status r;
#ifdef GRS_DIAG
  // diagnostic builds (tools/diag): the passes' bounds checks, reported per phase on stderr
  auto diag_set = [&](uint64_t out_lim, uint64_t in_lim) -> grs_status {
    const uint32_t lim[4] = {static_cast<uint32_t>(std::min<uint64_t>(out_lim, 0xFFFFFFFFu)),
                             static_cast<uint32_t>(std::min<uint64_t>(in_lim, 0xFFFFFFFFu)),
                             static_cast<uint32_t>(std::min<size_t>(s->status_words, 0xFFFFFFFFu)), 0u};
    GRS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(grs::diag_lim), lim, sizeof(lim), 0, hipMemcpyHostToDevice, stream));
    return GRS_OK;
  };
  auto diag_check = [&](const char* what) -> grs_status {
    GRS_HIP(hipStreamSynchronize(stream));
    uint32_t hit[24];
    GRS_HIP(hipMemcpyFromSymbol(hit, HIP_SYMBOL(grs::diag_hit), sizeof(hit)));
    if (hit[8] != 0u)
      fprintf(stderr, "diag %-12s first run past the bound: tile %u digit %u start %u gstart %u prefix %u seg_start %u "
              "seg_len %u publish %u gh %u base %u valid %u lstart %u\n", what, hit[9], hit[10], hit[11], hit[12],
              hit[13], hit[14], hit[15], hit[16], hit[17], hit[18], hit[19], hit[20]);
    uint32_t host_err[4] = {};
    GRS_HIP(hipMemcpy(host_err, err, sizeof(host_err), hipMemcpyDeviceToHost));
    fprintf(stderr, "diag %-12s bad stores %u (max %u)  bad loads %u (max %u)  status %u (tile row %u)  error word %u\n",
            what, hit[0], hit[1], hit[2], hit[3], hit[4], hit[5], host_err[0]);
    const uint32_t zero[24] = {};
    GRS_HIP(hipMemcpyToSymbol(HIP_SYMBOL(grs::diag_hit), zero, sizeof(zero)));
    const char* stop = getenv("GRS_DIAG_STOP");
    if (stop != nullptr && strcmp(stop, what) == 0) return set_err(GRS_EINVAL, std::string("diag stop after ") + what);
    return GRS_OK;
  };
#define GRS_DIAG_SET(o, i) if ((r = diag_set(o, i)) != GRS_OK) return r
#define GRS_DIAG_CHECK(w) if ((r = diag_check(w)) != GRS_OK) return r
#else
#define GRS_DIAG_SET(o, i)
#define GRS_DIAG_CHECK(w)
#endif
  if ((r = mark()) != GRS_OK) return r;
  s->last_msd_cb = s->cb_i;
  s->last_msd_spill2 = mb + L.spill2;
  if (s->cb_dirty && s->cb_i == 0) GRS_HIP(hipMemsetAsync(hist, 0, GRS_CTRL_ERROR * 4, stream));
  s->cb_dirty = false;
  if (s->alt_band_dirty) {   // an LSD record sort wrote across alt's inner guard band: restore it
    GRS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(static_cast<char*>(s->alt_keys) + s->alt_inner_band),
                              static_cast<int>(kGuardWord), kGuardBytes / 4, stream));
    s->alt_band_dirty = false;
  }
  // sample: the top byte's histogram; zeroes P1's status, the next call's control block, h2
  // and the big-segment counters
  hipLaunchKernelGGL((grs::grs_msd_sample<K>), dim3(std::max(1, s->cus)), dim3(256), 0, stream, src, n, samp, st[0],
                     static_cast<uint32_t>(words1), hist_next, h2, static_cast<uint32_t>(L.clear), span);
  GRS_HIP(hipGetLastError());
  s->cb_i ^= 1;
  if ((r = mark()) != GRS_OK) return r;
  // P1: stable scatter by the top digit (the sample's guess of it) into the sampled regions,
  // src -> alt (no counting read); its tiles OR the keys into span[0..3]
  const Dig d1{0, 255u};   // (+ *top)
  GRS_DIAG_SET(region_len, n);
  {
    const uint32_t tiles = (n + tile1 - 1) / tile1;
    auto go = [&](auto tshape, auto optc) {
      using T = decltype(tshape);
      constexpr uint32_t opt = decltype(optc)::value;
      hipLaunchKernelGGL((grs::grs_onesweep_region<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, opt>),
                         dim3(tiles), dim3(T::BLOCK), 0, stream, src, alt, vsrc, valt, n, d1, samp, mult,
                         pad, static_cast<uint32_t>(region_len), tickets, st[0], st[1], err, totals, span);
    };
    if (xl) go(XL{}, std::integral_constant<uint32_t, XL::OPT>{});
    else if (big) go(Big{}, std::integral_constant<uint32_t, Big::OPT>{});
    else go(Small{}, std::integral_constant<uint32_t, kSmallOpt>{});
    GRS_HIP(hipGetLastError());
  }
  if ((r = mark()) != GRS_OK) return r;
  // the exact span checks the guessed top digit; a run that outgrew its region or a varying bit
  // above the guess: P1 again into the exact layout at the exact digit (grs_msd_span plans it:
  // exact counts, persistent scatter); otherwise the two launches leave at once
  hipLaunchKernelGGL((grs::grs_msd_span<K, FT::TILE>), dim3(1), dim3(256), 0, stream, n, span, totals, recf, hdrf);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_seg_hist<K, 1>), dim3(2 * s->cus), dim3(256), 0, stream, src, recf, hdrf,
                     0, exact, st[0], 256u, top);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, FT::BLOCK, FT::ITEMS, FT::MINW, FT::OPT, true>),
                     dim3(s->cus), dim3(FT::BLOCK), 0, stream, src, alt, vsrc, valt, d1, recf, hdrf,
                     exact, 256u, tickets + 15 * GRS_XCDS, st[0], st[1], err, nullptr, nullptr, nullptr,
                     nullptr, top);
  GRS_HIP(hipGetLastError());
  GRS_DIAG_CHECK("P1");
  if ((r = mark()) != GRS_OK) return r;
  // P2's plans (the bucket table: P1's regions, or the redo's exact layout): the exact one for
  // the rare redo below, then H2 over a 1/2^k sample of P1's output and the region plan from it
  // (grs_msd_plan3); zeroes P2's status
  uint32_t* const tab = mb + L.tab;
  uint32_t* const spill2 = mb + L.spill2;
  uint32_t* const h2x = mb + L.h2x;
  uint32_t* const reg = mb + L.reg;
  uint32_t* const hdr2r = mb + L.hdr2r;
  auto* const rec2r = reinterpret_cast<grs::SegTile*>(mb + L.rec2r);
  K* const rk = static_cast<K*>(s->alt2_keys);
  uint32_t* const rv = PAIRS ? s->alt2_vals : nullptr;
  // H2 chunks: ~8 rounds of the resident blocks (2 per CU), 32K to 256K keys; the sample: one
  // 2^GRS_H2_PIECE_LOG-key piece in 2^k, k so that a uniform 16-bit bin still gets 512-1023
  // sampled keys (1/32 at 2^30: the regions' 6-sigma slack is then at most 26.5 %, inside the
  // region buffer's 30 %)
  uint32_t chunk = GRS_H2_CHUNK;
  while (chunk > 32768u && static_cast<uint64_t>(n) / chunk < 16u * static_cast<uint64_t>(std::max(1, s->cus)))
    chunk >>= 1;
  uint32_t shift = 0;
  while (shift < 6 && (static_cast<uint64_t>(n) >> (shift + 1)) >= 65536ull * 512) ++shift;
  chunk = std::min<uint32_t>(chunk << shift, 1u << 20);   // sampled: about as many keys a block
  if (s->h2_chunk != 0) chunk = s->h2_chunk;             // (GRS_OPT_H2_CHUNK: A/B runs)
  const uint32_t piece_log = s->h2_piece != 0 ? static_cast<uint32_t>(__builtin_ctz(s->h2_piece)) : GRS_H2_PIECE_LOG;
  // the region buffer's room (option msd = 2, a test hook: none, so the exact redo runs)
  const uint64_t cap2 = s->msd_mode == 2 ? 0 : static_cast<uint64_t>(msd_alt2_words(s->capacity));
  {
    if (xl)
      hipLaunchKernelGGL((grs::grs_msd_plan2<XL::TILE>), dim3(1), dim3(1024), 0, stream, samp, mult, pad,
                         totals, exact, chunk, tab, rec2, hdr2, shift == 0 ? 1u : 0u);
    else
      hipLaunchKernelGGL((grs::grs_msd_plan2<Big::TILE>), dim3(1), dim3(1024), 0, stream, samp, mult, pad,
                         totals, exact, chunk, tab, rec2, hdr2, shift == 0 ? 1u : 0u);
    GRS_HIP(hipGetLastError());
    hipLaunchKernelGGL((grs::grs_msd_hist2<K>), dim3(n / chunk + 257), dim3(1024), 0, stream, alt,
                       shift ? mb + L.h2s : h2x, st[1], static_cast<uint32_t>(words2), tab, chunk, shift,
                       (const uint32_t*)nullptr, top, piece_log);
    GRS_HIP(hipGetLastError());
    if (shift) {
      uint32_t* const room = mb + L.room;
      hipLaunchKernelGGL(grs::grs_msd_regions, dim3(256), dim3(256), 0, stream, tab, mb + L.h2s, reg, room);
      GRS_HIP(hipGetLastError());
      if (xl)
        hipLaunchKernelGGL((grs::grs_msd_plan3<XL::TILE>), dim3(1), dim3(1024), 0, stream, tab, room, cap2,
                           rec2r, hdr2r, spill2);
      else
        hipLaunchKernelGGL((grs::grs_msd_plan3<Big::TILE>), dim3(1), dim3(1024), 0, stream, tab, room, cap2,
                           rec2r, hdr2r, spill2);
      GRS_HIP(hipGetLastError());
    }
  }
  if ((r = mark()) != GRS_OK) return r;
  // P2: stable scatter by the second byte inside each top-byte bucket.  With a sample (large
  // sorts): alt -> the region buffer, each 16-bit segment in its region, its first tile writing
  // the region starts (dstart) and its last the totals (h2) and the spill flag; after a spill
  // (or for small sorts, always) the exact pass alt -> keys from H2's exact counts (h2x).
  {
    const Dig d2{-8, 255u};   // the byte below the top digit (+ *top)
    const dim3 grid(static_cast<uint32_t>(t2));
    constexpr uint32_t RG = 131072;
    auto go = [&](auto tshape) -> grs_status {
      using T = decltype(tshape);
      if (shift) {
        GRS_DIAG_CHECK("plans");
        GRS_DIAG_SET(cap2, region_len);
        hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT | RG, false>),
                           grid, dim3(T::BLOCK), 0, stream, alt, rk, valt, rv, d2, rec2r, hdr2r, reg, 256u,
                           tickets + GRS_XCDS, st[1], st[0], err, dstart, h2, spill2, (const uint32_t*)nullptr, top);
        GRS_HIP(hipGetLastError());
        GRS_DIAG_CHECK("P2region");
        GRS_DIAG_SET(n, region_len);
        // the redo: exact counts, then the exact pass in place (persistent, gated by the flag)
        hipLaunchKernelGGL((grs::grs_msd_hist2<K, T::TILE>), dim3(n / chunk + 257), dim3(1024), 0, stream, alt,
                           h2x, st[0], static_cast<uint32_t>(words2), tab, chunk, 0u, spill2, top, 8u, rec2, hdr2);
        GRS_HIP(hipGetLastError());
        hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT, true>),
                           dim3(s->cus), dim3(T::BLOCK), 0, stream, alt, keys, valt, vals, d2, rec2, hdr2, h2x,
                           256u, tickets + 14 * GRS_XCDS, st[0], st[1], err, (uint32_t*)nullptr,
                           (uint32_t*)nullptr, (uint32_t*)nullptr, spill2, top);
        GRS_HIP(hipGetLastError());
      } else {
        // no sample: the exact pass straight away (the flag says so to P3: in place)
        GRS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(spill2), 1, 1, stream));
        hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT, false>), grid,
                           dim3(T::BLOCK), 0, stream, alt, keys, valt, vals, d2, rec2, hdr2, h2x, 256u,
                           tickets + GRS_XCDS, st[1], st[0], err, (uint32_t*)nullptr, (uint32_t*)nullptr,
                           (uint32_t*)nullptr, (const uint32_t*)nullptr, top);
        GRS_HIP(hipGetLastError());
      }
      return GRS_OK;
    };
    if ((r = xl ? go(XL{}) : go(Big{})) != GRS_OK) return r;
    GRS_DIAG_CHECK("P2exact");
    hipLaunchKernelGGL(grs::grs_msd_starts, dim3(256), dim3(256), 0, stream, spill2, tab, h2, h2x, dstart,
                       mb + L.len2, mb + L.in2, mb + L.out2);
    GRS_HIP(hipGetLastError());
  }
  if ((r = mark()) != GRS_OK) return r;
  // P3: every 16-bit segment sorted by the bits below its prefix in LDS, from its region (in
  // place after a spill) to its sorted place in keys; longer ones listed: up to the largest LDS
  // shape's capacity for its persistent kernel (inputs narrower than the key, e.g. a rank's
  // range after the multi-GPU exchange), beyond that for the fallback (moved to their place
  // first: grs_msd_copy_big)
  using P3L = std::conditional_t<sizeof(K) == 4 && !PAIRS, MsdLocalC, MsdLocalB>;
  const uint32_t mid_max = P3L::SMAX > P3C::SMAX ? P3L::SMAX : P3C::SMAX;
  if constexpr (sizeof(K) == 4) {
    if (s->p3_mode == 1) {
      // persistent, the next segment's loads behind this one's stores (grs_msd_local_pf; the
      // ticket: big[16], zeroed by the sample kernel).  Measured slower than a workgroup per
      // segment (C4 P3 2.12 vs 1.97 ms, ns 0.80 vs 0.45: the ticket and the segment's table
      // reads are a serial latency per segment that the dispatcher's fresh workgroups do not
      // pay): an A/B option
      using LS = grs::LocalSort<K, PAIRS, P3C::BLOCK, P3C::I, P3C::C16>;
      constexpr int lds_per_cu = 160 * 1024 / static_cast<int>(sizeof(typename LS::Smem) + 16);
      // (u32 keys on 512 x 20: three workgroups' 80 registers spill the loop; two)
      constexpr int per_cu = std::min(std::min(lds_per_cu, 2048 / P3C::BLOCK), P3C::BLOCK == 512 && !PAIRS ? 2 : 8);
      constexpr int minw = std::max(1, per_cu * P3C::BLOCK / GRS_WAVE / 4);
      hipLaunchKernelGGL((grs::grs_msd_local_pf<K, PAIRS, P3C::BLOCK, P3C::I, P3C::C16, FT::TILE, minw>),
                         dim3(per_cu * std::max(1, s->cus)), dim3(P3C::BLOCK), 0, stream, keys, vals, rk, rv, spill2,
                         mb + L.len2, mb + L.in2, mb + L.out2, mid_max, mb + L.mid, bigc, mb + L.bin, mb + L.bstart,
                         mb + L.blen, mb + L.brow, rows, top, bigc + 16);
    } else if (!PAIRS && P3C::SMAX == MsdLocalC2::SMAX && s->p3_mode == 0) {
      // C4's 2^30 keys: the low halves in LDS, three workgroups a CU (grs_msd_local16; tools/lab8.py
      // round 6: 1.90 vs 1.96 ms uniform, 1.83 vs 1.99 on the reference's input).  Segments past
      // its 17408 keys (8 sigma above the mean at 2^30) take the mid list
      hipLaunchKernelGGL((grs::grs_msd_local16<512, 34, 6, FT::TILE>), dim3(65536), dim3(512), 0, stream,
                         (uint32_t*)keys, vals, (const uint32_t*)rk, rv, spill2, mb + L.len2, mb + L.in2, mb + L.out2,
                         mid_max, mb + L.mid, bigc, mb + L.bin, mb + L.bstart, mb + L.blen, mb + L.brow, rows, top);
    } else if (!PAIRS && P3C::SMAX == MsdLocalD::SMAX && s->p3_mode == 0 && msd_segment_need(n) <= 1024 * 34) {
      // past 1.13G keys up to ~2.18G: 1024 x 34 low halves, two workgroups a CU where LocalSort's
      // 1024 x 36 fits one (lab at 2^31: 4.81 vs ~5.3 ms).  No mid list in this shape's sort: a
      // segment past 34816 keys takes the fallback
      hipLaunchKernelGGL((grs::grs_msd_local16<1024, 34, 8, FT::TILE>), dim3(65536), dim3(1024), 0, stream,
                         (uint32_t*)keys, vals, (const uint32_t*)rk, rv, spill2, mb + L.len2, mb + L.in2, mb + L.out2,
                         1024u * 34u, mb + L.mid, bigc, mb + L.bin, mb + L.bstart, mb + L.blen, mb + L.brow, rows, top);
    } else {
      hipLaunchKernelGGL((grs::grs_msd_local<K, PAIRS, P3C::BLOCK, P3C::I, P3C::C16, FT::TILE>), dim3(65536),
                         dim3(P3C::BLOCK), 0, stream, keys, vals, rk, rv, spill2, mb + L.len2, mb + L.in2,
                         mb + L.out2, mid_max, mb + L.mid, bigc, mb + L.bin, mb + L.bstart, mb + L.blen, mb + L.brow,
                         rows, top);
    }
  } else {
    hipLaunchKernelGGL((grs::grs_msd_local<K, PAIRS, P3C::BLOCK, P3C::I, P3C::C16, FT::TILE>), dim3(65536),
                       dim3(P3C::BLOCK), 0, stream, keys, vals, rk, rv, spill2, mb + L.len2, mb + L.in2, mb + L.out2,
                       mid_max, mb + L.mid, bigc, mb + L.bin, mb + L.bstart, mb + L.blen, mb + L.brow, rows, top);
  }
  GRS_HIP(hipGetLastError());
  if (P3L::SMAX > P3C::SMAX) {
    constexpr int per_cu = P3L::SMAX * (sizeof(K) + (PAIRS ? 4 : 0)) <= 80 * 1024 ? 2 : 1;
    constexpr int minw = per_cu * P3L::BLOCK / GRS_WAVE / 4;
    // (with grs_msd_copy_big's work: one launch fewer)
    hipLaunchKernelGGL((grs::grs_msd_local_list<K, PAIRS, P3L::BLOCK, P3L::I, P3L::C16, minw>),
                       dim3(per_cu * s->cus), dim3(P3L::BLOCK), 0, stream, keys, vals, rk, rv, spill2, mb + L.mid,
                       top, (const uint32_t*)bigc, (const uint32_t*)(mb + L.bin), (const uint32_t*)(mb + L.bstart),
                       (const uint32_t*)(mb + L.blen));
    GRS_HIP(hipGetLastError());
  } else {
    hipLaunchKernelGGL((grs::grs_msd_copy_big<K, PAIRS>), dim3(4 * s->cus), dim3(256), 0, stream, rk, rv, keys, vals,
                       spill2, bigc, mb + L.bin, mb + L.bstart, mb + L.blen);
    GRS_HIP(hipGetLastError());
  }
  GRS_DIAG_CHECK("P3");
  GRS_DIAG_SET(n, n);
  if ((r = mark()) != GRS_OK) return r;
  // fallback: the listed segments by a segmented LSD on the bits below the prefix
  // (keys -> alt -> ... -> keys: ND is even)
  static_assert(ND % 2 == 0, "the fallback ends in keys");
  hipLaunchKernelGGL((grs::grs_seg_plan<FT::TILE, grs::kSegList>), dim3(1), dim3(1024), 0, stream,
                     mb + L.bstart, mb + L.blen, mb + L.brow, 0u, bigc, mb + L.spill, recf, hdrf);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_seg_hist<K, ND>), dim3(2 * s->cus), dim3(256), 0, stream, keys, recf, hdrf,
                     0, rows, st[0], 256u);
  GRS_HIP(hipGetLastError());
  for (int p = 0; p < ND; ++p) {
    K* const ik = (p & 1) ? alt : keys;
    K* const ok = (p & 1) ? keys : alt;
    uint32_t* const iv = (p & 1) ? valt : vals;
    uint32_t* const ov = (p & 1) ? vals : valt;
    hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, FT::BLOCK, FT::ITEMS, FT::MINW, FT::OPT, true>),
                       dim3(s->cus), dim3(FT::BLOCK), 0, stream, ik, ok, iv, ov, Dig{8 * p, 255u}, recf, hdrf,
                       rows + 256 * p, static_cast<uint32_t>(ND * 256), tickets + (2 + p) * GRS_XCDS,
                       st[p & 1], st[(p + 1) & 1], err, nullptr);
    GRS_HIP(hipGetLastError());
  }
  GRS_DIAG_CHECK("fallback");
  GRS_DIAG_SET(0, 0);
  if ((r = mark()) != GRS_OK) return r;
  if (evs) {
    s->info[s->calls % s->ring] = {ev, 6, false, 1};
    ++s->calls;
  }
  return GRS_OK;
}

template <typename K, bool PAIRS>
grs_status run_sort_msd(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, hipStream_t stream,
                        const K* src_in = nullptr, const uint32_t* vsrc_in = nullptr) {
  switch (msd_local_shape(n, sizeof(K) + (PAIRS ? 4 : 0))) {
    case 4: return run_msd<K, PAIRS, MsdLocalS>(s, keys, vals, n, stream, src_in, vsrc_in);
    case 5: return run_msd<K, PAIRS, MsdLocalM>(s, keys, vals, n, stream, src_in, vsrc_in);
    case 1:
      if constexpr (sizeof(K) == 8) return run_msd<K, PAIRS, MsdLocalW>(s, keys, vals, n, stream, src_in, vsrc_in);
      return run_msd<K, PAIRS, MsdLocalA>(s, keys, vals, n, stream, src_in, vsrc_in);
    case 2: return run_msd<K, PAIRS, MsdLocalB>(s, keys, vals, n, stream, src_in, vsrc_in);
    case 3:
      if constexpr (sizeof(K) == 4 && !PAIRS) return run_msd<K, PAIRS, MsdLocalC>(s, keys, vals, n, stream, src_in, vsrc_in);
      [[fallthrough]];
    case 6:
      if constexpr (sizeof(K) == 4 && !PAIRS) return run_msd<K, PAIRS, MsdLocalD>(s, keys, vals, n, stream, src_in, vsrc_in);
      [[fallthrough]];
    case 7:
      if constexpr (sizeof(K) == 4 && !PAIRS) return run_msd<K, PAIRS, MsdLocalC2>(s, keys, vals, n, stream, src_in, vsrc_in);
      [[fallthrough]];
    default: return set_err(GRS_EINVAL, "internal: no MSD shape for this n");
  }
}

// Stable key-range partition with N (compile-time) splitters: one bucket histogram + one pass
// whose digit is the bucket (grs::SplitterIdxDigit).  Buckets land contiguously in
// keys_out / vals_out in bucket order; the count + 1 bucket sizes go to d_counts (device).
// dig_dev: the functor in device memory (splitters computed on the device) or null.
// region > 0 (the sharded exchange): no bucket histogram; bucket b goes to
// keys_out[b * region, ...) instead of after the buckets before it (region >= n, and
// (count + 1) * region < 2^32), and the bucket sizes come from the look-back's group
// accumulators afterwards.  That skips one read of the keys.
template <typename K, bool PAIRS, int N>
grs_status run_partition_n(grs_sorter* s, const K* keys, const uint32_t* vals, K* keys_out,
                           uint32_t* vals_out, uint32_t n, const grs::SplitterIdxDigit<K, N>& dig,
                           const grs::SplitterIdxDigit<K, N>* dig_dev, int count,
                           uint32_t* d_counts, hipStream_t stream, uint32_t region = 0) {
  using T = PartTile<K, PAIRS>;
  using Dig = grs::SplitterIdxDigit<K, N>;
  const uint32_t tiles = (n + T::TILE - 1) / T::TILE;
  const size_t words = status_words_for(tiles, 16);
  if (words > s->status_words) return set_err(GRS_ECAPACITY, "status buffer too small");
  uint32_t* hist = s->ctrl;
  s->cb_dirty = true;   // run_sort's block may be this one (sorter.cb_i)
  if (region) {
    // "digit counts" of `region` each: the pass's digit-start scan yields b * region
    hipLaunchKernelGGL(grs::grs_part_init, dim3(std::max<uint32_t>(1u, std::min<uint32_t>(256u, static_cast<uint32_t>(words / 1024 + 1)))),
                       dim3(256), 0, stream, hist, static_cast<uint32_t>(GRS_CTRL_ERROR), region,
                       static_cast<uint32_t>(count + 1), s->status, static_cast<uint32_t>(words));
    GRS_HIP(hipGetLastError());
  } else {
    GRS_HIP(hipMemsetAsync(s->ctrl, 0, GRS_CTRL_ERROR * 4, stream));
    // one resident wave of workgroups (grid-stride loop): 2048 blocks at 6 per CU (76 VGPRs)
    // ran as 1536 + 512, a second, mostly empty round (tools/prof_partition.py)
    static const int per_cu = [] {
      int b = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, grs::grs_digit_hist<K, Dig>, GRS_HIST_BLOCK,
                                                       0) != hipSuccess || b < 1)
        b = 4;
      return b;
    }();
    const int grid = std::max(1, std::min<int>(per_cu * std::max(1, s->cus), (n + 4095) / 4096));
    hipLaunchKernelGGL((grs::grs_digit_hist<K, Dig>), dim3(grid), dim3(GRS_HIST_BLOCK), 0, stream,
                       keys, n, dig, dig_dev, hist, s->status, static_cast<uint32_t>(words));
    GRS_HIP(hipGetLastError());
  }
  grs_status r;
  if (s->rank_mode == 0)
    r = launch_pass<K, PAIRS, 4, T, kSmallOpt>(s, keys, keys_out, vals, vals_out, n, dig, dig_dev, hist,
                                             s->ctrl + GRS_CTRL_TICKETS, s->status,
                                             s->status + s->status_stride, stream);
  else
    r = launch_pass<K, PAIRS, 4, T, kMatchOpt>(s, keys, keys_out, vals, vals_out, n, dig, dig_dev, hist,
                                              s->ctrl + GRS_CTRL_TICKETS, s->status,
                                              s->status + s->status_stride, stream);
  if (r != GRS_OK) return r;
  if (region) {
    const uint32_t groups = (tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP;
    hipLaunchKernelGGL(grs::grs_lb_totals, dim3(1), dim3(256), 0, stream,
                       s->status + static_cast<size_t>(tiles) * 16, groups, 16u,
                       static_cast<uint32_t>(count + 1), d_counts);
    GRS_HIP(hipGetLastError());
  } else {
    GRS_HIP(hipMemcpyAsync(d_counts, hist, (count + 1) * 4, hipMemcpyDeviceToDevice, stream));
  }
  return GRS_OK;
}

// Host-side splitters (keys, optional shard-local thresholds) -> the smallest N >= count.
template <typename K, bool PAIRS>
grs_status run_partition(grs_sorter* s, const K* keys, const uint32_t* vals, K* keys_out,
                         uint32_t* vals_out, uint32_t n, const K* splitters, const uint32_t* th,
                         int count, uint32_t* d_counts, hipStream_t stream, uint32_t region = 0) {
  auto go = [&](auto nconst) {
    constexpr int N = decltype(nconst)::value;
    grs::SplitterIdxDigit<K, N> d{};
    d.count = N;
    for (int i = 0; i < GRS_MAX_SPLITTERS; ++i) {
      // padding splitters (i >= count) never count: (max key, max index) is above every element
      d.s[i] = i < count ? splitters[i] : static_cast<K>(~static_cast<K>(0));
      d.th[i] = i < count ? (th ? th[i] : 0u) : 0xFFFFFFFFu;
    }
    return run_partition_n<K, PAIRS, N>(s, keys, vals, keys_out, vals_out, n, d, nullptr, count,
                                        d_counts, stream, region);
  };
  if (count <= 1) return go(std::integral_constant<int, 1>{});
  if (count <= 3) return go(std::integral_constant<int, 3>{});
  if (count <= 7) return go(std::integral_constant<int, 7>{});
  return go(std::integral_constant<int, 15>{});
}

}  // namespace

extern "C" {

static grs_status partition_impl(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                                 void* d_keys_out, uint32_t* d_vals_out, size_t n,
                                 const void* splitters, const uint32_t* thresholds,
                                 int n_splitters, uint32_t* d_counts, void* stream,
                                 uint32_t region = 0) {
  if (!s) return set_err(GRS_EINVAL, "grs_partition: NULL sorter");
  if (n_splitters < 0 || n_splitters > GRS_MAX_SPLITTERS || (n_splitters > 0 && !splitters))
    return set_err(GRS_EINVAL, "grs_partition: 0..15 splitters required");
  if (!d_counts) return set_err(GRS_EINVAL, "grs_partition: d_counts is NULL");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_partition: n exceeds sorter capacity");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n == 0) {
    GRS_HIP(hipMemsetAsync(d_counts, 0, (n_splitters + 1) * 4, st));
    return GRS_OK;
  }
  if (!d_keys || !d_keys_out) return set_err(GRS_EINVAL, "grs_partition: NULL keys");
  if (s->pairs && (!d_vals || !d_vals_out))
    return set_err(GRS_EINVAL, "grs_partition: payload sorter needs d_vals / d_vals_out");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  const uint32_t n32 = static_cast<uint32_t>(n);
  grs_status r;
  if (s->key_type == GRS_KEY_U32) {
    if (s->pairs)
      r = run_partition<uint32_t, true>(s, (const uint32_t*)d_keys, d_vals, (uint32_t*)d_keys_out,
                                        d_vals_out, n32, (const uint32_t*)splitters, thresholds,
                                        n_splitters, d_counts, st, region);
    else
      r = run_partition<uint32_t, false>(s, (const uint32_t*)d_keys, nullptr, (uint32_t*)d_keys_out,
                                         nullptr, n32, (const uint32_t*)splitters, thresholds,
                                         n_splitters, d_counts, st, region);
  } else {
    if (s->pairs)
      r = run_partition<uint64_t, true>(s, (const uint64_t*)d_keys, d_vals, (uint64_t*)d_keys_out,
                                        d_vals_out, n32, (const uint64_t*)splitters, thresholds,
                                        n_splitters, d_counts, st, region);
    else
      r = run_partition<uint64_t, false>(s, (const uint64_t*)d_keys, nullptr, (uint64_t*)d_keys_out,
                                         nullptr, n32, (const uint64_t*)splitters, thresholds,
                                         n_splitters, d_counts, st, region);
  }
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_partition(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                         void* d_keys_out, uint32_t* d_vals_out, size_t n,
                         const void* splitters, int n_splitters, uint32_t* d_counts,
                         void* stream) {
  return partition_impl(s, d_keys, d_vals, d_keys_out, d_vals_out, n, splitters, nullptr,
                        n_splitters, d_counts, stream);
}

grs_status grs_partition_ranges(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                                void* d_keys_out, uint32_t* d_vals_out, size_t n,
                                const void* splitters, const uint32_t* thresholds,
                                int n_splitters, uint32_t* d_counts, void* stream) {
  if (n_splitters > 0 && !thresholds)
    return set_err(GRS_EINVAL, "grs_partition_ranges: thresholds are NULL");
  return partition_impl(s, d_keys, d_vals, d_keys_out, d_vals_out, n, splitters, thresholds,
                        n_splitters, d_counts, stream);
}

grs_status grs_partition_regions(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                                 void* d_keys_out, uint32_t* d_vals_out, size_t n,
                                 const void* splitters, const uint32_t* thresholds,
                                 int n_splitters, size_t region, uint32_t* d_counts, void* stream) {
  if (n_splitters > 0 && !thresholds)
    return set_err(GRS_EINVAL, "grs_partition_regions: thresholds are NULL");
  if (n > 0 && (region == 0 || static_cast<uint64_t>(n_splitters + 1) * region >= (uint64_t(1) << 32)))
    return set_err(GRS_EINVAL, "grs_partition_regions: need 0 < region and (n_splitters + 1) * region < 2^32");
  return partition_impl(s, d_keys, d_vals, d_keys_out, d_vals_out, n, splitters, thresholds,
                        n_splitters, d_counts, stream, static_cast<uint32_t>(region));
}

grs_status grs_sort_bits(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n, int begin_bit,
                         int end_bit, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_sort: NULL sorter");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort: n exceeds sorter capacity");
  const int kbits = s->key_type == GRS_KEY_U64 ? 64 : 32;
  if (begin_bit < 0 || end_bit > kbits || begin_bit >= end_bit)
    return set_err(GRS_EINVAL, "grs_sort: bad bit range");
  if (n == 0) return GRS_OK;  // the reference's N = 0 "won't crash" (PrefixSumSsbo.cpp:121-124)
  if (!d_keys) return set_err(GRS_EINVAL, "grs_sort: d_keys is NULL");
  if (s->pairs && !d_vals) return set_err(GRS_EINVAL, "grs_sort: payload sorter needs d_vals");
  // natural alignment of the element types (u32 pairs at 4-byte alignment are fine: the record
  // passes that move 8 bytes on the caller's arrays check for 8 and fall back, run_sort)
  if ((reinterpret_cast<uintptr_t>(d_keys) & (static_cast<uintptr_t>(kbits / 8) - 1)) != 0 ||
      (reinterpret_cast<uintptr_t>(d_vals) & 3u) != 0)
    return set_err(GRS_EINVAL, "grs_sort: d_keys / d_vals not aligned to their element size");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t n32 = static_cast<uint32_t>(n);
  grs_status r = GRS_EINVAL;
  const bool u64 = s->key_type == GRS_KEY_U64;
  s->last_msd_cb = -1;
  if (use_msd(s, n, begin_bit, end_bit)) {
    if (!u64 && !s->pairs)
      r = run_sort_msd<uint32_t, false>(s, (uint32_t*)d_keys, nullptr, n32, st);
    else if (!u64)
      r = run_sort_msd<uint32_t, true>(s, (uint32_t*)d_keys, d_vals, n32, st);
    else
      r = run_sort_msd<uint64_t, false>(s, (uint64_t*)d_keys, nullptr, n32, st);
  } else if (!u64 && !s->pairs && s->radix_bits == 8)
    r = run_sort<uint32_t, false, 8>(s, (uint32_t*)d_keys, nullptr, n32, begin_bit, end_bit, st);
  else if (!u64 && !s->pairs && s->radix_bits == 4)
    r = run_sort<uint32_t, false, 4>(s, (uint32_t*)d_keys, nullptr, n32, begin_bit, end_bit, st);
  else if (!u64 && s->pairs && s->radix_bits == 8)
    r = run_sort<uint32_t, true, 8>(s, (uint32_t*)d_keys, d_vals, n32, begin_bit, end_bit, st);
  else if (!u64 && s->pairs && s->radix_bits == 4)
    r = run_sort<uint32_t, true, 4>(s, (uint32_t*)d_keys, d_vals, n32, begin_bit, end_bit, st);
  else if (u64 && !s->pairs && s->radix_bits == 8)
    r = run_sort<uint64_t, false, 8>(s, (uint64_t*)d_keys, nullptr, n32, begin_bit, end_bit, st);
  else if (u64 && !s->pairs && s->radix_bits == 4)
    r = run_sort<uint64_t, false, 4>(s, (uint64_t*)d_keys, nullptr, n32, begin_bit, end_bit, st);
  else if (u64 && s->pairs && s->radix_bits == 8)
    r = run_sort<uint64_t, true, 8>(s, (uint64_t*)d_keys, d_vals, n32, begin_bit, end_bit, st);
  else if (u64 && s->pairs && s->radix_bits == 4)
    r = run_sort<uint64_t, true, 4>(s, (uint64_t*)d_keys, d_vals, n32, begin_bit, end_bit, st);
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_sort(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_sort: NULL sorter");
  return grs_sort_bits(s, d_keys, d_vals, n, 0, s->key_type == GRS_KEY_U64 ? 64 : 32, stream);
}

grs_status grs_timing_history(grs_sorter* s, int k, grs_timing* out) {
  if (!s || !out) return set_err(GRS_EINVAL, "grs_timing_history: NULL argument");
  std::memset(out, 0, sizeof(*out));
  if (s->ring == 0 || k < 0 || k >= s->ring || k >= s->calls)
    return set_err(GRS_EINVAL, "grs_timing_history: no such profiled call");
  const long long slot = (s->calls - 1 - k) % s->ring;
  const grs_sorter::CallInfo ci = s->info[slot];
  hipEvent_t* e = s->ev + slot * grs_sorter::EV_PER_CALL;
  GRS_HIP(hipEventSynchronize(e[ci.ev_used - 1]));
  out->passes = ci.passes;
  out->kind = ci.kind;
  float ms = 0;
  GRS_HIP(hipEventElapsedTime(&ms, e[0], e[1]));
  out->hist_ms = ms;
  for (int p = 0; p < ci.passes && p < 16; ++p) {
    GRS_HIP(hipEventElapsedTime(&ms, e[1 + p], e[2 + p]));
    out->pass_ms[p] = ms;
  }
  if (ci.copy) {
    GRS_HIP(hipEventElapsedTime(&ms, e[1 + ci.passes], e[2 + ci.passes]));
    out->copy_ms = ms;
  }
  GRS_HIP(hipEventElapsedTime(&ms, e[0], e[ci.ev_used - 1]));
  out->total_ms = ms;
  return GRS_OK;
}

grs_status grs_last_timing(grs_sorter* s, grs_timing* out) { return grs_timing_history(s, 0, out); }

grs_status grs_check_error(grs_sorter* s) {
  if (!s) return set_err(GRS_EINVAL, "grs_check_error: NULL sorter");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  uint32_t e = 0;
  grs_status r = GRS_OK;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&e, s->ctrl + GRS_CTRL_ERROR, 4, hipMemcpyDeviceToHost) != hipSuccess ||
      (e && hipMemset(s->ctrl + GRS_CTRL_ERROR, 0, 4) != hipSuccess))
    r = set_err(GRS_EHIP, "grs_check_error: HIP failure");
  if (prev != s->device) (void)hipSetDevice(prev);
  if (r != GRS_OK) return r;
  return e ? set_err(GRS_ETIMEOUT, "a look-back spin exceeded its bound") : GRS_OK;
}

grs_status grs_stream_check_error(grs_sorter* s, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_stream_check_error: NULL sorter");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  grs_status r = GRS_OK;
  *s->h_err = 0;
  if (hipMemcpyAsync(s->h_err, s->ctrl + GRS_CTRL_ERROR, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_stream_check_error: HIP failure");
  const uint32_t e = *s->h_err;
  if (r == GRS_OK && e && hipMemsetAsync(s->ctrl + GRS_CTRL_ERROR, 0, 4, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_stream_check_error: HIP failure");
  if (prev != s->device) (void)hipSetDevice(prev);
  if (r != GRS_OK) return r;
  return e ? set_err(GRS_ETIMEOUT, "a look-back spin exceeded its bound") : GRS_OK;
}

static int grid_for(size_t n, int block) {
  const size_t g = (n + block - 1) / block;
  return static_cast<int>(std::max<size_t>(1, std::min<size_t>(g, 8192)));
}

grs_status grs_iota_u32(uint32_t* d_out, size_t n, uint32_t start, void* stream) {
  if (n == 0) return GRS_OK;
  if (!d_out) return set_err(GRS_EINVAL, "grs_iota_u32: NULL");
  hipLaunchKernelGGL(grs::grs_iota_u32, dim3(grid_for(n, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_out, static_cast<uint64_t>(n), start);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

grs_status grs_copy_u32(const uint32_t* d_src, uint32_t* d_dst, size_t n, void* stream) {
  if (n == 0) return GRS_OK;
  if (!d_src || !d_dst) return set_err(GRS_EINVAL, "grs_copy_u32: NULL");
  hipLaunchKernelGGL(grs::grs_copy_u32, dim3(grid_for(n, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), d_src, d_dst, static_cast<uint64_t>(n));
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

static grs_status gather_records(const void* d_src, void* d_dst, const uint32_t* d_idx, size_t n,
                                 size_t record_bytes, void* stream, uint32_t idx_max) {
  if (n == 0) return GRS_OK;
  if (!d_src || !d_dst || !d_idx || record_bytes == 0 || record_bytes > 0xFFFFFFFFull)
    return set_err(GRS_EINVAL, "grs_gather_records: bad argument");
  hipLaunchKernelGGL(grs::grs_gather_records, dim3(grid_for(n * ((record_bytes + 3) / 4), 256)),
                     dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), d_idx,
                     static_cast<uint64_t>(n), static_cast<uint32_t>(record_bytes), idx_max);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

grs_status grs_gather_records(const void* d_src, void* d_dst, const uint32_t* d_idx, size_t n,
                              size_t record_bytes, void* stream) {
  return gather_records(d_src, d_dst, d_idx, n, record_bytes, stream, 0xFFFFFFFFu);
}

grs_status grs_fill_splitmix(void* d_keys, size_t n, int key_bytes, uint64_t seed,
                             uint64_t first_index, void* stream) {
  if (n == 0) return GRS_OK;
  if (!d_keys || (key_bytes != 4 && key_bytes != 8))
    return set_err(GRS_EINVAL, "grs_fill_splitmix: bad argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (key_bytes == 4)
    hipLaunchKernelGGL(grs::grs_fill_splitmix<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint32_t*>(d_keys), static_cast<uint64_t>(n), seed, first_index);
  else
    hipLaunchKernelGGL(grs::grs_fill_splitmix<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint64_t*>(d_keys), static_cast<uint64_t>(n), seed, first_index);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

grs_status grs_fill_permutation(void* d_keys, size_t n, int key_bytes, uint64_t total, uint64_t seed,
                                 uint64_t first_index, void* stream) {
  if (n == 0) return GRS_OK;
  if (!d_keys || (key_bytes != 4 && key_bytes != 8) || total == 0 || first_index > total ||
      n > total - first_index || (key_bytes == 4 && total > (uint64_t(1) << 32)) || total > (uint64_t(1) << 62))
    return set_err(GRS_EINVAL, "grs_fill_permutation: bad argument");
  grs::PermParams p{};
  int b = 1;
  while (b < 62 && (uint64_t(1) << b) < total) ++b;
  p.mask = (uint64_t(1) << b) - 1;
  p.half = b / 2 + 1;
  for (int r = 0; r < 4; ++r) {
    p.a[r] = grs::splitmix64(seed + 2 * r) | 1u;
    p.c[r] = grs::splitmix64(seed + 2 * r + 1);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (key_bytes == 4)
    hipLaunchKernelGGL(grs::grs_fill_permutation<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint32_t*>(d_keys), static_cast<uint64_t>(n), total, first_index, p);
  else
    hipLaunchKernelGGL(grs::grs_fill_permutation<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint64_t*>(d_keys), static_cast<uint64_t>(n), total, first_index, p);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

grs_status grs_count_inversions(const void* d_keys, size_t n, int key_bytes, uint64_t* out_count,
                                void* stream) {
  if (!out_count || (key_bytes != 4 && key_bytes != 8))
    return set_err(GRS_EINVAL, "grs_count_inversions: bad argument");
  *out_count = 0;
  if (n < 2) return GRS_OK;
  if (!d_keys) return set_err(GRS_EINVAL, "grs_count_inversions: NULL keys");
  hipStream_t st = static_cast<hipStream_t>(stream);
  unsigned long long* d_cnt = nullptr;
  GRS_HIP(hipMalloc(&d_cnt, sizeof(*d_cnt)));
  grs_status r = GRS_OK;
  if (hipMemsetAsync(d_cnt, 0, sizeof(*d_cnt), st) != hipSuccess) r = GRS_EHIP;
  if (r == GRS_OK) {
    if (key_bytes == 4)
      hipLaunchKernelGGL(grs::grs_count_inversions<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0,
                         st, static_cast<const uint32_t*>(d_keys), static_cast<uint64_t>(n), d_cnt);
    else
      hipLaunchKernelGGL(grs::grs_count_inversions<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0,
                         st, static_cast<const uint64_t*>(d_keys), static_cast<uint64_t>(n), d_cnt);
    if (hipGetLastError() != hipSuccess) r = GRS_EHIP;
  }
  unsigned long long h = 0;
  if (r == GRS_OK && hipMemcpyAsync(&h, d_cnt, sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess)
    r = GRS_EHIP;
  if (r == GRS_OK && hipStreamSynchronize(st) != hipSuccess) r = GRS_EHIP;
  (void)hipFree(d_cnt);
  if (r != GRS_OK) return set_err(r, "grs_count_inversions: HIP failure");
  *out_count = h;
  return GRS_OK;
}

grs_status grs_key_transform(void* d_keys, size_t n, int key_bytes, int kind, int inverse,
                             void* stream) {
  if ((key_bytes != 4 && key_bytes != 8) || kind < 0 || kind > 2)
    return set_err(GRS_EINVAL, "grs_key_transform: bad key_bytes or kind");
  if (n == 0 || kind == GRS_KEYS_UNSIGNED) return GRS_OK;
  if (!d_keys) return set_err(GRS_EINVAL, "grs_key_transform: NULL keys");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (key_bytes == 4)
    hipLaunchKernelGGL(grs::grs_key_transform<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint32_t*>(d_keys), static_cast<uint64_t>(n), kind, inverse);
  else
    hipLaunchKernelGGL(grs::grs_key_transform<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<uint64_t*>(d_keys), static_cast<uint64_t>(n), kind, inverse);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

// Scan scratch: [0] error word (set when a look-back spin gives up), [1] ticket, [2..3] pad,
// then one 64-bit look-back status word per tile.  Tiles of 8K items below 2^22 items, 32K from
// there (more tiles in flight at small n, fewer look-backs at large n; tools/ab_scan.py).
static constexpr size_t kScanTileSmall = (GRS_SCAN_OP_BLOCK / GRS_WAVE) * 8 * 4 * GRS_WAVE;
static constexpr size_t kScanTileLarge = (GRS_SCAN_OP_BLOCK / GRS_WAVE) * 32 * 4 * GRS_WAVE;
static constexpr size_t kScanLargeMin = size_t(1) << 22;

size_t grs_scan_scratch_bytes(size_t n) { return 16 + 8 * ((n + kScanTileSmall - 1) / kScanTileSmall); }

}  // extern "C"

// The one-pass scan.  err2 (nullable): a sorter's error word that a look-back timeout also
// sets, so the internal callers (segmented sort, presorted exchange) surface GRS_ETIMEOUT
// through grs_check_error / grs_stream_check_error like the sort passes.
static grs_status scan_u32_impl(const uint32_t* d_in, uint32_t* d_out, size_t n, uint32_t* d_total,
                                void* d_scratch, size_t scratch_bytes, void* stream,
                                uint32_t* err2) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n > GRS_SCAN_MAX_N) return set_err(GRS_ECAPACITY, "grs_exclusive_scan_u32: n too large");
  if (n == 0) {
    if (d_total) GRS_HIP(hipMemsetAsync(d_total, 0, 4, st));
    return GRS_OK;
  }
  if (!d_in || !d_out || !d_scratch)
    return set_err(GRS_EINVAL, "grs_exclusive_scan_u32: NULL argument");
  if (scratch_bytes < grs_scan_scratch_bytes(n))
    return set_err(GRS_EINVAL, "grs_exclusive_scan_u32: scratch too small");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out)) & 15u)
    return set_err(GRS_EINVAL, "grs_exclusive_scan_u32: d_in and d_out must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_scratch) & 7u)
    return set_err(GRS_EINVAL, "grs_exclusive_scan_u32: scratch must be 8-byte aligned");
  uint32_t* ctl = static_cast<uint32_t*>(d_scratch);
  const bool large = n >= kScanLargeMin;
  const size_t tile = large ? kScanTileLarge : kScanTileSmall;
  const uint32_t tiles = static_cast<uint32_t>((n + tile - 1) / tile);
  const uint32_t n32 = static_cast<uint32_t>(n);
  GRS_HIP(hipMemsetAsync(ctl, 0, 16 + 8 * static_cast<size_t>(tiles), st));
  if (large)
    hipLaunchKernelGGL(grs::grs_scan_onepass<32>, dim3(tiles), dim3(GRS_SCAN_OP_BLOCK), 0, st, d_in,
                       d_out, n32, ctl, d_total, err2);
  else
    hipLaunchKernelGGL(grs::grs_scan_onepass<8>, dim3(tiles), dim3(GRS_SCAN_OP_BLOCK), 0, st, d_in,
                       d_out, n32, ctl, d_total, err2);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

extern "C" {

grs_status grs_exclusive_scan_u32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                  uint32_t* d_total, void* d_scratch, size_t scratch_bytes,
                                  void* stream) {
  return scan_u32_impl(d_in, d_out, n, d_total, d_scratch, scratch_bytes, stream, nullptr);
}

grs_status grs_scan_check_error(const void* d_scratch, void* stream) {
  if (!d_scratch) return set_err(GRS_EINVAL, "grs_scan_check_error: NULL scratch");
  hipStream_t st = static_cast<hipStream_t>(stream);
  uint32_t e = 0;
  GRS_HIP(hipMemcpyAsync(&e, static_cast<const uint32_t*>(d_scratch), 4,
                         hipMemcpyDeviceToHost, st));
  GRS_HIP(hipStreamSynchronize(st));
  return e ? set_err(GRS_ETIMEOUT, "a scan look-back spin exceeded its bound") : GRS_OK;
}

// At most 16 segments, some longer than the LDS path takes: each segment is sorted on its own by
// the sorter (its keys and payload are contiguous: sub-range pointers), 16 B of traffic per
// pair per pass and no gather.  (A whole-array key sort + one partition pass by segment
// measured 2.97 ms for 4 x 2^24 pairs: its payload gather reads 4 B per 128-B line.)  The
// offsets are read back once (one stream synchronisation).  Keys-only calls carry a scratch
// rider.
static grs_status sort_segmented_few(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n,
                                     const uint32_t* d_offsets, int num_segments, void* stream) {
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  grs_status r = GRS_OK;
  uint32_t off[GRS_MAX_SPLITTERS + 2] = {};
  if (hipMemcpyAsync(off, d_offsets, (num_segments + 1) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_segmented: offsets");
  if (r == GRS_OK && !d_vals)   // the keys-only rider
    r = grow_buf(s, &s->seg_buf, &s->seg_bytes, n * 4, "grs_sort_segmented: scratch");
  for (int g = 0; g < num_segments && r == GRS_OK; ++g) {
    const uint32_t lo = off[g], hi = off[g + 1];
    if (hi <= lo + 1) continue;
    if (hi > n) {
      r = set_err(GRS_EINVAL, "grs_sort_segmented: offsets past n");
      break;
    }
    uint32_t* v = d_vals ? d_vals + lo : static_cast<uint32_t*>(s->seg_buf) + lo;
    r = grs_sort(s, static_cast<char*>(d_keys) + static_cast<size_t>(lo) * kb, v, hi - lo, stream);
  }
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

// u32 keys: one sort of u64 keys (segment << 32 | key) by bits [0, 32 + ceil(log2 S)), the
// payload riding along; no random gathers (grs_segment_marks / _compose / _split).
// Scratch (seg_buf): comp u64[n] | marks u32[n] | marks_excl u32[n] | scan scratch.
static grs_status sort_segmented_u32(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n,
                                     const uint32_t* d_offsets, int num_segments, void* stream) {
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t scan_bytes = grs_scan_scratch_bytes(n);
  const size_t need = al(n * 8) + 2 * al(n * 4) + al(scan_bytes);
  grs_status r = grow_buf(s, &s->seg_buf, &s->seg_bytes, need, "grs_sort_segmented: scratch");
  if (r == GRS_OK && (!s->seg64 || s->seg64->capacity < n)) {
    if (s->seg64) grs_destroy(s->seg64);
    s->seg64 = nullptr;
    r = grs_create(&s->seg64, s->capacity, GRS_KEY_U64, 1, 8, s->device);
  }
  char* b = static_cast<char*>(s->seg_buf);
  uint64_t* comp = reinterpret_cast<uint64_t*>(b);
  uint32_t* marks = reinterpret_cast<uint32_t*>(b + al(n * 8));
  uint32_t* excl = reinterpret_cast<uint32_t*>(b + al(n * 8) + al(n * 4));
  void* scan_scratch = b + al(n * 8) + 2 * al(n * 4);
  int segbits = 0;
  while ((1ll << segbits) < num_segments) ++segbits;
  if (r == GRS_OK && hipMemsetAsync(marks, 0, n * 4, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_segmented: memset");
  if (r == GRS_OK && num_segments > 1) {
    hipLaunchKernelGGL(grs::grs_segment_marks, dim3(grid_for(num_segments, 256)), dim3(256), 0, st,
                       d_offsets, static_cast<uint32_t>(num_segments) , static_cast<uint32_t>(n),
                       marks);
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (r == GRS_OK)
    r = scan_u32_impl(marks, excl, n, nullptr, scan_scratch, scan_bytes, stream, s->ctrl + GRS_CTRL_ERROR);
  if (r == GRS_OK) {
    hipLaunchKernelGGL(grs::grs_segment_compose, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<const uint32_t*>(d_keys), marks, excl, comp,
                       static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  // payload: the caller's values, or the marks buffer as a don't-care rider
  if (r == GRS_OK) r = grs_sort_bits(s->seg64, comp, d_vals ? d_vals : marks, n, 0, 32 + segbits, stream);
  if (r == GRS_OK) {   // the inner sorter's look-back timeouts surface through this sorter's checks
    hipLaunchKernelGGL(grs::grs_fold_error, dim3(1), dim3(64), 0, st, s->seg64->ctrl + GRS_CTRL_ERROR,
                       s->ctrl + GRS_CTRL_ERROR);
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (r == GRS_OK) {
    hipLaunchKernelGGL(grs::grs_segment_split, dim3(grid_for(n, 256)), dim3(256), 0, st, comp,
                       static_cast<uint32_t*>(d_keys), static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

}  // extern "C"

namespace {

// Segments of any length (round 5): a segmented LSD over the segment table -- one planner
// block (tiles never straddle a segment; a segment of one tile is solo), one histogram launch
// (digit counts per segment of several tiles; solo tiles count themselves), then one
// grs_onesweep_seg launch per 8-bit digit whose look-back chains restart at every segment.
// No host synchronisation.  Scratch (seg_buf): header | tile records | histogram rows | two
// status buffers | planner spill.
template <typename K, bool PAIRS>
grs_status sort_segmented_seg(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n,
                              const uint32_t* d_offsets, uint32_t nseg, hipStream_t st) {
  using T = BigTile<K, PAIRS>;
  constexpr int ND = static_cast<int>(sizeof(K));   // 8-bit digits
  constexpr uint32_t G = GRS_LB_GROUP;
  const size_t tiles_max = n / T::TILE + nseg + 1;
  const size_t multi_max = n / (T::TILE + 1) + 1;
  const size_t rows_tiles = 2 * (n / T::TILE) + 2;   // tiles of the segments of several tiles
  const size_t groups_max = rows_tiles / G + multi_max + 1;
  const size_t sw = (rows_tiles + 2 * groups_max) * 256;
  auto al = [](size_t w) { return (w + 63) & ~static_cast<size_t>(63); };
  const size_t o_rec = 64, o_rows = o_rec + al(tiles_max * 8), o_st0 = o_rows + al(multi_max * ND * 256);
  const size_t o_st1 = o_st0 + al(sw), o_spill = o_st1 + al(sw), words = o_spill + al(6 * (size_t(nseg) + 1));
  grs_status r = grow_buf(s, &s->seg_buf, &s->seg_bytes, words * 4, "grs_sort_segmented");
  if (r != GRS_OK) return r;
  uint32_t* const b = static_cast<uint32_t*>(s->seg_buf);
  uint32_t* const hdr = b;
  auto* const rec = reinterpret_cast<grs::SegTile*>(b + o_rec);
  uint32_t* const rows = b + o_rows;
  uint32_t* const st0 = b + o_st0;
  uint32_t* const st1 = b + o_st1;
  uint32_t* const err = s->ctrl + GRS_CTRL_ERROR;
  // per-pass tickets: the tail of the control block's ticket area (zeroed here: the sort
  // calls' alternation does not cover this path)
  uint32_t* const tickets = b + 16;
  GRS_HIP(hipMemsetAsync(tickets, 0, 16 * 4, st));
  GRS_HIP(hipMemsetAsync(rows, 0, multi_max * ND * 256 * 4, st));
  hipLaunchKernelGGL((grs::grs_seg_plan<T::TILE, grs::kSegOffsets>), dim3(1), dim3(1024), 0, st, d_offsets,
                     nullptr, nullptr, nseg, nullptr, b + o_spill, rec, hdr);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_seg_hist<K, ND>), dim3(8 * s->cus), dim3(256), 0, st, keys, rec, hdr, 0, rows,
                     st0, 256u);
  GRS_HIP(hipGetLastError());
  K* const alt = static_cast<K*>(s->alt_keys);
  uint32_t* const valt = PAIRS ? s->alt_vals : nullptr;
  const dim3 grid(static_cast<uint32_t>(tiles_max));
  for (int p = 0; p < ND; ++p) {
    K* const ik = (p & 1) ? alt : keys;
    K* const ok = (p & 1) ? keys : alt;
    uint32_t* const iv = (p & 1) ? valt : vals;
    uint32_t* const ov = (p & 1) ? vals : valt;
    hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT, false>), grid,
                       dim3(T::BLOCK), 0, st, ik, ok, iv, ov, grs::RadixDigit<K>{8 * p, 255u}, rec, hdr,
                       rows + 256 * p, static_cast<uint32_t>(ND * 256), tickets + p, (p & 1) ? st1 : st0,
                       (p & 1) ? st0 : st1, err, nullptr);
    GRS_HIP(hipGetLastError());
  }
  return GRS_OK;
}

// Segments of 16K keys and more on average, whose top-byte runs fit LDS (round 5): one stable
// scatter by the top byte inside every segment (keys -> alt; grs_onesweep_seg over a
// kSegOffsetsAll plan, each segment's first tile writing its 256 run starts), the runs as work
// lists (grs_seg_runs), each run sorted by the bits below the top byte in LDS (alt -> keys:
// grs_seg_local_list, a primary shape sized for the average run and the largest shape), and
// runs longer than the largest shape by a segmented LSD on those bits over the big list
// (kSegList plan, histograms, KB/8 - 1 persistent passes alt -> keys -> ... -> keys: an odd
// count; leave at once when the list is empty).  Two HBM round trips per key where runs fit,
// against KB/8 for the segmented LSD.  No host synchronisation.  Scratch (seg_buf): headers |
// tickets and list counters | tile records | top-byte rows | run starts | lists | fallback rows
// and records | two status buffers | planner spill.
template <typename K, bool PAIRS, typename P, typename L>
grs_status sort_segmented_msd(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, const uint32_t* d_offsets,
                              uint32_t nseg, hipStream_t st) {
  using T = BigTile<K, PAIRS>;
  constexpr int KB = 8 * static_cast<int>(sizeof(K));
  constexpr int NDF = KB / 8 - 1;   // fallback digits (odd: alt -> ... -> keys)
  constexpr uint32_t G = GRS_LB_GROUP, TF = T::TILE;
  static_assert(NDF % 2 == 1, "the fallback ends in keys");
  static_assert(L::SMAX >= P::SMAX, "shapes");
  const size_t tiles_max = n / TF + nseg + 1;
  const size_t ecap = std::min<size_t>(size_t(nseg) * 256, n) + 1;   // entries of a list
  const size_t bcap = std::min<size_t>(size_t(nseg) * 256, n / (L::SMAX + 1) + 1);
  const size_t mr = n / (TF + 1) + 1;                                // fallback histogram rows
  const size_t rows_tiles = 2 * (n / TF) + 2;
  const size_t groups_max = rows_tiles / G + std::max<size_t>(mr, n / (TF + 1) + 1) + 1;
  const size_t sw = (rows_tiles + 2 * groups_max) * 256;
  auto al = [](size_t w) { return (w + 63) & ~static_cast<size_t>(63); };
  const size_t o_tk = 64, o_cnt = o_tk + 64;   // 64 ticket words, then 4 list counters
  const size_t o_rec = 256, o_rows = o_rec + al(tiles_max * 8), o_ds = o_rows + al(size_t(nseg) * 256);
  const size_t o_prim = o_ds + al(size_t(nseg) * 256), o_mid = o_prim + al(2 * ecap);
  const size_t o_bst = o_mid + al(2 * ecap), o_bln = o_bst + al(bcap), o_brw = o_bln + al(bcap);
  const size_t o_rowf = o_brw + al(bcap), o_recf = o_rowf + al(mr * NDF * 256);
  const size_t o_st0 = o_recf + al((n / TF + bcap + 1) * 8), o_st1 = o_st0 + al(sw);
  const size_t o_spill = o_st1 + al(sw), words = o_spill + al(6 * (std::max<size_t>(nseg, bcap) + 1));
  grs_status r = grow_buf(s, &s->seg_buf, &s->seg_bytes, words * 4, "grs_sort_segmented");
  if (r != GRS_OK) return r;
  uint32_t* const b = static_cast<uint32_t*>(s->seg_buf);
  uint32_t* const hdr = b;
  uint32_t* const hdrf = b + 4;
  uint32_t* const tickets = b + o_tk;
  uint32_t* const cnt = b + o_cnt;
  auto* const rec = reinterpret_cast<grs::SegTile*>(b + o_rec);
  auto* const recf = reinterpret_cast<grs::SegTile*>(b + o_recf);
  uint32_t* const rows = b + o_rows;
  uint32_t* const ds = b + o_ds;
  uint32_t* const stt[2] = {b + o_st0, b + o_st1};
  uint32_t* const err = s->ctrl + GRS_CTRL_ERROR;
  K* const alt = static_cast<K*>(s->alt_keys);
  uint32_t* const valt = PAIRS ? s->alt_vals : nullptr;
  using Dig = grs::RadixDigit<K>;
  GRS_HIP(hipMemsetAsync(tickets, 0, (64 + 4) * 4, st));
  GRS_HIP(hipMemsetAsync(rows, 0, size_t(nseg) * 256 * 4, st));
  // the top-byte scatter inside every segment
  hipLaunchKernelGGL((grs::grs_seg_plan<TF, grs::kSegOffsetsAll>), dim3(1), dim3(1024), 0, st, d_offsets,
                     nullptr, nullptr, nseg, nullptr, b + o_spill, rec, hdr);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_seg_hist<K, 1>), dim3(8 * s->cus), dim3(256), 0, st, keys, rec, hdr, KB - 8, rows,
                     stt[0], 256u);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT, false>),
                     dim3(static_cast<uint32_t>(tiles_max)), dim3(T::BLOCK), 0, st, keys, alt, vals, valt,
                     Dig{KB - 8, 255u}, rec, hdr, rows, 256u, tickets, stt[0], stt[1], err, ds);
  GRS_HIP(hipGetLastError());
  // the runs as lists, then sorted in LDS, alt -> keys
  hipLaunchKernelGGL((grs::grs_seg_runs<P::SMAX, L::SMAX, TF, NDF>), dim3(nseg), dim3(256), 0, st, d_offsets, ds,
                     cnt, b + o_prim, b + o_mid, b + o_bst, b + o_bln, b + o_brw, b + o_rowf);
  GRS_HIP(hipGetLastError());
  auto local = [&](auto shape, const uint32_t* count, const uint32_t* list) {
    using S = decltype(shape);
    using LS = grs::LocalSort<K, PAIRS, S::BLOCK, S::I, S::C16, KB / 8>;
    constexpr int per_cu = std::max<int>(1, std::min<int>(2048 / S::BLOCK, 160 * 1024 / static_cast<int>(sizeof(typename LS::Smem))));
    constexpr int minw = std::max(1, per_cu * S::BLOCK / GRS_WAVE / 4);
    hipLaunchKernelGGL((grs::grs_seg_local_list<K, PAIRS, S::BLOCK, S::I, S::C16, minw>), dim3(per_cu * s->cus),
                       dim3(S::BLOCK), 0, st, alt, valt, keys, vals, count, list);
  };
  local(P{}, cnt, b + o_prim);
  GRS_HIP(hipGetLastError());
  if constexpr (L::SMAX > P::SMAX) {
    local(L{}, cnt + 1, b + o_mid);
    GRS_HIP(hipGetLastError());
  }
  // fallback: runs longer than the largest shape, a segmented LSD below the top byte
  hipLaunchKernelGGL((grs::grs_seg_plan<TF, grs::kSegList>), dim3(1), dim3(1024), 0, st, b + o_bst, b + o_bln,
                     b + o_brw, 0u, cnt + 2, b + o_spill, recf, hdrf);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_seg_hist<K, NDF>), dim3(2 * s->cus), dim3(256), 0, st, alt, recf, hdrf, 0,
                     b + o_rowf, stt[0], 256u);
  GRS_HIP(hipGetLastError());
  for (int p = 0; p < NDF; ++p) {
    K* const ik = (p & 1) ? keys : alt;
    K* const ok = (p & 1) ? alt : keys;
    uint32_t* const iv = (p & 1) ? vals : valt;
    uint32_t* const ov = (p & 1) ? valt : vals;
    hipLaunchKernelGGL((grs::grs_onesweep_seg<K, PAIRS, 8, T::BLOCK, T::ITEMS, T::MINW, T::OPT, true>), dim3(s->cus),
                       dim3(T::BLOCK), 0, st, ik, ok, iv, ov, Dig{8 * p, 255u}, recf, hdrf,
                       b + o_rowf + 256 * p, static_cast<uint32_t>(NDF * 256), tickets + 8 * (1 + p),
                       stt[p & 1], stt[(p + 1) & 1], err, nullptr);
    GRS_HIP(hipGetLastError());
  }
  return GRS_OK;
}

// The largest LDS shape of the segmented top-byte sort, and the primary shape for segments of
// n / nseg keys on average: a uniform run holds m = n / nseg / 256 keys, +- sqrt(m) (as
// msd_local_shape); 0 when even the largest shape would leave most runs to the fallback.
template <typename K, bool PAIRS>
using SegMsdLargest = std::conditional_t<sizeof(K) + (PAIRS ? 4 : 0) <= 8, MsdLocalC, MsdLocalB>;
template <typename K, bool PAIRS>
int seg_msd_shape(size_t n, size_t nseg) {
  const double m = static_cast<double>(n) / static_cast<double>(nseg) / 256.0;
  const double need = m + 8.0 * std::sqrt(m) + 64.0;
  // no smaller shape than A: short runs merge into entries of up to the shape's capacity
  if (need <= MsdLocalA::SMAX) return 1;
  if (need <= MsdLocalB::SMAX) return 2;
  if (need <= SegMsdLargest<K, PAIRS>::SMAX) return 3;
  return 0;
}

template <typename K, bool PAIRS>
grs_status sort_segmented_msd_any(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, const uint32_t* d_offsets,
                                  uint32_t nseg, hipStream_t st) {
  using L = SegMsdLargest<K, PAIRS>;
  switch (seg_msd_shape<K, PAIRS>(n, nseg)) {
    case 1: return sort_segmented_msd<K, PAIRS, MsdLocalA, L>(s, keys, vals, n, d_offsets, nseg, st);
    case 2: return sort_segmented_msd<K, PAIRS, MsdLocalB, L>(s, keys, vals, n, d_offsets, nseg, st);
    case 3: return sort_segmented_msd<K, PAIRS, L, L>(s, keys, vals, n, d_offsets, nseg, st);
    default: return set_err(GRS_EINVAL, "internal: no segmented LDS shape");
  }
}

}  // namespace

extern "C" {

// grs_sort_segmented: below this average segment length (and past the LDS-sized segments) the
// composite-key sort instead of the segmented passes, which launch a workgroup per segment at
// least (tools/bench_seg_route.py, one 16M-key segment beside short ones, 2^24-2^25 keys in all:
// 1M x 4 keys 318 vs 1.4 ms, 16K x 1024 5.1 vs 1.6, 8K x 2048 2.7 vs 1.6, 4K x 4096 0.85 vs 1.6)
static constexpr size_t kSegRouteMinAvg = 4096;

grs_status grs_sort_segmented(grs_sorter* s, void* d_keys, uint32_t* d_vals, size_t n,
                              const uint32_t* d_offsets, int num_segments, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_sort_segmented: NULL sorter");
  if (!s->pairs)
    return set_err(GRS_EINVAL, "grs_sort_segmented: needs a sorter created with a payload");
  if (num_segments < 1 || !d_offsets)
    return set_err(GRS_EINVAL, "grs_sort_segmented: bad segments");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort_segmented: n exceeds capacity");
  if (n == 0) return GRS_OK;
  if (!d_keys) return set_err(GRS_EINVAL, "grs_sort_segmented: NULL keys");
  // short segments: one workgroup per segment in LDS, the block radix sort up to 16384 (u32
  // keys) / 8192 (u64 keys) items, or the bitonic fallback up to 4096 where the lane order of
  // LDS atomics is not relied on (the device probe failed, or GRS_OPT_RANK = 1).  Reading the
  // longest length back costs one stream synchronisation; it is skipped where the average
  // segment already exceeds the bound.
  const bool radix = s->rank_mode == 0;
  const uint32_t small_max = !radix ? GRS_SEG_SMALL_MAX
                             : s->key_type == GRS_KEY_U32 ? GRS_SEG_RADIX_MAX32 : GRS_SEG_RADIX_MAX64;
  if (static_cast<uint64_t>(num_segments) * small_max >= n) {
    int prev = 0;
    GRS_HIP(hipGetDevice(&prev));
    if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint32_t* dmax = s->ctrl + GRS_CTRL_ERROR + 4;
    grs_status r = GRS_OK;
    bool small = false;
    if (hipMemsetAsync(dmax, 0, 4, st) != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: memset");
    if (r == GRS_OK) {
      hipLaunchKernelGGL(grs::grs_segment_maxlen, dim3(std::min<size_t>(grid_for(num_segments, 256), 1024)),
                         dim3(256), 0, st, d_offsets, static_cast<uint32_t>(num_segments), dmax);
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(s->h_err, dmax, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        r = set_err(GRS_EHIP, "grs_sort_segmented: longest segment");
      else
        small = *s->h_err <= small_max;
    }
    if (r == GRS_OK && small) {
      const uint32_t longest = *s->h_err;
      auto go = [&](auto kt, auto smax, auto block) {
        using KT = decltype(kt);
        constexpr uint32_t SM = decltype(smax)::value, BL = decltype(block)::value;
        if constexpr (SM <= (sizeof(KT) == 4 ? GRS_SEG_RADIX_MAX32 : GRS_SEG_RADIX_MAX64)) {
          if (radix)
            hipLaunchKernelGGL((grs::grs_segment_radix<KT, SM, BL>), dim3(num_segments), dim3(BL),
                               0, st, static_cast<KT*>(d_keys), d_vals, d_offsets);
        }
        if constexpr (SM <= GRS_SEG_SMALL_MAX) {
          if (!radix)
            hipLaunchKernelGGL((grs::grs_segment_bitonic<KT, SM>), dim3(num_segments),
                               dim3(GRS_SEG_SMALL_BLOCK), 0, st, static_cast<KT*>(d_keys), d_vals,
                               d_offsets);
        }
      };
      using B256 = std::integral_constant<uint32_t, 256>;
      using B1024 = std::integral_constant<uint32_t, 1024>;
      auto pick = [&](auto kt) {
        if (longest <= 512) go(kt, std::integral_constant<uint32_t, 512>{}, B256{});
        else if (longest <= 1024) go(kt, std::integral_constant<uint32_t, 1024>{}, B256{});
        else if (longest <= 2048) go(kt, std::integral_constant<uint32_t, 2048>{}, B256{});
        else if (longest <= 4096) go(kt, std::integral_constant<uint32_t, 4096>{}, B256{});
        else if (longest <= 8192) go(kt, std::integral_constant<uint32_t, 8192>{}, B1024{});
        else go(kt, std::integral_constant<uint32_t, 16384>{}, B1024{});
      };
      if (s->key_type == GRS_KEY_U32) pick(uint32_t{});
      else pick(uint64_t{});
      if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
    }
    if (prev != s->device) (void)hipSetDevice(prev);
    if (r != GRS_OK || small) return r;
  }
  // atomic ranking, 8-bit digits: a few segments of 4M keys and more on average are sorted one
  // by one (each a whole sort: MSD or LSD); segments of 4K keys and more on average whose top-byte
  // runs fit LDS take the top-byte scatter + LDS sorts; anything else the segmented LSD
  const size_t avg = n / static_cast<size_t>(num_segments);
  // segmented passes launch a workgroup per segment at least (a segment shorter than a tile is a
  // solo tile), so very many short segments beside a long one take the composite-key sort
  // (kSegRouteMinAvg: tools/bench_seg_route.py)
  const bool seg_passes = s->seg_route == 1 || (s->seg_route == 0 && avg >= kSegRouteMinAvg);
  if (s->rank_mode == 0 && s->radix_bits == 8 && seg_passes && s->seg_route != 2 &&
      !(num_segments <= GRS_MAX_SPLITTERS + 1 && avg >= (size_t(1) << 22))) {
    int prev = 0;
    GRS_HIP(hipGetDevice(&prev));
    if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t n32 = static_cast<uint32_t>(n), ns = static_cast<uint32_t>(num_segments);
    const bool u32 = s->key_type == GRS_KEY_U32;
    auto go = [&](auto kt, auto pairs) -> grs_status {
      using KT = decltype(kt);
      constexpr bool PR = decltype(pairs)::value;
      KT* const k = static_cast<KT*>(d_keys);
      uint32_t* const v = PR ? d_vals : nullptr;
      if (s->msd_mode != 0 && avg >= 4096 && seg_msd_shape<KT, PR>(n, ns) != 0)
        return sort_segmented_msd_any<KT, PR>(s, k, v, n32, d_offsets, ns, st);
      return sort_segmented_seg<KT, PR>(s, k, v, n32, d_offsets, ns, st);
    };
    grs_status r;
    if (u32 && d_vals) r = go(uint32_t{}, std::true_type{});
    else if (u32) r = go(uint32_t{}, std::false_type{});
    else if (d_vals) r = go(uint64_t{}, std::true_type{});
    else r = go(uint64_t{}, std::false_type{});
    if (prev != s->device) (void)hipSetDevice(prev);
    return r;
  }
  if (num_segments <= GRS_MAX_SPLITTERS + 1)
    return sort_segmented_few(s, d_keys, d_vals, n, d_offsets, num_segments, stream);
  if (s->key_type == GRS_KEY_U32) return sort_segmented_u32(s, d_keys, d_vals, n, d_offsets,
                                                            num_segments, stream);
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool u64 = s->key_type == GRS_KEY_U64;
  const size_t kb = u64 ? 8 : 4;
  // perm | pos | vals_out | segment keys (reused for the gathered keys), 256-B aligned parts
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t need = 3 * al(n * 4) + al(n * kb);
  grs_status r = grow_buf(s, &s->seg_buf, &s->seg_bytes, need, "grs_sort_segmented: scratch");
  char* b = static_cast<char*>(s->seg_buf);
  uint32_t* perm = reinterpret_cast<uint32_t*>(b);
  uint32_t* pos = reinterpret_cast<uint32_t*>(b + al(n * 4));
  uint32_t* vout = reinterpret_cast<uint32_t*>(b + 2 * al(n * 4));
  void* segk = b + 3 * al(n * 4);
  int segbits = 1;
  while ((1ll << segbits) < num_segments) ++segbits;
  const int kbits = u64 ? 64 : 32;
  // 1. stable sort of the keys, carrying each key's input index
  if (r == GRS_OK) r = grs_iota_u32(perm, n, 0, stream);
  if (r == GRS_OK) r = grs_sort_bits(s, d_keys, perm, n, 0, kbits, stream);
  // 2. segment of each sorted element; 3. stable sort by segment (key order kept inside one)
  if (r == GRS_OK) {
    if (u64)
      hipLaunchKernelGGL(grs::grs_segment_ids<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                         perm, d_offsets, static_cast<uint32_t>(num_segments),
                         static_cast<uint64_t*>(segk), static_cast<uint64_t>(n));
    else
      hipLaunchKernelGGL(grs::grs_segment_ids<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                         perm, d_offsets, static_cast<uint32_t>(num_segments),
                         static_cast<uint32_t*>(segk), static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (r == GRS_OK) r = grs_iota_u32(pos, n, 0, stream);
  if (r == GRS_OK && num_segments > 1)
    r = grs_sort_bits(s, segk, pos, n, 0, std::min(segbits, kbits), stream);
  // 4. gather keys (into the segment-key buffer) and payload, then copy back
  if (r == GRS_OK) {
    if (u64)
      hipLaunchKernelGGL(grs::grs_segment_gather<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0,
                         st, static_cast<const uint64_t*>(d_keys), static_cast<uint64_t*>(segk),
                         pos, perm, d_vals, vout, static_cast<uint64_t>(n));
    else
      hipLaunchKernelGGL(grs::grs_segment_gather<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0,
                         st, static_cast<const uint32_t*>(d_keys), static_cast<uint32_t*>(segk),
                         pos, perm, d_vals, vout, static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (r == GRS_OK && hipMemcpyAsync(d_keys, segk, n * kb, hipMemcpyDeviceToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_segmented: copy");
  if (r == GRS_OK && d_vals &&
      hipMemcpyAsync(d_vals, vout, n * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_segmented: copy");
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_sort_host(grs_sorter* s, const void* h_keys_in, void* h_keys_out,
                         const uint32_t* h_vals_in, uint32_t* h_vals_out, size_t n, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_sort_host: NULL sorter");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort_host: n exceeds capacity");
  if (n == 0) return GRS_OK;
  if (!h_keys_in || !h_keys_out) return set_err(GRS_EINVAL, "grs_sort_host: NULL keys");
  if (s->pairs != (h_vals_in != nullptr) || (h_vals_in != nullptr) != (h_vals_out != nullptr))
    return set_err(GRS_EINVAL, "grs_sort_host: payload pointers must match the sorter");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  const size_t kbytes = (n * kb + 255) & ~static_cast<size_t>(255);
  const size_t need = kbytes + (s->pairs ? n * 4 : 0);
  grs_status r = grow_buf(s, &s->host_stage, &s->host_stage_bytes, need, "grs_sort_host: staging");
  char* dk = static_cast<char*>(s->host_stage);
  uint32_t* dv = s->pairs ? reinterpret_cast<uint32_t*>(dk + kbytes) : nullptr;
  if (r == GRS_OK && hipMemcpyAsync(dk, h_keys_in, n * kb, hipMemcpyHostToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_host: upload");
  if (r == GRS_OK && dv && hipMemcpyAsync(dv, h_vals_in, n * 4, hipMemcpyHostToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_host: upload");
  if (r == GRS_OK) r = grs_sort(s, dk, dv, n, stream);
  if (r == GRS_OK && hipMemcpyAsync(h_keys_out, dk, n * kb, hipMemcpyDeviceToHost, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_host: download");
  if (r == GRS_OK && dv && hipMemcpyAsync(h_vals_out, dv, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_host: download");
  if (r == GRS_OK && hipStreamSynchronize(st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_host: synchronize");
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

// ---------------------------------------------------------------------------------------
// multi-GPU key-range sort: grs_sort_sharded
// ---------------------------------------------------------------------------------------

int grs_shard_samples_per_rank(int nranks) {
  return nranks <= 0 ? 0 : std::min(1024, GRS_SHARD_SAMPLES_MAX / nranks);
}

}  // extern "C"

namespace {

#define GRS_RCCL(call)                                                                     \
  do {                                                                                     \
    ncclResult_t e_ = (call);                                                              \
    if (e_ != ncclSuccess)                                                                 \
      return set_err(GRS_ERCCL, std::string(#call) + ": " + ncclGetErrorString(e_));       \
  } while (0)

// Exchange plan from the G x G count matrix (row r: rank r's bucket sizes).
void shard_plan(const uint32_t* mat, int g, int me, uint64_t* soff, uint64_t* roff, uint64_t* n_out) {
  uint64_t so = 0, ro = 0;
  for (int p = 0; p < g; ++p) {
    soff[p] = so;
    so += mat[me * g + p];
    roff[p] = ro;
    ro += mat[p * g + me];
  }
  *n_out = ro;
}

template <typename K>
constexpr ncclDataType_t nccl_type() { return sizeof(K) == 4 ? ncclUint32 : ncclUint64; }

// Exchange timing of grs_sort_sharded (profiling on): event k of the call.
grs_status xmark(grs_sorter* s, int k, hipStream_t st) {
  if (s->ring > 0 && s->xev[k]) GRS_HIP(hipEventRecord(s->xev[k], st));
  return GRS_OK;
}

// Pinned words of grs_sort_sharded's host read-back: G rows of at most 2G + 3 words.
constexpr size_t kShardHostWords = 16 * (2 * 16 + 3) + 16;

// The agreement before an exchange.  Each rank appends three words to the row it all-gathers
// (its counts / sizes): its sticky error word and its receive capacity min(out_cap, capacity)
// as two words.  Every rank then reads every row and takes the SAME decision -- a timeout or a
// too-small receive side on any rank aborts all of them before any data moves (a rank that
// returned alone would leave its peers waiting in the grouped send / recv for ever).
grs_status append_verdict(grs_sorter* s, uint32_t* tail, size_t cap, hipStream_t st) {
  GRS_HIP(hipMemcpyAsync(tail, s->ctrl + GRS_CTRL_ERROR, 4, hipMemcpyDeviceToDevice, st));
  GRS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(tail + 1),
                            static_cast<int>(static_cast<uint32_t>(cap)), 1, st));
  GRS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(tail + 2),
                            static_cast<int>(static_cast<uint32_t>(static_cast<uint64_t>(cap) >> 32)), 1, st));
  return GRS_OK;
}

// rows: g rows of w words, the verdict in the last three; recv[r] = what rank r would receive.
// GRS_OK, or the status every rank returns (the sticky error word is cleared on a timeout).
grs_status read_verdict(grs_sorter* s, const uint32_t* rows, int g, int w, const uint64_t* recv,
                        int me, hipStream_t st) {
  bool err = false;
  int short_rank = -1;
  for (int r = 0; r < g; ++r) {
    const uint32_t* v = rows + static_cast<size_t>(r) * w + (w - 3);
    err |= v[0] != 0u;
    const uint64_t cap = v[1] | (static_cast<uint64_t>(v[2]) << 32);
    if (recv[r] > cap && (short_rank < 0 || r == me)) short_rank = r;
  }
  if (err) {
    GRS_HIP(hipMemsetAsync(s->ctrl + GRS_CTRL_ERROR, 0, 4, st));
    return set_err(GRS_ETIMEOUT, "grs_sort_sharded: a look-back spin exceeded its bound (on this "
                                 "rank or a peer; every rank aborts before the exchange)");
  }
  if (short_rank >= 0)
    return set_err(GRS_ECAPACITY, "grs_sort_sharded: the received run of rank " +
                                      std::to_string(short_rank) + " (" + std::to_string(recv[short_rank]) +
                                      " items) exceeds its out_capacity or sorter capacity");
  return GRS_OK;
}

template <typename K, bool PAIRS, int N>
grs_status run_sharded_n(grs_sorter* s, const K* keys, const uint32_t* vals, uint32_t n, K* out_k,
                         uint32_t* out_v, size_t out_cap, size_t* n_out, ncclComm_t comm, int g,
                         int me, hipStream_t st) {
  using Dig = grs::SplitterIdxDigit<K, N>;
  const uint32_t S = static_cast<uint32_t>(grs_shard_samples_per_rank(g));
  // scratch: sk[S] | sp[S] | ak[G*S] | ap[G*S] | cnt[16] | mat[G*G] | digit, 256-B aligned parts
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t gs = static_cast<size_t>(g) * S;
  const int W = g + 3;   // words per rank in the count all-gather: counts + verdict
  const size_t need = al(S * sizeof(K)) + al(S * 4) + al(gs * sizeof(K)) + al(gs * 4) + al(4 * W) +
                      al(static_cast<size_t>(g) * W * 4) + al(sizeof(Dig));
  {
    const grs_status r = grow_buf(s, &s->shard_buf, &s->shard_bytes, need, "grs_sort_sharded: scratch");
    if (r != GRS_OK) return r;
  }
  if (!s->shard_host && hipHostMalloc(reinterpret_cast<void**>(&s->shard_host), kShardHostWords * 4,
                                      hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(GRS_ENOMEM, "grs_sort_sharded: pinned allocation failed");
  }
  char* b = static_cast<char*>(s->shard_buf);
  K* sk = reinterpret_cast<K*>(b);                  b += al(S * sizeof(K));
  uint32_t* sp = reinterpret_cast<uint32_t*>(b);     b += al(S * 4);
  K* ak = reinterpret_cast<K*>(b);                   b += al(gs * sizeof(K));
  uint32_t* ap = reinterpret_cast<uint32_t*>(b);     b += al(gs * 4);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(b);    b += al(4 * W);
  uint32_t* mat = reinterpret_cast<uint32_t*>(b);    b += al(static_cast<size_t>(g) * W * 4);
  Dig* dig = reinterpret_cast<Dig*>(b);

  if (xmark(s, 0, st) != GRS_OK) return GRS_EHIP;
  // 1-2. samples, all-gathered (rank-major)
  hipLaunchKernelGGL((grs::grs_shard_samples<K>), dim3((S + 255) / 256), dim3(256), 0, st, keys, n,
                     S, sk, sp);
  GRS_HIP(hipGetLastError());
  GRS_RCCL(ncclGroupStart());
  GRS_RCCL(ncclAllGather(sk, ak, S, nccl_type<K>(), comm, st));
  GRS_RCCL(ncclAllGather(sp, ap, S, ncclUint32, comm, st));
  GRS_RCCL(ncclGroupEnd());
  // 3. this rank's partition digit, on the device
  hipLaunchKernelGGL((grs::grs_shard_splitters<K, N>), dim3(1), dim3(1024), 0, st, ak, ap,
                     static_cast<uint32_t>(g), S, static_cast<uint32_t>(me), dig);
  GRS_HIP(hipGetLastError());
  // 4. partition into the send buffer: G regions of `region` items (bucket b at b * region), so
  //    no bucket histogram pass is needed (grs_partition's region mode).  region is the even
  //    share plus 25 % and 64K items of slack (a balanced bucket fits: the splitters are
  //    quantiles with ties broken by index); the buffer holds (G - 1) regions + n items, so even
  //    a last bucket of all n items stays inside it.  A bucket larger than its region spills
  //    into the next region: the count matrix shows it at the host synchronisation, and the
  //    partition is then redone with a bucket histogram into contiguous buckets in the sorter's
  //    ping-pong scratch (free until step 8) -- the counts, and so the exchange plan, are the
  //    same.  Contiguous buckets are also the path when G * region reaches 2^32.
  //    (GRS_OPT_SHARDED_SEND = 2, a test hook: regions of n / (2G), so that full buckets spill
  //    and the redo path runs even on one rank)
  //    Every rank computes every rank's region from that rank's n (its row sum of the count
  //    matrix), so all of them know whether any rank spilled (the options must agree).
  auto region_of = [&](uint64_t nr) -> uint32_t {
    return nr == 0 ? 0u
         : s->sharded_send == 2
             ? std::max<uint32_t>(1u, static_cast<uint32_t>(nr / (2u * static_cast<uint32_t>(g))))
             : static_cast<uint32_t>(std::min<uint64_t>(nr, nr * 5 / 4 / g + 65536));
  };
  auto regions_of = [&](uint64_t nr) {
    return nr > 0 && static_cast<uint64_t>(g) * region_of(nr) < (1ull << 32) && s->sharded_send != 1;
  };
  const uint32_t region = region_of(n);
  bool regions = regions_of(n);
  K* send_k = static_cast<K*>(s->alt_keys);
  uint32_t* send_v = s->alt_vals;
  const size_t xitems = static_cast<size_t>(g - 1) * region + n;   // region-mode buffer items
  if (regions) {
    const size_t need = xitems * (sizeof(K) + (PAIRS ? 4 : 0));
    const grs_status rx = grow_buf(s, &s->xbuf, &s->xbuf_bytes, need, "grs_sort_sharded: send buffer");
    if (rx != GRS_OK) return rx;
    send_k = static_cast<K*>(s->xbuf);
    send_v = PAIRS ? reinterpret_cast<uint32_t*>(send_k + xitems) : nullptr;
  }
  if (n > 0) {
    const grs_status r = run_partition_n<K, PAIRS, N>(s, keys, vals, send_k, send_v, n, Dig{}, dig,
                                                      g - 1, cnt, st, regions ? region : 0u);
    if (r != GRS_OK) return r;
  } else {
    GRS_HIP(hipMemsetAsync(cnt, 0, static_cast<size_t>(g) * 4, st));
  }
  // 5-6. count matrix + every rank's verdict to every rank, then the one host synchronisation
  if (append_verdict(s, cnt + g, std::min<size_t>(out_cap, s->capacity), st) != GRS_OK) return GRS_EHIP;
  GRS_RCCL(ncclAllGather(cnt, mat, W, ncclUint32, comm, st));
  GRS_HIP(hipMemcpyAsync(s->shard_host, mat, static_cast<size_t>(g) * W * 4, hipMemcpyDeviceToHost, st));
  GRS_HIP(hipStreamSynchronize(st));
  uint32_t* const h = s->shard_host;
  uint64_t recv_tot[16] = {};
  for (int r = 0; r < g; ++r)
    for (int p = 0; p < g; ++p) recv_tot[p] += h[static_cast<size_t>(r) * W + p];
  {
    const grs_status v = read_verdict(s, h, g, W, recv_tot, me, st);
    if (v != GRS_OK) return v;
  }
  // the verdict words read, compact the rows into the G x G count matrix (row r moves down)
  for (int r = 0; r < g; ++r)
    for (int p = 0; p < g; ++p) h[r * g + p] = h[static_cast<size_t>(r) * W + p];
  uint64_t soff[16], roff[16], total = 0;
  shard_plan(h, g, me, soff, roff, &total);
  bool spilled = false, spilled_any = false;
  for (int r = 0; r < g; ++r) {
    uint64_t nr = 0;
    for (int p = 0; p < g; ++p) nr += h[r * g + p];
    bool sp = false;
    for (int p = 0; regions_of(nr) && p < g; ++p) sp |= h[r * g + p] > region_of(nr);
    spilled_any |= sp;
    if (r == me) spilled = sp;
  }
  if (spilled) {   // a bucket outgrew its region: contiguous buckets instead (same counts)
    s->x_region_redo++;
    regions = false;
    send_k = static_cast<K*>(s->alt_keys);
    send_v = s->alt_vals;
    const grs_status r = run_partition_n<K, PAIRS, N>(s, keys, vals, send_k, send_v, n, Dig{}, dig,
                                                      g - 1, cnt, st, 0u);
    if (r != GRS_OK) return r;
  }
  if (spilled_any) {
    // the redone partitions' look-backs must not have timed out before their buckets are sent:
    // every rank all-gathers its error word once more (this rare path only) and all decide alike
    GRS_HIP(hipMemcpyAsync(cnt, s->ctrl + GRS_CTRL_ERROR, 4, hipMemcpyDeviceToDevice, st));
    GRS_RCCL(ncclAllGather(cnt, mat, 1, ncclUint32, comm, st));
    GRS_HIP(hipMemcpyAsync(h + g * g, mat, static_cast<size_t>(g) * 4, hipMemcpyDeviceToHost, st));
    GRS_HIP(hipStreamSynchronize(st));
    bool err = false;
    for (int r = 0; r < g; ++r) err |= h[g * g + r] != 0u;
    if (err) {
      GRS_HIP(hipMemsetAsync(s->ctrl + GRS_CTRL_ERROR, 0, 4, st));
      return set_err(GRS_ETIMEOUT, "grs_sort_sharded: a partition look-back spin exceeded its bound "
                                   "(on this rank or a peer)");
    }
  }
  if (regions)
    for (int p = 0; p < g; ++p) soff[p] = static_cast<uint64_t>(p) * region;
  // 7. exchange: keys and payload in one group; the self part is a device copy
  if (xmark(s, 1, st) != GRS_OK) return GRS_EHIP;
  GRS_RCCL(ncclGroupStart());
  for (int p = 0; p < g; ++p) {
    if (p == me) continue;
    const size_t sc = s->shard_host[me * g + p], rc = s->shard_host[p * g + me];
    if (sc) GRS_RCCL(ncclSend(send_k + soff[p], sc, nccl_type<K>(), p, comm, st));
    if (rc) GRS_RCCL(ncclRecv(out_k + roff[p], rc, nccl_type<K>(), p, comm, st));
    if (PAIRS && sc) GRS_RCCL(ncclSend(send_v + soff[p], sc, ncclUint32, p, comm, st));
    if (PAIRS && rc) GRS_RCCL(ncclRecv(out_v + roff[p], rc, ncclUint32, p, comm, st));
  }
  GRS_RCCL(ncclGroupEnd());
  const size_t self = s->shard_host[me * g + me];
  if (self) {
    GRS_HIP(hipMemcpyAsync(out_k + roff[me], send_k + soff[me], self * sizeof(K),
                           hipMemcpyDeviceToDevice, st));
    if (PAIRS)
      GRS_HIP(hipMemcpyAsync(out_v + roff[me], send_v + soff[me], self * 4,
                             hipMemcpyDeviceToDevice, st));
  }
  if (xmark(s, 2, st) != GRS_OK) return GRS_EHIP;
  *n_out = static_cast<size_t>(total);
  // 8. local stable sort of the received run (source-rank order = global order for ties)
  const grs_status rs = grs_sort(s, out_k, out_v, static_cast<size_t>(total), st);
  if (rs != GRS_OK || xmark(s, 3, st) != GRS_OK) return rs != GRS_OK ? rs : GRS_EHIP;
  uint64_t sent = 0, recvd = 0;
  for (int p = 0; p < g; ++p) {
    if (p == me) continue;
    sent += s->shard_host[me * g + p];
    recvd += s->shard_host[p * g + me];
  }
  const uint64_t ib = sizeof(K) + (PAIRS ? 4 : 0);
  s->xev_recorded = s->ring > 0;
  s->x_sent = sent * ib;
  s->x_recv = recvd * ib;
  s->x_presorted = 0;
  return GRS_OK;
}

// ---- presorted exchange (grs_codec.hpp): sort, encode the buckets, exchange, decode, merge --


size_t codec_blocks_max(size_t n, int g) { return n / grs::kCodecBlock + static_cast<size_t>(g); }

// Codec scratch: plan[2G+2] | sizes[2G] | blk_words[nb+1] | blk_woff[nb+1] | blk_meta[2nb] |
// scan scratch | co-ranks of the merge rounds
struct CodecScratch {
  uint32_t *plan, *sizes, *blk_words, *blk_woff, *blk_meta, *corank;
  void* scan;
  size_t scan_bytes;
};

grs_status codec_scratch(grs_sorter* s, size_t n_enc, size_t n_merge, int g, CodecScratch* cs) {
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t nb = codec_blocks_max(n_enc, g);
  const size_t scan = grs_scan_scratch_bytes(nb + 1);
  // co-ranks: the 2-way rounds' boundaries, or the k-way merge's samples + (tiles + 1) rows
  const size_t ns = n_merge / grs::kMkSpacing + grs::kMaxRanks + 1;
  const size_t cor = std::max(n_merge / grs::kMergeTile + 2 * grs::kMaxRanks + 2,
                              ns + 64 + (ns / grs::kMkSPT + 2) * grs::kMkStride);
  const size_t need = al(4 * (2 * g + 2)) + al(4 * 2 * g) + 2 * al(4 * (nb + 1)) + al(8 * nb) +
                      al(scan) + al(4 * cor);
  const grs_status r = grow_buf(s, &s->codec_buf, &s->codec_bytes, need, "presorted exchange scratch");
  if (r != GRS_OK) return r;
  char* b = static_cast<char*>(s->codec_buf);
  cs->plan = reinterpret_cast<uint32_t*>(b);      b += al(4 * (2 * g + 2));
  cs->sizes = reinterpret_cast<uint32_t*>(b);     b += al(4 * 2 * g);
  cs->blk_words = reinterpret_cast<uint32_t*>(b); b += al(4 * (nb + 1));
  cs->blk_woff = reinterpret_cast<uint32_t*>(b);  b += al(4 * (nb + 1));
  cs->blk_meta = reinterpret_cast<uint32_t*>(b);  b += al(8 * nb);
  cs->scan = b;                                   b += al(scan);
  cs->scan_bytes = scan;
  cs->corank = reinterpret_cast<uint32_t*>(b);
  return GRS_OK;
}

// Encode the buckets of a sorted shard (u32 keys) split by the device partition digit `dig`:
// d_send gets bucket 0's [directory][data], then bucket 1's, ...; cs.sizes[2b] / [2b+1] the
// keys / words of bucket b (device).
template <int N>
grs_status codec_encode(grs_sorter* s, const uint32_t* sorted, uint32_t n,
                        const grs::SplitterIdxDigit<uint32_t, N>* dig, int g, uint32_t* send,
                        const CodecScratch& cs, hipStream_t st) {
  hipLaunchKernelGGL((grs::grs_shard_bounds<uint32_t, N>), dim3(1), dim3(64), 0, st, sorted, n, dig,
                     static_cast<uint32_t>(g), cs.plan);
  GRS_HIP(hipGetLastError());
  const uint32_t nb = static_cast<uint32_t>(codec_blocks_max(n, g));
  const dim3 grid((nb + 4 * grs::kCodecBPW - 1) / (4 * grs::kCodecBPW));   // 4 waves per workgroup
  hipLaunchKernelGGL(grs::grs_codec_sizes, grid, dim3(256), 0, st, sorted, cs.plan,
                     static_cast<uint32_t>(g), nb, cs.blk_words, cs.blk_meta);
  GRS_HIP(hipGetLastError());
  GRS_HIP(hipMemsetAsync(cs.blk_words + nb, 0, 4, st));
  grs_status r = scan_u32_impl(cs.blk_words, cs.blk_woff, nb + 1, nullptr, cs.scan, cs.scan_bytes,
                               st, s->ctrl + GRS_CTRL_ERROR);
  if (r != GRS_OK) return r;
  hipLaunchKernelGGL(grs::grs_codec_pack, grid, dim3(256), 0, st, sorted, cs.plan,
                     static_cast<uint32_t>(g), nb, cs.blk_meta, cs.blk_woff, send, cs.sizes);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

// Decode the received runs (source p: lens[p] keys encoded at word_off[p] of d_recv) and merge
// them, in source order for ties, into out (n_total keys).  Scratch: the sorter's ping-pong
// buffer (capacity >= n_total).
grs_status codec_decode_merge(grs_sorter* s, const uint32_t* recv, int g, const uint64_t* word_off,
                              const uint32_t* lens, uint32_t* out, uint64_t n_total,
                              const CodecScratch& cs, hipStream_t st) {
  grs::CodecSources src{};
  src.g = static_cast<uint32_t>(g);
  uint32_t blocks = 0, run = 0;
  for (int p = 0; p < g; ++p) {
    src.blk_base[p] = blocks;
    src.len[p] = lens[p];
    src.run_off[p] = run;
    src.word_off[p] = word_off[p];
    blocks += (lens[p] + grs::kCodecBlock - 1) / grs::kCodecBlock;
    run += lens[p];
  }
  src.blk_base[g] = blocks;
  int rounds = 0;
  for (int k = g; k > 1; k = (k + 1) / 2) ++rounds;
  const bool kway = s->merge_mode == 1;
  if (kway) rounds = g > 1 ? 1 : 0;
  uint32_t* alt = static_cast<uint32_t*>(s->alt_keys);
  uint32_t* in = (rounds & 1) ? alt : out;   // the last round writes out
  uint32_t* o = (rounds & 1) ? out : alt;
  if (blocks > 0) {
    hipLaunchKernelGGL(grs::grs_codec_unpack, dim3((blocks + 4 * grs::kCodecBPW - 1) / (4 * grs::kCodecBPW)),
                       dim3(256), 0, st, recv, src, in);
    GRS_HIP(hipGetLastError());
  }
  if (kway) {
    if (g <= 1 || n_total == 0) return GRS_OK;
    grs::MergeK mk{};
    mk.k = static_cast<uint32_t>(g);
    mk.kp = 1;
    while (mk.kp < mk.k) mk.kp <<= 1;
    uint32_t ns = 0;
    for (int p = 0; p < g; ++p) {
      mk.off[p] = src.run_off[p];
      mk.sbase[p] = ns;
      ns += (lens[p] + grs::kMkSpacing - 1) / grs::kMkSpacing;
    }
    mk.off[g] = static_cast<uint32_t>(n_total);
    mk.sbase[g] = ns;
    uint32_t* samp = cs.corank;
    uint32_t* cor = cs.corank + ((ns + 63u) & ~63u);
    hipLaunchKernelGGL(grs::grs_mergek_samples, dim3((ns + 255) / 256), dim3(256), 0, st, in, mk, samp);
    GRS_HIP(hipGetLastError());
    const uint64_t threads = static_cast<uint64_t>(ns + 1) * mk.kp;
    hipLaunchKernelGGL(grs::grs_mergek_bounds, dim3(static_cast<uint32_t>((threads + 255) / 256)), dim3(256),
                       0, st, in, mk, samp, cor);
    GRS_HIP(hipGetLastError());
    hipLaunchKernelGGL(grs::grs_mergek_tiles, dim3(grs::mk_tiles(mk)), dim3(grs::kMkBlock), 0, st, in, o,
                       mk, cor);
    GRS_HIP(hipGetLastError());
    return GRS_OK;
  }
  uint32_t off[grs::kMaxRanks + 2];
  for (int p = 0; p < g; ++p) off[p] = src.run_off[p];
  off[g] = static_cast<uint32_t>(n_total);
  for (int k = g; k > 1;) {
    grs::MergeRound mr{};
    mr.pairs = static_cast<uint32_t>((k + 1) / 2);
    off[k + 1] = off[k];   // an odd last run merges with an empty one
    uint32_t bnd = 0;
    for (uint32_t i = 0; i < mr.pairs; ++i) {
      mr.bbase[i] = bnd;
      const uint32_t len = off[2 * i + 2] - off[2 * i];
      bnd += (len + grs::kMergeTile - 1) / grs::kMergeTile + 1;
    }
    mr.bbase[mr.pairs] = bnd;
    for (uint32_t i = 0; i <= 2 * mr.pairs; ++i) mr.off[i] = off[i];
    hipLaunchKernelGGL(grs::grs_merge_corank, dim3((bnd + 255) / 256), dim3(256), 0, st, in, mr,
                       cs.corank);
    GRS_HIP(hipGetLastError());
    const uint32_t tiles = bnd - mr.pairs;
    if (tiles > 0) {
      hipLaunchKernelGGL(grs::grs_merge_tiles, dim3(tiles), dim3(256), 0, st, in, o, mr, cs.corank);
      GRS_HIP(hipGetLastError());
    }
    for (uint32_t i = 0; i < mr.pairs; ++i) off[i] = off[2 * i];
    off[mr.pairs] = static_cast<uint32_t>(n_total);
    k = static_cast<int>(mr.pairs);
    std::swap(in, o);
  }
  return GRS_OK;
}

// grs_sort_sharded, presorted exchange (u32 keys, no payload): local sort into out_k, samples
// of the sorted shard, splitters, bounds + encode, the count / size matrix (the one host
// synchronisation), one send / recv of encoded words per peer, decode + merge into out_k.
template <int N>
grs_status run_sharded_presorted(grs_sorter* s, const uint32_t* keys, uint32_t n, uint32_t* out_k,
                                 size_t out_cap, size_t* n_out, ncclComm_t comm, int g, int me,
                                 hipStream_t st) {
  using Dig = grs::SplitterIdxDigit<uint32_t, N>;
  const uint32_t S = static_cast<uint32_t>(grs_shard_samples_per_rank(g));
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t gs = static_cast<size_t>(g) * S;
  const int W = 2 * g + 3;   // words per rank in the size all-gather: (keys, words) + verdict
  const size_t need = al(S * 4) + al(S * 4) + al(gs * 4) + al(gs * 4) + al(4 * static_cast<size_t>(g) * W) +
                      al(4 * W) + al(sizeof(Dig));
  grs_status r = grow_buf(s, &s->shard_buf, &s->shard_bytes, need, "grs_sort_sharded: scratch");
  if (r != GRS_OK) return r;
  if (!s->shard_host && hipHostMalloc(reinterpret_cast<void**>(&s->shard_host), kShardHostWords * 4,
                                      hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(GRS_ENOMEM, "grs_sort_sharded: pinned allocation failed");
  }
  char* b = static_cast<char*>(s->shard_buf);
  uint32_t* sk = reinterpret_cast<uint32_t*>(b);  b += al(S * 4);
  uint32_t* sp = reinterpret_cast<uint32_t*>(b);  b += al(S * 4);
  uint32_t* ak = reinterpret_cast<uint32_t*>(b);  b += al(gs * 4);
  uint32_t* ap = reinterpret_cast<uint32_t*>(b);  b += al(gs * 4);
  uint32_t* mat = reinterpret_cast<uint32_t*>(b); b += al(4 * static_cast<size_t>(g) * W);
  uint32_t* row = reinterpret_cast<uint32_t*>(b); b += al(4 * W);
  Dig* dig = reinterpret_cast<Dig*>(b);
  CodecScratch cs;
  if ((r = codec_scratch(s, n, s->capacity, g, &cs)) != GRS_OK) return r;
  const size_t send_words = n + grs::kCodecDir * codec_blocks_max(n, g);
  if ((r = grow_buf(s, &s->xbuf, &s->xbuf_bytes, 4 * send_words, "grs_sort_sharded: send buffer")) != GRS_OK)
    return r;
  uint32_t* send = static_cast<uint32_t*>(s->xbuf);

  if ((r = xmark(s, 0, st)) != GRS_OK) return r;
  // 1. local sort, out of place: the sorted shard lands in out_k
  if (n > 0) {
    r = use_msd(s, n, 0, 32) ? run_sort_msd<uint32_t, false>(s, out_k, nullptr, n, st, keys)
                             : run_sort<uint32_t, false, 8>(s, out_k, nullptr, n, 0, 32, st, keys);
    if (r != GRS_OK) return r;
  }
  // 2-3. samples of the sorted shard (rank-major gather), splitters on the device
  hipLaunchKernelGGL((grs::grs_shard_samples<uint32_t>), dim3((S + 255) / 256), dim3(256), 0, st,
                     out_k, n, S, sk, sp);
  GRS_HIP(hipGetLastError());
  GRS_RCCL(ncclGroupStart());
  GRS_RCCL(ncclAllGather(sk, ak, S, ncclUint32, comm, st));
  GRS_RCCL(ncclAllGather(sp, ap, S, ncclUint32, comm, st));
  GRS_RCCL(ncclGroupEnd());
  hipLaunchKernelGGL((grs::grs_shard_splitters_sorted<uint32_t, N>), dim3(1), dim3(1024), 0, st, ak, ap,
                     static_cast<uint32_t>(g), S, static_cast<uint32_t>(me), dig);
  GRS_HIP(hipGetLastError());
  // 4. bounds + encode
  if ((r = codec_encode<N>(s, out_k, n, dig, g, send, cs, st)) != GRS_OK) return r;
  // 5. (keys, words) of every bucket of every rank + every rank's verdict, then the one host
  //    synchronisation
  GRS_HIP(hipMemcpyAsync(row, cs.sizes, 4 * 2 * static_cast<size_t>(g), hipMemcpyDeviceToDevice, st));
  if ((r = append_verdict(s, row + 2 * g, std::min<size_t>(out_cap, s->capacity), st)) != GRS_OK) return r;
  GRS_RCCL(ncclAllGather(row, mat, W, ncclUint32, comm, st));
  GRS_HIP(hipMemcpyAsync(s->shard_host, mat, 4 * static_cast<size_t>(g) * W, hipMemcpyDeviceToHost, st));
  GRS_HIP(hipStreamSynchronize(st));
  uint32_t* const h = s->shard_host;
  {
    uint64_t recv_tot[grs::kMaxRanks] = {};
    for (int q = 0; q < g; ++q)
      for (int p = 0; p < g; ++p) recv_tot[p] += h[static_cast<size_t>(q) * W + 2 * p];
    if ((r = read_verdict(s, h, g, W, recv_tot, me, st)) != GRS_OK) return r;
  }
  // compact the rows into the G x 2G matrix
  for (int q = 0; q < g; ++q)
    for (int p = 0; p < 2 * g; ++p) h[q * 2 * g + p] = h[static_cast<size_t>(q) * W + p];
  uint64_t soff[grs::kMaxRanks], roff[grs::kMaxRanks], total = 0, so = 0, ro = 0;
  uint32_t lens[grs::kMaxRanks];
  for (int p = 0; p < g; ++p) {
    soff[p] = so;
    so += h[me * 2 * g + 2 * p + 1];
    roff[p] = ro;
    ro += h[p * 2 * g + 2 * me + 1];
    lens[p] = h[p * 2 * g + 2 * me];
    total += lens[p];
  }
  if ((r = grow_buf(s, &s->xrbuf, &s->xrbuf_bytes, std::max<size_t>(4 * ro, 4), "grs_sort_sharded: receive buffer")) != GRS_OK)
    return r;
  uint32_t* recv = static_cast<uint32_t*>(s->xrbuf);
  // 6. exchange of encoded words; the self part is a device copy
  if ((r = xmark(s, 1, st)) != GRS_OK) return r;
  GRS_RCCL(ncclGroupStart());
  for (int p = 0; p < g; ++p) {
    if (p == me) continue;
    const size_t sc = h[me * 2 * g + 2 * p + 1], rc = h[p * 2 * g + 2 * me + 1];
    if (sc) GRS_RCCL(ncclSend(send + soff[p], sc, ncclUint32, p, comm, st));
    if (rc) GRS_RCCL(ncclRecv(recv + roff[p], rc, ncclUint32, p, comm, st));
  }
  GRS_RCCL(ncclGroupEnd());
  const size_t self = h[me * 2 * g + 2 * me + 1];
  if (self)
    GRS_HIP(hipMemcpyAsync(recv + roff[me], send + soff[me], 4 * self, hipMemcpyDeviceToDevice, st));
  if ((r = xmark(s, 2, st)) != GRS_OK) return r;
  // 7. decode + merge into out_k
  if ((r = codec_decode_merge(s, recv, g, roff, lens, out_k, total, cs, st)) != GRS_OK) return r;
  if ((r = xmark(s, 3, st)) != GRS_OK) return r;
  s->xev_recorded = s->ring > 0;
  s->x_sent = 4 * (so - h[me * 2 * g + 2 * me + 1]);
  s->x_recv = 4 * (ro - h[me * 2 * g + 2 * me + 1]);
  s->x_presorted = 1;
  *n_out = static_cast<size_t>(total);
  return GRS_OK;
}

// grs_sort_sharded, chunked partition-first exchange (GRS_OPT_EXCHANGE = 3; keys without
// payload: the received runs are laid out chunk-major, so equal keys from different sources
// interleave, which only a payload could tell).  The partition of chunk c + 1 runs on the
// caller's stream while chunk c crosses the links from a second stream that carries every RCCL
// call of the exchange:
//   stream st:  samples, all-gather, splitters, chunk digits | partition chunk 0, 1, ..., C-1
//   stream X:   per chunk c: wait for partition c; all-gather its count rows (+ verdict);
//               copy them to the host; [host: the chunk's plan]; grouped send / recv of chunk c
//   then st waits for X and sorts the received run.
// A timeout or a receive side too small on any rank stops every rank at the same chunk (each
// reads every rank's rows of every chunk), before that chunk moves.  C (GRS_OPT_X_CHUNKS) must
// be the same on every rank.
template <typename K, int N>
grs_status run_sharded_chunked(grs_sorter* s, const K* keys, uint32_t n, K* out_k, size_t out_cap,
                               size_t* n_out, ncclComm_t comm, int g, int me, hipStream_t st) {
  using Dig = grs::SplitterIdxDigit<K, N>;
  const int C = s->x_chunks > 0 ? s->x_chunks : 4;
  const uint32_t S = static_cast<uint32_t>(grs_shard_samples_per_rank(g));
  const uint32_t chunk = (n + static_cast<uint32_t>(C) - 1) / static_cast<uint32_t>(C);
  const int W = g + 3;   // words per rank in a chunk's count all-gather: counts + verdict
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  const size_t gs = static_cast<size_t>(g) * S;
  // scratch: sk[S] | sp[S] | ak[G*S] | ap[G*S] | rows[C][W] | mats[C][G*W] | dig | digs[C]
  const size_t need = al(S * sizeof(K)) + al(S * 4) + al(gs * sizeof(K)) + al(gs * 4) +
                      al(static_cast<size_t>(C) * W * 4) + al(static_cast<size_t>(C) * g * W * 4) + al(sizeof(Dig)) +
                      al(static_cast<size_t>(C) * sizeof(Dig));
  grs_status r = grow_buf(s, &s->shard_buf, &s->shard_bytes, need, "grs_sort_sharded: scratch");
  if (r != GRS_OK) return r;
  if (!s->xstream) GRS_HIP(hipStreamCreateWithFlags(&s->xstream, hipStreamNonBlocking));
  for (int c = 0; c <= 16; ++c)
    if (!s->xcev[c]) GRS_HIP(hipEventCreateWithFlags(&s->xcev[c], hipEventDisableTiming));
  if (!s->xhev) GRS_HIP(hipEventCreateWithFlags(&s->xhev, hipEventDisableTiming));
  if (!s->xchunk_host && hipHostMalloc(reinterpret_cast<void**>(&s->xchunk_host), 16 * 19 * 4,
                                       hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(GRS_ENOMEM, "grs_sort_sharded: pinned allocation failed");
  }
  char* b = static_cast<char*>(s->shard_buf);
  K* sk = reinterpret_cast<K*>(b);                  b += al(S * sizeof(K));
  uint32_t* sp = reinterpret_cast<uint32_t*>(b);     b += al(S * 4);
  K* ak = reinterpret_cast<K*>(b);                   b += al(gs * sizeof(K));
  uint32_t* ap = reinterpret_cast<uint32_t*>(b);     b += al(gs * 4);
  uint32_t* rows = reinterpret_cast<uint32_t*>(b);   b += al(static_cast<size_t>(C) * W * 4);
  uint32_t* mats = reinterpret_cast<uint32_t*>(b);   b += al(static_cast<size_t>(C) * g * W * 4);
  Dig* dig = reinterpret_cast<Dig*>(b);              b += al(sizeof(Dig));
  Dig* digs = reinterpret_cast<Dig*>(b);
  hipStream_t X = s->xstream;
  K* send = static_cast<K*>(s->alt_keys);   // chunk c's buckets, contiguous from c * chunk
  const size_t cap = std::min<size_t>(out_cap, s->capacity);

  if (xmark(s, 0, st) != GRS_OK) return GRS_EHIP;
  // 1-3. samples, all-gathered; splitters; the chunks' digits
  hipLaunchKernelGGL((grs::grs_shard_samples<K>), dim3((S + 255) / 256), dim3(256), 0, st, keys, n, S, sk, sp);
  GRS_HIP(hipGetLastError());
  GRS_RCCL(ncclGroupStart());
  GRS_RCCL(ncclAllGather(sk, ak, S, nccl_type<K>(), comm, st));
  GRS_RCCL(ncclAllGather(sp, ap, S, ncclUint32, comm, st));
  GRS_RCCL(ncclGroupEnd());
  hipLaunchKernelGGL((grs::grs_shard_splitters<K, N>), dim3(1), dim3(1024), 0, st, ak, ap,
                     static_cast<uint32_t>(g), S, static_cast<uint32_t>(me), dig);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL((grs::grs_shard_chunk_digits<K, N>), dim3((C * GRS_MAX_SPLITTERS + 255) / 256), dim3(256), 0,
                     st, dig, static_cast<uint32_t>(C), chunk, digs);
  GRS_HIP(hipGetLastError());
  // 4. every chunk's partition on st, each followed by its verdict words and an event
  for (int c = 0; c < C; ++c) {
    const uint32_t c0 = std::min<uint32_t>(n, static_cast<uint32_t>(c) * chunk);
    const uint32_t cn = std::min<uint32_t>(n - c0, chunk);
    uint32_t* row = rows + static_cast<size_t>(c) * W;
    if (cn > 0) {
      r = run_partition_n<K, false, N>(s, keys + c0, nullptr, send + c0, nullptr, cn, Dig{}, digs + c, g - 1, row,
                                       st, 0u);
      if (r != GRS_OK) return r;
    } else {
      GRS_HIP(hipMemsetAsync(row, 0, static_cast<size_t>(g) * 4, st));
    }
    if (append_verdict(s, row + g, cap, st) != GRS_OK) return GRS_EHIP;
    GRS_HIP(hipEventRecord(s->xcev[c], st));
  }
  // 5. per chunk on X: count rows, the one host read of the chunk, its send / recv group
  GRS_HIP(hipStreamWaitEvent(X, s->xcev[0], 0));   // (the samples' all-gather precedes it on st)
  uint64_t recv_base = 0, recv_so_far[16] = {}, sent = 0, recvd = 0;
  uint64_t soff[16], roff[16];
  for (int c = 0; c < C; ++c) {
    GRS_HIP(hipStreamWaitEvent(X, s->xcev[c], 0));
    uint32_t* mat = mats + static_cast<size_t>(c) * g * W;
    GRS_RCCL(ncclAllGather(rows + static_cast<size_t>(c) * W, mat, W, ncclUint32, comm, X));
    GRS_HIP(hipMemcpyAsync(s->xchunk_host, mat, static_cast<size_t>(g) * W * 4, hipMemcpyDeviceToHost, X));
    GRS_HIP(hipEventRecord(s->xhev, X));
    GRS_HIP(hipEventSynchronize(s->xhev));
    uint32_t* h = s->xchunk_host;
    // every rank's cumulative receive after this chunk, for the verdict
    uint64_t recv_tot[16] = {};
    for (int q = 0; q < g; ++q) {
      for (int p = 0; p < g; ++p) recv_so_far[p] += h[static_cast<size_t>(q) * W + p];
    }
    for (int p = 0; p < g; ++p) recv_tot[p] = recv_so_far[p];
    if ((r = read_verdict(s, h, g, W, recv_tot, me, st)) != GRS_OK) return r;
    for (int q = 0; q < g; ++q)
      for (int p = 0; p < g; ++p) h[q * g + p] = h[static_cast<size_t>(q) * W + p];
    const uint32_t c0 = std::min<uint32_t>(n, static_cast<uint32_t>(c) * chunk);
    const uint64_t got = grs::shard_chunk_plan(h, g, me, c0, recv_base, soff, roff);
    if (c == 0 && xmark(s, 1, X) != GRS_OK) return GRS_EHIP;
    GRS_RCCL(ncclGroupStart());
    for (int p = 0; p < g; ++p) {
      if (p == me) continue;
      const size_t sc = h[me * g + p], rc = h[p * g + me];
      if (sc) GRS_RCCL(ncclSend(send + soff[p], sc, nccl_type<K>(), p, comm, X));
      if (rc) GRS_RCCL(ncclRecv(out_k + roff[p], rc, nccl_type<K>(), p, comm, X));
      sent += sc;
      recvd += rc;
    }
    GRS_RCCL(ncclGroupEnd());
    const size_t self = h[me * g + me];
    if (self)
      GRS_HIP(hipMemcpyAsync(out_k + roff[me], send + soff[me], self * sizeof(K), hipMemcpyDeviceToDevice, X));
    recv_base += got;
  }
  GRS_HIP(hipEventRecord(s->xcev[16], X));
  GRS_HIP(hipStreamWaitEvent(st, s->xcev[16], 0));
  if (xmark(s, 2, st) != GRS_OK) return GRS_EHIP;
  *n_out = static_cast<size_t>(recv_base);
  // 6. local sort of the received run
  const grs_status rs = grs_sort(s, out_k, nullptr, static_cast<size_t>(recv_base), st);
  if (rs != GRS_OK || xmark(s, 3, st) != GRS_OK) return rs != GRS_OK ? rs : GRS_EHIP;
  s->xev_recorded = s->ring > 0;
  s->x_sent = sent * sizeof(K);
  s->x_recv = recvd * sizeof(K);
  s->x_presorted = 0;
  return GRS_OK;
}

template <typename K, bool PAIRS>
grs_status run_sharded(grs_sorter* s, const K* keys, const uint32_t* vals, uint32_t n, K* out_k,
                       uint32_t* out_v, size_t out_cap, size_t* n_out, ncclComm_t comm, int g,
                       int me, hipStream_t st) {
  if constexpr (!PAIRS) {
    if (s->sharded_exchange == 3) {   // chunked partition-first (keys only)
      if (g <= 2) return run_sharded_chunked<K, 1>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      if (g <= 4) return run_sharded_chunked<K, 3>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      if (g <= 8) return run_sharded_chunked<K, 7>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      return run_sharded_chunked<K, 15>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
    }
  }
  if constexpr (sizeof(K) == 4 && !PAIRS) {
    // presorted exchange: u32 keys without payload, up to 4 ranks (GRS_OPT_EXCHANGE forces
    // either).  It moves ~1 byte a key instead of 4 but adds the
    // encode and ceil(log2 G) merge rounds; measured on one MI355X at C4 it is
    // ahead at 2 and 4 ranks and level at 8.  The sorted shard is staged in the output, and
    // encoded words count in u32.
    const bool want = s->sharded_exchange == 2 || (s->sharded_exchange == 0 && g <= 4);
    if (want && out_cap >= n && n < (1u << 31) && s->capacity < (1ull << 31)) {
      if (g <= 2) return run_sharded_presorted<1>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      if (g <= 4) return run_sharded_presorted<3>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      if (g <= 8) return run_sharded_presorted<7>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
      return run_sharded_presorted<15>(s, keys, n, out_k, out_cap, n_out, comm, g, me, st);
    }
  }
  if (g <= 2) return run_sharded_n<K, PAIRS, 1>(s, keys, vals, n, out_k, out_v, out_cap, n_out, comm, g, me, st);
  if (g <= 4) return run_sharded_n<K, PAIRS, 3>(s, keys, vals, n, out_k, out_v, out_cap, n_out, comm, g, me, st);
  if (g <= 8) return run_sharded_n<K, PAIRS, 7>(s, keys, vals, n, out_k, out_v, out_cap, n_out, comm, g, me, st);
  return run_sharded_n<K, PAIRS, 15>(s, keys, vals, n, out_k, out_v, out_cap, n_out, comm, g, me, st);
}

}  // namespace

extern "C" {

grs_status grs_sort_sharded(grs_sorter* s, const void* d_keys_in, const uint32_t* d_vals_in,
                            size_t n_local, void* d_keys_out, uint32_t* d_vals_out,
                            size_t out_capacity, size_t* n_out, void* nccl_comm, void* stream) {
  if (!s || !n_out || !nccl_comm) return set_err(GRS_EINVAL, "grs_sort_sharded: NULL argument");
  *n_out = 0;
  if (n_local > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort_sharded: n_local exceeds capacity");
  if ((n_local && !d_keys_in) || !d_keys_out)
    return set_err(GRS_EINVAL, "grs_sort_sharded: NULL keys");
  if (s->pairs && ((n_local && !d_vals_in) || !d_vals_out))
    return set_err(GRS_EINVAL, "grs_sort_sharded: payload sorter needs d_vals_in / d_vals_out");
  ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
  int g = 0, me = 0;
  GRS_RCCL(ncclCommCount(comm, &g));
  GRS_RCCL(ncclCommUserRank(comm, &me));
  if (g < 1 || g > GRS_MAX_SPLITTERS + 1)
    return set_err(GRS_EINVAL, "grs_sort_sharded: 1..16 ranks supported");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t n32 = static_cast<uint32_t>(n_local);
  grs_status r;
  if (g == 1 && !s->sharded_general) {   // one rank: nothing to partition or exchange
    if (out_capacity < n_local) {
      r = set_err(GRS_ECAPACITY, "grs_sort_sharded: out_capacity below n_local");
    } else {
      const size_t kb = s->key_type == GRS_KEY_U32 ? 4 : 8;
      r = GRS_OK;
      if (n_local && d_keys_out != d_keys_in &&
          hipMemcpyAsync(d_keys_out, d_keys_in, n_local * kb, hipMemcpyDeviceToDevice, st) != hipSuccess)
        r = set_err(GRS_EHIP, "grs_sort_sharded: copy");
      if (r == GRS_OK && s->pairs && n_local && d_vals_out != d_vals_in &&
          hipMemcpyAsync(d_vals_out, d_vals_in, n_local * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        r = set_err(GRS_EHIP, "grs_sort_sharded: copy");
      if (r == GRS_OK) r = grs_sort(s, d_keys_out, s->pairs ? d_vals_out : nullptr, n_local, stream);
      if (r == GRS_OK) *n_out = n_local;
    }
  } else if (s->key_type == GRS_KEY_U32)
    r = s->pairs ? run_sharded<uint32_t, true>(s, (const uint32_t*)d_keys_in, d_vals_in, n32, (uint32_t*)d_keys_out, d_vals_out, out_capacity, n_out, comm, g, me, st)
                 : run_sharded<uint32_t, false>(s, (const uint32_t*)d_keys_in, nullptr, n32, (uint32_t*)d_keys_out, nullptr, out_capacity, n_out, comm, g, me, st);
  else
    r = s->pairs ? run_sharded<uint64_t, true>(s, (const uint64_t*)d_keys_in, d_vals_in, n32, (uint64_t*)d_keys_out, d_vals_out, out_capacity, n_out, comm, g, me, st)
                 : run_sharded<uint64_t, false>(s, (const uint64_t*)d_keys_in, nullptr, n32, (uint64_t*)d_keys_out, nullptr, out_capacity, n_out, comm, g, me, st);
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_shard_sample(const void* d_keys, size_t n, int key_bytes, int samples,
                            void* d_sample_keys, uint32_t* d_sample_pos, void* stream) {
  if ((key_bytes != 4 && key_bytes != 8) || samples <= 0 || !d_sample_keys || !d_sample_pos ||
      (n > 0 && !d_keys))
    return set_err(GRS_EINVAL, "grs_shard_sample: bad argument");
  if (n > GRS_MAX_N) return set_err(GRS_ECAPACITY, "grs_shard_sample: n too large");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid((samples + 255) / 256);
  const uint32_t n32 = static_cast<uint32_t>(n), S = static_cast<uint32_t>(samples);
  if (key_bytes == 4)
    hipLaunchKernelGGL((grs::grs_shard_samples<uint32_t>), grid, dim3(256), 0, st,
                       static_cast<const uint32_t*>(d_keys), n32, S,
                       static_cast<uint32_t*>(d_sample_keys), d_sample_pos);
  else
    hipLaunchKernelGGL((grs::grs_shard_samples<uint64_t>), grid, dim3(256), 0, st,
                       static_cast<const uint64_t*>(d_keys), n32, S,
                       static_cast<uint64_t*>(d_sample_keys), d_sample_pos);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
}

size_t grs_shard_encode_words_max(size_t n, int nranks) {
  return n + grs::kCodecDir * codec_blocks_max(n, std::max(nranks, 1));
}

grs_status grs_shard_encode(grs_sorter* s, const uint32_t* d_sorted, size_t n,
                            const uint32_t* d_gathered_keys, const uint32_t* d_gathered_pos,
                            int nranks, int rank, uint32_t* d_send, size_t send_capacity_words,
                            uint32_t* d_sizes, void* stream) {
  if (!s || !d_gathered_keys || !d_gathered_pos || !d_send || !d_sizes || (n > 0 && !d_sorted))
    return set_err(GRS_EINVAL, "grs_shard_encode: NULL argument");
  if (nranks < 1 || nranks > grs::kMaxRanks || rank < 0 || rank >= nranks)
    return set_err(GRS_EINVAL, "grs_shard_encode: 1..16 ranks");
  if (n >= (1u << 31)) return set_err(GRS_ECAPACITY, "grs_shard_encode: n >= 2^31");
  if (send_capacity_words < grs_shard_encode_words_max(n, nranks))
    return set_err(GRS_ECAPACITY, "grs_shard_encode: send buffer below grs_shard_encode_words_max");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int g = nranks;
  const uint32_t S = static_cast<uint32_t>(grs_shard_samples_per_rank(g));
  auto go = [&](auto nconst) -> grs_status {
    constexpr int N = decltype(nconst)::value;
    using Dig = grs::SplitterIdxDigit<uint32_t, N>;
    grs_status r = grow_buf(s, &s->shard_buf, &s->shard_bytes, sizeof(Dig), "grs_shard_encode: scratch");
    if (r != GRS_OK) return r;
    Dig* dig = static_cast<Dig*>(s->shard_buf);
    CodecScratch cs;
    if ((r = codec_scratch(s, n, s->capacity, g, &cs)) != GRS_OK) return r;
    hipLaunchKernelGGL((grs::grs_shard_splitters_sorted<uint32_t, N>), dim3(1), dim3(1024), 0, st,
                       d_gathered_keys, d_gathered_pos, static_cast<uint32_t>(g), S,
                       static_cast<uint32_t>(rank), dig);
    GRS_HIP(hipGetLastError());
    if ((r = codec_encode<N>(s, d_sorted, static_cast<uint32_t>(n), dig, g, d_send, cs, st)) != GRS_OK)
      return r;
    GRS_HIP(hipMemcpyAsync(d_sizes, cs.sizes, 4 * 2 * g, hipMemcpyDeviceToDevice, st));
    return GRS_OK;
  };
  grs_status r;
  if (g <= 2) r = go(std::integral_constant<int, 1>{});
  else if (g <= 4) r = go(std::integral_constant<int, 3>{});
  else if (g <= 8) r = go(std::integral_constant<int, 7>{});
  else r = go(std::integral_constant<int, 15>{});
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_shard_decode_merge(grs_sorter* s, const uint32_t* d_recv, int nranks,
                                  const uint64_t* recv_word_offsets, const uint32_t* recv_keys,
                                  uint32_t* d_keys_out, size_t out_capacity, void* stream) {
  if (!s || !recv_word_offsets || !recv_keys || !d_keys_out)
    return set_err(GRS_EINVAL, "grs_shard_decode_merge: NULL argument");
  if (nranks < 1 || nranks > grs::kMaxRanks)
    return set_err(GRS_EINVAL, "grs_shard_decode_merge: 1..16 sources");
  if (s->key_type != GRS_KEY_U32) return set_err(GRS_EINVAL, "grs_shard_decode_merge: u32 sorter");
  uint64_t total = 0;
  for (int p = 0; p < nranks; ++p) total += recv_keys[p];
  if (total > out_capacity || total > s->capacity || total >= (1ull << 31))
    return set_err(GRS_ECAPACITY, "grs_shard_decode_merge: received keys exceed a capacity");
  if (total > 0 && !d_recv) return set_err(GRS_EINVAL, "grs_shard_decode_merge: NULL d_recv");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  CodecScratch cs;
  grs_status r = codec_scratch(s, 0, s->capacity, nranks, &cs);
  if (r == GRS_OK)
    r = codec_decode_merge(s, d_recv, nranks, recv_word_offsets, recv_keys, d_keys_out, total, cs, st);
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_sharded_redo_count(const grs_sorter* s, uint64_t* count) {
  if (!s || !count) return set_err(GRS_EINVAL, "grs_sharded_redo_count: NULL argument");
  *count = s->x_region_redo;
  return GRS_OK;
}

grs_status grs_sharded_last_timing(grs_sorter* s, grs_sharded_timing* out) {
  if (!s || !out) return set_err(GRS_EINVAL, "grs_sharded_last_timing: NULL argument");
  std::memset(out, 0, sizeof(*out));
  if (!s->xev_recorded)
    return set_err(GRS_EINVAL, "grs_sharded_last_timing: no profiled multi-rank grs_sort_sharded call");
  GRS_HIP(hipEventSynchronize(s->xev[3]));
  float ms = 0;
  GRS_HIP(hipEventElapsedTime(&ms, s->xev[0], s->xev[3]));
  out->total_ms = ms;
  GRS_HIP(hipEventElapsedTime(&ms, s->xev[0], s->xev[1]));
  out->before_ms = ms;
  GRS_HIP(hipEventElapsedTime(&ms, s->xev[1], s->xev[2]));
  out->exchange_ms = ms;
  GRS_HIP(hipEventElapsedTime(&ms, s->xev[2], s->xev[3]));
  out->after_ms = ms;
  out->bytes_sent = s->x_sent;
  out->bytes_received = s->x_recv;
  out->presorted = s->x_presorted;
  return GRS_OK;
}

grs_status grs_rccl_unique_id(void* id_out) {
  if (!id_out) return set_err(GRS_EINVAL, "grs_rccl_unique_id: NULL");
  static_assert(sizeof(ncclUniqueId) == GRS_RCCL_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  GRS_RCCL(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return GRS_OK;
}

grs_status grs_rccl_comm_init(void** comm_out, const void* id, int nranks, int rank, int device) {
  if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks)
    return set_err(GRS_EINVAL, "grs_rccl_comm_init: bad argument");
  *comm_out = nullptr;
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  GRS_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ncclResult_t e = ncclCommInitRank(&c, nranks, uid, rank);
  (void)hipSetDevice(prev);
  if (e != ncclSuccess)
    return set_err(GRS_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
  *comm_out = c;
  return GRS_OK;
}

void grs_rccl_comm_destroy(void* comm) {
  if (comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm));
}

grs_status grs_shard_splitters_host(const void* sorted_keys, const uint32_t* sorted_idx,
                                    const uint32_t* gathered_pos, int key_bytes, int nranks,
                                    int samples_per_rank, int rank, void* splitters_out,
                                    uint32_t* thresholds_out) {
  if (!sorted_keys || !sorted_idx || !gathered_pos || (nranks > 1 && (!splitters_out || !thresholds_out)) ||
      (key_bytes != 4 && key_bytes != 8) || nranks < 1 || nranks > 16 || samples_per_rank < 1 ||
      rank < 0 || rank >= nranks)
    return set_err(GRS_EINVAL, "grs_shard_splitters_host: bad argument");
  const uint32_t m = static_cast<uint32_t>(nranks * samples_per_rank);
  for (int bb = 0; bb + 1 < nranks; ++bb) {
    const uint32_t q = grs::shard_quantile(static_cast<uint32_t>(bb), m, static_cast<uint32_t>(nranks));
    const uint32_t j = sorted_idx[q];
    if (key_bytes == 4)
      static_cast<uint32_t*>(splitters_out)[bb] = static_cast<const uint32_t*>(sorted_keys)[q];
    else
      static_cast<uint64_t*>(splitters_out)[bb] = static_cast<const uint64_t*>(sorted_keys)[q];
    thresholds_out[bb] = grs::shard_threshold(j / static_cast<uint32_t>(samples_per_rank),
                                              static_cast<uint32_t>(rank), gathered_pos[j]);
  }
  return GRS_OK;
}

grs_status grs_shard_bounds_host(const void* sorted_keys, size_t n, int key_bytes,
                                const void* splitters, const uint32_t* thresholds, int nranks,
                                uint64_t* bounds_out) {
  if ((key_bytes != 4 && key_bytes != 8) || nranks < 1 || nranks > grs::kMaxRanks || !bounds_out ||
      (n > 0 && !sorted_keys) || (nranks > 1 && (!splitters || !thresholds)) || n > GRS_MAX_N)
    return set_err(GRS_EINVAL, "grs_shard_bounds_host: bad argument");
  const uint32_t n32 = static_cast<uint32_t>(n);
  bounds_out[0] = 0;
  bounds_out[nranks] = n;
  for (int b = 0; b + 1 < nranks; ++b)
    bounds_out[b + 1] = key_bytes == 4
        ? grs::shard_bound(static_cast<const uint32_t*>(sorted_keys), n32,
                           static_cast<const uint32_t*>(splitters)[b], thresholds[b])
        : grs::shard_bound(static_cast<const uint64_t*>(sorted_keys), n32,
                           static_cast<const uint64_t*>(splitters)[b], thresholds[b]);
  return GRS_OK;
}

grs_status grs_shard_plan_host(const uint32_t* count_matrix, int nranks, int rank,
                               uint64_t* send_off, uint64_t* recv_off, uint64_t* n_out) {
  if (!count_matrix || !send_off || !recv_off || !n_out || nranks < 1 || nranks > 16 || rank < 0 ||
      rank >= nranks)
    return set_err(GRS_EINVAL, "grs_shard_plan_host: bad argument");
  shard_plan(count_matrix, nranks, rank, send_off, recv_off, n_out);
  return GRS_OK;
}

grs_status grs_shard_chunk_plan_host(const uint32_t* count_matrices, int nchunks, int nranks, int rank,
                                     uint64_t chunk_len, uint64_t* send_off, uint64_t* recv_off, uint64_t* n_out) {
  if (!count_matrices || !send_off || !recv_off || !n_out || nchunks < 1 || nranks < 1 || nranks > 16 ||
      rank < 0 || rank >= nranks)
    return set_err(GRS_EINVAL, "grs_shard_chunk_plan_host: bad argument");
  const size_t gg = static_cast<size_t>(nranks) * nranks;
  uint64_t base = 0;
  for (int c = 0; c < nchunks; ++c)
    base += grs::shard_chunk_plan(count_matrices + c * gg, nranks, rank, static_cast<uint64_t>(c) * chunk_len, base,
                                  send_off + static_cast<size_t>(c) * nranks, recv_off + static_cast<size_t>(c) * nranks);
  *n_out = base;
  return GRS_OK;
}

// The record sort's scratch, two allocations so a small call never pays for the capacity:
//  - rec_kbuf: the key and index buffers grs_records_key_buffers hands out, laid out for the
//    sorter's CAPACITY (the same place whatever n a later call sorts) and independent of the
//    record size, allocated on first use and never moved;
//  - rec_buf: grown on demand to one call's needs -- grs_sort_records' own keys | indices |
//    record copy, or grs_sort_records_by_keys' record copy.  It never aliases rec_kbuf, so the
//    buffers a caller holds stay valid whatever record size a later call uses.
static grs_status records_key_scratch(grs_sorter* s, void** keys, uint32_t** idx) {
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  const size_t cap = std::max<size_t>(s->capacity, 1);
  const size_t koff = (cap * kb + 255) & ~static_cast<size_t>(255);
  if (!s->rec_kbuf) {
    const grs_status r = sbuf_alloc(s, &s->rec_kbuf, koff + cap * 4, "grs_records_key_buffers: scratch");
    if (r != GRS_OK) return r;
  }
  *keys = s->rec_kbuf;
  *idx = reinterpret_cast<uint32_t*>(static_cast<char*>(s->rec_kbuf) + koff);
  return GRS_OK;
}

// rec_buf of at least `need` bytes (grown on demand; its contents are per call).
static grs_status records_call_scratch(grs_sorter* s, size_t need) {
  return grow_buf(s, &s->rec_buf, &s->rec_bytes, need, "grs_sort_records: scratch");
}

grs_status grs_records_key_buffers(grs_sorter* s, size_t n, size_t record_bytes, void** d_keys,
                                   uint32_t** d_idx) {
  if (!s || !d_keys || !d_idx) return set_err(GRS_EINVAL, "grs_records_key_buffers: NULL argument");
  if (!s->pairs) return set_err(GRS_EINVAL, "grs_records_key_buffers: needs a sorter created with a payload");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_records_key_buffers: n exceeds capacity");
  if (record_bytes == 0 || record_bytes > 0xFFFFFFFFull)
    return set_err(GRS_EINVAL, "grs_records_key_buffers: bad record size");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  const grs_status r = records_key_scratch(s, d_keys, d_idx);
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_sort_records_by_keys(grs_sorter* s, void* d_records, size_t n, size_t record_bytes,
                                    void* d_keys, uint32_t* d_idx, void* stream) {
  if (!s) return set_err(GRS_EINVAL, "grs_sort_records_by_keys: NULL sorter");
  if (!s->pairs) return set_err(GRS_EINVAL, "grs_sort_records_by_keys: needs a sorter created with a payload");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort_records_by_keys: n exceeds capacity");
  if (record_bytes == 0 || record_bytes > 0xFFFFFFFFull)
    return set_err(GRS_EINVAL, "grs_sort_records_by_keys: bad record size");
  if (n == 0) return GRS_OK;
  if (!d_records || !d_keys || !d_idx) return set_err(GRS_EINVAL, "grs_sort_records_by_keys: NULL buffer");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  // the caller's keys / indices may live in rec_kbuf (grs_records_key_buffers) or anywhere;
  // the record copy goes to rec_buf, sized for this call
  grs_status r = records_call_scratch(s, n * record_bytes);
  void* copy = s->rec_buf;
  if (r == GRS_OK) r = grs_sort(s, d_keys, d_idx, n, stream);                     // stable pairs
  if (r == GRS_OK) r = gather_records(d_records, copy, d_idx, n, record_bytes, stream,
                                      static_cast<uint32_t>(n - 1));  // K5
  if (r == GRS_OK && hipMemcpyAsync(d_records, copy, n * record_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_records_by_keys: copy back");
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_sort_records(grs_sorter* s, void* d_records, size_t n, size_t record_bytes,
                            const grs_key_extract* key, void* stream) {
  if (!s || !key) return set_err(GRS_EINVAL, "grs_sort_records: NULL argument");
  if (!s->pairs) return set_err(GRS_EINVAL, "grs_sort_records: needs a sorter created with a payload");
  if (n > s->capacity) return set_err(GRS_ECAPACITY, "grs_sort_records: n exceeds capacity");
  const size_t kb = s->key_type == GRS_KEY_U64 ? 8 : 4;
  if (record_bytes == 0 || record_bytes > 0xFFFFFFFFull ||
      (key->kind != GRS_EXTRACT_FIELD && key->kind != GRS_EXTRACT_MORTON3) ||
      (key->kind == GRS_EXTRACT_FIELD && (key->offset + kb > record_bytes || key->transform < 0 ||
                                          key->transform > 2)) ||
      (key->kind == GRS_EXTRACT_MORTON3 && static_cast<size_t>(key->offset) + 12 > record_bytes))
    return set_err(GRS_EINVAL, "grs_sort_records: key field outside the record or bad kind");
  if (n == 0) return GRS_OK;
  if (!d_records) return set_err(GRS_EINVAL, "grs_sort_records: NULL records");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  // keys | indices | record copy, sized for this call
  auto al = [](size_t b) { return (b + 255) & ~static_cast<size_t>(255); };
  grs_status r = records_call_scratch(s, al(n * kb) + al(n * 4) + n * record_bytes);
  char* rb = static_cast<char*>(s->rec_buf);
  void* keys = rb;
  uint32_t* idx = reinterpret_cast<uint32_t*>(rb + al(n * kb));
  void* copy = rb + al(n * kb) + al(n * 4);
  const grs::KeyExtract kx{key->kind, key->offset, key->transform,
                           {key->lo[0], key->lo[1], key->lo[2]}, {key->hi[0], key->hi[1], key->hi[2]}};
  if (r == GRS_OK) {   // K1: one fused pre-pass, key + index
    if (kb == 4)
      hipLaunchKernelGGL(grs::grs_extract_keys<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                         static_cast<const uint8_t*>(d_records), static_cast<uint64_t>(n),
                         static_cast<uint32_t>(record_bytes), kx, static_cast<uint32_t*>(keys), idx);
    else
      hipLaunchKernelGGL(grs::grs_extract_keys<uint64_t>, dim3(grid_for(n, 256)), dim3(256), 0, st,
                         static_cast<const uint8_t*>(d_records), static_cast<uint64_t>(n),
                         static_cast<uint32_t>(record_bytes), kx, static_cast<uint64_t*>(keys), idx);
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_records: launch");
  }
  if (r == GRS_OK) r = grs_sort(s, keys, idx, n, stream);                        // stable pairs
  if (r == GRS_OK) r = gather_records(d_records, copy, idx, n, record_bytes, stream,
                                      static_cast<uint32_t>(n - 1));  // K5
  if (r == GRS_OK && hipMemcpyAsync(d_records, copy, n * record_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_sort_records: copy back");                          // copy-back
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

grs_status grs_lds_order_check(int device, int blocks, int items, unsigned long long* mismatches) {
  if (!mismatches || blocks < 1 || items < 1 || items > 512)
    return set_err(GRS_EINVAL, "grs_lds_order_check: blocks >= 1, 1 <= items <= 512, non-NULL out");
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != device) GRS_HIP(hipSetDevice(device));
  unsigned long long* d = nullptr;
  grs_status r = GRS_OK;
  if (hipMalloc(&d, 8) != hipSuccess) {
    (void)hipGetLastError();
    r = set_err(GRS_ENOMEM, "grs_lds_order_check: allocation");
  }
  if (r == GRS_OK && hipMemset(d, 0, 8) != hipSuccess) r = set_err(GRS_EHIP, "grs_lds_order_check: memset");
  for (uint32_t p = 0; r == GRS_OK && p < 5; ++p) {
    const uint32_t it = static_cast<uint32_t>(items);
    hipLaunchKernelGGL((grs_lds_order_scale<4, 1>), dim3(blocks), dim3(512), 0, 0, p, it, d);
    hipLaunchKernelGGL((grs_lds_order_scale<8, 1>), dim3(blocks), dim3(512), 0, 0, p, it, d);
    hipLaunchKernelGGL((grs_lds_order_scale<8, 2>), dim3(blocks), dim3(512), 0, 0, p, it, d);
    hipLaunchKernelGGL((grs_lds_order_scale<11, 1>), dim3(blocks), dim3(512), 0, 0, p, it, d);
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_lds_order_check: launch");
  }
  if (r == GRS_OK && hipMemcpy(mismatches, d, 8, hipMemcpyDeviceToHost) != hipSuccess)
    r = set_err(GRS_EHIP, "grs_lds_order_check: copy");
  if (d) (void)hipFree(d);
  if (prev != device) (void)hipSetDevice(prev);
  return r;
}

const char* grs_pass_kernel(const grs_sorter* s, size_t n) {
  if (!s || n == 0) return "";
  // the MSD-first schedule (grs_msd.hpp): its P1 scatter kernel (bench.py attributes the
  // roofline to the slowest of P1 / P2 / P3 from their phase times)
  if (use_msd(s, n, 0, s->key_type == GRS_KEY_U64 ? 64 : 32)) return "grs_onesweep_region";
  auto pick = [&](size_t big_tile, bool two_rounds = false) -> const char* {
    if (s->rank_mode != 0 || !use_big_tiles(s, n, big_tile) || two_rounds) return "grs_onesweep_v4";
    if (!use_persistent(s, (n + big_tile - 1) / big_tile, s->radix_bits)) return "grs_onesweep_v4";
    const bool rec = s->key_type == GRS_KEY_U32 && s->pairs && s->radix_bits == 8 && s->rec_mode != 0;
    const bool fused = !rec && s->pass_mode == 8;
    return fused ? "grs_onesweep_fused" : "grs_onesweep_v6";
  };
  const bool u32 = s->key_type == GRS_KEY_U32;
  if (s->radix_bits == 4)
    return u32 ? (s->pairs ? pick(BigTile4<uint32_t, true>::TILE) : pick(BigTile4<uint32_t, false>::TILE))
               : (s->pairs ? pick(BigTile4<uint64_t, true>::TILE) : pick(BigTile4<uint64_t, false>::TILE));
  return u32 ? (s->pairs ? pick(BigTile<uint32_t, true>::TILE, use_xl(s, n, XLTile<uint32_t, true>::TILE))
                         : pick(BigTile<uint32_t, false>::TILE, use_xl(s, n, XLTile<uint32_t, false>::TILE)))
             : (s->pairs ? pick(BigTile<uint64_t, true>::TILE, BigTile<uint64_t, true>::TWO_ROUNDS)
                         : pick(BigTile<uint64_t, false>::TILE, use_xl(s, n, XLTile<uint64_t, false>::TILE)));
}

}  // extern "C"
