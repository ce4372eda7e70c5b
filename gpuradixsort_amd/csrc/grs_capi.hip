// grs_capi.hip — C-ABI of libgrs (include/grs.h): sorter lifecycle, pass driver, helpers.
//
// The pass driver replaces ParallelSort::Sort (Source/ComputeControllers/ParallelSort.cpp:168-298):
// where the reference issues 1 + 32 x 4 GLSL dispatches with a glMemoryBarrier after each,
// one grs_sort call issues
//     hipMemsetAsync(control block)  -> grs_upfront_hist  -> P x grs_onesweep_pass
// on one stream (P = ceil((end_bit - begin_bit) / radix_bits); 4 launches for u32 at 8-bit
// digits), plus one D2D copy when P is odd so the result lands back in the caller's buffer
// (the reference's glCopyBufferSubData, ParallelSort.cpp:312-318).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "../../include/grs.h"
#include "grs_config.h"
#include "grs_kernels.hpp"

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
      return set_err(GRS_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));     \
  } while (0)

// Tile geometry per (key type, payload, radix) of the one-tile-per-workgroup passes (the
// atomic-rank pass grs_onesweep_ar and the ballot-match fallback grs_onesweep_pass).
// ITEMS keys per thread, GRS_BLOCK threads; measured on MI355X (tools/lab.py).
template <typename K, bool PAIRS, int RB>
struct TileCfg {
  static constexpr int BLOCK = GRS_BLOCK;
  // The largest tiles that fit one workgroup's LDS (128-144 KB of keys + payload): longer
  // digit runs per tile, fewer look-back steps.  Lab (2^27, ms per pass, two sweeps):
  // u32 pairs 16 / 24 / 32 items 0.55 / 0.53-0.60 / 0.56; u64 keys 16 / 24 / 32 items
  // 0.56 / 0.53-0.56 / 0.51; u64 pairs 8 / 12 / 16 / 24 items 1.02 / 0.90-0.96 / 0.81-0.87 /
  // 0.80; bench C3 48 -> 55 Gkeys/s and C5 28.5 -> 30 going to 24 / 24 / 16 items; 36 items
  // (147 KB) another 1-2 % over 32 for u32 pairs and u64 keys (15 interleaved rounds).
  static constexpr int ITEMS = sizeof(K) == 8 ? (PAIRS ? 24 : 36) : (PAIRS ? 36 : 24);
  static constexpr int TILE = BLOCK * ITEMS;
};

// The persistent pass grs_onesweep_v3 (u32 keys without payload): 16 waves x 16 keys, one
// workgroup per CU (double-buffered 64 KB tiles in LDS).  Smaller v3 tiles, or v3 with a
// payload or u64 keys (8K- or 4K-key tiles), measured 2-6x slower: a workgroup holds the
// ticket of the tile it prefetches for a whole iteration, and with more, shorter tiles in
// flight later tiles' look-backs wait on those held tiles.
struct V3Cfg {
  static constexpr int BLOCK = 1024;
  static constexpr int ITEMS = 16;
  static constexpr int TILE = BLOCK * ITEMS;
};

// One-tile-per-workgroup atomic-rank pass with 32K-36K-key tiles for u32 keys without payload
// (the default, 512 x 72; GRS_U32_PASS=ar1024 / ar512 select 1024 x 32 / 512 x 64): longer
// digit runs per tile beat v3's prefetching of 16K-key tiles (lab 0.276 vs 0.285 ms per pass,
// in the sort 109.8 vs 105.4 Gkeys/s).
template <int B, int I>
struct BigCfg {
  static constexpr int BLOCK = B;
  static constexpr int ITEMS = I;
  static constexpr int TILE = B * I;
};

constexpr int max_tile_min() { return 2048; }  // smallest TILE over configs (sizes status)

// Status words of one look-back buffer for `tiles` tiles: the larger of the one-tile passes'
// layout (tile words + group accumulators + group INCLUSIVE words) and v3's (tile words +
// group + 2 x supergroup words).
size_t status_words_for(size_t tiles, size_t radix) {
  const size_t groups = (tiles + GRS_LB_GROUP - 1) / GRS_LB_GROUP;
  return std::max((tiles + 2 * groups) * radix, grs::hier_status_words(tiles, radix));
}

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

// Rank mode per device: 0 = atomic ranking (probe passed), 1 = ballot-match fallback.
// GRS_RANK=match in the environment forces the fallback (tests cover both paths).
int device_rank_mode(int device) {
  static std::mutex mu;
  static int mode[64];
  static bool known[64];
  const char* env = std::getenv("GRS_RANK");
  if (env && std::strcmp(env, "match") == 0) return 1;
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
  int rank_mode = 0;               // 0: atomic ranking (v3 / ar passes), 1: ballot-match fallback
  int v3_grid = 0;                 // resident v3 workgroups (CUs x blocks per CU)
  size_t capacity = 0;
  void* alt_keys = nullptr;
  uint32_t* alt_vals = nullptr;
  uint32_t* status = nullptr;      // 2 x status_words
  size_t status_words = 0;         // per buffer
  uint32_t* ctrl = nullptr;        // GRS_CTRL_WORDS
  size_t scratch_bytes = 0;
  // Profiling ring: the last `ring` calls keep their per-phase hipEvents.
  static constexpr int EV_PER_CALL = GRS_MAX_PASSES + 3;
  int ring = 0;
  long long calls = 0;             // profiled calls recorded so far
  hipEvent_t* ev = nullptr;        // ring * EV_PER_CALL events
  struct CallInfo { int ev_used; int passes; bool copy; };
  CallInfo* info = nullptr;        // ring entries
  // grs_sort_segmented scratch (allocated on first use, grown on demand)
  void* seg_buf = nullptr;
  size_t seg_bytes = 0;
  grs_sorter* seg64 = nullptr;     // u64 pair sorter of (segment << 32 | key), u32 keys only
  void* host_stage = nullptr;      // grs_sort_host device staging (keys | payload), on first use
  size_t host_stage_bytes = 0;
  // tuning knobs read from the environment at grs_create (A/B measurements on one box)
  // GRS_V3_DMA=nt: nontemporal tile DMA.  One box, same process (tools/ab_v3_dma.sh): nt made
  // the pass 1 % faster but the next histogram 20 % slower (106.5 vs 104.2 Gkeys/s), so off.
  bool v3_dma_nt = false;
  int hist_grid_cap = 1024;             // GRS_HIST_GRID: cap of the upfront histogram grid
  // GRS_U32_PASS (u32 keys without payload): -1 = auto (default), 0 = v3, 1 = ar1024,
  // 2 = ar512, 3 = ar512x72.  Same box, same process (tools/ab_u32_pass.sh, ab_u32_size.sh):
  // at 2^27 keys v3 105.4, ar1024 109.5, ar512x72 109.8 Gkeys/s; but a one-tile-per-workgroup
  // grid of 36K-key tiles has a tail: at 2^24 / 2^25 / 2^26 keys v3 wins (77 / 89 / 97 vs
  // 53 / 71 / 87 Gkeys/s).  Auto = ar512x72 from 12 tiles per resident v3 workgroup (CU) up.
  int u32_pass = -1;
  bool part_match = false;              // GRS_PART_RANK=match: ballot-match partition pass
};

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
  }
  return "GRS_UNKNOWN";
}

const char* grs_last_error(void) { return g_last_error.c_str(); }

void grs_destroy(grs_sorter* s) {
  if (!s) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(s->device);
  if (s->alt_keys) (void)hipFree(s->alt_keys);
  if (s->alt_vals) (void)hipFree(s->alt_vals);
  if (s->status) (void)hipFree(s->status);
  if (s->ctrl) (void)hipFree(s->ctrl);
  if (s->seg_buf) (void)hipFree(s->seg_buf);
  if (s->seg64) grs_destroy(s->seg64);
  if (s->host_stage) (void)hipFree(s->host_stage);
  for (int i = 0; s->ev && i < s->ring * grs_sorter::EV_PER_CALL; ++i)
    if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
  delete[] s->ev;
  delete[] s->info;
  (void)hipSetDevice(prev);
  delete s;
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
    return set_err(GRS_ECAPACITY, "grs_create: capacity exceeds 2^30-1 items per device call");
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
  const size_t kb = key_type == GRS_KEY_U64 ? 8 : 4;
  const size_t cap = std::max<size_t>(capacity, 1);
  const size_t tiles = (cap + max_tile_min() - 1) / max_tile_min();
  s->status_words = status_words_for(tiles, size_t(1) << radix_bits);
  s->rank_mode = device_rank_mode(device);
  {
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (radix_bits == 8)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(&grs::grs_onesweep_v3<uint32_t, false, 8, V3Cfg::BLOCK, V3Cfg::ITEMS>),
          V3Cfg::BLOCK, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(&grs::grs_onesweep_v3<uint32_t, false, 4, V3Cfg::BLOCK, V3Cfg::ITEMS>),
          V3Cfg::BLOCK, 0);
    (void)hipGetLastError();
    s->v3_grid = std::max(1, cus) * std::max(1, per_cu);
  }
  if (const char* e = std::getenv("GRS_V3_DMA")) s->v3_dma_nt = std::strcmp(e, "nt") == 0;
  if (const char* e = std::getenv("GRS_HIST_GRID")) s->hist_grid_cap = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("GRS_PART_RANK")) s->part_match = std::strcmp(e, "match") == 0;
  if (const char* e = std::getenv("GRS_U32_PASS"))
    s->u32_pass = std::strcmp(e, "v3") == 0         ? 0
                  : std::strcmp(e, "ar1024") == 0   ? 1
                  : std::strcmp(e, "ar512") == 0    ? 2
                  : std::strcmp(e, "ar512x72") == 0 ? 3
                                                    : -1;
  grs_status st = GRS_OK;
  auto alloc = [&](void** p, size_t bytes) {
    if (st != GRS_OK) return;
    if (hipMalloc(p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      st = set_err(GRS_ENOMEM, "grs_create: hipMalloc of " + std::to_string(bytes) + " bytes failed");
      return;
    }
    s->scratch_bytes += bytes;
  };
  alloc(&s->alt_keys, cap * kb);
  if (s->pairs) alloc(reinterpret_cast<void**>(&s->alt_vals), cap * 4);
  alloc(reinterpret_cast<void**>(&s->status), 2 * s->status_words * 4);
  alloc(reinterpret_cast<void**>(&s->ctrl), GRS_CTRL_WORDS * 4);
  if (st == GRS_OK && hipMemset(s->ctrl, 0, GRS_CTRL_WORDS * 4) != hipSuccess)
    st = set_err(GRS_EHIP, "grs_create: hipMemset failed");
  (void)hipSetDevice(prev);
  if (st != GRS_OK) {
    grs_destroy(s);
    return st;
  }
  *out = s;
  return GRS_OK;
}

size_t grs_scratch_bytes(const grs_sorter* s) { return s ? s->scratch_bytes : 0; }

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
  }
  (void)hipSetDevice(prev);
  return st;
}

}  // extern "C"

namespace {

// Which pass kernel a sort call launches: the persistent v3 pass for u32 keys without payload,
// the one-tile-per-workgroup atomic-rank pass otherwise, the ballot-match pass if the LDS
// order probe failed (or GRS_RANK=match).
enum class PassKind { V3, AR, MATCH, AR1024, AR512, AR512X72 };

// u32 keys without payload, GRS_U32_PASS unset: the 36K-tile pass once the grid has >= 12
// tiles per CU (its tail is then small), the persistent v3 pass below that
int u32_pass_for(const grs_sorter* s, size_t n) {
  if (s->u32_pass >= 0) return s->u32_pass;
  const size_t tiles = (n + BigCfg<512, 72>::TILE - 1) / BigCfg<512, 72>::TILE;
  return tiles >= 12 * static_cast<size_t>(std::max(1, s->v3_grid)) ? 3 : 0;
}

template <typename K, bool PAIRS>
PassKind pass_kind(const grs_sorter* s, size_t n) {
  if (s->rank_mode != 0) return PassKind::MATCH;
  const int u32_pass = u32_pass_for(s, n);
  if (!PAIRS && sizeof(K) == 4)
    return u32_pass == 1   ? PassKind::AR1024
           : u32_pass == 2 ? PassKind::AR512
           : u32_pass == 3 ? PassKind::AR512X72
                              : PassKind::V3;
  return PassKind::AR;
}

template <typename K, bool PAIRS, int RB>
grs_status run_sort(grs_sorter* s, K* keys, uint32_t* vals, uint32_t n, int begin_bit,
                    int end_bit, hipStream_t stream) {
  using Cfg = TileCfg<K, PAIRS, RB>;
  constexpr int RADIX = 1 << RB;
  const PassKind kind = pass_kind<K, PAIRS>(s, n);
  const int passes = (end_bit - begin_bit + RB - 1) / RB;
  const uint32_t tile = kind == PassKind::V3       ? V3Cfg::TILE
                        : kind == PassKind::AR1024 ? BigCfg<1024, 32>::TILE
                        : kind == PassKind::AR512  ? BigCfg<512, 64>::TILE
                        : kind == PassKind::AR512X72 ? BigCfg<512, 72>::TILE
                                                   : Cfg::TILE;
  const uint32_t tiles = (n + tile - 1) / tile;
  const size_t words = status_words_for(tiles, RADIX);
  if (words > s->status_words) return set_err(GRS_ECAPACITY, "status buffer too small");
  uint32_t* st0 = s->status;
  uint32_t* st1 = s->status + s->status_words;
  uint32_t* hist = s->ctrl;
  uint32_t* tickets = s->ctrl + GRS_CTRL_TICKETS;
  uint32_t* err = s->ctrl + GRS_CTRL_ERROR;
  int ev = 0;
  hipEvent_t* evs = s->ring ? s->ev + (s->calls % s->ring) * grs_sorter::EV_PER_CALL : nullptr;
  auto mark = [&]() -> grs_status {
    if (evs) GRS_HIP(hipEventRecord(evs[ev++], stream));
    return GRS_OK;
  };

  grs_status r;
  if ((r = mark()) != GRS_OK) return r;
  // zero histograms + tickets (the error word is sticky: only grs_check_error clears it)
  GRS_HIP(hipMemsetAsync(s->ctrl, 0, GRS_CTRL_ERROR * 4, stream));
  {
    // > n / 2^18 blocks keeps every 16-bit bank-private counter below 2^16 (HistLayout)
    // 1024 blocks: 5 % faster than 2048 alone (tools/histlab.py) and 0.008 ms faster inside
    // the sort (tools/ab_v3_dma.sh); GRS_HIST_GRID overrides the cap
    const int grid = std::max<int>((n >> 18) + 1, std::min<int>(s->hist_grid_cap, (n + 4095) / 4096));
    hipLaunchKernelGGL((grs::grs_upfront_hist<K, RB>), dim3(grid), dim3(GRS_HIST_BLOCK), 0,
                       stream, keys, n, begin_bit, end_bit, passes, hist, st0,
                       static_cast<uint32_t>(words));
    GRS_HIP(hipGetLastError());
  }
  if ((r = mark()) != GRS_OK) return r;

  K* src = keys;
  K* dst = static_cast<K*>(s->alt_keys);
  uint32_t* vsrc = vals;
  uint32_t* vdst = s->alt_vals;
  for (int p = 0; p < passes; ++p) {
    const int shift = begin_bit + p * RB;
    const int bits = std::min(RB, end_bit - shift);
    uint32_t* st_cur = (p & 1) ? st1 : st0;
    uint32_t* st_nxt = (p & 1) ? st0 : st1;
    const grs::RadixDigit<K> dig{shift, (1u << bits) - 1u};
    if (kind == PassKind::V3) {
      if constexpr (!PAIRS && sizeof(K) == 4) {
        const uint32_t grid = std::min<uint32_t>(tiles, static_cast<uint32_t>(s->v3_grid));
        if (!s->v3_dma_nt)   // default cache policy for the tile DMA (see grs_create)
          hipLaunchKernelGGL((grs::grs_onesweep_v3<K, false, RB, V3Cfg::BLOCK, V3Cfg::ITEMS, 128>),
                             dim3(grid), dim3(V3Cfg::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig,
                             hist + p * RADIX, tickets + p, st_cur, st_nxt, err);
        else
          hipLaunchKernelGGL((grs::grs_onesweep_v3<K, false, RB, V3Cfg::BLOCK, V3Cfg::ITEMS>),
                             dim3(grid), dim3(V3Cfg::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig,
                             hist + p * RADIX, tickets + p, st_cur, st_nxt, err);
      }
    } else if (kind == PassKind::AR1024 || kind == PassKind::AR512 || kind == PassKind::AR512X72) {
      if constexpr (!PAIRS && sizeof(K) == 4) {
        if (kind == PassKind::AR512X72)
          hipLaunchKernelGGL((grs::grs_onesweep_ar<K, false, RB, 512, 72>), dim3(tiles), dim3(512),
                             0, stream, src, dst, vsrc, vdst, n, dig, hist + p * RADIX,
                             tickets + p, st_cur, st_nxt, err);
        else if (kind == PassKind::AR1024)
          hipLaunchKernelGGL((grs::grs_onesweep_ar<K, false, RB, 1024, 32>), dim3(tiles),
                             dim3(1024), 0, stream, src, dst, vsrc, vdst, n, dig,
                             hist + p * RADIX, tickets + p, st_cur, st_nxt, err);
        else
          hipLaunchKernelGGL((grs::grs_onesweep_ar<K, false, RB, 512, 64>), dim3(tiles), dim3(512),
                             0, stream, src, dst, vsrc, vdst, n, dig, hist + p * RADIX,
                             tickets + p, st_cur, st_nxt, err);
      }
    } else if (kind == PassKind::AR) {
      hipLaunchKernelGGL((grs::grs_onesweep_ar<K, PAIRS, RB, Cfg::BLOCK, Cfg::ITEMS>), dim3(tiles),
                         dim3(Cfg::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig, hist + p * RADIX,
                         tickets + p, st_cur, st_nxt, err);
    } else {
      hipLaunchKernelGGL((grs::grs_onesweep_pass<K, PAIRS, RB, Cfg::BLOCK, Cfg::ITEMS>), dim3(tiles),
                         dim3(Cfg::BLOCK), 0, stream, src, dst, vsrc, vdst, n, dig, hist + p * RADIX,
                         tickets + p, st_cur, st_nxt, err);
    }
    GRS_HIP(hipGetLastError());
    if ((r = mark()) != GRS_OK) return r;
    std::swap(src, dst);
    std::swap(vsrc, vdst);
  }
  const bool copy = (passes & 1) != 0;
  if (copy) {  // result sits in scratch: copy back (ParallelSort.cpp:312-318)
    GRS_HIP(hipMemcpyAsync(keys, src, static_cast<size_t>(n) * sizeof(K), hipMemcpyDeviceToDevice,
                           stream));
    if (PAIRS)
      GRS_HIP(hipMemcpyAsync(vals, vsrc, static_cast<size_t>(n) * 4, hipMemcpyDeviceToDevice,
                             stream));
    if ((r = mark()) != GRS_OK) return r;
  }
  if (evs) {
    s->info[s->calls % s->ring] = {ev, passes, copy};
    ++s->calls;
  }
  return GRS_OK;
}

// Stable key-range partition: one histogram launch + one pass with a splitter digit (4-bit
// slot, up to 16 buckets).  Buckets land contiguously in keys_out/vals_out in bucket order;
// bucket sizes are copied to d_counts[0..count].
template <typename K, bool PAIRS>
grs_status run_partition(grs_sorter* s, const K* keys, const uint32_t* vals, K* keys_out,
                         uint32_t* vals_out, uint32_t n, const K* splitters, int count,
                         uint32_t* d_counts, hipStream_t stream) {
  constexpr int RB = 4;
  using Cfg = TileCfg<K, PAIRS, RB>;
  grs::SplitterDigit<K> dig{};
  dig.count = static_cast<uint32_t>(count);
  for (int i = 0; i < GRS_MAX_SPLITTERS; ++i) dig.s[i] = i < count ? splitters[i] : K(0);
  const uint32_t tiles = (n + Cfg::TILE - 1) / Cfg::TILE;
  const size_t words = status_words_for(tiles, 1u << RB);
  if (words > s->status_words) return set_err(GRS_ECAPACITY, "status buffer too small");
  uint32_t* hist = s->ctrl;
  GRS_HIP(hipMemsetAsync(s->ctrl, 0, GRS_CTRL_ERROR * 4, stream));
  const int grid = std::max(1, std::min<int>(2048, (n + 4095) / 4096));
  if (count == 7) {
    grs::SplitterDigitN<K, 7> d7{};
    d7.count = 7;
    for (int i = 0; i < GRS_MAX_SPLITTERS; ++i) d7.s[i] = dig.s[i];
    hipLaunchKernelGGL((grs::grs_digit_hist<K, grs::SplitterDigitN<K, 7>>), dim3(grid),
                       dim3(GRS_HIST_BLOCK), 0, stream, keys, n, d7, hist, s->status,
                       static_cast<uint32_t>(words));
  } else {
    hipLaunchKernelGGL((grs::grs_digit_hist<K, grs::SplitterDigit<K>>), dim3(grid),
                       dim3(GRS_HIST_BLOCK), 0, stream, keys, n, dig, hist, s->status,
                       static_cast<uint32_t>(words));
  }
  GRS_HIP(hipGetLastError());
  // power-of-two rank counts get a compile-time splitter count (unrolled in SGPRs)
  auto fixed = [&](auto nconst) {
    constexpr int N = decltype(nconst)::value;
    grs::SplitterDigitN<K, N> dn{};
    dn.count = N;
    for (int i = 0; i < GRS_MAX_SPLITTERS; ++i) dn.s[i] = dig.s[i];
    hipLaunchKernelGGL((grs::grs_onesweep_ar<K, PAIRS, RB, Cfg::BLOCK, Cfg::ITEMS, 0,
                                             grs::SplitterDigitN<K, N>>),
                       dim3(tiles), dim3(Cfg::BLOCK), 0, stream, keys, keys_out, vals, vals_out, n,
                       dn, hist, s->ctrl + GRS_CTRL_TICKETS, s->status,
                       s->status + s->status_words, s->ctrl + GRS_CTRL_ERROR);
  };
  if (s->rank_mode == 0 && !s->part_match && count == 7)
    fixed(std::integral_constant<int, 7>{});
  else if (s->rank_mode == 0 && !s->part_match && count == 3)
    fixed(std::integral_constant<int, 3>{});
  else if (s->rank_mode == 0 && !s->part_match && count == 1)
    fixed(std::integral_constant<int, 1>{});
  else if (s->rank_mode == 0 && !s->part_match)
    hipLaunchKernelGGL((grs::grs_onesweep_ar<K, PAIRS, RB, Cfg::BLOCK, Cfg::ITEMS, 0,
                                             grs::SplitterDigit<K>>),
                       dim3(tiles), dim3(Cfg::BLOCK), 0, stream, keys, keys_out, vals, vals_out, n,
                       dig, hist, s->ctrl + GRS_CTRL_TICKETS, s->status,
                       s->status + s->status_words, s->ctrl + GRS_CTRL_ERROR);
  else
    hipLaunchKernelGGL((grs::grs_onesweep_pass<K, PAIRS, RB, Cfg::BLOCK, Cfg::ITEMS, 0,
                                               grs::SplitterDigit<K>>),
                       dim3(tiles), dim3(Cfg::BLOCK), 0, stream, keys, keys_out, vals, vals_out, n,
                       dig, hist, s->ctrl + GRS_CTRL_TICKETS, s->status,
                       s->status + s->status_words, s->ctrl + GRS_CTRL_ERROR);
  GRS_HIP(hipGetLastError());
  GRS_HIP(hipMemcpyAsync(d_counts, hist, (count + 1) * 4, hipMemcpyDeviceToDevice, stream));
  return GRS_OK;
}

}  // namespace

extern "C" {

grs_status grs_partition(grs_sorter* s, const void* d_keys, const uint32_t* d_vals,
                         void* d_keys_out, uint32_t* d_vals_out, size_t n,
                         const void* splitters, int n_splitters, uint32_t* d_counts,
                         void* stream) {
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
                                        d_vals_out, n32, (const uint32_t*)splitters, n_splitters,
                                        d_counts, st);
    else
      r = run_partition<uint32_t, false>(s, (const uint32_t*)d_keys, nullptr, (uint32_t*)d_keys_out,
                                         nullptr, n32, (const uint32_t*)splitters, n_splitters,
                                         d_counts, st);
  } else {
    if (s->pairs)
      r = run_partition<uint64_t, true>(s, (const uint64_t*)d_keys, d_vals, (uint64_t*)d_keys_out,
                                        d_vals_out, n32, (const uint64_t*)splitters, n_splitters,
                                        d_counts, st);
    else
      r = run_partition<uint64_t, false>(s, (const uint64_t*)d_keys, nullptr, (uint64_t*)d_keys_out,
                                         nullptr, n32, (const uint64_t*)splitters, n_splitters,
                                         d_counts, st);
  }
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
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
  int prev = 0;
  GRS_HIP(hipGetDevice(&prev));
  if (prev != s->device) GRS_HIP(hipSetDevice(s->device));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t n32 = static_cast<uint32_t>(n);
  grs_status r = GRS_EINVAL;
  const bool u64 = s->key_type == GRS_KEY_U64;
  if (!u64 && !s->pairs && s->radix_bits == 8)
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
  uint32_t e = 0;
  GRS_HIP(hipDeviceSynchronize());
  GRS_HIP(hipMemcpy(&e, s->ctrl + GRS_CTRL_ERROR, 4, hipMemcpyDeviceToHost));
  if (e) {
    GRS_HIP(hipMemset(s->ctrl + GRS_CTRL_ERROR, 0, 4));
    return set_err(GRS_ETIMEOUT, "a look-back spin exceeded its bound");
  }
  return GRS_OK;
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

grs_status grs_gather_records(const void* d_src, void* d_dst, const uint32_t* d_idx, size_t n,
                              size_t record_bytes, void* stream) {
  if (n == 0) return GRS_OK;
  if (!d_src || !d_dst || !d_idx || record_bytes == 0 || record_bytes > 0xFFFFFFFFull)
    return set_err(GRS_EINVAL, "grs_gather_records: bad argument");
  hipLaunchKernelGGL(grs::grs_gather_records, dim3(grid_for(n * ((record_bytes + 3) / 4), 256)),
                     dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), d_idx,
                     static_cast<uint64_t>(n), static_cast<uint32_t>(record_bytes));
  GRS_HIP(hipGetLastError());
  return GRS_OK;
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

// Scan scratch: [0] error word (kept for the ABI; reduce-then-scan never spins), [1..3]
// pad, then one uint32 prefix per 16K-item tile.
static constexpr size_t kScanTile = GRS_SCAN_BLOCK * GRS_SCAN_ITEMS;

size_t grs_scan_scratch_bytes(size_t n) { return 16 + 4 * ((n + kScanTile - 1) / kScanTile); }

grs_status grs_exclusive_scan_u32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                  uint32_t* d_total, void* d_scratch, size_t scratch_bytes,
                                  void* stream) {
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
  uint32_t* ctl = static_cast<uint32_t*>(d_scratch);
  uint32_t* sums = ctl + 4;
  const uint32_t tiles = static_cast<uint32_t>((n + kScanTile - 1) / kScanTile);
  const uint32_t n32 = static_cast<uint32_t>(n);
  GRS_HIP(hipMemsetAsync(ctl, 0, 16, st));
  hipLaunchKernelGGL(grs::grs_scan_reduce, dim3(tiles), dim3(GRS_SCAN_BLOCK), 0, st, d_in, n32,
                     sums);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL(grs::grs_scan_spine, dim3(1), dim3(GRS_SCAN_SPINE_BLOCK), 0, st, sums, tiles,
                     d_total);
  GRS_HIP(hipGetLastError());
  hipLaunchKernelGGL(grs::grs_scan_downsweep, dim3(tiles), dim3(GRS_SCAN_BLOCK), 0, st, d_in,
                     d_out, n32, sums);
  GRS_HIP(hipGetLastError());
  return GRS_OK;
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
  grs_status r = GRS_OK;
  if (s->seg_bytes < need) {
    if (s->seg_buf) (void)hipFree(s->seg_buf);
    s->seg_buf = nullptr;
    s->seg_bytes = 0;
    if (hipMalloc(&s->seg_buf, need) != hipSuccess) {
      (void)hipGetLastError();
      r = set_err(GRS_ENOMEM, "grs_sort_segmented: scratch allocation failed");
    } else {
      s->seg_bytes = need;
    }
  }
  if (r == GRS_OK && (!s->seg64 || s->seg64->capacity < n)) {
    if (s->seg64) grs_destroy(s->seg64);
  if (s->host_stage) (void)hipFree(s->host_stage);
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
  if (r == GRS_OK) r = grs_exclusive_scan_u32(marks, excl, n, nullptr, scan_scratch, scan_bytes, stream);
  if (r == GRS_OK) {
    hipLaunchKernelGGL(grs::grs_segment_compose, dim3(grid_for(n, 256)), dim3(256), 0, st,
                       static_cast<const uint32_t*>(d_keys), marks, excl, comp,
                       static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  // payload: the caller's values, or the marks buffer as a don't-care rider
  if (r == GRS_OK) r = grs_sort_bits(s->seg64, comp, d_vals ? d_vals : marks, n, 0, 32 + segbits, stream);
  if (r == GRS_OK) {
    hipLaunchKernelGGL(grs::grs_segment_split, dim3(grid_for(n, 256)), dim3(256), 0, st, comp,
                       static_cast<uint32_t*>(d_keys), static_cast<uint64_t>(n));
    if (hipGetLastError() != hipSuccess) r = set_err(GRS_EHIP, "grs_sort_segmented: launch");
  }
  if (prev != s->device) (void)hipSetDevice(prev);
  return r;
}

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
  grs_status r = GRS_OK;
  if (s->seg_bytes < need) {
    if (s->seg_buf) (void)hipFree(s->seg_buf);
  if (s->seg64) grs_destroy(s->seg64);
  if (s->host_stage) (void)hipFree(s->host_stage);
    s->seg_buf = nullptr;
    s->seg_bytes = 0;
    if (hipMalloc(&s->seg_buf, need) != hipSuccess) {
      (void)hipGetLastError();
      r = set_err(GRS_ENOMEM, "grs_sort_segmented: scratch allocation failed");
    } else {
      s->seg_bytes = need;
    }
  }
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
  grs_status r = GRS_OK;
  if (s->host_stage_bytes < need) {
    if (s->host_stage) (void)hipFree(s->host_stage);
    s->host_stage = nullptr;
    s->host_stage_bytes = 0;
    if (hipMalloc(&s->host_stage, need) != hipSuccess) {
      (void)hipGetLastError();
      r = set_err(GRS_ENOMEM, "grs_sort_host: staging allocation failed");
    } else {
      s->host_stage_bytes = need;
    }
  }
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

const char* grs_pass_kernel(const grs_sorter* s, size_t n) {
  if (!s) return "";
  if (s->rank_mode != 0) return "grs_onesweep_pass";
  if (s->key_type == GRS_KEY_U32 && !s->pairs && u32_pass_for(s, n) == 0) return "grs_onesweep_v3";
  return "grs_onesweep_ar";
}

}  // extern "C"
