// grs_codec.hpp — the presorted exchange of grs_sort_sharded (u32 keys, no payload).
//
// New with respect to the reference (single-context).  The partition-first
// exchange (grs_shard.hpp + the partition pass) sends every key as 4 bytes over xGMI, and at
// 8 ranks that transfer costs about as much as the whole local sort.  Sorting
// FIRST makes each bucket a sorted run, and a sorted run of uniform keys compresses to about
// one byte per key as bit-packed deltas:
//
//   local sort      grs_sort of the shard (out of place)
//   bounds          the splitters of grs_shard_splitters (samples of the SORTED shard, ties
//                   by global index) become G + 1 positions of the sorted shard: bucket b is
//                   the run [bounds[b], bounds[b+1])                      grs_shard_bounds
//   encode          per bucket: 256-key blocks; block = directory entry {first key, data word
//                   offset in the bucket, width | count << 8} + (count - 1) deltas of `width`
//                   bits; buckets land back to back: [directory][data]    grs_codec_sizes,
//                                                   exclusive scan of the block words, grs_codec_pack
//   exchange        one send / recv of u32 words per peer (RCCL, or any transport)
//   decode          every received block -> its run, runs in source-rank order  grs_codec_unpack
//   merge           ceil(log2 G) rounds of a 2-way merge path over the runs (ties: the lower
//                   run first, i.e. global input order)               grs_merge_corank/tiles
//                   or (option GRS_OPT_MERGE = 1) ONE k-way pass: sample-delimited tiles
//                   merged in LDS, grs_mergek_samples/bounds/tiles -- correct, and measured
//                   slower at 8 ranks
//
// The order of the result is the same as the partition-first path's: bucket b holds the
// range of the global (key, global index) order between splitters b-1 and b.
#pragma once

#include "grs_pass.hpp"

namespace grs {

constexpr int kCodecBlock = 256;     // keys per block (one wave, 4 per lane)
constexpr int kCodecDir = 3;         // directory words per block
constexpr int kMergeTile = 4096;     // outputs per merge workgroup
constexpr int kMergeVT = 16;         // outputs per merge thread
constexpr int kMaxRanks = GRS_MAX_SPLITTERS + 1;

// Sorted-shard positions of the buckets: plan[0..g] = bounds, plan[g+1..2g+1] = first block
// of each bucket (block_base[g] = blocks in total).  Splitter b (key, threshold th) splits the
// run of its key at clamp(th, lower_bound, upper_bound): th = 0 for a sample of an earlier
// rank (every local copy of the key follows it), all-ones for a later rank (every copy
// precedes it), the sample's own sorted position for this rank.  One 64-thread workgroup.
template <typename K>
__host__ __device__ __forceinline__ uint32_t shard_bound(const K* sorted, uint32_t n, K key, uint32_t th) {
  uint32_t lo = 0, hi = n;   // lower bound
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (sorted[mid] < key) lo = mid + 1; else hi = mid;
  }
  const uint32_t lb = lo;
  hi = n;                    // upper bound
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (sorted[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return th < lb ? lb : th > lo ? lo : th;
}

template <typename K, int N>
__global__ __launch_bounds__(64) void grs_shard_bounds(const K* __restrict__ sorted, uint32_t n,
                                                       const SplitterIdxDigit<K, N>* __restrict__ dig,
                                                       uint32_t g, uint32_t* __restrict__ plan) {
  __shared__ uint32_t b[kMaxRanks + 1];
  const uint32_t t = threadIdx.x;
  if (t == 0) {
    b[0] = 0;
    b[g] = n;
  }
  if (t + 1 < g) b[t + 1] = shard_bound(sorted, n, dig->s[t], dig->th[t]);
  __syncthreads();
  if (t <= g) plan[t] = b[t];
  if (t == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < g; ++i) {
      plan[g + 1 + i] = acc;
      acc += (b[i + 1] - b[i] + kCodecBlock - 1) / kCodecBlock;
    }
    plan[2 * g + 1] = acc;
  }
}

// Bucket of global block gb (block_base = plan + g + 1); g when gb is past the last block.
__device__ __forceinline__ uint32_t codec_bucket(const uint32_t* plan, uint32_t g, uint32_t gb) {
  const uint32_t* bb = plan + g + 1;
  uint32_t b = 0;
  while (b < g && bb[b + 1] <= gb) ++b;
  return b;
}

// Element i of a block sits in lane i % 64, row i / 64 (u): every load is 256 contiguous bytes.
constexpr int kCodecRows = kCodecBlock / GRS_WAVE;   // 4
constexpr int kCodecBPW = 4;                         // blocks per wave (loads of all in flight)

// Block position of global block gb: start in the sorted shard and key count (cnt 0: none).
struct CodecBlk {
  uint32_t b, start, cnt;
};
__device__ __forceinline__ CodecBlk codec_blk(const uint32_t* plan, uint32_t g, uint32_t gb,
                                              uint32_t nb_max) {
  CodecBlk k{g, 0, 0};
  if (gb >= nb_max) return k;
  k.b = codec_bucket(plan, g, gb);
  if (k.b >= g) return k;
  k.start = plan[k.b] + (gb - plan[g + 1 + k.b]) * kCodecBlock;
  k.cnt = min(static_cast<uint32_t>(kCodecBlock), plan[k.b + 1] - k.start);
  return k;
}

__device__ __forceinline__ void codec_load(const uint32_t* __restrict__ sorted, const CodecBlk& bk,
                                           uint32_t lane, uint32_t (&k)[kCodecRows]) {
#pragma unroll
  for (int u = 0; u < kCodecRows; ++u) {
    const uint32_t i = lane + GRS_WAVE * u;
    k[u] = bk.cnt ? sorted[bk.start + (i < bk.cnt ? i : bk.cnt - 1)] : 0u;
  }
}

// dl[u] = element i's key minus element i-1's (0 for element 0 and past cnt)
__device__ __forceinline__ void codec_deltas(const uint32_t (&k)[kCodecRows], uint32_t lane,
                                             uint32_t cnt, uint32_t (&dl)[kCodecRows]) {
#pragma unroll
  for (int u = 0; u < kCodecRows; ++u) {
    // both shuffles run in every lane (an inactive source lane would read garbage)
    const uint32_t up = __shfl_up(k[u], 1, GRS_WAVE);
    const uint32_t last = __shfl(k[u > 0 ? u - 1 : 0], GRS_WAVE - 1, GRS_WAVE);
    const uint32_t prev = lane ? up : last;
    const uint32_t i = lane + GRS_WAVE * u;
    dl[u] = (i == 0 || i >= cnt) ? 0u : k[u] - prev;
  }
}

__device__ __forceinline__ uint32_t codec_width(uint32_t maxd) { return maxd ? 32u - __clz(maxd) : 0u; }
__device__ __forceinline__ uint32_t codec_words(uint32_t cnt, uint32_t w) {
  return static_cast<uint32_t>((static_cast<uint64_t>(cnt - 1) * w + 31) / 32);
}

// kCodecBPW blocks per wave: width and packed size of each.  blk_words[gb] (0 past the last
// block: the scan runs over an upper bound of the block count), blk_meta[2gb..] = {first key,
// w | cnt << 8}.
__global__ __launch_bounds__(256) void grs_codec_sizes(const uint32_t* __restrict__ sorted,
                                                       const uint32_t* __restrict__ plan, uint32_t g,
                                                       uint32_t nb_max, uint32_t* __restrict__ blk_words,
                                                       uint32_t* __restrict__ blk_meta) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gb0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kCodecBPW;
  CodecBlk bk[kCodecBPW];
  uint32_t k[kCodecBPW][kCodecRows];
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) bk[q] = codec_blk(plan, g, gb0 + q, nb_max);
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) codec_load(sorted, bk[q], lane, k[q]);
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    const uint32_t gb = gb0 + q;
    if (gb >= nb_max) break;
    if (bk[q].cnt == 0) {
      if (lane == 0) blk_words[gb] = 0;
      continue;
    }
    uint32_t dl[kCodecRows];
    codec_deltas(k[q], lane, bk[q].cnt, dl);
    uint32_t m = max(max(dl[0], dl[1]), max(dl[2], dl[3]));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(m, o, GRS_WAVE)));
    const uint32_t w = codec_width(m);
    if (lane == 0) {
      blk_words[gb] = codec_words(bk[q].cnt, w);
      blk_meta[2 * static_cast<size_t>(gb)] = k[q][0];
      blk_meta[2 * static_cast<size_t>(gb) + 1] = w | (bk[q].cnt << 8);
    }
  }
}

// kCodecBPW blocks per wave: directory entry and packed deltas (field f = element f+1's delta
// at bits [f*w, f*w + w) of the block's data words), assembled in LDS.  blk_woff: exclusive
// scan of blk_words (nb_max + 1 entries).  sizes[2b] = keys of bucket b, [2b+1] = its words.
__global__ __launch_bounds__(256) void grs_codec_pack(const uint32_t* __restrict__ sorted,
                                                      const uint32_t* __restrict__ plan, uint32_t g,
                                                      uint32_t nb_max, const uint32_t* __restrict__ blk_meta,
                                                      const uint32_t* __restrict__ blk_woff,
                                                      uint32_t* __restrict__ send,
                                                      uint32_t* __restrict__ sizes) {
  __shared__ uint32_t words[4][kCodecBPW][kCodecBlock];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t* bb = plan + g + 1;
  if (blockIdx.x == 0 && threadIdx.x < g) {
    const uint32_t b = threadIdx.x;
    sizes[2 * b] = plan[b + 1] - plan[b];
    sizes[2 * b + 1] = kCodecDir * (bb[b + 1] - bb[b]) + (blk_woff[bb[b + 1]] - blk_woff[bb[b]]);
  }
  const uint32_t gb0 = (blockIdx.x * 4 + wv) * kCodecBPW;
  CodecBlk bk[kCodecBPW];
  uint32_t k[kCodecBPW][kCodecRows];
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) bk[q] = codec_blk(plan, g, gb0 + q, nb_max);
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) codec_load(sorted, bk[q], lane, k[q]);
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
#pragma unroll
    for (int u = 0; u < kCodecRows; ++u) words[wv][q][lane + GRS_WAVE * u] = 0;
  }
  // one wave's LDS operations execute in issue order: the zeroing precedes the ors below
  asm volatile("" ::: "memory");
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    if (bk[q].cnt == 0) continue;
    const uint32_t meta = blk_meta[2 * static_cast<size_t>(gb0 + q) + 1];
    const uint32_t w = meta & 0xFFu;
    if (w == 0) continue;
    uint32_t dl[kCodecRows];
    codec_deltas(k[q], lane, bk[q].cnt, dl);
    uint32_t* lw = words[wv][q];
#pragma unroll
    for (int u = 0; u < kCodecRows; ++u) {
      const uint32_t i = lane + GRS_WAVE * u;
      if (i >= 1 && i < bk[q].cnt) {
        const uint32_t bit = (i - 1) * w;
        const uint32_t wi = bit >> 5, sh = bit & 31u;
        atomicOr(&lw[wi], dl[u] << sh);
        if (sh + w > 32u) atomicOr(&lw[wi + 1], dl[u] >> (32u - sh));
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's ors are done
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    if (bk[q].cnt == 0) continue;
    const uint32_t gb = gb0 + q, b = bk[q].b;
    const uint32_t meta = blk_meta[2 * static_cast<size_t>(gb) + 1];
    const uint32_t nw = codec_words(bk[q].cnt, meta & 0xFFu);
    const size_t base = kCodecDir * static_cast<size_t>(bb[b]) + blk_woff[bb[b]];
    const uint32_t nb = bb[b + 1] - bb[b];
    const uint32_t rel = blk_woff[gb] - blk_woff[bb[b]];
    uint32_t* dst = send + base + kCodecDir * static_cast<size_t>(nb) + rel;
    for (uint32_t i = lane; i < nw; i += GRS_WAVE) dst[i] = words[wv][q][i];
    if (lane < static_cast<uint32_t>(kCodecDir)) {
      uint32_t* dir = send + base + kCodecDir * static_cast<size_t>(gb - bb[b]);
      dir[lane] = lane == 0 ? k[q][0] : lane == 1 ? rel : meta;
    }
  }
}

// Where the received runs are: source p's stream of u32 words at word_off[p] (directory of
// its blocks, then their data), holding len[p] keys, decoded to run_off[p] of the output.
struct CodecSources {
  uint32_t g;
  uint32_t blk_base[kMaxRanks + 1];   // first global block of each source
  uint32_t len[kMaxRanks];
  uint32_t run_off[kMaxRanks];
  uint64_t word_off[kMaxRanks];
};

// kCodecBPW received blocks per wave: directory words of all of them, then their packed
// fields, then per block: unpack, prefix-sum the deltas in element order (a DPP wave scan per
// row plus the rows before), add the first key.
__global__ __launch_bounds__(256) void grs_codec_unpack(const uint32_t* __restrict__ recv,
                                                        const CodecSources src,
                                                        uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gb0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kCodecBPW;
  const uint32_t nbt = src.blk_base[src.g];
  if (gb0 >= nbt) return;
  uint32_t p[kCodecBPW], dirv[kCodecBPW];
  const uint32_t* data[kCodecBPW];
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    const uint32_t gb = min(gb0 + q, nbt - 1);
    uint32_t pp = 0;
    while (pp + 1 < src.g && src.blk_base[pp + 1] <= gb) ++pp;
    p[q] = pp;
    const uint32_t j = gb - src.blk_base[pp];
    const uint32_t* stream = recv + src.word_off[pp];
    // lanes 0..2 hold the block's directory words
    dirv[q] = lane < static_cast<uint32_t>(kCodecDir) ? stream[kCodecDir * j + lane] : 0u;
    data[q] = stream + kCodecDir * static_cast<size_t>(src.blk_base[pp + 1] - src.blk_base[pp]);
  }
  uint32_t first[kCodecBPW], w[kCodecBPW], cnt[kCodecBPW];
  uint32_t f[kCodecBPW][kCodecRows][2];
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    first[q] = __shfl(dirv[q], 0, GRS_WAVE);
    const uint32_t rel = __shfl(dirv[q], 1, GRS_WAVE);
    const uint32_t meta = __shfl(dirv[q], 2, GRS_WAVE);
    w[q] = meta & 0xFFu;
    cnt[q] = gb0 + q < nbt ? meta >> 8 : 0u;
    data[q] += rel;
#pragma unroll
    for (int u = 0; u < kCodecRows; ++u) {
      const uint32_t i = lane + GRS_WAVE * u;
      f[q][u][0] = f[q][u][1] = 0;
      if (w[q] > 0 && i >= 1 && i < cnt[q]) {
        const uint32_t bit = (i - 1) * w[q];
        f[q][u][0] = data[q][bit >> 5];
        if ((bit & 31u) + w[q] > 32u) f[q][u][1] = data[q][(bit >> 5) + 1];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kCodecBPW; ++q) {
    if (cnt[q] == 0) continue;
    const uint32_t gb = gb0 + q;
    const uint32_t j = gb - src.blk_base[p[q]];
    const uint32_t mask = w[q] >= 32 ? 0xFFFFFFFFu : (1u << w[q]) - 1u;
    uint32_t* o = out + src.run_off[p[q]] + static_cast<size_t>(j) * kCodecBlock;
    uint32_t carry = first[q];
#pragma unroll
    for (int u = 0; u < kCodecRows; ++u) {
      const uint32_t i = lane + GRS_WAVE * u;
      uint32_t d = 0;
      if (w[q] > 0 && i >= 1 && i < cnt[q]) {
        const uint32_t sh = ((i - 1) * w[q]) & 31u;
        d = f[q][u][0] >> sh;
        if (sh + w[q] > 32u) d |= f[q][u][1] << (32u - sh);
        d &= mask;
      }
      const uint32_t incl = wave_scan_dpp(d);
      if (i < cnt[q]) o[i] = carry + incl;
      carry += __shfl(incl, GRS_WAVE - 1, GRS_WAVE);
    }
  }
}

// ---- 2-way merge-path rounds --------------------------------------------------------------
// One round merges runs (2i, 2i+1) of `in` (offsets off[0..k]) into `out` at off[2i]; an odd
// last run merges with an empty one (a copy).  Ties take the lower run first (stable).
struct MergeRound {
  uint32_t pairs;
  uint32_t off[kMaxRanks + 1];        // run offsets, k + 1 of them (pairs * 2 + 1 used)
  uint32_t bbase[kMaxRanks / 2 + 2];  // first boundary index of each pair (tiles + 1 per pair)
};

// Number of A items among the first d outputs of merge(A[0..a), B[0..b)), ties to A.
template <typename LdA, typename LdB>
__device__ __forceinline__ uint32_t merge_corank(uint32_t d, uint32_t a, uint32_t b, const LdA& A,
                                                 const LdB& B) {
  uint32_t lo = d > b ? d - b : 0u, hi = d < a ? d : a;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (A(mid) <= B(d - mid - 1)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t merge_pair_of(const MergeRound& r, uint32_t x) {
  uint32_t i = 0;
  while (i + 1 < r.pairs && r.bbase[i + 1] <= x) ++i;
  return i;
}

// One thread per tile boundary (tile t of pair i starts at output t * kMergeTile; the pair's
// last boundary is its end).
__global__ __launch_bounds__(256) void grs_merge_corank(const uint32_t* __restrict__ in,
                                                        const MergeRound r,
                                                        uint32_t* __restrict__ corank) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
  if (x >= r.bbase[r.pairs]) return;
  const uint32_t i = merge_pair_of(r, x);
  const uint32_t t = x - r.bbase[i];
  const uint32_t a = r.off[2 * i + 1] - r.off[2 * i];
  const uint32_t b = r.off[2 * i + 2] - r.off[2 * i + 1];
  const uint32_t d = min(t * static_cast<uint32_t>(kMergeTile), a + b);
  const uint32_t* A = in + r.off[2 * i];
  const uint32_t* B = in + r.off[2 * i + 1];
  corank[x] = merge_corank(d, a, b, [&](uint32_t q) { return A[q]; },
                           [&](uint32_t q) { return B[q]; });
}

// One workgroup per tile: the tile's inputs (positions t + 256 v of [A part | B part]) into
// registers, all loads in flight, then LDS; a co-rank per thread; kMergeVT unrolled merge steps
// into registers; the tile out through LDS (padded against bank conflicts), coalesced.
__global__ __launch_bounds__(256) void grs_merge_tiles(const uint32_t* __restrict__ in,
                                                       uint32_t* __restrict__ out,
                                                       const MergeRound r,
                                                       const uint32_t* __restrict__ corank) {
  constexpr uint32_t PAD = kMergeTile + kMergeTile / 32;
  __shared__ uint32_t lin[kMergeTile];
  __shared__ uint32_t lout[PAD];
  const uint32_t tile = blockIdx.x;
  // tile -> (pair, local tile): boundaries bbase[i] .. bbase[i+1]-1 hold tiles_i + 1 entries
  uint32_t i = 0;
  while (i + 1 < r.pairs && r.bbase[i + 1] - (i + 1) <= tile) ++i;
  const uint32_t t = tile - (r.bbase[i] - i);
  const uint32_t a = r.off[2 * i + 1] - r.off[2 * i];
  const uint32_t b = r.off[2 * i + 2] - r.off[2 * i + 1];
  const uint32_t d0 = t * kMergeTile;
  const uint32_t d1 = min(d0 + kMergeTile, a + b);
  const uint32_t i0 = corank[r.bbase[i] + t], i1 = corank[r.bbase[i] + t + 1];
  const uint32_t j0 = d0 - i0, j1 = d1 - i1;
  const uint32_t la = i1 - i0, lb = j1 - j0, len = la + lb;
  const uint32_t* A = in + r.off[2 * i] + i0;
  const uint32_t* B = in + r.off[2 * i + 1] + j0;
  uint32_t x[kMergeVT];
#pragma unroll
  for (int v = 0; v < kMergeVT; ++v) {
    const uint32_t q = threadIdx.x + 256 * v;
    x[v] = q < la ? A[q] : q < len ? B[q - la] : 0u;
  }
#pragma unroll
  for (int v = 0; v < kMergeVT; ++v) {
    const uint32_t q = threadIdx.x + 256 * v;
    if (q < len) lin[q] = x[v];
  }
  __syncthreads();
  const uint32_t xd = threadIdx.x * kMergeVT;
  if (xd < len) {
    uint32_t ia = merge_corank(xd, la, lb, [&](uint32_t q) { return lin[q]; },
                               [&](uint32_t q) { return lin[la + q]; });
    uint32_t ib = xd - ia;
    uint32_t ka = ia < la ? lin[ia] : 0u, kb = ib < lb ? lin[la + ib] : 0u;
#pragma unroll
    for (int v = 0; v < kMergeVT; ++v) {
      const bool takea = ib >= lb || (ia < la && ka <= kb);
      x[v] = takea ? ka : kb;
      if (takea) {
        ++ia;
        ka = ia < la ? lin[ia] : 0u;
      } else {
        ++ib;
        kb = ib < lb ? lin[la + ib] : 0u;
      }
    }
#pragma unroll
    for (int v = 0; v < kMergeVT; ++v) {
      const uint32_t o = xd + v;
      if (o < len) lout[o + (o >> 5)] = x[v];
    }
  }
  __syncthreads();
  uint32_t* O = out + r.off[2 * i] + d0;
#pragma unroll
  for (int v = 0; v < kMergeVT; ++v) {
    const uint32_t q = threadIdx.x + 256 * v;
    if (q < len) O[q] = lout[q + (q >> 5)];
  }
}

// ---- one-round k-way merge ----------------------------------------------------------------
// The k <= 16 received runs are merged in ONE pass over HBM (read 4 B + write 4 B per key)
// instead of ceil(log2 k) 2-way rounds.  Total order: (key, run, index), i.e. ties go to the
// lower run (= global input order).
//   samples   every kMkSpacing-th element of every run (the decoded blocks' first keys)
//   bounds    each sample's rank among ALL samples (k binary searches in the runs' sample
//             lists, one lane per run); every kMkSPT-th sample in that merged order is a tile
//             boundary, and since a boundary is an element of the input, its exact co-rank in
//             run q is one binary search inside the kMkSpacing-wide window the sample rank
//             leaves: for runs before its own the count of keys <= it, for runs after it the
//             count of keys < it, for its own run its index
//   tiles     tile j = the elements between boundaries j and j + 1: at most (kMkSPT + k)
//             blocks of kMkSpacing elements (each run adds at most one partial block to its
//             samples in the range), loaded into LDS, merged in log2(k) 2-way rounds inside
//             LDS (merge path per thread, ties to the lower group), written out contiguously
constexpr int kMkSpacing = kCodecBlock;
constexpr int kMkSPT = 16;
constexpr int kMkMaxTile = kMkSpacing * (kMkSPT + kMaxRanks);   // 8192
constexpr int kMkBlock = 1024;
constexpr int kMkVT = kMkMaxTile / kMkBlock;                      // 8 loads / stores per thread
// A tile holds at most (kMkSPT + k) blocks of kMkSpacing elements for k <= kMaxRanks runs (the
// boundaries are every kMkSPT-th sample, and each run adds at most one partial block), so the
// tile kernel's buffers must hold exactly that bound: changing kMaxRanks, kMkSPT or the block
// size without kMkMaxTile would otherwise truncate tiles.
static_assert(kMkMaxTile == kMkSpacing * (kMkSPT + kMaxRanks) && kMkVT * kMkBlock == kMkMaxTile,
              "k-way merge tile bound");
constexpr int kMkChunk = 8;                                       // outputs per merge step
constexpr int kMkStride = kMaxRanks;                              // co-rank row stride

struct MergeK {
  uint32_t k;                      // runs (1..kMaxRanks)
  uint32_t kp;                     // k rounded up to a power of two (lanes per sample)
  uint32_t off[kMaxRanks + 1];     // run q = in[off[q], off[q + 1])
  uint32_t sbase[kMaxRanks + 1];   // run q's samples = samp[sbase[q], sbase[q + 1])
};

__host__ __device__ __forceinline__ uint32_t mk_tiles(const MergeK& m) {
  return (m.sbase[m.k] + kMkSPT - 1) / kMkSPT;
}

__device__ __forceinline__ uint32_t mk_run_of(const MergeK& m, uint32_t s) {
  uint32_t p = 0;
  while (p + 1 < m.k && m.sbase[p + 1] <= s) ++p;
  return p;
}

// samp[s] = element kMkSpacing * (s - sbase[p]) of run p
__global__ __launch_bounds__(256) void grs_mergek_samples(const uint32_t* __restrict__ in,
                                                          const MergeK m,
                                                          uint32_t* __restrict__ samp) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  if (s >= m.sbase[m.k]) return;
  const uint32_t p = mk_run_of(m, s);
  samp[s] = in[m.off[p] + (s - m.sbase[p]) * kMkSpacing];
}

// First index i in [lo, hi) of a[] where key <= v (LE) / key < v (!LE) fails; the predicate
// holds before lo.
template <bool LE>
__device__ __forceinline__ uint32_t mk_search(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t v) {
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t x = a[mid];
    if (LE ? x <= v : x < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// kp lanes per sample: lane q resolves run q.  corank[j * kMkStride + q] = elements of run q
// before tile j's first element; row mk_tiles(m) = the run lengths.
__global__ __launch_bounds__(256) void grs_mergek_bounds(const uint32_t* __restrict__ in,
                                                         const MergeK m,
                                                         const uint32_t* __restrict__ samp,
                                                         uint32_t* __restrict__ corank) {
  // grid: (samples + 1) * kp threads; a lane group (kp lanes of one wave) shares its sample
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
  const uint32_t s = tid / m.kp, q = tid % m.kp;
  const uint32_t ns = m.sbase[m.k];
  if (s > ns) return;
  if (s == ns) {   // the end row
    if (q < m.k) corank[static_cast<size_t>(mk_tiles(m)) * kMkStride + q] = m.off[q + 1] - m.off[q];
    return;
  }
  const uint32_t p = mk_run_of(m, s);
  const uint32_t mi = s - m.sbase[p];
  const uint32_t v = samp[s];
  uint32_t rank = 0;
  if (q < m.k) {
    const uint32_t* sq = samp + m.sbase[q];
    const uint32_t nq = m.sbase[q + 1] - m.sbase[q];
    rank = q == p ? mi : q < p ? mk_search<true>(sq, 0, nq, v) : mk_search<false>(sq, 0, nq, v);
  }
  uint32_t r = rank;
  for (uint32_t o = 1; o < m.kp; o <<= 1) r += __shfl_xor(r, o, GRS_WAVE);
  if (r % kMkSPT != 0 || q >= m.k) return;
  uint32_t c;
  if (q == p) {
    c = mi * kMkSpacing;
  } else {
    const uint32_t len = m.off[q + 1] - m.off[q];
    const uint32_t lo = rank ? (rank - 1) * kMkSpacing + 1 : 0;
    const uint32_t hi = rank ? min(rank * kMkSpacing, len) : 0;
    const uint32_t* rq = in + m.off[q];
    c = q < p ? mk_search<true>(rq, lo, hi, v) : mk_search<false>(rq, lo, hi, v);
  }
  corank[static_cast<size_t>(r / kMkSPT) * kMkStride + q] = c;
}

// LDS address of tile element x: one pad word per 8 (a lane's 8-output chunk starts 9 words
// after its neighbour's: the chunk writes of a wave hit 64 different banks)
__device__ __forceinline__ uint32_t mk_pad(uint32_t x) { return x + (x >> 3); }

// One workgroup per tile (2 per CU: 2 x 72 KB of LDS, 32 waves).
__global__ __launch_bounds__(kMkBlock, 2) void grs_mergek_tiles(const uint32_t* __restrict__ in,
                                                                uint32_t* __restrict__ out,
                                                                const MergeK m,
                                                                const uint32_t* __restrict__ corank) {
  constexpr uint32_t PADN = kMkMaxTile + kMkMaxTile / 8;
  __shared__ uint32_t buf[2][PADN];
  __shared__ uint32_t P[kMaxRanks + 1];    // segment starts in the tile (kp segments, padded)
  __shared__ uint32_t S[kMaxRanks];        // segment starts in the runs
  __shared__ uint32_t O0;
  const uint32_t j = blockIdx.x, t = threadIdx.x;
  if (t < GRS_WAVE) {   // wave 0: lane q loads run q's two co-ranks (one round trip), DPP scans
    const uint32_t c0 = t < m.k ? corank[static_cast<size_t>(j) * kMkStride + t] : 0u;
    const uint32_t c1 = t < m.k ? corank[static_cast<size_t>(j + 1) * kMkStride + t] : 0u;
    const uint32_t l = c1 - c0;
    const uint32_t li = wave_scan_dpp(l), oi = wave_scan_dpp(c0);
    if (t <= m.kp) P[t] = li - l;   // lanes past k hold l = 0: P[kp] = the tile's length
    if (t < m.kp) S[t] = m.off[min(t, m.k)] + c0;
    if (t == GRS_WAVE - 1) O0 = oi;
  }
  __syncthreads();
  // <= kMkMaxTile by construction (static_assert above); the min only keeps a corrupt co-rank
  // table inside the LDS buffers
  const uint32_t len = min(P[m.kp], static_cast<uint32_t>(kMkMaxTile));
  // the tile's segments, all loads in flight, then LDS
  uint32_t x[kMkVT];
  uint32_t q = 0;   // segment of element e (e grows with v)
#pragma unroll
  for (int v = 0; v < kMkVT; ++v) {
    const uint32_t e = t + kMkBlock * v;
    x[v] = 0;
    if (e < len) {
      while (q + 1 < m.kp && P[q + 1] <= e) ++q;
      x[v] = in[S[q] + (e - P[q])];
    }
  }
#pragma unroll
  for (int v = 0; v < kMkVT; ++v) {
    const uint32_t e = t + kMkBlock * v;
    if (e < len) buf[0][mk_pad(e)] = x[v];
  }
  __syncthreads();
  // log2(kp) rounds; round w merges segment groups [g, g + w) and [g + w, g + 2w) in chunks of
  // kMkChunk outputs: a chunk's merge-path co-rank, kMkChunk candidates from each side (all
  // loads in flight), one 2 kMkChunk-element bitonic merge in registers, its first outputs.  (The values are
  // bare keys: which of two equal keys lands first cannot be told apart.)
  uint32_t cur = 0;
  for (uint32_t w = 1; w < m.kp; w <<= 1) {
    const uint32_t* src = buf[cur];
    uint32_t* dst = buf[cur ^ 1];
    const uint32_t npairs = m.kp / (2 * w);
    for (uint32_t c = t;; c += kMkBlock) {
      uint32_t acc = 0, a0 = 0, b0 = 0, b1 = 0;
      bool found = false;
      for (uint32_t g = 0; g < npairs; ++g) {
        a0 = P[2 * g * w];
        b0 = P[2 * g * w + w];
        b1 = P[2 * g * w + 2 * w];
        const uint32_t nch = (b1 - a0 + kMkChunk - 1) / kMkChunk;
        if (c < acc + nch) {
          found = true;
          break;
        }
        acc += nch;
      }
      if (!found) break;
      const uint32_t d = (c - acc) * kMkChunk;
      const uint32_t al = b0 - a0, bl = b1 - b0;
      const uint32_t nout = min(static_cast<uint32_t>(kMkChunk), al + bl - d);
      const uint32_t ia = merge_corank(d, al, bl, [&](uint32_t i) { return src[mk_pad(a0 + i)]; },
                                       [&](uint32_t i) { return src[mk_pad(b0 + i)]; });
      const uint32_t ib = d - ia;
      constexpr int C = kMkChunk;
      uint32_t v[2 * C];
#pragma unroll
      for (int i = 0; i < C; ++i) {
        v[i] = ia + i < al ? src[mk_pad(a0 + ia + i)] : 0xFFFFFFFFu;
        v[2 * C - 1 - i] = ib + i < bl ? src[mk_pad(b0 + ib + i)] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int st = C; st >= 1; st >>= 1) {
#pragma unroll
        for (int i = 0; i < 2 * C; ++i) {
          if ((i & st) == 0) {
            const uint32_t lo = min(v[i], v[i + st]), hi = max(v[i], v[i + st]);
            v[i] = lo;
            v[i + st] = hi;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < C; ++i)
        if (static_cast<uint32_t>(i) < nout) dst[mk_pad(a0 + d + i)] = v[i];
    }
    __syncthreads();
    cur ^= 1;
  }
  uint32_t* o = out + O0;
#pragma unroll
  for (int v = 0; v < kMkVT; ++v) {
    const uint32_t e = t + kMkBlock * v;
    if (e < len) o[e] = buf[cur][mk_pad(e)];
  }
}

}  // namespace grs
