// grs_msd.hpp — the MSD-first u32 sort and the segment-table kernels of libgrs (gfx950).
//
// The reference sorts with 32 stable one-bit LSD splits (ParallelSort.cpp:236-298), and the
// LSD path of this library (grs_pass.hpp) with 4 stable 8-bit scatter passes.  A scatter pass
// costs what its digit runs cost: 256 runs per tile, the boundary lines two tiles share, 0.56
// of 8 TB/s at the floor of its own loads and stores.  For u32 keys, two
// stable MSD scatters already sort the keys by their top 16 bits into 65536 segments of
// ~n / 65536 keys, which one workgroup can finish in LDS with contiguous HBM traffic:
//
//   H1  grs_upfront_hist2<.., QN = 1>   top-byte histogram (one LDS add per key)
//   P1  grs_onesweep_v4                 stable scatter by bits 24..31          keys -> alt
//   H2  grs_msd_hist2                   per top-byte bucket, the byte-2 histogram (65536 bins)
//                                       over P1's output (a block meets 1-2 buckets: LDS);
//                                       block 0 also plans P2's tiles (grs_seg_plan_block)
//   P2  grs_onesweep_seg                stable scatter by bits 16..23 inside each bucket
//                                                                              alt -> keys
//   P3  grs_msd_local                   one workgroup per 16-bit prefix: its keys read once,
//                                       sorted by bits 0..15 in LDS (two lane-ordered 8-bit
//                                       rounds, as the pass ranks), written once, in place
//
// Stable scatters and a stable LDS sort: equal keys keep their input order, so the output is
// the reference's (the stable sort by key).  A 16-bit segment longer than P3's LDS capacity is
// appended to a list instead, and sorted by a segmented LSD on bits 0..15 over the listed
// segments only (grs_seg_plan -> grs_seg_hist -> 2 x grs_onesweep_seg, persistent grids that
// leave at once when the list is empty): skewed inputs stay correct and pay only for the
// segments that need it.
#pragma once

#include "grs_kernels.hpp"
#include "grs_pass.hpp"

namespace grs {

// ---------------------------------------------------------------------------------------
// segment tables: one SegTile per tile of a segmented pass
// ---------------------------------------------------------------------------------------
// Segment sources of a plan: sizes (starts are their exclusive scan: the buckets of a pass),
// explicit (start, length) lists, or offsets (num + 1 words, segment i = [off[i], off[i+1])).
// kSegOffsetsAll: offsets, every segment's histogram row = its index (tables per segment).
enum SegSource : int { kSegSizes = 0, kSegList = 1, kSegOffsets = 2, kSegMoved = 3, kSegOffsetsAll = 4 };

// LDS of the planner: 6 words per segment (tile, row and group prefixes, start, length,
// histogram row); larger tables keep them in global scratch (`spill`, 6 * (nseg + 1) words).
#define GRS_PLAN_LDS_SEGS 2048
#define GRS_H2_PIECE_LOG 8   // keys of one piece of H2's sample, log2 (grs_msd_hist2)
#ifndef GRS_P3_LDS_LAYOUT   // P3's LDS positions (LocalSort::swz_t): 0 plain, 1 XOR swizzle, 2 padded
#define GRS_P3_LDS_LAYOUT 1
#endif
#define GRS_PLAN_LDS_WORDS (6 * GRS_PLAN_LDS_SEGS + 5 * 16)

// Block exclusive scan of NV values per thread over BLOCK threads (wsum: NV * waves words of
// LDS); tot = the block totals.
template <int BLOCK, int NV>
__device__ __forceinline__ void block_scan(uint32_t (&v)[NV], uint32_t* wsum, uint32_t (&tot)[NV]) {
  constexpr int W = BLOCK / GRS_WAVE;
  const uint32_t t = threadIdx.x, lane = t & (GRS_WAVE - 1), w = t >> 6;
  uint32_t inc[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    inc[q] = wave_scan_dpp(v[q]);
    if (lane == GRS_WAVE - 1) wsum[q * W + w] = inc[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    uint32_t p = 0;
    tot[q] = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const uint32_t x = wsum[q * W + k];
      p += static_cast<uint32_t>(k) < w ? x : 0u;
      tot[q] += x;
    }
    v[q] = p + inc[q] - v[q];
  }
  __syncthreads();   // wsum is reused by the next call
}

// One block (BLOCK threads) plans a segmented pass of TILE-key tiles: for every ticket, the
// tile's place (SegTile) -- tiles in segment order; a segment of several tiles gets status rows
// and starts new look-back groups, a segment of one tile is solo (no status words).
// Sources: kSegSizes a = sizes (starts = their scan; histogram row = segment index);
// kSegList a = starts, b = lengths, c = histogram rows; kSegOffsets a = offsets (histogram row =
// the segment's place among the segments of several tiles: solo segments need none);
// kSegMoved a = where each segment's keys are read, b = lengths, c = where its sorted runs go
// (histogram row = segment index).  hdr[0] = tiles, hdr[1] = groups, hdr[2] =
// status rows.  room (nullable): the records' seg_len = room[i] instead of the segment's length
// (a region pass: the room its runs may take).
// lds: GRS_PLAN_LDS_WORDS words.
template <uint32_t TILE, int BLOCK, int SRC>
__device__ void seg_plan_block(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                               const uint32_t* __restrict__ c, uint32_t nseg,
                               uint32_t* __restrict__ spill, SegTile* __restrict__ rec,
                               uint32_t* __restrict__ hdr, uint32_t* lds,
                               const uint32_t* __restrict__ room = nullptr) {
  constexpr uint32_t G = GRS_LB_GROUP;
  const uint32_t t = threadIdx.x;
  const bool in_lds = nseg < GRS_PLAN_LDS_SEGS;
  uint32_t* const tpre = in_lds ? lds : spill;
  const uint32_t cap = in_lds ? GRS_PLAN_LDS_SEGS : nseg + 1;
  uint32_t* const rpre = tpre + cap;
  uint32_t* const gpre = rpre + cap;
  uint32_t* const sst = gpre + cap;
  uint32_t* const sln = sst + cap;
  uint32_t* const shr = sln + cap;   // histogram row; kSegMoved: the output start
  uint32_t* const wsum = lds + 6 * GRS_PLAN_LDS_SEGS;
  uint32_t carry[5] = {0, 0, 0, 0, 0};   // tiles, rows, groups, start (sizes), multi ordinal
  for (uint32_t c0 = 0; c0 < nseg; c0 += BLOCK) {
    const uint32_t i = c0 + t;
    uint32_t len = 0, st = 0, hr = i;
    if (i < nseg) {
      if constexpr (SRC == kSegSizes) {
        len = a[i];
      } else if constexpr (SRC == kSegList || SRC == kSegMoved) {
        st = a[i];
        len = b[i];
        hr = c[i];
      } else {
        st = a[i];
        len = a[i + 1] - st;
      }
    }
    const uint32_t tl = len / TILE + (len % TILE != 0u ? 1u : 0u);
    const uint32_t multi = tl > 1 ? tl : 0u;
    uint32_t v[5] = {tl, multi, (multi + G - 1) / G, len, multi ? 1u : 0u}, tot[5];
    block_scan<BLOCK, 5>(v, wsum, tot);
    if (i < nseg) {
      tpre[i] = carry[0] + v[0];
      rpre[i] = carry[1] + v[1];
      gpre[i] = carry[2] + v[2];
      sst[i] = SRC == kSegSizes ? carry[3] + v[3] : st;
      sln[i] = len;
      shr[i] = SRC == kSegOffsets ? carry[4] + v[4] : hr;   // kSegOffsetsAll: hr = i
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) carry[q] += tot[q];
  }
  if (t == 0) tpre[nseg] = carry[0];
  __syncthreads();
  const uint32_t tiles = carry[0];
  for (uint32_t tk = t; tk < tiles; tk += BLOCK) {
    uint32_t lo = 0, hi = nseg;   // the largest i with tpre[i] <= tk (a non-empty segment)
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (tpre[mid] <= tk) lo = mid; else hi = mid;
    }
    const uint32_t j = tk - tpre[lo];
    const uint32_t tl = tpre[lo + 1] - tpre[lo];
    const uint32_t len = sln[lo];
    const uint32_t q = j / G;
    const uint32_t flags = (j % G) | (min(G, tl - q * G) << 4) | ((tl == 1 ? 1u : 0u) << 8) | (q << 9) |
                           (j + 1 == tl ? 0x80000000u : 0u);
    const uint32_t out = SRC == kSegMoved ? shr[lo] : sst[lo];
    rec[tk] = SegTile{rpre[lo] + j, gpre[lo] + q, flags, sst[lo] + j * TILE, min(TILE, len - j * TILE),
                      out, room != nullptr ? room[lo] : len, SRC == kSegMoved ? lo : shr[lo]};
  }
  if (t == 0) {
    hdr[0] = tiles;
    hdr[1] = carry[2];
    hdr[2] = carry[1];
  }
}

// Stand-alone planner (one block): nseg from the host, or from *nseg_dev when non-null.
template <uint32_t TILE, int SRC>
__global__ __launch_bounds__(1024) void grs_seg_plan(const uint32_t* __restrict__ a,
                                                     const uint32_t* __restrict__ b,
                                                     const uint32_t* __restrict__ c,
                                                     uint32_t nseg_host,
                                                     const uint32_t* __restrict__ nseg_dev,
                                                     uint32_t* __restrict__ spill,
                                                     SegTile* __restrict__ rec,
                                                     uint32_t* __restrict__ hdr) {
  __shared__ uint32_t lds[GRS_PLAN_LDS_WORDS];
  const uint32_t nseg = nseg_dev != nullptr ? *nseg_dev : nseg_host;
  seg_plan_block<TILE, 1024, SRC>(a, b, c, nseg, spill, rec, hdr, lds);
}

// Per-segment digit histograms of a segment table's keys: rows[seg * ND * 256 + p * 256 + d]
// counts digit d (bits [shift0 + 8p, +8)) of the segment's keys, p < ND (rows zeroed by the
// caller).  Solo segments (one tile) are skipped: their pass counts them itself.  Persistent
// grid over the plan's tiles; also zeroes the status words of the first segmented pass
// (`zero`, rows of `radix` words; the layout is known only from the plan).
// shift_dev (nullable): digit p is bits [*shift_dev + shift0 + 8p, +8) (a shift found on the device).
template <typename K, int ND>
__global__ __launch_bounds__(256) void grs_seg_hist(const K* __restrict__ keys,
                                                    const SegTile* __restrict__ rec,
                                                    const uint32_t* __restrict__ hdr, int shift0,
                                                    uint32_t* __restrict__ rows,
                                                    uint32_t* __restrict__ zero, uint32_t radix,
                                                    const uint32_t* __restrict__ shift_dev = nullptr) {
  __shared__ uint32_t h[ND * 256];
  const uint32_t t = threadIdx.x;
  const uint32_t tiles = hdr[0];
  if (shift_dev != nullptr) shift0 += static_cast<int>(__builtin_amdgcn_readfirstlane(*shift_dev));
  const size_t zw = static_cast<size_t>(hdr[2] + 2 * hdr[1]) * radix;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + t; i < zw; i += static_cast<size_t>(gridDim.x) * 256)
    zero[i] = 0;
  for (uint32_t k = blockIdx.x; k < tiles; k += gridDim.x) {
    const SegTile r = rec[k];
    if ((r.flags >> 8) & 1u) continue;   // solo (uniform: one record per workgroup)
    for (uint32_t i = t; i < ND * 256; i += 256) h[i] = 0;
    __syncthreads();
    // U loads in flight per thread before any is counted (a tile is 17-36K keys: 8-18 each)
    constexpr uint32_t U = 8;
    for (uint32_t i0 = t; i0 < r.valid; i0 += 256 * U) {
      K x[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * 256;
        x[u] = i < r.valid ? keys[r.base + i] : K(0);
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (i0 + u * 256 < r.valid) {
#pragma unroll
          for (int p = 0; p < ND; ++p)
            atomicAdd(&h[p * 256 + static_cast<uint32_t>((x[u] >> (shift0 + 8 * p)) & 255u)], 1u);
        }
      }
    }
    __syncthreads();
    for (uint32_t i = t; i < ND * 256; i += 256)
      if (h[i] != 0u) atomicAdd(&rows[static_cast<size_t>(r.seg) * ND * 256 + i], h[i]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// MSD u32 sort: H2 and P3
// ---------------------------------------------------------------------------------------
#define GRS_H2_CHUNK 262144
#define GRS_H2_COPIES 32
#ifndef GRS_H2_INFLIGHT
#define GRS_H2_INFLIGHT 8   // 16-B loads in flight per thread in H2
#endif
#define GRS_MSD_SAMPLE_CHUNKS 16384   // 64-key chunks the sample reads (2^20 keys)
#define GRS_MSD_GUESS_CHUNKS 64       // 64-key chunks every sample block reads for the span guess

// The MSD sort's span words in the call's control block (zeroed by the previous call):
// [0..1] OR of the keys (lo, hi), [2..3] OR of their complements, [4] the top digit's shift.
#define GRS_MSD_SPAN 1024

// The top digit of the MSD sort: the byte whose highest bit is the keys' highest VARYING bit
// (varying = OR(keys) & OR(~keys): bits that are not the same in every key), between bits
// [8, 16) and the key's top byte.  Bits above it are equal in every key, so sorting by bits
// [0, shift + 8) sorts the keys: the two scatters take bits [shift - 8, shift + 8) and the LDS
// sort the bits below (the reference's own input, a shuffled 0..n-1 (main.cpp:119-125), varies
// in its low log2(n) bits only; the top byte would leave 16 buckets at n = 2^28).
template <typename K>
__host__ __device__ inline uint32_t msd_top_shift(K varying) {
  constexpr int KB = 8 * static_cast<int>(sizeof(K));
  int hb = -1;
  for (int b = KB - 1; b >= 0; --b)
    if ((varying >> b) & K(1)) {
      hb = b;
      break;
    }
  const int s = hb - 7;
  return static_cast<uint32_t>(s < 8 ? 8 : s > KB - 8 ? KB - 8 : s);
}
template <typename K>
__device__ __forceinline__ K span_join(uint32_t lo, uint32_t hi) {
  if constexpr (sizeof(K) == 8) return (static_cast<K>(hi) << 32) | lo;
  else return static_cast<K>(lo);
}
// LDS rounds of P3 for top shift s: the bits below the 16-bit segment prefix, [0, s - 8)
template <int RMAX>
__device__ __forceinline__ int msd_p3_rounds(uint32_t s) {
  const int r = (static_cast<int>(s) - 8 + 7) / 8;
  return r < 1 ? 1 : r > RMAX ? RMAX : r;
}

// S: the top digit's histogram from an evenly spaced sample of 64-key chunks (all keys when
// n <= 64 * chunks), added into samp[256] (zero); also does the clearing the LSD sort's
// histogram kernel does (P1's status, the next call's control block) plus clear2 (h2 and the
// big-segment counters).  The digit's shift is a guess from GRS_MSD_GUESS_CHUNKS evenly spaced
// chunks that every block reads (so all blocks agree without communicating); block 0 writes it
// to span[4] for P1, whose tiles then find the exact span (grs_msd_span checks the guess).
template <typename K>
__global__ __launch_bounds__(256) void grs_msd_sample(const K* __restrict__ keys, uint32_t n,
                                                      uint32_t* __restrict__ samp,
                                                      uint32_t* __restrict__ clear, uint32_t clear_words,
                                                      uint32_t* __restrict__ clear_ctrl,
                                                      uint32_t* __restrict__ clear2, uint32_t clear2_words,
                                                      uint32_t* __restrict__ span) {
  __shared__ uint32_t h[256];
  __shared__ uint32_t sv[4];
  const uint32_t t = threadIdx.x, lane = t & (GRS_WAVE - 1);
  h[t] = 0;
  if (t < 4) sv[t] = 0;
  // the guess's keys first (16 per thread, in flight together)
  constexpr uint32_t GC = GRS_MSD_GUESS_CHUNKS, GK = GC * GRS_WAVE / 256;
  K g[GK];
#pragma unroll
  for (uint32_t u = 0; u < GK; ++u) {
    const uint32_t i = u * 256 + t;
    const uint32_t pos = n <= GC * GRS_WAVE
                             ? i
                             : static_cast<uint32_t>(static_cast<uint64_t>(i >> 6) * (n - GRS_WAVE) / (GC - 1)) + (i & 63u);
    g[u] = i < n ? keys[pos] : K(0);
  }
  const uint32_t gs = gridDim.x * 256;
  // the clears in 16-B stores (22 MB of P1's look-back words at 2^30: a dword a lane took most
  // of this kernel's 20 us); the buffers are 16-B aligned, the tails word by word
  auto zero16 = [&](uint32_t* p, uint32_t words) {
    uint4* const q = reinterpret_cast<uint4*>(p);
    const uint32_t nv = words / 4;
    for (uint32_t i = blockIdx.x * 256 + t; i < nv; i += gs) q[i] = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t i = nv * 4 + blockIdx.x * 256 + t; i < words; i += gs) p[i] = 0;
  };
  zero16(clear, clear_words);
  zero16(clear2, clear2_words);
  constexpr uint32_t H = GRS_CTRL_HIST_WORDS, TK = GRS_MAX_PASSES * GRS_XCDS;
  zero16(clear_ctrl, H + TK);
  K o = 0, no = 0;
#pragma unroll
  for (uint32_t u = 0; u < GK; ++u)
    if (u * 256 + t < n) {
      o |= g[u];
      no |= static_cast<K>(~g[u]);
    }
  uint32_t v[4] = {static_cast<uint32_t>(o), static_cast<uint32_t>(static_cast<uint64_t>(o) >> 32),
                   static_cast<uint32_t>(no), static_cast<uint32_t>(static_cast<uint64_t>(no) >> 32)};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) v[q] |= __shfl_xor(v[q], s);
  }
  __syncthreads();   // h and sv zeroed
  if (lane == 0)
    for (int q = 0; q < 4; ++q) atomicOr(&sv[q], v[q]);
  __syncthreads();
  const uint32_t top = msd_top_shift<K>(span_join<K>(sv[0], sv[1]) & span_join<K>(sv[2], sv[3]));
  if (blockIdx.x == 0 && t == 0) span[4] = top;
  auto bin = [&](K k) { return static_cast<uint32_t>(k >> top) & 255u; };
  constexpr uint32_t C = GRS_MSD_SAMPLE_CHUNKS;
  if (n <= C * GRS_WAVE) {
    for (uint32_t i0 = blockIdx.x * 256 + t; i0 < n; i0 += 4 * gs) {   // four loads in flight
      K x[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) x[u] = i0 + u * gs < n ? keys[i0 + u * gs] : K(0);
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u)
        if (i0 + u * gs < n) atomicAdd(&h[bin(x[u])], 1u);
    }
  } else {
    // every wave's chunks loaded before any is counted (the loads overlap): one block per CU, 16
    // chunks per wave in flight (1024 blocks adding 256 counts each into the same 256 words cost
    // 24 us at 2^28 under the profiler, round 5)
    constexpr uint32_t U = 16;
    const uint32_t waves = gridDim.x * 4;
    for (uint32_t c0 = blockIdx.x * 4 + (t >> 6); c0 < C; c0 += U * waves) {
      K k[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t c = c0 + u * waves;
        const uint32_t pos = static_cast<uint32_t>(static_cast<uint64_t>(c) * (n - GRS_WAVE) / (C - 1));
        k[u] = c < C ? keys[pos + lane] : K(0);
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u)
        if (c0 + u * waves < C) atomicAdd(&h[bin(k[u])], 1u);
    }
  }
  __syncthreads();
  if (h[t] != 0u) atomicAdd(&samp[t], h[t]);
}

// After P1 (one block): the exact span (P1's tiles ORed every key into span[0..3]) fixes the top
// digit's shift.  A shift above the sample's guess (a varying bit the guess missed) or a run
// that outgrew its region (totals[256], set by P1) plans the redo: P1 again with exact counts at
// the exact shift, the whole input as one segment of TILEF-key tiles (grs_seg_hist and a
// persistent grs_onesweep_seg), and sets totals[256] so that the plans downstream take the
// exact layout; an empty plan otherwise (the redo's launches leave at once).
template <typename K, uint32_t TILEF>
__global__ __launch_bounds__(256) void grs_msd_span(uint32_t n, uint32_t* __restrict__ span,
                                                    uint32_t* __restrict__ totals,
                                                    SegTile* __restrict__ rec, uint32_t* __restrict__ hdr) {
  __shared__ uint32_t tiles;
  const uint32_t t = threadIdx.x;
  if (t == 0) {
    const uint32_t sx = msd_top_shift<K>(span_join<K>(span[0], span[1]) & span_join<K>(span[2], span[3]));
    bool redo = totals[256] != 0u;
    if (sx != span[4]) {
      span[4] = sx;
      totals[256] = 1u;
      redo = true;
    }
    tiles = redo ? n / TILEF + (n % TILEF != 0u ? 1u : 0u) : 0u;
  }
  __syncthreads();
  constexpr uint32_t G = GRS_LB_GROUP;
  const uint32_t T = tiles;
  for (uint32_t k = t; k < T; k += 256) {
    const uint32_t q = k / G;
    const uint32_t flags = (k % G) | (min(G, T - q * G) << 4) | ((T == 1 ? 1u : 0u) << 8) | (q << 9) |
                           (k + 1 == T ? 0x80000000u : 0u);
    rec[k] = SegTile{k, q, flags, k * TILEF, min(TILEF, n - k * TILEF), 0u, n, 0u};
  }
  if (t == 0) {
    hdr[0] = T;
    hdr[1] = T > 1 ? (T + G - 1) / G : 0u;
    hdr[2] = T > 1 ? T : 0u;
  }
}

// The top-byte bucket table after P1: in[s] = where bucket s's keys lie in alt, len[s] = its
// keys, out[s] = where its sorted keys go, cpre[s] = H2 chunks of `chunk` keys before bucket s
// (cpre[256] = all).  P1's regions when no run outgrew its region (totals[256] == 0), the redone exact
// layout otherwise.  One block computes it into LDS (in, len, out, cpre: 4 x 257 words).
__device__ void msd_bucket_table(const uint32_t* __restrict__ samp, unsigned long long mult,
                                 uint32_t pad, const uint32_t* __restrict__ totals,
                                 const uint32_t* __restrict__ exact, uint32_t chunk, uint32_t* in,
                                 uint32_t* len, uint32_t* out, uint32_t* cpre, uint32_t* wsum) {
  const uint32_t t = threadIdx.x;   // blockDim == 1024
  const bool redo = totals[256] != 0u;
  uint32_t v[3] = {0, 0, 0}, tot[3];
  if (t < 256) {
    const uint32_t l = redo ? exact[t] : totals[t];
    const uint32_t r = redo ? l : static_cast<uint32_t>((static_cast<unsigned long long>(samp[t]) * mult) >> 20) + pad;
    v[0] = l;
    v[1] = r;
    v[2] = (l + chunk - 1) / chunk;
    len[t] = l;
  }
  block_scan<1024, 3>(v, wsum, tot);
  if (t < 256) {
    out[t] = v[0];
    in[t] = v[1];
    cpre[t] = v[2];
  }
  if (t == 0) cpre[256] = tot[2];
  __syncthreads();
}

// The plan of P2 (one block): the bucket table (tab: in | len | out | cpre, 4 x 257 words, for
// H2) and P2's tiles (bucket s read at in[s], its runs written from out[s]).
template <uint32_t TILE2>
__global__ __launch_bounds__(1024) void grs_msd_plan2(const uint32_t* __restrict__ samp,
                                                      unsigned long long mult, uint32_t pad,
                                                      const uint32_t* __restrict__ totals,
                                                      const uint32_t* __restrict__ exact,
                                                      uint32_t chunk, uint32_t* __restrict__ tab,
                                                      SegTile* __restrict__ rec2,
                                                      uint32_t* __restrict__ hdr2, uint32_t with_records = 1) {
  __shared__ uint32_t lds[GRS_PLAN_LDS_WORDS + 4 * 257 + 64];
  uint32_t* const in = lds + GRS_PLAN_LDS_WORDS;
  uint32_t* const len = in + 257;
  uint32_t* const out = len + 257;
  uint32_t* const cpre = out + 257;
  uint32_t* const wsum = cpre + 257;
  msd_bucket_table(samp, mult, pad, totals, exact, chunk, in, len, out, cpre, wsum);
  for (uint32_t i = threadIdx.x; i < 4 * 257; i += 1024) tab[i] = in[i];
  // (with_records 0, a sampled P2: its exact tiles are planned by the gated exact H2 only when
  // a region overflows -- the record loop was most of this kernel's 21 us at 2^30)
  if (with_records != 0u) seg_plan_block<TILE2, 1024, kSegMoved>(in, len, out, 256u, nullptr, rec2, hdr2, lds);
}

// H2: h2[(top byte) * 256 + byte 2] over P1's output, one chunk of one bucket per block (grid
// >= n / chunk + 256; tab from grs_msd_plan2 with the same chunk: 256K keys at 2^30, fewer
// below so the grid is several resident rounds, not 2.5 with a tail); zeroes `zero_words` of
// `zero` (P2's status).  Two 1024-thread blocks per CU (8 waves per SIMD).  (P1 writing the
// sample itself, the byte below its digit at one output position in 16 or in whole 1024-position
// windows, cost P1 230 us at 2^30 for the 110 us it saved here: round 6)
template <typename K, uint32_t TILE2 = 0>
__global__ __launch_bounds__(1024, TILE2 != 0 ? 4 : 8) void grs_msd_hist2(const K* __restrict__ keys,
                                                         uint32_t* __restrict__ h2,
                                                         uint32_t* __restrict__ zero,
                                                         uint32_t zero_words,
                                                         const uint32_t* __restrict__ tab, uint32_t chunk,
                                                         uint32_t sample_shift = 0,
                                                         const uint32_t* __restrict__ gate = nullptr,
                                                         const uint32_t* __restrict__ top_shift = nullptr,
                                                         uint32_t piece_log = 8,
                                                         SegTile* __restrict__ rec2 = nullptr,
                                                         uint32_t* __restrict__ hdr2 = nullptr) {
  constexpr uint32_t B = 1024;
  constexpr uint32_t LW = 256 * GRS_H2_COPIES;
  __shared__ __attribute__((aligned(16))) uint32_t h[LW];
  __shared__ uint32_t cpre[257];
  const uint32_t t = threadIdx.x;
  if (gate != nullptr && __builtin_amdgcn_readfirstlane(*gate) == 0u) return;   // (the exact redo)
  for (uint32_t i = blockIdx.x * B + t; i < zero_words; i += gridDim.x * B) zero[i] = 0;
  if constexpr (TILE2 != 0) {
    // the exact redo after a sampled P2: the last block (never one of the chunks: the grid has
    // 256 more blocks than n / chunk) plans the exact pass's tiles from tab's in / len / out,
    // which grs_msd_plan2 skipped
    __shared__ uint32_t plan_lds[GRS_PLAN_LDS_WORDS];
    if (blockIdx.x == gridDim.x - 1) {
      seg_plan_block<TILE2, 1024, kSegMoved>(tab, tab + 257, tab + 2 * 257, 256u, nullptr, rec2, hdr2, plan_lds);
      return;
    }
  }
  for (uint32_t i = t; i < LW; i += B) h[i] = 0;
  if (t < 257) cpre[t] = tab[3 * 257 + t];
  __syncthreads();
  const uint32_t b = blockIdx.x;
  if (b >= cpre[256]) return;
  uint32_t lo = 0, hi = 256;   // the largest s with cpre[s] <= b
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cpre[mid] <= b) lo = mid; else hi = mid;
  }
  const uint32_t s = lo, j = b - cpre[s];
  const uint32_t c0 = tab[s] + j * chunk;
  const uint32_t cl = min(chunk, tab[257 + s] - j * chunk);
  uint32_t* const base = h + (t & (GRS_H2_COPIES - 1));
  // the byte below the top digit (top_shift: the MSD sort's shift found on the device)
  const int SH = top_shift != nullptr ? static_cast<int>(__builtin_amdgcn_readfirstlane(*top_shift)) - 8
                                      : 8 * static_cast<int>(sizeof(K)) - 16;
  auto count = [&](K k) {
    atomicAdd(base + (static_cast<uint32_t>(k >> SH) & 255u) * GRS_H2_COPIES, 1u);
  };
  auto flush = [&]() {
    __syncthreads();
    if (t < 256) {
      const uint32_t* row = h + t * GRS_H2_COPIES;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < GRS_H2_COPIES; ++k) c += row[(k + t) & (GRS_H2_COPIES - 1)];
      if (c != 0) atomicAdd(&h2[s * 256 + t], c);
    }
  };
  constexpr uint32_t VEC = 16 / sizeof(K);
  const K* kc = keys + c0;
  // 16-B loads from the first aligned key on
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(kc) & 15u) / sizeof(K);
  const uint32_t head = min(cl, (VEC - mis) % VEC);
  const uint32_t nv = (cl - head) / VEC;
  const uint4* kv = reinterpret_cast<const uint4*>(kc + head);
  auto count4 = [&](const uint4& x) {
    const K* e = reinterpret_cast<const K*>(&x);
#pragma unroll
    for (uint32_t q = 0; q < VEC; ++q) count(e[q]);
  };
  if (sample_shift != 0) {
    // a sample: the first of every 2^sample_shift pieces of 2^piece_log keys (whatever the
    // input order, the pieces cover the chunk evenly); the bucket's scale is its length over its
    // sampled keys
    constexpr uint32_t VL = VEC == 4 ? 2 : 1;
    const uint32_t pul = piece_log - VL, PU = 1u << pul;   // 16-B loads per piece
    const uint32_t np = (nv + PU - 1) >> pul;
    const uint32_t ns = ((np + (1u << sample_shift) - 1) >> sample_shift) << pul;
    auto at = [&](uint32_t m) { return ((m >> pul) << (sample_shift + pul)) + (m & (PU - 1u)); };
    uint32_t m = t;
    // GRS_H2_INFLIGHT loads in flight per thread (a block's whole share in one or two rounds:
    // the loop is latency-bound, one at a time ran at 0.7 TB/s)
    constexpr int U = GRS_H2_INFLIGHT;
    for (; m + (U - 1) * B < ns; m += U * B) {
      uint4 x[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t v = at(m + u * B);
        ok[u] = v < nv;
        x[u] = kv[ok[u] ? v : 0u];   // (nv >= 1 here: ns > 0)
      }
      // every load issued before the first count (the scheduler otherwise pairs each load
      // with its wait and counts: one in flight)
#pragma unroll
      for (int u = 0; u < U; ++u) asm volatile("" ::"v"(x[u].x), "v"(x[u].y), "v"(x[u].z), "v"(x[u].w));
      // (the counts add 0 for a load past the chunk instead of branching round it: a branch
      // let the compiler sink each load into its branch and wait for it alone)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const K* e = reinterpret_cast<const K*>(&x[u]);
        const uint32_t one = ok[u] ? 1u : 0u;
#pragma unroll
        for (uint32_t q = 0; q < VEC; ++q)
          atomicAdd(base + (static_cast<uint32_t>(e[q] >> SH) & 255u) * GRS_H2_COPIES, one);
      }
    }
    for (; m < ns; m += B) {
      const uint32_t v = at(m);
      if (v < nv) count4(kv[v]);
    }
    flush();
    return;
  }
  if (t < head) count(kc[t]);
  uint32_t i = t;
  constexpr int U = GRS_H2_INFLIGHT;
  for (; i + (U - 1) * B < nv; i += U * B) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = kv[i + u * B];
#pragma unroll
    for (int u = 0; u < U; ++u) asm volatile("" ::"v"(x[u].x), "v"(x[u].y), "v"(x[u].z), "v"(x[u].w));
#pragma unroll
    for (int u = 0; u < U; ++u) count4(x[u]);
  }
  for (; i < nv; i += B) count4(kv[i]);
  for (uint32_t r = head + nv * VEC + t; r < cl; r += B) count(kc[r]);
  flush();
}

// The regions of P2 (one block of 256 per top-byte bucket s, a thread per byte-2 bin b), from
// the sampled byte-2 counts hs (H2 with a sample_shift) so that P2 needs no counting read of
// P1's output: the region of bin (s, b) holds its estimate c * scale (scale = the bucket's
// length over its sampled keys) + 6 standard errors (scale * sqrt(c + 1)) + 64, at most the
// bucket's length (a bucket with no sampled key: every bin its length).  reg[s * 256 + b] = the
// region (P2's "histogram" rows), room[s] = the bucket's total.
__global__ __launch_bounds__(256) void grs_msd_regions(const uint32_t* __restrict__ tab,
                                                       const uint32_t* __restrict__ hs,
                                                       uint32_t* __restrict__ reg, uint32_t* __restrict__ room) {
  __shared__ uint32_t wsum[4];
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  const uint32_t c = hs[s * 256 + t];
  uint32_t v[1] = {c}, ts[1];
  block_scan<256, 1>(v, wsum, ts);
  const uint32_t L = tab[257 + s];
  uint32_t r = L;
  if (ts[0] != 0u) {
    const float scale = static_cast<float>(L) / static_cast<float>(ts[0]);
    const float e = static_cast<float>(c) * scale + 6.0f * scale * sqrtf(static_cast<float>(c) + 1.0f) + 64.0f;
    r = e < static_cast<float>(L) ? static_cast<uint32_t>(e) : L;
  }
  reg[s * 256 + t] = r;
  // the bucket's total in 64 bits: past 2^31 it is reported as 2^32 - 1, which no region buffer
  // holds, so the exact path runs (each region stays below 2^32, and so does every prefix P2's
  // tiles take over a bucket's regions)
  __shared__ uint64_t part[4];
  uint64_t r64 = r;
  for (int o = 32; o > 0; o >>= 1) r64 += __shfl_xor(r64, o);
  if ((t & 63u) == 0) part[t >> 6] = r64;
  __syncthreads();
  if (t == 0) {
    const uint64_t all = part[0] + part[1] + part[2] + part[3];
    room[s] = all >= (uint64_t(1) << 31) ? 0xFFFFFFFFu : static_cast<uint32_t>(all);
  }
}

// The region plan of P2 (one block): the regions laid out bucket by bucket in the region buffer
// (cap2 elements) and P2's tiles planned with seg_len = room[s] (rec / hdr).  Regions past cap2:
// no tiles (hdr[0] = 0) and *spill = 1, so the exact path runs instead.
template <uint32_t TILE2>
__global__ __launch_bounds__(1024) void grs_msd_plan3(const uint32_t* __restrict__ tab,
                                                      const uint32_t* __restrict__ room_g, uint64_t cap2,
                                                      SegTile* __restrict__ rec, uint32_t* __restrict__ hdr,
                                                      uint32_t* __restrict__ spill) {
  __shared__ uint32_t lds[GRS_PLAN_LDS_WORDS + 4 * 257 + 64];
  uint32_t* const in = lds + GRS_PLAN_LDS_WORDS;
  uint32_t* const len = in + 257;
  uint32_t* const out = len + 257;
  uint32_t* const room = out + 257;
  uint32_t* const wsum = room + 257;
  const uint32_t t = threadIdx.x;
  uint64_t r64 = 0;
  if (t < 256) {
    in[t] = tab[t];
    len[t] = tab[257 + t];
    room[t] = room_g[t];
    r64 = room[t];
  }
  // the layout's total in 64 bits (a wave sum per wave, then thread 0)
  for (int o = 32; o > 0; o >>= 1) r64 += __shfl_xor(r64, o);
  __shared__ uint64_t wtot[16];
  if ((t & 63u) == 0) wtot[t >> 6] = r64;
  uint32_t v[1] = {t < 256 ? room[t] : 0u}, tot[1];
  block_scan<1024, 1>(v, wsum, tot);
  if (t < 256) out[t] = v[0];
  uint64_t all = 0;
  for (int k = 0; k < 16; ++k) all += wtot[k];
  __syncthreads();
  if (all > cap2 || all >= (uint64_t(1) << 32)) {
    if (t == 0) {
      hdr[0] = 0;
      hdr[1] = 0;
      hdr[2] = 0;
      *spill = 1u;
    }
    return;
  }
  seg_plan_block<TILE2, 1024, kSegMoved>(in, len, out, 256u, nullptr, rec, hdr, lds, room);
}

// The 16-bit segments for P3 after P2: without a spill (*spill == 0) the lengths are the
// region P2's digit totals (rtot) and each segment is read from its region start (rstart, in
// the region buffer); after a spill, the exact pass's counts (xcnt), in place.  out = where each
// sorted segment goes: its bucket's exact start (tab's out, grs_msd_plan2) + the lengths of
// the bucket's earlier segments.  One block of 256 per top-byte bucket.
__global__ __launch_bounds__(256) void grs_msd_starts(const uint32_t* __restrict__ spill,
                                                      const uint32_t* __restrict__ tab,
                                                      const uint32_t* __restrict__ rtot,
                                                      const uint32_t* __restrict__ xcnt,
                                                      const uint32_t* __restrict__ rstart,
                                                      uint32_t* __restrict__ len2, uint32_t* __restrict__ in2,
                                                      uint32_t* __restrict__ out2) {
  __shared__ uint32_t wsum[4];
  const bool sp = *spill != 0u;
  const uint32_t s = blockIdx.x, t = threadIdx.x, b = s * 256 + t;
  const uint32_t l = sp ? xcnt[b] : rtot[b];
  uint32_t v[1] = {l}, tot[1];
  block_scan<256, 1>(v, wsum, tot);
  const uint32_t o = tab[2 * 257 + s] + v[0];
  len2[b] = l;
  out2[b] = o;
  in2[b] = sp ? o : rstart[b];
}

// The big-list segments of P3 (longer than any LDS shape) from the region buffer into the
// caller's arrays at their sorted place, for the in-place fallback (persistent grid, every
// block on every entry; leaves at once without entries or after a spill, whose exact pass
// already wrote the caller's arrays).
template <typename K, bool PAIRS>
__global__ __launch_bounds__(256) void grs_msd_copy_big(const K* __restrict__ rk, const uint32_t* __restrict__ rv,
                                                        K* __restrict__ keys, uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ spill,
                                                        const uint32_t* __restrict__ big,
                                                        const uint32_t* __restrict__ big_in,
                                                        const uint32_t* __restrict__ big_out,
                                                        const uint32_t* __restrict__ big_len) {
  if (*spill != 0u) return;
  const uint32_t count = big[0];
  for (uint32_t e = 0; e < count; ++e) {
    const uint32_t a = big_in[e], o = big_out[e], n = big_len[e];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
      keys[o + i] = rk[a + i];
      if constexpr (PAIRS) vals[o + i] = rv[a + i];
    }
  }
}

// One workgroup sorts one segment [lo, lo + len) (len <= BLOCK * I) by its low 8 * rounds bits
// in LDS (rounds <= RMAX; the MSD sort: the bits below the 16-bit prefix, 2 rounds for u32 keys,
// 6 for u64), read from kin / vin and written to kout / vout (the same arrays: in place): 8-bit
// rounds of lane-ordered returning LDS adds, as the pass ranks.  C16: 16-bit wave counters (two
// per word), so that two 18K-key workgroups share a CU's LDS.
template <typename K, bool PAIRS, int BLOCK, int I, bool C16, int RMAX = (8 * static_cast<int>(sizeof(K)) - 16) / 8>
struct LocalSort {
  static constexpr uint32_t W = BLOCK / GRS_WAVE, SMAX = BLOCK * I;
  static constexpr int ROUNDS = RMAX;
  static_assert(W <= 16 && BLOCK >= 256, "digit threads: waves 0..3");
  static_assert(!C16 || SMAX < 65536, "16-bit positions");
  // 16-B vectors of keys / values; the arrays hold SMAX + one vector, so that element p can sit
  // at p + a (a < vector) with a the misalignment of the HBM run it comes from or goes to
  static constexpr uint32_t KV = 16 / sizeof(K), VV = 4;
  // LDS positions are swizzled: element x sits at swz(x), which XORs the 16-B group index inside
  // each 64-group with bits 8.. of x.  A rounds' scatter whose digit runs are all 256 long (the
  // reference's 0..N-1 shuffled: every 16-bit segment of 2^30 keys holds each value of its low 14
  // bits once) sends a wave-instruction's 64 keys to 64 run starts 256 apart -- one LDS bank,
  // a 64-way conflict that made P3 1.8x slower; swizzled, at most 4 lanes share a bank.  The
  // 16-B groups stay whole, so copy_out's vector reads stand.
  template <uint32_t V>   // V elements per 16-B group
  __device__ __forceinline__ static uint32_t swz_t(uint32_t x) {
#if GRS_P3_LDS_LAYOUT == 0
    return x;
#elif GRS_P3_LDS_LAYOUT == 2
    return x + ((x >> 8) * V);   // one 16-B group of padding every 256 elements
#else
    return x ^ (((x >> 8) & 15u) << (V == 4 ? 2 : V == 2 ? 1 : 0));
#endif
  }
  __device__ __forceinline__ static uint32_t swz(uint32_t x) { return swz_t<KV>(x); }
  __device__ __forceinline__ static uint32_t swzv(uint32_t x) { return swz_t<VV>(x); }
  // swz_t(base + lane) for a wave-uniform base that is a multiple of 64 (lane < 64): the part
  // that depends on the base is scalar, one VALU op per access is left
  template <uint32_t V>
  __device__ __forceinline__ static uint32_t swz_row(uint32_t base, uint32_t lane) {
#if GRS_P3_LDS_LAYOUT == 0
    return base + lane;
#elif GRS_P3_LDS_LAYOUT == 2
    return base + (base >> 8) * V + lane;
#else
    return base + (lane ^ (((base >> 8) & 15u) << (V == 4 ? 2 : V == 2 ? 1 : 0)));
#endif
  }
  template <uint32_t V>
  static constexpr uint32_t lds_len(uint32_t n) {   // (xor: stays inside a 64-group)
    return GRS_P3_LDS_LAYOUT == 2 ? (n + (n >> 8) * V + 63) / 64 * 64 : (n + 63) / 64 * 64;
  }
  static constexpr uint32_t SK = lds_len<KV>(SMAX + KV);
  struct Smem {
    alignas(16) K sk[SK];
    alignas(16) uint32_t sv[PAIRS ? lds_len<VV>(SMAX + VV) : 4];
    uint32_t cnt[W * 256 / (C16 ? 2 : 1)];
    uint32_t wtot[4];
    uint32_t slot;
  };
  using Vals = uint32_t[PAIRS ? I : 1];
  __device__ __forceinline__ static void run(Smem& sm, K* __restrict__ keys, uint32_t* __restrict__ vals,
                                             uint32_t lo, uint32_t len) {
    run(sm, keys, vals, keys, vals, lo, len, ROUNDS);
  }
  __device__ __forceinline__ static void run(Smem& sm, const K* kin, const uint32_t* vin, K* kout,
                                             uint32_t* vout, uint32_t lo, uint32_t len, int rounds) {
    K k[I];
    Vals v;
    load(k, v, kin, vin, lo, len);
    sort_rounds(sm, k, v, len, rounds);
    store(sm, kout, vout, lo, len);
  }
  // the segment's keys (and payload) into registers, wave-striped (item j of lane l of wave w is
  // key w*64*I + j*64 + l)
  // (t: threadIdx.x; a persistent caller passes an opaque copy per call, so that the compiler
  // does not keep the I per-item offsets live across its loop)
  __device__ __forceinline__ static void load(K (&k)[I], Vals& v, const K* kin, const uint32_t* vin,
                                              uint32_t lo, uint32_t len, uint32_t t = threadIdx.x) {
    const uint32_t lane = t & (GRS_WAVE - 1), w = t >> 6;
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
      k[j] = i < len ? kin[lo + i] : K(0);
      if constexpr (PAIRS) v[j] = i < len ? vin[lo + i] : 0u;
    }
  }
  // `rounds` stable 8-bit rounds from the registers; the sorted segment is left in sm.sk / sm.sv,
  // element p at sm.sk[p + ak] / sm.sv[p + av] (ak, av: store_vec's alignment shifts)
  __device__ __forceinline__ static void sort_rounds(Smem& sm, K (&k)[I], Vals& v, uint32_t len, int rounds,
                                                     uint32_t ak = 0, uint32_t av = 0, int shift0 = 0,
                                                     uint32_t t = threadIdx.x) {
    uint16_t* const c16 = reinterpret_cast<uint16_t*>(sm.cnt);
    auto cld = [&](uint32_t a) -> uint32_t { if constexpr (C16) return c16[a]; else return sm.cnt[a]; };
    auto cst = [&](uint32_t a, uint32_t x) {
      if constexpr (C16) c16[a] = static_cast<uint16_t>(x); else sm.cnt[a] = x;
    };
    const uint32_t lane = t & (GRS_WAVE - 1), w = t >> 6;
#pragma unroll
    for (int pass = 0; pass < ROUNDS; ++pass) {
      if (pass >= rounds) break;   // uniform
      const int shift = shift0 + 8 * pass;
      auto digit = [&](K x) { return static_cast<uint32_t>(x >> shift) & 255u; };
      for (uint32_t c = t; c < W * 256 / (C16 ? 2 : 1); c += BLOCK) sm.cnt[c] = 0;
      __syncthreads();
      uint32_t r[I];
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
        const uint32_t d = digit(k[j]);
        if constexpr (C16) {
          const uint32_t sh = (d & 1u) << 4;
          r[j] = i < len ? (atomicAdd(&sm.cnt[(w * 256 + d) >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
        } else {
          r[j] = i < len ? atomicAdd(&sm.cnt[w * 256 + d], 1u) : 0u;
        }
      }
      __syncthreads();
      uint32_t c[W], tot = 0, incl = 0;
      if (t < 256) {
#pragma unroll
        for (uint32_t ww = 0; ww < W; ++ww) {
          c[ww] = cld(ww * 256 + t);
          tot += c[ww];
        }
        incl = wave_scan_dpp(tot);
        if (lane == GRS_WAVE - 1) sm.wtot[w] = incl;
      }
      __syncthreads();
      if (t < 256) {
        uint32_t b = incl - tot;
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww) b += ww < w ? sm.wtot[ww] : 0u;
#pragma unroll
        for (uint32_t ww = 0; ww < W; ++ww) {
          cst(ww * 256 + t, b);
          b += c[ww];
        }
      }
      __syncthreads();
      const bool last = pass + 1 >= rounds;
      const uint32_t sk_off = last ? ak : 0u, sv_off = last ? av : 0u;
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t i = w * GRS_WAVE * I + j * GRS_WAVE + lane;
        if (i < len) {
          const uint32_t dst = cld(w * 256 + digit(k[j])) + r[j];
          sm.sk[swz(dst + sk_off)] = k[j];
          if constexpr (PAIRS) sm.sv[swzv(dst + sv_off)] = v[j];
        }
      }
      __syncthreads();
      if (pass + 1 < rounds) {
        const uint32_t ws = __builtin_amdgcn_readfirstlane(w);
#pragma unroll
        for (uint32_t j = 0; j < I; ++j) {
          const uint32_t base = ws * GRS_WAVE * I + j * GRS_WAVE;
          if (base + lane < len) {
            k[j] = sm.sk[swz_row<KV>(base, lane)];
            if constexpr (PAIRS) v[j] = sm.sv[swz_row<VV>(base, lane)];
          }
        }
      }
    }
  }
  // the sorted segment from LDS to HBM, consecutive threads on consecutive keys
  __device__ __forceinline__ static void store(Smem& sm, K* kout, uint32_t* vout, uint32_t lo, uint32_t len) {
    for (uint32_t i = threadIdx.x; i < len; i += BLOCK) {
      kout[lo + i] = sm.sk[swz(i)];
      if constexpr (PAIRS) vout[lo + i] = sm.sv[swzv(i)];
    }
  }

  // ---- 16-B accesses (one dwordx4 per lane) for runs at any element alignment ----
  // Where element p of a run starting at `at` sits relative to a 16-B boundary: (address / E) % V.
  template <typename T, uint32_t V>
  __device__ __forceinline__ static uint32_t mis(const T* at) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(at) / sizeof(T)) % V;
  }
  // lds[a, a + len) -> run[0, len) with a = mis(run) (sort_rounds' shift).  ROT: the workgroup
  // starts its vectors at a rotation of (blockIdx * 97 mod 256) x 256 B, so that the hundreds of
  // workgroups storing at once are not all at the same offset of their runs: runs that start at
  // multiples of 64 KB (the reference's 0..N-1 shuffled at 2^30: 16384-key segments) would
  // otherwise send every workgroup's stores to the same HBM channels at the same time
  template <typename T, uint32_t V, bool ROT = true>
  __device__ __forceinline__ static void copy_out(T* run, const T* lds, uint32_t len, uint32_t seed = blockIdx.x) {
    const uint32_t t = threadIdx.x, a = mis<T, V>(run);
    const uint32_t head = min(len, (V - a) % V);
    const uint32_t nv = (len - head) / V;
    if (t < head) run[t] = lds[swz_t<V>(a + t)];
    uint4* dst = reinterpret_cast<uint4*>(run + head);
    const uint32_t rot = ROT && nv != 0u ? ((seed * 97u & 255u) * 16u) % nv : 0u;
    for (uint32_t c = t; c < nv; c += BLOCK) {
      uint32_t r = c + rot;
      if (r >= nv) r -= nv;
      // the group's V elements: V-aligned in LDS, whole under the swizzle
      dst[r] = *reinterpret_cast<const uint4*>(lds + swz_t<V>(a + head + r * V));
    }
    const uint32_t r = head + nv * V + t;
    if (r < len) run[r] = lds[swz_t<V>(a + r)];
  }
  // run() with 16-B HBM stores (the loads stay one element per lane, wave-striped: staging them
  // through LDS with 16-B LDS-DMA loads measured slower, tools/lab8.py): kin / vin and kout /
  // vout are the segment's runs, at any alignment
  template <bool ROT = true>
  __device__ __forceinline__ static void run_vec(Smem& sm, const K* kin, const uint32_t* vin, K* kout,
                                                 uint32_t* vout, uint32_t len, int rounds) {
    K k[I];
    Vals v;
    auto ld = [&]() { load(k, v, kin, vin, 0u, len); };
    ld();
    const uint32_t ak = mis<K, KV>(kout), av = PAIRS ? mis<uint32_t, VV>(vout) : 0u;
    if (ROUNDS > 2 && rounds > 2) {
      // more than two rounds (u64 keys): two on the top 16 of the bits to sort, then the runs
      // of keys equal in them -- short in a uniform segment (4096 keys in 65536 bins: ~6 % of
      // the keys, runs of 2-4) -- finished by an insertion sort on the bits below, stable; a
      // run past kRunMax sends the segment through every round instead (its keys read again)
      if constexpr (ROUNDS > 2) {   // (u32 keys never take this branch: no code for it)
        sort_rounds(sm, k, v, len, 2, ak, av, 8 * rounds - 16);
        if (finish_runs(sm, len, 8 * rounds - 16, ak, av)) {
          ld();
          sort_rounds(sm, k, v, len, rounds, ak, av);
        }
      }
    } else {
      sort_rounds(sm, k, v, len, rounds, ak, av);   // (ends with a barrier after its scatter)
    }
    copy_out<K, KV, ROT>(kout, sm.sk, len);
    if constexpr (PAIRS) copy_out<uint32_t, VV, ROT>(vout, sm.sv, len);
  }
  static constexpr uint32_t kRunMax = 48;
  // The sorted segment in LDS (sm.sk[ak + p]) is ordered by key >> hb and, inside each run of equal
  // key >> hb, by input order; sort every run by the whole key with a stable insertion sort (one
  // thread per run; the runs are disjoint and their key >> hb never changes, so the run bounds
  // other threads read stay valid).  Returns true (uniform) if a run was longer than kRunMax
  // (left unsorted: the caller sorts the segment by every round instead).
  __device__ __forceinline__ static bool finish_runs(Smem& sm, uint32_t len, int hb, uint32_t ak, uint32_t av) {
    __syncthreads();   // the last round's scatter
    if (threadIdx.x == 0) sm.slot = 0;
    __syncthreads();
    auto A = [&](uint32_t p) -> K& { return sm.sk[swz(ak + p)]; };
    auto B = [&](uint32_t p) -> uint32_t& { return sm.sv[swzv(av + p)]; };
    for (uint32_t p = threadIdx.x; p < len; p += BLOCK) {
      const K hi = A(p) >> hb;
      if (p != 0 && (A(p - 1) >> hb) == hi) continue;   // not a run start
      uint32_t e = p + 1;
      while (e < len && (A(e) >> hb) == hi && e - p <= kRunMax) ++e;
      if (e - p > kRunMax) {
        sm.slot = 1;
        continue;
      }
      for (uint32_t q = p + 1; q < e; ++q) {   // insertion sort of [p, e): stable
        const K x = A(q);
        uint32_t y = 0;
        if constexpr (PAIRS) y = B(q);
        uint32_t r = q;
        while (r > p && A(r - 1) > x) {
          A(r) = A(r - 1);
          if constexpr (PAIRS) B(r) = B(r - 1);
          --r;
        }
        A(r) = x;
        if constexpr (PAIRS) B(r) = y;
      }
    }
    __syncthreads();
    return sm.slot != 0u;
  }
};

// P3 for u32 keys without payload: the keys of a 16-bit segment agree in bits 16..31 (the
// prefix and the bits above the top digit; the bits sorted are below 16 whatever the top shift),
// so LDS holds their low halves only and the registers two of them a VGPR -- half LocalSort's
// LDS and registers, so that four 17K-key workgroups share a CU (LocalSort<u32>'s 72-KB shape:
// two), and one segment's HBM loads and stores overlap three others' LDS rounds.  The rounds are
// LocalSort's (lane-ordered returning LDS adds on 16-bit wave counters, stable); copy_out widens
// each 8-B group of low halves to a 16-B store of whole keys.  rounds 1..2 (msd_p3_rounds).
#ifndef GRS_P3H_GROUP
#define GRS_P3H_GROUP 8
#endif
template <int BLOCK, int I>
struct LocalSort16 {
  static_assert(I % 2 == 0, "two keys a register");
  static constexpr uint32_t W = BLOCK / GRS_WAVE, SMAX = BLOCK * I, IP = I / 2;
  // LDS operations a wave keeps in flight in the rank and scatter loops (the scheduler would
  // issue all I of them at once and spill at eight waves a SIMD)
  static constexpr uint32_t G = GRS_P3H_GROUP;
  static_assert(W <= 16 && BLOCK >= 256 && SMAX < 65536, "digit threads: waves 0..3; 16-bit counters");
  // LocalSort::swz_t for 4-element groups: XOR of the group index inside each 64-element block
  // with bits 8.. of x (runs 256 long would otherwise send a wave's 64 scatter targets to one bank)
  __device__ __forceinline__ static uint32_t swz(uint32_t x) { return x ^ (((x >> 8) & 15u) << 2); }
  // swz(base + lane) for a wave-uniform base that is a multiple of 64 (lane < 64)
  __device__ __forceinline__ static uint32_t swz_row(uint32_t base, uint32_t lane) {
    return base + (lane ^ (((base >> 8) & 15u) << 2));
  }
  static constexpr uint32_t SK = (SMAX + 4 + 63) / 64 * 64;   // SMAX slots + an alignment shift < 4
  struct Smem {
    alignas(16) uint16_t sk[SK];
    uint32_t cnt[W * 128];   // 16-bit counters, two a word
    uint32_t spare[GRS_WAVE];   // the ranking's adds for slots past the keys
    uint32_t wtot[4];
    uint32_t slot;
  };
  __device__ __forceinline__ static uint32_t half(const uint32_t (&p)[IP], uint32_t j) {
    return (p[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
  }
  // kin[0, len) -> kout[0, len) sorted by bits 0 .. 8 * rounds (rounds 0: the load + store
  // skeleton of the lab, LDS left unwritten).  The slots past len skip the ranking (lanes of one
  // digit would serialise on its counter) and scatter to their own index, past the keys
  __device__ __forceinline__ static void run(Smem& sm, const uint32_t* kin, uint32_t* kout, uint32_t len,
                                             int rounds) {
    const uint32_t t = threadIdx.x, lane = t & (GRS_WAVE - 1), w = t >> 6;
    const uint32_t hi = __builtin_amdgcn_readfirstlane(kin[0]) & 0xFFFF0000u;
    // the low halves only (2-B buffer loads of the same lines: unpredicated, the descriptor's
    // range check drops the slots past len, one offset register for all I), packed two a register
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(kin), 0, static_cast<int>(4u * len),
                                                        0x00020000);
    // (wave-uniform bases: the per-item parts of offsets and bounds stay scalar)
    const uint32_t ws = __builtin_amdgcn_readfirstlane(w), wbase = ws * GRS_WAVE * I;
    const uint32_t wlen = len > wbase ? len - wbase : 0u;   // this wave's slots holding keys
    uint32_t kp[IP];
#pragma unroll
    for (uint32_t j = 0; j < IP; ++j) {
      const uint32_t a = __builtin_amdgcn_raw_buffer_load_b16(rsrc, 4u * lane, 4u * (wbase + 2u * j * GRS_WAVE), 0);
      const uint32_t b = __builtin_amdgcn_raw_buffer_load_b16(rsrc, 4u * lane, 4u * (wbase + (2u * j + 1u) * GRS_WAVE), 0);
      kp[j] = (a & 0xFFFFu) | (b << 16);
    }
    const uint32_t ak = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(kout) / 4u) % 4u;
    uint16_t* const c16 = reinterpret_cast<uint16_t*>(sm.cnt);
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (pass >= rounds) break;   // (uniform)
      const uint32_t shift = 8u * static_cast<uint32_t>(pass);
      for (uint32_t c = t; c < W * 128; c += BLOCK) sm.cnt[c] = 0;
      __syncthreads();
      uint32_t rp[IP];
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t d = (half(kp, j) >> shift) & 255u, sh = (d & 1u) << 4;
        // a slot past the keys adds to its lane's own spare word (no predicate, no serialising
        // lanes on one counter)
        const bool ok = lane + j * GRS_WAVE < wlen;
        const uint32_t r = (atomicAdd(ok ? &sm.cnt[(w * 256 + d) >> 1] : &sm.spare[lane], 1u << sh) >> sh) & 0xFFFFu;
        if (j & 1) rp[j >> 1] |= r << 16;
        else rp[j >> 1] = r;
        if (j % G == G - 1) __builtin_amdgcn_sched_barrier(0);   // G returning adds in flight
      }
      // opaque: the scatter recomputes each half and digit from the packed registers (the
      // compiler would keep I unpacked halves and I digits live across the scan and spill them)
#pragma unroll
      for (uint32_t j = 0; j < IP; ++j) asm volatile("" : "+v"(kp[j]), "+v"(rp[j]));
      __syncthreads();
      uint32_t c[W], tot = 0, incl = 0;
      if (t < 256) {
#pragma unroll
        for (uint32_t ww = 0; ww < W; ++ww) {
          c[ww] = c16[ww * 256 + t];
          tot += c[ww];
        }
        incl = wave_scan_dpp(tot);
        if (lane == GRS_WAVE - 1) sm.wtot[w] = incl;
      }
      __syncthreads();
      if (t < 256) {
        uint32_t b = incl - tot;
#pragma unroll
        for (uint32_t ww = 0; ww < 4; ++ww) b += ww < w ? sm.wtot[ww] : 0u;
#pragma unroll
        for (uint32_t ww = 0; ww < W; ++ww) {
          c16[ww * 256 + t] = static_cast<uint16_t>(b);
          b += c[ww];
        }
      }
      __syncthreads();
      const uint32_t off = pass + 1 >= rounds ? ak : 0u;
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t x = half(kp, j);
        const uint32_t dst = lane + j * GRS_WAVE < wlen ? c16[w * 256 + ((x >> shift) & 255u)] + half(rp, j)
                                                        : wbase + j * GRS_WAVE + lane;
        sm.sk[swz(dst + off)] = static_cast<uint16_t>(x);
        if (j % G == G - 1) __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
      if (pass + 1 < rounds) {
#pragma unroll
        for (uint32_t j = 0; j < IP; ++j) {
          const uint32_t b0 = wbase + 2u * j * GRS_WAVE, b1 = b0 + GRS_WAVE;
          kp[j] = static_cast<uint32_t>(sm.sk[swz_row(b0, lane)]) | (static_cast<uint32_t>(sm.sk[swz_row(b1, lane)]) << 16);
        }
      }
    }
    // sm.sk[ak + p] -> kout[p] in 16-B stores (head / tail peeled to kout's 16-B alignment), the
    // workgroup's vectors rotated as LocalSort::copy_out's
    const uint32_t head = min(len, (4u - ak) % 4u), nv = (len - head) / 4u;
    if (t < head) kout[t] = hi | sm.sk[swz(ak + t)];
    uint4* const dst = reinterpret_cast<uint4*>(kout + head);
    const uint32_t rot = nv != 0u ? ((blockIdx.x * 97u & 255u) * 16u) % nv : 0u;
    for (uint32_t c = t; c < nv; c += BLOCK) {
      uint32_t r = c + rot;
      if (r >= nv) r -= nv;
      const uint2 g = *reinterpret_cast<const uint2*>(sm.sk + swz(ak + head + r * 4u));
      dst[r] = make_uint4(hi | (g.x & 0xFFFFu), hi | (g.x >> 16), hi | (g.y & 0xFFFFu), hi | (g.y >> 16));
    }
    const uint32_t r = head + nv * 4u + t;
    if (r < len) kout[r] = hi | sm.sk[swz(ak + r)];
  }
};

// P3: one workgroup per 16-bit prefix b (grid 65536): its len2[b] keys (and payload), read at
// in2[b] of the region buffer (rk / rv) -- or, after a P2 spill, of the caller's arrays, in
// place -- sorted in LDS (LocalSort) and written to out2[b] of the caller's arrays
// (grs_msd_starts).  Longer segments are listed: up to MID keys in the mid list (mid[0] =
// count, (in, out, len) from mid[2] on) for grs_msd_local_list's larger shape, longer ones in
// the big list for the segmented LSD in place (grs_msd_copy_big moves them first): big[0] counts
// them, big[1] counts those longer than one fallback tile (TILEF keys), which get a histogram
// row (ND digits) zeroed here; big_in / big_start / big_len / big_row hold (region start,
// sorted start, length, row) per entry.
// A P3 segment that is not sorted in this shape's LDS: one key (copied to its place, unless in
// place), or longer than SMAX -- listed: up to mid_max keys in the mid list (mid[0] = count,
// (in, out, len) from mid[2] on) for grs_msd_local_list's larger shape, longer ones in the big
// list for the segmented LSD in place (grs_msd_copy_big moves them first): big[0] counts them,
// big[1] counts those longer than one fallback tile (TILEF keys), which get a histogram row (ND
// digits) zeroed here; big_in / big_start / big_len / big_row hold (region start, sorted start,
// length, row) per entry.  Uniform in the workgroup; slot: an LDS word.
template <typename K, bool PAIRS, int BLOCK, uint32_t SMAX, uint32_t ND, uint32_t TILEF>
__device__ __forceinline__ void msd_local_other(uint32_t len, uint32_t lo, uint32_t o, bool inplace, const K* kin,
                                                const uint32_t* vin, K* keys, uint32_t* vals, uint32_t mid_max,
                                                uint32_t* mid, uint32_t* big, uint32_t* big_in,
                                                uint32_t* big_start, uint32_t* big_len, uint32_t* big_row,
                                                uint32_t* rows, uint32_t& slot) {
  const uint32_t t = threadIdx.x;
  if (len == 1u) {
    if (!inplace && t == 0) {
      keys[o] = kin[lo];
      if constexpr (PAIRS) vals[o] = vin[lo];
    }
    return;
  }
  if (len <= SMAX) return;   // (0)
  if (len <= mid_max) {   // the mid list (a larger LDS shape)
    if (t == 0) {
      const uint32_t e = atomicAdd(&mid[0], 1u);
      mid[2 + 3 * e] = lo;
      mid[3 + 3 * e] = o;
      mid[4 + 3 * e] = len;
    }
    return;
  }
  if (t == 0) {
    const uint32_t e = atomicAdd(&big[0], 1u);
    const uint32_t row = len > TILEF ? atomicAdd(&big[1], 1u) : 0xFFFFFFFFu;
    big_in[e] = lo;
    big_start[e] = o;
    big_len[e] = len;
    big_row[e] = row;
    slot = row;
  }
  __syncthreads();
  const uint32_t row = slot;
  if (row != 0xFFFFFFFFu)
    for (uint32_t i = t; i < ND * 256; i += BLOCK) rows[static_cast<size_t>(row) * ND * 256 + i] = 0;
}

// P3: one workgroup per 16-bit prefix b (grid 65536): its len2[b] keys (and payload), read at
// in2[b] of the region buffer (rk / rv) -- or, after a P2 spill, of the caller's arrays, in
// place -- sorted in LDS (LocalSort) and written to out2[b] of the caller's arrays
// (grs_msd_starts); the others as msd_local_other says.
template <typename K, bool PAIRS, int BLOCK, int I, bool C16, uint32_t TILEF>
__global__ __launch_bounds__(BLOCK) void grs_msd_local(K* __restrict__ keys, uint32_t* __restrict__ vals,
                                                       const K* __restrict__ rk, const uint32_t* __restrict__ rv,
                                                       const uint32_t* __restrict__ spill,
                                                       const uint32_t* __restrict__ len2,
                                                       const uint32_t* __restrict__ in2,
                                                       const uint32_t* __restrict__ out2,
                                                       uint32_t mid_max, uint32_t* __restrict__ mid,
                                                       uint32_t* __restrict__ big,
                                                       uint32_t* __restrict__ big_in,
                                                       uint32_t* __restrict__ big_start,
                                                       uint32_t* __restrict__ big_len,
                                                       uint32_t* __restrict__ big_row,
                                                       uint32_t* __restrict__ rows,
                                                       const uint32_t* __restrict__ top_shift) {
  using LS = LocalSort<K, PAIRS, BLOCK, I, C16>;
  constexpr uint32_t ND = LS::ROUNDS;   // fallback digits (histogram row of ND x 256 words)
  __shared__ typename LS::Smem sm;
  const uint32_t len = len2[blockIdx.x];
  if (len == 0u) return;   // (the start of an empty segment was never written)
  const bool inplace = __builtin_amdgcn_readfirstlane(*spill) != 0u;
  const uint32_t lo = in2[blockIdx.x], o = out2[blockIdx.x];
  const K* const kin = inplace ? keys : rk;
  const uint32_t* const vin = inplace ? vals : rv;
  if (len == 1u || len > LS::SMAX) {
    msd_local_other<K, PAIRS, BLOCK, LS::SMAX, ND, TILEF>(len, lo, o, inplace, kin, vin, keys, vals, mid_max, mid,
                                                          big, big_in, big_start, big_len, big_row, rows, sm.slot);
    return;
  }
  // the bits below the segment's 16-bit prefix (bits above the top digit are equal in every key);
  // 16-B HBM loads and stores through LDS at the runs' own alignments
  const int rounds = msd_p3_rounds<LS::ROUNDS>(__builtin_amdgcn_readfirstlane(*top_shift));
  LS::template run_vec<>(sm, kin + lo, PAIRS ? vin + lo : nullptr, keys + o, PAIRS ? vals + o : nullptr, len,
                         rounds);
}

// P3 of u32 keys without payload on LocalSort16 (the low halves in LDS; three 512 x 34
// workgroups a CU at 2^30 keys instead of LocalSort's two 768 x 23): grs_msd_local's tables,
// lists and results.
template <int BLOCK, int I, int MINW, uint32_t TILEF>
__global__ __launch_bounds__(BLOCK, MINW) void grs_msd_local16(
    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, const uint32_t* __restrict__ rk,
    const uint32_t* __restrict__ rv, const uint32_t* __restrict__ spill, const uint32_t* __restrict__ len2,
    const uint32_t* __restrict__ in2, const uint32_t* __restrict__ out2, uint32_t mid_max, uint32_t* __restrict__ mid,
    uint32_t* __restrict__ big, uint32_t* __restrict__ big_in, uint32_t* __restrict__ big_start,
    uint32_t* __restrict__ big_len, uint32_t* __restrict__ big_row, uint32_t* __restrict__ rows,
    const uint32_t* __restrict__ top_shift) {
  using LS = LocalSort16<BLOCK, I>;
  __shared__ typename LS::Smem sm;
  const uint32_t len = len2[blockIdx.x];
  if (len == 0u) return;
  const bool inplace = __builtin_amdgcn_readfirstlane(*spill) != 0u;
  const uint32_t lo = in2[blockIdx.x], o = out2[blockIdx.x];
  const uint32_t* const kin = inplace ? keys : rk;
  if (len == 1u || len > LS::SMAX) {
    msd_local_other<uint32_t, false, BLOCK, LS::SMAX, 2, TILEF>(len, lo, o, inplace, kin, nullptr, keys, vals, mid_max,
                                                                mid, big, big_in, big_start, big_len, big_row, rows,
                                                                sm.slot);
    return;
  }
  LS::run(sm, kin + lo, keys + o, len, msd_p3_rounds<2>(__builtin_amdgcn_readfirstlane(*top_shift)));
}

// P3 persistent (keys sorted in at most two LDS rounds: u32 keys, u32 pairs): grid = resident
// workgroups, each drawing segments from a ticket (*ticket zero at launch) until past 65536.
// The next segment's keys are loaded into the registers as soon as this one's last round has
// scattered them into LDS, so the loads fly while this segment is stored (one workgroup per
// segment paid the full HBM latency of its loads after its predecessor's stores).  The same
// results as grs_msd_local.
template <typename K, bool PAIRS, int BLOCK, int I, bool C16, uint32_t TILEF, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void grs_msd_local_pf(
    K* __restrict__ keys, uint32_t* __restrict__ vals, const K* __restrict__ rk, const uint32_t* __restrict__ rv,
    const uint32_t* __restrict__ spill, const uint32_t* __restrict__ len2, const uint32_t* __restrict__ in2,
    const uint32_t* __restrict__ out2, uint32_t mid_max, uint32_t* __restrict__ mid, uint32_t* __restrict__ big,
    uint32_t* __restrict__ big_in, uint32_t* __restrict__ big_start, uint32_t* __restrict__ big_len,
    uint32_t* __restrict__ big_row, uint32_t* __restrict__ rows, const uint32_t* __restrict__ top_shift,
    uint32_t* __restrict__ ticket) {
  using LS = LocalSort<K, PAIRS, BLOCK, I, C16>;
  static_assert(LS::ROUNDS <= 2, "u64 keys: grs_msd_local (its run finish may reload the keys)");
  constexpr uint32_t ND = LS::ROUNDS, NSEG = 65536;
  __shared__ typename LS::Smem sm;
  __shared__ uint32_t nxt;
  const uint32_t t = threadIdx.x;
  const bool inplace = __builtin_amdgcn_readfirstlane(*spill) != 0u;
  const K* const kin = inplace ? keys : rk;
  const uint32_t* const vin = inplace ? vals : rv;
  const int rounds = msd_p3_rounds<LS::ROUNDS>(__builtin_amdgcn_readfirstlane(*top_shift));
  auto sorted_here = [](uint32_t l) { return l >= 2u && l <= LS::SMAX; };
  if (t == 0) nxt = atomicAdd(ticket, 1u);
  __syncthreads();
  uint32_t b = __builtin_amdgcn_readfirstlane(nxt);
  K k[I];
  typename LS::Vals v;
  uint32_t len = b < NSEG ? len2[b] : 0u;
  if (b < NSEG && sorted_here(len)) LS::load(k, v, kin, vin, in2[b], len);
  while (b < NSEG) {
    __syncthreads();   // every thread has read nxt
    if (t == 0) nxt = atomicAdd(ticket, 1u);
    const uint32_t lo = in2[b], o = out2[b];
    const bool here = sorted_here(len);
    if (here) {
      const uint32_t ak = LS::template mis<K, LS::KV>(keys + o);
      const uint32_t av = PAIRS ? LS::template mis<uint32_t, LS::VV>(vals + o) : 0u;
      uint32_t tt = t;
      asm volatile("" : "+v"(tt));
      LS::sort_rounds(sm, k, v, len, rounds, ak, av, 0, tt);   // (its barriers publish nxt)
    } else {
      if (len != 0u)
        msd_local_other<K, PAIRS, BLOCK, LS::SMAX, ND, TILEF>(len, lo, o, inplace, kin, vin, keys, vals, mid_max,
                                                              mid, big, big_in, big_start, big_len, big_row, rows,
                                                              sm.slot);
      __syncthreads();
    }
    const uint32_t nb = __builtin_amdgcn_readfirstlane(nxt);
    const uint32_t nlen = nb < NSEG ? len2[nb] : 0u;
    // the registers are free (the last round scattered them into LDS): the next segment's loads
    if (nb < NSEG && sorted_here(nlen)) {
      uint32_t tt = t;
      asm volatile("" : "+v"(tt));
      LS::load(k, v, kin, vin, in2[nb], nlen, tt);
    }
    if (here) {
      LS::template copy_out<K, LS::KV>(keys + o, sm.sk, len, b);
      if constexpr (PAIRS) LS::template copy_out<uint32_t, LS::VV>(vals + o, sm.sv, len, b);
    }
    b = nb;
    len = nlen;
  }
}

// P3's second shape: the mid list's segments (persistent grid, a segment per workgroup in
// turn; leaves at once when the list is empty).  MINW: waves per SIMD to keep the registers
// of two workgroups per CU where their LDS fits.
template <typename K, bool PAIRS, int BLOCK, int I, bool C16, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void grs_msd_local_list(K* __restrict__ keys,
                                                            uint32_t* __restrict__ vals,
                                                            const K* __restrict__ rk,
                                                            const uint32_t* __restrict__ rv,
                                                            const uint32_t* __restrict__ spill,
                                                            const uint32_t* __restrict__ mid,
                                                            const uint32_t* __restrict__ top_shift,
                                                            const uint32_t* __restrict__ big = nullptr,
                                                            const uint32_t* __restrict__ big_in = nullptr,
                                                            const uint32_t* __restrict__ big_out = nullptr,
                                                            const uint32_t* __restrict__ big_len = nullptr) {
  using LS = LocalSort<K, PAIRS, BLOCK, I, C16>;
  __shared__ typename LS::Smem sm;
  const bool inplace = *spill != 0u;
  // big (nullable): grs_msd_copy_big's work first, so that it needs no launch of its own (every
  // workgroup takes a slice of every entry; disjoint from the mid list's segments)
  if (big != nullptr && !inplace) {
    const uint32_t nb = big[0];
    for (uint32_t e = 0; e < nb; ++e) {
      const uint32_t a = big_in[e], o = big_out[e], n = big_len[e];
      for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        keys[o + i] = rk[a + i];
        if constexpr (PAIRS) vals[o + i] = rv[a + i];
      }
    }
  }
  const uint32_t count = mid[0];
  if (count == 0u) return;
  const K* const kin = inplace ? keys : rk;
  const uint32_t* const vin = inplace ? vals : rv;
  const int rounds = msd_p3_rounds<LS::ROUNDS>(__builtin_amdgcn_readfirstlane(*top_shift));
  for (uint32_t e = blockIdx.x; e < count; e += gridDim.x) {
    const uint32_t lo = mid[2 + 3 * e], o = mid[3 + 3 * e], len = mid[4 + 3 * e];
    LS::template run_vec<>(sm, kin + lo, PAIRS ? vin + lo : nullptr, keys + o, PAIRS ? vals + o : nullptr,
                           len, rounds);
    __syncthreads();   // every LDS read of this segment before the next one's
  }
}

// ---------------------------------------------------------------------------------------
// segmented sort of long segments (grs_sort_segmented): one stable scatter by the top byte
// inside every segment (grs_onesweep_seg over a kSegOffsetsAll plan; each segment's first tile
// writes its 256 run starts to ds[seg * 256 + d]), then every run sorted by the bits below the
// top byte in LDS, from the second buffer back into the caller's arrays
// ---------------------------------------------------------------------------------------
// The runs of segment blockIdx.x as work lists.  Consecutive runs merge greedily into entries
// of at most CP keys (sorted by the whole key: the runs keep their order); a longer run is an
// entry of its own.  Entries of up to CP keys go to the primary list (prim), up to CL to the mid list, longer
// ones to the big list (bstart / blen / brow) for a segmented LSD on the bits below the top
// byte.  cnt (zeroed by the caller): [0] primary entries, [1] mid entries, [2] big entries,
// [3] big entries longer than one fallback tile of TILEF keys, which get a histogram row of ND
// digits (zeroed here).  prim / mid: (start, length | merged << 31) per entry.
template <uint32_t CP, uint32_t CL, uint32_t TILEF, int ND>
__global__ __launch_bounds__(256) void grs_seg_runs(const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ ds, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ prim, uint32_t* __restrict__ mid,
                                                    uint32_t* __restrict__ bstart,
                                                    uint32_t* __restrict__ blen, uint32_t* __restrict__ brow,
                                                    uint32_t* __restrict__ rows) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  __shared__ uint32_t es[257], eb[257], rl[256], wsum[3 * 4], base[3];
  const uint32_t s = blockIdx.x, t = threadIdx.x;
  const uint32_t lo = off[s], hi = off[s + 1];
  if (hi <= lo) return;   // uniform: an empty segment (its run starts were never written)
  const uint32_t st = ds[static_cast<size_t>(s) * 256 + t];
  const uint32_t en = t < 255u ? ds[static_cast<size_t>(s) * 256 + t + 1] : hi;
  rl[t] = en - st;
  __syncthreads();
  // greedy packing by wave 0 on the scalar unit (lane j of quarter q holds run 64 q + j): run d
  // opens an entry when it is the first, longer than CP, or would overfill the open one; rl[d]
  // becomes the flag
  if (t < GRS_WAVE) {
    uint32_t cur = CP + 1;
    uint32_t q4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) q4[q] = rl[q * GRS_WAVE + t];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint64_t m = 0;
#pragma unroll
      for (int j = 0; j < GRS_WAVE; ++j) {
        const uint32_t l = __builtin_amdgcn_readlane(q4[q], j);
        const bool open = cur > CP || l > CP - cur;
        cur = open ? l : cur + l;
        if (l > CP) cur = CP + 1;
        m |= static_cast<uint64_t>(open) << j;
      }
      rl[q * GRS_WAVE + t] = static_cast<uint32_t>(m >> t) & 1u;
    }
  }
  __syncthreads();
  uint32_t f[1] = {rl[t]}, ne[1];
  const uint32_t is_first = f[0];
  block_scan<256, 1>(f, wsum, ne);
  const uint32_t E = ne[0];
  if (is_first) {
    es[f[0]] = st;
    eb[f[0]] = t;
  }
  if (t == 0) {
    es[E] = hi;
    eb[E] = 256;
  }
  __syncthreads();
  uint32_t s0 = 0, l = 0, nb = 0;
  if (t < E) {
    s0 = es[t];
    l = es[t + 1] - s0;
    nb = eb[t + 1] - eb[t];
  }
  uint32_t cls[3] = {l != 0u && l <= CP ? 1u : 0u, l > CP && l <= CL ? 1u : 0u, l > CL ? 1u : 0u}, tot[3];
  const uint32_t k0 = cls[0], k1 = cls[1], k2 = cls[2];
  block_scan<256, 3>(cls, wsum, tot);
  if (t == 0) {
    base[0] = tot[0] ? atomicAdd(&cnt[0], tot[0]) : 0u;
    base[1] = tot[1] ? atomicAdd(&cnt[1], tot[1]) : 0u;
    base[2] = tot[2] ? atomicAdd(&cnt[2], tot[2]) : 0u;
  }
  __syncthreads();
  const uint32_t lw = l | (nb > 1u ? 0x80000000u : 0u);
  if (k0) {
    const uint32_t e = base[0] + cls[0];
    prim[2 * e] = s0;
    prim[2 * e + 1] = lw;
  } else if (k1) {
    const uint32_t e = base[1] + cls[1];
    mid[2 * e] = s0;
    mid[2 * e + 1] = lw;
  } else if (k2) {
    const uint32_t e = base[2] + cls[2];
    const uint32_t row = l > TILEF ? atomicAdd(&cnt[3], 1u) : NONE;
    bstart[e] = s0;
    blen[e] = l;
    brow[e] = row;
    if (row != NONE)
      for (uint32_t i = 0; i < ND * 256; ++i) rows[static_cast<size_t>(row) * ND * 256 + i] = 0;
  }
}

// The *count entries of a list of grs_seg_runs sorted in LDS from kin / vin into kout / vout: a
// run by the bits below the top byte, a merged entry by the whole key (persistent grid; leaves
// at once when the list is empty).
template <typename K, bool PAIRS, int BLOCK, int I, bool C16, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void grs_seg_local_list(const K* __restrict__ kin,
                                                                  const uint32_t* __restrict__ vin,
                                                                  K* __restrict__ kout,
                                                                  uint32_t* __restrict__ vout,
                                                                  const uint32_t* __restrict__ count_p,
                                                                  const uint32_t* __restrict__ list) {
  constexpr int KR = static_cast<int>(sizeof(K));   // 8-bit rounds of the whole key
  using LS = LocalSort<K, PAIRS, BLOCK, I, C16, KR>;
  __shared__ typename LS::Smem sm;
  const uint32_t count = *count_p;
  for (uint32_t e = blockIdx.x; e < count; e += gridDim.x) {
    const uint32_t lw = list[2 * e + 1];
    LS::run(sm, kin, vin, kout, vout, list[2 * e], lw & 0x7FFFFFFFu, (lw >> 31) ? KR : KR - 1);
    __syncthreads();   // every LDS read of this entry before the next one's
  }
}

}  // namespace grs
