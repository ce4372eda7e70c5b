// grs_shard.hpp — device steps of the multi-GPU key-range sort (grs_sort_sharded).
//
// New with respect to the reference, which is single-context.  One
// process per GPU; rank r holds the contiguous global input range that follows ranks < r.
// The exchange needs bucket boundaries ("splitters") that every rank agrees on; here they are
// computed on the device, so the only host synchronisation of a sharded sort is reading the
// G x G count matrix before the all-to-all:
//
//   grs_shard_samples    S regularly spaced (key, position) samples of the local shard
//   (RCCL all-gather of the G*S samples, rank-major: gathered index j = rank * S + i)
//   grs_shard_splitters  one workgroup: bitonic sort of the gathered samples by (key, j) in
//                        LDS -- (key, j) order IS (key, global index) order, because ranks
//                        hold consecutive global ranges and a rank's samples are in position
//                        order -- then the G-1 quantiles become this rank's partition digit
//                        (grs::SplitterIdxDigit: splitter keys + shard-local thresholds)
//
// Ties are broken by global index (SURVEY.md §7 "Hard parts"): an input of equal keys splits
// evenly across ranks instead of landing on one, and the buckets are still ranges of the
// global stable order, so concatenating the ranks' outputs gives the stable sort.
#pragma once

#include "grs_kernels.hpp"

namespace grs {

#define GRS_SHARD_SAMPLES_MAX 8192   // gathered samples sorted in one workgroup's LDS

// Threshold of splitter (key, sample from rank rr at shard position p) for the shard of
// `rank` (SplitterIdxDigit): elements of earlier ranks precede it, of later ranks follow it.
__host__ __device__ __forceinline__ uint32_t shard_threshold(uint32_t rr, uint32_t rank, uint32_t p) {
  return rr < rank ? 0u : rr > rank ? 0xFFFFFFFFu : p;
}

// Index of splitter b (b < G - 1) in the sorted samples of M = G * S entries.
__host__ __device__ __forceinline__ uint32_t shard_quantile(uint32_t b, uint32_t m, uint32_t g) {
  return static_cast<uint32_t>((static_cast<uint64_t>(b) + 1) * m / g);
}

// Sample i at shard position floor(i * n / S); an empty shard contributes (max key, max pos).
template <typename K>
__global__ void grs_shard_samples(const K* __restrict__ keys, uint32_t n, uint32_t s,
                                  K* __restrict__ skeys, uint32_t* __restrict__ spos) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < s; i += gridDim.x * blockDim.x) {
    if (n == 0) {
      skeys[i] = static_cast<K>(~static_cast<K>(0));
      spos[i] = 0xFFFFFFFFu;
    } else {
      const uint32_t p = static_cast<uint32_t>((static_cast<uint64_t>(i) * n) / s);
      skeys[i] = keys[p];
      spos[i] = p;
    }
  }
}

// One 1024-thread workgroup.  skeys / spos: the gathered samples (m = g * s, rank-major).
// Writes this rank's partition digit with N = compile-time splitter slots (>= g - 1; the
// unused slots never count).
template <typename K, int N>
__global__ __launch_bounds__(1024) void grs_shard_splitters(const K* __restrict__ skeys,
                                                            const uint32_t* __restrict__ spos,
                                                            uint32_t g, uint32_t s, uint32_t rank,
                                                            SplitterIdxDigit<K, N>* __restrict__ out) {
  __shared__ K lk[GRS_SHARD_SAMPLES_MAX];
  __shared__ uint32_t lj[GRS_SHARD_SAMPLES_MAX];
  const uint32_t m = g * s;
  uint32_t p2 = 1;
  while (p2 < m) p2 <<= 1;
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < p2; i += blockDim.x) {
    lk[i] = i < m ? skeys[i] : static_cast<K>(~static_cast<K>(0));
    lj[i] = i < m ? i : 0xFFFFFFFFu;   // padding sorts after every sample
  }
  __syncthreads();
  // bitonic sort, ascending by (key, j)
  for (uint32_t k = 2; k <= p2; k <<= 1) {
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      for (uint32_t i = t; i < p2; i += blockDim.x) {
        const uint32_t l = i ^ jj;
        if (l > i) {
          const K ka = lk[i], kb = lk[l];
          const uint32_t ja = lj[i], jb = lj[l];
          const bool a_gt_b = ka > kb || (ka == kb && ja > jb);
          const bool up = (i & k) == 0;
          if (a_gt_b == up) {
            lk[i] = kb;
            lk[l] = ka;
            lj[i] = jb;
            lj[l] = ja;
          }
        }
      }
      __syncthreads();
    }
  }
  if (t < static_cast<uint32_t>(GRS_MAX_SPLITTERS)) {
    K key = static_cast<K>(~static_cast<K>(0));
    uint32_t th = 0xFFFFFFFFu;
    if (t + 1 < g && t < static_cast<uint32_t>(N)) {
      const uint32_t q = shard_quantile(t, m, g);
      const uint32_t j = lj[q];
      key = lk[q];
      th = shard_threshold(j / s, rank, spos[j]);
    }
    out->s[t] = key;
    out->th[t] = th;
    if (t == 0) out->count = N;
  }
}

// The same splitters when every rank's samples are SORTED (samples of a sorted shard, the
// presorted exchange): the rank of gathered sample j = (r, i) in (key, j) order is i plus, for
// every other rank r', the samples of r' before it -- upper_bound of its key in r' < r,
// lower_bound in r' > r -- found by binary search in LDS instead of a bitonic sort.  One
// 1024-thread workgroup; output identical to grs_shard_splitters.
template <typename K, int N>
__global__ __launch_bounds__(1024) void grs_shard_splitters_sorted(const K* __restrict__ skeys,
                                                                   const uint32_t* __restrict__ spos,
                                                                   uint32_t g, uint32_t s, uint32_t rank,
                                                                   SplitterIdxDigit<K, N>* __restrict__ out) {
  __shared__ K lk[GRS_SHARD_SAMPLES_MAX];
  const uint32_t m = g * s;
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < m; i += blockDim.x) lk[i] = skeys[i];
  if (t < static_cast<uint32_t>(GRS_MAX_SPLITTERS)) {   // unused slots never count
    out->s[t] = static_cast<K>(~static_cast<K>(0));
    out->th[t] = 0xFFFFFFFFu;
    if (t == 0) out->count = N;
  }
  __syncthreads();
  for (uint32_t j = t; j < m; j += blockDim.x) {
    const uint32_t r = j / s;
    const K key = lk[j];
    uint32_t q = j - r * s;
    for (uint32_t rr = 0; rr < g; ++rr) {
      if (rr == r) continue;
      const K* l = lk + rr * s;
      uint32_t lo = 0, hi = s;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rr < r ? l[mid] <= key : l[mid] < key) lo = mid + 1; else hi = mid;
      }
      q += lo;
    }
    // sample j is splitter b when its rank is quantile b (ranks are a permutation of [0, m))
    for (uint32_t b = 0; b + 1 < g && b < static_cast<uint32_t>(N); ++b) {
      if (shard_quantile(b, m, g) == q) {
        out->s[b] = key;
        out->th[b] = shard_threshold(r, rank, spos[j]);
      }
    }
  }
}

}  // namespace grs

namespace grs {

// Chunked exchange (GRS_OPT_EXCHANGE = 3): the partition digit of chunk c of the shard (shard
// positions [c * chunk, ...)) takes chunk-local indices, so its thresholds move down by
// c * chunk (a threshold at or below the chunk's start becomes 0: every element of the chunk is
// at or past it).  One thread per (chunk, splitter slot).
template <typename K, int N>
__global__ void grs_shard_chunk_digits(const SplitterIdxDigit<K, N>* __restrict__ dig, uint32_t chunks,
                                       uint32_t chunk, SplitterIdxDigit<K, N>* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= chunks * GRS_MAX_SPLITTERS) return;
  const uint32_t c = i / GRS_MAX_SPLITTERS, j = i % GRS_MAX_SPLITTERS;
  const uint64_t base = static_cast<uint64_t>(c) * chunk;
  if (j == 0) out[c].count = dig->count;
  out[c].s[j] = dig->s[j];
  const uint32_t th = dig->th[j];
  out[c].th[j] = th == 0xFFFFFFFFu ? th : th <= base ? 0u : static_cast<uint32_t>(th - base);
}

// The chunked exchange's plan for chunk c: mat = the G x G count matrix of that chunk (row r:
// what rank r's chunk c sends to each bucket), its buckets contiguous from c * chunk of the send
// buffer; received chunk-major: chunk c's runs from every source follow everything received in
// chunks < c (recv_base), in source-rank order.  send_off / recv_off: G entries; returns the
// items received in this chunk.
__host__ __forceinline__ uint64_t shard_chunk_plan(const uint32_t* mat, int g, int me, uint64_t chunk_start,
                                                   uint64_t recv_base, uint64_t* send_off, uint64_t* recv_off) {
  uint64_t so = chunk_start, ro = recv_base;
  for (int p = 0; p < g; ++p) {
    send_off[p] = so;
    so += mat[me * g + p];
    recv_off[p] = ro;
    ro += mat[p * g + me];
  }
  return ro - recv_base;
}

}  // namespace grs
