// lab5.hip — round-5 laboratory (not part of libgrs): the pieces of an MSD-first u32 sort,
// timed one by one so the whole can be priced before it is built (tools/lab5.py).
//
//   H1  histogram of the top byte only (one LDS add per key): the read floor of the keys
//   H2  histogram of byte 2 per top-byte bucket, over data already grouped by top byte
//       (a block's chunk meets at most a few buckets: LDS counters for a window of 2 buckets,
//       global atomics for keys past it)
//   P3  one workgroup per 16-bit-prefix segment: the segment is read once, sorted by its low
//       16 bits in LDS (two 8-bit digit rounds of lane-ordered returning LDS adds, as in the
//       pass), written once -- contiguous HBM traffic instead of two scatter passes
//   copy  a contiguous read + write of the same bytes (P3's HBM floor)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

namespace {

constexpr int kH2Copies = 32;
constexpr int kH2Win = 2;   // buckets counted in LDS per block

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void msd_h2(const uint32_t* __restrict__ keys, uint32_t n,
                                                uint32_t chunk, uint32_t* __restrict__ g_h2) {
  __shared__ __attribute__((aligned(16))) uint32_t h[kH2Win * 256 * kH2Copies];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < kH2Win * 256 * kH2Copies; i += BLOCK) h[i] = 0;
  const uint32_t c0 = blockIdx.x * chunk;
  const uint32_t c1 = min(n, c0 + chunk);
  const uint32_t s0 = keys[c0] >> 24;
  __syncthreads();
  uint32_t* const base = h + (t & (kH2Copies - 1));
  auto count = [&](uint32_t k) {
    const uint32_t s = (k >> 24) - s0;
    if (s < kH2Win)
      atomicAdd(base + (s * 256 + ((k >> 16) & 255u)) * kH2Copies, 1u);
    else
      atomicAdd(&g_h2[k >> 16], 1u);
  };
  const uint4* kv = reinterpret_cast<const uint4*>(keys + c0);
  const uint32_t nv = (c1 - c0) / 4;
  uint32_t v = t;
  for (; v + 3 * BLOCK < nv; v += 4 * BLOCK) {
    uint4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = kv[v + u * BLOCK];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      count(x[u].x);
      count(x[u].y);
      count(x[u].z);
      count(x[u].w);
    }
  }
  for (; v < nv; v += BLOCK) {
    const uint4 x = kv[v];
    count(x.x);
    count(x.y);
    count(x.z);
    count(x.w);
  }
  for (uint32_t i = c0 + nv * 4 + t; i < c1; i += BLOCK) count(keys[i]);
  __syncthreads();
  for (uint32_t i = t; i < kH2Win * 256; i += BLOCK) {
    const uint32_t* row = h + i * kH2Copies;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kH2Copies; ++k) c += row[(k + t) & (kH2Copies - 1)];
    const uint32_t s = s0 + i / 256;
    if (c != 0 && s < 256) atomicAdd(&g_h2[s * 256 + i % 256], c);
  }
}

// P3: segment = [off[b], off[b+1]); keys sorted by bits [0, 16) in LDS, stably; out-of-place.
template <int BLOCK, int I, bool C16>
__global__ __launch_bounds__(BLOCK) void msd_p3(const uint32_t* __restrict__ in,
                                                uint32_t* __restrict__ out,
                                                const uint32_t* __restrict__ off,
                                                uint32_t* __restrict__ err) {
  constexpr uint32_t W = BLOCK / 64, SMAX = BLOCK * I;
  __shared__ uint32_t sk[SMAX];
  __shared__ uint32_t cnt[W * 256 / (C16 ? 2 : 1)];
  __shared__ uint32_t wtot[4];
  uint16_t* const c16 = reinterpret_cast<uint16_t*>(cnt);
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t lo = off[blockIdx.x];
  const uint32_t len = off[blockIdx.x + 1] - lo;
  if (len > SMAX) {
    if (t == 0) atomicAdd(err, 1u);
    return;
  }
  if (len == 0) return;
  uint32_t k[I];
#pragma unroll
  for (uint32_t j = 0; j < I; ++j) {
    const uint32_t i = w * 64 * I + j * 64 + lane;
    k[j] = i < len ? in[lo + i] : 0u;
  }
  for (int pass = 0; pass < 2; ++pass) {
    const int shift = 8 * pass;
    for (uint32_t c = t; c < W * 256 / (C16 ? 2 : 1); c += BLOCK) cnt[c] = 0;
    __syncthreads();
    uint32_t r[I];
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * 64 * I + j * 64 + lane;
      const uint32_t d = (k[j] >> shift) & 255u;
      if constexpr (C16) {
        const uint32_t sh = (d & 1u) << 4;
        r[j] = i < len ? (atomicAdd(&cnt[(w * 256 + d) >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
      } else {
        r[j] = i < len ? atomicAdd(&cnt[w * 256 + d], 1u) : 0u;
      }
    }
    __syncthreads();
    auto cld = [&](uint32_t a) -> uint32_t { if constexpr (C16) return c16[a]; else return cnt[a]; };
    auto cst = [&](uint32_t a, uint32_t v) { if constexpr (C16) c16[a] = static_cast<uint16_t>(v); else cnt[a] = v; };
    uint32_t c[W], tot = 0, incl = 0;
    if (t < 256) {
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        c[ww] = cld(ww * 256 + t);
        tot += c[ww];
      }
      incl = grs::wave_scan_dpp(tot);
      if (lane == 63) wtot[w] = incl;
    }
    __syncthreads();
    if (t < 256) {
      uint32_t b = incl - tot;
#pragma unroll
      for (uint32_t ww = 0; ww < 4; ++ww) b += ww < w ? wtot[ww] : 0u;
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        cst(ww * 256 + t, b);
        b += c[ww];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * 64 * I + j * 64 + lane;
      if (i < len) sk[cld(w * 256 + ((k[j] >> shift) & 255u)) + r[j]] = k[j];
    }
    __syncthreads();
    if (pass == 0) {
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t i = w * 64 * I + j * 64 + lane;
        if (i < len) k[j] = sk[i];
      }
    }
  }
  // sorted segment in LDS: stored by consecutive threads
  for (uint32_t i = t; i < len; i += BLOCK) out[lo + i] = sk[i];
}

// P3 with 16-bit keys in LDS: a segment's keys share their top 16 bits (its prefix), so only
// the low halves are ranked, moved and stored; half the LDS per key.  PK: the low half and the
// rank share one register per key.
template <int BLOCK, int I, bool C16>
__global__ __launch_bounds__(BLOCK) void msd_p3h(const uint32_t* __restrict__ in,
                                                 uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ off,
                                                 uint32_t* __restrict__ err) {
  constexpr uint32_t W = BLOCK / 64, SMAX = BLOCK * I;
  __shared__ uint16_t sk[SMAX];
  __shared__ uint32_t cnt[W * 256 / (C16 ? 2 : 1)];
  __shared__ uint32_t wtot[4];
  uint16_t* const c16 = reinterpret_cast<uint16_t*>(cnt);
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t lo = off[blockIdx.x];
  const uint32_t len = off[blockIdx.x + 1] - lo;
  if (len > SMAX) {
    if (t == 0) atomicAdd(err, 1u);
    return;
  }
  if (len == 0) return;
  const uint32_t prefix = blockIdx.x << 16;
  uint32_t k[I];   // low 16 bits; the rank in the high half during a round
#pragma unroll
  for (uint32_t j = 0; j < I; ++j) {
    const uint32_t i = w * 64 * I + j * 64 + lane;
    k[j] = i < len ? (in[lo + i] & 0xFFFFu) : 0u;
  }
  auto cld = [&](uint32_t a) -> uint32_t { if constexpr (C16) return c16[a]; else return cnt[a]; };
  auto cst = [&](uint32_t a, uint32_t v) { if constexpr (C16) c16[a] = static_cast<uint16_t>(v); else cnt[a] = v; };
  for (int pass = 0; pass < 2; ++pass) {
    const int shift = 8 * pass;
    for (uint32_t c = t; c < W * 256 / (C16 ? 2 : 1); c += BLOCK) cnt[c] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * 64 * I + j * 64 + lane;
      const uint32_t d = (k[j] >> shift) & 255u;
      uint32_t r;
      if constexpr (C16) {
        const uint32_t sh = (d & 1u) << 4;
        r = i < len ? (atomicAdd(&cnt[(w * 256 + d) >> 1], 1u << sh) >> sh) & 0xFFFFu : 0u;
      } else {
        r = i < len ? atomicAdd(&cnt[w * 256 + d], 1u) : 0u;
      }
      k[j] = (k[j] & 0xFFFFu) | (r << 16);
    }
    __syncthreads();
    uint32_t c[W], tot = 0, incl = 0;
    if (t < 256) {
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        c[ww] = cld(ww * 256 + t);
        tot += c[ww];
      }
      incl = grs::wave_scan_dpp(tot);
      if (lane == 63) wtot[w] = incl;
    }
    __syncthreads();
    if (t < 256) {
      uint32_t b = incl - tot;
#pragma unroll
      for (uint32_t ww = 0; ww < 4; ++ww) b += ww < w ? wtot[ww] : 0u;
#pragma unroll
      for (uint32_t ww = 0; ww < W; ++ww) {
        cst(ww * 256 + t, b);
        b += c[ww];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < I; ++j) {
      const uint32_t i = w * 64 * I + j * 64 + lane;
      const uint32_t v = k[j] & 0xFFFFu;
      if (i < len) sk[cld(w * 256 + ((v >> shift) & 255u)) + (k[j] >> 16)] = static_cast<uint16_t>(v);
    }
    __syncthreads();
    if (pass == 0) {
#pragma unroll
      for (uint32_t j = 0; j < I; ++j) {
        const uint32_t i = w * 64 * I + j * 64 + lane;
        k[j] = i < len ? sk[i] : 0u;
      }
    }
  }
  for (uint32_t i = t; i < len; i += BLOCK) out[lo + i] = prefix | sk[i];
}

__global__ __launch_bounds__(256) void copy4(const uint4* __restrict__ in, uint4* __restrict__ out,
                                             uint32_t n4) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) out[i] = in[i];
}

}  // namespace

extern "C" {

int lab5_h1(const uint32_t* keys, uint32_t n, uint32_t* hist, int cus, int qn, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int slots = 2 * cus;
  const int need = static_cast<int>(n >> 20) + 1;
  int grid = slots;
  if (grid < need) grid = (need + slots - 1) / slots * slots;
  if (qn == 1)
    hipLaunchKernelGGL((grs::grs_upfront_hist2<uint32_t, 8, false, 1>), dim3(grid), dim3(512), 0, s,
                       keys, n, 24, 32, 1, hist, (uint32_t*)nullptr, 0u, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u);
  else
    hipLaunchKernelGGL((grs::grs_upfront_hist2<uint32_t, 8, true>), dim3(grid), dim3(512), 0, s,
                       keys, n, 0, 32, 4, hist, (uint32_t*)nullptr, 0u, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab5_h2(const uint32_t* keys, uint32_t n, uint32_t chunk, uint32_t* h2, int block, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t grid = (n + chunk - 1) / chunk;
  if (block == 512)
    hipLaunchKernelGGL(msd_h2<512>, dim3(grid), dim3(512), 0, s, keys, n, chunk, h2);
  else if (block == 1024)
    hipLaunchKernelGGL(msd_h2<1024>, dim3(grid), dim3(1024), 0, s, keys, n, chunk, h2);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab5_p3(int block, int items, int c16, const uint32_t* in, uint32_t* out, const uint32_t* off,
            uint32_t nseg, uint32_t* err, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3(B, I, C)                                                                           \
  if (block == B && items == I && c16 == C) {                                                \
    hipLaunchKernelGGL((msd_p3<B, I, C != 0>), dim3(nseg), dim3(B), 0, s, in, out, off, err); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                          \
  }
  P3(256, 20, 0) P3(256, 24, 0) P3(512, 10, 0) P3(256, 20, 1) P3(1024, 20, 0) P3(1024, 20, 1)
  P3(512, 40, 0) P3(512, 40, 1) P3(1024, 24, 1) P3(768, 24, 1)
#undef P3
#define P3H(B, I, C)                                                                          \
  if (block == B && items == I && c16 == C + 10) {                                            \
    hipLaunchKernelGGL((msd_p3h<B, I, C != 0>), dim3(nseg), dim3(B), 0, s, in, out, off, err); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                           \
  }
  P3H(256, 20, 0) P3H(256, 20, 1) P3H(256, 24, 0) P3H(512, 10, 0) P3H(512, 12, 0)
  P3H(768, 24, 1) P3H(768, 24, 0) P3H(512, 36, 1) P3H(512, 36, 0) P3H(1024, 18, 1) P3H(1024, 20, 1)
  P3H(256, 72, 1) P3H(384, 48, 1)
#undef P3H
  return -1;
}

int lab5_copy(const uint32_t* in, uint32_t* out, uint32_t n, int grid, void* stream) {
  hipLaunchKernelGGL(copy4, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
