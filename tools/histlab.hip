// histlab.hip — laboratory for the upfront digit histogram (not part of libgrs).
// Built by tools/Makefile into tools/libhistlab.so; driven by tools/histlab.py on the GPU box.
//
// hist_var is the library's grs_upfront_hist with its knobs exposed:
//   BLOCK     threads per workgroup
//   COPIES    bank-private histogram copies (lane t adds into copy t % COPIES)
//   PACK16    two digits per 32-bit word as 16-bit halves (else one 32-bit counter)
//   MODE      0 = real, 1 = loads only (HBM floor), 2 = LDS atomics only on hashed keys
//   UNROLL    16-byte loads in flight per thread
#include <hip/hip_runtime.h>

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

namespace {

template <int BLOCK, int COPIES, bool PACK16, int MODE, int UNROLL>
__global__ __launch_bounds__(BLOCK) void hist_var(const uint32_t* __restrict__ keys, uint32_t n,
                                                  uint32_t* __restrict__ g_hist) {
  constexpr int RB = 8, RADIX = 256, P = 4;
  constexpr int PER_COPY = P * (PACK16 ? RADIX / 2 : RADIX);
  constexpr int WORDS = PER_COPY * COPIES;
  __shared__ uint32_t s_hist[WORDS];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < static_cast<uint32_t>(WORDS); i += BLOCK) s_hist[i] = 0;
  __syncthreads();
  const uint32_t copy = t % COPIES;
  uint32_t sink = 0;
  auto count = [&](uint32_t k) {
    if constexpr (MODE == 1) {
      sink ^= k;
    } else {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const uint32_t d = (k >> (p * RB)) & 255u;
        if constexpr (PACK16)
          atomicAdd(&s_hist[(p * (RADIX / 2) + (d >> 1)) * COPIES + copy], 1u << ((d & 1u) << 4));
        else
          atomicAdd(&s_hist[(p * RADIX + d) * COPIES + copy], 1u);
      }
    }
  };
  const uint32_t nvec = n / 4;
  const uint4* kv = reinterpret_cast<const uint4*>(keys);
  const uint32_t stride = gridDim.x * BLOCK;
  uint32_t v = blockIdx.x * BLOCK + t;
  if constexpr (MODE == 2) {
    for (; v < nvec; v += stride) {
      uint32_t h = v * 0x9E3779B9u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h = (h ^ (h >> 15)) * 0x2C1B3C6Du;
        count(h);
      }
    }
  } else {
    for (; v + (UNROLL - 1) * stride < nvec; v += UNROLL * stride) {
      uint4 x[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) x[u] = kv[v + u * stride];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        count(x[u].x);
        count(x[u].y);
        count(x[u].z);
        count(x[u].w);
      }
    }
    for (; v < nvec; v += stride) {
      const uint4 x = kv[v];
      count(x.x);
      count(x.y);
      count(x.z);
      count(x.w);
    }
  }
  __syncthreads();
  if constexpr (MODE == 1) {
    if (sink == 0x12345678u) g_hist[0] = sink;
    return;
  }
  for (uint32_t i = t; i < static_cast<uint32_t>(P * RADIX); i += BLOCK) {
    const uint32_t p = i / RADIX, d = i % RADIX;
    uint32_t c = 0;
    if constexpr (PACK16) {
      const uint32_t* row = &s_hist[(p * (RADIX / 2) + (d >> 1)) * COPIES];
#pragma unroll
      for (int k = 0; k < COPIES; ++k) c += (row[(k + t) % COPIES] >> ((d & 1u) << 4)) & 0xFFFFu;
    } else {
      const uint32_t* row = &s_hist[(p * RADIX + d) * COPIES];
#pragma unroll
      for (int k = 0; k < COPIES; ++k) c += row[(k + t) % COPIES];
    }
    if (c) atomicAdd(&g_hist[i], c);
  }
}

}  // namespace

extern "C" {

// variant ids: see tools/histlab.py
int histlab_run(int variant, int grid, const uint32_t* keys, uint32_t n, uint32_t* hist,
                void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (variant) {
    case 0:  // the library kernel
      hipLaunchKernelGGL((grs::grs_upfront_hist<uint32_t, 8>), dim3(grid), dim3(GRS_HIST_BLOCK), 0,
                         s, keys, n, 0, 32, 4, hist, hist + 4096, 0u);
      break;
#define HV(id, B, C, P16, M, U)                                                              \
  case id:                                                                                   \
    hipLaunchKernelGGL((hist_var<B, C, P16, M, U>), dim3(grid), dim3(B), 0, s, keys, n, hist); \
    break;
    HV(1, 256, 16, true, 0, 4)    // lab copy of the library kernel
    HV(2, 256, 16, true, 1, 4)    // loads only
    HV(3, 256, 16, true, 2, 4)    // atomics only
    HV(4, 512, 32, true, 0, 4)    // 32 copies (exact bank per lane group), 64 KB
    HV(5, 512, 16, false, 0, 4)   // 32-bit counters, 16 copies, 64 KB
    HV(6, 256, 16, true, 0, 8)    // 8 loads in flight
    HV(7, 1024, 32, true, 0, 4)   // one 1024-thread workgroup, 64 KB
    HV(8, 512, 32, true, 2, 4)    // atomics only, 32 copies
    HV(9, 256, 8, true, 0, 4)     // 8 copies, 16 KB
#undef HV
    default:
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
