// lab7.hip — round-5 laboratory (not part of libgrs): the MSD sort's LDS segment sort
// (grs::LocalSort, grs_msd.hpp) timed with 0, 1 and 2 of its 8-bit rounds, one workgroup per
// segment (P3's launch), to split its time between HBM and LDS work (tools/lab7.py).
#include <hip/hip_runtime.h>

#include "../gpuradixsort_amd/csrc/grs_msd.hpp"

namespace {

template <int BLOCK, int I, bool C16>
__global__ __launch_bounds__(BLOCK) void lab_p3(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                const uint32_t* __restrict__ off, int rounds) {
  using LS = grs::LocalSort<uint32_t, false, BLOCK, I, C16, 2>;
  __shared__ typename LS::Smem sm;
  const uint32_t lo = off[blockIdx.x], len = off[blockIdx.x + 1] - lo;
  if (len == 0) return;
  LS::run(sm, in, nullptr, out, nullptr, lo, len, rounds);
}

// persistent: workgroup g sorts segments g, g + grid, ...; the next segment's keys are loaded
// into registers after the rounds have left this one in LDS, so they fly during its stores
template <int BLOCK, int I, bool C16, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void lab_p3p(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       const uint32_t* __restrict__ off, uint32_t nseg) {
  using LS = grs::LocalSort<uint32_t, false, BLOCK, I, C16, 2>;
  __shared__ typename LS::Smem sm;
  uint32_t b = blockIdx.x;
  if (b >= nseg) return;
  uint32_t lo = off[b], len = off[b + 1] - lo;
  uint32_t k[I];
  typename LS::Vals v;
  LS::load(k, v, in, nullptr, lo, len);
  for (;;) {
    LS::sort_rounds(sm, k, v, len, 2);
    const uint32_t nb = b + gridDim.x;
    uint32_t nlo = 0, nlen = 0;
    if (nb < nseg) {
      nlo = off[nb];
      nlen = off[nb + 1] - nlo;
      LS::load(k, v, in, nullptr, nlo, nlen);
    }
    LS::store(sm, out, nullptr, lo, len);
    __syncthreads();
    if (nb >= nseg) break;
    b = nb;
    lo = nlo;
    len = nlen;
  }
}

}  // namespace

extern "C" int lab7_p3p(int block, int items, int c16, int per_cu, int cus, const uint32_t* in, uint32_t* out,
                        const uint32_t* off, uint32_t nseg, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3P(B, I, C, M)                                                                              \
  if (block == B && items == I && c16 == C && per_cu * B / 256 == M) {                              \
    hipLaunchKernelGGL((lab_p3p<B, I, C != 0, M>), dim3(per_cu * cus), dim3(B), 0, s, in, out, off, nseg); \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                \
  }
  P3P(768, 24, 1, 6) P3P(256, 20, 0, 4) P3P(256, 20, 0, 5) P3P(256, 20, 0, 6) P3P(512, 20, 0, 6)
#undef P3P
  return -1;
}

extern "C" int lab7_p3(int block, int items, int c16, int rounds, const uint32_t* in, uint32_t* out,
                       const uint32_t* off, uint32_t nseg, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3(B, I, C)                                                                                 \
  if (block == B && items == I && c16 == C) {                                                      \
    hipLaunchKernelGGL((lab_p3<B, I, C != 0>), dim3(nseg), dim3(B), 0, s, in, out, off, rounds);   \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                               \
  }
  P3(256, 20, 0) P3(512, 20, 0) P3(768, 24, 1) P3(256, 12, 0) P3(256, 8, 0) P3(1024, 18, 1) P3(512, 36, 1)
  P3(640, 28, 1) P3(896, 20, 1)
#undef P3
  return -1;
}
