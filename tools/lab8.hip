// lab8.hip — round-6 laboratory (not part of libgrs): P3 (grs::LocalSort, grs_msd.hpp) with
// one-dword-per-lane HBM accesses (the shipped round-5 form) against 16-B accesses through LDS,
// on segments of P3's real geometry: variable lengths, read from regions at any alignment,
// written packed at any alignment (tools/lab8.py).
//   MODE 0  dword striped loads, dword stores (LocalSort::run, round 5)
//   MODE 1  dword striped loads, 16-B stores rotated per workgroup (LocalSort::run_vec, shipped)
//   MODE 3  as 1 without the rotation (run_vec<false>)
// (MODE 2, 16-B LDS-DMA loads through LDS, measured in session r6s3 and removed: 2^30 2025 us
// against 1829 for MODE 3; skeleton 1634 vs 1670)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../gpuradixsort_amd/csrc/grs_msd.hpp"

namespace {

template <int BLOCK, int I, bool C16, int MODE>
__global__ __launch_bounds__(BLOCK) void lab_p3v(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ inoff,
                                                 const uint32_t* __restrict__ outoff,
                                                 const uint32_t* __restrict__ lens, int rounds) {
  using LS = grs::LocalSort<uint32_t, false, BLOCK, I, C16, 2>;
  __shared__ typename LS::Smem sm;
  const uint32_t len = lens[blockIdx.x];
  if (len == 0) return;
  const uint32_t* kin = in + inoff[blockIdx.x];
  uint32_t* kout = out + outoff[blockIdx.x];
  if constexpr (MODE == 0) LS::run(sm, kin, nullptr, kout, nullptr, 0u, len, rounds);
  else if constexpr (MODE == 3) LS::template run_vec<false>(sm, kin, nullptr, kout, nullptr, len, rounds);
  else LS::template run_vec<>(sm, kin, nullptr, kout, nullptr, len, rounds);
}

// u64 keys (C5's P3): MODE 0 = LocalSort::run (6 rounds), 1 = run_vec (2 rounds + the runs
// finished by insertion, 16-B stores)
template <int BLOCK, int I, int MODE>
__global__ __launch_bounds__(BLOCK) void lab_p3w(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                 const uint32_t* __restrict__ inoff,
                                                 const uint32_t* __restrict__ outoff,
                                                 const uint32_t* __restrict__ lens, int rounds) {
  using LS = grs::LocalSort<uint64_t, false, BLOCK, I, false>;
  __shared__ typename LS::Smem sm;
  const uint32_t len = lens[blockIdx.x];
  if (len == 0) return;
  const uint64_t* kin = in + inoff[blockIdx.x];
  uint64_t* kout = out + outoff[blockIdx.x];
  if constexpr (MODE == 0) LS::run(sm, kin, nullptr, kout, nullptr, 0u, len, rounds);
  else LS::template run_vec<>(sm, kin, nullptr, kout, nullptr, len, rounds);
}

// u32 keys, low halves in LDS (grs::LocalSort16, round 7 of the lab): MINW waves a SIMD
template <int BLOCK, int I, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void lab_p3h(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       const uint32_t* __restrict__ inoff,
                                                       const uint32_t* __restrict__ outoff,
                                                       const uint32_t* __restrict__ lens, int rounds) {
  using LS = grs::LocalSort16<BLOCK, I>;
  __shared__ typename LS::Smem sm;
  const uint32_t len = lens[blockIdx.x];
  if (len == 0) return;
  LS::run(sm, in + inoff[blockIdx.x], out + outoff[blockIdx.x], len, rounds);
}

// persistent P3 with a static segment stride (no ticket): the next segment's table entries are
// read while this one sorts, and its key loads follow this one's stores at once (HALF: LocalSort16)
template <int BLOCK, int I, int MINW, bool HALF>
__global__ __launch_bounds__(BLOCK, MINW) void lab_p3s(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       const uint32_t* __restrict__ inoff,
                                                       const uint32_t* __restrict__ outoff,
                                                       const uint32_t* __restrict__ lens, uint32_t nseg, int rounds) {
  using LS = grs::LocalSort<uint32_t, false, BLOCK, I, (BLOCK > 256), 2>;
  using LH = grs::LocalSort16<BLOCK, (I + 1) / 2 * 2>;
  __shared__ std::conditional_t<HALF, typename LH::Smem, typename LS::Smem> sm;
  uint32_t b = blockIdx.x;
  uint32_t len = lens[b], io = inoff[b], oo = outoff[b];
  for (; b < nseg; b += gridDim.x) {
    const uint32_t nb = b + gridDim.x;
    uint32_t nlen = 0, nio = 0, noo = 0;
    if (nb < nseg) {
      nlen = lens[nb];
      nio = inoff[nb];
      noo = outoff[nb];
    }
    if (len != 0) {
      if constexpr (HALF) LH::run(sm, in + io, out + oo, len, rounds);
      else LS::template run_vec<>(sm, in + io, nullptr, out + oo, nullptr, len, rounds);
    }
    __syncthreads();   // (LDS reuse by the next segment)
    len = nlen;
    io = nio;
    oo = noo;
  }
}

}  // namespace

extern "C" int lab8_p3s(int block, int items, int minw, int half, int grid, int rounds, const uint32_t* in,
                        uint32_t* out, const uint32_t* inoff, const uint32_t* outoff, const uint32_t* lens,
                        uint32_t nseg, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (grid <= 0 || static_cast<uint32_t>(grid) > nseg) return -3;
#define P3S(B, I, M, H)                                                                                   \
  if (block == B && items == I && minw == M && half == H) {                                               \
    hipLaunchKernelGGL((lab_p3s<B, I, M, H != 0>), dim3(grid), dim3(B), 0, s, in, out, inoff, outoff, lens, \
                       nseg, rounds);                                                                     \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                      \
  }
  P3S(256, 20, 6, 0) P3S(256, 20, 8, 0) P3S(768, 23, 6, 0) P3S(512, 34, 6, 1) P3S(256, 20, 8, 1)
#undef P3S
  return -1;
}

extern "C" int lab8_p3h(int block, int items, int minw, int rounds, const uint32_t* in, uint32_t* out,
                        const uint32_t* inoff, const uint32_t* outoff, const uint32_t* lens, uint32_t nseg,
                        void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3H(B, I, M)                                                                                          \
  if (block == B && items == I && minw == M) {                                                              \
    hipLaunchKernelGGL((lab_p3h<B, I, M>), dim3(nseg), dim3(B), 0, s, in, out, inoff, outoff, lens, rounds);   \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                        \
  }
  P3H(512, 34, 8) P3H(512, 36, 6) P3H(256, 68, 4) P3H(768, 24, 6) P3H(512, 34, 6) P3H(256, 68, 5)
  P3H(256, 20, 8) P3H(256, 16, 8) P3H(512, 10, 8) P3H(768, 46, 6) P3H(1024, 34, 8) P3H(512, 68, 4)
  P3H(1024, 36, 4)
#undef P3H
  return -1;
}

extern "C" int lab8_p3w(int block, int items, int mode, int rounds, const uint64_t* in, uint64_t* out,
                        const uint32_t* inoff, const uint32_t* outoff, const uint32_t* lens, uint32_t nseg,
                        void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3W(B, I, M)                                                                                          \
  if (block == B && items == I && mode == M)                                                                  \
    hipLaunchKernelGGL((lab_p3w<B, I, M>), dim3(nseg), dim3(B), 0, s, in, out, inoff, outoff, lens, rounds);   \
  else
  P3W(256, 20, 0) P3W(256, 20, 1) P3W(512, 10, 0) P3W(512, 10, 1) P3W(1024, 5, 0) P3W(1024, 5, 1)
    return -1;
#undef P3W
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int lab8_p3(int block, int items, int c16, int mode, int rounds, const uint32_t* in, uint32_t* out,
                       const uint32_t* inoff, const uint32_t* outoff, const uint32_t* lens, uint32_t nseg,
                       void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
#define P3(B, I, C, M)                                                                                     \
  if (block == B && items == I && c16 == C && mode == M) {                                                \
    hipLaunchKernelGGL((lab_p3v<B, I, C != 0, M>), dim3(nseg), dim3(B), 0, s, in, out, inoff, outoff, lens, \
                       rounds);                                                                           \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                                      \
  }
  P3(768, 24, 1, 0) P3(768, 24, 1, 1) P3(768, 24, 1, 3)
  P3(256, 20, 0, 0) P3(256, 20, 0, 1) P3(256, 20, 0, 3)
  P3(512, 10, 0, 1) P3(1024, 5, 0, 1) P3(1024, 5, 1, 1)
  P3(1024, 18, 1, 1) P3(512, 36, 1, 1) P3(768, 23, 1, 1) P3(640, 28, 1, 1)
  P3(256, 19, 0, 1) P3(768, 22, 1, 1)
#undef P3
  return -1;
}
