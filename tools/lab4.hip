// lab4.hip — round-4 laboratory for the SHIPPED pass kernel (gpuradixsort_amd/csrc/grs_pass.hpp):
// the library's tile shapes with candidate OPT bits, timed by tools/lab2.py ("p4" variants).
// Not part of libgrs.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../gpuradixsort_amd/csrc/grs_pass.hpp"

extern "C" {

// one pass of the shipped kernel: kb, pairs, block, items, minw, opt (same arguments as
// lab2_v4; hist_stride / range_tiles are ignored)
int lab4_v4(int kb, int pairs, int block, int items, int minw, int opt, const void* in, void* out,
            const uint32_t* vin, uint32_t* vout, uint32_t n, const uint32_t* hist,
            uint32_t* ticket, uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream,
            uint32_t, uint32_t) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long code = (((((long)kb * 2 + pairs) * 10000 + block) * 1000 + items) * 10 + minw) * 10000000L + opt;
  switch (code) {
#define V(KB, P, B, I, M, O)                                                                   \
  case (((((long)KB * 2 + P) * 10000 + B) * 1000 + I) * 10 + M) * 10000000L + O: {             \
    using KT = std::conditional_t<KB == 32, uint32_t, uint64_t>;                               \
    const uint32_t tiles = (n + B * I - 1) / (B * I);                                          \
    hipLaunchKernelGGL((grs::grs_onesweep_v4<KT, P != 0, 8, B, I, M, O>), dim3(tiles), dim3(B), \
                       0, s, (const KT*)in, (KT*)out, vin, vout, n,                            \
                       grs::RadixDigit<KT>{shift, 255u}, hist, ticket, st, st2, err,           \
                       (const grs::RadixDigit<KT>*)nullptr);                                   \
  } break;
    V(32, 0, 1024, 36, 1, 272) V(32, 0, 768, 64, 1, 1040) V(64, 0, 768, 44, 1, 1040)
    V(32, 1, 768, 40, 1, 1040)
#undef V
    default:
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
