// lab.hip — kernel laboratory (not part of libgrs): timing ablations of one onesweep pass.
// Built by tools/Makefile into tools/liblab*.so; driven by tools/lab.py on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "r1_kernels.hpp"

namespace {

__global__ void copy_x4(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t n4) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
    out[i] = in[i];
}

int g_persist_grid = 0;
int g_stream = 0;

template <typename K, bool PAIRS, int BLOCK, int ITEMS, int DBG>
void launch(const void* in, void* out, const uint32_t* vin, uint32_t* vout, uint32_t n,
            const uint32_t* hist, uint32_t* ticket, uint32_t* st, uint32_t* st2, uint32_t* err,
            int shift, hipStream_t s) {
  constexpr int TILE = BLOCK * ITEMS;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  const K* ki = static_cast<const K*>(in);
  K* ko = static_cast<K*>(out);
  if (g_stream > 0) {
    if constexpr (DBG == 0 && ITEMS * (PAIRS ? 2 : 1) <= 63 &&
                  sizeof(grs::StreamSmem<K, PAIRS, 8, BLOCK, ITEMS>) <= 160 * 1024)
      hipLaunchKernelGGL((grs::grs_onesweep_stream<K, PAIRS, 8, BLOCK, ITEMS>), dim3(g_stream),
                         dim3(BLOCK), 0, s, ki, ko, vin, vout, n, grs::RadixDigit<K>{shift, 255u},
                         hist, ticket, st, st2, err);
  } else if (g_persist_grid > 0)
    hipLaunchKernelGGL((grs::grs_onesweep_persistent<K, PAIRS, 8, BLOCK, ITEMS, DBG>),
                       dim3(g_persist_grid), dim3(BLOCK), 0, s, ki, ko, vin, vout, n,
                       grs::RadixDigit<K>{shift, 255u}, hist, ticket, st, st2, err);
  else
    hipLaunchKernelGGL((grs::grs_onesweep_pass<K, PAIRS, 8, BLOCK, ITEMS, DBG>), dim3(tiles),
                       dim3(BLOCK), 0, s, ki, ko, vin, vout, n, grs::RadixDigit<K>{shift, 255u},
                       hist, ticket, st, st2, err);
}

}  // namespace

extern "C" {

void lab_set_persistent(int grid) {
  // grid > 0: register-prefetch persistent kernel; grid < 0: LDS-DMA stream kernel (-grid WGs)
  g_persist_grid = grid > 0 ? grid : 0;
  g_stream = grid < 0 ? -grid : 0;
}

// key (kb = 32/64), payload, block, items, dbg
int lab_pass2(int kb, int pairs, int block, int items, int dbg, const void* in, void* out,
              const uint32_t* vin, uint32_t* vout, uint32_t n, const uint32_t* hist,
              uint32_t* ticket, uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long code = ((((long)kb * 2 + pairs) * 10000 + block) * 100 + items) * 100 + dbg;
#ifdef LAB_MIN
  (void)s; (void)code; (void)in; (void)out; (void)vin; (void)vout; (void)n; (void)hist;
  (void)ticket; (void)st; (void)st2; (void)err; (void)shift;
  return -1;
#else
  switch (code) {
#define V(KB, P, B, I, D)                                                                     \
  case ((((long)KB * 2 + P) * 10000 + B) * 100 + I) * 100 + D:                                  \
    launch<std::conditional_t<KB == 32, uint32_t, uint64_t>, P != 0, B, I, D>(                \
        in, out, vin, vout, n, hist, ticket, st, st2, err, shift, s);                         \
    break;
    // u32 keys-only
    V(32, 0, 256, 16, 0) V(32, 0, 256, 16, 16) V(32, 0, 256, 32, 0) V(32, 0, 256, 32, 16)
    V(32, 0, 512, 16, 0) V(32, 0, 512, 16, 16) V(32, 0, 256, 24, 16) V(32, 0, 512, 24, 16)
    V(32, 0, 256, 32, 24) V(32, 0, 256, 32, 25) V(32, 0, 512, 16, 24) V(32, 0, 256, 32, 17)
    V(32, 0, 256, 32, 19)
    V(32, 0, 512, 24, 0) V(32, 0, 512, 24, 8) V(32, 0, 512, 16, 1536) V(32, 0, 512, 16, 1280)
    V(32, 0, 512, 16, 1544) V(32, 0, 512, 24, 1280) V(32, 0, 256, 16, 2048) V(32, 0, 256, 24, 1536)
    V(32, 0, 512, 32, 0) V(32, 0, 1024, 16, 0) V(32, 0, 1024, 12, 0) V(32, 0, 512, 20, 0)
    V(32, 0, 512, 24, 32) V(32, 0, 512, 24, 1) V(32, 0, 512, 12, 0) V(32, 0, 256, 24, 0)
    V(32, 0, 512, 16, 1024) V(32, 0, 256, 16, 1024) V(32, 0, 256, 32, 1024)
    V(32, 0, 512, 8, 0) V(32, 1, 512, 8, 0) V(64, 0, 512, 8, 0)
    V(32, 0, 512, 24, 65) V(32, 0, 512, 24, 129) V(32, 0, 512, 24, 4097) V(32, 0, 512, 24, 4289)
    V(32, 0, 512, 24, 3)
    // u32 pairs
    V(32, 1, 256, 16, 16) V(32, 1, 256, 24, 16) V(32, 1, 256, 32, 16) V(32, 1, 512, 16, 16)
    V(32, 1, 512, 8, 16) V(32, 1, 256, 16, 0) V(32, 1, 256, 32, 0)
    // u64 keys-only
    V(64, 0, 256, 16, 16) V(64, 0, 256, 24, 16) V(64, 0, 256, 32, 16) V(64, 0, 512, 16, 16)
    V(64, 0, 256, 8, 16) V(64, 0, 256, 16, 0)
    // u64 pairs
    V(64, 1, 256, 12, 16) V(64, 1, 256, 16, 16) V(64, 1, 512, 8, 16)
#undef V
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
#endif
}

// atomic-rank pass: grid 0 = one tile per workgroup, grid > 0 = persistent with that grid
int lab_ar(int kb, int pairs, int block, int items, int dbg, int grid, const void* in, void* out,
           const uint32_t* vin, uint32_t* vout, uint32_t n, const uint32_t* hist, uint32_t* ticket,
           uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long code = ((((long)kb * 2 + pairs) * 10000 + block) * 100 + items) * 100 + dbg;
  switch (code) {
#define A(KB, P, B, I, D)                                                                     \
  case ((((long)KB * 2 + P) * 10000 + B) * 100 + I) * 100 + D: {                                \
    using KT = std::conditional_t<KB == 32, uint32_t, uint64_t>;                              \
    const uint32_t tiles = (n + B * I - 1) / (B * I);                                         \
    if (grid > 0)                                                                             \
      hipLaunchKernelGGL((grs::grs_onesweep_ar_persist<KT, P != 0, 8, B, I, D>), dim3(grid),   \
                         dim3(B), 0, s, (const KT*)in, (KT*)out, vin, vout, n,                \
                         grs::RadixDigit<KT>{shift, 255u}, hist, ticket, st, st2, err);       \
    else                                                                                      \
      hipLaunchKernelGGL((grs::grs_onesweep_ar<KT, P != 0, 8, B, I, D>), dim3(tiles), dim3(B), \
                         0, s, (const KT*)in, (KT*)out, vin, vout, n,                         \
                         grs::RadixDigit<KT>{shift, 255u}, hist, ticket, st, st2, err);       \
  } break;
#ifdef LAB_MIN
    A(32, 0, 512, 24, 64) A(32, 1, 512, 16, 64) A(32, 1, 512, 12, 64) A(64, 0, 512, 16, 64)
    A(64, 0, 512, 12, 64) A(64, 1, 512, 8, 64) A(64, 1, 512, 12, 64) A(32, 0, 1024, 16, 64)
#else
    A(32, 0, 512, 24, 0) A(32, 0, 512, 16, 0) A(32, 0, 512, 20, 0) A(32, 0, 512, 32, 0)
    A(32, 0, 256, 16, 0) A(32, 0, 256, 24, 0) A(32, 0, 256, 32, 0) A(32, 0, 1024, 16, 0)
    A(32, 0, 512, 12, 0) A(32, 0, 1024, 12, 0) A(32, 0, 512, 8, 0)
    A(32, 1, 512, 16, 0) A(32, 1, 512, 12, 0) A(32, 1, 256, 16, 0) A(32, 1, 512, 8, 0)
    A(64, 0, 512, 16, 0) A(64, 0, 512, 12, 0) A(64, 0, 256, 16, 0) A(64, 0, 512, 8, 0)
    A(64, 1, 512, 8, 0) A(64, 1, 512, 12, 0) A(64, 1, 256, 12, 0)
    A(32, 1, 512, 20, 0) A(32, 1, 512, 24, 0) A(64, 0, 512, 20, 0) A(64, 0, 512, 24, 0)
    A(64, 1, 512, 16, 0) A(32, 1, 1024, 12, 0) A(64, 0, 1024, 12, 0)
    A(32, 1, 512, 32, 0) A(64, 0, 512, 32, 0) A(64, 1, 512, 24, 0) A(32, 1, 1024, 16, 0)
    A(64, 0, 1024, 16, 0) A(32, 0, 1024, 32, 0) A(32, 0, 512, 64, 0) A(32, 0, 512, 48, 0)
    A(32, 0, 1024, 24, 0) A(32, 1, 512, 36, 0) A(64, 0, 512, 36, 0)
    A(32, 0, 512, 24, 8192) A(32, 0, 512, 16, 8192) A(32, 0, 1024, 16, 8192)
    A(32, 0, 512, 24, 8) A(32, 0, 512, 16, 8) A(32, 0, 1024, 16, 8)
    A(32, 0, 512, 24, 16) A(32, 0, 1024, 16, 16)
    A(32, 0, 512, 24, 48) A(32, 0, 512, 24, 64) A(32, 0, 512, 24, 72) A(32, 0, 512, 24, 80)
    A(32, 0, 512, 16, 64) A(32, 0, 1024, 16, 64) A(32, 0, 512, 20, 64) A(32, 0, 512, 24, 32) A(32, 0, 512, 24, 40) A(32, 0, 1024, 16, 32) A(32, 0, 512, 16, 32) A(32, 0, 512, 16, 40)
#endif
#undef A
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ar2 (one-wave vectorised two-level look-back), one tile per workgroup
int lab_ar2(int kb, int pairs, int block, int items, int dbg, const void* in, void* out,
            const uint32_t* vin, uint32_t* vout, uint32_t n, const uint32_t* hist, uint32_t* ticket,
            uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long code = ((((long)kb * 2 + pairs) * 10000 + block) * 100 + items) * 100 + dbg;
  switch (code) {
#define A(KB, P, B, I, D)                                                                     \
  case ((((long)KB * 2 + P) * 10000 + B) * 100 + I) * 100 + D: {                                \
    using KT = std::conditional_t<KB == 32, uint32_t, uint64_t>;                              \
    const uint32_t tiles = (n + B * I - 1) / (B * I);                                         \
    hipLaunchKernelGGL((grs::grs_onesweep_ar2<KT, P != 0, 8, B, I, D>), dim3(tiles), dim3(B),  \
                       0, s, (const KT*)in, (KT*)out, vin, vout, n,                           \
                       grs::RadixDigit<KT>{shift, 255u}, hist, ticket, st, st2, err);         \
  } break;
#ifdef LAB_MIN
    A(32, 0, 512, 24, 0)
#else
    A(32, 0, 512, 24, 0) A(32, 0, 512, 16, 0) A(32, 0, 512, 20, 0) A(32, 0, 1024, 16, 0)
    A(32, 0, 512, 24, 8) A(32, 0, 512, 16, 8) A(32, 0, 256, 24, 0) A(32, 0, 256, 32, 0)
    A(32, 1, 512, 16, 0) A(32, 1, 512, 12, 0) A(64, 0, 512, 16, 0) A(64, 0, 512, 12, 0)
    A(64, 1, 512, 8, 0) A(64, 1, 512, 12, 0)
#endif
#undef A
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// v3 (library default pass): persistent grid of `grid` workgroups (0 = one per tile)
int lab_v3(int kb, int pairs, int block, int items, int dbg, int grid, const void* in, void* out,
           const uint32_t* vin, uint32_t* vout, uint32_t n, const uint32_t* hist, uint32_t* ticket,
           uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long code = ((((long)kb * 2 + pairs) * 10000 + block) * 100 + items) * 100 + dbg;
  switch (code) {
#define C3(KB, P, B, I, D)                                                                    \
  case ((((long)KB * 2 + P) * 10000 + B) * 100 + I) * 100 + D: {                               \
    using KT = std::conditional_t<KB == 32, uint32_t, uint64_t>;                             \
    const uint32_t tiles = (n + B * I - 1) / (B * I);                                        \
    const uint32_t g = grid > 0 ? std::min<uint32_t>(grid, tiles) : tiles;                   \
    hipLaunchKernelGGL((grs::grs_onesweep_v3<KT, P != 0, 8, B, I, D>), dim3(g), dim3(B), 0, s, \
                       (const KT*)in, (KT*)out, vin, vout, n, grs::RadixDigit<KT>{shift, 255u}, \
                       hist, ticket, st, st2, err);                                          \
  } break;
    C3(32, 0, 512, 16, 0) C3(32, 0, 512, 16, 16) C3(32, 0, 512, 12, 0) C3(32, 0, 512, 16, 32)
    C3(32, 0, 512, 16, 48) C3(32, 0, 1024, 16, 32) C3(32, 0, 1024, 16, 8) C3(32, 0, 512, 16, 8)
    C3(32, 0, 1024, 16, 64) C3(32, 0, 512, 16, 64) C3(32, 0, 1024, 16, 72)
    C3(32, 0, 1024, 16, 0) C3(32, 0, 1024, 16, 16) C3(32, 0, 1024, 16, 1) C3(32, 0, 1024, 16, 2)
    C3(32, 0, 1024, 16, 3) C3(32, 0, 1024, 16, 9) C3(32, 0, 1024, 16, 128)
    C3(32, 0, 1024, 16, 256) C3(32, 0, 1024, 16, 384) C3(32, 0, 1024, 16, 130)
    C3(32, 0, 1024, 16, 65) C3(32, 0, 1024, 16, 577) C3(32, 0, 1024, 16, 705) C3(32, 0, 1024, 16, 193) C3(32, 0, 1024, 12, 0) C3(32, 0, 512, 8, 0)
    C3(32, 1, 512, 8, 0) C3(32, 1, 1024, 8, 0) C3(64, 0, 512, 8, 0) C3(64, 0, 1024, 8, 0)
    C3(64, 1, 512, 4, 0) C3(64, 1, 1024, 4, 0)
#undef C3
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab_hist(int kb, const void* in, uint32_t n, uint32_t* hist, uint32_t* clear, uint32_t cw,
             void* stream) {
  if (kb == 32)
    hipLaunchKernelGGL((grs::grs_upfront_hist<uint32_t, 8>), dim3(2048), dim3(GRS_HIST_BLOCK), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint32_t*>(in), n, 0,
                       32, 4, hist, clear, cw);
  else
    hipLaunchKernelGGL((grs::grs_upfront_hist<uint64_t, 8>), dim3(2048), dim3(GRS_HIST_BLOCK), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint64_t*>(in), n, 0,
                       64, 8, hist, clear, cw);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab_copy(const uint32_t* in, uint32_t* out, uint32_t n, void* stream) {
  hipLaunchKernelGGL(copy_x4, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
