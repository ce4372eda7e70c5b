// lab.hip — kernel laboratory (not part of libgrs): timing ablations of one onesweep pass.
// Built by tools/Makefile into tools/liblab.so; driven by tools/lab.py on the GPU box.
#include <hip/hip_runtime.h>

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

namespace {

__global__ void copy_dword(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = in[i];
}

__global__ void copy_x4(const uint4* __restrict__ in, uint4* __restrict__ out, uint32_t n4) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
    out[i] = in[i];
}

int g_persist_grid = 0;

template <int BLOCK, int ITEMS, int DBG>
void launch(const uint32_t* in, uint32_t* out, uint32_t n, const uint32_t* hist, uint32_t* ticket,
            uint32_t* st, uint32_t* st2, uint32_t* err, int shift, hipStream_t s) {
  constexpr int TILE = BLOCK * ITEMS;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  if (g_persist_grid > 0)
    hipLaunchKernelGGL((grs::grs_onesweep_persistent<uint32_t, false, 8, BLOCK, ITEMS, DBG>),
                       dim3(g_persist_grid), dim3(BLOCK), 0, s, in, out, nullptr, nullptr, n,
                       grs::RadixDigit<uint32_t>{shift, 255u}, hist, ticket, st, st2, err);
  else
    hipLaunchKernelGGL((grs::grs_onesweep_pass<uint32_t, false, 8, BLOCK, ITEMS, DBG>), dim3(tiles),
                       dim3(BLOCK), 0, s, in, out, nullptr, nullptr, n,
                       grs::RadixDigit<uint32_t>{shift, 255u}, hist, ticket, st, st2, err);
}

}  // namespace

extern "C" {

// variant = BLOCK * 10000 + ITEMS * 16 + DBG
void lab_set_persistent(int grid) { g_persist_grid = grid; }

int lab_pass(int variant, const uint32_t* in, uint32_t* out, uint32_t n, const uint32_t* hist,
             uint32_t* ticket, uint32_t* st, uint32_t* st2, uint32_t* err, int shift, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (variant) {
#define V(B, I, D) \
  case B * 10000 + I * 16 + D: launch<B, I, D>(in, out, n, hist, ticket, st, st2, err, shift, s); break;
    V(256, 8, 0) V(256, 16, 0) V(256, 16, 1) V(256, 16, 2) V(256, 16, 3) V(256, 16, 4) V(256, 16, 7)
    V(256, 24, 0) V(256, 32, 0) V(256, 32, 1) V(256, 32, 2) V(256, 32, 3) V(256, 32, 4)
    V(512, 8, 0) V(512, 12, 0) V(512, 16, 0) V(512, 16, 1) V(512, 16, 3) V(512, 16, 4)
    V(1024, 8, 0) V(1024, 16, 0)
#undef V
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab_hist(const uint32_t* in, uint32_t n, uint32_t* hist, uint32_t* clear, uint32_t cw, void* stream) {
  hipLaunchKernelGGL((grs::grs_upfront_hist<uint32_t, 8>), dim3(2048), dim3(GRS_HIST_BLOCK), 0,
                     static_cast<hipStream_t>(stream), in, n, 0, 32, 4, hist, clear, cw);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab_copy(int wide, const uint32_t* in, uint32_t* out, uint32_t n, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (wide)
    hipLaunchKernelGGL(copy_x4, dim3(4096), dim3(256), 0, s, reinterpret_cast<const uint4*>(in),
                       reinterpret_cast<uint4*>(out), n / 4);
  else
    hipLaunchKernelGGL(copy_dword, dim3(4096), dim3(256), 0, s, in, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
