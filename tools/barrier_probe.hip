// Lab probe (round 5): what a grid barrier costs between the passes of one persistent launch
// (grs_onesweep_fused) against a kernel boundary.  256 x 1024-thread workgroups, one per CU;
// each round every workgroup stores `words` u32 (a pass's writes), then the barrier.
//   mode 0: arrival counter only (no fences: the sync cost alone, NOT a correct barrier)
//   mode 1: every workgroup: release add (buffer_wbl2) + acquire fence (buffer_inv)
//   mode 2: every workgroup: acquire fence only; the LAST arriver of each XCD writes its L2
//           back (one buffer_wbl2 per XCD) before the global arrival
//   mode 3: every workgroup: release add only
// Separate launches of the store kernel give the kernel-boundary cost (barrier_probe.py).
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 15u;
}

__device__ __forceinline__ void stores(uint32_t* out, uint32_t words, uint32_t round) {
  uint32_t* o = out + static_cast<size_t>(blockIdx.x) * words;
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) o[i] = i + round;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ctl: [0] global arrivals, [8 + x] arrivals of XCD x, [32 + x] workgroups of XCD x, [48] XCDs
__global__ __launch_bounds__(1024) void probe_fused(uint32_t* out, uint32_t words, int rounds, int mode,
                                                    uint32_t* ctl, uint32_t* err) {
  const uint32_t x = xcc_id();
  const uint32_t G = gridDim.x;
  if (threadIdx.x == 0) {
    if (atomicAdd(&ctl[32 + x], 1u) == 0u) atomicAdd(&ctl[48], 1u);
    atomicAdd(&ctl[1], 1u);
    while (ld_relaxed(&ctl[1]) < G) __builtin_amdgcn_s_sleep(2);
  }
  __syncthreads();
  for (int r = 0; r < rounds; ++r) {
    stores(out, words, r);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t target = static_cast<uint32_t>(r + 1) * G;
      if (mode == 1 || mode == 3) {
        __hip_atomic_fetch_add(&ctl[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else if (mode == 2) {
        const uint32_t nx = ld_relaxed(&ctl[32 + x]);
        const uint32_t a = atomicAdd(&ctl[8 + x], 1u) + 1u;
        target = static_cast<uint32_t>(r + 1) * ld_relaxed(&ctl[48]);
        if (a == static_cast<uint32_t>(r + 1) * nx) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          atomicAdd(&ctl[0], 1u);
        }
      } else {
        atomicAdd(&ctl[0], 1u);
      }
      uint32_t spins = 0;
      while (ld_relaxed(&ctl[0]) < target) {
        if (++spins > (1u << 22)) {
          atomicOr(err, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (mode == 1 || mode == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void probe_store(uint32_t* out, uint32_t words, int round) {
  stores(out, words, static_cast<uint32_t>(round));
}

}  // namespace

extern "C" int barrier_probe_fused(uint32_t* out, uint32_t words, int rounds, int mode, uint32_t* ctl,
                                   uint32_t* err, int grid, void* stream) {
  hipLaunchKernelGGL(probe_fused, dim3(grid), dim3(1024), 0, static_cast<hipStream_t>(stream), out, words,
                     rounds, mode, ctl, err);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int barrier_probe_launches(uint32_t* out, uint32_t words, int rounds, int grid, void* stream) {
  for (int r = 0; r < rounds; ++r)
    hipLaunchKernelGGL(probe_store, dim3(grid), dim3(1024), 0, static_cast<hipStream_t>(stream), out, words, r);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
