// Does a scalar (SMEM) load with glc observe a store another XCD made?  (Round-3 verdict item
// 1 suggested polling the look-back words on the scalar unit, whose loads count in lgkmcnt and
// would not queue behind a prefetch.)  Block 0 stores flag = 1 (relaxed agent-scope atomic
// store, as the pass publishes its status words) about 20 us after it starts; every other block
// polls the flag and records how many polls and how long it took to see it, and on which XCC.
//   mode 0: scalar loads with glc
//   mode 1: a plain scalar load of the flag first (the line in the scalar cache, stale-to-be),
//           then scalar loads with glc
//   mode 2: vector loads (relaxed agent-scope atomic load, the pass's ld_status), for reference
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ uint32_t smem_glc(const uint32_t* p) {
  uint32_t v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t smem_plain(const uint32_t* p) {
  uint32_t v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}

__global__ void smem_probe(uint32_t* flag, uint32_t* out, int mode, uint32_t max_polls) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) {
      while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(8);   // 20 us
      __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      out[0] = xcc;
    }
    return;
  }
  if (threadIdx.x != 0) return;
  uint32_t polls = 0, v = 0;
  if (mode == 1) v = smem_plain(flag);
  for (; polls < max_polls; ++polls) {
    v = mode == 2 ? __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : smem_glc(flag);
    if (v == 1u) break;
    __builtin_amdgcn_s_sleep(1);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  uint32_t* o = out + 4 * blockIdx.x;
  o[0] = xcc;
  o[1] = v;
  o[2] = polls;
  o[3] = static_cast<uint32_t>(t1 - t0);   // 100 MHz ticks
}

extern "C" int smem_probe_run(uint32_t* flag, uint32_t* out, int mode, int blocks,
                              uint32_t max_polls) {
  if (hipMemset(flag, 0, 4) != hipSuccess) return -1;
  hipLaunchKernelGGL(smem_probe, dim3(blocks), dim3(64), 0, 0, flag, out, mode, max_polls);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
