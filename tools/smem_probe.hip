// Does a scalar (SMEM) load with glc observe a store another XCD made?  (Round-3 verdict item
// 1 suggested polling the look-back words on the scalar unit, whose loads count in lgkmcnt and
// would not queue behind a prefetch.)  Block 0 stores flag = 1 (relaxed agent-scope atomic
// store, as the pass publishes its status words) about 20 us after it starts; every other block
// polls the flag and records how many polls and how long it took to see it, and on which XCC.
//   mode 0: scalar loads with glc
//   mode 1: a plain scalar load of the flag first (the line in the scalar cache, stale-to-be),
//           then scalar loads with glc
//   mode 2: vector loads (relaxed agent-scope atomic load, the pass's ld_status), for reference
//   mode 3: a 64-word row through scalar x16 loads into the lanes (smem_row_lane)
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

// One wave row of 64 status words into the lanes (lane l gets row[l]): 4 scalar x16 loads with
// glc and 64 v_writelane -- what a scalar look-back re-poll would cost per row.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ u32x16 smem_x16_glc(const uint32_t* p) {
  u32x16 v;
  asm volatile("s_load_dwordx16 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t smem_row_lane(const uint32_t* row) {
  u32x16 v[4];
  // all four loads in flight under one wait
  asm volatile(
      "s_load_dwordx16 %0, %4, 0x0 glc\n\t"
      "s_load_dwordx16 %1, %4, 0x40 glc\n\t"
      "s_load_dwordx16 %2, %4, 0x80 glc\n\t"
      "s_load_dwordx16 %3, %4, 0xc0 glc\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=s"(v[0]), "=s"(v[1]), "=s"(v[2]), "=s"(v[3]) : "s"(row) : "memory");
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(out) : "s"(v[q][i]), "i"(16 * q + i));
  return out;
}

// mode 3: block 0's wave 0 stores a row of 64 words (word l = l + 1) at ~20 us; the readers
// poll the row with smem_row_lane until every lane holds its own word
__global__ void smem_probe_row(uint32_t* row, uint32_t* out, uint32_t max_polls) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint32_t lane = threadIdx.x & 63;
  if (blockIdx.x == 0) {
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x < 64) __hip_atomic_store(row + lane, lane + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) out[0] = xcc;
    return;
  }
  if (threadIdx.x >= 64) return;
  uint32_t polls = 0, ok = 0;
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (; polls < max_polls; ++polls) {
    const uint32_t v = smem_row_lane(row);
    if (__builtin_amdgcn_ballot_w64(v != lane + 1) == 0) {
      ok = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    uint32_t* o = out + 4 * blockIdx.x;
    o[0] = xcc;
    o[1] = ok;
    o[2] = polls;
    o[3] = static_cast<uint32_t>(t1 - t0);
    out[4 * 64 + blockIdx.x] = static_cast<uint32_t>((c1 - c0) / (polls + 1));   // cycles per poll
  }
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
  if (hipMemset(flag, 0, 256) != hipSuccess) return -1;
  if (mode == 3)
    hipLaunchKernelGGL(smem_probe_row, dim3(blocks), dim3(64), 0, 0, flag, out, max_polls);
  else
    hipLaunchKernelGGL(smem_probe, dim3(blocks), dim3(64), 0, 0, flag, out, mode, max_polls);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
