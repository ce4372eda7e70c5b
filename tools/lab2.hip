// lab2.hip — kernel laboratory (not part of libgrs): memory-pattern replays and emulations of
// the pass, LDS-atomic rates, streaming-copy ceilings, the one-pass scan.  The pass kernel
// itself is timed from the shipped source (tools/lab4.hip includes grs_pass.hpp: lab2.py's "p4"
// variants).  The round 2-4 fork of the pass with its rejected variants (tools/lab_pass.hpp)
// was removed in round 5; `git show 729d494:tools/lab_pass.hpp` has it.
// Built by tools/Makefile into tools/liblab2.so; driven by tools/lab2.py on the GPU box.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../gpuradixsort_amd/csrc/grs_kernels.hpp"

namespace grs_lab {
// XCC id of the calling wave: HW_REG_XCC_ID (hwreg 20 on gfx940+), bits [3:0]
__device__ __forceinline__ uint32_t xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & (GRS_XCDS - 1);
}
// Per-XCD ticket heads (round 4's rejected schedule, kept for the replay's X8 mode): tile ids
// 8 j + c are handed out by counter c in increasing j; a workgroup draws from its own XCD's
// counter and, once that is exhausted, from the others in turn.
__device__ __forceinline__ uint32_t draw_ticket_x8(uint32_t* ticket, uint32_t tiles) {
  const uint32_t x = xcc_id();
  for (uint32_t k = 0; k < GRS_XCDS; ++k) {
    const uint32_t c = (x + k) & (GRS_XCDS - 1);
    if (c >= tiles) continue;
    const uint32_t cnt = (tiles - c + GRS_XCDS - 1) / GRS_XCDS;   // tiles with id = c mod 8
    const uint32_t v = atomicAdd(ticket + c, 1u);
    if (v < cnt) return v * GRS_XCDS + c;
  }
  return 0xFFFFFFFFu;   // every tile drawn
}
}  // namespace grs_lab


namespace {

// Streaming copy: U independent 16-B loads in flight per thread, then U stores.
template <int U>
__global__ __launch_bounds__(256) void copy_u(const uint4* __restrict__ in, uint4* __restrict__ out,
                                              uint32_t n4) {
  const uint32_t stride = gridDim.x * 256;
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = in[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) out[i + u * stride] = x[u];
  }
  for (; i < n4; i += stride) out[i] = in[i];
}

// Read-only stream (HBM read ceiling).
template <int U>
__global__ __launch_bounds__(256) void read_u(const uint4* __restrict__ in, uint32_t* __restrict__ sink,
                                              uint32_t n4) {
  const uint32_t stride = gridDim.x * 256;
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = in[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Memory pattern of one pass without its compute: tile T = blockIdx.x is loaded wave-striped
// into registers and stored by tile position i = k*BLOCK + t to
//   MODE 0: T*TILE + i (contiguous), MODE 1: 256 equal digit runs of RUN = TILE/256 keys:
//   dst = (i / RUN) * (n / 256) + T * RUN + i % RUN (the uniform-key scatter of a pass);
//   MODE 2: as 1, with consecutive tiles on one XCD (block b -> tile (b%8)*tiles/8 + b/8)
//   MODE 3: as 1, every destination shifted by one key (run boundaries 4 B past a 64-B line:
//   the unaligned boundaries of real digit runs); MODE 5: as 3 with MODE 2's tile mapping
// POL (store policy): 0 default, 1 nontemporal, 2 agent-scope (sc1, write-through),
// 3 nontemporal for lines inside a run and default for the run's partial head / tail lines
// MODE 8: the runs of MODE 3 (every destination one key past alignment), but stored
// destination-aligned: wave w writes runs w, w + WAVES, ...; a run starting at D is cut into
// 64-key chunks at (D & ~63) + 64 k, lane l writing key A + l of its chunk when inside the run
// (every wave-instruction writes one aligned 256-B window of one run).  POL 3: nontemporal
// for lines wholly inside the run, default for its head / tail lines.
template <int BLOCK, int ITEMS, int POL>
__global__ __launch_bounds__(BLOCK) void scatter_emu_aligned(const uint32_t* __restrict__ in,
                                                             uint32_t* __restrict__ out,
                                                             uint32_t n) {
  constexpr uint32_t TILE = BLOCK * ITEMS, RUN = TILE / 256, WAVES = BLOCK / 64;
  extern __shared__ uint32_t pad_lds[];
  const uint32_t T = blockIdx.x;
  if ((T + 1) * TILE > n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t key[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) key[j] = in[T * TILE + w * 64 * ITEMS + j * 64 + lane];
  if (n == 0) pad_lds[threadIdx.x] = key[0];
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) acc ^= key[j];
  for (uint32_t r = w; r < 256; r += WAVES) {
    const uint32_t rs = r * (n / 256) + T * RUN + 1, re = rs + RUN;   // run [rs, re)
    for (uint32_t A = rs & ~63u; A < re; A += 64) {
      const uint32_t dst = A + lane;
      if (dst >= rs && dst < re && dst < n) {
        const uint32_t v = acc + dst;
        const uint32_t ls = dst & ~31u;
        if (POL == 3 && ls >= rs && ls + 32 <= re) __builtin_nontemporal_store(v, &out[dst]);
        else out[dst] = v;
      }
    }
  }
}

template <int BLOCK, int ITEMS, int MODE, int POL = 0>
__global__ __launch_bounds__(BLOCK) void scatter_emu(const uint32_t* __restrict__ in,
                                                     uint32_t* __restrict__ out, uint32_t n) {
  constexpr uint32_t TILE = BLOCK * ITEMS, RUN = TILE / 256;
  extern __shared__ uint32_t pad_lds[];
  const uint32_t tiles8 = (n / TILE) / 8 * 8;
  constexpr bool XL = MODE == 2 || MODE == 5 || MODE == 6;
  const uint32_t T = MODE == 6 ? ((blockIdx.x / 8) / 32 * 8 + blockIdx.x % 8) * 32 + (blockIdx.x / 8) % 32
                   : XL ? (blockIdx.x % 8) * (tiles8 / 8) + blockIdx.x / 8 : blockIdx.x;
  if (XL && blockIdx.x >= tiles8) return;
  if ((T + 1) * TILE > n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t key[ITEMS];
  if constexpr (MODE == 7) {   // gather: read the 256 runs of a pass's digit-major layout
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = j * BLOCK + threadIdx.x;
      key[j] = in[(i / RUN) * (n / 256) + T * RUN + i % RUN];
    }
  } else {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) key[j] = in[T * TILE + w * 64 * ITEMS + j * 64 + lane];
  }
  if (n == 0) pad_lds[threadIdx.x] = key[0];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + threadIdx.x;
    uint32_t dst = (MODE == 0 || MODE == 7) ? T * TILE + i : (i / RUN) * (n / 256) + T * RUN + i % RUN;
    if (MODE >= 3) dst = dst + 1 == n ? 0u : dst + 1;
    if constexpr (POL == 0) {
      out[dst] = key[k];
    } else if constexpr (POL == 1) {
      __builtin_nontemporal_store(key[k], &out[dst]);
    } else if constexpr (POL == 2) {
      __hip_atomic_store(&out[dst], key[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t rs = dst - i % RUN, re = rs + RUN;   // run [rs, re)
      const uint32_t ls = dst & ~31u;                     // 128-B line of dst
      if (ls >= rs && ls + 32 <= re) __builtin_nontemporal_store(key[k], &out[dst]);
      else out[dst] = key[k];
    }
  }
}

// Key + payload pass memory pattern (BASELINE C3) without compute: 256 equal digit runs per
// tile, stored as two u32 arrays (AOS = 0, the library's SoA) or as one array of 8-byte
// (key, value) records (AOS = 1): the same bytes, runs twice as long.
template <int BLOCK, int ITEMS, int AOS>
__global__ __launch_bounds__(BLOCK) void scatter_emu_pairs(const uint32_t* __restrict__ kin,
                                                           const uint32_t* __restrict__ vin,
                                                           uint32_t* __restrict__ kout,
                                                           uint32_t* __restrict__ vout, uint32_t n) {
  constexpr uint32_t TILE = BLOCK * ITEMS, RUN = TILE / 256;
  extern __shared__ uint32_t pad_lds[];
  const uint32_t T = blockIdx.x;
  if ((T + 1) * TILE > n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t k[ITEMS], v[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t src = T * TILE + w * 64 * ITEMS + j * 64 + lane;
    if constexpr (AOS) {
      const uint2 x = reinterpret_cast<const uint2*>(kin)[src];
      k[j] = x.x;
      v[j] = x.y;
    } else {
      k[j] = kin[src];
      v[j] = vin[src];
    }
  }
  if (n == 0) pad_lds[threadIdx.x] = k[0] + v[0];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = j * BLOCK + threadIdx.x;
    const uint32_t dst = (i / RUN) * (n / 256) + T * RUN + i % RUN;
    if constexpr (AOS) {
      reinterpret_cast<uint2*>(kout)[dst] = make_uint2(k[j], v[j]);
    } else {
      kout[dst] = k[j];
      vout[dst] = v[j];
    }
  }
}

// MODE 3's runs (every run boundary 4 B past a 128-B line; tiles T and T + 1 = blocks b, b + 1
// on different XCDs) with the boundary lines HANDED OFF instead of written twice partially:
// tile T writes the tail of each run, [floor32(E), E), into one whole 128-B slot line of a ring
// (sc1 stores), publishes a flag (vmcnt(0), barrier, sc1 flag store), stores the rest of its
// runs, then waits for tile T - 1's flag and writes the head of each of its runs,
// [floor32(D), D), from T - 1's slot line: every boundary line reaches memory once, whole,
// from one CU.  VAR 0: as described; 1: no flag wait (timing of the traffic alone, wrong
// data); 2: the slot lines are written by plain stores (no sc1) and no flag (traffic, wrong).
// C2's memory pattern: the pass's loads and stores at 4-bit digits (16 runs per tile, every run
// one key past alignment), no compute; lab2.py runs it 8 times back to back (the 8 passes of a
// 2^24-key sort, ping-pong, MALL-resident) for the floor of the C2 passes.
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void scatter_emu16(const uint32_t* __restrict__ in,
                                                       uint32_t* __restrict__ out, uint32_t n) {
  constexpr uint32_t TILE = BLOCK * ITEMS, RUN = TILE / 16;
  const uint32_t T = blockIdx.x;
  if ((T + 1) * TILE > n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t key[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) key[j] = in[T * TILE + w * 64 * ITEMS + j * 64 + lane];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + threadIdx.x;
    uint32_t dst = (i / RUN) * (n / 16) + T * RUN + i % RUN + 1;
    out[dst >= n ? 0u : dst] = key[k];
  }
}

constexpr uint32_t kEmuRing = 2048;
template <int BLOCK, int ITEMS, int VAR>
__global__ __launch_bounds__(BLOCK) void scatter_emu_handoff(const uint32_t* __restrict__ in,
                                                             uint32_t* __restrict__ out, uint32_t n,
                                                             uint32_t* __restrict__ ring,
                                                             uint32_t* __restrict__ flags,
                                                             uint32_t epoch, uint32_t* err) {
  constexpr uint32_t TILE = BLOCK * ITEMS, RUN = TILE / 256, WAVES = BLOCK / 64;
  extern __shared__ uint32_t pad_lds[];
  const uint32_t T = blockIdx.x;
  const uint32_t tiles = n / TILE;
  if (T >= tiles) return;
  const uint32_t region = n / 256;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t key[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) key[j] = in[T * TILE + w * 64 * ITEMS + j * 64 + lane];
  if (n == 0) pad_lds[threadIdx.x] = key[0];
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) acc ^= key[j];
  // run r of tile T: [D, E) with D = r * region + T * RUN + 1
  const bool defer_tail = T + 1 < tiles;   // every E is 4 B past a line here (RUN % 32 = 16)
  const bool take_head = T > 0;
  // (1) slot lines: two runs per wave-instruction (lanes 0-31: run r, 32-63: run r + 1)
  uint32_t* slot = ring + static_cast<size_t>(T % kEmuRing) * 256 * 32;
  if (defer_tail) {
    for (uint32_t r = w * 2 + (lane >> 5); r < 256; r += 2 * WAVES) {
      const uint32_t E = r * region + T * RUN + 1 + RUN;
      const uint32_t j = lane & 31;
      const uint32_t v = acc + (E & ~31u) + j;
      if (VAR == 2) slot[r * 32 + j] = v;
      else __hip_atomic_store(&slot[r * 32 + j], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (VAR == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        __hip_atomic_store(&flags[T % kEmuRing], epoch * 65536u + T, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // (2) the runs, minus the deferred tails
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + threadIdx.x;
    const uint32_t r = i / RUN;
    const uint32_t dst = r * region + T * RUN + i % RUN + 1;
    const uint32_t E = r * region + T * RUN + 1 + RUN;
    if (!(defer_tail && dst >= (E & ~31u))) out[dst] = key[k];
  }
  // (3) the heads from T - 1's slot lines
  if (take_head) {
    const uint32_t* ps = ring + static_cast<size_t>((T - 1) % kEmuRing) * 256 * 32;
    if (VAR == 0) {
      if (threadIdx.x == 0) {
        const uint32_t want = epoch * 65536u + (T - 1);
        uint32_t spins = 0;
        while (__hip_atomic_load(&flags[(T - 1) % kEmuRing], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) != want) {
          if (++spins > (1u << 20)) {
            atomicOr(err, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
    }
    for (uint32_t r = w * 2 + (lane >> 5); r < 256; r += 2 * WAVES) {
      const uint32_t D = r * region + T * RUN + 1;
      const uint32_t j = lane & 31;
      if (j < (D & 31u)) {
        const uint32_t v = VAR == 2 ? ps[r * 32 + j]
                                    : __hip_atomic_load(&ps[r * 32 + j], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        out[(D & ~31u) + j] = v;
      }
    }
  }
}

}  // namespace


// LDS returning-atomic throughput by same-address multiplicity: each wave does ITER returning
// ds_add_u32 on counter (lane % DISTINCT) of its own 256-word region (+ a per-iteration rotation
// so that consecutive instructions hit different words); cycles per wave-instruction from
// s_memtime.  DISTINCT = 64: no two lanes share an address; 16: 4 lanes per address; 1: all.
template <int DISTINCT>
__global__ __launch_bounds__(1024) void lds_atomic_rate(uint32_t* out, int iters) {
  __shared__ uint32_t c[16 * 256];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (uint32_t i = t; i < 16 * 256; i += 1024) c[i] = 0;
  __syncthreads();
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const uint32_t a = w * 256 + ((lane % DISTINCT) * 4 + it) % 256;
    acc += atomicAdd(&c[a], 1u);
  }
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (t == 0) out[blockIdx.x] = static_cast<uint32_t>(t1 - t0);
  if (acc == 0xFFFFFFFFu) out[1023] = acc;
}

// XCC id of every block (placement check of draw_ticket_xr's counter choice)
__global__ void xcc_probe(uint32_t* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = grs_lab::xcc_id();
}


// Replay of a pass's memory traffic (round 4): the input is PRE-REORDERED (each tile's keys
// already stably grouped by digit, as the real pass holds them in LDS after its reorder) and
// table[tile][d] = global destination of tile position 0 of digit d (the real pass's base[]).
// A workgroup takes a ticket, loads its tile (ITEMS keys per thread, positions k*BLOCK + t)
// and stores key i to table[d] + i: exactly the real pass's load lines and store addresses,
// in its store order, without the ranking, reorder or look-back.  Its time is the floor of
// that access pattern.
template <int BLOCK, int ITEMS, int RB, bool X8>
__global__ __launch_bounds__(BLOCK) void replay_pass(const uint32_t* __restrict__ pre,
                                                     uint32_t* __restrict__ out,
                                                     const uint32_t* __restrict__ table, uint32_t n,
                                                     int shift, uint32_t* __restrict__ ticket) {
  constexpr int R = 1 << RB;
  constexpr uint32_t TILE = BLOCK * ITEMS;
  __shared__ uint32_t tb[R];
  __shared__ uint32_t tk;
  if (threadIdx.x == 0)
    tk = X8 ? grs_lab::draw_ticket_x8(ticket, (n + TILE - 1) / TILE) : atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tile = tk;
  for (uint32_t i = threadIdx.x; i < static_cast<uint32_t>(R); i += BLOCK)
    tb[i] = table[static_cast<size_t>(tile) * R + i];
  const uint32_t base = tile * TILE;
  const uint32_t valid = min(TILE, n - base);
  uint32_t key[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + threadIdx.x;
    key[k] = i < valid ? pre[base + i] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const uint32_t i = k * BLOCK + threadIdx.x;
    if (i < valid) out[tb[(key[k] >> shift) & (R - 1)] + i] = key[k];
  }
}

extern "C" {

int lab2_xcc(uint32_t* out, int blocks, void* stream) {
  hipLaunchKernelGGL(xcc_probe, dim3(blocks), dim3(64), 0, static_cast<hipStream_t>(stream), out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// pass memory-pattern emulation: block, items, mode, dynamic LDS bytes (occupancy control)
int lab2_emu(int block, int items, int mode, int lds, const void* in, void* out, uint32_t n,
             void* stream) {
  // mode = layout (0 contiguous, 1 runs, 2 runs + XCD-local tiles) + 10 * store policy
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t tiles = n / (block * items);
  const uint32_t* i = static_cast<const uint32_t*>(in);
  uint32_t* o = static_cast<uint32_t*>(out);
  const void* k = nullptr;
  const int code = block * 100000 + items * 100 + mode;
  switch (code) {
    case 51207200: k = (const void*)scatter_emu<512, 72, 0>; break;
    case 51207201: k = (const void*)scatter_emu<512, 72, 1>; break;
    case 51207202: k = (const void*)scatter_emu<512, 72, 2>; break;
    case 51207211: k = (const void*)scatter_emu<512, 72, 1, 1>; break;
    case 51207221: k = (const void*)scatter_emu<512, 72, 1, 2>; break;
    case 51207231: k = (const void*)scatter_emu<512, 72, 1, 3>; break;
    case 51206401: k = (const void*)scatter_emu<512, 64, 1>; break;
    case 51206411: k = (const void*)scatter_emu<512, 64, 1, 1>; break;
    case 51206421: k = (const void*)scatter_emu<512, 64, 1, 2>; break;
    case 51206601: k = (const void*)scatter_emu<512, 66, 1>; break;
    case 51206611: k = (const void*)scatter_emu<512, 66, 1, 1>; break;
    case 51206621: k = (const void*)scatter_emu<512, 66, 1, 2>; break;
    case 51206631: k = (const void*)scatter_emu<512, 66, 1, 3>; break;
    case 102403600: k = (const void*)scatter_emu<1024, 36, 0>; break;
    case 102403607: k = (const void*)scatter_emu<1024, 36, 7>; break;
    case 102403601: k = (const void*)scatter_emu<1024, 36, 1>; break;
    case 102403621: k = (const void*)scatter_emu<1024, 36, 1, 2>; break;
    case 102403611: k = (const void*)scatter_emu<1024, 36, 1, 1>; break;
    case 102403613: k = (const void*)scatter_emu<1024, 36, 3, 1>; break;
    case 102403623: k = (const void*)scatter_emu<1024, 36, 3, 2>; break;
    case 102404800: k = (const void*)scatter_emu<1024, 48, 0>; break;
    case 102407200: k = (const void*)scatter_emu<1024, 72, 0>; break;
    case 102403631: k = (const void*)scatter_emu<1024, 36, 1, 3>; break;
    case 102403603: k = (const void*)scatter_emu<1024, 36, 3>; break;
    case 102403605: k = (const void*)scatter_emu<1024, 36, 5>; break;
    case 102403602: k = (const void*)scatter_emu<1024, 36, 2>; break;
    case 102403606: k = (const void*)scatter_emu<1024, 36, 6>; break;
    case 102404801: k = (const void*)scatter_emu<1024, 48, 1>; break;
    case 102404803: k = (const void*)scatter_emu<1024, 48, 3>; break;
    case 102404805: k = (const void*)scatter_emu<1024, 48, 5>; break;
    case 102407201: k = (const void*)scatter_emu<1024, 72, 1>; break;
    case 102407203: k = (const void*)scatter_emu<1024, 72, 3>; break;
    case 102407205: k = (const void*)scatter_emu<1024, 72, 5>; break;
    case 102403608: k = (const void*)scatter_emu_aligned<1024, 36, 0>; break;
    case 102403638: k = (const void*)scatter_emu_aligned<1024, 36, 3>; break;
    case 102404808: k = (const void*)scatter_emu_aligned<1024, 48, 0>; break;
    case 102404838: k = (const void*)scatter_emu_aligned<1024, 48, 3>; break;
    default: return -1;
  }
  void* args[] = {&i, &o, &n};
  if (hipLaunchKernel(k, dim3(tiles), dim3(block), args, lds, s) != hipSuccess) return -2;
  return 0;
}

// C2 memory-pattern emulation: `passes` launches of scatter_emu16, ping-pong between a and b
int lab2_emu16(int block, int items, int passes, void* a, void* b, uint32_t n, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t tiles = n / (block * items);
  for (int p = 0; p < passes; ++p) {
    const uint32_t* i = static_cast<const uint32_t*>(p & 1 ? b : a);
    uint32_t* o = static_cast<uint32_t*>(p & 1 ? a : b);
    if (block == 1024 && items == 32)
      hipLaunchKernelGGL((scatter_emu16<1024, 32>), dim3(tiles), dim3(1024), 0, s, i, o, n);
    else if (block == 512 && items == 32)
      hipLaunchKernelGGL((scatter_emu16<512, 32>), dim3(tiles), dim3(512), 0, s, i, o, n);
    else if (block == 256 && items == 16)
      hipLaunchKernelGGL((scatter_emu16<256, 16>), dim3(tiles), dim3(256), 0, s, i, o, n);
    else
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// boundary-line hand-off emulation (scatter_emu_handoff): block, items, variant
int lab2_emu_handoff(int block, int items, int var, int lds, const void* in, void* out, uint32_t n,
                     uint32_t* ring, uint32_t* flags, uint32_t epoch, uint32_t* err, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t tiles = n / (block * items);
  const void* k = nullptr;
  switch (block * 100000 + items * 100 + var) {
    case 102403600: k = (const void*)scatter_emu_handoff<1024, 36, 0>; break;
    case 102403601: k = (const void*)scatter_emu_handoff<1024, 36, 1>; break;
    case 102403602: k = (const void*)scatter_emu_handoff<1024, 36, 2>; break;
    case 102404800: k = (const void*)scatter_emu_handoff<1024, 48, 0>; break;
    case 102404801: k = (const void*)scatter_emu_handoff<1024, 48, 1>; break;
    default: return -1;
  }
  const uint32_t* i = static_cast<const uint32_t*>(in);
  uint32_t* o = static_cast<uint32_t*>(out);
  void* args[] = {&i, &o, &n, &ring, &flags, &epoch, &err};
  if (hipLaunchKernel(k, dim3(tiles), dim3(block), args, lds, s) != hipSuccess) return -2;
  return 0;
}

// pairs memory-pattern emulation: block, items, aos, dynamic LDS bytes; AoS buffers are 2n words
int lab2_emu_pairs(int block, int items, int aos, int lds, const void* kin, const void* vin, void* kout,
                   void* vout, uint32_t n, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t tiles = n / (block * items);
  const void* k = nullptr;
  const int code = block * 10000 + items * 10 + aos;
  switch (code) {
    case 10240320: k = (const void*)scatter_emu_pairs<1024, 32, 0>; break;
    case 10240321: k = (const void*)scatter_emu_pairs<1024, 32, 1>; break;
    case 7680400: k = (const void*)scatter_emu_pairs<768, 40, 0>; break;
    case 7680401: k = (const void*)scatter_emu_pairs<768, 40, 1>; break;
    default: return -1;
  }
  const uint32_t* a = static_cast<const uint32_t*>(kin);
  const uint32_t* b = static_cast<const uint32_t*>(vin);
  uint32_t* c = static_cast<uint32_t*>(kout);
  uint32_t* d = static_cast<uint32_t*>(vout);
  void* args[] = {&a, &b, &c, &d, &n};
  if (hipLaunchKernel(k, dim3(tiles), dim3(block), args, lds, s) != hipSuccess) return -2;
  return 0;
}

// copy / read ceilings: kind 0 = copy, 1 = read; unroll 1/4/8; grid
// cycles per returning ds_add wave-instruction (16 waves per CU) for DISTINCT addresses per wave
int lab2_lds_atomic(int distinct, int iters, uint32_t* out, int blocks, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (distinct) {
    case 64: hipLaunchKernelGGL(lds_atomic_rate<64>, dim3(blocks), dim3(1024), 0, s, out, iters); break;
    case 32: hipLaunchKernelGGL(lds_atomic_rate<32>, dim3(blocks), dim3(1024), 0, s, out, iters); break;
    case 16: hipLaunchKernelGGL(lds_atomic_rate<16>, dim3(blocks), dim3(1024), 0, s, out, iters); break;
    case 8: hipLaunchKernelGGL(lds_atomic_rate<8>, dim3(blocks), dim3(1024), 0, s, out, iters); break;
    case 1: hipLaunchKernelGGL(lds_atomic_rate<1>, dim3(blocks), dim3(1024), 0, s, out, iters); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lab2_stream(int kind, int unroll, int grid, const void* in, void* out, uint64_t bytes,
                void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t n4 = static_cast<uint32_t>(bytes / 16);
  const uint4* i4 = static_cast<const uint4*>(in);
  uint4* o4 = static_cast<uint4*>(out);
  if (kind == 0) {
    if (unroll == 1) hipLaunchKernelGGL(copy_u<1>, dim3(grid), dim3(256), 0, s, i4, o4, n4);
    else if (unroll == 4) hipLaunchKernelGGL(copy_u<4>, dim3(grid), dim3(256), 0, s, i4, o4, n4);
    else hipLaunchKernelGGL(copy_u<8>, dim3(grid), dim3(256), 0, s, i4, o4, n4);
  } else {
    if (unroll == 1) hipLaunchKernelGGL(read_u<1>, dim3(grid), dim3(256), 0, s, i4, (uint32_t*)out, n4);
    else if (unroll == 4) hipLaunchKernelGGL(read_u<4>, dim3(grid), dim3(256), 0, s, i4, (uint32_t*)out, n4);
    else hipLaunchKernelGGL(read_u<8>, dim3(grid), dim3(256), 0, s, i4, (uint32_t*)out, n4);
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


// replay of one pass's memory traffic: block, items, radix bits (see replay_pass)
int lab2_replay(int block, int items, int rb, int x8, const uint32_t* pre, uint32_t* out,
                const uint32_t* table, uint32_t n, int shift, uint32_t* ticket, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t tiles = (n + block * items - 1) / (block * items);
#define RP(B, I, RB_)                                                                        \
  if (block == B && items == I && rb == RB_) {                                               \
    if (x8)                                                                                  \
      hipLaunchKernelGGL((replay_pass<B, I, RB_, true>), dim3(tiles), dim3(B), 0, s, pre, out, \
                         table, n, shift, ticket);                                           \
    else                                                                                     \
      hipLaunchKernelGGL((replay_pass<B, I, RB_, false>), dim3(tiles), dim3(B), 0, s, pre, out, \
                         table, n, shift, ticket);                                           \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                         \
  }
  RP(1024, 36, 8) RP(768, 64, 8) RP(1024, 32, 4) RP(1024, 48, 8) RP(1024, 16, 8) RP(1024, 40, 8)
  RP(768, 56, 8) RP(768, 60, 8)
  // round 5: 3-pass u32 (11/11/10-bit digits) floors
  RP(768, 64, 11) RP(1024, 36, 11) RP(1024, 48, 11) RP(768, 64, 10) RP(1024, 36, 10)
#undef RP
  return -1;
}

// single-pass scan (grs_scan_onepass<rows>) beside the library's scan (tools/ab_scan.py)
int lab2_scan2(int rows, const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* ctl,
               uint32_t* total, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint32_t TILE = GRS_SCAN_OP_BLOCK / 64 * rows * 256;
  const uint32_t tiles = (n + TILE - 1) / TILE;
  if (hipMemsetAsync(ctl, 0, 16 + 8 * static_cast<size_t>(tiles), s) != hipSuccess) return -2;
  if (rows == 16)
    hipLaunchKernelGGL(grs::grs_scan_onepass<16>, dim3(tiles), dim3(GRS_SCAN_OP_BLOCK), 0, s, in, out, n, ctl, total, (uint32_t*)nullptr);
  else if (rows == 8)
    hipLaunchKernelGGL(grs::grs_scan_onepass<8>, dim3(tiles), dim3(GRS_SCAN_OP_BLOCK), 0, s, in, out, n, ctl, total, (uint32_t*)nullptr);
  else if (rows == 32)
    hipLaunchKernelGGL(grs::grs_scan_onepass<32>, dim3(tiles), dim3(GRS_SCAN_OP_BLOCK), 0, s, in, out, n, ctl, total, (uint32_t*)nullptr);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
}  // extern "C"
