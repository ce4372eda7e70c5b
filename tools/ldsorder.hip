// ldsorder.hip — probe: do conflicting lanes of ONE ds_add_rtn_u32 wave-instruction get their
// old values in ascending lane order?  If so, a per-wave digit counter bumped by one returning
// LDS atomic per item yields a stable rank directly (tools only; the library does not rely on
// an unprobed property — see DESIGN.md).
//
// build: hipcc --offload-arch=gfx950 -O3 -o ldsorder ldsorder.hip ; run: ./ldsorder
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

// Each wave: ITEMS rounds; in round j lane l adds `inc` to counter[dig] where dig comes from the
// input; records the returned old value.  Host checks old == sum of inc of (earlier rounds, same
// digit) + (lower lanes of this round, same digit).
template <int RADIX, int PACK>
__global__ void probe(const uint32_t* __restrict__ dig, uint32_t* __restrict__ out, int items) {
  __shared__ uint32_t cnt[8][RADIX / PACK];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 8 * RADIX / PACK; i += blockDim.x) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const size_t base = (static_cast<size_t>(blockIdx.x) * blockDim.x + (threadIdx.x & ~63)) * items;
  const int lane = threadIdx.x & 63;
  for (int j = 0; j < items; ++j) {
    const uint32_t d = dig[base + j * 64 + lane];
    uint32_t old;
    if (PACK == 2)
      old = atomicAdd(&cnt[w][d >> 1], 1u << ((d & 1) * 16));
    else
      old = atomicAdd(&cnt[w][d], 1u);
    out[base + j * 64 + lane] = PACK == 2 ? ((old >> ((d & 1) * 16)) & 0xFFFF) : old;
  }
}

static uint64_t rng = 88172645463325252ull;
static uint32_t xr() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return static_cast<uint32_t>(rng);
}

template <int RADIX, int PACK>
long run(int mode, int blocks, int items) {
  const size_t n = static_cast<size_t>(blocks) * 512 * items;
  std::vector<uint32_t> h(n), o(n);
  for (size_t i = 0; i < n; ++i) {
    switch (mode) {
      case 0: h[i] = xr() % RADIX; break;                  // uniform
      case 1: h[i] = 7 % RADIX; break;                     // all equal
      case 2: h[i] = (xr() % 4) * (RADIX / 4); break;      // 4 values, same bank
      case 3: h[i] = (i % 64) < 32 ? 3 : xr() % RADIX; break;
      case 4: h[i] = (xr() & 1) ? 5 : (xr() % 2) * 32; break;  // bank-colliding pair + one
      default: h[i] = (xr() % 16) * 32 % RADIX; break;     // 16 values on one bank
    }
  }
  uint32_t *dd, *od;
  hipMalloc(&dd, n * 4);
  hipMalloc(&od, n * 4);
  hipMemcpy(dd, h.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((probe<RADIX, PACK>), dim3(blocks), dim3(512), 0, 0, dd, od, items);
  hipMemcpy(o.data(), od, n * 4, hipMemcpyDeviceToHost);
  hipFree(dd);
  hipFree(od);
  long bad = 0;
  for (size_t wv = 0; wv < n / (64 * items); ++wv) {
    std::vector<uint32_t> c(RADIX, 0);
    for (int j = 0; j < items; ++j)
      for (int l = 0; l < 64; ++l) {
        const size_t i = wv * 64 * items + j * 64 + l;
        if (o[i] != c[h[i]]) ++bad;
        c[h[i]]++;
      }
  }
  return bad;
}

int main() {
  long tot = 0;
  for (int mode = 0; mode < 6; ++mode) {
    long b1 = run<256, 1>(mode, 2048, 24);
    long b2 = run<256, 2>(mode, 2048, 24);
    long b3 = run<2048, 2>(mode, 1024, 16);
    printf("mode %d: mismatches r256=%ld r256packed=%ld r2048packed=%ld\n", mode, b1, b2, b3);
    tot += b1 + b2 + b3;
  }
  printf(tot == 0 ? "LANE-ORDERED\n" : "NOT lane-ordered\n");
  return 0;
}
