/* ref_restatement.c — TEST INFRASTRUCTURE ONLY (the parity oracle; never shipped, never
 * called by the product path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * A plain-C restatement of the reference's GLSL sort path (amdreallyfast/GpuRadixSort), one
 * function per compute program, each citing the file:line it follows.  The reference cannot
 * be built or run here (OpenGL 4.5 compute + MSVC-only host code), so this
 * restatement is pinned instead by the reference's own known-answer data (PrefixScan.xlsx
 * scan trace, the 16-key vector of main.cpp:128-143 — see tests/golden/) and cross-checked
 * against a stable merge sort.
 *
 * GLSL invocations of one dispatch touch disjoint elements within each barrier-separated
 * step, so running each step's invocations sequentially reproduces the shader exactly.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Shaders/ParallelSort/ParallelSortConstants.comp:17,24 */
#define WORK_GROUP_SIZE_X 512u
#define ITEMS_PER_WORK_GROUP (WORK_GROUP_SIZE_X * 2u)
/* PrefixScanBuffer.comp:36: PrefixSumsByGroup is exactly one work group's worth */
#define MAX_ITEMS (ITEMS_PER_WORK_GROUP * ITEMS_PER_WORK_GROUP)

/* Padded item count P = ceil(N / 1024) * 1024 (Source/SSBOs/PrefixSumSsbo.cpp:125-127). */
uint32_t ref_padded_count(uint32_t n) {
  uint32_t p = n / ITEMS_PER_WORK_GROUP;
  p += (n % ITEMS_PER_WORK_GROUP == 0) ? 0 : 1;
  return p * ITEMS_PER_WORK_GROUP;
}

/* Work-efficient (Blelloch) exclusive scan of one group of `size` items held in `a`
 * (power of two), exactly as ParallelPrefixScan.comp:56-141 does it in shared memory:
 * up-sweep (70-90), store + zero the root (93-104), down-sweep (114-135).  Returns the
 * group total.  `size` = ITEMS_PER_WORK_GROUP in the reference; the PrefixScan.xlsx worked
 * example uses size 32. */
uint32_t ref_blelloch_scan_group(uint32_t* a, uint32_t size) {
  uint32_t threads = size / 2u;
  uint32_t mult = 1; /* indexMultiplierDueToDepth */
  for (uint32_t pairs = size >> 1; pairs > 0; pairs >>= 1) {
    for (uint32_t tid = 0; tid < threads; ++tid) {
      if (tid < pairs) {
        uint32_t dbl = tid * 2u;
        uint32_t lesser = mult * (dbl + 1u) - 1u;
        uint32_t greater = mult * (dbl + 2u) - 1u;
        a[greater] += a[lesser];
      }
    }
    mult *= 2u;
  }
  uint32_t total = a[size - 1u];
  a[size - 1u] = 0;
  mult >>= 1;
  for (uint32_t pairs = 1; pairs < size; pairs *= 2u) {
    for (uint32_t tid = 0; tid < threads; ++tid) {
      if (tid < pairs) {
        uint32_t dbl = tid * 2u;
        uint32_t lesser = mult * (dbl + 1u) - 1u;
        uint32_t greater = mult * (dbl + 2u) - 1u;
        uint32_t tmp = a[lesser];
        a[lesser] = a[greater];
        a[greater] += tmp;
      }
    }
    mult >>= 1;
  }
  return total;
}

/* K1 OriginalDataToIntermediateData.comp:36-51: idx = tid; key = tid < N ? value : ~0. */
void ref_k1_original_to_intermediate(const uint32_t* orig, uint32_t n, uint32_t p,
                                     uint32_t* data, uint32_t* idx) {
  for (uint32_t tid = 0; tid < p; ++tid) {
    idx[tid] = tid;
    data[tid] = tid < n ? orig[tid] : 0xffffffffu;
  }
}

/* K2 GetBitForPrefixScan.comp:33-64: PrefixSumsWithinGroup[tid] = (key >> bit) & 1 and
 * work group 0 zeroes PrefixSumsByGroup[0..1023]. */
void ref_k2_get_bit(const uint32_t* data, uint32_t p, uint32_t bit, uint32_t* within,
                    uint32_t* by_group) {
  for (uint32_t tid = 0; tid < p; ++tid) within[tid] = (data[tid] >> bit) & 1u;
  memset(by_group, 0, ITEMS_PER_WORK_GROUP * sizeof(uint32_t));
}

/* K3a ParallelPrefixScan.comp:41-142 with uCalculateAll = 1: per-1024 Blelloch scan of
 * PrefixSumsWithinGroup, group totals to PrefixSumsByGroup[wg] (line 100). */
void ref_k3a_scan_all(uint32_t* within, uint32_t p, uint32_t* by_group) {
  for (uint32_t wg = 0; wg < p / ITEMS_PER_WORK_GROUP; ++wg)
    by_group[wg] = ref_blelloch_scan_group(within + wg * ITEMS_PER_WORK_GROUP, ITEMS_PER_WORK_GROUP);
}

/* K3b ParallelPrefixScan.comp:151-196 with uCalculateAll = 0: the same scan over the 1024
 * group totals, root value -> totalNumberOfOnes (line 175). */
uint32_t ref_k3b_scan_group_sums(uint32_t* by_group) {
  return ref_blelloch_scan_group(by_group, ITEMS_PER_WORK_GROUP);
}

/* K4 SortIntermediateData.comp:32-67: stable split by one bit.
 *   ones  = PrefixSumsByGroup[wg/2] + PrefixSumsWithinGroup[tid]   (line 272-274, wg of 512)
 *   zeros = tid - ones;  totalZeros = P - totalNumberOfOnes          (lines 281-282)
 *   dst   = bit ? totalZeros + ones : zeros                          (line 292)          */
void ref_k4_sort_intermediate(const uint32_t* data_r, const uint32_t* idx_r, uint32_t* data_w,
                              uint32_t* idx_w, uint32_t p, uint32_t bit, const uint32_t* within,
                              const uint32_t* by_group, uint32_t total_ones) {
  for (uint32_t tid = 0; tid < p; ++tid) {
    uint32_t wg = tid / WORK_GROUP_SIZE_X;
    uint32_t ones = by_group[wg / 2u] + within[tid];
    uint32_t zeros = tid - ones;
    uint32_t total_zeros = p - total_ones;
    uint32_t b = (data_r[tid] >> bit) & 1u;
    uint32_t dst = b == 0 ? zeros : total_zeros + ones;
    data_w[dst] = data_r[tid];
    idx_w[dst] = idx_r[tid];
  }
}

/* K5 SortOriginalData.comp:33-50: copy[i] = original[idx[i]] for i < N. */
void ref_k5_sort_original(const uint32_t* orig, const uint32_t* idx, uint32_t n, uint32_t* copy) {
  for (uint32_t i = 0; i < n; ++i) copy[i] = orig[idx[i]];
}

/* ParallelSort::Sort() (Source/ComputeControllers/ParallelSort.cpp:168-320): K1, then for
 * bit 0..31 {K2, K3a, K3b, K4, flip halves}, then K5 and the copy back into `data`.
 * Writes the final carried index (the stable permutation) to perm_out[0..n) if non-NULL.
 * Returns 0, or -1 if n exceeds the reference's 1,048,576 capacity (where the GLSL path
 * silently corrupts memory: PrefixScanBuffer.comp:36), or -2 on allocation failure. */
int ref_parallel_sort(uint32_t* data, uint32_t n, uint32_t* perm_out) {
  if (n > MAX_ITEMS) return -1;
  if (n == 0) return 0; /* PrefixSumSsbo.cpp:121-124: no work groups, no work */
  uint32_t p = ref_padded_count(n);
  uint32_t* key = malloc(2u * p * sizeof(uint32_t)); /* IntermediateDataSsbo: 2 halves */
  uint32_t* idx = malloc(2u * p * sizeof(uint32_t));
  uint32_t* within = malloc(p * sizeof(uint32_t));
  uint32_t* copy = malloc(n * sizeof(uint32_t));
  uint32_t by_group[ITEMS_PER_WORK_GROUP];
  if (!key || !idx || !within || !copy) {
    free(key); free(idx); free(within); free(copy);
    return -2;
  }
  ref_k1_original_to_intermediate(data, n, p, key, idx);
  int write_second = 1; /* ParallelSort.cpp:235 */
  for (uint32_t bit = 0; bit < 32; ++bit) {
    uint32_t roff = (uint32_t)(!write_second) * p; /* lines 239-240 */
    uint32_t woff = (uint32_t)write_second * p;
    ref_k2_get_bit(key + roff, p, bit, within, by_group);
    ref_k3a_scan_all(within, p, by_group);
    uint32_t total_ones = ref_k3b_scan_group_sums(by_group);
    ref_k4_sort_intermediate(key + roff, idx + roff, key + woff, idx + woff, p, bit, within,
                             by_group, total_ones);
    write_second = !write_second; /* line 297 */
  }
  uint32_t roff = (uint32_t)(!write_second) * p; /* line 304 */
  ref_k5_sort_original(data, idx + roff, n, copy);
  memcpy(data, copy, n * sizeof(uint32_t)); /* glCopyBufferSubData, lines 312-318 */
  if (perm_out) memcpy(perm_out, idx + roff, n * sizeof(uint32_t));
  free(key); free(idx); free(within); free(copy);
  return 0;
}

/* ---- independent cross-check: stable merge sort of (key, index) ----------------------- */

static void merge_pass_u64(uint64_t* a, uint32_t* ia, uint64_t* b, uint32_t* ib, size_t n,
                           size_t w) {
  for (size_t lo = 0; lo < n; lo += 2 * w) {
    size_t mid = lo + w < n ? lo + w : n;
    size_t hi = lo + 2 * w < n ? lo + 2 * w : n;
    size_t i = lo, j = mid, k = lo;
    while (i < mid && j < hi) {
      if (a[j] < a[i]) { b[k] = a[j]; ib[k++] = ia[j++]; }   /* ties take the left: stable */
      else { b[k] = a[i]; ib[k++] = ia[i++]; }
    }
    while (i < mid) { b[k] = a[i]; ib[k++] = ia[i++]; }
    while (j < hi) { b[k] = a[j]; ib[k++] = ia[j++]; }
  }
}

/* Stable ascending sort of 64-bit keys; perm[i] = input index of the i-th output key.
 * keys are sorted in place.  Returns 0 or -2 on allocation failure. */
int oracle_stable_sort_u64(uint64_t* keys, uint32_t* perm, size_t n) {
  uint64_t* tk = malloc((n ? n : 1) * sizeof(uint64_t));
  uint32_t* ti = malloc((n ? n : 1) * sizeof(uint32_t));
  if (!tk || !ti) { free(tk); free(ti); return -2; }
  for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
  uint64_t *a = keys, *b = tk;
  uint32_t *ia = perm, *ib = ti;
  for (size_t w = 1; w < n; w *= 2) {
    merge_pass_u64(a, ia, b, ib, n, w);
    uint64_t* t = a; a = b; b = t;
    uint32_t* u = ia; ia = ib; ib = u;
  }
  if (a != keys) {
    memcpy(keys, a, n * sizeof(uint64_t));
    memcpy(perm, ia, n * sizeof(uint32_t));
  }
  free(tk); free(ti);
  return 0;
}

int oracle_stable_sort_u32(uint32_t* keys, uint32_t* perm, size_t n) {
  uint64_t* k = malloc((n ? n : 1) * sizeof(uint64_t));
  if (!k) return -2;
  for (size_t i = 0; i < n; ++i) k[i] = keys[i];
  int r = oracle_stable_sort_u64(k, perm, n);
  for (size_t i = 0; i < n; ++i) keys[i] = (uint32_t)k[i];
  free(k);
  return r;
}

/* splitmix64 synthetic keys: key[i] = splitmix64(seed ^ (first + i)). */
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void oracle_fill_splitmix_u32(uint32_t* out, size_t n, uint64_t seed, uint64_t first) {
  for (size_t i = 0; i < n; ++i) out[i] = (uint32_t)splitmix64(seed ^ (first + i));
}

void oracle_fill_splitmix_u64(uint64_t* out, size_t n, uint64_t seed, uint64_t first) {
  for (size_t i = 0; i < n; ++i) out[i] = splitmix64(seed ^ (first + i));
}
