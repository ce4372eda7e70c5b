// lab6.hip — round-5 laboratory (not part of libgrs): the multi-GPU partition pass
// (grs_onesweep_v4 over PartTile, 1024 x 36 keys, 16-bucket digit) with its digit computed
// different ways, to price the digit against the rest of the pass (tools/lab6.py):
//   0  SplitterIdxDigit<7>   the shipped digit: 7 composite (key, index) 64-bit compares
//   1  SplitterDigitN<7>     7 compares of the key alone (no tie-break index)
//   2  RadixDigit{29, 7}     the top 3 bits (what uniform splitters amount to): a shift
//   3  LutIdxDigit<7>        a 4096-entry byte table on the top 12 bits (global memory), the
//                            composite compares only for a prefix a splitter falls in
// opt: the pass's OPT bits (16 = look-back after the reorder; 272 = also 16-bit wave counters,
// not for indexed digits).
#include <hip/hip_runtime.h>

#include "../gpuradixsort_amd/csrc/grs_pass.hpp"

namespace {

template <typename K, int N>
struct LutIdxDigit {
  static constexpr bool kIndexed = true;
  grs::SplitterIdxDigit<K, N> full;
  const uint8_t* lut;   // bucket of the top 12 bits, 0xFF: a splitter lies in that prefix
  __device__ __forceinline__ uint32_t operator()(K k, uint32_t i) const {
    const uint32_t b = lut[static_cast<uint32_t>(k >> (8 * sizeof(K) - 12))];
    return b != 0xFFu ? b : full(k, i);
  }
  __device__ __forceinline__ uint32_t max_digit() const { return N; }
};

// the shipped digit without its LDS bucket table (the compares for every key)
template <typename K, int N>
struct NoLutIdxDigit {
  static constexpr bool kIndexed = true;
  grs::SplitterIdxDigit<K, N> full;
  __device__ __forceinline__ uint32_t operator()(K k, uint32_t i) const { return full(k, i); }
  __device__ __forceinline__ uint32_t max_digit() const { return N; }
};

// 32-bit compares of the key; the index only for a key equal to a splitter key (rare: a branch
// no lane of a wave usually takes)
template <typename K, int N>
struct TieIdxDigit {
  static constexpr bool kIndexed = true;
  grs::SplitterIdxDigit<K, N> full;
  __device__ __forceinline__ uint32_t operator()(K k, uint32_t i) const {
    uint32_t b = 0;
    bool eq = false;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      b += full.s[j] < k;
      eq |= full.s[j] == k;
    }
    if (eq) b = full(k, i);
    return b;
  }
  __device__ __forceinline__ uint32_t max_digit() const { return N; }
};

template <int OPT, typename D, int ITEMS = 36>
int launch(const D& dig, const uint32_t* in, uint32_t* out, uint32_t n, const uint32_t* hist,
           uint32_t* ticket, uint32_t* st0, uint32_t* st1, uint32_t* err, hipStream_t s) {
  constexpr int BLOCK = 1024;
  const uint32_t tiles = (n + BLOCK * ITEMS - 1) / (BLOCK * ITEMS);
  hipLaunchKernelGGL((grs::grs_onesweep_v4<uint32_t, false, 4, BLOCK, ITEMS, 1, OPT, D>), dim3(tiles),
                     dim3(BLOCK), 0, s, in, out, nullptr, nullptr, n, dig, hist, ticket, st0, st1, err,
                     static_cast<const D*>(nullptr));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

extern "C" int lab6_part(int mode, int opt, const uint32_t* in, uint32_t* out, uint32_t n,
                         const uint32_t* hist, uint32_t* ticket, uint32_t* st0, uint32_t* st1,
                         uint32_t* err, const uint8_t* lut, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  grs::SplitterIdxDigit<uint32_t, 7> idx{};
  grs::SplitterDigitN<uint32_t, 7> plain{};
  idx.count = plain.count = 7;
  for (int j = 0; j < GRS_MAX_SPLITTERS; ++j) {
    const uint32_t sp = j < 7 ? static_cast<uint32_t>(j + 1) << 29 : 0xFFFFFFFFu;
    idx.s[j] = plain.s[j] = sp;
    idx.th[j] = j < 7 ? 0u : 0xFFFFFFFFu;
  }
  if (mode == 0) return opt == 16 ? launch<16>(idx, in, out, n, hist, ticket, st0, st1, err, s) : 2;
  // the shipped digit on smaller tiles (fewer VGPRs: the 36-key tile spills)
  if (mode == 4) return launch<16, decltype(idx), 32>(idx, in, out, n, hist, ticket, st0, st1, err, s);
  if (mode == 5) return launch<16, decltype(idx), 28>(idx, in, out, n, hist, ticket, st0, st1, err, s);
  if (mode == 6) return launch<16, decltype(idx), 24>(idx, in, out, n, hist, ticket, st0, st1, err, s);
  if (mode == 7) {
    const NoLutIdxDigit<uint32_t, 7> nl{idx};
    return launch<16, decltype(nl), 32>(nl, in, out, n, hist, ticket, st0, st1, err, s);
  }
  if (mode == 8) {
    const NoLutIdxDigit<uint32_t, 7> nl{idx};
    return launch<16, decltype(nl), 36>(nl, in, out, n, hist, ticket, st0, st1, err, s);
  }
  if (mode == 9) {
    const TieIdxDigit<uint32_t, 7> td{idx};
    return launch<16, decltype(td), 32>(td, in, out, n, hist, ticket, st0, st1, err, s);
  }
  if (mode == 1)
    return opt == 16 ? launch<16>(plain, in, out, n, hist, ticket, st0, st1, err, s)
                     : launch<272>(plain, in, out, n, hist, ticket, st0, st1, err, s);
  if (mode == 2) {
    const grs::RadixDigit<uint32_t> rd{29, 7u};
    return opt == 16 ? launch<16>(rd, in, out, n, hist, ticket, st0, st1, err, s)
                     : launch<272>(rd, in, out, n, hist, ticket, st0, st1, err, s);
  }
  if (mode == 3) {
    LutIdxDigit<uint32_t, 7> ld{idx, lut};
    return opt == 16 ? launch<16>(ld, in, out, n, hist, ticket, st0, st1, err, s) : 2;
  }
  return 2;
}

extern "C" size_t lab6_status_words(uint32_t n) {
  const uint32_t tiles = (n + 24575) / 24576;   // the smallest tile of the modes
  return grs::lb3_status_words(tiles, 16);
}
