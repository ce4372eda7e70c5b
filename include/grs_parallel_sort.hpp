// grs_parallel_sort.hpp — C++ host facade that keeps the reference's dispatch surface.
//
// Reference interface (amdreallyfast/GpuRadixSort):
//   struct OriginalData { unsigned int _value; }            Include/SSBOs/OriginalData.h:14-31
//   struct IntermediateData { _data; _globalIndexOfOriginalData; }
//                                                           Include/SSBOs/IntermediateData.h:12-30
//   class OriginalDataSsbo(unsigned numItems), NumItems()   Include/SSBOs/OriginalDataSsbo.h:16-20,
//                                                           Source/SSBOs/OriginalDataSsbo.cpp:20-33
//   class ParallelSort(const OriginalDataSsbo::SHARED_PTR&), Sort()
//                                                           Include/ComputeControllers/ParallelSort.h:46-48
//
// The GL shader-storage buffers become HIP device buffers; BufferId() becomes DevicePtr().
// Behaviour kept: the caller's buffer is sorted in place, ascending, stably; the controller
// is bound to one data buffer and owns its scratch.  Behaviour changed on purpose: errors
// throw grs::Error instead of being printed (ShaderStorage.cpp:338-339) or ignored, and
// there is no 1,048,576-item ceiling (PrefixScanBuffer.comp:36).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "grs.h"

namespace grs {

struct Error : std::runtime_error {
  grs_status status;
  Error(grs_status s, const std::string& what)
      : std::runtime_error(what + ": " + grs_status_string(s) + " (" + grs_last_error() + ")"),
        status(s) {}
};

inline void check(grs_status s, const char* what) {
  if (s != GRS_OK) throw Error(s, what);
}

inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace grs

// 4-byte user record; the sort key is _value (OriginalData.h:14-31).
struct OriginalData {
  unsigned int _value;
};

// {key, original index} pair (IntermediateData.h:12-30) — the payload form of grs_sort.
struct IntermediateData {
  unsigned int _data;
  unsigned int _globalIndexOfOriginalData;
};

// Device buffer of OriginalData records (OriginalDataSsbo.cpp:20-33: allocate + zero-fill).
class OriginalDataSsbo {
 public:
  typedef std::shared_ptr<OriginalDataSsbo> SHARED_PTR;

  explicit OriginalDataSsbo(unsigned int numItems) : _numItems(numItems) {
    if (numItems) {
      grs::check_hip(hipMalloc(&_data, sizeof(OriginalData) * numItems), "OriginalDataSsbo");
      grs::check_hip(hipMemset(_data, 0, sizeof(OriginalData) * numItems), "OriginalDataSsbo");
    }
  }
  ~OriginalDataSsbo() {
    if (_data) (void)hipFree(_data);
  }
  OriginalDataSsbo(const OriginalDataSsbo&) = delete;
  OriginalDataSsbo& operator=(const OriginalDataSsbo&) = delete;

  unsigned int NumItems() const { return _numItems; }
  OriginalData* DevicePtr() const { return _data; }

  // glBufferSubData upload (main.cpp:146-149) / glMapBufferRange readback (ParallelSort.cpp:330-333)
  void Upload(const std::vector<OriginalData>& v) {
    if (v.size() != _numItems) throw std::invalid_argument("OriginalDataSsbo::Upload: size mismatch");
    if (_numItems)
      grs::check_hip(hipMemcpy(_data, v.data(), sizeof(OriginalData) * _numItems, hipMemcpyHostToDevice),
                     "OriginalDataSsbo::Upload");
  }
  std::vector<OriginalData> Download() const {
    std::vector<OriginalData> v(_numItems);
    if (_numItems)
      grs::check_hip(hipMemcpy(v.data(), _data, sizeof(OriginalData) * _numItems, hipMemcpyDeviceToHost),
                     "OriginalDataSsbo::Download");
    return v;
  }

 private:
  unsigned int _numItems = 0;
  OriginalData* _data = nullptr;
};

// Device buffer of user records of any size (a Particle struct, ...): the record form of
// OriginalDataSsbo for ParallelSort's record constructor.
template <typename Record>
class RecordSsbo {
 public:
  typedef std::shared_ptr<RecordSsbo<Record>> SHARED_PTR;

  explicit RecordSsbo(unsigned int numItems) : _numItems(numItems) {
    if (numItems) {
      grs::check_hip(hipMalloc(&_data, sizeof(Record) * numItems), "RecordSsbo");
      grs::check_hip(hipMemset(_data, 0, sizeof(Record) * numItems), "RecordSsbo");
    }
  }
  ~RecordSsbo() {
    if (_data) (void)hipFree(_data);
  }
  RecordSsbo(const RecordSsbo&) = delete;
  RecordSsbo& operator=(const RecordSsbo&) = delete;

  unsigned int NumItems() const { return _numItems; }
  Record* DevicePtr() const { return _data; }
  void Upload(const std::vector<Record>& v) {
    if (v.size() != _numItems) throw std::invalid_argument("RecordSsbo::Upload: size mismatch");
    if (_numItems)
      grs::check_hip(hipMemcpy(_data, v.data(), sizeof(Record) * _numItems, hipMemcpyHostToDevice),
                     "RecordSsbo::Upload");
  }
  std::vector<Record> Download() const {
    std::vector<Record> v(_numItems);
    if (_numItems)
      grs::check_hip(hipMemcpy(v.data(), _data, sizeof(Record) * _numItems, hipMemcpyDeviceToHost),
                     "RecordSsbo::Download");
    return v;
  }

 private:
  unsigned int _numItems = 0;
  Record* _data = nullptr;
};

// Key-extraction specs for the record constructor (the K1 hook, grs_sort_records).
namespace grs {
inline grs_key_extract FieldKey(uint32_t offset, int transform = GRS_KEYS_UNSIGNED) {
  grs_key_extract k{};
  k.kind = GRS_EXTRACT_FIELD;
  k.offset = offset;
  k.transform = transform;
  return k;
}
inline grs_key_extract MortonKey(uint32_t offset, const float lo[3], const float hi[3]) {
  grs_key_extract k{};
  k.kind = GRS_EXTRACT_MORTON3;
  k.offset = offset;
  for (int i = 0; i < 3; ++i) {
    k.lo[i] = lo[i];
    k.hi[i] = hi[i];
  }
  return k;
}
}  // namespace grs

// The compute controller: bound to one data buffer, owns the sort scratch.
//  * ParallelSort(OriginalDataSsbo)           the reference's constructor (ParallelSort.h:46):
//                                             4-byte records whose key is the record
//  * ParallelSort(RecordSsbo<Record>, key)    records of any size sorted by a key extracted
//                                             from each record (a field, or a Morton code of a
//                                             float3 position: "sort the particles ... by Morton
//                                             codes", ParallelSort.h:13-31)
class ParallelSort {
 public:
  explicit ParallelSort(const OriginalDataSsbo::SHARED_PTR& dataToSort, void* stream = nullptr)
      : _keep(dataToSort), _stream(stream) {
    if (!dataToSort) throw std::invalid_argument("ParallelSort: null OriginalDataSsbo");
    _data = dataToSort->DevicePtr();
    _numItems = dataToSort->NumItems();
    int dev = 0;
    grs::check_hip(hipGetDevice(&dev), "ParallelSort");
    // 4-byte records whose key is the record itself: a keys-only u32 sort at 8-bit digits.
    grs::check(grs_create(&_sorter, _numItems, GRS_KEY_U32, 0, 8, dev), "ParallelSort: grs_create");
  }

  // u32 keys (key_bits = 32) or u64 keys (64) extracted by `key`; stable.
  template <typename Record>
  ParallelSort(const std::shared_ptr<RecordSsbo<Record>>& dataToSort, const grs_key_extract& key,
               int key_bits = 32, void* stream = nullptr)
      : _keep(dataToSort), _stream(stream), _records(true), _recordBytes(sizeof(Record)), _key(key) {
    if (!dataToSort) throw std::invalid_argument("ParallelSort: null RecordSsbo");
    if (key_bits != 32 && key_bits != 64) throw std::invalid_argument("ParallelSort: key_bits 32 or 64");
    _data = dataToSort->DevicePtr();
    _numItems = dataToSort->NumItems();
    int dev = 0;
    grs::check_hip(hipGetDevice(&dev), "ParallelSort");
    grs::check(grs_create(&_sorter, _numItems, key_bits == 64 ? GRS_KEY_U64 : GRS_KEY_U32, 1, 8, dev),
               "ParallelSort: grs_create");
  }
  ~ParallelSort() { grs_destroy(_sorter); }
  ParallelSort(const ParallelSort&) = delete;
  ParallelSort& operator=(const ParallelSort&) = delete;

  // Sorts the bound buffer in place (ParallelSort.cpp:168-422) and synchronises the stream:
  // like the reference's Sort(), which ends by mapping the buffer (ParallelSort.cpp:330-333),
  // it returns with the data sorted, and it throws grs::Error (GRS_ETIMEOUT) if a look-back
  // spin of the sort gave up.  SortAsync() only enqueues (check later with CheckError()).
  void Sort() {
    SortAsync();
    CheckError();
  }
  void SortAsync() {
    if (_records)
      grs::check(grs_sort_records(_sorter, _data, _numItems, _recordBytes, &_key, _stream),
                 "ParallelSort::Sort");
    else
      grs::check(grs_sort(_sorter, _data, nullptr, _numItems, _stream), "ParallelSort::Sort");
  }
  void CheckError() { grs::check(grs_stream_check_error(_sorter, _stream), "ParallelSort::CheckError"); }

  // Pins a kernel choice of the sorter (grs_set_option; A/B runs, and the error path's test
  // hook GRS_OPT_FAULT_TILE).
  void SetOption(grs_option opt, int value) {
    grs::check(grs_set_option(_sorter, opt, value), "ParallelSort::SetOption");
  }

  // Per-phase GPU times of the last Sort() when profiling is on (durations.txt successor).
  void SetProfiling(bool on) { grs::check(grs_set_profiling(_sorter, on ? 1 : 0), "SetProfiling"); }
  grs_timing LastTiming() {
    grs_timing t;
    grs::check(grs_last_timing(_sorter, &t), "LastTiming");
    return t;
  }

 private:
  std::shared_ptr<void> _keep;   // the bound buffer stays alive as long as the controller
  void* _data = nullptr;
  unsigned int _numItems = 0;
  grs_sorter* _sorter = nullptr;
  void* _stream = nullptr;
  bool _records = false;
  size_t _recordBytes = 4;
  grs_key_extract _key{};
};

// ---- user-defined key functors (the reference's K1 hook) ----------------------------------
// The reference's K1 is written to "adapt to whatever needs to be sorted": structs with
// integers, floats and vec4s (Shaders/ParallelSort/OriginalDataToIntermediateData.comp:12-19,
// 42; ParallelSort.h:15-18,27-31).  ParallelSortBy<Record, KeyFn> takes any device-callable
// key function of a record; the caller's hipcc instantiates its extraction kernel here, and
// libgrs sorts the (key, index) pairs and gathers the records (grs_sort_records_by_keys).
namespace grs {

// Order-preserving bit maps for functors whose key is signed or floating point: a < b (as
// int / float, IEEE-754 total order: -NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN) iff
// OrderedBits(a) < OrderedBits(b) as unsigned (the maps of grs_key_transform).
__host__ __device__ inline uint32_t OrderedBits(int32_t v) { return static_cast<uint32_t>(v) ^ 0x80000000u; }
__host__ __device__ inline uint64_t OrderedBits(int64_t v) {
  return static_cast<uint64_t>(v) ^ 0x8000000000000000ull;
}
__host__ __device__ inline uint32_t OrderedBits(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline uint64_t OrderedBits(double f) {
  uint64_t u;
  __builtin_memcpy(&u, &f, 8);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// K1 with the caller's functor: keys[i] = fn(rec[i]), idx[i] = i (grid-stride).
template <typename Key, typename Record, typename KeyFn>
__global__ void ExtractKeysWith(const Record* __restrict__ rec, uint32_t n, KeyFn fn,
                                Key* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    keys[i] = static_cast<Key>(fn(rec[i]));
    idx[i] = i;
  }
}

}  // namespace grs

// Controller bound to a RecordSsbo<Record> that sorts it in place, stably, by key_fn(record):
// KeyFn is a functor with a __device__ (or __host__ __device__) const operator() taking a
// const Record& and returning uint32_t or uint64_t (use grs::OrderedBits for int / float keys).
template <typename Record, typename KeyFn>
class ParallelSortBy {
 public:
  using Key = std::decay_t<decltype(std::declval<const KeyFn&>()(std::declval<const Record&>()))>;
  static_assert(std::is_same<Key, uint32_t>::value || std::is_same<Key, uint64_t>::value,
                "the key functor must return uint32_t or uint64_t (grs::OrderedBits maps signed "
                "and floating-point keys)");

  ParallelSortBy(const std::shared_ptr<RecordSsbo<Record>>& dataToSort, KeyFn keyFn,
                 void* stream = nullptr)
      : _keep(dataToSort), _fn(keyFn), _stream(stream) {
    if (!dataToSort) throw std::invalid_argument("ParallelSortBy: null RecordSsbo");
    _data = dataToSort->DevicePtr();
    _numItems = dataToSort->NumItems();
    int dev = 0;
    grs::check_hip(hipGetDevice(&dev), "ParallelSortBy");
    grs::check(grs_create(&_sorter, _numItems, sizeof(Key) == 8 ? GRS_KEY_U64 : GRS_KEY_U32, 1, 8, dev),
               "ParallelSortBy: grs_create");
  }
  ~ParallelSortBy() { grs_destroy(_sorter); }
  ParallelSortBy(const ParallelSortBy&) = delete;
  ParallelSortBy& operator=(const ParallelSortBy&) = delete;

  // Blocking, like ParallelSort::Sort(); SortAsync() only enqueues.
  void Sort() {
    SortAsync();
    grs::check(grs_stream_check_error(_sorter, _stream), "ParallelSortBy::CheckError");
  }
  void SortAsync() {
    if (_numItems == 0) return;
    void* keys = nullptr;
    uint32_t* idx = nullptr;
    grs::check(grs_records_key_buffers(_sorter, _numItems, sizeof(Record), &keys, &idx),
               "ParallelSortBy: key buffers");
    const unsigned grid = std::min<unsigned>((_numItems + 255) / 256, 8192u);
    hipLaunchKernelGGL((grs::ExtractKeysWith<Key, Record, KeyFn>), dim3(grid), dim3(256), 0,
                       static_cast<hipStream_t>(_stream), _data, _numItems, _fn,
                       static_cast<Key*>(keys), idx);
    grs::check_hip(hipGetLastError(), "ParallelSortBy: extract launch");
    grs::check(grs_sort_records_by_keys(_sorter, _data, _numItems, sizeof(Record), keys, idx, _stream),
               "ParallelSortBy::Sort");
  }

 private:
  std::shared_ptr<void> _keep;
  Record* _data = nullptr;
  unsigned int _numItems = 0;
  KeyFn _fn;
  grs_sorter* _sorter = nullptr;
  void* _stream = nullptr;
};

// Multi-GPU controller (one process per GPU): sorts this rank's shard as part
// of the global input over an RCCL communicator (grs_sort_sharded).  Output: this rank's
// contiguous range of the global stable order.
class ShardedParallelSort {
 public:
  // capacity: max(shard, received run) items; nccl_comm: an initialised ncclComm_t
  ShardedParallelSort(size_t capacity, void* nccl_comm, int key_bits = 32, bool pairs = false,
                      void* stream = nullptr)
      : _comm(nccl_comm), _stream(stream) {
    int dev = 0;
    grs::check_hip(hipGetDevice(&dev), "ShardedParallelSort");
    grs::check(grs_create(&_sorter, capacity, key_bits == 64 ? GRS_KEY_U64 : GRS_KEY_U32,
                          pairs ? 1 : 0, 8, dev),
               "ShardedParallelSort: grs_create");
  }
  ~ShardedParallelSort() { grs_destroy(_sorter); }
  ShardedParallelSort(const ShardedParallelSort&) = delete;
  ShardedParallelSort& operator=(const ShardedParallelSort&) = delete;

  // Returns the number of items this rank holds after the sort (in d_keys_out / d_vals_out).
  size_t Sort(const void* d_keys_in, const uint32_t* d_vals_in, size_t n_local, void* d_keys_out,
              uint32_t* d_vals_out, size_t out_capacity) {
    size_t n_out = 0;
    grs::check(grs_sort_sharded(_sorter, d_keys_in, d_vals_in, n_local, d_keys_out, d_vals_out,
                                out_capacity, &n_out, _comm, _stream),
               "ShardedParallelSort::Sort");
    grs::check(grs_stream_check_error(_sorter, _stream), "ShardedParallelSort::Sort");
    return n_out;
  }

  // Per-phase timing of the last Sort() (EnableProfiling first): before / of / after the
  // exchange, and the bytes that crossed the links (grs_sharded_last_timing).
  void EnableProfiling(int ring = 1) {
    grs::check(grs_set_profiling(_sorter, ring), "ShardedParallelSort::EnableProfiling");
  }
  grs_sharded_timing LastExchangeTiming() {
    grs_sharded_timing t{};
    grs::check(grs_sharded_last_timing(_sorter, &t), "ShardedParallelSort::LastExchangeTiming");
    return t;
  }

 private:
  grs_sorter* _sorter = nullptr;
  void* _comm = nullptr;
  void* _stream = nullptr;
};
