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

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
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

// The compute controller: bound to one OriginalDataSsbo, owns the sort scratch.
class ParallelSort {
 public:
  explicit ParallelSort(const OriginalDataSsbo::SHARED_PTR& dataToSort, void* stream = nullptr)
      : _originalDataSsbo(dataToSort), _stream(stream) {
    if (!dataToSort) throw std::invalid_argument("ParallelSort: null OriginalDataSsbo");
    int dev = 0;
    grs::check_hip(hipGetDevice(&dev), "ParallelSort");
    // 4-byte records whose key is the record itself: a keys-only u32 sort at 8-bit digits.
    grs::check(grs_create(&_sorter, dataToSort->NumItems(), GRS_KEY_U32, 0, 8, dev),
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
    grs::check(grs_sort(_sorter, _originalDataSsbo->DevicePtr(), nullptr,
                        _originalDataSsbo->NumItems(), _stream),
               "ParallelSort::Sort");
  }
  void CheckError() { grs::check(grs_stream_check_error(_sorter, _stream), "ParallelSort::CheckError"); }

  // Per-phase GPU times of the last Sort() when profiling is on (durations.txt successor).
  void SetProfiling(bool on) { grs::check(grs_set_profiling(_sorter, on ? 1 : 0), "SetProfiling"); }
  grs_timing LastTiming() {
    grs_timing t;
    grs::check(grs_last_timing(_sorter, &t), "LastTiming");
    return t;
  }

 private:
  OriginalDataSsbo::SHARED_PTR _originalDataSsbo;
  grs_sorter* _sorter = nullptr;
  void* _stream = nullptr;
};
