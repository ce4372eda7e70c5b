"""Python mirror of the reference's controller surface (same names, same argument meaning).

Reference (amdreallyfast/GpuRadixSort):
  OriginalDataSsbo(numItems)      Include/SSBOs/OriginalDataSsbo.h:16-20, Source/SSBOs/OriginalDataSsbo.cpp:20-33
  ParallelSort(dataToSort)        Include/ComputeControllers/ParallelSort.h:46
  ParallelSort.Sort()             Include/ComputeControllers/ParallelSort.h:48, ParallelSort.cpp:168-422

The SSBO becomes a device tensor of uint32 `_value`s; Sort() sorts it in place with the
HIP kernels of libgrs (no CPU path).  Errors raise GrsError instead of printing.
RecordSort generalises the reference's IntermediateData design (ParallelSort.h:27-31,
IntermediateSortBuffers.comp:5-25): sort (key, original index) pairs, then gather whole
records by index (K5, SortOriginalData.comp:27-51) and copy them back (ParallelSort.cpp:311-318).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from .sorter import RadixSorter, gather_records, iota_u32


class OriginalDataSsbo:
    """Device buffer of `numItems` OriginalData records (uint32 `_value`), zero-filled."""

    def __init__(self, numItems: int, device: Optional[int] = None):
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._data = torch.zeros(int(numItems), dtype=torch.uint32, device=dev)

    def NumItems(self) -> int:
        return self._data.numel()

    def Buffer(self) -> torch.Tensor:
        """The device tensor (the reference's BufferId())."""
        return self._data

    def Upload(self, values) -> None:
        """glBufferSubData (main.cpp:146-149)."""
        t = torch.as_tensor(values).to(torch.int64).to(torch.uint32)
        if t.numel() != self.NumItems():
            raise ValueError("Upload: size mismatch")
        self._data.copy_(t.to(self._data.device))

    def Download(self) -> torch.Tensor:
        """glMapBufferRange readback (ParallelSort.cpp:330-333)."""
        return self._data.cpu()


class ParallelSort:
    """Bound to one OriginalDataSsbo; owns the sort scratch (ParallelSort.cpp:36-145)."""

    def __init__(self, dataToSort: OriginalDataSsbo, stream: Optional[torch.cuda.Stream] = None):
        if dataToSort is None:
            raise ValueError("ParallelSort: dataToSort is None")
        self._originalDataSsbo = dataToSort
        self._stream = stream
        # the record is its own key: a keys-only u32 sort at 8-bit digits
        self._sorter = RadixSorter(max(dataToSort.NumItems(), 1), key_bits=32, pairs=False,
                                   radix_bits=8, device=dataToSort.Buffer().device.index)

    def Sort(self) -> None:
        """Sort the bound buffer in place and synchronise the stream (the reference's Sort()
        ends with a blocking map, ParallelSort.cpp:330-333); raises GrsError (GRS_ETIMEOUT) if
        a look-back spin gave up.  SortAsync() only enqueues."""
        self.SortAsync()
        self._sorter.check_error(self._stream)

    def SortAsync(self) -> None:
        buf = self._originalDataSsbo.Buffer()
        self._sorter.sort(buf, stream=self._stream)


class RecordSort:
    """Sort fixed-size records (a Particle struct, ...) by a key — the reference's intended
    use (ParallelSort.h:13-31: "sort the particles ... by Morton codes").

    records: contiguous device tensor whose first dimension is N (e.g. uint8 (N, record_bytes)).
    The key comes from ONE of:
      field=offset [, transform]   the key-width field at that byte offset of every record
                                   (transform: KEYS_UNSIGNED / KEYS_SIGNED / KEYS_FLOAT)
      morton=(offset, lo, hi)      Morton code of the float x, y, z at offset (10 bits per axis
                                   with key_bits=32, 21 with 64), normalised by lo / hi
    — both run the K1 key-extraction hook inside libgrs (grs_sort_records: fused extraction
    pre-pass, stable (key, index) sort, K5 gather, copy back) — or
      keys=tensor                  precomputed device keys (sorted along with the records, in
                                   place: the caller's tensor ends up in key order)
    """

    def __init__(self, capacity: int, key_bits: int = 32, radix_bits: int = 8,
                 device: Optional[int] = None):
        self.capacity = int(capacity)
        self.key_bits = int(key_bits)
        self._sorter = RadixSorter(max(self.capacity, 1), key_bits=key_bits, pairs=True,
                                   radix_bits=radix_bits, device=device)
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._idx = torch.empty(max(self.capacity, 1), dtype=torch.uint32, device=dev)

    def sort(self, records: torch.Tensor, keys: Optional[torch.Tensor] = None, *,
             field: Optional[int] = None, transform: int = 0, morton=None,
             stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        if not records.is_cuda or not records.is_contiguous():
            raise ValueError("records must be a contiguous device tensor")
        n = records.shape[0] if records.dim() else 0
        if sum(x is not None for x in (keys, field, morton)) != 1:
            raise ValueError("give exactly one of keys=, field=, morton=")
        if n > self.capacity:
            raise ValueError("more records than the capacity")
        if n == 0:
            return records
        rb = records.numel() * records.element_size() // n
        if keys is not None:
            if keys.numel() < n:
                raise ValueError("records and keys disagree on N")
            idx = self._idx[:n]
            iota_u32(idx, 0, stream)                       # K1: _globalIndexOfOriginalData = tid
            self._sorter.sort(keys, idx, n=n, stream=stream)  # stable (key, idx) sort, in place
            copy = torch.empty_like(records)
            gather_records(records, copy, idx, n, rb, stream)  # K5 gather
            records.copy_(copy)                             # copy back
            return records
        from ._lib import GRS_EXTRACT_FIELD, GRS_EXTRACT_MORTON3, check, grs_key_extract, lib
        from .sorter import _ptr, _stream_ptr

        kx = grs_key_extract()
        if field is not None:
            kx.kind, kx.offset, kx.transform = GRS_EXTRACT_FIELD, int(field), int(transform)
        else:
            off, lo, hi = morton
            kx.kind, kx.offset = GRS_EXTRACT_MORTON3, int(off)
            for a in range(3):
                kx.lo[a], kx.hi[a] = float(lo[a]), float(hi[a])
        check(lib().grs_sort_records(self._sorter._h, _ptr(records), n, rb, ctypes.byref(kx),
                                     _stream_ptr(stream)), "grs_sort_records")
        return records
