"""gpuradixsort_amd — MI355X-native (gfx950) stable radix sort behind the reference's
ParallelSort controller surface (amdreallyfast/GpuRadixSort).  Large sorts (from 48M keys) run
an MSD-first schedule (two stable scatters by the keys' top two varying bytes, then every 16-bit
segment sorted in LDS); smaller ones and 4-bit digits the stable LSD passes.  Both give the
reference's output (the stable sort by key) bit for bit.

  RadixSorter          the C-ABI sorter (include/grs.h) over torch device tensors
  OriginalDataSsbo,
  ParallelSort         the reference's names and call pattern (ParallelSort.h:46-48)
  RecordSort           sort whole records by a key (K1 key hook + pair sort + K5 gather)
  key_transform        order-preserving signed / float key bits (sort them as unsigned)
  exclusive_scan_u32   stand-alone device-wide scan (the reference's K3a + K3b)
  RadixSorter.sort_segmented   batched sort of independent segments
  sharded.ShardedSorter        multi-GPU key-range sort (grs_sort_sharded): device splitters,
                       one exchange of grouped RCCL ncclSend / ncclRecv over xGMI, local sort
                       (or presorted runs bit-packed, exchanged and merged)
  fill_splitmix, fill_permutation   synthetic inputs on the device (uniform keys; the
                       reference's own shuffled 0..N-1)

All compute runs in libgrs.so's HIP kernels; there is no CPU fallback.
"""
from ._lib import GRS_MAX_N, GrsError, lib
from .parallel_sort import OriginalDataSsbo, ParallelSort, RecordSort
from .sorter import (KEYS_FLOAT, KEYS_SIGNED, KEYS_UNSIGNED, RadixSorter, count_inversions,
                     exclusive_scan_u32, fill_permutation, fill_splitmix, gather_records, iota_u32,
                     key_transform)

__all__ = ["GRS_MAX_N", "GrsError", "lib", "OriginalDataSsbo", "ParallelSort", "RecordSort",
           "RadixSorter", "count_inversions", "fill_splitmix", "fill_permutation", "gather_records",
           "iota_u32", "key_transform", "exclusive_scan_u32", "KEYS_UNSIGNED", "KEYS_SIGNED",
           "KEYS_FLOAT"]
