"""RadixSorter: the C-ABI sorter (grs_create / grs_sort) over torch device tensors.

torch is only plumbing here: it owns the device buffers and the stream; every byte of the
sort is moved by libgrs's HIP kernels (gpuradixsort_amd/csrc/grs_kernels.hpp).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from ._lib import GRS_KEY_U32, GRS_KEY_U64, OPTIONS, check, grs_timing, lib

_KEY_TYPES = {torch.int32: GRS_KEY_U32, torch.uint32: GRS_KEY_U32,
              torch.int64: GRS_KEY_U64, torch.uint64: GRS_KEY_U64}


def _stream_ptr(stream: Optional[torch.cuda.Stream]) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


class RadixSorter:
    """Stable ascending LSD radix sort of unsigned keys (u32 or u64), optionally carrying a
    uint32 payload; mirrors ParallelSort's ctor/Sort() split (ParallelSort.cpp:36-145 /
    168-422): scratch is sized once at construction, sort() is asynchronous on the stream.

    Keys are interpreted as UNSIGNED integers of their width whatever torch dtype holds
    them (torch.int32 / torch.uint32 / torch.int64 / torch.uint64)."""

    def __init__(self, capacity: int, key_bits: int = 32, pairs: bool = False,
                 radix_bits: int = 8, device: Optional[int] = None,
                 options: Optional[dict] = None):
        L = lib()
        if device is None:
            device = torch.cuda.current_device()
        self.capacity = int(capacity)
        self.key_bits = int(key_bits)
        self.pairs = bool(pairs)
        self.radix_bits = int(radix_bits)
        self.device = int(device)
        kt = GRS_KEY_U32 if key_bits == 32 else GRS_KEY_U64
        if key_bits not in (32, 64):
            raise ValueError("key_bits must be 32 or 64")
        h = ctypes.c_void_p()
        check(L.grs_create(ctypes.byref(h), self.capacity, kt, int(self.pairs), self.radix_bits,
                           self.device), "grs_create")
        self._h = h
        for name, value in (options or {}).items():
            self.set_option(name, value)

    def set_option(self, name: str, value) -> None:
        """Pin a kernel choice the defaults make by size (grs_set_option): name is one of
        _lib.OPTIONS ("tile", "xl", "pass", "records", "rank", "sharded_path", "sharded_send",
        "exchange", "merge"), value an int or one of that option's value names."""
        opt, names = OPTIONS[name]
        v = names[value] if isinstance(value, str) else int(value)
        check(lib().grs_set_option(self._h, opt, v), f"grs_set_option({name}={value})")

    def get_option(self, name: str) -> int:
        v = ctypes.c_int()
        check(lib().grs_get_option(self._h, OPTIONS[name][0], ctypes.byref(v)), "grs_get_option")
        return v.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().grs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def scratch_bytes(self) -> int:
        return int(lib().grs_scratch_bytes(self._h))

    def check_guards(self) -> int:
        """Guard words of the sorter's scratch that a kernel overwrote since the last check
        (grs_debug_check_guards; synchronises the device, restores them): 0 expected."""
        bad = ctypes.c_uint64()
        check(lib().grs_debug_check_guards(self._h, ctypes.byref(bad)), "grs_debug_check_guards")
        return int(bad.value)

    def msd_flags(self) -> dict:
        """What the last sort did in the MSD schedule (grs_debug_msd_flags; synchronises):
        p1_redo (P1 ran twice), p2_exact (P2 took the exact path), top_shift (the top digit's
        shift).  GrsError when the last sort took the LSD passes."""
        f = (ctypes.c_uint32 * 3)()
        check(lib().grs_debug_msd_flags(self._h, f), "grs_debug_msd_flags")
        return {"p1_redo": bool(f[0]), "p2_exact": bool(f[1]), "top_shift": int(f[2])}

    @property
    def rank_mode(self) -> str:
        """'atomic' (lane-ordered LDS atomics, the default) or 'match' (ballot fallback)."""
        return {0: "atomic", 1: "match"}[int(lib().grs_rank_mode(self._h))]

    @property
    def pass_kernel(self) -> str:
        """Name of the pass kernel a sort() of `capacity` items launches (roofline reports)."""
        return self.pass_kernel_for(self.capacity)

    def pass_kernel_for(self, n: int) -> str:
        """Name of the pass kernel a sort() of n items launches (grs_pass_kernel)."""
        return lib().grs_pass_kernel(self._h, int(n)).decode()

    def _check_keys(self, keys: torch.Tensor, vals: Optional[torch.Tensor]) -> None:
        if not keys.is_cuda or not keys.is_contiguous():
            raise ValueError("keys must be a contiguous device tensor")
        if keys.element_size() * 8 != self.key_bits:
            raise ValueError(f"keys must be {self.key_bits}-bit")
        if self.pairs:
            if vals is None or vals.numel() < keys.numel() or vals.element_size() != 4 \
                    or not vals.is_contiguous() or not vals.is_cuda:
                raise ValueError("pairs sorter needs a contiguous 32-bit device payload tensor")
        elif vals is not None:
            raise ValueError("this sorter was created without a payload")

    @staticmethod
    def _check_n(n: Optional[int], *tensors: Optional[torch.Tensor]) -> int:
        """n defaults to the first tensor's length; every given tensor must hold n items
        (libgrs cannot see tensor extents: a larger n would read and write past them)."""
        n = tensors[0].numel() if n is None else int(n)
        if n < 0:
            raise ValueError("n must be >= 0")
        for t in tensors:
            if t is not None and t.numel() < n:
                raise ValueError(f"n = {n} exceeds a tensor of {t.numel()} items")
        return n

    def sort(self, keys: torch.Tensor, vals: Optional[torch.Tensor] = None, n: Optional[int] = None,
             begin_bit: int = 0, end_bit: Optional[int] = None,
             stream: Optional[torch.cuda.Stream] = None) -> None:
        """Sort keys[:n] (and vals[:n]) in place, stably, on `stream` (default: current).
        Asynchronous: call check_error(stream) to surface a look-back timeout."""
        self._check_keys(keys, vals)
        n = self._check_n(n, keys, vals)
        end_bit = self.key_bits if end_bit is None else int(end_bit)
        vp = _ptr(vals) if vals is not None else ctypes.c_void_p(0)
        check(lib().grs_sort_bits(self._h, _ptr(keys), vp, n, int(begin_bit), end_bit,
                                  _stream_ptr(stream)), "grs_sort")

    def partition(self, keys: torch.Tensor, keys_out: torch.Tensor, splitters, counts: torch.Tensor,
                  vals: Optional[torch.Tensor] = None, vals_out: Optional[torch.Tensor] = None,
                  n: Optional[int] = None, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Stable key-range partition (grs_partition): bucket(k) = #splitters <= k; buckets
        land contiguously in keys_out (and vals_out); bucket sizes -> counts (device u32)."""
        import numpy as np

        self._check_keys(keys, vals)
        if not keys_out.is_cuda or not keys_out.is_contiguous() or keys_out.element_size() != keys.element_size():
            raise ValueError("keys_out must be a contiguous device tensor of the key width")
        if not counts.is_cuda or counts.element_size() != 4 or not counts.is_contiguous():
            raise ValueError("counts must be a contiguous 32-bit device tensor")
        n = self._check_n(n, keys, vals, keys_out, vals_out)
        sp = np.ascontiguousarray(np.asarray(splitters, dtype=np.uint32 if self.key_bits == 32
                                             else np.uint64))
        if counts.numel() < sp.size + 1:
            raise ValueError("counts needs len(splitters) + 1 entries")
        if self.pairs and (vals_out is None or not vals_out.is_cuda or not vals_out.is_contiguous()
                           or vals_out.element_size() != 4):
            raise ValueError("pairs partition needs a contiguous 32-bit device vals_out")
        vp = _ptr(vals) if vals is not None else ctypes.c_void_p(0)
        vo = _ptr(vals_out) if vals_out is not None else ctypes.c_void_p(0)
        check(lib().grs_partition(self._h, _ptr(keys), vp, _ptr(keys_out), vo, n,
                                  ctypes.c_void_p(sp.ctypes.data), int(sp.size), _ptr(counts),
                                  _stream_ptr(stream)), "grs_partition")

    def partition_regions(self, keys: torch.Tensor, keys_out: torch.Tensor, splitters, counts: torch.Tensor,
                          region: int, thresholds=None, vals: Optional[torch.Tensor] = None,
                          vals_out: Optional[torch.Tensor] = None, n: Optional[int] = None,
                          stream: Optional[torch.cuda.Stream] = None) -> None:
        """The same partition into regions (grs_partition_regions, the exchange's send step):
        bucket b from keys_out[b * region] on, no bucket histogram; keys_out (and vals_out) hold
        len(splitters) * region + n items; a count > region means that bucket ran on into the
        next region.  thresholds: shard-local index thresholds (ties by position), default 0."""
        import numpy as np

        self._check_keys(keys, vals)
        n = keys.numel() if n is None else int(n)
        sp = np.ascontiguousarray(np.asarray(splitters, dtype=np.uint32 if self.key_bits == 32
                                             else np.uint64))
        th = np.ascontiguousarray(np.zeros(sp.size, np.uint32) if thresholds is None
                                  else np.asarray(thresholds, dtype=np.uint32))
        need = sp.size * int(region) + n
        if (not keys_out.is_cuda or not keys_out.is_contiguous() or keys_out.numel() < need
                or keys_out.element_size() != keys.element_size()):
            raise ValueError(f"keys_out must be a contiguous device tensor of >= {need} keys")
        if self.pairs and (vals_out is None or vals_out.numel() < need or not vals_out.is_contiguous()):
            raise ValueError(f"pairs partition needs a contiguous vals_out of >= {need} items")
        if counts.numel() < sp.size + 1 or counts.element_size() != 4:
            raise ValueError("counts needs len(splitters) + 1 32-bit entries")
        vp = _ptr(vals) if vals is not None else ctypes.c_void_p(0)
        vo = _ptr(vals_out) if vals_out is not None else ctypes.c_void_p(0)
        check(lib().grs_partition_regions(self._h, _ptr(keys), vp, _ptr(keys_out), vo, n,
                                          ctypes.c_void_p(sp.ctypes.data), ctypes.c_void_p(th.ctypes.data),
                                          int(sp.size), int(region), _ptr(counts), _stream_ptr(stream)),
              "grs_partition_regions")

    def sort_host(self, keys, vals=None, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Sort host numpy arrays in place through device staging (grs_sort_host; BASELINE C1
        plumbing, PCIe both ways).  keys: uint32/uint64 numpy array; vals: uint32 or None."""
        import numpy as np

        if not isinstance(keys, np.ndarray) or not keys.flags.c_contiguous \
                or keys.dtype.itemsize * 8 != self.key_bits:
            raise ValueError(f"keys must be a contiguous {self.key_bits}-bit numpy array")
        if (vals is not None) != self.pairs:
            raise ValueError("payload presence must match the sorter")
        if vals is not None and (vals.dtype.itemsize != 4 or vals.size < keys.size
                                 or not vals.flags.c_contiguous):
            raise ValueError("vals must be a contiguous 32-bit numpy array")
        kp = ctypes.c_void_p(keys.ctypes.data)
        vp = ctypes.c_void_p(vals.ctypes.data) if vals is not None else ctypes.c_void_p(0)
        check(lib().grs_sort_host(self._h, kp, kp, vp, vp, keys.size, _stream_ptr(stream)),
              "grs_sort_host")

    def sort_segmented(self, keys: torch.Tensor, offsets: torch.Tensor,
                       vals: Optional[torch.Tensor] = None, n: Optional[int] = None,
                       stream: Optional[torch.cuda.Stream] = None) -> None:
        """Sort every segment [offsets[s], offsets[s+1]) of keys[:n] (and vals) on its own,
        stably, in place (grs_sort_segmented).  offsets: device u32/i32 tensor of
        num_segments + 1 non-decreasing entries, offsets[0] = 0, offsets[-1] = n.  Needs a
        sorter built with pairs=True (the payload slot carries the input index)."""
        if not self.pairs:
            raise ValueError("sort_segmented needs a sorter created with pairs=True")
        if not keys.is_cuda or not keys.is_contiguous() or keys.element_size() * 8 != self.key_bits:
            raise ValueError(f"keys must be a contiguous {self.key_bits}-bit device tensor")
        if not offsets.is_cuda or not offsets.is_contiguous() or offsets.element_size() != 4:
            raise ValueError("offsets must be a contiguous 32-bit device tensor")
        if vals is not None and (not vals.is_cuda or not vals.is_contiguous()
                                 or vals.element_size() != 4):
            raise ValueError("vals must be a contiguous 32-bit device tensor")
        n = self._check_n(n, keys, vals)
        if offsets.numel() < 2:
            raise ValueError("offsets needs num_segments + 1 >= 2 entries")
        vp = _ptr(vals) if vals is not None else ctypes.c_void_p(0)
        check(lib().grs_sort_segmented(self._h, _ptr(keys), vp, n, _ptr(offsets),
                                       offsets.numel() - 1, _stream_ptr(stream)),
              "grs_sort_segmented")

    def set_profiling(self, ring: int) -> None:
        """Keep per-phase hipEvent timings of the last `ring` sort calls (0 = off)."""
        check(lib().grs_set_profiling(self._h, int(ring)), "grs_set_profiling")

    def timing(self, k: int = 0) -> dict:
        """Per-phase GPU ms of the k-th most recent profiled call (synchronises)."""
        t = grs_timing()
        check(lib().grs_timing_history(self._h, int(k), ctypes.byref(t)), "grs_timing_history")
        return {"passes": t.passes, "total_ms": t.total_ms, "hist_ms": t.hist_ms,
                "pass_ms": list(t.pass_ms)[: t.passes], "copy_ms": t.copy_ms,
                "kind": {1: "msd", 2: "fused"}.get(t.kind, "lsd")}

    def check_error(self, stream: Optional[torch.cuda.Stream] = None, device_wide: bool = False) -> None:
        """Raise GrsError(GRS_ETIMEOUT) if a look-back spin of an earlier call gave up.
        Synchronises `stream` (default: current; grs_stream_check_error), or the whole device
        with device_wide=True (grs_check_error)."""
        if device_wide:
            check(lib().grs_check_error(self._h), "grs_check_error")
        else:
            check(lib().grs_stream_check_error(self._h, _stream_ptr(stream)), "grs_stream_check_error")


# ---- boundary helpers -----------------------------------------------------------------

def fill_splitmix(out: torch.Tensor, seed: int, first_index: int = 0,
                  stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """key[i] = splitmix64(seed ^ (first_index + i)) truncated to out's width (device)."""
    check(lib().grs_fill_splitmix(_ptr(out), out.numel(), out.element_size(),
                                  seed & (2**64 - 1), first_index, _stream_ptr(stream)),
          "grs_fill_splitmix")
    return out


def fill_permutation(out: torch.Tensor, seed: int, total: Optional[int] = None, first_index: int = 0,
                     stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """The reference's own input (main.cpp:119-125: 0..N-1 shuffled): out[i] = pi(first_index + i)
    for a seeded bijection pi of [0, total) (total defaults to out.numel()), on the device."""
    total = out.numel() if total is None else int(total)
    check(lib().grs_fill_permutation(_ptr(out), out.numel(), out.element_size(), total,
                                     seed & (2**64 - 1), first_index, _stream_ptr(stream)),
          "grs_fill_permutation")
    return out


def iota_u32(out: torch.Tensor, start: int = 0, stream=None) -> torch.Tensor:
    check(lib().grs_iota_u32(_ptr(out), out.numel(), start, _stream_ptr(stream)), "grs_iota_u32")
    return out


def gather_records(src: torch.Tensor, dst: torch.Tensor, idx: torch.Tensor, n: int,
                   record_bytes: int, stream=None) -> torch.Tensor:
    check(lib().grs_gather_records(_ptr(src), _ptr(dst), _ptr(idx), n, record_bytes,
                                   _stream_ptr(stream)), "grs_gather_records")
    return dst


def count_inversions(keys: torch.Tensor, n: Optional[int] = None, stream=None) -> int:
    n = keys.numel() if n is None else n
    out = ctypes.c_uint64()
    check(lib().grs_count_inversions(_ptr(keys), n, keys.element_size(), ctypes.byref(out),
                                     _stream_ptr(stream)), "grs_count_inversions")
    return int(out.value)


KEYS_UNSIGNED, KEYS_SIGNED, KEYS_FLOAT = 0, 1, 2
_KINDS = {torch.int32: KEYS_SIGNED, torch.int64: KEYS_SIGNED, torch.float32: KEYS_FLOAT,
          torch.float64: KEYS_FLOAT, torch.uint32: KEYS_UNSIGNED, torch.uint64: KEYS_UNSIGNED}


def key_transform(keys: torch.Tensor, inverse: bool = False, kind: Optional[int] = None,
                  stream=None) -> torch.Tensor:
    """Order-preserving bit transform in place (grs_key_transform) so signed / float keys sort
    as unsigned: kind defaults from keys.dtype (int -> signed, float -> IEEE-754)."""
    k = _KINDS[keys.dtype] if kind is None else int(kind)
    check(lib().grs_key_transform(_ptr(keys), keys.numel(), keys.element_size(), k, int(inverse),
                                  _stream_ptr(stream)), "grs_key_transform")
    return keys


def exclusive_scan_u32(inp: torch.Tensor, out: Optional[torch.Tensor] = None,
                       total: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """Device-wide exclusive prefix sum of uint32 (mod 2^32), one launch (grs_exclusive_scan_u32);
    out may be inp (in place); total (device, >= 1 word) receives the sum of all items."""
    if inp.element_size() != 4 or not inp.is_cuda or not inp.is_contiguous():
        raise ValueError("scan input must be a contiguous 32-bit device tensor")
    out = torch.empty_like(inp) if out is None else out
    n = inp.numel()
    L = lib()
    scratch = torch.empty(max(1, (L.grs_scan_scratch_bytes(n) + 3) // 4), dtype=torch.int32,
                          device=inp.device)
    tp = _ptr(total) if total is not None else ctypes.c_void_p(0)
    check(L.grs_exclusive_scan_u32(_ptr(inp), _ptr(out), n, tp, _ptr(scratch),
                                   scratch.numel() * 4, _stream_ptr(stream)),
          "grs_exclusive_scan_u32")
    check(L.grs_scan_check_error(_ptr(scratch), _stream_ptr(stream)), "grs_scan_check_error")
    return out
