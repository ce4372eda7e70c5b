"""Multi-GPU sort: one process per GPU, key-range sharding with ONE all-to-all exchange.

New with respect to the reference (which is single-context).  Input: each
rank r holds a contiguous shard of the global input (the global range that follows ranks < r).
Output: rank r holds a contiguous, sorted range of the global stable order; the concatenation
over ranks in rank order equals the stable sort of the whole input.

All of it runs in libgrs's C-ABI entry point grs_sort_sharded (include/grs.h) on an RCCL
communicator that libgrs owns (RcclComm below; a C++ caller passes its own ncclComm_t).

u32 keys without payload take the PRESORTED exchange (grs_codec.hpp): local sort first, then
samples / splitters of the sorted shard, each bucket encoded as bit-packed deltas (about a
byte per key instead of four), the encoded words exchanged, decoded and merged.  The same
steps are exported for other transports (shard_sample / shard_encode / shard_decode_merge
below; the one-device simulation of tests/test_gpu_presorted.py uses them).

Other key types take the PARTITION-FIRST exchange:
  1. samples     S regularly spaced (key, position) samples of the shard, RCCL all-gather
  2. splitters   on the device: the G*S samples sorted by (key, global index) in one
                 workgroup, G-1 quantiles -> this rank's partition digit; ties are broken by
                 global index, so equal keys split evenly across ranks
  3. partition   the grs pass kernel with the splitter digit: G contiguous send buckets
  4. counts      RCCL all-gather of the G x G bucket counts -> the ONE host synchronisation
  5. exchange    grouped ncclSend / ncclRecv of keys and payload (xGMI: one link per peer)
  6. local sort  grs_sort of the received run, which arrived in source-rank order = global
                 input order for equal keys, so the result is the global stable order

torch.distributed only carries the 128-byte RCCL id from rank 0 to the others.  The CPU tests
run the same orchestration under gloo (tests/sharded_sim.py) with libgrs's host twins of the
splitter and plan arithmetic (grs_shard_splitters_host, grs_shard_plan_host).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from ._lib import GRS_RCCL_ID_BYTES, check, lib
from .sorter import RadixSorter, _ptr, _stream_ptr


class RcclComm:
    """An RCCL communicator over the ranks of a torch.distributed group, one rank per GPU,
    created by libgrs (grs_rccl_comm_init); `handle` is the ncclComm_t."""

    def __init__(self, group=None, device: Optional[int] = None):
        L = lib()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.cuda.current_device() if device is None else int(device)
        idbuf = ctypes.create_string_buffer(GRS_RCCL_ID_BYTES)
        if self.rank == 0:
            check(L.grs_rccl_unique_id(idbuf), "grs_rccl_unique_id")
        obj = [bytes(idbuf.raw) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group else 0,
                                   group=group)
        idbuf = ctypes.create_string_buffer(obj[0], GRS_RCCL_ID_BYTES)
        h = ctypes.c_void_p()
        check(L.grs_rccl_comm_init(ctypes.byref(h), idbuf, self.world, self.rank, self.device),
              "grs_rccl_comm_init")
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().grs_rccl_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedSorter:
    """Stable sort of a key (+ uint32 payload) array sharded over the ranks of `group`
    (grs_sort_sharded).  capacity_local bounds this rank's input; the received run may be
    larger on skewed inputs: recv_slack sizes the output buffer (and the sorter) for it."""

    def __init__(self, capacity_local: int, key_bits: int = 32, pairs: bool = False,
                 radix_bits: int = 8, group=None, device: Optional[torch.device] = None,
                 recv_slack: float = 1.25, comm: Optional[RcclComm] = None,
                 options: Optional[dict] = None):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.key_bits = key_bits
        self.pairs = pairs
        self.comm = comm if comm is not None else RcclComm(group, device.index)
        self.world = self.comm.world
        self.rank = self.comm.rank
        if self.world > 16:
            raise ValueError("grs_sort_sharded supports at most 16 ranks per exchange")
        self.cap = int(capacity_local)
        self.out_cap = max(int(self.cap * recv_slack), self.cap, 1)
        self.sorter = RadixSorter(self.out_cap, key_bits=key_bits, pairs=pairs,
                                  radix_bits=radix_bits, device=device.index, options=options)
        kdt = torch.uint32 if key_bits == 32 else torch.uint64
        self.out_k = torch.empty(self.out_cap, dtype=kdt, device=device)
        self.out_v = torch.empty(self.out_cap, dtype=torch.uint32, device=device) if pairs else None
        self.last_n_out = 0

    def sort(self, keys: torch.Tensor, vals: Optional[torch.Tensor] = None,
             n: Optional[int] = None, stream: Optional[torch.cuda.Stream] = None, check_error=True):
        """Returns (keys_out, vals_out): views of this rank's sorted output range (valid until
        the next call).  check_error=True synchronises the stream once more to surface a
        look-back timeout of the local sort (the exchange itself already synchronised)."""
        self.sorter._check_keys(keys, vals)
        n = RadixSorter._check_n(n, keys, vals)
        if n > self.cap:
            raise ValueError("shard exceeds capacity_local")
        n_out = ctypes.c_size_t(0)
        vp = _ptr(vals) if vals is not None else ctypes.c_void_p(0)
        vo = _ptr(self.out_v) if self.pairs else ctypes.c_void_p(0)
        check(lib().grs_sort_sharded(self.sorter._h, _ptr(keys), vp, n, _ptr(self.out_k), vo,
                                     self.out_cap, ctypes.byref(n_out), self.comm.handle,
                                     _stream_ptr(stream)), "grs_sort_sharded")
        if check_error:
            self.sorter.check_error(stream)
        self.last_n_out = int(n_out.value)
        m = self.last_n_out
        return self.out_k[:m], (self.out_v[:m] if self.pairs else None)

    # ---- bench plumbing ---------------------------------------------------------------------
    def set_profiling(self, ring: int) -> None:
        self.sorter.set_profiling(ring)

    def timing(self, k: int = 0) -> dict:
        return self.sorter.timing(k)

    def exchange_timing(self) -> dict:
        """Phases of the last multi-rank sort() (profiling on; grs_sharded_last_timing): ms
        before / of / after the exchange and the bytes that crossed the links."""
        from ._lib import grs_sharded_timing

        t = grs_sharded_timing()
        check(lib().grs_sharded_last_timing(self.sorter._h, ctypes.byref(t)), "grs_sharded_last_timing")
        return {"total_ms": t.total_ms, "before_ms": t.before_ms, "exchange_ms": t.exchange_ms,
                "after_ms": t.after_ms, "bytes_sent": int(t.bytes_sent),
                "bytes_received": int(t.bytes_received),
                "exchange": "presorted" if t.presorted else "partition-first"}

    def redo_count(self) -> int:
        """Partition-first calls redone into contiguous buckets after a region spill."""
        c = ctypes.c_uint64()
        check(lib().grs_sharded_redo_count(self.sorter._h, ctypes.byref(c)), "grs_sharded_redo_count")
        return int(c.value)

    def count_inversions(self) -> int:
        from .sorter import count_inversions

        return count_inversions(self.out_k[: self.last_n_out])

    def close(self) -> None:
        self.sorter.close()
        self.comm.close()


# ---- presorted-exchange steps (transport-independent; include/grs.h) --------------------------

def shard_sample(keys: torch.Tensor, n: int, samples: int,
                 stream: Optional[torch.cuda.Stream] = None):
    """S regularly spaced (key, position) samples of keys[:n] (grs_shard_sample)."""
    sk = torch.empty(samples, dtype=keys.dtype, device=keys.device)
    sp = torch.empty(samples, dtype=torch.uint32, device=keys.device)
    check(lib().grs_shard_sample(_ptr(keys), int(n), keys.element_size(), int(samples), _ptr(sk),
                                 _ptr(sp), _stream_ptr(stream)), "grs_shard_sample")
    return sk, sp


def shard_encode(sorter: RadixSorter, sorted_keys: torch.Tensor, n: int, gathered_keys: torch.Tensor,
                 gathered_pos: torch.Tensor, nranks: int, rank: int,
                 stream: Optional[torch.cuda.Stream] = None):
    """Encode the G buckets of a sorted u32 shard (grs_shard_encode).  Returns (send, sizes):
    send holds the buckets back to back (u32 words), sizes[2b] / [2b+1] bucket b's keys / words."""
    if sorted_keys.element_size() != 4 or sorted_keys.numel() < n:
        raise ValueError("sorted_keys: a u32 device tensor of >= n keys")
    L = lib()
    cap = int(L.grs_shard_encode_words_max(int(n), int(nranks)))
    send = torch.empty(max(cap, 1), dtype=torch.uint32, device=sorted_keys.device)
    sizes = torch.empty(2 * nranks, dtype=torch.uint32, device=sorted_keys.device)
    check(L.grs_shard_encode(sorter._h, _ptr(sorted_keys), int(n), _ptr(gathered_keys),
                             _ptr(gathered_pos), int(nranks), int(rank), _ptr(send), cap,
                             _ptr(sizes), _stream_ptr(stream)), "grs_shard_encode")
    return send, sizes


def shard_decode_merge(sorter: RadixSorter, recv: torch.Tensor, word_offsets, lens,
                       out: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> int:
    """Decode the received runs (source p: lens[p] keys at recv[word_offsets[p]:]) and merge them
    into out (grs_shard_decode_merge); returns the number of keys written."""
    g = len(lens)
    wo = (ctypes.c_uint64 * g)(*[int(x) for x in word_offsets])
    ln = (ctypes.c_uint32 * g)(*[int(x) for x in lens])
    check(lib().grs_shard_decode_merge(sorter._h, _ptr(recv), g, wo, ln, _ptr(out), out.numel(),
                                       _stream_ptr(stream)), "grs_shard_decode_merge")
    return int(sum(int(x) for x in lens))
