"""Multi-GPU sort: one process per GPU, key-range sharding with ONE all-to-all-v exchange.

New with respect to the reference (which is single-context).  Input: each
rank r holds a contiguous shard of the global input (global indices [r*n, (r+1)*n) in rank
order).  Output: rank r holds a contiguous, sorted range of the global stable order; the
concatenation over ranks in rank order equals the stable sort of the whole input.

Per call:
  1. splitters  every rank contributes `oversample` regularly spaced keys of its shard;
                one all_gather; every rank sorts the G*oversample samples on the host
                (tiny) and picks the same G-1 quantiles as splitters
  2. partition  grs_partition: stable key-range partition into G contiguous send buckets
                (bucket = number of splitters <= key, monotone in the key)
  3. counts     all_to_all of the G bucket sizes -> receive sizes (one D2H sync)
  4. exchange   all_to_all_single of the keys (and payload) -- on the "nccl" backend this is
                RCCL over xGMI, every peer pair on its own link
  5. local sort the received buckets are concatenated in SOURCE-RANK order, i.e. global
                input order for equal keys; the stable LSD sort then gives the global stable
                order (ties broken by global index, exactly the reference's order)

Correctness does not depend on the splitters (any non-decreasing splitters give the right
global order); they only set the balance.  Equal keys never straddle two ranks.

The device steps go through an `ops` object: HipOps (libgrs, the only production path) by
default.  tests/ substitute a numpy implementation to run the orchestration under `gloo`
on CPU; the collective pattern is identical.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist


class HipOps:
    """Device steps on libgrs (HIP, gfx950)."""

    def __init__(self, capacity: int, key_bits: int, pairs: bool, radix_bits: int, device):
        from .sorter import RadixSorter

        self.device = device
        self.key_bits = key_bits
        self.pairs = pairs
        self.radix_bits = radix_bits
        self.part = RadixSorter(capacity, key_bits=key_bits, pairs=pairs, radix_bits=radix_bits,
                                device=device.index)
        self.local = None
        self.local_cap = 0

    def partition(self, keys, vals, keys_out, vals_out, splitters, counts):
        self.part.partition(keys, keys_out, splitters, counts, vals, vals_out)

    def local_sort(self, keys, vals, n):
        if self.local is None or self.local_cap < n:
            if self.local is not None:
                self.local.close()
            self.local_cap = max(n, 1)
            from .sorter import RadixSorter

            self.local = RadixSorter(self.local_cap, key_bits=self.key_bits, pairs=self.pairs,
                                     radix_bits=self.radix_bits, device=self.device.index)
            if getattr(self, "_ring", 0):
                self.local.set_profiling(self._ring)
        self.local.sort(keys, vals, n=n)

    def set_profiling(self, ring):
        self._ring = ring
        if self.local is not None:
            self.local.set_profiling(ring)

    def timing(self, k=0):
        return self.local.timing(k)

    def count_inversions(self, keys):
        from .sorter import count_inversions

        return count_inversions(keys)


def _comm_view(t: torch.Tensor) -> torch.Tensor:
    """Collectives move bytes: view unsigned keys as the signed type of the same width."""
    if t.dtype == torch.uint32:
        return t.view(torch.int32)
    if t.dtype == torch.uint64:
        return t.view(torch.int64)
    return t


class ShardedSorter:
    """Stable sort of a key (+ uint32 payload) array sharded over the ranks of `group`."""

    def __init__(self, capacity_local: int, key_bits: int = 32, pairs: bool = False,
                 radix_bits: int = 8, group=None, device: Optional[torch.device] = None,
                 oversample: int = 1024, recv_slack: float = 1.25, ops=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.key_bits = key_bits
        self.pairs = pairs
        self.oversample = int(oversample)
        if self.world - 1 > 15:
            raise ValueError("grs_partition supports at most 16 ranks per exchange")
        self.kdt = torch.uint32 if key_bits == 32 else torch.uint64
        self.ndt = np.uint32 if key_bits == 32 else np.uint64
        self.ops = ops if ops is not None else HipOps(capacity_local, key_bits, pairs, radix_bits,
                                                      device)
        self.cap = int(capacity_local)
        self.send_k = torch.empty(max(self.cap, 1), dtype=self.kdt, device=device)
        self.send_v = torch.empty(max(self.cap, 1), dtype=torch.uint32, device=device) if pairs else None
        self.recv_cap = max(int(self.cap * recv_slack), 1)
        self.recv_k = torch.empty(self.recv_cap, dtype=self.kdt, device=device)
        self.recv_v = torch.empty(self.recv_cap, dtype=torch.uint32, device=device) if pairs else None
        self.counts = torch.zeros(self.world, dtype=torch.uint32, device=device)
        self.last_local_n = 0
        self.last_send_counts = None
        self.last_recv_counts = None

    # ---- step 1 ---------------------------------------------------------------------------
    def splitters(self, keys: torch.Tensor, n: int) -> np.ndarray:
        G, S = self.world, self.oversample
        if n > 0:
            idx = (torch.arange(S, device=keys.device, dtype=torch.int64) * n) // S
            local = _comm_view(keys[:n]).index_select(0, idx)
        else:   # an empty shard contributes max keys (they only bias the top splitter)
            local = torch.full((S,), -1, dtype=_comm_view(keys[:0]).dtype, device=keys.device)
        gathered = torch.empty(G * S, dtype=local.dtype, device=keys.device)
        dist.all_gather_into_tensor(gathered, local.contiguous(), group=self.group)
        samples = np.sort(gathered.cpu().numpy().view(self.ndt))
        q = (np.arange(1, G, dtype=np.int64) * samples.size) // G
        return samples[q]

    # ---- steps 2-5 ------------------------------------------------------------------------
    def sort(self, keys: torch.Tensor, vals: Optional[torch.Tensor] = None,
             n: Optional[int] = None, splitters=None):
        """Returns (keys_out, vals_out) views of this rank's sorted output range."""
        n = keys.numel() if n is None else int(n)
        if n > self.cap:
            raise ValueError("shard exceeds capacity_local")
        if (vals is not None) != self.pairs:
            raise ValueError("payload presence must match the sorter")
        sp = self.splitters(keys, n) if splitters is None else np.asarray(splitters, self.ndt)
        self.ops.partition(keys, vals, self.send_k, self.send_v, sp, self.counts)

        send_counts = self.counts.to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc = send_counts.cpu().tolist()   # the one host sync of the call
        rc = recv_counts.cpu().tolist()
        n_out = int(sum(rc))
        if n_out > self.recv_cap:          # skewed input: grow the receive buffers
            self.recv_cap = int(n_out * 1.1) + 1
            self.recv_k = torch.empty(self.recv_cap, dtype=self.kdt, device=self.device)
            if self.pairs:
                self.recv_v = torch.empty(self.recv_cap, dtype=torch.uint32, device=self.device)
        dist.all_to_all_single(_comm_view(self.recv_k[:n_out]), _comm_view(self.send_k[:n]),
                               output_split_sizes=rc, input_split_sizes=sc, group=self.group)
        if self.pairs:
            dist.all_to_all_single(_comm_view(self.recv_v[:n_out]), _comm_view(self.send_v[:n]),
                                   output_split_sizes=rc, input_split_sizes=sc, group=self.group)
        self.ops.local_sort(self.recv_k, self.recv_v, n_out)
        self.last_local_n = n_out
        self.last_send_counts, self.last_recv_counts = sc, rc
        return self.recv_k[:n_out], (self.recv_v[:n_out] if self.pairs else None)

    # ---- bench plumbing ---------------------------------------------------------------------
    def set_profiling(self, ring: int) -> None:
        self.ops.set_profiling(ring)

    def timing(self, k: int = 0) -> dict:
        return self.ops.timing(k)

    def count_inversions(self, _keys=None) -> int:
        return self.ops.count_inversions(self.recv_k[: self.last_local_n])

    def phase_summary(self) -> dict:
        return {"recv_keys_this_rank": self.last_local_n,
                "send_counts": self.last_send_counts, "recv_counts": self.last_recv_counts}
