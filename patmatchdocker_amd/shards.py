"""Sharding of a sequence database over the GPUs of one node + hit gather.

The reference scans one file with one CPU process per strand
(``www/FlaskApp/FlaskApp/patmatch.py:733-743``).  Here the database is cut
into contiguous runs of whole records, one run per GPU (one process per
GPU, ``torch.distributed`` over RCCL/xGMI).  Every rank scans only its own
records -- there is no data-path collective -- and the (small) hit lists
are gathered to rank 0 once per query: counts first, then the padded key and
length vectors with one ``all_gather`` each, then an O(n) merge on rank 0
(ranks own increasing position ranges, so each pattern's hits are the
ranks' sorted slices in rank order).  Keys are ``pattern << 48 |
global_beg``, so the result is exactly the single-GPU order.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

POS_BITS = 48
POS_MASK = (1 << POS_BITS) - 1


def shard_range(n_records: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous record range [first, first+count) owned by ``rank``."""
    base, extra = divmod(n_records, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def to_global(keys: torch.Tensor, offset: int) -> torch.Tensor:
    """Shift the position field of ``pattern<<48 | beg`` keys by ``offset``."""
    if offset == 0 or keys.numel() == 0:
        return keys
    return keys + offset          # the pattern field never overflows (beg + offset < 2^48)


def gather_hits(keys: torch.Tensor, lens: torch.Tensor, group=None, dst: int = 0
                ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """All ranks' (keys, lens) -> sorted (keys, lens) on rank ``dst``.

    Works with any backend (RCCL for device tensors, gloo for CPU tensors).
    Non-destination ranks return None.
    """
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return keys, lens          # one rank: the engine already sorted them
    if dist.get_backend(group) == "gloo" and keys.is_cuda:   # gloo gathers host tensors
        out = gather_hits(keys.cpu(), lens.cpu(), group, dst)
        return None if out is None else (out[0].to(keys.device), out[1].to(lens.device))
    world = dist.get_world_size(group)
    count = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count, group=group)
    sizes = [int(c.item()) for c in counts]
    width = max(max(sizes), 1)
    pk = torch.zeros(width, dtype=keys.dtype, device=keys.device)
    pl = torch.zeros(width, dtype=lens.dtype, device=lens.device)
    pk[:keys.numel()] = keys
    pl[:lens.numel()] = lens
    all_k = [torch.empty_like(pk) for _ in range(world)]
    all_l = [torch.empty_like(pl) for _ in range(world)]
    dist.all_gather(all_k, pk, group=group)
    dist.all_gather(all_l, pl, group=group)
    if dist.get_rank(group) != dst:
        return None
    parts = [t[:n] for t, n in zip(all_k, sizes)]
    k = torch.cat(parts)
    ln = torch.cat([t[:n] for t, n in zip(all_l, sizes)])
    if k.numel() == 0:
        return k, ln
    return _merge(parts, k, ln)


def _merge(parts, k, ln):
    """Rank-major concatenation -> (pattern, beg) order without a sort: each
    rank's list is sorted and ranks own increasing position ranges, so the
    output is, pattern by pattern, the ranks' pattern slices in rank order.
    Every element's destination is computed from per-(rank, pattern) counts
    (torch.searchsorted) and scattered once."""
    dev = k.device
    npat = int((k >> POS_BITS).max().item()) + 1
    bounds = torch.arange(npat + 1, device=dev, dtype=torch.int64) << POS_BITS
    start = torch.stack([torch.searchsorted(t, bounds) for t in parts])   # [world, npat + 1]
    cnt = start[:, 1:] - start[:, :-1]                                    # [world, npat]
    # destination base of (rank, pattern): all earlier patterns, then earlier ranks
    per_pat = cnt.sum(0)
    pat_base = torch.cumsum(per_pat, 0) - per_pat                         # [npat]
    rank_off = torch.cumsum(cnt, 0) - cnt                                 # [world, npat]
    base = pat_base.unsqueeze(0) + rank_off - start[:, :-1]               # dest = base[r, p] + index in rank
    sizes = torch.tensor([t.numel() for t in parts], device=dev)
    rank = torch.repeat_interleave(torch.arange(len(parts), device=dev), sizes)
    idx = torch.arange(k.numel(), device=dev) - (torch.cumsum(sizes, 0) - sizes)[rank]
    dest = base[rank, k >> POS_BITS] + idx
    out_k = torch.empty_like(k)
    out_l = torch.empty_like(ln)
    out_k[dest] = k
    out_l[dest] = ln
    return out_k, out_l


def hits_to_tensors(hits_handle, device: torch.device):
    """Device copy of a ``pm_hits`` list into torch tensors (keys int64, lens int32)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    n = ctypes.c_uint64()
    _lib.check(lib.pm_hits_count(hits_handle, ctypes.byref(n)))
    keys = torch.empty(n.value, dtype=torch.int64, device=device)
    lens = torch.empty(n.value, dtype=torch.int32, device=device)
    if n.value:
        # ordered on torch's current stream after the scan (no host sync)
        stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream) if keys.is_cuda else None
        _lib.check(lib.pm_hits_copy_device(hits_handle, keys.data_ptr(), lens.data_ptr(), n.value, stream))
    return keys, lens
