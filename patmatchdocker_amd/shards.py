r"""Sharding of a sequence database over the GPUs of one node + hit gather.

The reference scans one file with one CPU process per strand
(``www/FlaskApp/FlaskApp/patmatch.py:733-743``).  Here the database is cut
into contiguous runs of whole records, one run per GPU (one process per
GPU, ``torch.distributed`` over RCCL/xGMI).  Every rank scans only its own
records -- there is no data-path collective -- and the (small) hit lists
are gathered once per query: counts first, then the padded key and length
vectors with one ``all_gather`` each, then an O(n) merge (ranks own
increasing position ranges, so each pattern's hits are the ranks' sorted
slices in rank order).  Keys are ``pattern << 48 | global_beg``, so the
result is exactly the single-GPU order.

Real files (:class:`ShardedDatabase`, :func:`scan_sharded`): the file is cut
at header lines (``/^>\S/``, ``generate_sequence_index.pl:33-38``) into
``world`` byte ranges of about equal size; each rank holds its range plus a
short halo in HBM and reports hits in file offsets.  Only one thing couples
the pieces: nrgrep's report rule (a match is printed, the scan resumes at its
end) -- the simple engine's windows (k = 0, a class accepting
'\n') may run from one record into the next, so a report that crosses a cut
moves the next piece's resume point.  The pieces exchange the end of their
last report (one small all_gather); a piece entered past its start re-chains
its candidates from that point (rare: only such cross-line windows reach past
a cut), so the result equals the single-process scan byte for byte.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
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


def gather_hits(keys: torch.Tensor, lens: torch.Tensor, group=None, dst: Optional[int] = 0
                ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """All ranks' (keys, lens) -> sorted (keys, lens) on rank ``dst``
    (``dst=None``: on every rank).

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
    if dst is not None and dist.get_rank(group) != dst:
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


# ---------------------------------------------------------------------------
# real FASTA files: record-aligned pieces, one per rank
# ---------------------------------------------------------------------------

HALO = 4096   # bytes held past a piece's end: >= any window that can cross a cut (<= 64 positions)
_SPACE = np.frombuffer(b" \t\n\r\f\x0b", dtype=np.uint8)


def header_lines(data: bytes) -> Tuple[np.ndarray, np.ndarray]:
    """(start, end) of every header line: '>' at a line start followed by a
    non-space (``/^>(\\S+)/``, generate_sequence_index.pl:33); end = the
    offset of its '\\n' (or len(data))."""
    arr = np.frombuffer(data, dtype=np.uint8)
    gt = np.flatnonzero(arr == ord(">"))
    if gt.size:
        at_line = (gt == 0) | (arr[np.maximum(gt - 1, 0)] == 10)
        nxt = gt + 1
        named = nxt < arr.size
        named[named] = ~np.isin(arr[nxt[named]], _SPACE)
        gt = gt[at_line & named]
    nl = np.flatnonzero(arr == 10)
    i = np.searchsorted(nl, gt)
    ends = np.full(gt.size, arr.size, dtype=np.int64)
    has = i < nl.size
    ends[has] = nl[i[has]]
    return gt.astype(np.int64), ends


def split_fasta(data: bytes, world: int) -> List[Tuple[int, int]]:
    """``world`` contiguous byte ranges covering ``data``, cut only at header
    lines, of about equal size (a range may be empty: fewer records than
    ranks)."""
    n = len(data)
    starts, _ = header_lines(data)
    cuts = [0]
    for i in range(1, world):
        j = int(np.searchsorted(starts, (n * i) // world))
        cut = int(starts[j]) if j < starts.size else n
        cuts.append(max(cut, cuts[-1]))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def drop_header_starts(beg: np.ndarray, end: np.ndarray, hs: np.ndarray, he: np.ndarray):
    """Remove hits starting on a header line, its '\\n' included (what
    process_output discards, patmatch.py:548-550)."""
    if beg.size == 0 or hs.size == 0:
        return beg, end
    i = np.searchsorted(hs, beg, side="right") - 1
    on = (i >= 0) & (beg <= he[np.maximum(i, 0)])
    return beg[~on], end[~on]


class ShardedDatabase:
    """Rank ``rank``'s piece of a FASTA file (``split_fasta``) in HBM, with
    ``HALO`` bytes of the next piece so windows that start in the piece are
    evaluated on the file's own bytes.  ``raw`` is the whole file (hit text
    and line-start checks); hit offsets are file offsets."""

    def __init__(self, data: bytes, world: int, rank: int, device: int = 0, alphabet: Optional[str] = None,
                 halo: int = HALO, open_db: bool = True):
        self.raw = data
        self.world, self.rank = world, rank
        self.ranges = split_fasta(data, world)
        self.beg, self.end = self.ranges[rank]
        self.stop = min(len(data), self.end + halo) if self.end > self.beg else self.end
        hs, he = header_lines(data[self.beg:self.end])
        self.headers = (hs, he)
        self.db = None
        if open_db and self.stop > self.beg:
            from . import engine
            self.db = engine.SequenceDatabase.from_bytes(data[self.beg:self.stop],
                                                         alphabet or engine.choose_alphabet(data), device)

    @classmethod
    def from_file(cls, path: str, world: int, rank: int, device: int = 0) -> "ShardedDatabase":
        with open(path, "rb") as fh:
            return cls(fh.read(), world, rank, device)

    def __len__(self):
        return self.end - self.beg

    def scanner(self):
        return _EngineScanner(self.db)

    def close(self):
        if self.db is not None:
            self.db.close()
            self.db = None


class _EngineScanner:
    """The two scans :func:`scan_sharded` needs, on the GPU engine (local
    offsets of the piece's database)."""

    def __init__(self, db):
        self.db = db

    def reported(self, progs, k, types):
        """What nrgrep_coords reports, header-line starts kept."""
        from . import engine
        return engine.scan(self.db, progs, k=k, types=types, keep_headers=True)[0]

    def candidates(self, prog, k, types):
        """Every start with a match (shortest end; '$' applied, '^' not),
        header-line starts kept."""
        from . import engine
        return engine.scan(self.db, [prog], k=k, types=types, report=engine.REPORT_ALL, keep_headers=True,
                           start_anchor=False)[0][0]


def _coll_device(group=None) -> torch.device:
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _rechain(piece: ShardedDatabase, prog, cand, chain, R: int):
    """The piece's report chain for one program when the scan enters it at
    local offset ``R`` > 0 instead of 0: the report rule replayed over the
    candidates from R until it takes a candidate the original chain took
    (from there on the two chains agree)."""
    cb, ce = (np.asarray(x, dtype=np.int64) for x in cand)
    keep = cb < len(piece)
    cb, ce = cb[keep], ce[keep]
    ob, oe = chain
    text, base = piece.raw, piece.beg
    out_b, out_e = [], []
    i = int(np.searchsorted(cb, R))
    while i < cb.size:
        s = int(cb[i])
        if prog.anchor_start and not (s == R or s == 0 or text[base + s - 1] == 10):
            i += 1
            continue
        j = int(np.searchsorted(ob, s))
        if j < ob.size and int(ob[j]) == s:   # resynchronized
            return (np.concatenate([np.array(out_b, dtype=np.int64), ob[j:]]),
                    np.concatenate([np.array(out_e, dtype=np.int64), oe[j:]]))
        out_b.append(s)
        out_e.append(int(ce[i]))
        R = int(ce[i])
        i = int(np.searchsorted(cb, R))
    return np.array(out_b, dtype=np.int64), np.array(out_e, dtype=np.int64)


def scan_sharded(piece: ShardedDatabase, progs: Sequence, k: int = 0, types: str = "ids", group=None,
                 scanner=None) -> List[Tuple[np.ndarray, np.ndarray]]:
    """Every rank scans its piece; returns, on every rank, [(beg, end) per
    program] in file offsets -- equal to the single-process scan of the
    whole file (what nrgrep_coords reports, header-line starts dropped)."""
    scanner = scanner or piece.scanner()
    P = len(progs)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    n_local = len(piece)
    empty = (np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64))
    if n_local:
        chains = []
        for b, e in scanner.reported(progs, k, types):
            b, e = np.asarray(b, dtype=np.int64), np.asarray(e, dtype=np.int64)
            keep = b < n_local
            chains.append((b[keep], e[keep]))
    else:
        chains = [empty] * P
    if world > 1:
        # the chain state leaving each piece: the end of its last report
        dev = _coll_device(group)
        last = torch.tensor([int(e[-1]) + piece.beg if e.size else -1 for _, e in chains], dtype=torch.int64,
                            device=dev)
        rows = [torch.empty_like(last) for _ in range(world)]
        dist.all_gather(rows, last, group=group)
        state = rows[0].cpu().numpy()
        for r in range(1, world):
            beg_r = piece.ranges[r][0]
            need = [p for p in range(P) if state[p] > beg_r]
            if not need:
                state = np.maximum(state, rows[r].cpu().numpy())
                continue
            out = torch.empty_like(last)
            if r == piece.rank:
                cand_cache = {}
                for p in need:
                    if n_local:
                        cand_cache[p] = scanner.candidates(progs[p], k, types)
                        chains[p] = _rechain(piece, progs[p], cand_cache[p], chains[p], int(state[p]) - beg_r)
                mine = np.array([int(e[-1]) + piece.beg if e.size else -1 for _, e in chains], dtype=np.int64)
                out.copy_(torch.from_numpy(np.maximum(mine, state)))
            dist.broadcast(out, src=r, group=group)
            state = out.cpu().numpy()
    hs, he = piece.headers
    chains = [drop_header_starts(b, e, hs, he) for b, e in chains]
    if world == 1:
        return [(b + piece.beg, e + piece.beg) for b, e in chains]
    dev = _coll_device(group)
    keys = np.concatenate([(np.int64(p) << POS_BITS) | (b + piece.beg) for p, (b, _) in enumerate(chains)]
                          or [np.zeros(0, dtype=np.int64)])
    lens = np.concatenate([(e - b).astype(np.int32) for b, e in chains] or [np.zeros(0, dtype=np.int32)])
    gk, gl = gather_hits(torch.from_numpy(keys).to(dev), torch.from_numpy(lens).to(dev), group, dst=None)
    gk, gl = gk.cpu().numpy(), gl.cpu().numpy().astype(np.int64)
    pat = gk >> POS_BITS
    beg = gk & POS_MASK
    res = []
    for p in range(P):
        sel = pat == p
        res.append((beg[sel], beg[sel] + gl[sel]))
    return res
