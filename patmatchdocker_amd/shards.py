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

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.utils.dlpack

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


def gather_hits(keys: torch.Tensor, lens: Optional[torch.Tensor], group=None, dst: Optional[int] = 0,
                fixed_len: Optional[Sequence[int]] = None) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """All ranks' (keys, lens) -> sorted (keys, lens) on rank ``dst``
    (``dst=None``: on every rank).

    Byte budget per query: one int64 count per rank (all_gather), then the
    count-padded key vector of every rank moves to ``dst`` only
    (``dist.gather``: (world - 1) x width x 8 bytes into dst over xGMI; with
    ``dst=None`` an all_gather sends it to every rank).  ``fixed_len[p]``:
    every hit of pattern p has that length (a class sequence searched with
    substitutions), so the length vector is not sent at all and is rebuilt
    from the pattern field.  Works with any backend (RCCL for device tensors,
    gloo for CPU tensors).  Non-destination ranks return None.
    """
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        if lens is None:
            lens = _fixed_lens(keys, fixed_len)
        return keys, lens          # one rank: the engine already sorted them
    if dist.get_backend(group) == "gloo" and keys.is_cuda:   # gloo gathers host tensors
        out = gather_hits(keys.cpu(), None if lens is None else lens.cpu(), group, dst, fixed_len)
        return None if out is None else (out[0].to(keys.device), out[1].to(keys.device))
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    # dst is a rank of ``group``; dist.gather takes the global rank
    gdst = dst if dst is None or group is None else dist.get_global_rank(group, dst)
    send_lens = fixed_len is None
    if send_lens and lens is None:
        raise ValueError("lens are needed unless fixed_len is given")
    count = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    counts = [torch.zeros_like(count) for _ in range(world)]
    dist.all_gather(counts, count, group=group)
    sizes = [int(c.item()) for c in counts]
    width = max(max(sizes), 1)
    pk = torch.zeros(width, dtype=keys.dtype, device=keys.device)
    pk[:keys.numel()] = keys
    if send_lens:
        pl = torch.zeros(width, dtype=lens.dtype, device=lens.device)
        pl[:lens.numel()] = lens
    # the receive buffers are views of one allocation (rank r's list at
    # r * width), so the merge reads the parts where they landed: no cat
    recv = me == dst or dst is None
    buf_k = torch.empty(world * width, dtype=keys.dtype, device=keys.device) if recv else None
    all_k = list(buf_k.split(width)) if recv else None
    if send_lens:
        buf_l = torch.empty(world * width, dtype=pl.dtype, device=pl.device) if recv else None
        all_l = list(buf_l.split(width)) if recv else None
    if dst is None:
        dist.all_gather(all_k, pk, group=group)
        if send_lens:
            dist.all_gather(all_l, pl, group=group)
    else:
        dist.gather(pk, all_k, dst=gdst, group=group)
        if send_lens:
            dist.gather(pl, all_l, dst=gdst, group=group)
        if me != dst:
            return None
    if buf_k.is_cuda:
        return merge_parts(buf_k, buf_l if send_lens else None, [r * width for r in range(world)], sizes,
                           fixed_len if not send_lens else None)
    parts = [t[:n] for t, n in zip(all_k, sizes)]
    k = torch.cat(parts)
    ln = torch.cat([t[:n] for t, n in zip(all_l, sizes)]) if send_lens else _fixed_lens(k, fixed_len)
    if k.numel() == 0:
        return k, ln
    return _merge(parts, k, ln)


def merge_parts(buf_k: torch.Tensor, buf_l: Optional[torch.Tensor], begs: Sequence[int], sizes: Sequence[int],
                fixed_len: Optional[Sequence[int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The ranks' lists (part r = buf[begs[r] : begs[r] + sizes[r]] of a
    device buffer, each sorted, position ranges increasing with r) ->
    (keys, lens) sorted by key, on the device by ``pm_merge_parts`` (one
    pass, no sort), ordered on torch's current stream.  Lengths move with
    their keys (``buf_l``) or come from the pattern field (``fixed_len``)."""
    from . import _lib
    dev = buf_k.device
    total = int(sum(sizes))
    out_k = torch.empty(total, dtype=torch.int64, device=dev)
    out_l = torch.empty(total, dtype=torch.int32, device=dev)
    if total == 0:
        return out_k, out_l
    if buf_l is None:
        table = torch.tensor(list(fixed_len), dtype=torch.int32, device=dev)
        npat = table.numel()
        lens_p = None
    else:
        npat = int((buf_k[begs[0]:begs[0] + sizes[0]] >> POS_BITS).max().item()) + 1 if sizes[0] else 1
        for b, n in zip(begs[1:], sizes[1:]):
            if n:
                npat = max(npat, int((buf_k[b:b + n] >> POS_BITS).max().item()) + 1)
        table = None
        lens_p = buf_l.to(torch.int32) if buf_l.dtype != torch.int32 else buf_l
    lib = _lib.load()
    n = len(sizes)
    beg_a = (_ct.c_uint64 * n)(*begs)
    len_a = (_ct.c_uint64 * n)(*sizes)
    wb = _ct.c_uint64()
    stream = _ct.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(lib.pm_merge_parts(None, None, beg_a, len_a, n, npat, None, None, None, None, _ct.byref(wb),
                                  dev.index or 0, stream))
    work = torch.empty(max(1, wb.value), dtype=torch.uint8, device=dev)
    _lib.check(lib.pm_merge_parts(_ct.c_void_p(buf_k.data_ptr()),
                                  _ct.c_void_p(lens_p.data_ptr()) if lens_p is not None else None,
                                  beg_a, len_a, n, npat,
                                  _ct.c_void_p(table.data_ptr()) if table is not None else None,
                                  _ct.c_void_p(out_k.data_ptr()), _ct.c_void_p(out_l.data_ptr()),
                                  _ct.c_void_p(work.data_ptr()), _ct.byref(wb), dev.index or 0, stream))
    return out_k, out_l


def _fixed_lens(keys: torch.Tensor, fixed_len: Optional[Sequence[int]]) -> torch.Tensor:
    table = torch.tensor(list(fixed_len), dtype=torch.int32, device=keys.device)
    return table[keys >> POS_BITS] if keys.numel() else torch.zeros(0, dtype=torch.int32, device=keys.device)


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` on every rank (one all_reduce MIN): a
    rank that failed locally makes the others fail instead of leaving them
    blocked in the next collective."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_coll_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


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


# --- zero-copy hand-over of a hit list (DLPack) ------------------------------
import ctypes as _ct


class _DLDevice(_ct.Structure):
    _fields_ = [("device_type", _ct.c_int32), ("device_id", _ct.c_int32)]


class _DLDataType(_ct.Structure):
    _fields_ = [("code", _ct.c_uint8), ("bits", _ct.c_uint8), ("lanes", _ct.c_uint16)]


class _DLTensor(_ct.Structure):
    _fields_ = [("data", _ct.c_void_p), ("device", _DLDevice), ("ndim", _ct.c_int32), ("dtype", _DLDataType),
                ("shape", _ct.POINTER(_ct.c_int64)), ("strides", _ct.POINTER(_ct.c_int64)),
                ("byte_offset", _ct.c_uint64)]


_DL_DELETER = _ct.CFUNCTYPE(None, _ct.c_void_p)


class _DLManagedTensor(_ct.Structure):
    _fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", _ct.c_void_p), ("deleter", _DL_DELETER)]


_KDL_ROCM, _KDL_INT, _KDL_UINT = 10, 0, 1
_LIVE = {}    # DLManagedTensor address -> (struct, shape, owner, device)
_OWNERS = {}  # hit-list handle -> tensors still alive


@_DL_DELETER
def _dl_release(addr):
    try:
        _dl_release_impl(addr)
    except Exception:   # interpreter teardown: the module's globals may be gone
        pass


def _dl_release_impl(addr):
    entry = _LIVE.pop(addr, None)
    if entry is None:
        return
    h, dev = entry[2], entry[3]
    _OWNERS[h] -= 1
    if _OWNERS[h] == 0:
        del _OWNERS[h]
        from . import _lib
        lib = _lib.load()
        recorded = False
        try:
            # torch frees external memory at once: the buffers go back to
            # the pool only after the work queued on torch's stream so far
            rc = lib.pm_hits_record_use(_ct.c_void_p(h), _ct.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
            recorded = rc == 0
        finally:
            if not recorded:
                # no use recorded: wait for every stream of the device, so no
                # queued reader sees the buffers reused
                torch.cuda.synchronize(dev)
            lib.pm_hits_destroy(_ct.c_void_p(h))


_capsule_new = _ct.pythonapi.PyCapsule_New
_capsule_new.restype = _ct.py_object
_capsule_new.argtypes = [_ct.c_void_p, _ct.c_char_p, _ct.c_void_p]


def _dl_tensor(h: int, ptr: int, n: int, bits: int, device: torch.device) -> torch.Tensor:
    shape = (_ct.c_int64 * 1)(n)
    mt = _DLManagedTensor()
    mt.dl_tensor.data = ptr
    mt.dl_tensor.device = _DLDevice(_KDL_ROCM, device.index if device.index is not None else 0)
    mt.dl_tensor.ndim = 1
    mt.dl_tensor.dtype = _DLDataType(_KDL_INT, bits, 1)
    mt.dl_tensor.shape = shape
    mt.dl_tensor.strides = None
    mt.dl_tensor.byte_offset = 0
    mt.deleter = _dl_release
    addr = _ct.addressof(mt)
    _LIVE[addr] = (mt, shape, h, device)
    _OWNERS[h] = _OWNERS.get(h, 0) + 1
    try:
        return torch.utils.dlpack.from_dlpack(_capsule_new(addr, b"dltensor", None))
    except Exception:
        _dl_release_impl(addr)
        raise


def hits_as_tensors(hits_handle, device: torch.device):
    """A ``pm_hits`` list's own device buffers as torch tensors (keys int64,
    lens int32), no copy: the tensors take the list over and destroy it
    (``pm_hits_destroy``) when both are freed -- the caller must not destroy
    it.  An empty list is destroyed at once.

    Stream contract: when the last tensor is freed, the buffers go back to
    the library's pool after the work queued so far on torch's CURRENT
    stream of ``device`` (``pm_hits_record_use``).  A caller that reads the
    tensors on another stream (``with torch.cuda.stream(s2)``) must free them
    while that stream is current, or synchronize it first (or
    ``record_stream`` a clone) -- as with any tensor torch's caching
    allocator hands back early.  If the use cannot be recorded, the release
    synchronizes the device before the buffers are returned."""
    from . import _lib
    lib = _lib.load()
    keys_p, lens_p, n = _ct.c_void_p(), _ct.c_void_p(), _ct.c_uint64()
    # waits for the list's producing work (the pointers are read by torch's streams)
    _lib.check(lib.pm_hits_device(hits_handle, _ct.byref(keys_p), _ct.byref(lens_p), _ct.byref(n)))
    h = hits_handle.value if isinstance(hits_handle, _ct.c_void_p) else int(hits_handle)
    if n.value == 0:
        _lib.check(lib.pm_hits_destroy(_ct.c_void_p(h)))
        return (torch.empty(0, dtype=torch.int64, device=device), torch.empty(0, dtype=torch.int32, device=device))
    keys = _dl_tensor(h, keys_p.value, n.value, 64, device)
    lens = _dl_tensor(h, lens_p.value, n.value, 32, device)
    return keys, lens


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

# bytes held past a piece's end: >= any window that can cross a cut (the
# simple engine's cross-line windows, up to PM_MAX_POSITIONS positions)
HALO = 4096
_SPACE = np.frombuffer(b" \t\n\r\f\x0b", dtype=np.uint8)


def _check_halo():
    from . import _lib
    assert HALO >= _lib.PM_MAX_POSITIONS, "HALO must cover the longest automaton window"


_check_halo()


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


_NAME_STOP = (b" ", b"\t", b"\n", b"\r", b"\f", b"\x0b")


def _next_header(data, target: int) -> int:
    """The first header-line start at or after ``target`` ('>' at a line
    start, then a non-space, as header_lines), or len(data).  Reads only
    from target - 1 on, so on a memory map it touches the pages around the
    cut alone."""
    n = len(data)

    def named(h):
        return h + 1 < n and data[h + 1:h + 2] not in _NAME_STOP

    if target <= 0:
        if n and data[0:1] == b">" and named(0):
            return 0
        target = 1
    pos = target - 1
    while True:
        q = data.find(b"\n>", pos)
        if q < 0:
            return n
        if named(q + 1):
            return q + 1
        pos = q + 1


def split_fasta(data, world: int) -> List[Tuple[int, int]]:
    """``world`` contiguous byte ranges covering ``data`` (bytes or a memory
    map), cut only at header lines, of about equal size (a range may be
    empty: fewer records than ranks).  Cut i is the first header line at or
    after n*i/world, found by scanning forward from there."""
    n = len(data)
    cuts = [0]
    for i in range(1, world):
        cuts.append(max(_next_header(data, (n * i) // world), cuts[-1]))
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


def _lib_bufsize() -> int:
    from . import _lib
    return _lib.PM_NRGREP_BUFFER


def shared_regions(data, bufsize: Optional[int] = None, group=None, failed: Optional[BaseException] = None):
    """nrgrep's search regions of the whole file (``engine.nrgrep_regions``),
    read once: with torch.distributed initialised over more than one rank,
    rank 0 computes them (a one-line record over the buffer size makes that
    a pass over the file) and broadcasts the table -- a collective, every
    rank of ``group`` calls it, also one that could not read the file
    (``failed``: rank 0 then broadcasts the failure, so every rank raises).
    Otherwise computed here."""
    from . import engine
    bufsize = _lib_bufsize() if bufsize is None else bufsize
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        obj = [None]
        if dist.get_rank(group) == 0:
            try:
                if failed is not None:
                    raise failed
                obj[0] = engine.nrgrep_regions(data, bufsize)
            except Exception as exc:   # still broadcast: the peers raise too
                obj[0] = {"failed": repr(exc)}
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if isinstance(obj[0], dict):
            raise RuntimeError("shared_regions: rank 0 could not read the file: %s" % obj[0]["failed"])
        return obj[0]
    return engine.nrgrep_regions(data, bufsize)


class ShardedDatabase:
    """Rank ``rank``'s piece of a FASTA file (``split_fasta``) in HBM, with
    ``HALO`` bytes of the next piece so windows that start in the piece are
    evaluated on the file's own bytes.  ``raw`` is the whole file as bytes
    or, from :meth:`from_file`, a read-only memory map: a rank reads only its
    piece (+ halo) and the pages around the cuts, and the hit text of any
    piece is sliced from the map on demand.  Hit offsets are file offsets."""

    def __init__(self, data, world: int, rank: int, device: int = 0, alphabet: Optional[str] = None,
                 halo: int = HALO, open_db: bool = True, bufsize: Optional[int] = None, regions=None):
        self.raw = data
        self.world, self.rank = world, rank
        self.ranges = split_fasta(data, world)
        self.beg, self.end = self.ranges[rank]
        self.stop = min(len(data), self.end + halo) if self.end > self.beg else self.end
        local = bytes(data[self.beg:self.stop])
        hs, he = header_lines(local[:self.end - self.beg])
        self.headers = (hs, he)
        # nrgrep's search regions are the whole file's (buffers of -b bytes
        # from offset 0): the piece takes those over [beg, stop), shifted to
        # its offsets (the first clipped to 0); ``regions`` = the whole
        # file's table when the caller has it (shared_regions)
        from . import engine
        gt, ge = regions if regions is not None else engine.nrgrep_regions(
            data, _lib_bufsize() if bufsize is None else bufsize)
        gt, ge = np.asarray(gt, dtype=np.int64), np.asarray(ge, dtype=np.int64)
        sel = (gt < self.stop) & (ge > self.beg)
        if self.stop > self.beg and sel.any():
            lt = np.maximum(gt[sel], self.beg) - self.beg
            le = np.minimum(ge[sel], self.stop) - self.beg
        else:
            lt, le = np.zeros(1, dtype=np.int64), np.full(1, self.stop - self.beg, dtype=np.int64)
        self.regions = (lt, le)
        self.db = None
        if open_db and self.stop > self.beg:
            self.db = engine.SequenceDatabase.from_bytes(local, alphabet or engine.choose_alphabet(local), device)
            self.db.set_regions(lt, le)

    @classmethod
    def from_file(cls, path: str, world: int, rank: int, device: int = 0, open_db: bool = True,
                  group=None) -> "ShardedDatabase":
        """Memory-maps ``path``.  With torch.distributed initialised this is
        a collective (``shared_regions``): every rank of ``group`` opens its
        piece together, and only rank 0 reads the whole file."""
        import mmap
        failed = None
        try:
            with open(path, "rb") as fh:
                size = os.fstat(fh.fileno()).st_size
                data = mmap.mmap(fh.fileno(), size, access=mmap.ACCESS_READ) if size else b""
        except (OSError, ValueError) as exc:   # still take part in the broadcast
            failed, data = exc, b""
        regions = shared_regions(data, group=group, failed=failed)
        if failed is not None:
            raise failed
        return cls(data, world, rank, device, open_db=open_db, regions=regions)

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
    (from there on the two chains agree).  The rule restarts at every
    search region's start (R = that start, recSearchFile); the incoming
    report lies in the piece's first region."""
    cb, ce = (np.asarray(x, dtype=np.int64) for x in cand)
    keep = cb < len(piece)
    cb, ce = cb[keep], ce[keep]
    ob, oe = chain
    text, base = piece.raw, piece.beg
    lt = piece.regions[0]
    out_b, out_e = [], []
    cur = 0   # the region of the last report

    def first_from(R, cur):
        # the next candidate at or after R -- or at the next region's start,
        # which may lie before R (the '\n' two regions share)
        lim = min(R, int(lt[cur + 1])) if cur + 1 < lt.size else R
        return int(np.searchsorted(cb, lim))

    i = first_from(R, cur)
    while i < cb.size:
        s = int(cb[i])
        reg = int(np.searchsorted(lt, s, side="right")) - 1
        if reg > cur:   # a new region: its search starts at its first byte
            cur, R = reg, int(lt[reg])
        if s < R:
            i += 1
            continue
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
        i = first_from(R, cur)
    return np.array(out_b, dtype=np.int64), np.array(out_e, dtype=np.int64)


_RECHAIN_FAILED = -2   # a re-chaining rank's broadcast when its re-chain raised


def scan_sharded(piece: ShardedDatabase, progs: Sequence, k: int = 0, types: str = "ids", group=None,
                 scanner=None, dst: Optional[int] = None) -> Optional[List[Tuple[np.ndarray, np.ndarray]]]:
    """Every rank scans its piece; returns [(beg, end) per program] in file
    offsets -- equal to the single-process scan of the whole file (what
    nrgrep_coords reports, header-line starts dropped) -- on rank ``dst``
    (the hits travel there only: ``dist.gather``), None on the other ranks;
    ``dst=None``: on every rank (``all_gather``).

    Collective: every rank of ``group`` must call it with the same programs,
    in the same order as its other collective calls.  A rank whose local
    scan raises still takes part in the first collective (``agree``), and a
    rank whose re-chain raises still broadcasts (a failure marker), so the
    other ranks raise too instead of blocking.  A failure inside the final
    hit gather itself (e.g. out of memory) is left to the process group's
    timeout."""
    scanner = scanner or piece.scanner()
    P = len(progs)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    n_local = len(piece)
    empty = (np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64))
    failure = None
    chains = [empty] * P
    try:
        if n_local:
            chains = []
            for b, e in scanner.reported(progs, k, types):
                b, e = np.asarray(b, dtype=np.int64), np.asarray(e, dtype=np.int64)
                keep = b < n_local
                chains.append((b[keep], e[keep]))
    except Exception as exc:   # every rank takes part in the agreement below
        failure = exc
    if not agree(failure is None, group):
        if failure is not None:
            raise failure
        raise RuntimeError("scan_sharded: another rank's scan failed")
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
                try:
                    for p in need:
                        if n_local:
                            cand = scanner.candidates(progs[p], k, types)
                            chains[p] = _rechain(piece, progs[p], cand, chains[p], int(state[p]) - beg_r)
                    mine = np.array([int(e[-1]) + piece.beg if e.size else -1 for _, e in chains], dtype=np.int64)
                    out.copy_(torch.from_numpy(np.maximum(mine, state)))
                except Exception as exc:   # the broadcast below still happens: the peers see the failure
                    failure = exc
                    out.fill_(_RECHAIN_FAILED)
            dist.broadcast(out, src=r, group=group)
            state = out.cpu().numpy()
            if (state == _RECHAIN_FAILED).any():
                if failure is not None:
                    raise failure
                raise RuntimeError("scan_sharded: rank %d's re-chain failed" % r)
    hs, he = piece.headers
    chains = [drop_header_starts(b, e, hs, he) for b, e in chains]
    if world == 1:
        return [(b + piece.beg, e + piece.beg) for b, e in chains]
    dev = _coll_device(group)
    keys = np.concatenate([(np.int64(p) << POS_BITS) | (b + piece.beg) for p, (b, _) in enumerate(chains)]
                          or [np.zeros(0, dtype=np.int64)])
    lens = np.concatenate([(e - b).astype(np.int32) for b, e in chains] or [np.zeros(0, dtype=np.int32)])
    out = gather_hits(torch.from_numpy(keys).to(dev), torch.from_numpy(lens).to(dev), group, dst=dst)
    if out is None:
        return None
    gk, gl = out[0].cpu().numpy(), out[1].cpu().numpy().astype(np.int64)
    pat = gk >> POS_BITS
    beg = gk & POS_MASK
    res = []
    for p in range(P):
        sel = pat == p
        res.append((beg[sel], beg[sel] + gl[sel]))
    return res
