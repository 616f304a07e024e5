"""Scan-pipeline dispatch: compiled patterns -> HIP kernels -> hits.

This is the host half of the replacement for one or more
``nrgrep_coords -i -b .. -k <k><types> '<pattern>' '<datafile>'`` runs
(``www/FlaskApp/FlaskApp/patmatch.py:733-742``).  A
:class:`SequenceDatabase` uploads a FASTA file into HBM once; :func:`scan`
routes every compiled :class:`~patmatchdocker_amd.regex.Program` to a kernel:

* ``linear`` -- fixed-length class sequences with substitutions only go to
  ``pm_scan_linear``: the bit-sliced Hamming kernel on a nucleotide database
  (all strands/patterns of a query in ONE pass over the data), a per-window
  byte kernel on a peptide database; at k = 0 this is nrgrep's "simple"
  engine, whose windows may span a line break;
* ``nfa``    -- everything else goes to the Glushkov reverse-scan + verify
  kernels (``pm_scan_nfa_errs``), which stay inside one line.

Every scan returns what nrgrep_coords PRINTS (``report="nrgrep"``): the
kernels' candidates reduced on the GPU by the binary's report rule (first
match found wins, the scan resumes at its end) and its '^'/'$' checks --
DESIGN.md §1.

Queries with insertions/deletions (``-k <k>ids``, the web form's default
when mismatches > 0) go to the Glushkov kernels with the error-type mask.
Unbounded ``*``/``+`` (``{m,}``) also run there (chunk states relaxed
across chunks, :func:`scan_nfa`), as do class sequences longer than 64
positions or with more than 3 errors (up to 256 positions and 15 errors,
7 above 128 positions).  Anything else (deletions with k >= the shortest
match, longer automata) raises :class:`UnsupportedOnGPU`; there is no CPU
fallback by design.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import UnsupportedOnGPU, check
from .regex import ALL_BYTES, Program, fold_byte

ANY_FOLDED = frozenset(fold_byte(b) for b in ALL_BYTES)   # '.': every byte value a folded text can hold

REPORT_NRGREP = "nrgrep"   # what nrgrep_coords prints (non-overlapping, first found wins)
REPORT_ALL = "all"         # every candidate start (shortest end)


def report_flags(prog: Program, report: str = REPORT_NRGREP, keep_headers: bool = False,
                 start_anchor: bool = True) -> int:
    """PM_REPORT_* / PM_ANCHOR_* / PM_KEEP_HEADERS flags of one program
    (include/patmatch_hip.h).  ``start_anchor=False`` leaves the '^' check to
    the caller (shards.py re-chains candidates across pieces of a file)."""
    if report not in (REPORT_NRGREP, REPORT_ALL):
        raise ValueError("report must be %r or %r" % (REPORT_NRGREP, REPORT_ALL))
    f = _lib.PM_REPORT_NRGREP if report == REPORT_NRGREP else _lib.PM_REPORT_ALL
    if keep_headers:
        f |= _lib.PM_KEEP_HEADERS
    if prog.anchor_start and start_anchor:
        f |= _lib.PM_ANCHOR_START
    if prog.anchor_end:
        f |= _lib.PM_ANCHOR_END
    return f
_ACGT = tuple(ord(c) for c in "ACGT")

NUC = "nuc"
BYTE = "byte"


def choose_alphabet(data: bytes, sample: int = 1 << 22) -> str:
    """Nucleotide planes when >= 90 % of the sampled sequence bytes are ACGTN."""
    head = data[:sample]
    seq = bytearray()
    for line in head.split(b"\n"):
        if not line.startswith(b">"):
            seq += line
    if not seq:
        return NUC
    arr = np.frombuffer(bytes(seq), dtype=np.uint8)
    folded = np.where((arr >= 97) & (arr <= 122), arr - 32, arr)
    good = np.isin(folded, np.frombuffer(b"ACGTN", dtype=np.uint8)).mean()
    return NUC if good >= 0.9 else BYTE


def nrgrep_regions(data, bufsize: int = _lib.PM_NRGREP_BUFFER):
    """nrgrep's search regions of a file read in buffers of ``bufsize`` bytes:
    (starts, ends) int64 arrays, region r = [starts[r], ends[r]).

    ``nrgrep_coords -b 1600000`` (patmatch.py:733-743) reads the file in
    buffers of 1,600,000 BYTES (OptBufSize = atoi(optarg), 0x401162; bufCreate
    allocates it, 0x41bb6b).  recSearchFile (0x402250) searches a full buffer
    up to and including its last '\n' (simpleRevSearch, 0x402475) and loads
    the next buffer from that '\n' on (bufLoad, 0x4023e6); a buffer with no
    '\n' but at its start is searched whole and the next starts after it
    (0x4024a0 -> 0x4022ba); the last buffer (bufEof 0x41bfc0: not full)
    reaches the end of the file.  ``data``: bytes or an mmap (rfind)."""
    n = len(data)
    starts, ends = [], []
    at = 0
    while True:
        starts.append(at)
        if bufsize <= 0 or at + bufsize > n:
            ends.append(n)
            break
        d = data.rfind(b"\n", at, at + bufsize)
        if d > at:
            ends.append(d + 1)
            at = d
        else:
            ends.append(at + bufsize)
            at += bufsize
        if at >= n:
            break
    return np.array(starts, dtype=np.int64), np.array(ends, dtype=np.int64)


class SequenceDatabase:
    """A FASTA file resident in the HBM of one GPU (``pm_db``)."""

    def __init__(self, handle, alphabet: str, device: int, raw: Optional[bytes] = None):
        self._h = handle
        self.alphabet = alphabet
        self.device = device
        self.raw = raw

    @classmethod
    def from_bytes(cls, data: bytes, alphabet: Optional[str] = None, device: int = 0,
                   stream: Optional[int] = None) -> "SequenceDatabase":
        lib = _lib.load()
        alphabet = alphabet or choose_alphabet(data)
        code = _lib.PM_ALPHA_NUC if alphabet == NUC else _lib.PM_ALPHA_BYTE
        h = ctypes.c_void_p()
        check(lib.pm_db_create(data, len(data), code, device, stream, ctypes.byref(h)))
        return cls(h, alphabet, device, raw=data)

    @classmethod
    def from_file(cls, path: str, alphabet: Optional[str] = None, device: int = 0) -> "SequenceDatabase":
        with open(path, "rb") as fh:
            return cls.from_bytes(fh.read(), alphabet, device)

    @classmethod
    def synthetic(cls, n_records: int, rec_len: int, seed: int = 1, device: int = 0,
                  stream: Optional[int] = None) -> "SequenceDatabase":
        lib = _lib.load()
        h = ctypes.c_void_p()
        check(lib.pm_db_create_synthetic(n_records, rec_len, seed, device, stream, ctypes.byref(h)))
        return cls(h, NUC, device, raw=None)

    @property
    def handle(self):
        if self._h is None:
            raise ValueError("database closed")
        return self._h

    def info(self):
        n, alpha, nx, nbytes = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.load().pm_db_info(self.handle, ctypes.byref(n), ctypes.byref(alpha), ctypes.byref(nx),
                                     ctypes.byref(nbytes)))
        return {"positions": n.value, "alphabet": NUC if alpha.value == 0 else BYTE,
                "exception_words": nx.value, "device_bytes": nbytes.value}

    def residue_codes(self):
        """BYTE databases: (number of 5-bit residue codes, code of each byte
        as a 256-entry uint8 array); 0 codes = no residue planes."""
        n = ctypes.c_int()
        table = np.zeros(256, dtype=np.uint8)
        check(_lib.load().pm_db_residue_codes(self.handle, ctypes.byref(n), table.ctypes.data))
        return n.value, table

    def __len__(self):
        return self.info()["positions"]

    def regions(self):
        """nrgrep's search regions of the loaded text (nrgrep_regions):
        (starts, ends) int64 arrays."""
        lib = _lib.load()
        cnt = ctypes.c_uint64()
        check(lib.pm_db_regions(self.handle, 0, None, None, ctypes.byref(cnt)))
        t = np.empty(cnt.value, dtype=np.uint64)
        e = np.empty(cnt.value, dtype=np.uint64)
        check(lib.pm_db_regions(self.handle, cnt.value, t.ctypes.data, e.ctypes.data, ctypes.byref(cnt)))
        return t.astype(np.int64), e.astype(np.int64)

    def set_regions(self, starts, ends):
        """Replace the search regions (a piece of a larger file takes the
        file's regions shifted into its coordinates; one region [0, n): no
        cuts)."""
        t = np.ascontiguousarray(starts, dtype=np.uint64)
        e = np.ascontiguousarray(ends, dtype=np.uint64)
        if t.shape != e.shape or t.size == 0:
            raise ValueError("starts and ends: equal non-empty lengths")
        check(_lib.load().pm_db_set_regions(self.handle, t.size, t.ctypes.data, e.ctypes.data))

    def decode(self, beg: int, length: int) -> bytes:
        buf = ctypes.create_string_buffer(max(length, 1))
        check(_lib.load().pm_db_decode(self.handle, beg, length, buf))
        return buf.raw[:length]

    def text(self, beg: int, end: int) -> bytes:
        """Original (not case-folded) bytes when the file is held, else decoded."""
        if self.raw is not None:
            return self.raw[beg:end]
        return self.decode(beg, end - beg)

    def close(self):
        if self._h is not None:
            check(_lib.load().pm_db_destroy(self._h))
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Hits:
    """Hits of one scan call, sorted by (pattern, beg)."""

    pattern: np.ndarray
    beg: np.ndarray
    end: np.ndarray
    kernel_ms: float

    def for_pattern(self, i: int):
        sel = self.pattern == i
        return self.beg[sel], self.end[sel]


def _collect(handle) -> Hits:
    lib = _lib.load()
    try:
        n = ctypes.c_uint64()
        check(lib.pm_hits_count(handle, ctypes.byref(n)))
        count = n.value
        pat = np.empty(count, dtype=np.int32)
        beg = np.empty(count, dtype=np.int64)
        end = np.empty(count, dtype=np.int64)
        if count:
            check(lib.pm_hits_copy(handle, pat.ctypes.data, beg.ctypes.data, end.ctypes.data, count))
        ms = ctypes.c_double()
        check(lib.pm_hits_kernel_ms(handle, ctypes.byref(ms)))
        return Hits(pat, beg, end, ms.value)
    finally:
        lib.pm_hits_destroy(handle)


def parse_error_types(k: int, types: str) -> str:
    return (types or "ids") if k else ""


def nfa_words(m: int) -> int:
    """64-bit words of a position set in the automaton kernels."""
    return 1 if m <= 64 else 2 if m <= 128 else 4


def route(prog: Program, alphabet: str, k: int, types: str) -> str:
    """Which kernel handles ``prog``; raises UnsupportedOnGPU if none does."""
    indel = bool(k) and ("i" in types or "d" in types)
    if prog.linear and not indel and prog.m <= _lib.PM_MAX_LINEAR_POSITIONS and k <= _lib.PM_MAX_LINEAR_K:
        return "linear"   # nucleotide planes (bit-sliced) or the byte layout (k_bytes_linear)
    if prog.m > _lib.PM_MAX_POSITIONS:
        raise UnsupportedOnGPU("patterns longer than %d positions are not supported" % _lib.PM_MAX_POSITIONS)
    if k > _lib.PM_MAX_K or (nfa_words(prog.m) == 4 and k > 7):
        raise UnsupportedOnGPU("k=%d errors is not supported by the GPU kernels for %d positions" % (k, prog.m))
    # deletions with k >= the shortest match route too: a class sequence runs
    # nrgrep's esimple report, whose walk then takes every position of every
    # line (pm_esimple.hip, es_all_positions); an extended pattern its
    # eextended report, every line a cluster (pm_eextended.hip,
    # ee_add_lines); a regular one its eregular report, likewise
    # (pm_regular.hip) -- every engine kind, so no shape is refused here
    return "nfa"   # automaton kernels: anything else, long oligos and k > 3 included


def _linear_tables(progs: Sequence[Program]):
    classes, index = [], {}
    pos_class = np.zeros((len(progs), 64), dtype=np.uint8)
    lengths = np.zeros(len(progs), dtype=np.int32)
    for p, prog in enumerate(progs):
        lengths[p] = prog.m
        for j, cls in enumerate(prog.classes):
            if cls not in index:
                index[cls] = len(classes)
                classes.append(cls)
            pos_class[p, j] = index[cls]
    nc = len(classes)
    acgt = np.zeros(nc, dtype=np.uint8)
    is_any = np.zeros(nc, dtype=np.uint8)
    bits = np.zeros((nc, 8), dtype=np.uint32)
    for c, cls in enumerate(classes):
        acgt[c] = sum(1 << i for i, b in enumerate(_ACGT) if b in cls)
        is_any[c] = 1 if ANY_FOLDED <= cls else 0   # accepts every byte, '\n' included
        for b in cls:
            bits[c, b >> 5] |= np.uint32(1 << (b & 31))
    return lengths, pos_class, nc, acgt, bits, is_any


class LinearBatch:
    """Pre-built class/position tables of a batch of linear programs."""

    def __init__(self, progs: Sequence[Program]):
        for p in progs:
            if not p.linear:
                raise ValueError("LinearBatch needs linear programs: %s" % p.source)
        self.lengths, self.pos_class, self.nc, self.acgt, self.bits, self.is_any = _linear_tables(progs)
        self.n = len(progs)

    def launch(self, db: SequenceDatabase, k: int, pipelined: bool = False, flags: int = None):
        """Run pm_scan_linear; returns the raw pm_hits handle (caller destroys).

        ``pipelined``: pm_scan_linear_async -- returns before the scan ends
        (the handle resolves on first use), so a caller can launch the next
        query before collecting this one.  ``flags``: PM_REPORT_* /
        PM_ANCHOR_* (default: what nrgrep_coords reports)."""
        out = ctypes.c_void_p()
        lib = _lib.load()
        fn = lib.pm_scan_linear_async if pipelined else lib.pm_scan_linear
        flags = _lib.PM_REPORT_NRGREP if flags is None else flags
        check(fn(db.handle, self.n, self.lengths.ctypes.data, self.pos_class.ctypes.data, self.nc,
                 self.acgt.ctypes.data, self.bits.ctypes.data, self.is_any.ctypes.data, k, flags,
                 ctypes.byref(out)))
        return out


def jit_compile(progs: Sequence[Program], k: int) -> int:
    """Generate + hipRTC-compile the specialized linear kernel (no GPU needed);
    returns the code-object size in bytes."""
    t = LinearBatch(progs)
    nbytes = ctypes.c_uint64()
    check(_lib.load().pm_linear_jit_compile(t.n, t.lengths.ctypes.data, t.pos_class.ctypes.data, t.nc,
                                            t.acgt.ctypes.data, t.is_any.ctypes.data, k, ctypes.byref(nbytes)))
    return nbytes.value


def ids_jit_compile(prog: Program, k: int, types: str = "ids") -> int:
    """Generate + hipRTC-compile the bit-sliced start pass for a class
    sequence with insertions/deletions (no GPU needed); returns the
    code-object size in bytes."""
    bm = np.array(prog.byte_masks(), dtype=np.uint64)
    bm[10] = 0
    nbytes = ctypes.c_uint64()
    check(_lib.load().pm_ids_jit_compile(prog.m, bm.ctypes.data, k, error_mask(types) if k else _lib.PM_ERR_SUB,
                                         ctypes.byref(nbytes)))
    return nbytes.value


def esimple_plan(prog: Program, k: int) -> dict:
    """The scan plan nrgrep's esimplePreproc derives for ``prog`` at ``k``
    errors (pm_esimple_plan, host only): ``type`` 1 = k+1 pieces of
    ``piece_len`` (BNDM), 2 = the ``window`` backward (ABNDM), 3 = the prefix
    forward (shift-or); ``L`` = pattern positions left of each piece."""
    w = nfa_words(prog.m)
    bm = np.array([_words(x, w) for x in prog.byte_masks()], dtype=np.uint64)
    out = (ctypes.c_int32 * (6 + _lib.PM_MAX_K))()
    check(_lib.load().pm_esimple_plan(prog.m, w, bm.ctypes.data, k, out))
    return {"type": out[0], "piece_len": out[1], "window": (out[2], out[3]),
            "L": [out[5 + i] for i in range(out[4])]}


def extended_plan(prog: Program) -> dict:
    """The scan plan nrgrep's extendedPreproc derives for an extended
    pattern (pm_extended_plan, host only): ``type`` 2 = the ``window``
    scanned backward, 3 = the prefix scanned forward; ``fwd`` = the window's
    non-optional positions; ``L`` = pattern positions left of a candidate;
    ``simple`` = the window holds no '?*+'."""
    w = nfa_words(prog.m)
    bm = np.array([_words(x, w) for x in prog.byte_masks()], dtype=np.uint64)
    opt = np.array(_words(prog.opt_mask, w), dtype=np.uint64)
    rep = np.array(_words(prog.rep_mask, w), dtype=np.uint64)
    out = (ctypes.c_int32 * 6)()
    check(_lib.load().pm_extended_plan(prog.m, w, bm.ctypes.data, opt.ctypes.data, rep.ctypes.data, out))
    return {"type": out[0], "fwd": out[1], "window": (out[2], out[3]), "L": out[4], "simple": bool(out[5])}


def eextended_plan(prog: Program, k: int) -> dict:
    """The scan plan nrgrep's eextendedPreproc derives for an extended
    pattern at ``k`` > 0 errors (pm_eextended_plan, host only): ``type`` 1 =
    k + 1 ``pieces`` of ``plen`` characters searched exactly, 2 = a window
    backward, 3 = the prefix forward (``pieces`` then holds it); ``simple``
    = the scanned positions hold no '?*+' (nrgrep's esimple scanners);
    ``window`` = extendedFindBest's, ``fwd`` its non-optional positions."""
    w = nfa_words(prog.m)
    bm = np.array([_words(x, w) for x in prog.byte_masks()], dtype=np.uint64)
    opt = np.array(_words(prog.opt_mask, w), dtype=np.uint64)
    rep = np.array(_words(prog.rep_mask, w), dtype=np.uint64)
    out = (ctypes.c_int32 * (6 + 2 * (_lib.PM_MAX_K + 1)))()
    check(_lib.load().pm_eextended_plan(prog.m, w, bm.ctypes.data, opt.ctypes.data, rep.ctypes.data, k, out))
    np_ = out[2]
    return {"type": out[0], "simple": bool(out[1]), "plen": out[3] if out[0] == 1 else 0,
            "fwd": out[3] if out[0] != 1 else 0, "window": (out[4], out[5]),
            "pieces": [(out[6 + 2 * i], out[7 + 2 * i]) for i in range(np_)]}


def kernel_ms(handle) -> float:
    ms = ctypes.c_double()
    check(_lib.load().pm_hits_kernel_ms(handle, ctypes.byref(ms)))
    return ms.value


def destroy_hits(handle):
    check(_lib.load().pm_hits_destroy(handle))


def scan_linear(db: SequenceDatabase, progs: Sequence[Program], k: int, flags: int = None) -> Hits:
    return _collect(LinearBatch(progs).launch(db, k, flags=flags))


def graded_tail_start(positions: int) -> Optional[int]:
    """First file offset that pm_linear_jit's graded tail scans (the last
    output segments' tiles go to workgroups of tpw / 4 tiles), or None when
    the tail does not engage (tpw < 4, below ~2 Gbp).  Mirrors scan_linear's
    partition in csrc/pm_linear.hip (JIT_WG_PER_CU = 4, split = 8, tiles of
    65,536 positions, tiles_for in pm_db.hip); tests and bench.py use it to
    point the oracle at the tiles the tail owns."""
    tile, wg_per_cu, split = 65536, 4, 8
    ntiles = (positions + 4096 + 2048 + tile - 1) // tile
    nwg = min(ntiles, 256 * wg_per_cu * split)
    tpw = -(-ntiles // nwg)
    nwg = -(-ntiles // tpw)
    nout = -(-nwg // split)
    tpo = tpw * split
    ogb = -(-(256 * wg_per_cu * tpw) // tpo)
    if os.environ.get("PM_JIT_GRADED", "1") == "0" or tpw < 4 or ogb >= nout:
        return None
    return (nout - ogb) * tpo * tile


def error_mask(types: str) -> int:
    """'-k' type letters -> PM_ERR_* mask (patmatch.py:299-309)."""
    return ((_lib.PM_ERR_INS if "i" in types else 0) | (_lib.PM_ERR_DEL if "d" in types else 0)
            | (_lib.PM_ERR_SUB if "s" in types else 0))


def _words(x: int, w: int) -> List[int]:
    return [(x >> (64 * q)) & 0xFFFFFFFFFFFFFFFF for q in range(w)]


def _nfa_tables(prog: Program):
    """The automaton's tables as pm_scan_nfa_wide takes them, built once per
    program (a compiled Program is not modified; building them costs a few
    hundred microseconds of Python per query)."""
    t = prog.__dict__.get("_nfa_tables")
    if t is None:
        w = nfa_words(prog.m)
        t = (w, np.array([_words(x, w) for x in prog.byte_masks()], dtype=np.uint64),
             np.array([_words(x, w) for x in prog.follow], dtype=np.uint64),
             np.array(_words(prog.first, w), dtype=np.uint64), np.array(_words(prog.last, w), dtype=np.uint64))
        prog.__dict__["_nfa_tables"] = t
    return t


def _tree_tables(prog: Program):
    """Program.tree as pm_scan_nfa_tree takes it (int32 [nodes][4], [nodes])."""
    t = prog.__dict__.get("_tree_tables")
    if t is None:
        t = (np.array([v for node in prog.tree for v in node], dtype=np.int32),
             np.array(prog.tree_nullable, dtype=np.int32))
        prog.__dict__["_tree_tables"] = t
    return t


def regular_plan(prog: Program) -> dict:
    """The plan nrgrep's regularPreproc derives for a regular pattern
    (pm_regular_plan, host only): ``type`` 2 = a window of ``ell``
    characters scanned backward, 3 = the automaton forward; ``cls`` = the
    window's detClass (1 / 2: nrgrep prints nothing); ``window`` / ``init``
    / ``final`` = state sets (position + 1)."""
    w = nfa_words(prog.m)
    bm = np.array([_words(x, w) for x in prog.byte_masks()], dtype=np.uint64)
    tree, tnull = _tree_tables(prog)
    out = (ctypes.c_int32 * 4)()
    masks = np.zeros(15, dtype=np.uint64)
    check(_lib.load().pm_regular_plan(prog.m, w, bm.ctypes.data, len(prog.tree), tree.ctypes.data,
                                      tnull.ctypes.data, out, masks.ctypes.data))

    def as_int(ws):
        return sum(int(x) << (64 * q) for q, x in enumerate(ws))
    return {"type": out[0], "ell": out[1], "cls": out[2], "states": out[3], "window": as_int(masks[0:5]),
            "init": as_int(masks[5:10]), "final": as_int(masks[10:15])}


def eregular_plan(prog: Program, k: int) -> dict:
    """The plan nrgrep's eregularPreproc derives at ``k`` errors
    (pm_eregular_plan, host only): ``type`` 1 = k + 1 pieces of ``ell``
    characters found exactly, 2 = a window of ``ell`` characters scanned
    backward with k errors, 3 = the automaton forward; ``cls`` = detClass of
    the first window (2: nothing prints); ``windows`` = [(window, init,
    final)]; ``match`` = checkMatch's state word for class 1."""
    if prog.kind != "regular":
        raise ValueError("not a regular pattern: %s" % prog.source)
    w, bm, _, _, _ = _nfa_tables(prog)
    tree, tnull = _tree_tables(prog)
    out = np.zeros(5, dtype=np.int32)
    nw = 5   # RG_NW: words per state set
    masks = np.zeros((3 * (_lib.PM_MAX_K + 1) + 1) * nw, dtype=np.uint64)
    check(_lib.load().pm_eregular_plan(prog.m, w, bm.ctypes.data, len(prog.tree), tree.ctypes.data, tnull.ctypes.data,
                                       k, out.ctypes.data, masks.ctypes.data))

    def word_set(j):
        return sum(int(masks[j * nw + q]) << (64 * q) for q in range(nw))
    wins = [(word_set(3 * i), word_set(3 * i + 1), word_set(3 * i + 2)) for i in range(int(out[4]))]
    return {"type": int(out[0]), "ell": int(out[1]), "cls": int(out[2]), "defined": bool(out[3]),
            "windows": wins, "match": int(masks[3 * (_lib.PM_MAX_K + 1) * nw])}


def nfa_launch(db: SequenceDatabase, prog: Program, k: int, pattern_id: int = 0, types: str = "s",
               flags: int = None, pipelined: bool = False):
    """pm_scan_nfa_wide; returns the raw pm_hits handle (caller destroys),
    keys ``pattern_id << 48 | beg`` -- see :func:`scan_nfa`.
    ``pipelined`` (PM_PIPELINED): returns once the report pass is queued;
    the list's count resolves on first use, so the caller can launch its
    next scan (the other strand) before collecting this one."""
    w, bm, fol, first, last = _nfa_tables(prog)
    errs = error_mask(types) if k else _lib.PM_ERR_SUB
    flags = report_flags(prog) if flags is None else flags
    if pipelined:
        flags |= _lib.PM_PIPELINED
    if k == 0 and prog.linear and any(10 in c for c in prog.classes):
        flags |= _lib.PM_CROSS_LINES
    if k > 0 and prog.linear and prog.kind == "simple":
        flags |= _lib.PM_ESIMPLE   # nrgrep's esimple engine decides the report
    if prog.kind == "extended":
        flags |= _lib.PM_EXTENDED  # nrgrep's extended / eextended engine decides the report
    out = ctypes.c_void_p()
    if prog.kind == "regular" and (flags & _lib.PM_REPORT_NRGREP):
        # nrgrep's regular (k = 0) / eregular (k > 0) engine decides the
        # report; its plan is priced over nrgrep's parse tree
        tree, tnull = _tree_tables(prog)
        check(_lib.load().pm_scan_nfa_tree(db.handle, prog.m, w, bm.ctypes.data, fol.ctypes.data, first.ctypes.data,
                                           last.ctypes.data, prog.max_len or 0, prog.min_len, k, errs, pattern_id,
                                           flags | _lib.PM_REGULAR, len(prog.tree), tree.ctypes.data,
                                           tnull.ctypes.data, ctypes.byref(out)))
        return out
    check(_lib.load().pm_scan_nfa_wide(db.handle, prog.m, w, bm.ctypes.data, fol.ctypes.data, first.ctypes.data,
                                       last.ctypes.data, prog.max_len or 0, prog.min_len, k, errs, pattern_id,
                                       flags, ctypes.byref(out)))
    return out


def scan_nfa(db: SequenceDatabase, prog: Program, k: int, pattern_id: int = 0, types: str = "s",
             flags: int = None) -> Hits:
    """The automaton kernels (pm_scan_nfa_wide).  A class sequence at k = 0
    runs as nrgrep's simple engine (PM_CROSS_LINES: windows may span a line
    break when a class accepts '\\n'), as in the fixed-length kernel."""
    return _collect(nfa_launch(db, prog, k, pattern_id, types, flags))


def _same_automaton(a: Program, b: Program) -> bool:
    # (the regular engine's plan also depends on nrgrep's tree)
    return (a.classes == b.classes and a.follow == b.follow and a.first == b.first and a.last == b.last
            and a.anchor_start == b.anchor_start and a.anchor_end == b.anchor_end and a.tree == b.tree)


def scan(db: SequenceDatabase, progs: Sequence[Program], k: int = 0, types: str = "ids",
         report: str = REPORT_NRGREP, keep_headers: bool = False, start_anchor: bool = True):
    """Scan all programs; returns ([(beg, end) arrays per program], kernel_ms).

    ``report``: "nrgrep" (default) = exactly the matches nrgrep_coords prints
    (one run per program), "all" = every candidate start.
    ``keep_headers``: also return hits starting on a header line (they take
    part in the report rule; process_output drops them).  ``start_anchor``:
    False = no '^' check (the caller applies it).
    Programs equal as automata (a palindromic site and its reverse
    complement, e.g. GAATTC) are scanned once and their hits reported for
    each of them, as the reference's two nrgrep runs would.
    """
    types = parse_error_types(k, types)
    routes = [route(p, db.alphabet, k, types) for p in progs]
    canonical: List[int] = []
    for i, p in enumerate(progs):
        twin = next((j for j in range(i) if canonical[j] == j and _same_automaton(progs[j], p)), None)
        canonical.append(i if twin is None else twin)
    results: List[Optional[tuple]] = [None] * len(progs)
    total_ms = 0.0
    # one linear batch per distinct flag set (anchors are per program)
    groups = {}
    for i in range(len(progs)):
        if routes[i] == "linear" and canonical[i] == i:
            groups.setdefault(report_flags(progs[i], report, keep_headers, start_anchor), []).append(i)
    for flags, linear_ids in groups.items():
        hits = scan_linear(db, [progs[i] for i in linear_ids], k, flags)
        total_ms += hits.kernel_ms
        for slot, i in enumerate(linear_ids):
            results[i] = hits.for_pattern(slot)
    # the automaton scans are all launched before the first is collected
    # (PM_PIPELINED): each one's report pass runs while the host launches
    # the next scan
    nfa_ids = [i for i in range(len(progs)) if routes[i] == "nfa" and canonical[i] == i]
    handles = []
    try:
        for i in nfa_ids:
            handles.append(nfa_launch(db, progs[i], k, 0, types,
                                      report_flags(progs[i], report, keep_headers, start_anchor), pipelined=True))
    except BaseException:
        for h in handles:
            destroy_hits(h)
        raise
    for j, i in enumerate(nfa_ids):
        try:
            hits = _collect(handles[j])
        except BaseException:
            for h in handles[j + 1:]:
                destroy_hits(h)
            raise
        total_ms += hits.kernel_ms
        results[i] = (hits.beg, hits.end)
    for i in range(len(progs)):
        if results[i] is None:
            results[i] = results[canonical[i]]
    return results, total_ms
