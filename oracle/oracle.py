"""Python front-end of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  It wraps ``liboracle.so``
(``pm_oracle.c``: per-start forward NFA simulation) and also carries a tiny
pure-Python set-based restatement (``scan_py``) used to cross-check the C
code on small inputs.  Parity of the scan against the reference binary is
UNPINNED (``nrgrep_coords`` is prebuilt and cannot be run); the pattern
converter and host logic are pinned by ``tests/golden``.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

ERR_INS, ERR_DEL, ERR_SUB = 1, 2, 4


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    srcs = [os.path.join(_HERE, f) for f in ("pm_oracle.c", "pm_cpuscan.c", "pm_nrgrep.c", "pm_nrgrep_ext.c", "pm_nrgrep_reg.c",
                                              "Makefile")]
    if not os.path.exists(path) or os.path.getmtime(path) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        p64 = ctypes.POINTER(ctypes.c_int64)
        pu64 = ctypes.POINTER(ctypes.c_uint64)
        _LIB.pmo_scan.restype = ctypes.c_int64
        _LIB.pmo_scan.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_uint64,
                                  ctypes.c_uint64, pu64, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, p64, p64, ctypes.c_int64]
        _LIB.pmo_scan2.restype = ctypes.c_int64
        _LIB.pmo_scan2.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_uint64,
                                   ctypes.c_uint64, pu64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, p64, p64, ctypes.c_int64]
        _LIB.pmc_ids_scan.restype = ctypes.c_int64
        _LIB.pmc_ids_scan.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                      ctypes.c_int64]
        _LIB.pmc_shiftadd.restype = ctypes.c_int64
        _LIB.pmc_shiftadd.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, p64, ctypes.c_int64]
        _LIB.pmn_plan.restype = ctypes.c_int
        _LIB.pmn_plan.argtypes = [pu64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        _LIB.pmn_esimple.restype = ctypes.c_int64
        _LIB.pmn_esimple.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, p64, p64, ctypes.c_int64]
        _LIB.pmx_plan.restype = ctypes.c_int
        _LIB.pmx_plan.argtypes = [pu64, ctypes.c_int, pu64, pu64, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        _LIB.pmx_extended.restype = ctypes.c_int64
        _LIB.pmx_extended.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_int, pu64, pu64, ctypes.c_int,
                                      ctypes.c_int, p64, p64, ctypes.c_int64]
        _LIB.pmx_eplan.restype = ctypes.c_int
        _LIB.pmx_eplan.argtypes = [pu64, ctypes.c_int, ctypes.c_int, pu64, pu64, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int)]
        _LIB.pmx_eextended.restype = ctypes.c_int64
        _LIB.pmx_eextended.argtypes = [ctypes.c_char_p, ctypes.c_int64, pu64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, pu64, pu64, ctypes.c_int, ctypes.c_int, p64, p64,
                                       ctypes.c_int64]
        pi32 = ctypes.POINTER(ctypes.c_int32)
        _LIB.pmr_plan.restype = ctypes.c_int
        _LIB.pmr_plan.argtypes = [pi32, pi32, ctypes.c_int, pu64, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int), pu64]
        _LIB.pmr_regular.restype = ctypes.c_int64
        _LIB.pmr_regular.argtypes = [ctypes.c_char_p, ctypes.c_int64, pi32, pi32, ctypes.c_int, pu64, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, p64, p64, ctypes.c_int64]
        _LIB.pmr_eplan.restype = ctypes.c_int
        _LIB.pmr_eplan.argtypes = [pi32, pi32, ctypes.c_int, pu64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.POINTER(ctypes.c_int), pu64]
        _LIB.pmr_eregular.restype = ctypes.c_int64
        _LIB.pmr_eregular.argtypes = [ctypes.c_char_p, ctypes.c_int64, pi32, pi32, ctypes.c_int, pu64, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, p64, p64,
                                      ctypes.c_int64]
        _LIB.pmo_index.restype = ctypes.c_int64
        _LIB.pmo_index.argtypes = [ctypes.c_char_p, ctypes.c_int64, p64, p64, p64, p64,
                                   ctypes.c_int64]
    return _LIB


def err_flags(types: str) -> int:
    return (ERR_INS if "i" in types else 0) | (ERR_DEL if "d" in types else 0) | \
           (ERR_SUB if "s" in types else 0)


def header_spans(text: bytes):
    """[beg, end) of every header line (/^>\\S/, generate_sequence_index.pl:33)."""
    spans = []
    for off, name in record_index(text):
        if name.startswith(">"):
            nl = text.find(b"\n", off)
            spans.append((off, len(text) if nl < 0 else nl))
    return spans


def drop_header_hits(text: bytes, hits):
    """Remove hits starting on a header line, its terminating '\n' included:
    process_output maps such a start to the '>name' record offset
    (get_name_offset, patmatch.py:214-238) and discards it (:548-550)."""
    hits = [h for h in hits if h[0] >= 0]   # eextended: a start before the file (its first byte read, pm_nrgrep_ext.c)
    spans = header_spans(text)
    if not spans:
        return hits
    import bisect
    starts = [b for b, _ in spans]
    out = []
    for beg, end in hits:
        i = bisect.bisect_right(starts, beg) - 1
        if i >= 0 and spans[i][0] <= beg <= spans[i][1]:
            continue
        out.append((beg, end))
    return out


PMO_NRGREP, PMO_START, PMO_END, PMO_SIMPLE = 1, 2, 4, 8

# nrgrep_coords -b 1600000 (patmatch.py:733-743): buffers of 1,600,000 bytes
# (main() stores atoi(optarg), 0x401162; bufCreate mallocs that, 0x41bb6b)
NRGREP_BUFFER = 1600000


def regions(text: bytes, bufsize: int = NRGREP_BUFFER):
    """The regions recSearchFile (0x402250) searches: a full buffer up to and
    including its last '\n' (simpleRevSearch 0x402475), the next buffer
    loaded from that '\n' (bufLoad 0x4023e6 with r13 = its start); with no
    '\n' in it (or only at its start) the whole buffer, the next one after
    it (0x4024a0 -> 0x4022ba); the last buffer (not full: bufEof 0x41bfc0)
    to the end of the file.  [(beg, end)]."""
    out, at, n = [], 0, len(text)
    while True:
        if not bufsize or at + bufsize > n:
            out.append((at, n))
            return out
        d = text.rfind(b"\n", at, at + bufsize)
        if d > at:
            out.append((at, d + 1))
            at = d
        else:
            out.append((at, at + bufsize))
            at += bufsize
        if at >= n:
            return out


def by_region(text: bytes, scan_one, skip_headers: bool, bufsize: int = NRGREP_BUFFER, threads: int = 1,
              regs=None):
    """recSearchFile's loop: every region searched as a text of its own (its
    start is R, its end the end of the text), the printed matches in file
    order -- a match over a region's last '\n' is found in both regions and
    printed twice, as the binary does.  Header-line starts are dropped with
    the whole file as context."""
    regs = regions(text, bufsize) if regs is None else [(int(a), int(b)) for a, b in regs]
    if len(regs) == 1:
        hits = scan_one(text)
    else:
        def one(r):
            a, b = r
            return [(x + a, y + a) for x, y in scan_one(text[a:b])]
        if threads > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=threads) as ex:
                parts = list(ex.map(one, regs))
        else:
            parts = [one(r) for r in regs]
        hits = [h for part in parts for h in part]
    return drop_header_hits(text, hits) if skip_headers else hits


def mode_of(prog, k: int, report: str = "nrgrep", simple=None) -> int:
    """pmo_scan2 mode bits for a compiled program: nrgrep's engine choice
    (simple = k 0 + class sequence, searchPreproc 0x402660), the anchors and
    the report rule ("nrgrep" / "leftmost": first found = leftmost start)."""
    m = PMO_NRGREP if report in ("nrgrep", "leftmost") else 0
    if prog.anchor_start:
        m |= PMO_START
    if prog.anchor_end:
        m |= PMO_END
    if (k == 0 and prog.linear) if simple is None else simple:
        m |= PMO_SIMPLE
    return m


def scan_candidates(text: bytes, prog, k: int = 0, types: str = "ids", bufsize: int = NRGREP_BUFFER, regs=None):
    """Every start with a match under nrgrep's engine choice (shortest end;
    '$' applied, '^' not, header-line starts kept), region by region: what
    the sharded scan re-chains when a report crosses into the next piece."""
    m = mode_of(prog, k, "all") & ~PMO_START
    return scan_reported(text, prog, k, types, mode=m, bufsize=bufsize, regs=regs)


def scan_reported(text: bytes, prog, k: int = 0, types: str = "ids", skip_headers: bool = False,
                  report: str = "nrgrep", simple=None, mode=None, bufsize: int = NRGREP_BUFFER, regs=None):
    """What ``nrgrep_coords`` prints for ``prog``.  A class sequence at
    k > 0 runs nrgrep's esimple engine (``scan_esimple``, pm_nrgrep.c: its
    own candidate order and verify).  Everything else (pmo_scan2): the
    candidates of ``scan`` (or the simple engine's whole-text windows at
    k = 0) reduced by the binary's report rule -- first found wins, the
    scan resumes at the match end -- and its '^'/'$' checks, the first found
    being the leftmost start (``report="leftmost"`` forces that rule for a
    class sequence too).  ``skip_headers`` then drops the header-line hits
    process_output throws away.  ``simple`` overrides the engine choice
    (False: line-bounded windows even at k = 0).  The file is searched in
    nrgrep's regions (``regions``: buffers of ``bufsize`` bytes; 0 = one)."""
    if report == "nrgrep" and simple is None and mode is None and k > 0 and is_esimple(prog):
        return scan_esimple(text, prog, k, types, skip_headers, bufsize, regs)
    if report == "nrgrep" and simple is None and mode is None and k == 0 and prog.kind == "extended":
        return scan_extended(text, prog, skip_headers, bufsize, regs)
    if report == "nrgrep" and simple is None and mode is None and k > 0 and prog.kind == "extended":
        return scan_eextended(text, prog, k, types, skip_headers, bufsize, regs)
    if report == "nrgrep" and simple is None and mode is None and k == 0 and prog.kind == "regular":
        return scan_regular(text, prog, skip_headers, bufsize, regs)
    if report == "nrgrep" and simple is None and mode is None and k > 0 and prog.kind == "regular":
        return scan_eregular(text, prog, k, types, skip_headers, bufsize, regs)
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_reported(t, prog, k, types, False, report, simple, mode, 0),
                         skip_headers, bufsize, regs=regs)
    L = lib()
    B = np.array(prog.byte_masks(), dtype=np.uint64)
    F = np.array(prog.follow + [0], dtype=np.uint64)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = L.pmo_scan2(text, len(text), B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                        prog.first, prog.last, F.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                        prog.m, k, err_flags(types) if k else 0, 1 if prog.ignore_case else 0,
                        mode_of(prog, k, report, simple) if mode is None else mode,
                        beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                        end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("oracle rejected k=%d" % k)
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def scan(text: bytes, prog, k: int = 0, types: str = "ids", skip_headers: bool = False):
    """All (beg, end) hits of compiled program ``prog`` in ``text`` (what
    nrgrep_coords prints); ``skip_headers`` drops the header-line hits that
    the reference's process_output throws away."""
    L = lib()
    B = np.array(prog.byte_masks(), dtype=np.uint64)
    F = np.array(prog.follow + [0], dtype=np.uint64)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = L.pmo_scan(text, len(text), B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                       prog.first, prog.last, F.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                       prog.m, k, err_flags(types) if k else 0, 1 if prog.ignore_case else 0,
                       beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                       end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("oracle rejected k=%d" % k)
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def scan_threads(text: bytes, prog, k: int = 0, types: str = "ids", skip_headers: bool = False,
                 threads: int = 1, report: str = None):
    """``scan`` over ``threads`` host threads: the text is cut after line
    breaks (no hit spans a '\\n'; header lines stay whole, so
    the header filter is unchanged -- and a database decoded from HBM renders
    headers as '\\n' bytes, so it has no '>' to cut at), each piece is scanned by
    ``pmo_scan`` (ctypes releases the GIL) and the hits are shifted back to
    file offsets.  Same output as ``scan``; used for the bench's CPU baseline."""
    def one_piece(t):
        if report is None:
            return scan(t, prog, k, types, skip_headers)
        return scan_reported(t, prog, k, types, skip_headers, report)
    if report is not None and len(text) >= NRGREP_BUFFER:
        # nrgrep's regions are independent searches: one per task
        return by_region(text, lambda t: scan_reported(t, prog, k, types, False, report, bufsize=0),
                         skip_headers, NRGREP_BUFFER, threads)
    # the simple engine's windows may span a line break: no cut is safe
    cross = report is not None and k == 0 and prog.linear and any(10 in c for c in prog.classes)
    if threads <= 1 or len(text) < (1 << 20) or cross or prog.anchor_start:
        return one_piece(text)
    from concurrent.futures import ThreadPoolExecutor
    cuts = [0]
    step = len(text) // threads
    for t in range(1, threads):
        c = text.find(b"\n", max(cuts[-1], t * step))
        if c < 0:
            break
        if c + 1 > cuts[-1]:
            cuts.append(c + 1)
    cuts.append(len(text))
    pieces = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def one(span):
        a, b = span
        return [(x + a, y + a) for x, y in one_piece(text[a:b])]

    with ThreadPoolExecutor(max_workers=len(pieces)) as ex:
        parts = list(ex.map(one, pieces))
    return [h for part in parts for h in part]


def record_index(text: bytes):
    """generate_sequence_index.pl restated: [(offset, name)] in file order."""
    L = lib()
    cap = max(16, text.count(b">") + 1)
    arrs = [np.empty(cap, dtype=np.int64) for _ in range(4)]
    n = L.pmo_index(text, len(text), *[a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) for a in arrs], cap)
    out = []
    hdr, data, nb, nl = (a[:n].tolist() for a in arrs)
    for h, d, b, ln in zip(hdr, data, nb, nl):
        name = text[b:b + ln].decode("latin-1")
        out.append((h, ">" + name))
        out.append((d, name))
    return out


# ---------------------------------------------------------------------------
# nrgrep's esimple engine (pm_nrgrep.c): the -k <k><ids> path of a class
# sequence, restated from the binary's disassembly
# ---------------------------------------------------------------------------

def is_esimple(prog) -> bool:
    """nrgrep's esimple engine (searchPreproc 0x402710): a plain class
    sequence (detClass 1) searched with errors."""
    return prog.linear and prog.kind == "simple"


def wide_masks(prog) -> np.ndarray:
    """[256][4] uint64 position sets (bit i = position i accepts the folded
    byte), up to 256 positions."""
    B = np.zeros((256, 4), dtype=np.uint64)
    for i, cls in enumerate(prog.classes):
        for b in cls:
            B[b, i >> 6] |= np.uint64(1 << (i & 63))
    return B


def nrgrep_plan(prog, k: int):
    """nrgrep's scan plan for ``prog`` at k errors (esimplePreproc): a dict
    with ``type`` (1 pieces, 2 backward window, 3 forward window),
    ``piece_len``, ``window`` and ``L`` (left length of every piece)."""
    B = wide_masks(prog)
    out = (ctypes.c_int * 24)()
    n = lib().pmn_plan(B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), prog.m, k,
                       1 if prog.ignore_case else 0, out)
    if n < 0:
        raise ValueError("no esimple plan for m=%d k=%d" % (prog.m, k))
    return {"type": out[0], "piece_len": out[1], "window": (out[2], out[3]),
            "L": [out[4 + i] for i in range(n)]}


def scan_esimple(text: bytes, prog, k: int, types: str = "ids", skip_headers: bool = False,
                 bufsize: int = NRGREP_BUFFER, regs=None):
    """What nrgrep_coords prints for a class sequence at k > 0 (pmn_esimple:
    nrgrep's own scanners, record lookup, two-phase verify and report rule),
    region by region (``regions``)."""
    if not prog.linear or k < 1:
        raise ValueError("scan_esimple needs a class sequence and k > 0")
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_esimple(t, prog, k, types, False, 0), skip_headers, bufsize,
                         regs=regs)
    B = wide_masks(prog)
    mode = (PMO_START if prog.anchor_start else 0) | (PMO_END if prog.anchor_end else 0)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = lib().pmn_esimple(text, len(text), B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), prog.m, k,
                              err_flags(types), 1 if prog.ignore_case else 0, mode,
                              beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                              end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pmn_esimple rejected m=%d k=%d" % (prog.m, k))
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


# ---------------------------------------------------------------------------
# nrgrep's extended engine at k = 0 (pm_nrgrep_ext.c): classes with '?*+',
# restated from the binary's disassembly
# ---------------------------------------------------------------------------

def _mask_words(x: int) -> np.ndarray:
    return np.array([(x >> (64 * q)) & 0xFFFFFFFFFFFFFFFF for q in range(4)], dtype=np.uint64)


def extended_plan(prog):
    """nrgrep's extendedPreproc plan for ``prog`` (pmx_plan): ``type`` 2 = a
    window scanned backward, 3 = the prefix scanned forward; ``window``
    [beg, end); ``L`` = the left part's length; ``simple`` = the window holds
    no '?*+' (simpleScan)."""
    if prog.kind != "extended":
        raise ValueError("not an extended pattern: %s" % prog.source)
    B = wide_masks(prog)
    out = (ctypes.c_int * 8)()
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    opt, rep = _mask_words(prog.opt_mask), _mask_words(prog.rep_mask)
    if lib().pmx_plan(B.ctypes.data_as(pu64), prog.m, opt.ctypes.data_as(pu64), rep.ctypes.data_as(pu64),
                      1 if prog.ignore_case else 0, out) < 0:
        raise ValueError("no extended plan for %s" % prog.source)
    return {"type": out[0], "fwd": out[1], "window": (out[2], out[3]), "L": out[4], "simple": bool(out[5])}


def scan_extended(text: bytes, prog, skip_headers: bool = False, bufsize: int = NRGREP_BUFFER, regs=None):
    """What nrgrep_coords prints for a class-2 pattern at k = 0 (pmx_extended:
    nrgrep's plan, scanners, two-phase verify and report rule), region by
    region (``regions``)."""
    if prog.kind != "extended":
        raise ValueError("scan_extended needs an extended pattern")
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_extended(t, prog, False, 0), skip_headers, bufsize, regs=regs)
    B = wide_masks(prog)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    opt, rep = _mask_words(prog.opt_mask), _mask_words(prog.rep_mask)
    mode = (PMO_START if prog.anchor_start else 0) | (PMO_END if prog.anchor_end else 0)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = lib().pmx_extended(text, len(text), B.ctypes.data_as(pu64), prog.m, opt.ctypes.data_as(pu64),
                               rep.ctypes.data_as(pu64), 1 if prog.ignore_case else 0, mode,
                               beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pmx_extended rejected %s" % prog.source)
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def eextended_plan(prog, k: int):
    """nrgrep's eextendedPreproc plan for ``prog`` at k errors (pmx_eplan):
    ``type`` 1 = k + 1 pieces, 2 = a window scanned backward, 3 = the prefix
    scanned forward; ``simple`` = the scanned positions hold no '?*+' (the
    esimple scanners); ``pieces`` = [(off, end)] (the window / prefix for
    types 2 and 3); ``plen`` = the pieces' length in characters (type 1),
    ``fwd`` = the window's (type 2); ``window`` = extendedFindBest's."""
    if prog.kind != "extended":
        raise ValueError("not an extended pattern: %s" % prog.source)
    B = wide_masks(prog)
    out = (ctypes.c_int * (6 + 2 * 17))()
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    opt, rep = _mask_words(prog.opt_mask), _mask_words(prog.rep_mask)
    if lib().pmx_eplan(B.ctypes.data_as(pu64), prog.m, k, opt.ctypes.data_as(pu64), rep.ctypes.data_as(pu64),
                       1 if prog.ignore_case else 0, out) < 0:
        raise ValueError("no eextended plan for %s at k=%d" % (prog.source, k))
    np_ = out[2]
    return {"type": out[0], "simple": bool(out[1]), "plen": out[3] if out[0] == 1 else 0,
            "fwd": out[3] if out[0] != 1 else 0, "window": (out[4], out[5]),
            "pieces": [(out[6 + 2 * i], out[7 + 2 * i]) for i in range(np_)]}


def scan_eextended(text: bytes, prog, k: int, types: str = "ids", skip_headers: bool = False,
                   bufsize: int = NRGREP_BUFFER, regs=None):
    """What nrgrep_coords prints for a class-2 pattern at k > 0 (pmx_eextended:
    nrgrep's eextended plan, scanners, checkMatch1 and report rule), region
    by region (``regions``)."""
    if prog.kind != "extended" or k < 1:
        raise ValueError("scan_eextended needs an extended pattern and k > 0")
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_eextended(t, prog, k, types, False, 0), skip_headers, bufsize,
                         regs=regs)
    B = wide_masks(prog)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    opt, rep = _mask_words(prog.opt_mask), _mask_words(prog.rep_mask)
    mode = (PMO_START if prog.anchor_start else 0) | (PMO_END if prog.anchor_end else 0)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = lib().pmx_eextended(text, len(text), B.ctypes.data_as(pu64), prog.m, k, err_flags(types),
                                opt.ctypes.data_as(pu64), rep.ctypes.data_as(pu64), 1 if prog.ignore_case else 0,
                                mode, beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pmx_eextended rejected %s at k=%d" % (prog.source, k))
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


# ---------------------------------------------------------------------------
# nrgrep's regular engine at k = 0 (pm_nrgrep_reg.c): '|' and repeated
# groups, restated from the binary's disassembly
# ---------------------------------------------------------------------------

def _tree_arrays(prog):
    pi32 = ctypes.POINTER(ctypes.c_int32)
    tree = np.array([v for node in prog.tree for v in node], dtype=np.int32)
    null = np.array(prog.tree_nullable, dtype=np.int32)
    return tree, null, tree.ctypes.data_as(pi32), null.ctypes.data_as(pi32)


def regular_plan(prog):
    """nrgrep's regularPreproc plan for ``prog`` (pmr_plan): ``type`` 2 = a
    window of ``ell`` characters scanned backward, 3 = the automaton scanned
    forward; ``cls`` = detClass of the window (1 / 2: the binary never prints
    a match, pm_nrgrep_reg.c); ``window`` / ``init`` / ``final`` = state sets
    (nrgrep numbering: position + 1); ``states`` = the window's m'."""
    if prog.kind != "regular":
        raise ValueError("not a regular pattern: %s" % prog.source)
    B = wide_masks(prog)
    tree, null, tp, np_ = _tree_arrays(prog)
    out = (ctypes.c_int * 4)()
    masks = np.zeros(15, dtype=np.uint64)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    if lib().pmr_plan(tp, np_, len(prog.tree), B.ctypes.data_as(pu64), prog.m, 1 if prog.ignore_case else 0, out,
                      masks.ctypes.data_as(pu64)) < 0:
        raise ValueError("no regular plan for %s" % prog.source)

    def as_int(ws):
        return sum(int(w) << (64 * q) for q, w in enumerate(ws))
    return {"type": out[0], "ell": out[1], "cls": out[2], "states": out[3], "window": as_int(masks[0:5]),
            "init": as_int(masks[5:10]), "final": as_int(masks[10:15])}


def scan_regular(text: bytes, prog, skip_headers: bool = False, bufsize: int = NRGREP_BUFFER, regs=None):
    """What nrgrep_coords prints for a class-3 pattern at k = 0 (pmr_regular:
    nrgrep's plan, regularScan, checkMatch and report rule), region by
    region (``regions``)."""
    if prog.kind != "regular":
        raise ValueError("scan_regular needs a regular pattern")
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_regular(t, prog, False, 0), skip_headers, bufsize, regs=regs)
    B = wide_masks(prog)
    tree, null, tp, np_ = _tree_arrays(prog)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    mode = (PMO_START if prog.anchor_start else 0) | (PMO_END if prog.anchor_end else 0)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = lib().pmr_regular(text, len(text), tp, np_, len(prog.tree), B.ctypes.data_as(pu64), prog.m,
                              1 if prog.ignore_case else 0, mode, beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                              end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pmr_regular rejected %s" % prog.source)
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def eregular_plan(prog, k: int, types: str = "ids"):
    """nrgrep's eregularPreproc plan for ``prog`` at ``k`` errors (pmr_eplan):
    ``type`` 1 = K + 1 pieces of ``ell`` characters found exactly, 2 = a
    window of ``ell`` characters scanned backward with k errors, 3 = the
    automaton forward; ``cls`` = detClass of the first window (1: esimple's
    scanners, 2: the binary dies, nothing prints); ``windows`` = [(window,
    init, final)] state sets (nrgrep numbering); ``match`` = checkMatch's
    state word for class 1; ``defined`` = False when nrgrep reads memory it
    never wrote for this plan (pm_nrgrep_reg.c, parity unpinned)."""
    if prog.kind != "regular":
        raise ValueError("not a regular pattern: %s" % prog.source)
    B = wide_masks(prog)
    tree, null, tp, np_ = _tree_arrays(prog)
    out = (ctypes.c_int * 6)()
    nw = 5   # PMR_NW
    masks = np.zeros((3 * 17 + 1) * nw, dtype=np.uint64)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    if lib().pmr_eplan(tp, np_, len(prog.tree), B.ctypes.data_as(pu64), prog.m, 1 if prog.ignore_case else 0, k,
                       err_flags(types), out, masks.ctypes.data_as(pu64)) < 0:
        raise ValueError("no eregular plan for %s at k=%d" % (prog.source, k))
    def word_set(j):
        return sum(int(masks[j * nw + q]) << (64 * q) for q in range(nw))
    wins = [(word_set(3 * i), word_set(3 * i + 1), word_set(3 * i + 2)) for i in range(out[5])]
    return {"type": out[0], "ell": out[1], "cls": out[2], "states": out[3], "defined": bool(out[4]),
            "windows": wins, "match": int(masks[51 * nw])}


def scan_eregular(text: bytes, prog, k: int, types: str = "ids", skip_headers: bool = False,
                  bufsize: int = NRGREP_BUFFER, regs=None):
    """What nrgrep_coords prints for a class-3 pattern at k > 0 (pmr_eregular:
    nrgrep's eregular plan, its scanners, checkMatch and report rule), region
    by region (``regions``).  Automata of up to 319 positions."""
    if prog.kind != "regular":
        raise ValueError("scan_eregular needs a regular pattern")
    if regs is not None or (bufsize and len(text) >= bufsize):
        return by_region(text, lambda t: scan_eregular(t, prog, k, types, False, 0), skip_headers, bufsize,
                         regs=regs)
    B = wide_masks(prog)
    tree, null, tp, np_ = _tree_arrays(prog)
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    mode = (PMO_START if prog.anchor_start else 0) | (PMO_END if prog.anchor_end else 0)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = lib().pmr_eregular(text, len(text), tp, np_, len(prog.tree), B.ctypes.data_as(pu64), prog.m,
                               1 if prog.ignore_case else 0, mode, k, err_flags(types),
                               beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pmr_eregular rejected %s at k=%d" % (prog.source, k))
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


# ---------------------------------------------------------------------------
# pure-Python restatement (explicit (position, errors) state sets), small n
# ---------------------------------------------------------------------------

def scan_py(text: bytes, prog, k: int = 0, types: str = "ids", to_line_end: bool = False):
    """Every start of a line-bounded match and its shortest end (any number
    of positions); ``to_line_end``: the end must be the line end ('$')."""
    types = types if k else ""
    fold = (lambda c: c - 32 if 97 <= c <= 122 else c) if prog.ignore_case else (lambda c: c)
    START = -1

    def succ(state):
        if state == START:
            return [i for i in range(prog.m) if prog.first >> i & 1]
        return [i for i in range(prog.m) if prog.follow[state] >> i & 1]

    def closure(states):
        out, todo = dict(states), list(states.items())
        while todo:
            st, e = todo.pop()
            if "d" in types and e < k:
                for nx in succ(st):
                    if out.get(nx, k + 1) > e + 1:
                        out[nx] = e + 1
                        todo.append((nx, e + 1))
        return out

    hits = []
    pos = 0
    for line in text.split(b"\n"):
        for s in range(len(line)):
            cur = closure({START: 0})
            for p in range(s, len(line)):
                c = fold(line[p])
                nxt = {}

                def put(st, e):
                    if e <= k and nxt.get(st, k + 1) > e:
                        nxt[st] = e
                for st, e in cur.items():
                    for nx in succ(st):
                        if c in prog.classes[nx]:
                            put(nx, e)
                        elif "s" in types:
                            put(nx, e + 1)
                    if "i" in types:
                        put(st, e + 1)
                cur = closure(nxt)
                if any(st != START and prog.last >> st & 1 for st in cur) and (not to_line_end or p + 1 == len(line)):
                    hits.append((pos + s, pos + p + 1))
                    break
                if not cur:
                    break
        pos += len(line) + 1
    return hits


def scan_py_reported(text: bytes, prog, k: int = 0, types: str = "ids", skip_headers: bool = False):
    """What nrgrep_coords prints for a line-bounded engine (k > 0, or k = 0
    with no class accepting '\n'), restated in pure Python for automata of
    any size (pm_oracle.c holds 64 positions): the candidates of scan_py,
    the report rule (first found wins, resume at its end) and the '^'
    check (a line start or the resume point, pmo_scan2).  A class sequence
    at k > 0 is nrgrep's esimple engine: ``scan_esimple`` (256 positions)."""
    if k > 0 and is_esimple(prog):
        return scan_esimple(text, prog, k, types, skip_headers)
    out, R = [], 0
    for b, e in scan_py(text, prog, k, types, to_line_end=prog.anchor_end):
        if b < R:
            continue
        if prog.anchor_start and not (b == R or b == 0 or text[b - 1] == 10):
            continue
        out.append((b, e))
        R = e
    return drop_header_hits(text, out) if skip_headers else out


# ---------------------------------------------------------------------------
# bit-parallel CPU scan (pm_cpuscan.c): the bench's CPU baseline
# ---------------------------------------------------------------------------

def shiftadd_scan(text: bytes, prog, k: int, skip_headers: bool = False):
    """Reported windows of a fixed-length class sequence with <= k
    substitutions, by the Shift-Add bit-parallel automaton (pm_cpuscan.c);
    same output as ``scan_reported(text, prog, k, "s")``."""
    if not prog.linear:
        raise ValueError("shiftadd_scan needs a class sequence")
    L = lib()
    B = np.array(prog.byte_masks(), dtype=np.uint64)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        n = L.pmc_shiftadd(text, len(text), B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), prog.m, k,
                           1 if prog.ignore_case else 0, beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("pattern too long for one Shift-Add word (m=%d, k=%d)" % (prog.m, k))
        if n <= cap:
            hits = [(b, b + prog.m) for b in beg[:n].tolist()]
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def shiftadd_threads(text: bytes, prog, k: int, skip_headers: bool = False, threads: int = 1):
    """``shiftadd_scan`` over host threads, the text cut after line breaks
    (k > 0: windows never span one, so the pieces are independent)."""
    if threads <= 1 or k == 0 or len(text) < (1 << 20):
        return shiftadd_scan(text, prog, k, skip_headers)
    from concurrent.futures import ThreadPoolExecutor
    cuts = [0]
    step = len(text) // threads
    for t in range(1, threads):
        c = text.find(b"\n", max(cuts[-1], t * step))
        if c < 0:
            break
        if c + 1 > cuts[-1]:
            cuts.append(c + 1)
    cuts.append(len(text))
    pieces = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def one(span):
        a, b = span
        return [(x + a, y + a) for x, y in shiftadd_scan(text[a:b], prog, k, skip_headers)]

    with ThreadPoolExecutor(max_workers=len(pieces)) as ex:
        parts = list(ex.map(one, pieces))
    return [h for part in parts for h in part]


def ids_scan(text: bytes, prog, k: int, types: str = "ids", skip_headers: bool = False):
    """Reported matches of a class sequence with <= k insertions / deletions /
    substitutions by the bit-parallel Wu-Manber recurrence (pm_cpuscan.c
    pmc_ids_scan: reverse pass for starts, forward pass for the shortest
    end, report rule); same output as ``scan_reported(text, prog, k, types)``
    for k > 0."""
    if not prog.linear or k < 1:
        raise ValueError("ids_scan needs a class sequence and k > 0")
    L = lib()
    B = np.array(prog.byte_masks(), dtype=np.uint64)
    cap = 1 << 16
    while True:
        beg = np.empty(cap, dtype=np.int64)
        end = np.empty(cap, dtype=np.int64)
        n = L.pmc_ids_scan(text, len(text), B.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), prog.m, k,
                           err_flags(types), 1 if prog.ignore_case else 0,
                           beg.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                           end.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap)
        if n < 0:
            raise ValueError("shape not covered by pmc_ids_scan (m=%d, k=%d)" % (prog.m, k))
        if n <= cap:
            hits = list(zip(beg[:n].tolist(), end[:n].tolist()))
            return drop_header_hits(text, hits) if skip_headers else hits
        cap = int(n)


def ids_threads(text: bytes, prog, k: int, types: str = "ids", skip_headers: bool = False, threads: int = 1):
    """``ids_scan`` over host threads, the text cut after line breaks (the
    e* engines' matches never span one, so the pieces are independent)."""
    if threads <= 1 or len(text) < (1 << 20):
        return ids_scan(text, prog, k, types, skip_headers)
    from concurrent.futures import ThreadPoolExecutor
    cuts = [0]
    step = len(text) // threads
    for t in range(1, threads):
        c = text.find(b"\n", max(cuts[-1], t * step))
        if c < 0:
            break
        if c + 1 > cuts[-1]:
            cuts.append(c + 1)
    cuts.append(len(text))
    pieces = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def one(span):
        a, b = span
        return [(x + a, y + a) for x, y in ids_scan(text[a:b], prog, k, types, skip_headers)]

    with ThreadPoolExecutor(max_workers=len(pieces)) as ex:
        parts = list(ex.map(one, pieces))
    return [h for part in parts for h in part]
