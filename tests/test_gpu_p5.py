"""The 5-bit residue planes of BYTE (peptide) databases (pm_db::p5,
k_p5_linear): class sequences at k = 0..3 substitutions scanned on the
planes report what the byte kernel and the oracle report (nrgrep's simple /
esimple engines, patmatch.py:733-743 with -p patterns), on proteome-shaped
FASTA with headers, ragged lines, lower case, X / B / Z / '*', and on files
with more than 30 distinct bytes besides '\\n' (no planes: the byte copy
is scanned).  At k = 0 a class that takes '\\n' ('X', a negated class)
lets nrgrep's simple engine match across lines: '\\n' is then a residue
of its own and the windows over header bytes are checked on the file's
bytes (k_p5_cross_fix)."""
import random

import pytest

from patmatchdocker_amd import _lib
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

pytestmark = pytest.mark.gpu

AA = "ACDEFGHIKLMNPQRSTVWY"


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import engine as eng
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def proteome(rng, n_records=40, extra="XBZ*", lower=0.05):
    recs = []
    for r in range(n_records):
        n = rng.randint(1, 900)
        seq = []
        for _ in range(n):
            x = rng.random()
            c = rng.choice(extra) if x < 0.02 else rng.choice("CCKLGST" if x < 0.3 else AA)
            seq.append(c.lower() if rng.random() < lower else c)
        s = "".join(seq)
        w = rng.choice([60, 70, 1000])
        recs.append(">YP%04d protein %d\n%s\n" % (r, r, "\n".join(s[i:i + w] for i in range(0, len(s), w))))
    return "".join(recs).encode()


PATTERNS = ["CXXC", "C-x(2)-C", "[LIVM]XXG", "RGD", "NX[ST]", "CX{3}[LIVMFYWC]", "GXGXXG", "KK",
            "[ST]X[RK]", "CC", "W", "C-x-[DN]-x(4)-[FY]-x-C-x-C", "LXXLL"]


def _progs():
    progs = []
    for p in PATTERNS:
        prog = compile_pattern(convert("-p", p))
        if prog.kind == "simple" and prog.m <= _lib.PM_MAX_LINEAR_POSITIONS:
            progs.append(prog)
    assert len(progs) >= 10
    return progs


def _pairs(r):
    return list(zip(r[0].tolist(), r[1].tolist()))


def _launch(engine, db, progs, k, flags):
    batch = engine.LinearBatch(progs)
    h = engine._collect(batch.launch(db, k, flags=flags))
    out = []
    for i in range(len(progs)):
        sel = h.pattern == i
        out.append(list(zip(h.beg[sel].tolist(), h.end[sel].tolist())))
    return out


@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_planes_match_the_oracle(engine, oracle_mod, k):
    rng = random.Random(50 + k)
    text = proteome(rng)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        n_codes, table = db.residue_codes()
        assert 20 <= n_codes <= 31
        assert table[ord("\n")] == 1 and table[ord("A")] > 1   # 0: header bytes
        progs = _progs()
        res, _ = engine.scan(db, progs, k=k, types="s")
        for prog, r in zip(progs, res):
            assert _pairs(r) == oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True), (prog.source, k)
    finally:
        db.close()


@pytest.mark.parametrize("k", [0, 2])
def test_planes_equal_the_byte_kernel(engine, k):
    """Every candidate (PM_REPORT_ALL, headers kept) of the plane kernel
    equals the byte kernel's on the same database."""
    rng = random.Random(70 + k)
    text = proteome(rng, n_records=60)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        progs = _progs()
        base = _lib.PM_REPORT_ALL | _lib.PM_KEEP_HEADERS
        planes = _launch(engine, db, progs, k, base)
        direct = _launch(engine, db, progs, k, base | _lib.PM_SCAN_BYTES)
        assert planes == direct
        assert sum(len(x) for x in planes) > 100
    finally:
        db.close()


def test_long_patterns_and_many_classes(engine, oracle_mod):
    """Patterns over 32 positions (three plane words per lane) and a batch
    with 16 distinct classes."""
    rng = random.Random(91)
    text = proteome(rng, n_records=30, lower=0.0)
    classes = ["[%s]" % "".join(rng.sample(AA, rng.randint(1, 12))) for _ in range(16)]
    pats = ["".join(rng.choice(classes + ["X"]) for _ in range(rng.randint(33, 60))) for _ in range(3)]
    pats.append("".join(classes))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        progs = [compile_pattern(convert("-p", p)) for p in pats]
        progs = [p for p in progs if p.kind == "simple" and p.m <= _lib.PM_MAX_LINEAR_POSITIONS]
        assert len(progs) >= 3
        for k in (2, 3):
            res, _ = engine.scan(db, progs, k=k, types="s")
            for prog, r in zip(progs, res):
                assert _pairs(r) == oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True), (prog.source, k)
    finally:
        db.close()


def test_more_than_31_distinct_bytes_scans_the_byte_copy(engine, oracle_mod):
    rng = random.Random(7)
    text = proteome(rng, n_records=20, extra="XBZ*0123456789#%&", lower=0.0)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        assert db.residue_codes()[0] == 0
        progs = _progs()
        res, _ = engine.scan(db, progs, k=1, types="s")
        for prog, r in zip(progs, res):
            assert _pairs(r) == oracle_mod.scan_reported(text, prog, 1, "s", skip_headers=True), prog.source
    finally:
        db.close()


def test_nucleotide_databases_have_no_residue_planes(engine):
    db = engine.SequenceDatabase.from_bytes(b">a\nACGTNACGT\n", alphabet=engine.NUC, device=0)
    try:
        assert db.residue_codes()[0] == 0
    finally:
        db.close()


def test_cross_line_windows_over_headers(engine, oracle_mod):
    """k = 0 with 'X': windows across '\\n' and into header lines whose
    text holds the pattern's letters (hits starting in a header are kept with
    PM_KEEP_HEADERS and dropped by the report, as process_output does)."""
    rng = random.Random(12)
    recs = []
    for r in range(80):
        hdr = ">%s CKLC%d %s" % ("".join(rng.choice("CKLGST") for _ in range(5)), r, "LCK" * rng.randint(0, 3))
        seq = "".join(rng.choice("CKLGSTAW") for _ in range(rng.randint(1, 40)))
        w = rng.choice([3, 5, 7, 60])
        recs.append(hdr + "\n" + "\n".join(seq[i:i + w] for i in range(0, len(seq), w)) + "\n")
    text = "".join(recs).encode()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        assert db.residue_codes()[0] > 0
        progs = [compile_pattern(convert("-p", p)) for p in ("CXXC", "KXL", "CX", "XKXXL", "LXC", "GXXXXXXS")]
        progs = [p for p in progs if p.kind == "simple"]
        assert len(progs) >= 5
        res, _ = engine.scan(db, progs, k=0, types="s")
        for prog, r in zip(progs, res):
            assert _pairs(r) == oracle_mod.scan_reported(text, prog, 0, "s", skip_headers=True), prog.source
        base = _lib.PM_REPORT_ALL | _lib.PM_KEEP_HEADERS
        planes = _launch(engine, db, progs, 0, base)
        assert planes == _launch(engine, db, progs, 0, base | _lib.PM_SCAN_BYTES)
        assert sum(len(x) for x in planes) > 200
    finally:
        db.close()


@pytest.mark.parametrize("text", [
    b"",
    b">only a header\n",
    b">h1\n>h2\nC\n",
    b">a\nC\nC\nW\nCC\n>b desc\nCCWCC",          # no final newline
    b"CWC\nCCC\n",                                # no header at all
    b">x\n" + b"C" * 100 + b"\n",
])
def test_edge_files(engine, oracle_mod, text):
    """Empty and header-only files, one-residue lines, a missing final
    newline, headerless text, a run longer than any window."""
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        progs = [compile_pattern(convert("-p", p)) for p in ("C", "CC", "CXC", "WC", "CCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCCC")]
        for k in (0, 1, 2):
            res, _ = engine.scan(db, progs, k=k, types="s")
            for prog, r in zip(progs, res):
                assert _pairs(r) == oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True), (prog.source, k, text)
    finally:
        db.close()


def test_many_patterns_one_batch(engine, oracle_mod):
    """A batch of 24 patterns (the byte path takes them in one scan)."""
    rng = random.Random(44)
    text = proteome(rng, n_records=25)
    pats = ["".join(rng.choice(AA + "X") for _ in range(rng.randint(2, 9))) for _ in range(24)]
    progs = [compile_pattern(convert("-p", p)) for p in pats]
    progs = [p for p in progs if p.kind == "simple"]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        for k in (0, 2):
            res, _ = engine.scan(db, progs, k=k, types="s")
            for prog, r in zip(progs, res):
                assert _pairs(r) == oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True), (prog.source, k)
    finally:
        db.close()


NFA_PATTERNS = ["C-x(2,4)-C-x(3)-[LIVMFYWC]", "CX{1,3}CK", "C(AG){1,3}L", "KX{2,}C", "N-{P}-[ST]-{P}",
                "[RK](2)-x-[ST]", "C-x(10,60)-C", "GXGXXG", "<M-x(0,5)-K", "KDEL>"]


@pytest.mark.parametrize("k,types", [(0, ""), (1, "ids"), (2, "s"), (1, "d")])
def test_automaton_start_pass_on_the_planes(engine, oracle_mod, k, types):
    """The automaton kernels' start pass (k_nfa_rev; k_nfa_carry for
    unbounded patterns) reads the residue planes of a peptide file (round 6):
    every candidate (PM_REPORT_ALL, headers kept) equals the byte copy's
    (PM_SCAN_BYTES), and the reported matches equal the oracle's, for ranges,
    group repeats, an unbounded range, a 62-position range (two state words)
    and anchors."""
    rng = random.Random(90 + k)
    text = proteome(rng, n_records=50)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
    try:
        assert db.residue_codes()[0] > 0
        total = 0
        for p in NFA_PATTERNS:
            prog = compile_pattern(convert("-p", p))
            if prog.linear and k == 0:
                continue   # the fixed-length kernels (tested above)
            base = _lib.PM_REPORT_ALL | _lib.PM_KEEP_HEADERS
            try:
                planes = engine.scan_nfa(db, prog, k, types=types or "s", flags=base)
                direct = engine.scan_nfa(db, prog, k, types=types or "s", flags=base | _lib.PM_SCAN_BYTES)
            except _lib.UnsupportedOnGPU:
                continue
            got = list(zip(planes.beg.tolist(), planes.end.tolist()))
            assert got == list(zip(direct.beg.tolist(), direct.end.tolist())), (p, k, types)
            total += len(got)
            res, _ = engine.scan(db, [prog], k=k, types=types)
            assert _pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, types, skip_headers=True), (p, k, types)
        assert total > 100
    finally:
        db.close()
