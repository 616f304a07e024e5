"""The automaton kernels beyond one state word and three errors
(pm_scan_nfa_wide): long oligos, unrolled N{m,n} ranges, unbounded repeats
over two state words, k = 4..15, and the simple engine's cross-line windows
for a long k = 0 class sequence -- each against an oracle restatement
(pure-Python state sets for > 64 positions, pm_oracle.c otherwise,
nrgrep_simple.py for the simple engine)."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.fastagen import dna_fasta, pep_fasta

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine as eng
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def _pairs(r):
    return list(zip(r[0].tolist(), r[1].tolist()))


def _mutate(s, n, seed):
    rng = random.Random(seed)
    s = bytearray(s)
    for _ in range(n):
        i = rng.randrange(len(s))
        s[i] = rng.choice(b"ACGT".replace(bytes([s[i]]), b""))
    return bytes(s)


@pytest.fixture(scope="module")
def dna():
    return dna_fasta(71, n_records=4, min_len=2000, max_len=4500)


@pytest.fixture(scope="module")
def dna_db(engine, dna):
    db = engine.SequenceDatabase.from_bytes(dna, alphabet=engine.NUC)
    yield db
    db.close()


def _oligo(text, length, seed):
    rng = random.Random(seed)
    lines = [ln for ln in text.split(b"\n") if ln and not ln.startswith(b">") and len(ln) > length + 10]
    ln = rng.choice(lines)
    i = rng.randrange(len(ln) - length)
    return ln[i:i + length].upper()


@pytest.mark.parametrize("length,k,types,mut", [(100, 0, "s", 0), (100, 3, "s", 3), (100, 5, "s", 4),
                                               (130, 4, "ids", 3), (200, 7, "s", 6), (80, 2, "ids", 2)])
def test_long_oligo(engine, oracle_mod, dna, dna_db, length, k, types, mut):
    oligo = _mutate(_oligo(dna, length, length + k), mut, k)
    prog = compile_pattern(convert("-n", oligo.decode()), ignore_case=True)
    assert prog.m == length
    assert engine.route(prog, engine.NUC, k, types) == "nfa"
    (got,), _ = engine.scan(dna_db, [prog], k=k, types=types)
    want = oracle_mod.scan_py_reported(dna, prog, k, types, skip_headers=True)
    assert _pairs(got) == want
    assert want   # the oligo is found


@pytest.mark.parametrize("k,types", [(4, "s"), (5, "ids"), (6, "id"), (9, "s"), (15, "s")])
def test_more_than_three_errors(engine, oracle_mod, dna, dna_db, k, types):
    fwd = convert("-n", "TGCTGASTCAGCANW")
    progs = [compile_pattern(fwd, ignore_case=True), compile_pattern(convert("-c", fwd), ignore_case=True)]
    res, _ = engine.scan(dna_db, progs, k=k, types=types)
    for prog, r in zip(progs, res):
        assert _pairs(r) == oracle_mod.scan_reported(dna, prog, k, types, skip_headers=True), (k, types)


@pytest.mark.parametrize("pattern,k,types", [("GATAN{10,100}TTAT", 0, "s"), ("GATAN{40,70}TTAT", 1, "ids"),
                                             ("CCN{60,90}GG", 0, "s")])
def test_unrolled_ranges(engine, oracle_mod, dna, dna_db, pattern, k, types):
    prog = compile_pattern(convert("-n", pattern), ignore_case=True)
    assert prog.m > 64 and not prog.linear
    (got,), _ = engine.scan(dna_db, [prog], k=k, types=types)
    # an extended pattern: nrgrep's extended / eextended engine (256 positions)
    want = oracle_mod.scan_reported(dna, prog, k, types, skip_headers=True)
    assert _pairs(got) == want
    assert want


def test_unbounded_repeat_over_two_words(engine, oracle_mod, dna, dna_db):
    # 66 positions then '.*': the carry relaxation with 2-word states
    oligo = _oligo(dna, 64, 3)
    prog = compile_pattern("(" + oligo.decode() + "A.*C)", ignore_case=True)
    assert prog.m > 64 and prog.max_len is None
    (got,), _ = engine.scan(dna_db, [prog], k=1, types="s")
    assert prog.kind == "extended"   # nrgrep's eextended engine
    assert _pairs(got) == oracle_mod.scan_reported(dna, prog, 1, "s", skip_headers=True)


def test_long_simple_pattern_spans_line_breaks(engine):
    """k = 0 class sequence with '.' (nrgrep's simple engine): windows run
    over '\\n' (and header lines) -- the cross-line automaton scan."""
    from oracle import nrgrep_simple
    text = dna_fasta(72, n_records=5, min_len=400, max_len=1500, width=60)
    i = text.index(b"\n", 500) - 40
    piece = text[i:i + 90].decode().replace("\n", ".")
    pat = piece[:30] + "." + piece[31:]
    prog = compile_pattern(pat, ignore_case=True)
    assert prog.m == 90 and prog.linear
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        (got,), _ = engine.scan(db, [prog], k=0)
    finally:
        db.close()
    want = nrgrep_simple.scan(text, pat)
    assert _pairs(got) == want
    assert (i, i + 90) in want


def test_long_peptide_pattern(engine, oracle_mod):
    text = pep_fasta(73, n_records=30, max_len=900)
    rng = random.Random(5)
    recs = [ln for ln in text.split(b"\n") if ln and not ln.startswith(b">") and len(ln) > 120]
    ln = rng.choice(recs)
    sub = ln[10:90].decode()
    pat = sub[:20] + "." + sub[21:50] + "[" + sub[50] + "W]" + sub[51:]
    prog = compile_pattern(pat, ignore_case=True)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        for k, types in [(0, "s"), (3, "s"), (2, "ids"), (8, "s")]:
            (got,), _ = engine.scan(db, [prog], k=k, types=types)
            assert _pairs(got) == oracle_mod.scan_py_reported(text, prog, k, types, skip_headers=True), (k, types)
    finally:
        db.close()
