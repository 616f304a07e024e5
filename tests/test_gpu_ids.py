"""The bit-sliced start pass for class sequences with insertions /
deletions (pm_ids.hip, PM_IDS_JIT=1 forces it on small databases): the
candidates and the reported matches equal the oracle's (pmo_scan2) on
multi-tile databases with N runs, IUPAC letters, lower case, wrapped lines
and motif-laden headers."""
import os
import sys

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.fastagen import dna_fasta

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_report import repeat_fasta  # noqa: E402

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


TEXTS = {
    "dna": lambda: dna_fasta(81, n_records=4, min_len=60000, max_len=140000),
    "repeats": lambda: repeat_fasta(82, n_records=3, min_len=50000, max_len=90000),
    "wrapped": lambda: dna_fasta(83, n_records=3, min_len=20000, max_len=50000, width=60),
}


@pytest.mark.parametrize("name", sorted(TEXTS))
def test_ids_pass_equals_oracle(engine, oracle_mod, monkeypatch, name):
    monkeypatch.setenv("PM_IDS_JIT", "1")
    text = TEXTS[name]()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat, k, types in [("TGCTGASTCAGCANW", 2, "ids"), ("TATAWAWR", 1, "ids"), ("GAATTC", 1, "id"),
                              ("GAATTC", 2, "i"), ("TGCTGASTCAGCANW", 3, "ds"), ("AWA", 1, "is"),
                              ("CAACAACAA", 2, "ids"), ("TANNA", 1, "ids")]:
            fwd = convert("-n", pat)
            progs = [compile_pattern(fwd, ignore_case=True), compile_pattern(convert("-c", fwd), ignore_case=True)]
            for prog in progs:
                for report in ("nrgrep", "all"):
                    r = engine.scan_nfa(db, prog, k, 0, types, engine.report_flags(prog, report))
                    want = oracle_mod.scan_reported(text, prog, k, types, skip_headers=True, report=report)
                    assert list(zip(r.beg.tolist(), r.end.tolist())) == want, (name, prog.source, k, types, report)
    finally:
        db.close()


def test_ids_pass_substitutions_only(engine, oracle_mod, monkeypatch):
    """errs = s through the automaton path (the linear kernel's job normally)."""
    monkeypatch.setenv("PM_IDS_JIT", "1")
    text = dna_fasta(84, n_records=3, min_len=40000, max_len=90000)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat, k in [("TGCTGASTCAGCANW", 2), ("TATAWAWR", 1), ("GAATTC", 3)]:
            prog = compile_pattern(convert("-n", pat), ignore_case=True)
            r = engine.scan_nfa(db, prog, k, 0, "s")
            want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)
            assert _pairs((r.beg, r.end)) == want, (pat, k)
    finally:
        db.close()


def test_ids_pass_through_engine_scan(engine, oracle_mod, monkeypatch):
    """engine.scan routes '-k 2ids' to the automaton kernels, which take the
    bit-sliced start pass: both strands, reported."""
    monkeypatch.setenv("PM_IDS_JIT", "1")
    text = dna_fasta(85, n_records=3, min_len=30000, max_len=70000)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        fwd = convert("-n", "TGCTGASTCAGCANW")
        progs = [compile_pattern(fwd, ignore_case=True), compile_pattern(convert("-c", fwd), ignore_case=True)]
        res, _ = engine.scan(db, progs, k=2, types="ids")
        for prog, r in zip(progs, res):
            assert _pairs(r) == oracle_mod.scan_reported(text, prog, 2, "ids", skip_headers=True)
    finally:
        db.close()


def test_ids_pass_classes_that_take_n(engine, oracle_mod, monkeypatch):
    """Two classes with the same A/C/G/T subset, one taking N and one not
    ([ACGN] / [ACG]): they need their own match registers (an N takes its
    membership from the plane mark), and kernels for the two cache apart."""
    monkeypatch.setenv("PM_IDS_JIT", "1")
    text = TEXTS["dna"]()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for src, k in [("A[ACGN]GT[ACG]TTAC", 1), ("A[ACG]GT[ACG]TTAC", 1), ("A[ACGN]GT[ACGN]TTAC", 1),
                       ("[ACGN][ACGN]A[ACG]", 1)]:
            prog = compile_pattern(src, ignore_case=True)
            r = engine.scan_nfa(db, prog, k, 0, "ids", engine.report_flags(prog, "all"))
            want = oracle_mod.scan_reported(text, prog, k, "ids", skip_headers=True, report="all")
            assert list(zip(r.beg.tolist(), r.end.tolist())) == want, src
    finally:
        db.close()


def test_pipelined_scans_equal_synchronous(engine, monkeypatch):
    """PM_PIPELINED (engine.scan's automaton scans, bench --types ids): the
    report pass is queued and the count resolves on first use.  Several
    scans of every report kind are launched before any is collected, some
    are destroyed uncollected, and each collected list equals the same
    query run synchronously."""
    from patmatchdocker_amd import _lib
    monkeypatch.setenv("PM_IDS_JIT", "1")
    text = TEXTS["dna"]()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        cases = []
        for src, k, types in [(convert("-n", "TGCTGASTCAGCANW"), 2, "ids"),
                              (convert("-c", convert("-n", "TGCTGASTCAGCANW")), 2, "ids"),
                              ("GA*TTC+A", 1, "ids"), ("(GATC){2,3}A", 0, ""), ("(CA|GT)TTG", 1, "s"),
                              ("TATA[AT]A", 1, "ids")]:
            prog = compile_pattern(src, ignore_case=True)
            for report in ("nrgrep", "all"):
                cases.append((prog, k, types, engine.report_flags(prog, report)))
        want = []
        for prog, k, types, flags in cases:
            r = engine.scan_nfa(db, prog, k, 0, types or "s", flags)
            want.append(_pairs((r.beg, r.end)))
        handles = [engine.nfa_launch(db, prog, k, 0, types or "s", flags, pipelined=True)
                   for prog, k, types, flags in cases]
        for i, h in enumerate(handles):
            if i % 3 == 1:
                engine.destroy_hits(h)   # never collected
                continue
            r = engine._collect(h)
            assert _pairs((r.beg, r.end)) == want[i], (cases[i][0].source, cases[i][1], cases[i][3])
        assert _lib.PM_PIPELINED == 1024
    finally:
        db.close()
