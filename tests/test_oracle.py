"""The CPU oracle (oracle/pm_oracle.c) cross-checked against two independent
restatements: the pure-Python state-set simulation and, for k = 0, Python's
own `re` engine (shortest full match from every start)."""
import random
import re

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.fastagen import dna_fasta, pep_fasta

# no '?', '*', '+' at a pattern edge: nrgrep's simplify (regex.py) drops or
# shortens those, Python's re does not
PATTERNS = ["(GAATTC)", "(TATA[AT]A[AT][AG])", "(C..?.?C...[LIVMFYWC])", "(A(CG)*T)", "(AC|GT.)", "(A[^C]G)",
            "(C(GA)?TTC)", "(GC?.?.TG)", "(GA+C)", "(#A)"]


def _to_python_re(source):
    # nrgrep syntax used by these patterns is a subset of Python's
    return source.replace("#", r"[^0-9A-Za-z\n]")


@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_python_state_sets(oracle_mod, seed):
    rng = random.Random(seed)
    text = dna_fasta(seed, n_records=3, max_len=50) if seed % 2 else pep_fasta(seed, 3, 40)
    for p in PATTERNS:
        prog = compile_pattern(p)
        for k, t in [(0, "ids"), (1, "s"), (1, "ids"), (2, "i"), (2, "d"), (1, "id"), (rng.randint(0, 3), "s")]:
            assert oracle_mod.scan(text, prog, k, t) == oracle_mod.scan_py(text, prog, k, t), (p, k, t)


@pytest.mark.parametrize("seed", range(4))
def test_oracle_vs_python_re_exact(oracle_mod, seed):
    text = dna_fasta(seed + 10, n_records=3, max_len=120)
    folded = text.upper()
    for p in PATTERNS:
        prog = compile_pattern(p)
        rx = re.compile(_to_python_re(p).encode())
        want = []
        pos = 0
        for line in folded.split(b"\n"):
            for s in range(len(line)):
                for e in range(s + 1, len(line) + 1):
                    if rx.fullmatch(line, s, e):
                        want.append((pos + s, pos + e))
                        break
            pos += len(line) + 1
        assert oracle_mod.scan(text, prog, 0) == want, p


def test_header_filter(oracle_mod):
    t = b">a GAATTC\nGAATTC\n> b GAATTC\n"
    p = compile_pattern("(GAATTC)")
    assert oracle_mod.scan(t, p) == [(3, 9), (10, 16), (21, 27)]
    assert oracle_mod.scan(t, p, skip_headers=True) == [(10, 16), (21, 27)]


def test_record_index_restatement(oracle_mod):
    assert oracle_mod.record_index(b">chrI a\nACGT\n>chrII\nAC\n>\n> x\nGG") == \
        [(0, ">chrI"), (8, "chrI"), (13, ">chrII"), (20, "chrII")]


def test_reverse_complement_strand(oracle_mod):
    text = b">s\nAAGAATTCAA\nCTTTTATAGG\n"
    fwd = compile_pattern(convert("-n", "TATAWAWR"))
    rev = compile_pattern(convert("-c", convert("-n", "TATAWAWR")))
    assert oracle_mod.scan(text, fwd) == []
    assert oracle_mod.scan(text, rev) == [(14, 22)]     # CTTTTATA = revcomp of TATAAAAG


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_oracle_threaded_scan_matches_serial(oracle_mod, threads):
    """The bench's multi-threaded CPU baseline (records split across host
    threads) returns exactly the serial scan's hits, header filter included."""
    text = dna_fasta(77, n_records=400, min_len=2000, max_len=6000)
    assert len(text) >= (1 << 20)
    for p, k in [("(GAATTC)", 0), ("(TATA[AT]A[AT][AG])", 1), ("(AC|GT.)", 0)]:
        prog = compile_pattern(p)
        want = oracle_mod.scan(text, prog, k, "s", skip_headers=True)
        got = oracle_mod.scan_threads(text, prog, k, "s", skip_headers=True, threads=threads)
        assert got == want, (p, k, threads)


def test_oracle_threaded_scan_on_decoded_layout(oracle_mod):
    """Cuts at line breaks also split a text without '>' (a database decoded
    from HBM renders header bytes as '\\n'), and hits stay identical."""
    text = dna_fasta(78, n_records=300, min_len=3000, max_len=8000).replace(b">", b"\n")
    prog = compile_pattern("(TATA[AT]A[AT][AG])")
    want = oracle_mod.scan(text, prog, 1, "s")
    assert oracle_mod.scan_threads(text, prog, 1, "s", threads=8) == want


@pytest.mark.parametrize("seed", range(3))
def test_shiftadd_cpu_scan_equals_reported_oracle(oracle_mod, seed):
    """The bit-parallel Shift-Add CPU scan (pm_cpuscan.c) reports exactly what
    pmo_scan2's leftmost-start rule reports for class sequences with
    substitutions (nrgrep's own order: test_nrgrep_esimple.py)."""
    text = dna_fasta(seed + 60, n_records=5, max_len=4000, width=(70 if seed == 1 else None))
    for pat in ["TGCTGASTCAGCANW", "TATAWAWR", "GAATTC", "NNGCNN", "AAAA", "TANNNNTA"]:
        for strand in ("-n", "-c"):
            fwd = convert("-n", pat)
            prog = compile_pattern(fwd if strand == "-n" else convert("-c", fwd))
            for k in (0, 1, 2, 3):
                if k >= prog.m:
                    continue
                want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True,
                                                report="leftmost" if k else "nrgrep")
                assert oracle_mod.shiftadd_scan(text, prog, k, skip_headers=True) == want, (pat, k)
                assert oracle_mod.shiftadd_threads(text, prog, k, skip_headers=True, threads=3) == want, (pat, k)


@pytest.mark.parametrize("seed", range(4))
def test_python_reported_oracle_equals_c_oracle(oracle_mod, seed):
    """scan_py_reported (any number of positions; checks the >64-position
    GPU scans) against pmo_scan2 on automata it holds, line-bounded engines."""
    text = dna_fasta(seed + 30, n_records=3, max_len=150, width=40) if seed % 2 else pep_fasta(seed, 4, 60)
    for p in PATTERNS + ["^(A.C)", "(G.T)$", "^(AC|GT.)$"]:
        prog = compile_pattern(p)
        for k, t in [(0, "s"), (1, "s"), (1, "ids"), (2, "id"), (2, "s")]:
            want = oracle_mod.scan_reported(text, prog, k, t, skip_headers=True, simple=False)
            if k and oracle_mod.is_esimple(prog):
                want = oracle_mod.scan_esimple(text, prog, k, t, skip_headers=True)
            assert oracle_mod.scan_py_reported(text, prog, k, t, skip_headers=True) == want, (p, k, t)


@pytest.mark.parametrize("seed", range(4))
def test_ids_cpu_scan_equals_reported_oracle(oracle_mod, seed):
    """The bit-parallel `-k <k>ids` CPU scan (pmc_ids_scan) reports exactly
    what the oracle's leftmost-start rule does."""
    from tests.test_gpu_report import repeat_fasta
    text = dna_fasta(seed + 40, n_records=4, max_len=4000) if seed % 2 else repeat_fasta(seed + 40, 3, 1000, 4000)
    for pat in ["TGCTGASTCAGCANW", "TATAWAWR", "GAATTC", "AWA", "CAACAACAA", "TANNA"]:
        prog = compile_pattern(convert("-n", pat), ignore_case=True)
        for k, t in [(1, "ids"), (2, "ids"), (2, "i"), (1, "d"), (3, "ds"), (2, "is"), (1, "s")]:
            if "d" in t and k >= prog.m:
                continue
            want = oracle_mod.scan_reported(text, prog, k, t, skip_headers=True, report="leftmost")
            assert oracle_mod.ids_scan(text, prog, k, t, skip_headers=True) == want, (pat, k, t)
            assert oracle_mod.ids_threads(text, prog, k, t, skip_headers=True, threads=3) == want, (pat, k, t)
