"""nrgrep_coords report semantics, CPU side.

The rules were read from the disassembly of the reference binary
(www/bin/nrgrep_coords, never executed).  Checked here:

* the C restatement (oracle/pm_oracle.c pmo_scan2, fed by regex.py's
  compiled program) against the independent string-level restatement of the
  simple engine (oracle/nrgrep_simple.py, its own parser) on every
  converter-golden pattern that is a plain class sequence, over texts with
  headers, line breaks, N runs, lower case and IUPAC letters;
* the report rule (first found wins, resume at the match end) against a
  direct Python restatement over the candidate list, for line-bounded
  patterns and k > 0 (the leftmost-start rule; a class sequence at k > 0
  runs nrgrep's esimple engine instead, tests/test_nrgrep_esimple.py);
* anchors, '.' accepting the delimiter, reversed ranges.
"""
import json
import os
import random

import pytest

from oracle import nrgrep_simple
from patmatchdocker_amd.regex import RegexSyntaxError, compile_pattern
from tests.fastagen import dna_fasta, pep_fasta

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "converter.json")


def _simple_golden_patterns():
    out = []
    for e in json.load(open(GOLDEN)):
        o = e.get("output")
        if not o:
            continue
        try:
            nrgrep_simple.parse(o)
            prog = compile_pattern(o)
        except (nrgrep_simple.NotSimple, RegexSyntaxError):
            continue
        if prog.linear and prog.m <= 64:
            out.append(o)
    return sorted(set(out))


SIMPLE = _simple_golden_patterns()


def _texts():
    yield dna_fasta(3, n_records=4, max_len=700)
    yield dna_fasta(4, n_records=3, max_len=500, width=50)
    yield pep_fasta(5, n_records=6, max_len=200)
    rng = random.Random(9)
    yield bytes(rng.choice(b"ACGTNacgt\n>RY .,-#^$") for _ in range(3000))


def test_golden_has_many_simple_patterns():
    assert len(SIMPLE) > 300


@pytest.mark.parametrize("ti", range(4))
def test_c_restatement_matches_string_level_simple_engine(oracle_mod, ti):
    text = list(_texts())[ti]
    for pat in SIMPLE:
        prog = compile_pattern(pat)
        want = nrgrep_simple.scan(text, pat)
        got = oracle_mod.scan_reported(text, prog, 0, "")
        assert got == want, pat


def _greedy(cands, text, a_start=False, a_end=False):
    out, R, cur = [], 0, None
    for s, e in cands:
        if a_end and not (e == len(text) or text[e] == 10):
            continue
        if s < R:
            continue
        if a_start and not (s == R or s == 0 or text[s - 1] == 10):
            continue
        out.append((s, e))
        R = e
    return out


@pytest.mark.parametrize("seed", range(4))
def test_report_rule_on_candidates(oracle_mod, seed):
    text = dna_fasta(seed + 40, n_records=4, max_len=800)
    pats = ["(TATA[AT]A[AT][AG])", "(GA...?TC)", "(A(CG)*T)", "(AA)", "(AC|GT.)", "(TT.?.?.?AA)"]
    for p in pats:
        prog = compile_pattern(p)
        for k, t in [(0, ""), (1, "s"), (1, "ids"), (2, "s")]:
            if k == 0 and prog.linear:
                continue   # the simple engine is not line-bounded (tested above)
            cands = oracle_mod.scan(text, prog, k, t)
            got = oracle_mod.scan_reported(text, prog, k, t, report="leftmost")
            assert got == _greedy(cands, text), (p, k, t)


def test_overlaps_are_not_reported(oracle_mod):
    text = b">s\nTATATATATA\nAAAAAA\n"
    assert oracle_mod.scan_reported(text, compile_pattern("(TATA)"), 0, "") == [(3, 7), (7, 11)]
    assert oracle_mod.scan_reported(text, compile_pattern("(AAA)"), 0, "") == [(14, 17), (17, 20)]
    # the raw candidate list keeps every start
    assert oracle_mod.scan(text, compile_pattern("(TATA)"), 0, "") == [(3, 7), (5, 9), (7, 11), (9, 13)]


def test_dot_spans_a_line_break_in_the_simple_engine(oracle_mod):
    text = b">a\nGAATTCA\n>b\nCCC\n"
    prog = compile_pattern("(TCA.)")
    # k = 0: the window may take the '\n' (process_output keeps it: its start
    # is in the sequence line)
    assert oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True) == [(7, 11)]
    assert nrgrep_simple.scan(text, "(TCA.)") == [(7, 11)]
    # k = 1 (esimple verifies inside the line): no window crosses it
    assert (7, 11) not in oracle_mod.scan_reported(text, prog, 1, "s")


def test_cross_line_match_from_a_header_suppresses_an_overlap(oracle_mod):
    # ">hX\nXAXA\n": the window [2, 5) = "X\nX" starts on the header line
    # (process_output drops it) and hides the overlapping sequence match
    # [4, 7); the scan resumes at 5 and reports [5, 8)
    text = b">hX\nXAXA\n"
    pat = "([AX].[AX])"
    assert nrgrep_simple.scan(text, pat) == [(2, 5), (5, 8)]
    prog = compile_pattern(pat)
    assert oracle_mod.scan_reported(text, prog, 0, "") == [(2, 5), (5, 8)]
    assert oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True) == [(5, 8)]
    assert (4, 7) in oracle_mod.scan_reported(text, prog, 0, "", report="all")


def test_anchors(oracle_mod):
    text = b">s\nACAC\nCACA\n"
    p = compile_pattern("^(AC)")
    assert p.anchor_start and not p.anchor_end and p.m == 2
    # line start, then the scan resumes at R = 5 where '^' passes again
    assert oracle_mod.scan_reported(text, p, 0, "") == [(3, 5), (5, 7)]
    assert nrgrep_simple.scan(text, "^(AC)") == [(3, 5), (5, 7)]
    q = compile_pattern("(CA)$")
    assert oracle_mod.scan_reported(text, q, 0, "") == [(10, 12)]
    assert nrgrep_simple.scan(text, "(CA)$") == [(10, 12)]
    # '^' / '$' inside the pattern are ordinary characters
    r = compile_pattern("(A^C)")
    assert not r.anchor_start and r.m == 3


def test_reversed_range_is_empty_not_an_error():
    p = compile_pattern("([T-A]C)")
    assert p.classes[0] == frozenset()
    assert nrgrep_simple.parse("([T-A]C)")[0][0] == set()


def test_dot_and_negated_classes_accept_the_delimiter():
    p = compile_pattern("(.[^A]#)")
    assert all(10 in c for c in p.classes)
