"""nrgrep's extended engine at k = 0 (patterns with '?', '*', '+': every
PatMatch range X{m,n}), restated from the binary's disassembly in
oracle/pm_nrgrep_ext.c: its plan against the library's own C++ restatement
(pm_extended_plan), and its report against a second statement of the rule
with explicit position sets (tests/extended_model.py) on texts where
candidates overlap densely.  The GPU is checked against the replay in
tests/test_gpu_extended.py."""
import json
import os
import random

import pytest

from oracle import oracle
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern, RegexSyntaxError
from tests.extended_model import ExtendedModel

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "converter.json")


def _golden_extended():
    out = set()
    for e in json.load(open(GOLDEN)):
        o = e.get("output")
        if not o:
            continue
        try:
            prog = compile_pattern(o)
        except RegexSyntaxError:
            continue
        if prog.kind == "extended":
            out.add(o)
    return sorted(out)


def random_extended(rng, alphabet="dna"):
    syms = (["A", "C", "G", "T", "[AG]", "[CT]", ".", "[^A]", "[AT]", "[GC]"] if alphabet == "dna"
            else ["C", "K", "L", "[LIVM]", ".", "[ST]", "G", "[^P]"])
    while True:
        parts = []
        for _ in range(rng.randint(2, 10)):
            node = rng.choice(syms)
            q = rng.random()
            node += "?" if q < 0.3 else "*" if q < 0.37 else "+" if q < 0.44 else ""
            parts.append(node)
        pat = "(" + "".join(parts) + ")"
        if rng.random() < 0.1:
            pat = "^" + pat
        if rng.random() < 0.1:
            pat += "$"
        try:
            prog = compile_pattern(pat)
        except RegexSyntaxError:
            continue
        if prog.kind == "extended":
            return pat, prog


def dense_text(rng, alphabet, n_lines=12, width=(20, 90)):
    letters = {"dna": ["ACGT", "AT", "AAT", "GC", "ACG"], "pep": ["CKLGST", "CCAK", "LIVMC", "ACDEFGHIKLMNPQRSTVWY"]}
    lines = []
    for r in range(n_lines):
        if rng.random() < 0.2:
            lines.append(">seq%d" % r)
        al = rng.choice(letters[alphabet])
        line = "".join(rng.choice(al) for _ in range(rng.randint(*width)))
        if rng.random() < 0.2:
            line = line.lower()
        lines.append(line)
    return ("\n".join(lines) + "\n").encode()


def test_golden_patterns_include_windows_away_from_the_start():
    pats = _golden_extended()
    assert len(pats) >= 15
    plans = [oracle.extended_plan(compile_pattern(p)) for p in pats]
    assert any(p["L"] > 0 for p in plans) and any(p["type"] == 3 for p in plans) and any(p["L"] == 0 for p in plans)


@pytest.mark.parametrize("seed", range(3))
def test_library_plan_matches_the_replay(seed):
    """pm_extended_plan (C++, the GPU's host side) vs pmx_plan (C, the
    oracle): the cost model decides the window, so the scanner and the
    candidate order."""
    rng = random.Random(700 + seed)
    progs = [compile_pattern(p) for p in _golden_extended()]
    while len(progs) < 600:
        progs.append(random_extended(rng, rng.choice(["dna", "pep"]))[1])
    for prog in progs:
        assert engine.extended_plan(prog) == oracle.extended_plan(prog), prog.source


def test_long_patterns_plan():
    rng = random.Random(11)
    for _ in range(40):
        parts = [rng.choice(["A", "C", "G", "T", ".", "[AG]"]) + ("?" if rng.random() < 0.2 else "")
                 for _ in range(rng.randint(60, 200))]
        try:
            prog = compile_pattern("(" + "".join(parts) + "T)")
        except RegexSyntaxError:
            continue
        if prog.kind == "extended":
            assert engine.extended_plan(prog) == oracle.extended_plan(prog)


@pytest.mark.parametrize("seed", range(6))
def test_replay_matches_the_set_model(seed):
    rng = random.Random(900 + seed)
    checked = 0
    while checked < 40:
        alpha = rng.choice(["dna", "pep"])
        pat, prog = random_extended(rng, alpha)
        plan = oracle.extended_plan(prog)
        if not ExtendedModel.covers(prog, plan):
            continue
        text = dense_text(rng, alpha)
        want = ExtendedModel(prog, plan).report(text)
        got = oracle.scan_extended(text, prog, bufsize=0)
        assert got == want, (pat, plan, text[:200])
        checked += 1


def test_golden_patterns_replay_vs_model():
    rng = random.Random(5)
    for pat in _golden_extended():
        prog = compile_pattern(pat)
        plan = oracle.extended_plan(prog)
        if not ExtendedModel.covers(prog, plan):
            continue
        for alpha in ("dna", "pep"):
            text = dense_text(rng, alpha, n_lines=8)
            assert oracle.scan_extended(text, prog, bufsize=0) == ExtendedModel(prog, plan).report(text), pat


def test_nearest_start_from_a_window_past_the_start():
    """AN{0,3}GAATTC: the window is GAATTC, the left part A.?.?.? is read
    back from it and the nearest start wins -- except that the two optional
    positions next to the window cannot both be skipped before a character
    is read (the initial state is not closed)."""
    prog = compile_pattern(convert("-n", "AN{0,3}GAATTC"))
    plan = oracle.extended_plan(prog)
    assert plan["type"] == 2 and plan["L"] == 4
    # starts at 0, 1, 2 all match; leftmost would print [0, 9)
    assert oracle.scan_extended(b"AAAGAATTC\n", prog) == [(1, 9)]
    assert oracle.scan_extended(b"xAGAATTC\n", prog) == []            # A right before G: needs three skips
    assert oracle.scan_extended(b"xAxGAATTC\n", prog) == [(1, 9)]


def test_every_printed_match_is_a_match():
    rng = random.Random(42)
    for _ in range(60):
        alpha = rng.choice(["dna", "pep"])
        pat, prog = random_extended(rng, alpha)
        text = dense_text(rng, alpha)
        got = oracle.scan_extended(text, prog, bufsize=0)
        cands = dict(oracle.scan_candidates(text, prog, 0, "", bufsize=0))   # '^' left to the report
        prev = 0
        for b, e in got:
            assert b >= prev and e > b
            assert b in cands, (pat, b)
            prev = e
