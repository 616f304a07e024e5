"""nrgrep's esimple engine (a class sequence at k > 0), CPU side.

The behaviour was read from the disassembly of www/bin/nrgrep_coords (never
executed).  Three statements of it are checked against each
other here:

* oracle/pm_nrgrep.c -- the binary's own loops replayed (BNDM / ABNDM /
  shift-or scanners, bit-parallel verify rows), the parity oracle;
* tests/esimple_model.py -- the candidate/verify rules as the GPU walk
  (pm_esimple.hip) uses them, every phase computed by an edit-distance
  table;
* the library's host plan (pm_esimple_plan, C++) against the oracle's
  (pmn_plan, C): two transcriptions of esimplePreproc's cost model.
"""
import random

import numpy as np
import pytest

from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern, fold_byte
from tests import esimple_model

IUPAC = {"R": "[AG]", "Y": "[CT]", "S": "[GC]", "W": "[AT]", "K": "[GT]", "M": "[AC]", "B": "[CGT]",
         "D": "[AGT]", "H": "[ACT]", "V": "[ACG]", "N": "."}
AMINO = "ACDEFGHIKLMNPQRSTVWY"


def _dna_pattern(rng, m):
    s = "".join(rng.choice("ACGT") if rng.random() < 0.8 else rng.choice("RYSWKMBDHVN") for _ in range(m))
    return "".join(IUPAC.get(c, c) for c in s)


def _mutate(rng, s, edits, alpha):
    s = list(s)
    for _ in range(edits):
        j = rng.randrange(len(s))
        r = rng.random()
        if r < 0.4:
            s[j] = rng.choice(alpha)
        elif r < 0.7:
            s.insert(j, rng.choice(alpha))
        elif len(s) > 1:
            del s[j]
    return "".join(s)


def _text(rng, alpha, n, plant=None, copies=0, edits=2, width=60):
    t = [rng.choice(alpha) for _ in range(n)]
    for _ in range(copies):
        cp = _mutate(rng, plant, rng.randint(0, edits), alpha)
        at = rng.randrange(max(1, n - len(cp)))
        t[at:at + len(cp)] = cp
    t = "".join(t)
    return (">s1 test\n" + "\n".join(t[i:i + width] for i in range(0, n, width)) + "\n").encode()


def _plain(pat_classes_str):
    """A plain string whose bytes fall in each class (for planting)."""
    out, i = [], 0
    s = pat_classes_str
    while i < len(s):
        if s[i] == "[":
            j = s.index("]", i)
            out.append(s[i + 1])
            i = j + 1
        elif s[i] == ".":
            out.append("A")
            i += 1
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def test_plan_library_equals_oracle(oracle_mod):
    rng = random.Random(11)
    n = 0
    for _ in range(600):
        if rng.random() < 0.6:
            prog = compile_pattern(_dna_pattern(rng, rng.randint(2, 200)))
        else:
            prog = compile_pattern("".join(rng.choice(AMINO) for _ in range(rng.randint(2, 120))))
        for k in (1, 2, 3, 5, 9, 15):
            if k >= prog.m or (prog.m > 128 and k > 7):
                continue
            a, b = oracle_mod.nrgrep_plan(prog, k), engine.esimple_plan(prog, k)
            assert a["type"] == b["type"] and a["L"] == b["L"], (prog.source, k, a, b)
            if a["type"] == 1:
                assert a["piece_len"] == b["piece_len"]
            else:
                assert a["window"] == b["window"]
            n += 1
    assert n > 1500


def test_plan_of_the_bench_motif(oracle_mod):
    """configs[2]'s motif at -k 2: three pieces of 4 at positions 1, 5, 9
    (the cost model over letterProb picks them, not an even split)."""
    for strand in ("-n", "-c"):
        fwd = convert("-n", "TGCTGASTCAGCANW")
        prog = compile_pattern(fwd if strand == "-n" else convert("-c", fwd))
        plan = oracle_mod.nrgrep_plan(prog, 2)
        assert plan["type"] == 1 and plan["piece_len"] == 4
        assert engine.esimple_plan(prog, 2) == plan
    assert oracle_mod.nrgrep_plan(compile_pattern(convert("-n", "TGCTGASTCAGCANW")), 2)["L"] == [1, 5, 9]


def test_every_scanner_type_occurs(oracle_mod):
    seen = set()
    rng = random.Random(3)
    for _ in range(400):
        prog = compile_pattern(_dna_pattern(rng, rng.randint(4, 40)) if rng.random() < 0.5
                               else "".join(rng.choice("WYCHMFQK") for _ in range(rng.randint(8, 40))))
        seen.add(oracle_mod.nrgrep_plan(prog, rng.randint(1, 3))["type"])
    assert seen == {1, 2, 3}


def _cases(seed, n_cases):
    rng = random.Random(seed)
    for _ in range(n_cases):
        r = rng.random()
        if r < 0.45:
            pat = _dna_pattern(rng, rng.randint(4, 22))
            alpha = rng.choice(["ACGT", "AT", "ACGTN", "AAAT", "A", "CA"])
        elif r < 0.75:
            pat = "".join(rng.choice("WYCHMFQK" if rng.random() < 0.5 else AMINO) for _ in range(rng.randint(8, 40)))
            alpha = AMINO
        else:
            pat = "".join(rng.choice("ACGT") for _ in range(rng.randint(30, 70)))
            alpha = "ACGT"
        a = rng.random()
        if a < 0.08:
            pat = "^" + pat
        elif a < 0.16:
            pat = pat + "$"
        prog = compile_pattern(pat)
        k = rng.randint(1, max(1, min(4, prog.m // 3)))
        types = rng.choice(["s", "ids", "ids", "i", "d", "is", "ds", "id"])
        if "d" in types and k >= prog.m:
            types = "s"
        text = _text(rng, alpha, rng.randint(100, 1200), _plain(pat.strip("^$")), rng.randint(0, 8), k + 1,
                     width=rng.choice([7, 60, 5000]))
        yield prog, k, types, text


@pytest.mark.parametrize("seed", range(6))
def test_literal_replay_equals_event_model(oracle_mod, seed):
    """pm_nrgrep.c's replay of the binary's scanners and bit-parallel
    verify == the candidate/verify rules with edit-distance phases."""
    for prog, k, types, text in _cases(seed, 60):
        plan = oracle_mod.nrgrep_plan(prog, k)
        got = oracle_mod.scan_esimple(text, prog, k, types)
        assert got == esimple_model.report(text, prog, k, types, plan), (prog.source, k, types, plan)


def _dist(prog, s, types):
    INF = 1 << 30
    m, n = prog.m, len(s)
    D = [[INF] * (n + 1) for _ in range(m + 1)]
    D[0][0] = 0
    for i in range(m + 1):
        for j in range(n + 1):
            if i == 0 and j == 0:
                continue
            v = INF
            if i and j:
                v = D[i - 1][j - 1] + (0 if fold_byte(s[j - 1]) in prog.classes[i - 1] else (1 if "s" in types else INF))
            if j and "i" in types:
                v = min(v, D[i][j - 1] + 1)
            if i and "d" in types:
                v = min(v, D[i - 1][j] + 1)
            D[i][j] = v
    return D[m][n]


@pytest.mark.parametrize("seed", range(3))
def test_reported_matches_are_valid_and_disjoint(oracle_mod, seed):
    for prog, k, types, text in _cases(seed + 100, 40):
        prev = 0
        for b, e in oracle_mod.scan_esimple(text, prog, k, types):
            assert prev <= b <= e and b"\n" not in text[b:e]
            assert _dist(prog, text[b:e], types) <= k, (prog.source, k, types, b, e)
            prev = e


def test_piece_order_can_beat_the_leftmost_start(oracle_mod):
    """nrgrep finds windows by their first exact piece (type 1): a later
    window whose piece 0 matches is printed before an overlapping earlier
    window whose only exact piece lies further right, which the leftmost-start
    rule would print.  Self-similar texts make such overlaps common."""
    rng = random.Random(5)
    found = 0
    for _ in range(600):
        prog = compile_pattern(_dna_pattern(rng, rng.randint(8, 18)))
        k = rng.randint(1, 2)
        if oracle_mod.nrgrep_plan(prog, k)["type"] != 1:
            continue
        text = _text(rng, rng.choice(["AT", "ACGT", "CA"]), 800)
        a = oracle_mod.scan_esimple(text, prog, k, "s")
        b = oracle_mod.scan_reported(text, prog, k, "s", report="leftmost")
        if a != b:
            found += 1
            assert all(e - s == prog.m and _dist(prog, text[s:e], "s") <= k for s, e in a)
            # every window nrgrep prints is one of the candidate windows
            assert set(a) <= set(oracle_mod.scan(text, prog, k, "s"))
    assert found >= 2


def test_ids_reports_differ_from_shortest_end(oracle_mod):
    """With indels the verify keeps the nearest start/end with the fewest
    errors, not the leftmost start with its shortest end."""
    prog = compile_pattern(convert("-n", "GAATTC"))
    text = b">s\nTTGAATTTCAAAGAATTCGAATC\nGGAAATTCCC\n"
    got = oracle_mod.scan_esimple(text, prog, 1, "ids")
    assert got == esimple_model.report(text, prog, 1, "ids", oracle_mod.nrgrep_plan(prog, 1))
    assert got != oracle_mod.scan_reported(text, prog, 1, "ids", report="leftmost")


@pytest.mark.parametrize("case", [("ACG", 3, "ids"), ("ACG", 4, "d"), ("AT", 2, "id"), ("GAT", 3, "ds"),
                                  ("[AC]GT", 3, "ids")])
def test_deletions_reaching_the_pattern_length(oracle_mod, case):
    """k >= m with deletions (the whole pattern may be deleted; the web form
    lets a 3-residue pattern run at -k 3ids, patmatch.py:308-314): the plan
    falls back to the forward prefix scanner (simpleFindBest finds no window,
    no pieces fit), every position is a candidate, and empty matches are
    printed -- the replay and the model agree."""
    from tests.fastagen import dna_fasta
    pat, k, types = case
    prog = compile_pattern(pat)
    plan = oracle_mod.nrgrep_plan(prog, k)
    assert plan["type"] == 3
    text = dna_fasta(5, n_records=3, max_len=200, width=30)
    got = oracle_mod.scan_esimple(text, prog, k, types)
    assert got == esimple_model.report(text, prog, k, types, plan)
    assert any(b == e for b, e in got) and any(e > b for b, e in got)
