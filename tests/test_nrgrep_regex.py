"""The scan candidates and the report of non-simple patterns (``? * + |``,
groups: nrgrep's extended and regular engines) at k >= 0, checked against an
independent restatement that parses the nrgrep pattern STRING itself and
matches with a different algorithm (oracle/nrgrep_regex.py: a relation over
the parse tree, no position automaton) -- so a bug in
``patmatchdocker_amd.regex.compile_pattern`` or in ``pm_oracle.c`` cannot hide
behind an oracle that consumes the same compiled program.  The GPU kernels
are checked against ``pm_oracle.c`` (tests/test_gpu_*.py); this closes the
loop for every converter-golden non-simple pattern and for random patterns
with alternation and repetition."""
import json
import os
import random

import pytest

from oracle import nrgrep_regex
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import RegexSyntaxError, compile_pattern
from tests.fastagen import dna_fasta, pep_fasta

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "converter.json")
ERRORS = [(0, ""), (1, "ids"), (1, "s"), (1, "d"), (2, "id"), (2, "ids")]


def _golden_non_simple():
    out = set()
    for e in json.load(open(GOLDEN)):
        o = e.get("output")
        if not o:
            continue
        try:
            prog = compile_pattern(o)
        except RegexSyntaxError:
            continue
        if not prog.linear:
            out.add(o)
    return sorted(out)


NON_SIMPLE = _golden_non_simple()


def _reported(oracle_mod, text, prog, k, types):
    # line-bounded windows (the simple engine's whole-text windows at k = 0
    # only apply to class sequences, tests/test_nrgrep_semantics.py); the
    # leftmost-start report rule (a class sequence at k > 0 runs esimple,
    # tests/test_nrgrep_esimple.py)
    if k == 0:
        return oracle_mod.scan_reported(text, prog, 0, "", simple=False)
    return oracle_mod.scan_reported(text, prog, k, types, report="leftmost")


def test_golden_has_non_simple_patterns():
    assert len(NON_SIMPLE) >= 20
    # every golden '*' comes from a trailing {m,}: simplify drops it (a nullable
    # tail), so the golden set's non-simple patterns are '?' ranges only
    assert any("?" in p for p in NON_SIMPLE)


@pytest.mark.parametrize("ti", range(2))
def test_golden_non_simple_candidates_and_report(oracle_mod, ti):
    text = [dna_fasta(3, n_records=3, max_len=300), pep_fasta(4, n_records=5, max_len=120)][ti]
    for pat in NON_SIMPLE:
        prog = compile_pattern(pat)
        for k, types in ERRORS:
            if k and "d" in types and k >= prog.min_len:
                continue   # refused by the engine (engine.route)
            assert oracle_mod.scan(text, prog, k, types) == nrgrep_regex.candidates(text, pat, k, types), (pat, k, types)
            assert _reported(oracle_mod, text, prog, k, types) == nrgrep_regex.reported(text, pat, k, types), \
                (pat, k, types)


def _random_pattern(rng, depth=0):
    parts = []
    for _ in range(rng.randint(1, 4)):
        r = rng.random()
        if r < 0.15 and depth < 2:
            node = "(" + _random_pattern(rng, depth + 1)
            if rng.random() < 0.4:
                node += "|" + _random_pattern(rng, depth + 1)
            node += ")"
        elif r < 0.3:
            node = rng.choice(["[AG]", "[CT]", "[GC]", "[^A]", ".", "[a-c]"])
        else:
            node = rng.choice("ACGTacgt")
        q = rng.random()
        node += "?" if q < 0.15 else "*" if q < 0.22 else "+" if q < 0.29 else ""
        parts.append(node)
    return "".join(parts)


@pytest.mark.parametrize("seed", range(3))
def test_random_regular_patterns(oracle_mod, seed):
    """Alternation, '+', nested groups and anchors (the converter never
    emits '|' or '+', nrgrep's syntax has them)."""
    rng = random.Random(100 + seed)
    text = dna_fasta(20 + seed, n_records=3, max_len=200)
    checked = 0
    while checked < 60:
        pat = _random_pattern(rng)
        if rng.random() < 0.15:
            pat = "^" + pat
        if rng.random() < 0.15:
            pat += "$"
        try:
            prog = compile_pattern(pat)
        except RegexSyntaxError:
            continue
        if prog.m > 64:
            continue
        checked += 1
        for k, types in [(0, ""), (1, "ids"), (1, "s"), (2, "is"), (1, "d")]:
            if k and "d" in types and k >= prog.min_len:
                continue
            assert oracle_mod.scan(text, prog, k, types) == nrgrep_regex.candidates(text, pat, k, types), (pat, k, types)
            assert _reported(oracle_mod, text, prog, k, types) == nrgrep_regex.reported(text, pat, k, types), \
                (pat, k, types)


def test_prosite_config3_pattern(oracle_mod):
    """configs[3]: C-x(2,4)-C-x(3)-[LIVMFYWC] through the converter, on
    peptides with planted instances, k = 0 and k = 1 ids."""
    pat = convert("-p", "C-x(2,4)-C-x(3)-[LIVMFYWC]")
    prog = compile_pattern(pat)
    rng = random.Random(5)
    recs = []
    for r in range(12):
        seq = "".join(rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(150))
        for _ in range(3):
            at = rng.randrange(140)
            inst = "C" + "".join(rng.choice("AGST") for _ in range(rng.randint(1, 5))) + "C" + "KLM" + rng.choice("LIVMFYWC")
            seq = seq[:at] + inst + seq[at:]
        recs.append(">p%d\n%s\n" % (r, seq))
    text = "".join(recs).encode()
    for k, types in [(0, ""), (1, "ids"), (1, "s")]:
        assert oracle_mod.scan(text, prog, k, types) == nrgrep_regex.candidates(text, pat, k, types)
        assert _reported(oracle_mod, text, prog, k, types) == nrgrep_regex.reported(text, pat, k, types)
