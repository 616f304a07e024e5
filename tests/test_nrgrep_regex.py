"""The scan candidates and the report of non-simple patterns (``? * + |``,
groups: nrgrep's extended / eextended and regular / eregular engines) at
k >= 0, checked against an independent restatement that parses the nrgrep
pattern STRING itself and matches with a different algorithm
(oracle/nrgrep_regex.py: a relation over the parse tree, no position
automaton) -- so a bug in ``patmatchdocker_amd.regex.compile_pattern`` or in
the oracle's C cannot hide behind an oracle that consumes the same compiled
program.  The candidates must be equal; the report is nrgrep's own (each
engine's scanner order and nearest-boundary verify, restated from the binary
in oracle/pm_nrgrep_*.c), so every printed match must be a match of the
pattern string with at most k errors of the allowed kinds, start at a
candidate start, and never overlap the previous one.  The GPU kernels are
checked against the oracle (tests/test_gpu_*.py); this closes the loop for
every converter-golden non-simple pattern and for random patterns with
alternation and repetition."""
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


def _approx(tree, text: bytes, s: int, e: int, k: int, types: str) -> bool:
    nl = text.find(b"\n", s + 1 if s < len(text) and text[s] == 10 else s)
    m = nrgrep_regex._Matcher(text, len(text) if nl < 0 else nl, k, "i" in types, "d" in types, "s" in types)
    ends = m.insert(m.reach(tree, {(s, False): 0}))
    return any(j == e and err <= k for (j, _), err in ends.items())


def _check_report(oracle_mod, text, pat, prog, k, types):
    """nrgrep's report (the engine nrgrep_coords runs for this pattern) is a
    sequence of non-overlapping matches of the pattern string, each starting
    at a candidate start."""
    got = oracle_mod.scan_reported(text, prog, k, types)
    starts = {s for s, _ in nrgrep_regex.candidates(text, pat, k, types)}
    tree, _, _ = nrgrep_regex.parse(pat, True)
    last = -1
    # the eextended engine's phases report one character past the boundary
    # they found (pm_nrgrep_ext.c eleft 0x40e849 / eright 0x40f2a3: the start
    # is the character before the last one read, the end the one after the
    # next): its printed [s, e) holds the alignment in [s, s + 1] .. [e - 1, e]
    # and may begin one before the previous end or on the '\n' before a line
    ee = prog.kind == "extended" and k > 0
    if k == 0 and prog.linear:
        # the simple engine: windows of the whole text (a class holding '\n'
        # spans lines, tests/test_nrgrep_semantics.py)
        for s, e in got:
            assert s >= last and e - s == prog.m, (pat, got)
            last = e
            assert all(text[s + i] in cls or (97 <= text[s + i] <= 122 and text[s + i] - 32 in cls)
                       for i, cls in enumerate(prog.classes)), (pat, s, e)
        return len(got)
    for s, e in got:
        assert s >= last - (1 if ee else 0), (pat, k, types, got)
        last = e
        assert text[s] != 10 or ee, (pat, k, types, s, e)
        spans = [(s, e)] if not ee else [(a, b) for a in (s, s + 1) for b in (e, e - 1) if a <= b]
        assert any(a in starts and _approx(tree, text, a, b, k, types if k else "") for a, b in spans), \
            (pat, k, types, s, e)
    return len(got)


def _refused(prog, k, types):
    # engine.route: deletions that can empty the pattern walk every line
    # (empty matches: not candidates), eregular restated up to 63 positions
    return bool(k) and (("d" in types and k >= prog.min_len) or (prog.kind == "regular" and prog.m + 1 > 64))


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
            if _refused(prog, k, types):
                continue
            assert oracle_mod.scan(text, prog, k, types) == nrgrep_regex.candidates(text, pat, k, types), (pat, k, types)
            _check_report(oracle_mod, text, pat, prog, k, types)


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
            if _refused(prog, k, types):
                continue
            assert oracle_mod.scan(text, prog, k, types) == nrgrep_regex.candidates(text, pat, k, types), (pat, k, types)
            _check_report(oracle_mod, text, pat, prog, k, types)


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
        _check_report(oracle_mod, text, pat, prog, k, types)
