"""nrgrep's eregular engine (the regular patterns of test_nrgrep_regular.py at
k > 0: PatMatch's group repeats with mismatches), restated from the binary's
disassembly (oracle/pm_nrgrep_reg.c, eregularPreproc 0x406a20 .. checkMatch
0x406010).

* the library's host plan (pm_eregular_plan, C++) equals the oracle's (C):
  pieces against windows, detClass of the first window, checkMatch's state
  word for class 1;
* every printed match is an approximate occurrence of the pattern STRING with
  at most k errors of the allowed kinds (oracle/nrgrep_regex.py's own
  matcher), and printed matches never overlap;
* a plan whose first window is an extended sequence prints nothing (the
  binary dies in eregularPreproc);
* deletions with k >= the shortest match print empty matches too."""
import random

import pytest

from oracle import nrgrep_regex
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.test_nrgrep_regular import GROUP_REPEATS, _dense_text, _patterns

ERRS = [(1, "ids"), (1, "s"), (2, "ids"), (1, "d"), (2, "is"), (1, "i"), (3, "ids")]


def _small(pats):
    return [(p, prog) for p, prog in pats if prog.m + 1 <= 64]


def _group_progs():
    out = []
    for mode, pat in GROUP_REPEATS:
        for strand in ([mode, "-c"] if mode == "-n" else [mode]):
            p = convert(strand, pat) if strand != "-c" else convert("-c", convert("-n", pat))
            prog = compile_pattern(p)
            if prog.kind == "regular":
                out.append((p, prog))
    return out


def test_plan_library_equals_oracle(oracle_mod):
    pats = _small(_patterns(200, 3) + _patterns(80, 4, "ACDEFGHIKLMNPQRSTVWY") + _group_progs())
    kinds = set()
    for pat, prog in pats:
        for k in (1, 2, 3):
            want = oracle_mod.eregular_plan(prog, k)
            got = engine.eregular_plan(prog, k)
            for key in ("type", "ell", "cls", "defined", "windows", "match"):
                assert got[key] == want[key], (pat, k, key, got, want)
            kinds.add((want["type"], want["cls"]))
    # pieces and windows of both classes, forward plans and dying plans occur
    assert {(1, 1), (1, 3), (2, 3), (3, 3)} <= kinds, kinds
    assert any(c == 2 for _, c in kinds), kinds


def _approx(pattern: str, text: bytes, s: int, e: int, k: int, types: str) -> bool:
    tree, _, _ = nrgrep_regex.parse(pattern, True)
    nl = text.find(b"\n", s)
    m = nrgrep_regex._Matcher(text, len(text) if nl < 0 else nl, k, "i" in types, "d" in types, "s" in types)
    ends = m.insert(m.reach(tree, {(s, False): 0}))
    return any(j == e and err <= k for (j, _), err in ends.items())


@pytest.mark.parametrize("seed", range(3))
def test_printed_matches_are_approximate_occurrences(oracle_mod, seed):
    rng = random.Random(70 + seed)
    pats = _small(_patterns(14, 80 + seed)) + (_group_progs() if seed == 0 else [])
    checked = 0
    for pat, prog in pats:
        tokens = [c for c in pat if c.isalpha()] + ["A", "C", "G", "T"]
        pieces = ["".join(rng.choice(tokens) for _ in range(rng.randint(1, 4))) for _ in range(8)]
        text = _dense_text(rng, pieces, n_lines=4)
        for k, types in ERRS[:4] if seed else ERRS:
            got = oracle_mod.scan_reported(text, prog, k, types, bufsize=0)
            last = -1
            for s, e in got:
                assert s >= last, (pat, k, types, got)
                last = e
                assert _approx(prog.source, text, s, e, k, types), (pat, k, types, s, e, text[s:e])
            checked += len(got)
    assert checked > 200


def test_extended_first_window_prints_nothing(oracle_mod):
    """detClass 2 on the first window: eregularPreproc writes through a null
    pointer (0x4081ed) and nrgrep_coords dies before it scans."""
    prog, k = compile_pattern("(CA)+C(T)+(TGT|TT)+."), 1
    plan = oracle_mod.eregular_plan(prog, k)
    assert plan["cls"] == 2 and engine.eregular_plan(prog, k)["cls"] == 2
    text = _dense_text(random.Random(1), [c for c in prog.source if c.isalpha()] + ["ACGT"])
    assert oracle_mod.scan_reported(text, prog, k, "ids", bufsize=0) == []
    assert oracle_mod.scan_reported(text, prog, k, "ids", report="leftmost", bufsize=0)


def test_deletions_to_nothing_print_empty_matches(oracle_mod):
    """k >= the shortest match with deletions: the whole pattern can be
    deleted, nrgrep prints empty matches as well."""
    prog = compile_pattern("(G(CA)?(CA)?T)")
    assert prog.min_len == 2
    text = b">x\nAAAGCACATAAAAAAAAAAAAGCATTTTTTTT\n"
    got = oracle_mod.scan_reported(text, prog, 2, "ids", bufsize=0)
    assert any(s == e for s, e in got) and any(e > s for s, e in got)
    for s, e in got:
        assert _approx(prog.source, text, s, e, 2, "ids")


def test_group_repeat_mismatches_converter_patterns(oracle_mod):
    """GA(TC){1,2}A at -k 1ids (PatMatch's default letters) over tandem
    repeats (its -c strand, ((T?(GA)(GA)TC)), is an extended pattern): the
    plan and the printed matches."""
    prog = compile_pattern(convert("-n", "GA(TC){1,2}A"))
    for k in (1, 2):
        plan = oracle_mod.eregular_plan(prog, k)
        got_plan = engine.eregular_plan(prog, k)
        assert all(got_plan[key] == plan[key] for key in got_plan)
    rng = random.Random(11)
    text = _dense_text(rng, ["GATC", "GATCTCA", "GA", "TCA", "A", "TC", "GC"], n_lines=5)
    got = oracle_mod.scan_reported(text, prog, 1, "ids", bufsize=0)
    assert len(got) > 5
    for s, e in got:
        assert _approx(prog.source, text, s, e, 1, "ids")


# Group repeats past 63 positions (round 6): the eregular verify's rows span
# several words.  fwdCheck / bwdCheck read the regularMakeDet tables (states
# t W .. t W + W - 1, W = ceil(m / ceil(m / 16))) by SLICE with an offset that
# jumps to the next word when a slice would cross one (0x403530), so where W
# does not divide 64 the states past the jump take other states' transitions
# (oracle etab).  With W = 16 the verify is the automaton's own.
LONG_REPEATS = [
    ("-n", "(CA){37,38}G"),      # 78 states, W = 16: exact
    ("-n", "(CA){37,38}GT"),     # 79 states, W = 16
    ("-n", "(GATC){8,16}T"),     # 66 states, W = 14: a jump over states 56 .. 63
    ("-c", "(GATC){8,16}"),      # 65 states, W = 13
    ("-n", "(CA){20,40}GT"),     # 83 states, W = 14
    ("-c", "(CA){20,40}GT"),
    ("-c", "AC(GT){30,35}"),     # 73 states
]


def _long_progs():
    out = []
    for strand, pat in LONG_REPEATS:
        src = convert("-n", pat) if strand == "-n" else convert("-c", convert("-n", pat))
        prog = compile_pattern(src)
        assert prog.kind == "regular" and prog.m + 1 > 64, (strand, pat, prog.kind, prog.m)
        out.append(((strand, pat), prog))
    return out


def _slice_width(states):
    nt0 = (states + 15) // 16
    return (states + nt0 - 1) // nt0


def test_long_plan_library_equals_oracle(oracle_mod):
    for name, prog in _long_progs():
        for k in (1, 2, 3):
            want = oracle_mod.eregular_plan(prog, k)
            got = engine.eregular_plan(prog, k)
            for key in ("type", "ell", "cls", "defined", "windows", "match"):
                assert got[key] == want[key], (name, k, key)
            assert want["states"] == prog.m + 1 if want["cls"] == 1 else want["states"] <= 64


def _planted(rng, units, lines=30):
    def mutate(s, n):
        s = list(s)
        for _ in range(n):
            i, op = rng.randrange(len(s)), rng.randrange(3)
            if op == 0:
                s[i] = rng.choice("ACGT")
            elif op == 1:
                del s[i]
            else:
                s.insert(i, rng.choice("ACGT"))
        return "".join(s)
    out = []
    for r in range(lines):
        line = "".join(rng.choice("ACGT") for _ in range(rng.randint(5, 30)))
        line += mutate(rng.choice(units), rng.randint(0, 2)) + "".join(rng.choice("ACGT") for _ in range(rng.randint(0, 9)))
        out.append(">s%d\n%s\n" % (r, line))
    return "".join(out).encode()


def test_long_repeats_with_aligned_slices_print_approximate_occurrences(oracle_mod):
    """W = 16: every slice is one word's, the verify follows the automaton:
    every print is an occurrence with <= k errors, prints never overlap."""
    rng = random.Random(606)
    for (strand, pat), prog in _long_progs()[:2]:
        assert _slice_width(prog.m + 1) == 16
        text = _planted(rng, ["CA" * 37 + "G", "CA" * 38 + "GT", "CA" * 36 + "G", "CA" * 40])
        for k, types in [(1, "ids"), (2, "ids"), (1, "s"), (2, "d")]:
            got = oracle_mod.scan_reported(text, prog, k, types, bufsize=0)
            assert len(got) >= 5, (pat, k, types)
            last = -1
            for s, e in got:
                assert s >= last and _approx(prog.source, text, s, e, k, types), (pat, k, types, s, e)
                last = e


def test_long_repeat_whose_slices_jump_prints_nothing(oracle_mod):
    """(CA){20,40}GT: 83 states, W = 14, the fifth slice jumps from state 56
    to 64; states 56 .. 63 take no transition in fwdCheck, the piece
    candidates' forward phase dies there, nothing is printed (the restated
    binary; parity unpinned)."""
    rng = random.Random(607)
    (_, prog) = _long_progs()[4]
    text = _planted(rng, ["CA" * 20 + "GT", "CA" * 30 + "GT", "CA" * 40 + "GT"])
    assert oracle_mod.scan_py_reported(text[:3000], prog, 1, "ids")   # real occurrences exist
    for k, types in [(1, "ids"), (2, "ids"), (1, "s")]:
        assert oracle_mod.scan_reported(text, prog, k, types, bufsize=0) == []
