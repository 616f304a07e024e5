"""nrgrep's eextended engine (patterns with '?', '*', '+' searched with
k > 0 errors: every PatMatch range under the web form's default -k <k>ids),
restated from the binary's disassembly in oracle/pm_nrgrep_ext.c
(pmx_eextended): its plan against the library's own C++ restatement
(pm_eextended_plan), every printed match against an independent matcher
(oracle/nrgrep_regex.py, the pattern string's own dynamic program), and the
quirks derived by hand from the code.  The GPU is checked against the
replay in tests/test_gpu_eextended.py."""
import random

import pytest

from oracle import oracle
from oracle import nrgrep_regex
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.test_nrgrep_extended import random_extended, dense_text, _golden_extended


@pytest.mark.parametrize("seed", range(2))
def test_library_plan_matches_the_replay(seed):
    """pm_eextended_plan (C++, the GPU's host side) vs pmx_eplan (C, the
    oracle): extendedFindBest at K = k, the piece DP over the overlapping
    cost table, the trims and thresholds decide the scanner."""
    rng = random.Random(1700 + seed)
    progs = [compile_pattern(p) for p in _golden_extended()]
    while len(progs) < 400:
        progs.append(random_extended(rng, rng.choice(["dna", "pep"]))[1])
    kinds = set()
    for prog in progs:
        for k in (1, 2, 3, 4):
            want = oracle.eextended_plan(prog, k)
            assert engine.eextended_plan(prog, k) == want, (prog.source, k)
            kinds.add((want["type"], want["simple"]))
    # pieces (both scanners) and the prefix; a window is rare at k > 0
    assert {(1, True), (1, False), (3, False)} <= kinds


def test_plans_of_patmatch_ranges():
    """configs[3] runs the extended prefix scanner; GAN{2,3}TC at -k 1 splits
    into the simple pieces GA / TC, so nrgrep runs esimpleScan's BNDM."""
    p3 = compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))
    assert oracle.eextended_plan(p3, 1)["type"] == 3
    p = compile_pattern(convert("-n", "GAN{2,3}TC"))
    plan = oracle.eextended_plan(p, 1)
    assert (plan["type"], plan["simple"], plan["plen"], plan["pieces"]) == (1, True, 2, [(0, 2), (5, 7)])


def _alignments(text, prog, k, types, a, b):
    """(s, e) with s in {a, a + 1}, e in {b - 1, b} aligning the pattern with
    <= k errors of the given types, by the pattern string's own matcher."""
    tree, _, _ = nrgrep_regex.parse(prog.source, True)
    nl = text.find(b"\n", max(a, 0))
    end = len(text) if nl < 0 else nl
    out = []
    for s in (a, a + 1):
        if s < 0:
            continue
        m = nrgrep_regex._Matcher(text, max(end, b), k, "i" in types, "d" in types, "s" in types)
        ends = m.insert(m.reach(tree, {(s, False): 0}))
        out += [(s, e) for (e, u), err in ends.items() if e in (b - 1, b) and err <= k]
    return out


@pytest.mark.parametrize("seed", range(3))
def test_every_print_is_an_alignment_within_one(seed):
    """checkMatch1 records a boundary found after reading a character one
    position further out, so a print [a, b) is an alignment [s, e) with
    s - a, b - e in {0, 1}."""
    rng = random.Random(2100 + seed)
    checked = 0
    while checked < 25:
        alpha = rng.choice(["dna", "pep"])
        _, prog = random_extended(rng, alpha)
        k = rng.choice([1, 2, 3])
        types = rng.choice(["ids", "ids", "s", "is", "id"])
        text = dense_text(rng, alpha, n_lines=10, width=(10, 80))
        for a, b in oracle.scan_eextended(text, prog, k, types, bufsize=0):
            assert _alignments(text, prog, k, types, a, b), (prog.source, k, types, (a, b), text[max(0, a - 5):b + 5])
        checked += 1


def test_exact_match_prints_one_past_its_end():
    """GAN{2,3}TC at -k 1 (GA...?TC): piece GA found at 6 (L = 0, the start is
    the candidate itself), the right phase reads GAATTC and reaches the last
    position on the C at 11 -- recorded as Y + 1 = 13 (checkMatch1 0x40f3da,
    0x40ed59): nrgrep prints [6, 13), "GAATTCG"."""
    text = b">s\nTTTGAATTCGGG\n"
    prog = compile_pattern(convert("-n", "GAN{2,3}TC"))
    assert (6, 13) in oracle.scan_eextended(text, prog, 1, "ids", bufsize=0)
    assert (6, 13) in oracle.scan_reported(text, prog, 1, "ids")


def test_start_before_the_file_is_dropped():
    """A match reading the file's first byte prints start -1; process_output
    maps it to the first record's header (get_name_offset, patmatch.py
    :217-238) and drops it (:548-550); the header filter does the same."""
    prog = compile_pattern("(A..?.?.?A)")
    text = b">r0\nAAAAAAAA\n"
    raw = oracle.scan_eextended(text, prog, 2, "ids", bufsize=0)
    assert raw and raw[0][0] == -1
    assert all(a >= 0 for a, _ in oracle.scan_eextended(text, prog, 2, "ids", skip_headers=True, bufsize=0))


def test_header_line_match_prints_on_the_previous_line():
    """An alignment starting a header line is printed from the '\\n' before
    it, which process_output keeps (it maps to the previous record):
    the GPU walk therefore starts a cluster at every header line."""
    rng = random.Random(600)
    progs = [random_extended(rng, "dna")[1] for _ in range(10)]
    text = b"".join(dense_text(rng, "dna", n_lines=50, width=(20, 300)) for _ in range(3))
    prog = [p for p in progs if p.source == "([CT]?T.+.?[CT][GC][AG]*)"][0]
    hits = oracle.scan_reported(text, prog, 3, "ids", skip_headers=True)
    assert (1116, 1118) in hits and text[1116:1118] == b"\n>"


@pytest.mark.parametrize("k", [1, 2])
def test_regions_restart_the_report(k):
    """by_region over nrgrep's 1.6 MB buffers equals each region searched as
    a text of its own."""
    rng = random.Random(40 + k)
    body = "".join(rng.choice("ACGT") for _ in range(1_700_000))
    text = (">c\n" + "\n".join(body[i:i + 70] for i in range(0, len(body), 70)) + "\n").encode()
    prog = compile_pattern(convert("-n", "AN{0,3}GAATTC"))
    regs = oracle.regions(text)
    assert len(regs) == 2
    got = oracle.scan_eextended(text, prog, k, "ids")
    want = []
    for a, b in regs:
        want += [(x + a, y + a) for x, y in oracle.scan_eextended(text[a:b], prog, k, "ids", bufsize=0)]
    assert got == want
