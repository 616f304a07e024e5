"""The GPU's regular report (pm_regular.hip: nrgrep's regularFindBest plan
over its parse tree, regularScan's backward window / forward automaton and
checkMatch's nearest boundaries, replayed per cluster of match starts)
against the oracle's literal replay of the binary's loops
(oracle/pm_nrgrep_reg.c), k = 0.  Group repeats through the converter
(GA(TC){1,2}A -> (GA(TC)(TC)?A), patmatch_to_nrgrep.pl:307-348, 462-495) on
tandem repeats where matches overlap densely, an unbounded repeat (lines
mode), a forward plan, peptide group repeats on the byte layout, random
regular patterns with '|' and anchors, N runs, lower case, both layouts, and
a group repeat whose window is a class sequence (nrgrep prints nothing)."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.test_nrgrep_regular import _patterns

pytestmark = pytest.mark.gpu

DNA_GROUPS = ["GA(TC){1,2}A", "G(TATA){2,}C", "(CA){2,4}GT", "A(TG){0,2}C", "(GA){1,3}(TC){2}",
              "NN(TC){1,2}GAATTC", "GAATTC(CA){2,3}N", "T(AT){1,3}[AG]", "(TA){2,3}(GC){1,2}"]
PEP_GROUPS = ["C(AG){1,3}L", "K(RK){1,2}XXC", "(GH){2,4}W", "W(CP){1,2}[LIV]", "(RK){2,}G", "KX(RK){1,2}C"]


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine as eng
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def _pairs(r):
    return list(zip(r[0].tolist(), r[1].tolist()))


def tandem_fasta(seed, units, n_records=6, rec_len=5000, width=60, letters="ACGT", n_runs=True):
    rng = random.Random(seed)
    out = []
    for r in range(n_records):
        parts = []
        while sum(map(len, parts)) < rec_len:
            x = rng.random()
            if x < 0.5:
                parts.append(rng.choice(units) * rng.randint(1, 12))
            elif x < 0.56 and n_runs:
                parts.append("N" * rng.randint(1, 20))
            else:
                parts.append("".join(rng.choice(letters) for _ in range(rng.randint(3, 60))))
        seq = "".join(parts)[:rec_len]
        if rng.random() < 0.25:
            seq = seq.lower()
        body = "\n".join(seq[i:i + width] for i in range(0, len(seq), width)) if width else seq
        out.append(">r%d tandem repeats\n%s\n" % (r, body))
    return "".join(out).encode()


def _check(engine, oracle_mod, text, progs, alphabet=None, k=0, types=""):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alphabet, device=0)
    total = 0
    try:
        res, _ = engine.scan(db, progs, k=k, types=types)
        for prog, r in zip(progs, res):
            want = oracle_mod.scan_reported(text, prog, k, types, skip_headers=True)
            got = _pairs(r)
            plan = oracle_mod.regular_plan(prog) if k == 0 else oracle_mod.eregular_plan(prog, k, types)
            assert got == want, (prog.source, k, types, plan, len(got), len(want),
                                 sorted(set(got) ^ set(want))[:6])
            total += len(want)
    finally:
        db.close()
    return total


@pytest.mark.parametrize("width", [60, None])
def test_dna_group_repeats_on_tandem_repeats(engine, oracle_mod, width):
    progs = []
    for p in DNA_GROUPS:
        progs += [compile_pattern(convert("-n", p)), compile_pattern(convert("-c", p))]
    progs = [p for p in progs if p.kind == "regular"]
    assert len(progs) >= 14
    plans = [oracle_mod.regular_plan(p) for p in progs]
    assert any(pl["type"] == 3 for pl in plans) and any(pl["cls"] == 1 for pl in plans)
    text = tandem_fasta(3, ["GATC", "GATCTCA", "TATA", "CA", "TC", "GA", "TG", "GAATTC", "GC", "AT"], width=width)
    assert _check(engine, oracle_mod, text, progs) > 200


def test_peptide_group_repeats(engine, oracle_mod):
    progs = [compile_pattern(convert("-p", p)) for p in PEP_GROUPS]
    progs = [p for p in progs if p.kind == "regular"]
    assert len(progs) == len(PEP_GROUPS)
    text = tandem_fasta(4, ["CAG", "AG", "CP", "GH", "RK", "C", "W", "L", "CAGL", "KRKRK", "WCPL", "GHW", "RKG"],
                        letters="ACDEFGHIKLMNPQRSTVWY", n_runs=False)
    assert _check(engine, oracle_mod, text, progs, alphabet="byte") > 50


@pytest.mark.parametrize("seed", range(3))
def test_random_regular_patterns(engine, oracle_mod, seed):
    """'|', groups with '?*+', classes, '.', anchors; nucleotide layout."""
    pats = [p for _, p in _patterns(30, 200 + seed)]
    tokens = ["A", "C", "G", "T", "AC", "GT", "TA", "CCG", "AAT", "GAGA"]
    text = tandem_fasta(10 + seed, tokens, n_records=4, rec_len=3000)
    _check(engine, oracle_mod, text, pats)


def test_class_sequence_window_prints_nothing(engine, oracle_mod):
    prog = compile_pattern(convert("-n", "GAATTC(CA){2,3}N"))
    assert oracle_mod.regular_plan(prog)["cls"] == 1
    text = b">x\nAAGAATTCCACAGTTTGAATTCCACACATT\nGAATTCCACACAGG\n"
    db = engine.SequenceDatabase.from_bytes(text, device=0)
    try:
        res, _ = engine.scan(db, [prog], k=0)
        assert _pairs(res[0]) == [] == oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True)
        # the leftmost-start rule would have printed them
        assert oracle_mod.scan_reported(text, prog, 0, "", report="leftmost")
    finally:
        db.close()


def test_long_records_many_clusters(engine, oracle_mod):
    """2 Mbp of one-line records with planted tandem instances: thousands of
    clusters, a file over nrgrep's 1.6 MB buffer (two search regions)."""
    rng = random.Random(9)
    recs = []
    for r in range(2):
        seq = []
        n = 0
        while n < 1_000_000:
            x = rng.random()
            piece = (rng.choice(["GATC", "GATCTC", "TCTC"]) + "A") if x < 0.05 else \
                "".join(rng.choice("ACGT") for _ in range(rng.randint(20, 400)))
            seq.append(piece)
            n += len(piece)
        recs.append(">chr%d\n%s\n" % (r, "".join(seq)))
    text = "".join(recs).encode()
    progs = [compile_pattern(convert("-n", "GA(TC){1,2}A")), compile_pattern(convert("-c", "GA(TC){1,2}A"))]
    assert _check(engine, oracle_mod, text, progs) > 1000


# ---------------------------------------------------------------------------
# k > 0: nrgrep's eregular engine (pieces, backward windows with k errors,
# the automaton forward; esimple's scanners when the first window is a class
# sequence) against the oracle's replay (pm_nrgrep_reg.c)
# ---------------------------------------------------------------------------

EREG_ERRS = [(1, "ids"), (1, "s"), (2, "ids"), (1, "d"), (2, "is")]


@pytest.mark.parametrize("k,types", EREG_ERRS)
def test_dna_group_repeats_with_errors(engine, oracle_mod, k, types):
    progs = []
    for p in DNA_GROUPS:
        progs += [compile_pattern(convert("-n", p)), compile_pattern(convert("-c", convert("-n", p)))]
    progs = [p for p in progs if p.kind == "regular" and p.m + 1 <= 64]
    plans = [oracle_mod.eregular_plan(p, k, types) for p in progs]
    assert {pl["type"] for pl in plans} >= {1, 3}
    text = tandem_fasta(5 + k, ["GATC", "GATCTCA", "TATA", "CA", "TC", "GA", "TG", "GAATTC", "GC", "AT"],
                        n_records=4, rec_len=3000)
    assert _check(engine, oracle_mod, text, progs, k=k, types=types) > 100


@pytest.mark.parametrize("k,types", [(1, "ids"), (1, "s"), (2, "ids")])
def test_peptide_group_repeats_with_errors(engine, oracle_mod, k, types):
    progs = [compile_pattern(convert("-p", p)) for p in PEP_GROUPS]
    progs = [p for p in progs if p.kind == "regular"]
    text = tandem_fasta(6, ["CAG", "AG", "CP", "GH", "RK", "C", "W", "L", "CAGL", "KRKRK", "WCPL", "GHW", "RKG"],
                        letters="ACDEFGHIKLMNPQRSTVWY", n_runs=False, n_records=4, rec_len=3000)
    assert _check(engine, oracle_mod, text, progs, alphabet="byte", k=k, types=types) > 20


@pytest.mark.parametrize("seed", range(2))
def test_random_regular_patterns_with_errors(engine, oracle_mod, seed):
    pats = [p for _, p in _patterns(20, 300 + seed) if p.m + 1 <= 64]
    tokens = ["A", "C", "G", "T", "AC", "GT", "TA", "CCG", "AAT", "GAGA"]
    text = tandem_fasta(20 + seed, tokens, n_records=3, rec_len=2000)
    for k, types in [(1, "ids"), (2, "s"), (1, "d")]:
        ok = [p for p in pats if not ("d" in types and p.min_len <= k)]
        _check(engine, oracle_mod, text, ok, k=k, types=types)


def test_deletions_to_nothing_every_line(engine, oracle_mod):
    """k >= the shortest match with deletions: every position is a key, every
    line a cluster; nrgrep prints empty matches too."""
    progs = [compile_pattern("(G(CA)?(CA)?T)"), compile_pattern(convert("-n", "GA(TC){1,2}A"))]
    text = tandem_fasta(31, ["GCAT", "GT", "CA", "GATC", "TCA"], n_records=3, rec_len=600)
    assert _check(engine, oracle_mod, text, progs[:1], k=2, types="ids") > 100
    assert _check(engine, oracle_mod, text, progs[1:], k=5, types="d") > 10


def test_long_records_with_errors(engine, oracle_mod):
    """2 Mbp of one-line records, planted GA(TC){1,2}A variants, -k 1ids: two
    search regions, clusters inside a line."""
    rng = random.Random(19)
    recs = []
    for r in range(2):
        seq, n = [], 0
        while n < 1_000_000:
            piece = rng.choice(["GATCA", "GATCTCA", "GTTCA", "GATTCA", "GACTCA"]) if rng.random() < 0.05 else \
                "".join(rng.choice("ACGT") for _ in range(rng.randint(20, 400)))
            seq.append(piece)
            n += len(piece)
        recs.append(">chr%d\n%s\n" % (r, "".join(seq)))
    text = "".join(recs).encode()
    progs = [compile_pattern(convert("-n", "GA(TC){1,2}A"))]
    assert _check(engine, oracle_mod, text, progs, k=1, types="ids") > 1000


@pytest.mark.parametrize("width", [60, None])
def test_long_group_repeats_at_k_above_zero(engine, oracle_mod, width):
    """Group repeats past 63 positions (round 6): the eregular verify over
    several words, the sliced transition tables of fwdCheck / bwdCheck with
    their word jumps (tests/test_nrgrep_eregular.py LONG_REPEATS) -- the
    verdict's (GATC){8,16} and (CA){20,40}GT among them -- over tandem
    repeats long enough to match, -k 1ids / 2ids / 1s / 2d, both layouts."""
    from tests.test_nrgrep_eregular import _long_progs
    progs = [p for _, p in _long_progs()]
    text = tandem_fasta(606, ["CA" * 37 + "G", "CA" * 38 + "GT", "GATC" * 9 + "T", "GATC" * 13, "CA" * 25 + "GT",
                              "AC" * 31 + "GT", "CA", "GATC", "TG"], n_records=5, rec_len=6000, width=width)
    total = 0
    for k, types in [(1, "ids"), (2, "ids"), (1, "s"), (2, "d")]:
        total += _check(engine, oracle_mod, text, progs, k=k, types=types)
    assert total > 30
