"""The GPU's eextended report (pm_eextended.hip: nrgrep's eextendedPreproc
plan, its piece / window / prefix scanners and checkMatch1 replayed per
cluster of alignment starts) against the oracle's literal replay
(oracle/pm_nrgrep_ext.c, pmx_eextended), k = 1..3 with every error-type
combination the web form builds (patmatch.py:299-314), on texts where
approximate matches overlap densely: PatMatch ranges on DNA repeats,
configs[3]'s PROSITE pattern on Cys-rich peptides (configs[3] at -k 1ids is
the verdict's done-criterion), random extended patterns, both layouts and
nrgrep's search regions."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.engine import UnsupportedOnGPU
from patmatchdocker_amd.regex import compile_pattern
from tests.test_gpu_extended import repeats_fasta, DNA_RANGES
from tests.test_nrgrep_extended import random_extended, dense_text

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


def _check(engine, oracle_mod, text, progs, k, types, alphabet=None):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alphabet, device=0)
    try:
        ran = 0
        for prog in progs:
            try:
                res, _ = engine.scan(db, [prog], k=k, types=types)
            except UnsupportedOnGPU:
                assert "d" in types and prog.min_len <= k, prog.source
                continue
            want = oracle_mod.scan_reported(text, prog, k, types, skip_headers=True)
            assert _pairs(res[0]) == want, (prog.source, k, types, oracle_mod.eextended_plan(prog, k))
            ran += 1
        return ran
    finally:
        db.close()


@pytest.mark.parametrize("k,types", [(1, "ids"), (2, "ids"), (3, "ids"), (1, "s"), (2, "is"), (1, "d")])
def test_dna_ranges_on_repeats(engine, oracle_mod, k, types):
    text = repeats_fasta(4, n_records=4, rec_len=5000)
    progs = [compile_pattern(convert(f, p)) for p in DNA_RANGES for f in ("-n", "-c")]
    progs = [p for p in progs if p.kind == "extended"]
    assert _check(engine, oracle_mod, text, progs, k, types, alphabet="nuc") >= 8


@pytest.mark.parametrize("k", [1, 2])
def test_prosite_config3_on_cys_rich_peptides(engine, oracle_mod, k):
    """configs[3] C-x(2,4)-C-x(3)-[LIVMFYWC] at -k <k>ids on peptides full of
    overlapping Cys pairs (the CACAACAAAL shape)."""
    prog = compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))
    rng = random.Random(18 + k)
    recs = []
    for r in range(30):
        seq = []
        while len(seq) < 300:
            x = rng.random()
            if x < 0.4:
                seq += list("C" + "".join(rng.choice("ACKS") for _ in range(rng.randint(0, 5))))
            elif x < 0.6:
                seq += list("CACAACAAAL")
            else:
                seq += [rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(rng.randint(1, 20))]
        recs.append(">p%d\n%s\n" % (r, "".join(seq)))
    text = "".join(recs).encode()
    assert _check(engine, oracle_mod, text, [prog], k, "ids", alphabet="byte") == 1
    assert _check(engine, oracle_mod, repeats_fasta(9, alphabet="pep", width=60), [prog], k, "ids",
                  alphabet="byte") == 1


def test_three_residue_range_at_k3(engine, oracle_mod):
    """A 3-residue ranged pattern at -k 3ids (the verdict's second case):
    deletions reach the shortest match, so the GPU refuses it unless the
    shortest match is longer than k."""
    rng = random.Random(3)
    text = b"".join(dense_text(rng, "pep", n_lines=40, width=(30, 200)) for _ in range(3))
    progs = [compile_pattern(convert("-p", p)) for p in ("CX{1,3}CK", "LX{0,2}GKS", "C-x(2)-[ST]-x(0,2)-K")]
    progs = [p for p in progs if p.kind == "extended"]
    assert len(progs) >= 2
    _check(engine, oracle_mod, text, progs, 3, "ids", alphabet="byte")
    _check(engine, oracle_mod, text, progs, 3, "s", alphabet="byte")


@pytest.mark.parametrize("alphabet", ["dna", "pep"])
def test_deletions_reaching_the_shortest_match(engine, oracle_mod, alphabet):
    """-k <k>ids with k >= the shortest match: empty alignments anywhere, so
    the walk takes every line (ee_add_lines) instead of refusing."""
    rng = random.Random(77)
    text = b"".join(dense_text(rng, alphabet, n_lines=30, width=(10, 120)) for _ in range(2))
    pats = ["GAN{0,1}TC", "AN{0,2}T"] if alphabet == "dna" else ["CX{0,2}C", "KX{1,2}L"]
    mode = "-n" if alphabet == "dna" else "-p"
    progs = [compile_pattern(convert(mode, p)) for p in pats]
    progs = [p for p in progs if p.kind == "extended"]
    assert progs
    layout = "nuc" if alphabet == "dna" else "byte"
    for prog in progs:
        k = prog.min_len
        assert _check(engine, oracle_mod, text, [prog], k, "ids", alphabet=layout) == 1
        assert _check(engine, oracle_mod, text, [prog], k, "d", alphabet=layout) == 1


@pytest.mark.parametrize("seed", range(4))
def test_random_extended_patterns(engine, oracle_mod, seed):
    rng = random.Random(600 + seed)
    for alpha, layout in (("dna", "nuc"), ("pep", "byte")):
        progs = [random_extended(rng, alpha)[1] for _ in range(10)]
        text = b"".join(dense_text(rng, alpha, n_lines=50, width=(20, 300)) for _ in range(3))
        for k, types in ((1, "ids"), (2, rng.choice(["ids", "is", "s", "id"])), (3, "ids")):
            _check(engine, oracle_mod, text, progs, k, types, alphabet=layout)


def test_eextended_over_search_regions(engine, oracle_mod):
    """A file over nrgrep's 1.6 MB buffer, including a 2 Mbp one-line record
    cut blind: the report restarts at every region start."""
    rng = random.Random(23)
    recs = []
    for r in range(3):
        seq = "".join(rng.choice("AAT" if r == 1 else "ACGT") for _ in range(rng.randint(700_000, 2_100_000)))
        recs.append(">c%d\n%s\n" % (r, seq if r == 1 else "\n".join(seq[i:i + 60] for i in range(0, len(seq), 60))))
    text = "".join(recs).encode()
    progs = [compile_pattern(convert("-n", p)) for p in ("AN{0,3}GAATTC", "TAN{0,3}TA", "GAN{2,3}TC")]
    _check(engine, oracle_mod, text, progs, 1, "ids", alphabet="nuc")
    _check(engine, oracle_mod, text, progs[:1], 2, "ids", alphabet="nuc")
