"""The GPU's extended report (pm_extended.hip: nrgrep's extendedFindBest
plan, window / prefix scanners and nearest-boundary checkMatch replayed per
cluster of match starts) against the oracle's replay of the binary's loops
(oracle/pm_nrgrep_ext.c), k = 0, on texts where matches overlap densely:
PatMatch ranges X{m,n} and {m,} (every one becomes X..?.? / X*, an extended
pattern), configs[3]'s PROSITE pattern on Cys-rich peptides, windows away
from the pattern start (the nearest start wins there), prefix scans, '*' and
'+', anchors, headers, N runs, lower case, both layouts, search regions."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.test_nrgrep_extended import random_extended, dense_text

pytestmark = pytest.mark.gpu

DNA_RANGES = ["GAN{2,3}TC", "GA{2,}TC", "AN{0,3}GAATTC", "TTTTN{0,2}CCCC", "AN{1,4}A", "W{1,3}N{0,2}GG",
              "[AG]N{2,5}[CT]", "TAN{0,3}TA", "AT{1,3}A{1,2}T", "RN{0,4}GG", "CN{0,3}G{2,}"]


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine as eng
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def _pairs(r):
    return list(zip(r[0].tolist(), r[1].tolist()))


def repeats_fasta(seed, n_records=5, rec_len=6000, width=60, alphabet="dna"):
    rng = random.Random(seed)
    out = []
    units = (["AT", "A", "GAA", "GGCC", "AAT", "TTTTCCCC", "CG"] if alphabet == "dna"
             else ["C", "CA", "CAAC", "CCK", "LIVC", "CKLM"])
    letters = "ACGT" if alphabet == "dna" else "ACDEFGHIKLMNPQRSTVWY"
    for r in range(n_records):
        parts = []
        while sum(map(len, parts)) < rec_len:
            x = rng.random()
            if x < 0.45:
                parts.append(rng.choice(units) * rng.randint(2, 40))
            elif x < 0.55 and alphabet == "dna":
                parts.append("N" * rng.randint(1, 30))
            else:
                parts.append("".join(rng.choice(letters) for _ in range(rng.randint(5, 200))))
        seq = "".join(parts)[:rec_len]
        if rng.random() < 0.3:
            seq = seq.lower()
        body = "\n".join(seq[i:i + width] for i in range(0, len(seq), width)) if width else seq
        out.append(">r%d some description\n%s\n" % (r, body))
    return "".join(out).encode()


def _check(engine, oracle_mod, text, progs, alphabet=None):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alphabet, device=0)
    try:
        res, _ = engine.scan(db, progs, k=0)
        for prog, r in zip(progs, res):
            want = oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True)
            assert _pairs(r) == want, (prog.source, oracle_mod.extended_plan(prog) if prog.kind == "extended" else "")
    finally:
        db.close()


@pytest.mark.parametrize("width", [60, None])
def test_dna_ranges_on_repeats(engine, oracle_mod, width):
    text = repeats_fasta(3, width=width)
    progs = []
    for p in DNA_RANGES:
        f = convert("-n", p)
        progs += [compile_pattern(f), compile_pattern(convert("-c", p))]
    progs = [p for p in progs if p.kind == "extended"]
    assert len(progs) >= 12
    assert any(oracle_mod.extended_plan(p)["L"] > 0 for p in progs)
    _check(engine, oracle_mod, text, progs, alphabet="nuc")


def test_prosite_config3_on_cys_rich_peptides(engine, oracle_mod):
    """configs[3]: C-x(2,4)-C-x(3)-[LIVMFYWC] (PatMatch CX{2,4}CX{3}[LIVMFYWC])
    on peptides full of overlapping Cys pairs (the CACAACAAAL shape)."""
    prog = compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))
    assert prog.kind == "extended"
    rng = random.Random(8)
    recs = []
    for r in range(40):
        seq = []
        while len(seq) < 400:
            x = rng.random()
            if x < 0.4:
                seq += list("C" + "".join(rng.choice("ACKS") for _ in range(rng.randint(0, 5))))
            elif x < 0.6:
                seq += list("CACAACAAAL")
            else:
                seq += [rng.choice("ACDEFGHIKLMNPQRSTVWY") for _ in range(rng.randint(1, 20))]
        recs.append(">p%d\n%s\n" % (r, "".join(seq)))
    text = "".join(recs).encode()
    _check(engine, oracle_mod, text, [prog], alphabet="byte")
    _check(engine, oracle_mod, repeats_fasta(9, alphabet="pep", width=None), [prog], alphabet="byte")


@pytest.mark.parametrize("seed", range(3))
def test_random_extended_patterns(engine, oracle_mod, seed):
    rng = random.Random(300 + seed)
    for alpha, layout in (("dna", "nuc"), ("pep", "byte")):
        progs = [random_extended(rng, alpha)[1] for _ in range(12)]
        text = b"".join(dense_text(rng, alpha, n_lines=60, width=(20, 400)) for _ in range(4))
        _check(engine, oracle_mod, text, progs, alphabet=layout)


def test_extended_over_search_regions(engine, oracle_mod):
    """A file over nrgrep's 1.6 MB buffer: the report restarts at every
    region start, including inside a 2 Mbp one-line record (blind cuts)."""
    rng = random.Random(17)
    recs = []
    for r in range(3):
        seq = "".join(rng.choice("AAT" if r == 1 else "ACGT") for _ in range(rng.randint(700_000, 2_100_000)))
        recs.append(">c%d\n%s\n" % (r, seq if r == 1 else "\n".join(seq[i:i + 60] for i in range(0, len(seq), 60))))
    text = "".join(recs).encode()
    progs = [compile_pattern(convert("-n", p)) for p in ("AN{0,3}GAATTC", "TAN{0,3}TA", "AT{1,3}A{1,2}T")]
    _check(engine, oracle_mod, text, progs, alphabet="nuc")
