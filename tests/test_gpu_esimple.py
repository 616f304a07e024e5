"""The GPU's esimple report (pm_esimple.hip: nrgrep's candidate order and
two-phase verify replayed per cluster of candidate starts) against the
oracle's replay of the binary's own loops (oracle/pm_nrgrep.c), on texts
where candidates overlap densely: AT repeats, homopolymers, tandem copies of
the motif with edits, wrapped lines, headers, N runs and lower case.  Both
layouts (nucleotide planes, peptide bytes), the linear kernel (substitutions)
and the automaton path (indels, > 64 positions), all three of nrgrep's
scanner types."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

pytestmark = pytest.mark.gpu

IUPAC = {"R": "[AG]", "Y": "[CT]", "S": "[GC]", "W": "[AT]", "K": "[GT]", "M": "[AC]", "B": "[CGT]",
         "D": "[AGT]", "H": "[ACT]", "V": "[ACG]", "N": "."}
AMINO = "ACDEFGHIKLMNPQRSTVWY"


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine as eng
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def _pairs(r):
    return list(zip(r[0].tolist(), r[1].tolist()))


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


def dense_fasta(seed, motif, n_records=6, rec_len=20000, width=60):
    """Records mixing AT repeats, homopolymers, random DNA with N runs and
    lower case, and tandem runs of edited motif copies."""
    rng = random.Random(seed)
    out = []
    for r in range(n_records):
        parts = []
        while sum(map(len, parts)) < rec_len:
            kind = rng.random()
            if kind < 0.2:
                parts.append("AT" * rng.randint(10, 200))
            elif kind < 0.3:
                parts.append(rng.choice("ACGT") * rng.randint(10, 300))
            elif kind < 0.55:
                parts.append("".join(_mutate(rng, motif, rng.randint(0, 3), "ACGT") for _ in range(rng.randint(2, 20))))
            elif kind < 0.6:
                parts.append("N" * rng.randint(1, 80))
            else:
                seg = "".join(rng.choice("ACGT") for _ in range(rng.randint(50, 2000)))
                parts.append(seg.lower() if rng.random() < 0.2 else seg)
        seq = "".join(parts)[:rec_len]
        out.append(">rec%d %s\n" % (r, motif[:8]))
        out.append("\n".join(seq[i:i + width] for i in range(0, len(seq), width)) + "\n")
    return "".join(out).encode()


def _plain(motif):
    return "".join(c if c in "ACGT" else "A" for c in motif)


DNA_CASES = [   # (IUPAC motif, k, types)
    ("TGCTGASTCAGCANW", 2, "s"), ("TGCTGASTCAGCANW", 1, "s"), ("TGCTGASTCAGCANW", 3, "s"),
    ("TGCTGASTCAGCANW", 2, "ids"), ("TGCTGASTCAGCANW", 1, "ids"), ("TATAWAWR", 1, "s"), ("TATAWAWR", 2, "ids"),
    ("GAATTC", 1, "ids"), ("GAATTC", 2, "s"), ("ATATATAT", 2, "ids"), ("AAAAAAAAAA", 2, "s"),
    ("CAACAACAA", 2, "ids"), ("ACGTTGCAACGTTGCAACGT", 3, "ids"), ("ACGTTGCAACGTTGCAACGT", 2, "is"),
    ("TANNNNTA", 1, "ds"), ("GGATCCNNNNNGGATCC", 2, "ids"),
]


@pytest.mark.parametrize("case", range(len(DNA_CASES)))
def test_esimple_report_dense_dna(engine, oracle_mod, case):
    motif, k, types = DNA_CASES[case]
    text = dense_fasta(200 + case, _plain(motif))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        fwd = convert("-n", motif)
        progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
        res, _ = engine.scan(db, progs, k=k, types=types)
        for prog, r in zip(progs, res):
            want = oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True)
            assert _pairs(r) == want, (motif, k, types, oracle_mod.nrgrep_plan(prog, k))
    finally:
        db.close()


def test_esimple_random_patterns_all_scanner_types(engine, oracle_mod):
    """Random IUPAC patterns 4..40 positions at k 1..4 (every scanner type
    occurs), anchors included, on one dense database."""
    rng = random.Random(7)
    text = dense_fasta(300, "TGCTGACTCAGCAAA", n_records=4, rec_len=15000)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    seen = set()
    try:
        for _ in range(40):
            m = rng.randint(4, 40)
            s = "".join(rng.choice("ACGT") if rng.random() < 0.8 else rng.choice("RYSWN") for _ in range(m))
            pat = "(" + "".join(IUPAC.get(c, c) for c in s) + ")"
            a = rng.random()
            pat = ("^" + pat) if a < 0.1 else (pat + "$") if a < 0.2 else pat
            prog = compile_pattern(pat)
            k = rng.randint(1, max(1, min(4, prog.m // 3)))
            types = rng.choice(["s", "ids", "is", "ds", "i", "d"])
            if "d" in types and k >= prog.min_len:
                types = "s"
            seen.add(oracle_mod.nrgrep_plan(prog, k)["type"])
            res, _ = engine.scan(db, [prog], k=k, types=types)
            want = oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True)
            assert _pairs(res[0]) == want, (pat, k, types)
        assert len(seen) >= 2
    finally:
        db.close()


def test_esimple_long_patterns(engine, oracle_mod):
    """65..160 positions (the automaton path, several words per position set)."""
    rng = random.Random(9)
    motif = "".join(rng.choice("ACGT") for _ in range(160))
    text = dense_fasta(301, motif, n_records=3, rec_len=20000, width=80)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for m, k, types in [(70, 3, "ids"), (100, 5, "s"), (160, 7, "ids"), (65, 2, "ds")]:
            prog = compile_pattern(motif[:m])
            res, _ = engine.scan(db, [prog], k=k, types=types)
            assert _pairs(res[0]) == oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True), (m, k, types)
    finally:
        db.close()


def test_esimple_peptides(engine, oracle_mod):
    """The byte layout: peptide class sequences with k = 1..3 (types 1, 2, 3
    of nrgrep's plan), planted edited copies."""
    rng = random.Random(13)
    recs = []
    pats = ["".join(rng.choice(AMINO) for _ in range(n)) for n in (9, 14, 22, 30)]
    for r in range(40):
        seq = "".join(rng.choice(AMINO) for _ in range(rng.randint(200, 900)))
        for p in pats:
            for _ in range(rng.randint(0, 2)):
                at = rng.randrange(len(seq))
                seq = seq[:at] + _mutate(rng, p, rng.randint(0, 3), AMINO) + seq[at:]
        recs.append(">p%d\n%s\n" % (r, "\n".join(seq[i:i + 60] for i in range(0, len(seq), 60))))
    text = "".join(recs).encode()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        for p in pats:
            prog = compile_pattern(p)
            for k, types in [(1, "ids"), (2, "s"), (3, "ids")]:
                if k >= prog.m // 3 + 1 and k > 1:
                    continue
                res, _ = engine.scan(db, [prog], k=k, types=types)
                want = oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True)
                assert _pairs(res[0]) == want, (p, k, types, oracle_mod.nrgrep_plan(prog, k))
    finally:
        db.close()


def test_esimple_lone_starts_and_the_shift_quirk(engine, oracle_mod):
    """Substitution-only lone starts are reported without a walk -- except
    where a piece's test bit is wrong (bit >= 32 under the 32-bit shift,
    0x41384b): this 35-mer at k = 2 has pieces of 11 at 1, 12, 23 (end bits
    10, 21, 32; the last tested as bit 0), so a copy whose two errors sit in
    the first two pieces is never verified by nrgrep.  Copies of both kinds,
    far apart, inside lines of random DNA."""
    rng = random.Random(21)
    motif = "TCGACCTTTCGCCAGGAACTAGAGACTATTGCTGA"
    prog = compile_pattern(motif)
    plan = oracle_mod.nrgrep_plan(prog, 2)
    assert plan["type"] == 1 and plan["piece_len"] == 11 and plan["L"] == [1, 12, 23], plan

    def edit(copy, j):
        copy[j] = "ACGT"[("ACGT".index(copy[j]) + 1) % 4]

    recs = []
    for r in range(30):
        seq = [rng.choice("ACGT") for _ in range(3000)]
        for c in range(4):
            at = 70 * (3 + 10 * c) + 5   # inside one 70-column line
            copy = list(motif)
            if c % 2 == 0:
                edit(copy, 1 + rng.randrange(11))
                edit(copy, 12 + rng.randrange(11))
            else:
                edit(copy, 23 + rng.randrange(12))
            seq[at:at + len(motif)] = copy
        s = "".join(seq)
        recs.append(">c%d\n%s\n" % (r, "\n".join(s[i:i + 70] for i in range(0, len(s), 70))))
    text = "".join(recs).encode()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, [prog], k=2, types="s")
        want = oracle_mod.scan_esimple(text, prog, 2, "s", skip_headers=True)
        leftmost = oracle_mod.scan_reported(text, prog, 2, "s", skip_headers=True, report="leftmost")
        assert len(leftmost) >= 120 and len(want) <= len(leftmost) - 55   # the copies nrgrep never verifies
        assert _pairs(res[0]) == want
    finally:
        db.close()


@pytest.mark.parametrize("layout", ["nuc", "byte"])
def test_deletions_reaching_the_pattern_length(engine, oracle_mod, layout):
    """-k 3ids on a 3-residue pattern (patmatch.py:308-314 passes it through):
    every position of every line is a candidate and nrgrep prints empty
    matches too; the walk takes each line as a cluster
    (pm_esimple.hip, es_all_positions)."""
    rng = random.Random(31)
    if layout == "nuc":
        text = dense_fasta(33, "TACGATT", n_records=4, rec_len=3000, width=61)
        cases = [("ACG", 3, "ids"), ("GAT", 4, "d"), ("[AC]GT", 3, "ds"), ("AT", 2, "id")]
    else:
        recs = []
        for r in range(20):
            seq = "".join(rng.choice(AMINO) for _ in range(rng.randint(50, 400)))
            recs.append(">p%d\n%s\n" % (r, "\n".join(seq[i:i + 60] for i in range(0, len(seq), 60))))
        text = "".join(recs).encode()
        cases = [("CWK", 3, "ids"), ("LL", 2, "d"), ("[ST]P", 2, "ids")]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC if layout == "nuc" else engine.BYTE)
    try:
        for pat, k, types in cases:
            prog = compile_pattern(pat)
            res, _ = engine.scan(db, [prog], k=k, types=types)
            want = oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True)
            assert len(want) > 100
            assert _pairs(res[0]) == want, (pat, k, types)
    finally:
        db.close()
