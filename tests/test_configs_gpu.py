"""BASELINE.json configs at full size on one GPU, hits bit-exact vs the CPU
oracle (parity of the reference binary itself is unpinned):

* configs[0]/[1]: EcoRI GAATTC (exact) and the TATA box TATAWAWR (IUPAC,
  0 mismatches), both strands, vs a 12.1 Mbp genome-shaped FASTA (17
  chromosome-length records, the S. cerevisiae S288C sizes; synthetic bases
  -- the genome itself is not in the reference and there is no network);
* configs[3]: the PROSITE-style peptide pattern C-x(2,4)-C-x(3)-[LIVMFYWC]
  vs a yeast-proteome-shaped protein FASTA (6,000 ORFs, ~3 MB).
"""
import numpy as np
import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

pytestmark = pytest.mark.gpu

# S288C chromosome lengths (I..XVI, mitochondrion), bp
CHROM = [230218, 813184, 316620, 1531933, 576874, 270161, 1090940, 562643, 439888, 745751,
         666816, 1078177, 924431, 784333, 1091291, 948066, 85779]


def genome_fasta(seed=1):
    rng = np.random.default_rng(seed)
    out = bytearray()
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    for i, n in enumerate(CHROM):
        out += b">chr%d [organism=Saccharomyces cerevisiae] synthetic\n" % (i + 1)
        seq = acgt[rng.integers(0, 4, n)]
        # a few N runs and lowercase stretches, as assemblies have
        for _ in range(3):
            j = int(rng.integers(0, n - 100))
            seq[j:j + int(rng.integers(1, 60))] = ord("N")
        j = int(rng.integers(0, n - 5000))
        seq[j:j + 5000] += 32
        out += seq.tobytes() + b"\n"
    return bytes(out)


def proteome_fasta(seed=2, n=6000):
    rng = np.random.default_rng(seed)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    # yeast-like composition skew
    p = np.array([5.5, 1.3, 5.8, 6.5, 4.5, 5.0, 2.2, 6.6, 7.3, 9.6, 2.1, 6.1, 4.4, 4.0, 4.4, 9.0, 5.9, 5.6, 1.0, 3.4])
    p /= p.sum()
    out = bytearray()
    for i in range(n):
        ln = int(rng.gamma(2.2, 230)) + 30
        out += b">Y%05dW G%d SGDID:S%09d, Verified ORF\n" % (i, i, i)
        out += b"M" + aa[rng.choice(20, ln, p=p)].tobytes() + b"*\n"
    return bytes(out)


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import engine as eng
    from patmatchdocker_amd import _lib
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


@pytest.mark.parametrize("motif", ["GAATTC", "TATAWAWR"])
def test_genome_both_strands(engine, oracle_mod, motif):
    text = genome_fasta()
    assert len(text) > 12_000_000
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        fwd = convert("-n", motif)
        progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
        res, ms = engine.scan(db, progs, k=0, types="")
        for prog, (beg, end) in zip(progs, res):
            want = oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True)
            assert list(zip(beg.tolist(), end.tolist())) == want, prog.source
            assert len(want) > 1000
    finally:
        db.close()


def test_proteome_prosite(engine, oracle_mod):
    text = proteome_fasta()
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        prog = compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))
        res, ms = engine.scan(db, [prog], k=0, types="")
        beg, end = res[0]
        want = oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True)
        assert list(zip(beg.tolist(), end.tolist())) == want
        assert len(want) > 100
    finally:
        db.close()
