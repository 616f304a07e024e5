"""GPU parity: the HIP kernels (through the C ABI) vs the CPU oracle.

Bit-exact (beg, end) equality on seeded synthetic FASTA files, per strand
pattern, for the linear (bit-sliced Hamming) and the Glushkov kernels.
"""
import numpy as np
import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from tests.fastagen import dna_fasta, pep_fasta

pytestmark = pytest.mark.gpu

DNA_PATTERNS = ["GAATTC", "TATAWAWR", "TGANTCAGNNNTGAC", "ACGTACGTACGTACGTACGTACGTACGTACGTACG",
                "NNNGCNNN", "YYYYYYYYYYYYYYYYYYYYRRRRRRRRRRRRRRRRRRRRNNNNNNNNNNNNNNNNNNNNNNNN",
                "CCAAT", "GGGCGG", "AN{2,3}TC", "GA(TC){1,2}A", "TTNNNN{0,3}AA"]
PEP_PATTERNS = ["CX{2,4}CX{3}[LIVMFYWC]", "NXS", "RGD", "C{2}", "[ST]X[RK]", "LXXLL", "KDEL>",
                "JOBZ", "W{1,3}Y", "P[^P]G"]


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import engine as eng
    from patmatchdocker_amd import _lib
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def _oracle_hits(oracle_mod, text, prog, k):
    return oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)


def _gpu_pairs(res):
    beg, end = res
    return list(zip(beg.tolist(), end.tolist()))


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("k", [0, 1, 2])
def test_dna_patterns_both_strands(engine, oracle_mod, seed, k):
    text = dna_fasta(seed, n_records=5, max_len=4000, width=(60 if seed == 3 else None))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in DNA_PATTERNS:
            fwd = convert("-n", pat)
            comp = convert("-c", fwd)
            progs = [compile_pattern(fwd), compile_pattern(comp)]
            res, _ = engine.scan(db, progs, k=k, types="s")
            for prog, r in zip(progs, res):
                want = _oracle_hits(oracle_mod, text, prog, k)
                assert _gpu_pairs(r) == want, (pat, prog.source, k)
    finally:
        db.close()


@pytest.mark.parametrize("k", [0, 1])
def test_peptide_patterns(engine, oracle_mod, k):
    text = pep_fasta(7, n_records=40)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        for pat in PEP_PATTERNS:
            prog = compile_pattern(convert("-p", pat))
            res, _ = engine.scan(db, [prog], k=k, types="s")
            assert _gpu_pairs(res[0]) == _oracle_hits(oracle_mod, text, prog, k), (pat, k)
    finally:
        db.close()


def test_dna_db_through_nfa_kernel(engine, oracle_mod):
    """Linear patterns forced through the Glushkov kernel on the 2-bit planes."""
    text = dna_fasta(11, n_records=4, max_len=5000)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in ["GAATTC", "TATAWAWR", "NNGCNN"]:
            prog = compile_pattern(convert("-n", pat))
            for k in (0, 2):
                r = engine.scan_nfa(db, prog, k)
                # a class sequence at k = 0 is nrgrep's simple engine in the
                # automaton kernels too (PM_CROSS_LINES: 'N' = '.' takes
                # '\n'); otherwise they stay inside a line
                want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)
                assert list(zip(r.beg.tolist(), r.end.tolist())) == want
    finally:
        db.close()


def test_edge_cases(engine, oracle_mod):
    cases = [b"", b">only header\n", b"GAATTC", b"gaattc\n", b">a\n\n\n>b\nGAATTCGAATTC\n",
             b"GAATT\nC\n", b"> not a header GAATTC\nGAATTC", b"\n" * 100 + b"GAATTC",
             b">x\n" + b"A" * 70000 + b"GAATTC\n"]
    prog = compile_pattern("(GAATTC)")
    for text in cases:
        for alpha in (engine.NUC, engine.BYTE):
            db = engine.SequenceDatabase.from_bytes(text, alphabet=alpha)
            try:
                for k in (0, 1):
                    res, _ = engine.scan(db, [prog], k=k, types="s")
                    assert _gpu_pairs(res[0]) == _oracle_hits(oracle_mod, text, prog, k), (text[:30], alpha, k)
            finally:
                db.close()


def test_many_patterns_batch(engine, oracle_mod):
    rng = np.random.default_rng(3)
    text = dna_fasta(21, n_records=3, max_len=20000, noise=False)
    pats = ["".join(rng.choice(list("ACGTRYN"), size=int(rng.integers(6, 20)))) for _ in range(13)]
    progs = [compile_pattern(convert("-n", p)) for p in pats]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=1, types="s")
        for prog, r in zip(progs, res):
            assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, 1), prog.source
    finally:
        db.close()


def test_synthetic_db_decode_and_scan(engine, oracle_mod):
    db = engine.SequenceDatabase.synthetic(n_records=7, rec_len=30011, seed=5)
    try:
        n = db.info()["positions"]
        text = db.decode(0, n)
        # the device holds the header bytes too (">r%08u", folded)
        assert text.count(b"\n") == 7 * 2 and text.startswith(b">R00000000\n")
        prog = compile_pattern(convert("-n", "TGANTCAG"))
        res, _ = engine.scan(db, [prog], k=1, types="s")
        assert _gpu_pairs(res[0]) == _oracle_hits(oracle_mod, text, prog, 1)
    finally:
        db.close()


@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_specialized_linear_kernel(engine, oracle_mod, monkeypatch, k):
    """The hipRTC pattern-specialized k_linear (PM_JIT=1) vs the oracle,
    including N runs, lowercase, wrapped lines and 33..64-position patterns."""
    monkeypatch.setenv("PM_JIT", "1")
    text = dna_fasta(31 + k, n_records=5, max_len=6000, width=(70 if k % 2 else None))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in ["GAATTC", "TATAWAWR", "TGCTGASTCAGCANW", "ACGTACGTACGTACGTACGTACGTACGTACGTACG",
                    "YYYYYYYYYYYYYYYYYYYYRRRRRRRRRRRRRRRRRRRRNNNNNNNNNNNNNNNNNNNNNNNN"]:
            fwd = convert("-n", pat)
            progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
            res, _ = engine.scan(db, progs, k=k, types="s")
            for prog, r in zip(progs, res):
                assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, k), (pat, prog.source, k)
    finally:
        db.close()


@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_specialized_shared_blocks(engine, oracle_mod, monkeypatch, k):
    """Patterns whose class runs agree at small offsets (shared carry-save
    blocks in the generated kernel): shifted copies, strands of palindromic
    and near-palindromic motifs, and a degenerate pair with N inside, vs the
    oracle."""
    monkeypatch.setenv("PM_JIT", "1")
    text = dna_fasta(211 + k, n_records=4, min_len=40000, max_len=80000, width=None)
    pats = ["ACGGTCATTGCAGT", "TTACGGTCATTGCA", "GGTCATTGCAGTCCAA", "ACGGTCATTGCAGT",
            "GAATTC", "TGCTGASTCAGCANW", "RGCCNNNNNGGCY", "ACGTTGCAAGGC"]
    progs = [compile_pattern(convert("-n", p)) for p in pats[:4]]
    for p in pats[4:]:
        fwd = convert("-n", p)
        progs += [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=k, types="s")
        for prog, r in zip(progs, res):
            assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, k), (prog.source, k)
    finally:
        db.close()


def test_specialized_matches_generic_on_synthetic(engine, oracle_mod, monkeypatch):
    """Both linear kernels on the bench's synthetic database (N runs, IUPAC
    letters, headers generated on the device), each vs the oracle on the
    decoded text (the bench motif, both strands, k = 2)."""
    db = engine.SequenceDatabase.synthetic(n_records=40, rec_len=100_003, seed=9)
    try:
        text = db.decode(0, db.info()["positions"])
        fwd = convert("-n", "TGCTGASTCAGCANW")
        progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
        monkeypatch.setenv("PM_JIT", "0")
        generic, _ = engine.scan(db, progs, k=2, types="s")
        monkeypatch.setenv("PM_JIT", "1")
        special, _ = engine.scan(db, progs, k=2, types="s")
        for prog, g, s_ in zip(progs, generic, special):
            want = oracle_mod.scan_threads(text, prog, 2, "s", skip_headers=True, threads=16, report="nrgrep")
            assert _gpu_pairs(g) == want, prog.source
            assert _gpu_pairs(s_) == want, prog.source
    finally:
        db.close()


@pytest.mark.parametrize("jit", ["0", "1"])
def test_multi_tile_stream_layout(engine, oracle_mod, monkeypatch, jit):
    """~450 KB over 7+ stream tiles: records crossing stream and tile
    boundaries, wrapped lines, N runs and lowercase, generic and specialized
    kernels, k = 0..3, against the oracle."""
    monkeypatch.setenv("PM_JIT", jit)
    text = dna_fasta(77, n_records=9, min_len=20000, max_len=90000, width=(None if jit == "1" else 80))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        assert len(db) > 6 * 65536
        for pat, ks in [("TGCTGASTCAGCANW", (0, 2, 3)), ("GAATTC", (0, 1)), ("TATAWAWR", (1,)),
                        ("ACGTACGTACGTACGTACGTACGTACGTACGTACG", (3,))]:
            fwd = convert("-n", pat)
            progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
            for k in ks:
                res, _ = engine.scan(db, progs, k=k, types="s")
                for prog, r in zip(progs, res):
                    assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, k), (pat, prog.source, k)
    finally:
        db.close()


def test_decode_roundtrip_multi_tile(engine):
    """pm_db_decode(0, n) reproduces the folded file, header lines included
    (their bytes live in the exception side table)."""
    text = dna_fasta(78, n_records=5, min_len=30000, max_len=60000, width=61)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        got = db.decode(0, len(text))
    finally:
        db.close()
    assert got == text.upper()


INDEL_DNA = ["GAATTC", "TATAWAWR", "TGANTCAG", "AN{2,3}TC", "GA(TC){1,2}A", "CCAATNNNNNGG",
             "ACGTACGTACGTACGTACGTACGTACGTACGTACG"]
INDEL_PEP = ["CX{2,4}CX{3}[LIVMFYWC]", "NXS", "RGDX", "LXXLL", "KDEL>", "W{1,3}YP", "P[^P]GA"]


@pytest.mark.parametrize("types", ["ids", "i", "d", "id", "is", "ds"])
@pytest.mark.parametrize("k", [1, 2, 3])
def test_indel_scan_dna(engine, oracle_mod, types, k):
    """-k <k><types> with insertions/deletions (the web default when
    mismatches > 0) through the Glushkov kernels, both strands, vs the oracle
    (pm_oracle.c's forward recurrence; parity of the binary itself unpinned)."""
    text = dna_fasta(200 + k, n_records=4, max_len=3000, width=(70 if k == 2 else None))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in INDEL_DNA:
            fwd = convert("-n", pat)
            progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
            if "d" in types and min(p.min_len for p in progs) <= k:
                continue
            res, _ = engine.scan(db, progs, k=k, types=types)
            for prog, r in zip(progs, res):
                want = oracle_mod.scan_reported(text, prog, k, types, skip_headers=True)
                assert _gpu_pairs(r) == want, (pat, prog.source, k, types)
    finally:
        db.close()


@pytest.mark.parametrize("types", ["ids", "id", "s", "d"])
@pytest.mark.parametrize("k", [1, 2])
def test_indel_scan_peptide(engine, oracle_mod, types, k):
    text = pep_fasta(300 + k, n_records=30)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        for pat in INDEL_PEP:
            prog = compile_pattern(convert("-p", pat))
            if "d" in types and prog.min_len <= k:
                continue
            res, _ = engine.scan(db, [prog], k=k, types=types)
            want = oracle_mod.scan_reported(text, prog, k, types, skip_headers=True)
            assert _gpu_pairs(res[0]) == want, (pat, k, types)
    finally:
        db.close()


def test_indel_multi_tile(engine, oracle_mod):
    """Insertions/deletions across stream and tile boundaries of the
    nucleotide layout (~330 KB, wrapped lines, N runs)."""
    text = dna_fasta(404, n_records=6, min_len=30000, max_len=80000, width=60)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        assert len(db) > 4 * 65536
        for pat, k in [("TGCTGASTCAGCANW", 2), ("GAATTC", 1), ("TATAWAWR", 1)]:
            prog = compile_pattern(convert("-n", pat))
            res, _ = engine.scan(db, [prog], k=k, types="ids")
            assert _gpu_pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, "ids", skip_headers=True), pat
    finally:
        db.close()


@pytest.mark.parametrize("k", [0, 2])
def test_specialized_batch_chunks(engine, oracle_mod, monkeypatch, k):
    """A batch of 11 patterns through the specialized kernel (chunks of 4, 4
    and 3 -> 4 + 4 + 2 + 1 launches), record expansion per chunk, vs oracle."""
    monkeypatch.setenv("PM_JIT", "1")
    rng = np.random.default_rng(17 + k)
    text = dna_fasta(91 + k, n_records=5, min_len=30000, max_len=70000, width=None)
    pats = ["".join(rng.choice(list("ACGTACGTRYSWN"), size=int(rng.integers(8, 16)))) for _ in range(11)]
    progs = [compile_pattern(convert("-n", p)) for p in pats]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=k, types="s")
        for prog, r in zip(progs, res):
            assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, k), (prog.source, k)
    finally:
        db.close()


def test_specialized_dense_hits(engine, oracle_mod, monkeypatch):
    """Patterns matching a large fraction of all windows (records overflow
    the first guess, per-pattern segment capacities grow on the retry, LDS
    sort replaced by the radix sort) next to a sparse one, vs the oracle."""
    monkeypatch.setenv("PM_JIT", "1")
    text = dna_fasta(131, n_records=4, min_len=60000, max_len=90000, width=None)
    progs = [compile_pattern(convert("-n", p)) for p in ["NNNNNANN", "TGCTGASTCAGCANW", "RRYY", "GAATTC"]]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=1, types="s")
        for prog, r in zip(progs, res):
            assert _gpu_pairs(r) == _oracle_hits(oracle_mod, text, prog, 1), prog.source
    finally:
        db.close()


UNBOUNDED_DNA = ["GA{2,}T", "A(TC){1,}G", "TATA{1,}GG", "GN{3,}CC", "C{4,}A"]   # (a trailing {m,} is dropped by simplify)
UNBOUNDED_PEP = ["CX{3,}C", "W{2,}Y", "KX{1,}DEL", "R{2,}GD", "NX{0,}S{2,}"]


@pytest.mark.parametrize("k,types", [(0, ""), (1, "s"), (1, "ids"), (2, "id")])
def test_unbounded_repeats(engine, oracle_mod, k, types):
    """{m,} repeats (nrgrep '*'): matches may run to the end of their record;
    chunk states are relaxed across chunks (k_nfa_carry) before the emitting
    reverse scan, on both layouts, multi-tile, vs the oracle."""
    text = dna_fasta(500 + k, n_records=5, min_len=20000, max_len=60000, width=(None if k else 90))
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in UNBOUNDED_DNA:
            prog = compile_pattern(convert("-n", pat))
            assert prog.max_len is None
            if "d" in types and prog.min_len <= k:
                continue
            res, _ = engine.scan(db, [prog], k=k, types=types)
            assert _gpu_pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, types or "s", skip_headers=True), (pat, k)
    finally:
        db.close()
    text = pep_fasta(600 + k, n_records=40, max_len=3000)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        for pat in UNBOUNDED_PEP:
            prog = compile_pattern(convert("-p", pat))
            if "d" in types and prog.min_len <= k:
                continue
            res, _ = engine.scan(db, [prog], k=k, types=types)
            assert _gpu_pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, types or "s", skip_headers=True), (pat, k)
    finally:
        db.close()


def _hits_pairs(h, n_pat):
    return [list(zip(*[a.tolist() for a in h.for_pattern(i)])) for i in range(n_pat)]


def test_pipelined_scans_match_synchronous(engine, oracle_mod, monkeypatch):
    """pm_scan_linear_async: three different batches launched back to back
    before any is collected, collected out of order, one destroyed
    unresolved, and a dense batch whose speculative layout overflows (the
    resolution re-runs it synchronously); every list equals the oracle's."""
    monkeypatch.setenv("PM_JIT", "1")
    text = dna_fasta(301, n_records=4, min_len=50000, max_len=90000, width=None)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    batches = []
    for pats in (["TGCTGASTCAGCANW"], ["GAATTC", "TATAWAWR"], ["NNNNNANN", "RRYY", "CCAAT"]):
        progs = []
        for p in pats:
            fwd = convert("-n", p)
            progs += [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
        batches.append((progs, engine.LinearBatch(progs)))
    try:
        for k in (1, 2):
            handles = [b.launch(db, k, pipelined=True) for _, b in batches]
            extra = batches[0][1].launch(db, k, pipelined=True)
            engine.destroy_hits(extra)   # never resolved
            for i in (2, 0, 1):
                progs = batches[i][0]
                got = _hits_pairs(engine._collect(handles[i]), len(progs))
                for prog, g in zip(progs, got):
                    assert g == _oracle_hits(oracle_mod, text, prog, k), (prog.source, k)
        # pending lists resolve before their database goes away
        handles = [b.launch(db, 2, pipelined=True) for _, b in batches]
    finally:
        db.close()
    for (progs, _), h in zip(batches, handles):
        got = _hits_pairs(engine._collect(h), len(progs))
        for prog, g in zip(progs, got):
            assert g == _oracle_hits(oracle_mod, text, prog, 2), prog.source


@pytest.mark.parametrize("pipelined", [False, True])
def test_sort_regimes_around_thresholds(engine, oracle_mod, monkeypatch, pipelined):
    """Hit bins of every size class of the collection path, vs the oracle:
    ~128 keys (rank sort), ~256 (the rank/bitonic boundary), ~512 (bitonic),
    ~2,048 (the LDS capacity boundary) and ~8,192 (radix sort) per bin, on
    a database whose bins cover ~8 stream tiles, synchronous and pipelined."""
    monkeypatch.setenv("PM_JIT", "1")
    text = dna_fasta(907, n_records=4, min_len=250000, max_len=300000, width=None)
    progs = [compile_pattern(convert("-n", p)) for p in ["ACGTAC", "ACGTAS", "ACGTA", "ACGT", "ACG"]]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for k in (0, 1):
            batch = engine.LinearBatch(progs)
            got = _hits_pairs(engine._collect(batch.launch(db, k, pipelined=pipelined)), len(progs))
            for prog, g in zip(progs, got):
                assert g == _oracle_hits(oracle_mod, text, prog, k), (prog.source, k)
    finally:
        db.close()
