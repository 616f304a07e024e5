"""nrgrep's search regions on the GPU (pm_db regions; DESIGN.md §1
"Regions"): ``nrgrep_coords -b 1600000`` searches the file buffer by buffer,
so no match spans a region end, the report rule restarts at each region
start and '^' passes there.  The GPU against the oracle, which searches
region by region (oracle.by_region), with small buffers so that every text
holds many regions: the simple engine's windows over a line break (k = 0,
classes taking '\\n'), '^' anchors, the esimple engine on one-line records
cut blind (no '\\n' in a buffer), the automaton path and the peptide layout.
Patterns that match a lone '\\n' (printed twice by the binary where two
regions share it) are not used: see DESIGN.md §1."""
import pytest

from fastagen import dna_fasta, pep_fasta
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

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


def _with_regions(engine, db, text, bufsize):
    t, e = engine.nrgrep_regions(text, bufsize)
    db.set_regions(t, e)
    got_t, got_e = db.regions()
    assert got_t.tolist() == t.tolist() and got_e.tolist() == e.tolist()
    return len(t)


def test_default_regions_match_the_oracle(engine, oracle_mod):
    """pm_db_create's regions (C++, PM_NRGREP_BUFFER) = the oracle's, for a
    wrapped file and a one-line-record file over several buffers; the
    synthetic database's from its layout."""
    for text in (dna_fasta(11, n_records=40, min_len=90000, max_len=120000, width=60),
                 dna_fasta(12, n_records=3, min_len=1_700_000, max_len=2_100_000, width=None)):
        db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
        try:
            t, e = db.regions()
            assert list(zip(t.tolist(), e.tolist())) == oracle_mod.regions(text)
            assert len(t) > 1
        finally:
            db.close()
    db = engine.SequenceDatabase.synthetic(5, 1_000_000, seed=3)
    try:
        text = db.decode(0, len(db))
        t, e = db.regions()
        assert list(zip(t.tolist(), e.tolist())) == oracle_mod.regions(text)
    finally:
        db.close()


@pytest.mark.parametrize("jit", ["0", "1"])
def test_simple_engine_windows_at_region_ends(engine, oracle_mod, monkeypatch, jit):
    """k = 0 class sequences whose classes take '\\n' (IUPAC N -> '.'): the
    simple engine's windows span line breaks but not a region end; '^'
    passes at a region start.  Both linear kernels."""
    monkeypatch.setenv("PM_JIT", jit)
    text = dna_fasta(21, n_records=8, min_len=3000, max_len=9000, width=50)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for bufsize in (997, 4096):
            assert _with_regions(engine, db, text, bufsize) > 4
            for pat in ["ANNNNNNNNNNNNNNT", "GNNNC", "<ACNNNNNNNN", "TNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNA"]:
                prog = compile_pattern(convert("-n", pat))
                res, _ = engine.scan(db, [prog], k=0)
                want = oracle_mod.scan_reported(text, prog, 0, skip_headers=True, bufsize=bufsize)
                assert _pairs(res[0]) == want, (pat, bufsize)
    finally:
        db.close()


@pytest.mark.parametrize("types", ["s", "ids"])
def test_esimple_on_blind_cuts(engine, oracle_mod, types):
    """One-line records longer than a buffer: regions cut them blind, so
    the esimple engine's matches must lie inside a region, its search
    restarts at the cut, and its window / piece limits use the region end."""
    text = dna_fasta(31, n_records=3, min_len=20000, max_len=30000, width=None)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        assert _with_regions(engine, db, text, 1500) > 10
        for motif, k in [("TGCTGASTCAGCANW", 2), ("TATAWAWR", 1), ("GAATTC", 1), ("ACGTAC", 2)]:
            prog = compile_pattern(convert("-n", motif))
            res, _ = engine.scan(db, [prog], k=k, types=types)
            want = oracle_mod.scan_esimple(text, prog, k, types, skip_headers=True, bufsize=1500)
            assert _pairs(res[0]) == want, (motif, k, types, oracle_mod.nrgrep_plan(prog, k))
    finally:
        db.close()


def test_automaton_and_peptides_in_regions(engine, oracle_mod):
    """The automaton path (ranges, k = 1 ids) on DNA and the peptide layout
    (PROSITE C-x(2,4)-C-x(3)-[LIVMFYWC]) over many regions."""
    text = dna_fasta(41, n_records=6, min_len=4000, max_len=8000, width=None)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        _with_regions(engine, db, text, 2000)
        for pat, k, types in [("GA{2,4}TC", 0, ""), ("ACG{1,3}TNNA", 1, "ids"), ("<TATAWAWR", 0, "")]:
            prog = compile_pattern(convert("-n", pat))
            res, _ = engine.scan(db, [prog], k=k, types=types)
            assert _pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, types or "ids", skip_headers=True,
                                                              bufsize=2000), pat
    finally:
        db.close()
    text = pep_fasta(42, n_records=60, max_len=900)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE)
    try:
        _with_regions(engine, db, text, 3000)
        for pat, k in [("C-x(2,4)-C-x(3)-[LIVMFYWC]", 0), ("C-x(2,4)-C-x(3)-[LIVMFYWC]", 1), ("KKR", 1)]:
            prog = compile_pattern(convert("-p", pat))
            res, _ = engine.scan(db, [prog], k=k, types="ids")
            assert _pairs(res[0]) == oracle_mod.scan_reported(text, prog, k, "ids", skip_headers=True,
                                                              bufsize=3000), (pat, k)
    finally:
        db.close()
