"""GPU parity of what nrgrep_coords REPORTS: the report pass
(pm_hits.hip k_rep_*) and the simple engine's cross-line windows
(k_linear_others / k_linear_generic with `cross`), through the C ABI, vs
the CPU oracle's pmo_scan2 -- on texts rich in overlapping matches
(AT-repeats, homopolymer runs), multi-line records, headers that match
the pattern, and '^'/'$' anchors; both linear kernels (run-time tables,
PM_JIT=0; hipRTC-specialized, PM_JIT=1), synchronous and pipelined, and
the Glushkov kernels."""
import random

import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import engine as eng
    from patmatchdocker_amd import _lib
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


def repeat_fasta(seed, n_records=6, min_len=2000, max_len=9000, width=None):
    """FASTA with dense self-overlapping matches: AT repeats, A/T runs, TATA
    boxes, GAATTC sites, N runs and lower case; headers that contain the
    motifs themselves."""
    rng = random.Random(seed)
    pieces = [b"TATATATATATA", b"AAAAAAAAAA", b"TTTTTTT", b"TATAAAAG", b"GAATTCGAATTC", b"NNNNN",
              b"tatatata", b"CAACAACAA", b"ACACACAC"]
    out = bytearray()
    for r in range(n_records):
        out += b">rec%d TATATA GAATTC AAAA %d\n" % (r, rng.randint(0, 9))
        n = rng.randint(min_len, max_len)
        s = bytearray()
        while len(s) < n:
            s += rng.choice(pieces) if rng.random() < 0.3 else bytes(rng.choice(b"ACGT") for _ in range(rng.randint(1, 12)))
        s = s[:n]
        if width:
            for i in range(0, len(s), width):
                out += s[i:i + width] + b"\n"
        else:
            out += s + b"\n"
    return bytes(out)


DNA = ["TATA", "AAA", "TATAWAWR", "AWA", "GAATTC", "TANN", "NNT", "ACA", "RRRR", "TGCTGASTCAGCANW"]


def _pairs(res):
    beg, end = res
    return list(zip(beg.tolist(), end.tolist()))


@pytest.mark.parametrize("jit", ["0", "1"])
@pytest.mark.parametrize("width", [None, 60])
def test_linear_reported_vs_oracle(engine, oracle_mod, monkeypatch, jit, width):
    monkeypatch.setenv("PM_JIT", jit)
    text = repeat_fasta(11 if width else 12, width=width)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in DNA:
            fwd = convert("-n", pat)
            progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
            for k in (0, 1, 2):
                if k >= len(pat):
                    continue
                for report in ("nrgrep", "all"):
                    res, _ = engine.scan(db, progs, k=k, types="s", report=report)
                    for prog, r in zip(progs, res):
                        want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True, report=report)
                        assert _pairs(r) == want, (pat, prog.source, k, report, jit)
    finally:
        db.close()


@pytest.mark.parametrize("pipelined", [False, True])
def test_linear_reported_large_pipelined(engine, oracle_mod, monkeypatch, pipelined):
    """Multi-tile database through the specialized kernel, speculative sort
    + report pass driven by the device-side list length (pipelined)."""
    monkeypatch.setenv("PM_JIT", "1")
    text = repeat_fasta(13, n_records=5, min_len=150000, max_len=260000)
    progs = []
    for p in ("TATA", "AWA", "TGCTGASTCAGCANW", "GAATTC"):
        fwd = convert("-n", p)
        progs += [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for k in (0, 1):
            batch = engine.LinearBatch(progs)
            h = engine._collect(batch.launch(db, k, pipelined=pipelined))
            for i, prog in enumerate(progs):
                got = list(zip(*[a.tolist() for a in h.for_pattern(i)]))
                want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)
                assert got == want, (prog.source, k)
    finally:
        db.close()


def test_cross_line_windows_and_headers(engine, oracle_mod, monkeypatch):
    """k = 0 simple engine: '.' / negated classes take '\\n' and header
    bytes; a match starting on a header line hides an overlapping sequence
    match (then dropped itself)."""
    text = (b">hX AXA\nXAXA\nTCAA\n>TCA.q\nACCA\nAC\nC\n>x\nGAATTCA\n" * 3) + b"TCAG"
    for jit in ("0", "1"):
        monkeypatch.setenv("PM_JIT", jit)
        db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
        try:
            for pat in ("([AX].[AX])", "(TCA.)", "(.C)", "(C[^G])", "(A.)", "(..)", "(.)", "(#)", "(C.A.C)"):
                prog = compile_pattern(pat)
                for report in ("nrgrep", "all"):
                    res, _ = engine.scan(db, [prog], k=0, types="", report=report)
                    want = oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True, report=report)
                    assert _pairs(res[0]) == want, (pat, report, jit)
        finally:
            db.close()


def test_anchors_on_gpu(engine, oracle_mod):
    text = repeat_fasta(17, n_records=4, min_len=100, max_len=600, width=40)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        for pat in ("^(TA)", "(TA)$", "^(TATA)$", "^(A.)", "(.A)$", "^(TA.?A)", "(A(TA)*)$"):
            prog = compile_pattern(pat)
            for k in (0, 1):
                res, _ = engine.scan(db, [prog], k=k, types="s")
                want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)
                assert _pairs(res[0]) == want, (pat, k)
    finally:
        db.close()


def test_anchored_patterns_on_a_large_database(engine, oracle_mod):
    """'^' on a 256 Mbp database (the converter turns every '<' pattern into
    '^(...)'): the report pass handles anchored candidates in parallel (no
    serial walk over the list), dense cross-line '^' windows included, within
    a time bound, and equals the oracle over the whole text (256 records,
    a few hundred search regions)."""
    import time
    # (records, pattern, k): '^(..)' chains a report from every line start to
    # the end of its region (p == R passes '^'), the densest anchored case
    for recs, pat, k in ((256, "^(A.)", 0), (256, "^(TA.?A)", 0), (256, "^(TAT[AT]A[AT]A[AG])", 1), (4, "^(..)", 0)):
        db = engine.SequenceDatabase.synthetic(recs, 1_000_000, seed=77)
        try:
            text = db.decode(0, len(db))
            prog = compile_pattern(pat)
            t0 = time.perf_counter()
            res, _ = engine.scan(db, [prog], k=k, types="s")
            assert time.perf_counter() - t0 < 30.0, pat
            want = oracle_mod.scan_reported(text, prog, k, "s", skip_headers=True)
            assert _pairs(res[0]) == want, (pat, k)
        finally:
            db.close()


@pytest.mark.parametrize("alpha", ["nuc", "byte"])
def test_nfa_reported_vs_oracle(engine, oracle_mod, alpha):
    """Variable-length patterns and indels: candidates (leftmost start,
    shortest end) reduced by the report rule, vs pmo_scan2."""
    text = repeat_fasta(19, n_records=4, min_len=1000, max_len=5000, width=70)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alpha)
    try:
        for pat, k, t in [("(TA(TA)?A)", 0, ""), ("(A+T)", 0, ""), ("(GA...?TC)", 1, "s"), ("(TATA)", 1, "ids"),
                          ("(AAA)", 1, "id"), ("(T.?A.?T)", 2, "s"), ("(CAA|ACA)", 0, "")]:
            prog = compile_pattern(pat)
            for report in ("nrgrep", "all"):
                r = engine.scan_nfa(db, prog, k, 0, t or "s", engine.report_flags(prog, report))
                want = oracle_mod.scan_reported(text, prog, k, t or "s", skip_headers=True, report=report) \
                    if not (k == 0 and prog.linear) else None
                if want is None:
                    continue
                assert list(zip(r.beg.tolist(), r.end.tolist())) == want, (pat, k, t, report)
    finally:
        db.close()


def test_synthetic_db_headers_are_reported_like_a_file(engine, oracle_mod):
    """The synthetic database's header bytes (">r%08u") live on the device:
    a cross-line pattern over the decoded text equals the GPU."""
    db = engine.SequenceDatabase.synthetic(n_records=5, rec_len=20011, seed=3)
    try:
        text = db.decode(0, db.info()["positions"])
        for pat in ("(.R0)", "(..)", "(A.)", "(TCA.)"):
            prog = compile_pattern(pat)
            res, _ = engine.scan(db, [prog], k=0, types="")
            assert _pairs(res[0]) == oracle_mod.scan_reported(text, prog, 0, "", skip_headers=True), pat
    finally:
        db.close()


@pytest.mark.parametrize("k,mbp", [(0, 6.0), (1, 1.5)])
def test_config4_batch_of_256_patterns(engine, oracle_mod, monkeypatch, k, mbp):
    """BASELINE configs[4]'s batch (bench.batch_patterns(256): degenerate
    12-nt IUPAC motifs) in ONE query through the specialized kernel on a
    multi-tile database, every pattern's report list vs the oracle."""
    import bench
    monkeypatch.setenv("PM_JIT", "1")
    rng = random.Random(404)
    text = bytearray()
    r = 0
    while len(text) < mbp * 1e6:
        text += b">chr%d batch test\n" % r
        text += bytes(rng.choice(b"ACGT") for _ in range(rng.randint(200000, 700000))) + b"\n"
        r += 1
    text = bytes(text)
    progs = [compile_pattern(convert("-n", m)) for m in bench.batch_patterns(256)]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=k, types="s")
    finally:
        db.close()
    total = 0
    for prog, r in zip(progs, res):
        want = oracle_mod.scan_threads(text, prog, k, "s", skip_headers=True, threads=16, report="nrgrep")
        assert _pairs(r) == want, (prog.source, k)
        total += len(want)
    assert total > 1000


def test_config4_batch_at_scale_on_the_synthetic_database(engine, oracle_mod, monkeypatch):
    """configs[4]'s batch on the bench's own synthetic database (N runs,
    IUPAC letters, ~70 search regions) at 70 Mbp: the q-gram filter, the
    per-class exception pass over cross-line windows and the report rule
    restarting at every region start, every pattern vs the oracle on the
    decoded text."""
    import bench
    monkeypatch.setenv("PM_JIT", "1")
    progs = [compile_pattern(convert("-n", m)) for m in bench.batch_patterns(256)]
    db = engine.SequenceDatabase.synthetic(70, 1_000_000, seed=321)
    try:
        text = db.decode(0, len(db))
        assert len(db.regions()[0]) > 40
        res, _ = engine.scan(db, progs, k=0, types="")
    finally:
        db.close()
    total = 0
    for prog, r in list(zip(progs, res))[::4]:   # every 4th pattern: the oracle takes ~0.4 s each
        want = oracle_mod.scan_threads(text, prog, 0, "", skip_headers=True, threads=16, report="nrgrep")
        assert _pairs(r) == want, prog.source
        total += len(want)
    assert total > 10000


def _exception_rich_fasta(seed, mbp, width, headless):
    """Multi-line records with N runs, IUPAC letters and lower case: windows
    over breaks (the simple engine's cross windows) and over "other" bytes
    are the exception pass's, the rest the q-gram filter's."""
    rng = random.Random(seed)
    out = bytearray()
    r = 0
    while len(out) < mbp * 1e6:
        if r or not headless:
            out += b">chr%d q-gram batch %d\n" % (r, rng.randint(0, 99))
        n = rng.randint(50000, 400000)
        s = bytearray(rng.choice(b"ACGT") for _ in range(n))
        for _ in range(rng.randint(0, 3)):   # N runs
            a = rng.randrange(n)
            s[a:a + rng.randint(5, 300)] = b"N" * len(s[a:a + rng.randint(5, 300)])
        for _ in range(n // 20000):          # IUPAC letters
            s[rng.randrange(n)] = rng.choice(b"RYKMSWBDHV")
        a = rng.randrange(n)
        s[a:a + 500] = s[a:a + 500].lower()
        s = bytes(s[:n])
        for i in range(0, len(s), width):
            out += s[i:i + width] + b"\n"
        r += 1
    return bytes(out)


@pytest.mark.parametrize("width,headless,minlen", [(60, False, 10), (80, True, 11)])
def test_batch_filter_with_exceptions(engine, oracle_mod, monkeypatch, width, headless, minlen):
    """The q-gram batch filter (pm_batch.hip, k = 0, >= 16 patterns of 10-16
    positions) on a multi-tile database full of exceptions, patterns of
    every length 10..16 (different piece offsets o_p) + configs[4]'s motifs,
    every pattern's report list vs the oracle; and the same query with the
    filter off (PM_BATCH=0: the bit-sliced kernel in 8-pattern chunks) and
    with the unordered verify (PM_BATCH_ORDERED=0) and the ordered lists
    radix sorted instead of scattered (PM_BATCH_SCATTER=0).
    minlen 11 also runs the stride-2 probes (PM_BATCH_STRIDE=2: every other
    position, two indexed pieces per pattern)."""
    import bench
    monkeypatch.setenv("PM_JIT", "1")
    text = _exception_rich_fasta(21 + width, 3.0, width, headless)
    rng = random.Random(width)
    motifs = bench.batch_patterns(40, seed=width)
    for L in range(minlen, 17):
        for _ in range(3):
            motifs.append("".join(rng.choice("ACGT") if rng.random() < 0.75 else rng.choice("RYSWKMN")
                                  for _ in range(L)))
    motifs += [m for m in ("GAATTCGAATTC", "TATATATATA", "NNNNNNNNNNAC", "AAAAAAAAAAAAAAAA") if len(m) >= minlen]
    progs = [compile_pattern(convert("-n", m)) for m in motifs]
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        res, _ = engine.scan(db, progs, k=0, types="s")
        res_s2 = None
        if minlen >= 11:
            monkeypatch.setenv("PM_BATCH_STRIDE", "2")
            res_s2, _ = engine.scan(db, progs, k=0, types="s")
            monkeypatch.delenv("PM_BATCH_STRIDE")
        # the ordered lists sorted by a radix pass instead of the stable scatter
        monkeypatch.setenv("PM_BATCH_SCATTER", "0")
        res_radix, _ = engine.scan(db, progs, k=0, types="s")
        monkeypatch.delenv("PM_BATCH_SCATTER")
        # the unordered verify (per-(pattern, segment) bins + sort)
        monkeypatch.setenv("PM_BATCH_ORDERED", "0")
        res_unord, _ = engine.scan(db, progs, k=0, types="s")
        monkeypatch.setenv("PM_BATCH", "0")
        res_chunks, _ = engine.scan(db, progs, k=0, types="s")
    finally:
        db.close()
    total = 0
    for i, (prog, r, rc) in enumerate(zip(progs, res, res_chunks)):
        want = oracle_mod.scan_threads(text, prog, 0, "s", skip_headers=True, threads=16, report="nrgrep")
        assert _pairs(r) == want, prog.source
        assert _pairs(rc) == want, prog.source
        assert _pairs(res_unord[i]) == want, prog.source
        assert _pairs(res_radix[i]) == want, prog.source
        if res_s2 is not None:
            assert _pairs(res_s2[i]) == want, prog.source
        total += len(want)
    assert total > 1000


def test_ordered_batch_retries_and_falls_back(engine, oracle_mod, monkeypatch):
    """The ordered batch verify's two escape paths, every pattern vs the
    oracle: lists that overflow their first capacity (PM_BATCH_ORD_CAP=8:
    grown and re-run), and a batch whose candidates match more patterns
    than a lane keeps per candidate (the same motif eight times: the
    unordered verify takes over)."""
    import bench
    monkeypatch.setenv("PM_JIT", "1")
    text = _exception_rich_fasta(77, 2.0, 60, False)
    motifs = bench.batch_patterns(24, seed=5)
    db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
    try:
        monkeypatch.setenv("PM_BATCH_ORD_CAP", "8")
        progs = [compile_pattern(convert("-n", m)) for m in motifs]
        res, _ = engine.scan(db, progs, k=0, types="s")
        monkeypatch.delenv("PM_BATCH_ORD_CAP")
        dup = [compile_pattern(convert("-n", motifs[0])) for _ in range(8)] + progs[1:12]
        res_dup, _ = engine.scan(db, dup, k=0, types="s")
    finally:
        db.close()
    total = 0
    for prog, r in zip(progs, res):
        want = oracle_mod.scan_threads(text, prog, 0, "s", skip_headers=True, threads=16, report="nrgrep")
        assert _pairs(r) == want, prog.source
        total += len(want)
    assert total > 100   # ~16 lists of 8 keys: the first capacity overflows
    for prog, r in zip(dup, res_dup):
        want = oracle_mod.scan_threads(text, prog, 0, "s", skip_headers=True, threads=16, report="nrgrep")
        assert _pairs(r) == want, prog.source
