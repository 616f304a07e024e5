"""pm_linear_jit's graded tail (pm_linear.hip, scan_linear: the last output
segments' tiles go to workgroups of fewer tiles).  It engages only when a
workgroup owns >= 4 tiles, i.e. from ~2 Gbp on, so it is checked here on
synthetic databases of 2.5 Gbp (5 tiles per workgroup, tail workgroups of 1)
and 11 Gbp (21 tiles, tail workgroups of 5: a segment's 168 tiles end in a
shorter one) against the uniform partition of the same scan
(PM_JIT_GRADED=0; that partition is the one the oracle-checked tests run):
every hit key equal, both strands."""
import numpy as np
import pytest

from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

pytestmark = pytest.mark.gpu


def _keys(engine, db, progs, k):
    h = engine._collect(engine.LinearBatch(progs).launch(db, k))
    return np.stack([np.asarray(h.pattern), np.asarray(h.beg), np.asarray(h.end)])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("records,ks", [(2500, (0, 1, 2, 3)), (11000, (2,))])
def test_graded_tail_equals_the_uniform_partition(monkeypatch, records, ks):
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    monkeypatch.setenv("PM_JIT", "1")
    fwd = convert("-n", "TGCTGASTCAGCANW")
    progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    db = engine.SequenceDatabase.synthetic(records, 1_000_000, seed=77, device=0)
    try:
        for k in ks:
            monkeypatch.setenv("PM_JIT_GRADED", "1")
            graded = _keys(engine, db, progs, k)
            monkeypatch.setenv("PM_JIT_GRADED", "0")
            uniform = _keys(engine, db, progs, k)
            assert graded.shape == uniform.shape and graded.shape[1] > 0, k
            assert np.array_equal(graded, uniform), k
    finally:
        db.close()


@pytest.mark.timeout(300)
def test_graded_tail_against_the_oracle(monkeypatch):
    """The tiles the graded tail owns, checked against the CPU oracle (not
    only against the other partition): a 2.5 Gbp synthetic database, the
    text from just before the tail's first tile to the end of the file
    decoded from HBM, nrgrep's esimple report (oracle/pm_nrgrep.c) over it
    at k = 1 and k = 2, both strands, every hit key equal."""
    from oracle import oracle as oracle_mod
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd import engine
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    monkeypatch.setenv("PM_JIT", "1")
    monkeypatch.delenv("PM_JIT_GRADED", raising=False)
    fwd = convert("-n", "TGCTGASTCAGCANW")
    progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    db = engine.SequenceDatabase.synthetic(2500, 1_000_000, seed=78, device=0)
    try:
        n = db.info()["positions"]
        ts = engine.graded_tail_start(n)
        assert ts is not None and ts < n - 100_000_000, "the graded tail must engage at 2.5 Gbp"
        beg = max(0, ts - 3_000_000)
        text = db.decode(beg, n - beg)
        cut = text.find(b"\n") + 1          # start at a line start (<= ts)
        off = beg + cut
        assert off <= ts
        text = text[cut:]
        for k in (1, 2):
            h = engine._collect(engine.LinearBatch(progs).launch(db, k))
            for pid, prog in enumerate(progs):
                sel = (np.asarray(h.pattern) == pid) & (np.asarray(h.beg) >= off)
                got = list(zip((np.asarray(h.beg)[sel] - off).tolist(), (np.asarray(h.end)[sel] - off).tolist()))
                want = oracle_mod.scan_threads(text, prog, k, "s", skip_headers=True, threads=16,
                                               report="nrgrep")
                assert len(want) > 50, (k, pid, len(want))
                assert got == want, (k, pid, len(got), len(want))
    finally:
        db.close()
