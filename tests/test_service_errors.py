"""run_patmatch answers a query shape that no GPU kernel takes with an
explicit error (like check_pattern's, patmatch.py:718-720), not a 500 and
not an empty hit list; nothing touches the GPU (CPU test)."""
import pytest


class FakeArgs(dict):
    def get(self, k, d=None):
        return super().get(k, d)


class FakeRequest:
    def __init__(self, **kw):
        self.args = FakeArgs(kw)
        self.form = FakeArgs()


@pytest.fixture()
def svc(tmp_path, monkeypatch):
    from patmatchdocker_amd import engine, service
    (tmp_path / "orf_dna.seq").write_bytes(b">a\nACGTACGT\n")
    monkeypatch.setattr(service, "dataDir", str(tmp_path) + "/")
    monkeypatch.setattr(service, "tmpDir", str(tmp_path) + "/")

    def no_gpu(*a, **k):
        raise AssertionError("the database must not be opened for a refused query")
    monkeypatch.setattr(engine.SequenceDatabase, "from_file", classmethod(no_gpu))
    return service


@pytest.mark.parametrize("kw", [
    dict(pattern="A" * 300, seqtype="dna", mismatch="1"),             # 300 automaton positions
    dict(pattern="A(TC){0,1}G" + "A" * 200, seqtype="dna", mismatch="8"),   # 4 words: at most 7 errors
    dict(pattern="A" * 40, seqtype="dna", mismatch="16", substitution="s"),   # 16 errors
])
def test_refused_shapes_answer_with_an_error(svc, kw):
    out = svc.run_patmatch(FakeRequest(**kw), "t1")
    assert set(out) == {"error"}
    assert "not supported by the GPU scan" in out["error"]


def test_supported_shapes_reach_the_database(svc):
    with pytest.raises(AssertionError, match="must not be opened"):
        svc.run_patmatch(FakeRequest(pattern="ACGTAC" * 20, seqtype="dna", mismatch="5"), "t2")   # 120 pos, k=5
    with pytest.raises(AssertionError, match="must not be opened"):   # a class sequence: the esimple walk
        svc.run_patmatch(FakeRequest(pattern="ACG", seqtype="dna", mismatch="3"), "t3")
    with pytest.raises(AssertionError, match="must not be opened"):   # a range: the eextended walk
        svc.run_patmatch(FakeRequest(pattern="AN{0,1}G", seqtype="dna", mismatch="2"), "t4")
    for i, kw in enumerate([dict(mismatch="1"), dict(mismatch="2", deletion="d")]):   # a group, 66 positions, k > 0
        with pytest.raises(AssertionError, match="must not be opened"):   # (round 6: the multi-word eregular walk)
            svc.run_patmatch(FakeRequest(pattern="A(TC){0,1}G" + "A" * 62, seqtype="dna", **kw), "t5%d" % i)
