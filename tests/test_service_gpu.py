"""End-to-end: patmatchdocker_amd.service.run_test on the GPU vs the
reference's own run_test pipeline (Perl converter, index script and
process_output of www/FlaskApp/FlaskApp/patmatch.py) with the CPU oracle in
place of the prebuilt nrgrep_coords (fixture: tests/golden/e2e.json)."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu

E2E = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "e2e.json")))


@pytest.fixture()
def service(tmp_path, monkeypatch):
    from patmatchdocker_amd import service as svc
    for name, data in E2E["files"].items():
        (tmp_path / name).write_bytes(data.encode("latin-1"))
    (tmp_path / "locus.txt").write_text(E2E["locus"])
    monkeypatch.setattr(svc, "dataDir", str(tmp_path) + "/")
    monkeypatch.setattr(svc, "tmpDir", str(tmp_path) + "/")
    yield svc
    svc.DATABASES.clear()


@pytest.mark.parametrize("case", E2E["cases"], ids=lambda c: "%s:%s" % (c["query"][0], c["query"][1]))
def test_run_test_matches_reference_pipeline(service, tmp_path, case):
    pattern, seqtype, strand, ins, dele, sub, mm, maxhits = case["query"]
    res = service.run_test(pattern, seqtype=seqtype, strand=strand, insertion=ins, deletion=dele,
                           substitution=sub, mismatch=mm, max_hits=maxhits)
    assert list(res) == case["result"]
    dl = tmp_path / "patmatch.6688"
    if case["file"] is not None:
        assert dl.read_text() == case["file"]


def test_nrgrep_coords_cli(service, tmp_path, capsys):
    from oracle import oracle
    from patmatchdocker_amd import nrgrep_coords
    from patmatchdocker_amd.regex import compile_pattern
    path = str(tmp_path / "orf_dna.seq")
    assert nrgrep_coords.main(["-i", "-b", "1600000", "-k", "1s", "(GAA[CT]TC)", path]) == 0
    got = capsys.readouterr().out
    text = open(path, "rb").read()
    want = "ESIMPLE search\n" + "".join("[%d, %d]: %s\n" % (b, e, text[b:e].decode("latin-1"))
                   for b, e in oracle.scan_reported(text, compile_pattern("(GAA[CT]TC)"), 1, "s", skip_headers=True))
    assert got == want


def test_concurrent_requests_share_one_database(service, tmp_path):
    """Request threads (mod_wsgi runs 15) scanning the same resident
    database at once -- linear and Glushkov scans, both alphabets -- each get
    exactly the single-threaded answer (the library serializes calls per
    database; the cache never closes a database under a scan)."""
    from concurrent.futures import ThreadPoolExecutor
    queries = [(["(GAA[CT]TC)", "(GA[AG]TTC)"], "1s", "orf_dna.seq"), (["(TATA[AT]A[AT][AG])"], "0ids", "orf_dna.seq"),
               (["(C..?.?C...[LIVMFYWC])"], "0ids", "orf_pep.seq"), (["(GA...?TC)"], "1ids", "orf_dna.seq"),
               (["(RGD)"], "1s", "orf_pep.seq")]
    want = [service.search_output(p, o, str(tmp_path / f)) for p, o, f in queries]
    jobs = [queries[i % len(queries)] for i in range(40)]
    with ThreadPoolExecutor(max_workers=12) as ex:
        got = list(ex.map(lambda q: service.search_output(q[0], q[1], str(tmp_path / q[2])), jobs))
    for i, g in enumerate(got):
        assert g == want[i % len(queries)], jobs[i]


def test_replaced_file_is_rescanned_without_closing_a_busy_database(service, tmp_path):
    path = tmp_path / "orf_dna.seq"
    before = service.search_output(["(GAATTC)"], "0ids", str(path))
    with service.DATABASES.lease(str(path)) as db_old:
        path.write_bytes(path.read_bytes() + b">new rec\nGAATTCGAATTC\n")
        after = service.search_output(["(GAATTC)"], "0ids", str(path))
        assert db_old.info()["positions"] > 0   # still open under the lease
    assert after[0].count("\n") == before[0].count("\n") + 2
