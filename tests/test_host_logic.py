"""Host-side restatements vs the reference's own Python/Perl outputs
(tests/golden/host_logic.json and index.json)."""
import json
import os

import pytest

from patmatchdocker_amd import service

HERE = os.path.dirname(__file__)
HOST = json.load(open(os.path.join(HERE, "golden", "host_logic.json")))
INDEX = json.load(open(os.path.join(HERE, "golden", "index.json")))


@pytest.mark.parametrize("case", HOST["check_pattern"])
def test_check_pattern(case):
    assert service.check_pattern(case["pattern"], case["seqtype"]) == case["out"]


@pytest.mark.parametrize("case", HOST["cleanup_pattern"])
def test_cleanup_pattern(case):
    assert service.cleanup_pattern(case["pattern"]) == case["out"]


@pytest.mark.parametrize("case", HOST["find_exclusion_offset"])
def test_find_exclusion_offset(case):
    assert service.find_exclusion_offset(case["pattern"]) == case["out"]


def test_get_name_offset():
    for case in HOST["get_name_offset"]:
        assert service.get_name_offset(case["offset"], case["list"]) == case["out"], case


def test_process_pattern():
    for case in HOST["process_pattern"]:
        assert list(service.process_pattern(*case["args"])) == case["out"], case["args"]


def test_set_seq_length(tmp_path):
    for case in HOST["set_seq_length"]:
        f = tmp_path / "x.seq"
        f.write_bytes(case["fasta"].encode("latin-1"))
        lengths = {}
        stops = service.set_seq_length(lengths, str(f))
        assert lengths == case["lengths"] and stops == case["stops"]


@pytest.mark.parametrize("case", INDEX)
def test_record_index(case, tmp_path):
    f = tmp_path / "db.seq"
    f.write_bytes(case["fasta"].encode("latin-1"))
    offsets, names = service.get_record_offset(str(f))
    want_off, want_names = [], {}
    for line in case["index"].split("\n"):        # patmatch.py:206-213 parsing
        pieces = line.strip().split("\t")
        if len(pieces) < 2:
            continue
        want_off.append(int(pieces[0]))
        want_names[int(pieces[0])] = pieces[1]
    assert offsets == want_off and names == want_names


def test_process_output(tmp_path, monkeypatch):
    monkeypatch.setattr(service, "dataDir", str(tmp_path) + "/")
    for i, case in enumerate(HOST["process_output"]):
        datafile = tmp_path / case["fasta_name"]
        datafile.write_bytes(case["fasta"].encode("latin-1"))
        (tmp_path / "locus.txt").write_text(case["locus"])
        offsets, names = service.get_record_offset(str(datafile))
        dl = tmp_path / "dl.txt"
        res = service.process_output(offsets, names, case["output"], str(datafile), case["maxhits"],
                                     case["begMatch"], case["endMatch"], str(dl), case["pattern"])
        assert [res[0], res[1], res[2], res[3]] == case["result"], i
        assert dl.read_text() == case["file"], i
