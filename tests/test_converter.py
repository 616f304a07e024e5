"""patmatch_to_nrgrep.pl restatement vs outputs of the Perl script itself
(tests/golden/converter.json, made by tests/golden/make_golden.py)."""
import json
import os

import pytest

from patmatchdocker_amd.convert import PatternSyntaxError, convert

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "converter.json")))


def test_golden_count():
    assert len(GOLDEN) > 1000


@pytest.mark.parametrize("case", GOLDEN, ids=lambda c: "%s:%s" % (c["mode"], c["pattern"]))
def test_converter_matches_perl(case):
    if case["output"] is None:          # the Perl script never terminates on it
        with pytest.raises(PatternSyntaxError):
            convert(case["mode"], case["pattern"])
    else:
        assert convert(case["mode"], case["pattern"]) == case["output"]


def test_known_examples():
    assert convert("-n", "GAATTC") == "(GAATTC)"
    assert convert("-n", "TATAWAWR") == "(TATA[AT]A[AT][AG])"
    assert convert("-p", "CX{2,4}CX{3}[LIVMFYWC]") == "(C...?.?C...[LIVMFYWC])"
    assert convert("-c", "(GAATTC)") == "((GAATTC))"
    assert convert("-c", "(CA.?G)") == "((C?.TG))"      # the reference's own quirk


def test_invalid_class():
    with pytest.raises(ValueError):
        convert("-x", "ACG")
