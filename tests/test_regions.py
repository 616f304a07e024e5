"""nrgrep's search regions (``-b 1600000``: buffers of 1,600,000 bytes, each
searched up to its last '\\n', the next one loaded from that '\\n'): the
library's restatement (engine.nrgrep_regions, the one pm_db_create* apply in
C++) against the oracle's, on the edge cases recSearchFile's loop has --
no '\\n' in a buffer, a '\\n' only at its start, a file that fills its last
buffer exactly, an empty file."""
import random

import pytest

from patmatchdocker_amd import engine


@pytest.fixture(scope="module")
def oracle_regions():
    from oracle import oracle
    return oracle.regions


def _ours(text, b):
    t, e = engine.nrgrep_regions(text, b)
    return list(zip(t.tolist(), e.tolist()))


CASES = [
    (b"", 8),
    (b"ACGT", 8),
    (b"ACGTACGT", 8),              # fills its only buffer: cut at its last '\n' (none) -> whole buffer
    (b"ACG\nACGT", 8),             # exactly one buffer, '\n' inside
    (b"\nACGTACGTACGTACGT", 8),    # '\n' only at a buffer start
    (b"AC\nGT\nACGTACGTACG\nT\n", 4),
    (b"ACGTACGTACGTACGTACGTACGT", 8),   # no '\n' at all: fixed cuts
    (b">h\nACGT\nAC\n" * 5, 7),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_region_edge_cases(oracle_regions, case):
    text, b = CASES[case]
    assert _ours(text, b) == oracle_regions(text, b)


def test_regions_random(oracle_regions):
    rng = random.Random(7)
    for trial in range(300):
        n = rng.randint(0, 400)
        p_nl = rng.choice([0.0, 0.01, 0.05, 0.3])
        text = bytes(10 if rng.random() < p_nl else rng.choice(b"ACGT") for _ in range(n))
        b = rng.randint(1, 60)
        got = _ours(text, b)
        assert got == oracle_regions(text, b), (text, b)
        # the regions tile the file, overlapping by the '\n' a region ends with
        assert got[0][0] == 0 and got[-1][1] == n
        for (a0, e0), (a1, e1) in zip(got, got[1:]):
            assert a1 in (e0 - 1, e0) and (a1 == e0 or text[a1] == 10)


def test_default_buffer_is_the_reference_flag():
    """-b 1600000 in patmatch.py:733-743, taken as bytes by the binary."""
    from patmatchdocker_amd import _lib
    assert _lib.PM_NRGREP_BUFFER == 1600000
    text = (b">chr\n" + b"ACGT" * 500000 + b"\n") * 2
    t, e = engine.nrgrep_regions(text)
    # a 2 Mbp line: the buffer after a header holds no '\n' but at its start
    # and is cut blind; the buffer over the record end ends at the next header
    assert t.tolist() == [0, 4, 1600004, 2000010, 3600010]
    assert e.tolist() == [5, 1600004, 2000011, 3600010, 4000012]
