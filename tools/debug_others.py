"""Debug: candidates of one pattern near a position, JIT path, lane vs wave
exception pass (PM_OTHERS_LANE), against the oracle.
usage: python tools/debug_others.py <seed> <k> <pattern> <lo> <hi>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PM_JIT"] = "1"
from oracle import oracle  # noqa: E402
from patmatchdocker_amd import _lib, engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402
from tests.fastagen import dna_fasta  # noqa: E402

seed, k, pat, lo, hi = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
text = dna_fasta(seed, n_records=4, min_len=40000, max_len=80000, width=None)
fwd = convert("-n", pat)
progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
print("text", repr(text[lo:hi]))
for lane in ("1", "0"):
    os.environ["PM_OTHERS_LANE"] = lane
    for flags in (_lib.PM_REPORT_ALL, _lib.PM_REPORT_NRGREP):
        h = engine.scan_linear(db, progs, k, flags)
        got = [(b, e) for b, e in zip(*[x.tolist() for x in h.for_pattern(0)]) if lo <= b < hi]
        print("lane" if lane == "1" else "wave", "all" if flags == 0 else "nrgrep", got)
print("oracle all", [x for x in oracle.scan_reported(text, progs[0], k, "s", skip_headers=True, report="all") if lo <= x[0] < hi])
db.close()
