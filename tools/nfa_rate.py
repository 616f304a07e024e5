"""Throughput of the Glushkov path on the synthetic nucleotide database:
a 15-nt motif with k = 1 insertions/deletions/substitutions (the web
default), and a bounded-gap pattern, on --gbp Gbp (default 1)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

gbp = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1_000_000, seed=7)
for pat, k, types in [("TGCTGASTCAGCANW", 1, "ids"), ("TGCTGASTCAGCANW", 2, "ids"), ("GAN{2,6}TC", 0, ""),
                      ("TGCTGASTCAGCANW", 2, "s")]:
    prog = compile_pattern(convert("-n", pat))
    engine.scan(db, [prog], k=k, types=types)
    dt = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        res, ms = engine.scan(db, [prog], k=k, types=types)
        dt = min(dt, time.perf_counter() - t0)
    print("%-20s k=%d %-3s hits %9d  kernel %8.2f ms  query %8.2f ms  %7.1f Gbases/s" % (
        pat, k, types, len(res[0][0]), ms, dt * 1e3, gbp / dt), flush=True)
db.close()
