"""configs[3] (C-x(2,4)-C-x(3)-[LIVMFYWC] vs the 3.5 MB proteome) at k = 0
and k = 1 ids: repeated queries for a kernel trace (rocprofv3) and the
host-side wall time per query."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402
from tests.test_configs_gpu import proteome_fasta  # noqa: E402

p = proteome_fasta()
prog = compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))
db = engine.SequenceDatabase.from_bytes(p, alphabet=engine.BYTE)
for k, types in ((0, ""), (1, "ids")):
    engine.scan(db, [prog], k=k, types=types)
    wall = []
    for _ in range(10):
        t0 = time.perf_counter()
        engine.scan(db, [prog], k=k, types=types)
        wall.append((time.perf_counter() - t0) * 1e3)
    print("k=%d query_ms %.3f" % (k, statistics.median(wall)), file=sys.stderr)
db.close()
