"""Walk cycles per cluster (PM_ES_MODE=3) on the same random FASTA text in
both layouts (nucleotide stream tiles vs plain bytes), to see what the
walk's text reads cost.  usage: walk_layouts.py [mbp] [types]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PM_ES_MODE"] = os.environ.get("PM_ES_MODE", "3")
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

mbp = int(sys.argv[1]) if len(sys.argv) > 1 else 500
types = sys.argv[2] if len(sys.argv) > 2 else "ids"
rng = np.random.default_rng(5)
rec = 1_000_000
parts = []
for r in range(mbp):
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, rec)]
    parts.append(b">r%07d\n" % r + seq.tobytes() + b"\n")
text = b"".join(parts)
fwd = convert("-n", "TGCTGASTCAGCANW")
prog = compile_pattern(fwd)
for alpha in (engine.NUC, engine.BYTE):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alpha)
    for rep in range(2):
        t0 = time.perf_counter()
        h = engine.scan_nfa(db, prog, 2, 0, types)
        dt = time.perf_counter() - t0
    ln = (h.end - h.beg).astype(np.int64)
    cyc = (ln & 0xFFFFFF) * 16
    size = ln >> 24
    w = size > 0
    print(alpha, "clusters", ln.size, "walked", int(w.sum()), "cycles median", int(np.median(cyc[w])) if w.any() else 0,
          "p90", int(np.percentile(cyc[w], 90)) if w.any() else 0, "scan s %.4f" % dt, flush=True)
    db.close()
