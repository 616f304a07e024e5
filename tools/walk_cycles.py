"""PM_ES_MODE=3: one hit per esimple cluster whose length field holds the
walk's cycles / 16 (low 24 bits) and the cluster size (high 8): where the
walk's time goes, cluster by cluster.  usage: walk_cycles.py s|ids [gbp]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PM_ES_MODE"] = os.environ.get("PM_ES_MODE", "3")
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

types = sys.argv[1] if len(sys.argv) > 1 else "s"
gbp = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
fwd = convert("-n", "TGCTGASTCAGCANW")
progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1000000, seed=12345, device=0)
if types == "s":
    h = engine.scan_linear(db, progs, 2)
else:
    h = engine.scan_nfa(db, progs[0], 2, 0, types)
ln = (h.end - h.beg).astype(np.int64)
cyc = (ln & 0xFFFFFF) * 16
size = ln >> 24
walked = size > 0
print("clusters", ln.size, "walked", int(walked.sum()))
if os.environ["PM_ES_MODE"] == "4":
    it, ve = ln & 4095, (ln >> 12) & 4095
    print("iterations: median", int(np.median(it[walked])), "max", int(it[walked].max()), "hist",
          np.bincount(np.minimum(it[walked], 40)).tolist())
    print("verifies: median", int(np.median(ve[walked])), "max", int(ve[walked].max()), "hist",
          np.bincount(np.minimum(ve[walked], 40)).tolist())
    sys.exit(0)
if walked.any():
    c = cyc[walked]
    print("cycles: median", int(np.median(c)), "p90", int(np.percentile(c, 90)), "p99", int(np.percentile(c, 99)),
          "max", int(c.max()), "sum", int(c.sum()))
    print("size hist", np.bincount(np.minimum(size[walked], 30)).tolist())
    order = np.argsort(cyc)[-8:]
    for o in order:
        print("cyc", int(cyc[o]), "size", int(size[o]), "pos", int(h.beg[o]), db.decode(int(h.beg[o]) - 5, 70))
db.close()
