"""Cluster statistics of the candidate starts (PM_REPORT_ALL) of the bench
workload: how many clusters the esimple walk gets, and their sizes."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import _lib, engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

gbp = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
fwd = convert("-n", "TGCTGASTCAGCANW")
progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1000000, seed=12345, device=0)
h = engine.scan_linear(db, progs, 2, flags=_lib.PM_REPORT_ALL)
keys = (h.pattern.astype(np.int64) << 48) | h.beg
print("starts", keys.size)
gap = 2 * (15 + 2) + 2
d = np.diff(keys)
heads = np.concatenate([[True], d > gap])
sizes = np.diff(np.concatenate([np.nonzero(heads)[0], [keys.size]]))
print("clusters", sizes.size, "lone", int((sizes == 1).sum()), "max", int(sizes.max()),
      "hist", np.bincount(np.minimum(sizes, 20)).tolist())
big = np.argsort(sizes)[-5:]
hidx = np.nonzero(heads)[0]
for b in big:
    k0 = int(keys[hidx[b]])
    print("cluster", int(sizes[b]), "pid", k0 >> 48, "pos", k0 & ((1 << 48) - 1),
          db.decode(k0 & ((1 << 48) - 1), 60))
db.close()
