"""Time the esimple report pass on the bench workload (configs[2]) with
PM_ES_MODE experiments; run under rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

types = sys.argv[1] if len(sys.argv) > 1 else "s"
gbp = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
fwd = convert("-n", "TGCTGASTCAGCANW")
progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1000000, seed=12345, device=0)
for it in range(4):
    if types == "s":
        h = engine.LinearBatch(progs).launch(db, 2)
        print(it, flush=True)
        engine.destroy_hits(h)
    else:
        for pid, prog in enumerate(progs):
            h = engine.nfa_launch(db, prog, 2, pid, types)
            engine.destroy_hits(h)
        print(it, flush=True)
db.close()
