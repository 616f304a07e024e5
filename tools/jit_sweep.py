"""Times the specialized linear kernel on the bench workload under env-var
variants of the generator (PM_JIT_* knobs), e.g.
    python tools/jit_sweep.py 10 TGCTGASTCAGCANW 2 "" "PM_JIT_EMIT=0" "PM_JIT_WAVES=3"
Each variant is a comma-separated list of NAME=VALUE.  PM_SWEEP_GAP_MS=<ms>
idles between launches so that every variant is timed at the recovered
clock (back-to-back launches settle ~15 % slower: power limit)."""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import _lib, engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

gbp = float(sys.argv[1])
motif = sys.argv[2]
k = int(sys.argv[3])
variants = sys.argv[4:] or [""]
os.environ["PM_JIT"] = "1"
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1_000_000, seed=1)
fwd = convert("-n", motif)
batch = engine.LinearBatch([compile_pattern(fwd), compile_pattern(convert("-c", fwd))])
for var in variants:
    env = dict(kv.split("=", 1) for kv in var.split(",") if kv)
    saved = {kk: os.environ.get(kk) for kk in env}
    os.environ.update(env)
    times, count = [], None
    gap = float(os.environ.get("PM_SWEEP_GAP_MS", "0")) * 1e-3   # idle between launches (clock recovery)
    time.sleep(10 * gap)
    for i in range(6):
        time.sleep(gap)
        h = batch.launch(db, k)
        times.append(engine.kernel_ms(h))
        n = ctypes.c_uint64()
        _lib.load().pm_hits_count(h, ctypes.byref(n))
        count = n.value
        engine.destroy_hits(h)
    for kk, v in saved.items():
        if v is None:
            os.environ.pop(kk, None)
        else:
            os.environ[kk] = v
    med = statistics.median(times[1:])
    print("%-40s %.3f ms  %6.0f Gbases/s  %6.0f GB/s alg  hits %d" % (
        var or "(default)", med, gbp * 1e9 / (med * 1e-3) / 1e9, gbp * 1e9 * 0.2539 / (med * 1e-3) / 1e9, count),
        flush=True)
db.close()
