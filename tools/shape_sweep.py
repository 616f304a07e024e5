"""Times k_linear lane shapes (PM_LINEAR_SHAPE) on the bench workload."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

gbp = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
motif = sys.argv[2] if len(sys.argv) > 2 else "TGCTGASTCAGCANW"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
shapes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["4d", "4s", "2d", "2s", "8d", "8s"]
db = engine.SequenceDatabase.synthetic(int(gbp * 1000), 1_000_000, seed=1)
fwd = convert("-n", motif)
batch = engine.LinearBatch([compile_pattern(fwd), compile_pattern(convert("-c", fwd))])
ref = None
for shape in shapes:
    os.environ["PM_LINEAR_SHAPE"] = shape
    times, count = [], None
    for i in range(6):
        h = batch.launch(db, k)
        times.append(engine.kernel_ms(h))
        import ctypes
        from patmatchdocker_amd import _lib
        n = ctypes.c_uint64()
        _lib.load().pm_hits_count(h, ctypes.byref(n))
        count = n.value
        engine.destroy_hits(h)
    ref = ref or count
    med = statistics.median(times[1:])
    print("shape %s: %.3f ms  %.0f Gbases/s  hits %d %s" % (shape, med, gbp * 1e9 / (med * 1e-3) / 1e9, count,
                                                          "" if count == ref else "MISMATCH"), flush=True)
db.close()
