"""Host-side timing of the pipelined bench step: how long launch (async)
and collect take on the host, per step (is the launch really async?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from patmatchdocker_amd import engine, shards  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

os.environ.setdefault("PM_JIT", "1")
dev = torch.device("cuda", 0)
db = engine.SequenceDatabase.synthetic(10000, 1_000_000, seed=1)
fwd = convert("-n", "TGCTGASTCAGCANW")
batch = engine.LinearBatch([compile_pattern(fwd), compile_pattern(convert("-c", fwd))])
pend = batch.launch(db, 2, pipelined=True)
for i in range(12):
    t0 = time.perf_counter()
    nxt = batch.launch(db, 2, pipelined=True)
    t1 = time.perf_counter()
    n = engine.ctypes.c_uint64()
    engine.check(engine._lib.load().pm_hits_count(pend, engine.ctypes.byref(n)))
    t2 = time.perf_counter()
    keys, lens = shards.hits_to_tensors(pend, dev)
    t3 = time.perf_counter()
    ms = engine.kernel_ms(pend)
    engine.destroy_hits(pend)
    t4 = time.perf_counter()
    pend = nxt
    print("step %2d launch %7.1f us  resolve %7.1f us  tensors %7.1f us  destroy %7.1f us  kernel %.3f ms" % (
        i, (t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t4 - t3) * 1e6, ms), flush=True)
engine.destroy_hits(pend)
db.close()
