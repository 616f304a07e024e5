"""Host cost of one pipelined configs[2] step, split: launch (the async
scan call) and collect (hits -> torch, kernel time, destroy), each timed
with the GPU idle (the previous work synchronized), medians in us."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from patmatchdocker_amd import engine, shards  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

fwd = convert("-n", bench.MOTIF)
progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
batch = engine.LinearBatch(progs)
db = engine.SequenceDatabase.synthetic(10000, 1_000_000, seed=12345)
dev = torch.device("cuda", 0)
L, C, F = [], [], []
for it in range(25):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = batch.launch(db, 2, pipelined=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    keys, lens = shards.hits_to_tensors(h, dev)
    ms = engine.kernel_ms(h)
    engine.destroy_hits(h)
    keys = shards.to_global(keys, 0)
    out = shards.gather_hits(keys, lens, fixed_len=[p.m for p in progs])
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    if it >= 5:
        L.append((t1 - t0) * 1e6)
        C.append((t3 - t2) * 1e6)
        F.append((t2 - t1) * 1e6)
print({"launch_us": round(statistics.median(L), 1), "collect_us": round(statistics.median(C), 1),
       "gpu_after_launch_us": round(statistics.median(F), 1)})
db.close()
