"""Host-side breakdown of one bench step (configs[2], 10 Gbp): scan call
(pm_scan_linear incl. its count sync), device copy into torch, destroy,
global-offset add.  Prints medians in microseconds."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from patmatchdocker_amd import engine, shards  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

fwd = convert("-n", "TGCTGASTCAGCANW")
batch = engine.LinearBatch([compile_pattern(fwd), compile_pattern(convert("-c", fwd))])
db = engine.SequenceDatabase.synthetic(10000, 1_000_000, seed=12345)
dev = torch.device("cuda", 0)
parts = {"scan": [], "to_tensors": [], "destroy": [], "offset": [], "total": [], "kernel": []}
for it in range(15):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = batch.launch(db, 2)
    t1 = time.perf_counter()
    keys, lens = shards.hits_to_tensors(h, dev)
    t2 = time.perf_counter()
    parts["kernel"].append(engine.kernel_ms(h) * 1e3)
    engine.destroy_hits(h)
    t3 = time.perf_counter()
    keys = shards.to_global(keys, 12345)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    if it >= 3:
        for k, v in zip(("scan", "to_tensors", "destroy", "offset", "total"), (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0)):
            parts[k].append(v * 1e6)
print({k: round(statistics.median(v), 1) for k, v in parts.items()})
db.close()
