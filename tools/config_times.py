"""Per-query device time of BASELINE.json configs[1] (TATAWAWR both strands
vs a 12.1 Mbp genome-shaped FASTA) and configs[3] (PROSITE C-x(2,4)-C-x(3)-
[LIVMFYWC] vs a 3.5 MB proteome-shaped FASTA) on one GPU, beside the CPU
oracle's time on the same input (single thread).  Prints one JSON line."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402  (checker / CPU baseline only)
from patmatchdocker_amd import engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402
from tests.test_configs_gpu import genome_fasta, proteome_fasta  # noqa: E402


def run(text, alphabet, progs, k, types, reps=10):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alphabet)
    try:
        engine.scan(db, progs, k=k, types=types)
        ms, wall = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            res, kms = engine.scan(db, progs, k=k, types=types)
            wall.append((time.perf_counter() - t0) * 1e3)
            ms.append(kms)
    finally:
        db.close()
    t0 = time.perf_counter()
    want = [oracle.scan_reported(text, p, k, types, skip_headers=True) for p in progs]
    cpu = (time.perf_counter() - t0) * 1e3
    ok = all(list(zip(b.tolist(), e.tolist())) == w for (b, e), w in zip(res, want))
    return {"kernel_ms": round(statistics.median(ms), 4), "query_ms": round(statistics.median(wall), 3),
            "cpu_oracle_ms": round(cpu, 1), "hits": sum(len(w) for w in want), "bit_exact": ok,
            "bytes": len(text)}


out = {}
g = genome_fasta()
fwd = convert("-n", "TATAWAWR")
out["configs[1] TATAWAWR both strands k=0, 12.1 Mbp genome-shaped"] = run(
    g, engine.NUC, [compile_pattern(fwd), compile_pattern(convert("-c", fwd))], 0, "")
fwd = convert("-n", "GAATTC")
out["configs[0] GAATTC both strands k=0, 12.1 Mbp genome-shaped"] = run(
    g, engine.NUC, [compile_pattern(fwd), compile_pattern(convert("-c", fwd))], 0, "")
p = proteome_fasta()
out["configs[3] CX{2,4}CX{3}[LIVMFYWC] k=0, 3.5 MB proteome-shaped"] = run(
    p, engine.BYTE, [compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))], 0, "")
out["configs[3] same, k=1 ids"] = run(
    p, engine.BYTE, [compile_pattern(convert("-p", "CX{2,4}CX{3}[LIVMFYWC]"))], 1, "ids")
print(json.dumps(out))
