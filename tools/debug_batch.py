"""Debug: configs[4] batch on a multi-tile DB, report=all vs nrgrep, per pattern vs the oracle."""
import os, random, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PM_JIT", "1")
import bench
from oracle import oracle
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern

rng = random.Random(404)
text = bytearray(); r = 0
while len(text) < float(sys.argv[1]) * 1e6:
    text += b">chr%d batch test\n" % r
    text += bytes(rng.choice(b"ACGT") for _ in range(rng.randint(200000, 700000))) + b"\n"
    r += 1
text = bytes(text)
n = int(sys.argv[2])
progs = [compile_pattern(convert("-n", m)) for m in bench.batch_patterns(256)][:n]
db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.NUC)
for report in ("all", "nrgrep"):
    res, _ = engine.scan(db, progs, k=0, types="s", report=report)
    bad = 0
    for i, (prog, (b, e)) in enumerate(zip(progs, res)):
        got = list(zip(b.tolist(), e.tolist()))
        want = oracle.scan_reported(text, prog, 0, "s", skip_headers=True, report=report)
        if got != want:
            bad += 1
            gs, ws = set(got), set(want)
            print(report, i, prog.source, "got", len(got), "want", len(want), "extra", sorted(gs - ws)[:6],
                  "missing", sorted(ws - gs)[:6], "sorted", got == sorted(got), "dups", len(got) - len(gs))
    print(report, "bad patterns:", bad, "of", len(progs))
db.close()
