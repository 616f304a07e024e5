"""Peptide scans on the 5-bit residue planes vs the byte copy: a synthetic
proteome-shaped FASTA (60-residue lines, a header every ~400 residues,
the 20 amino acids), fixed-length PROSITE-style patterns at k = 0..2
substitutions; kernel ms of each path (HIP events around the scan kernel)
and the planes' algorithmic HBM rate (0.625 byte per residue)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from patmatchdocker_amd import _lib, engine  # noqa: E402
from patmatchdocker_amd.convert import convert  # noqa: E402
from patmatchdocker_amd.regex import compile_pattern  # noqa: E402

MB = int(os.environ.get("P5_MB", "512"))
rng = np.random.default_rng(5)
aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
n_lines = MB * 1_000_000 // 61
body = aa[rng.integers(0, 20, size=(n_lines, 61))]
body[:, 60] = ord("\n")
hdr = np.flatnonzero(rng.random(n_lines) < 0.15)
body[hdr, 0] = ord(">")
text = body.tobytes()
db = engine.SequenceDatabase.from_bytes(text, alphabet=engine.BYTE, device=0)
print("residue codes", db.residue_codes()[0], "bytes", len(text), file=sys.stderr)
out = {"bytes": len(text)}
for pat in ("CXXC", "[LIVM]XXG", "CX[DN]XXXX[FY]XCXC", "RGD"):
    progs = [compile_pattern(convert("-p", pat))]
    batch = engine.LinearBatch(progs)
    for k in (0, 1, 2):
        row = {}
        for name, extra in (("planes", 0), ("bytes", _lib.PM_SCAN_BYTES)):
            ms, hits = [], 0
            for it in range(6):
                h = engine._collect(batch.launch(db, k, flags=_lib.PM_REPORT_ALL | extra))
                if it:
                    ms.append(h.kernel_ms)
                hits = len(h.beg)
            row[name] = {"kernel_ms": round(statistics.median(ms), 4), "hits": hits}
        assert row["planes"]["hits"] == row["bytes"]["hits"]
        row["planes"]["GB_s"] = round(0.625 * len(text) / (row["planes"]["kernel_ms"] * 1e-3) / 1e9, 1)
        row["speedup"] = round(row["bytes"]["kernel_ms"] / row["planes"]["kernel_ms"], 2)
        out["%s k=%d" % (pat, k)] = row
        print(pat, k, row, file=sys.stderr)
db.close()
print(json.dumps(out))
