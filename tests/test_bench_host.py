"""bench.py's host side, on CPU: the argument rules that decide whether the
extra workloads (configs4, north_star_100gbp) run, the region-aligned CPU
sample of configs[4], and the vectorized bit-exact comparison of a GPU hit
list with the CPU's matches -- fed here with a database stand-in that holds
the text on the host and a hit list built by the oracle itself."""
import random

import numpy as np
import pytest
import torch

import bench
from oracle import oracle
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern


class HostDb:
    """The three calls the CPU legs make on a SequenceDatabase."""

    def __init__(self, text, bufsize):
        self.text = text
        self.regs = engine.nrgrep_regions(text, bufsize)

    def info(self):
        return {"positions": len(self.text)}

    def decode(self, beg, length):
        return self.text[beg:beg + length]

    def regions(self):
        return self.regs


def _fasta(seed, records, rec_len):
    rng = random.Random(seed)
    out = bytearray()
    for r in range(records):
        out += b">R%08d\n" % r
        s = bytearray(rng.choice(b"ACGT") for _ in range(rec_len))
        for _ in range(3):
            at = rng.randrange(rec_len - 60)
            s[at:at + rng.randint(5, 50)] = b"N" * 5
        out += s + b"\n"
    return bytes(out)


def _gpu_like_hits(text, progs, bufsize):
    """What the engine hands the bench: sorted pattern << 48 | beg keys and
    lengths over the whole file (here from the oracle over nrgrep's regions)."""
    keys, lens = [], []
    regs = list(zip(*(a.tolist() for a in engine.nrgrep_regions(text, bufsize))))
    for pid, p in enumerate(progs):
        for b, e in oracle.by_region(text, lambda t: oracle.shiftadd_scan(t, p, 0), skip_headers=True, regs=regs):
            keys.append((pid << 48) | b)
            lens.append(e - b)
    return torch.tensor(keys, dtype=torch.int64), torch.tensor(lens, dtype=torch.int32)


def test_extras_run_only_for_the_default_workload():
    assert bench.parse_args([]).run_extras
    assert bench.parse_args(["--steps", "20", "--warmup", "5", "--gpus", "1"]).run_extras
    assert not bench.parse_args(["--gbp", "1"]).run_extras
    assert not bench.parse_args(["--config", "4"]).run_extras
    assert not bench.parse_args(["--types=ids"]).run_extras
    assert not bench.parse_args(["--extras", "off"]).run_extras
    assert bench.parse_args(["--gbp", "0.1", "--extras", "on"]).run_extras
    a = bench.parse_args(["--config", "4"])
    assert a.gbp == 12.5 and a.k == 0


def test_region_pieces_start_at_region_starts():
    text = _fasta(3, 12, 5000)
    db = HostDb(text, 7001)
    pieces = bench.region_pieces(db, 15000)
    starts, ends = (a.tolist() for a in db.regions())
    assert len(pieces) == 2
    (a0, t0, r0), (a1, t1, r1) = pieces
    assert a0 == 0 and a0 + len(t0) in ends and a1 in starts and a1 + len(t1) == len(text)
    for off, txt, regs in pieces:
        assert txt == text[off:off + len(txt)]
        assert regs[0][0] == 0 and regs[-1][1] == len(txt)
        for t, e in regs:
            assert t + off in starts and e + off in ends


@pytest.mark.parametrize("bufsize", [7001, 1600000])
def test_batch_cpu_baseline_matches_and_catches_a_difference(bufsize):
    """The configs[4] CPU leg on a sample of the file: bit-exact with a hit
    list that is right, not with one that lost a key or moved one."""
    text = _fasta(7, 16, 6000)
    db = HostDb(text, bufsize)
    progs = [compile_pattern(convert("-n", m)) for m in bench.batch_patterns(24, seed=11)]
    progs += [compile_pattern(convert("-n", "ACGN")), compile_pattern(convert("-n", "NNACG"))]
    keys, lens = _gpu_like_hits(text, progs, bufsize)
    assert keys.numel() > 50
    cb, ok, detail = bench.cpu_baseline_batch(db, progs, 20000, (keys, lens), 4)
    assert ok and detail["hits_checked"] > 0
    assert cb["kind"] == "port" and cb["cores"] == 4 and cb["value"] > 0
    # a key inside the sample dropped, or shifted by one
    sample_end = detail["pieces"][0][1]
    inside = [i for i, kk in enumerate(keys.tolist()) if (kk & ((1 << 48) - 1)) + 20 < sample_end]
    i = inside[len(inside) // 2]
    _, bad, _ = bench.cpu_baseline_batch(db, progs, 20000, (torch.cat([keys[:i], keys[i + 1:]]),
                                                            torch.cat([lens[:i], lens[i + 1:]])), 4)
    assert not bad
    moved = keys.clone()
    moved[i] += 1
    _, bad, _ = bench.cpu_baseline_batch(db, progs, 20000, (moved, lens), 4)
    assert not bad


def test_compare_sample_vectorized_against_the_scalar_rule():
    rng = np.random.default_rng(5)
    pieces = [(0, b"x" * 1000), (5000, b"y" * 800)]
    want = [[sorted({(int(b), int(b) + 12) for b in rng.integers(0, 980, 7)}) for _ in range(3)],
            [sorted({(int(b), int(b) + 12) for b in rng.integers(0, 780, 5)}) for _ in range(3)]]
    keys, lens = [], []
    for p in range(3):
        for (off, _), per in zip(pieces, want):
            for b, e in per[p]:
                keys.append((p << 48) | (b + off))
                lens.append(e - b)
    # hits outside the pieces, and one crossing a piece end, are not compared
    keys += [(1 << 48) | 3000, (2 << 48) | 995]
    lens += [12, 12]
    order = np.argsort(keys, kind="stable")
    kt = torch.tensor(np.asarray(keys)[order])
    lt = torch.tensor(np.asarray(lens)[order])
    ok, n = bench.compare_sample(pieces, want, (kt, lt), 3)
    assert ok and n == sum(len(x) for per in want for x in per)
    want[1][2] = want[1][2][1:]
    ok, _ = bench.compare_sample(pieces, want, (kt, lt), 3)
    assert not ok
