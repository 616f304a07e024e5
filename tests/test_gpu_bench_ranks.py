"""bench.py's multi-rank path, rehearsed on a one-GPU box: `--gpus 2`
spawns torch.distributed.run (spawn_ranks), the two ranks share the card
(PM_BENCH_REHEARSE=1: gloo instead of RCCL), each scans its own synthetic
records, shifts its keys to node-wide offsets (to_global) and gathers them
to rank 0 (gather_hits, fixed lengths for substitutions), and rank 0 takes
the slowest rank's time (the elapsed all_reduce).  The gathered hit count
must equal the two ranks' databases scanned one by one in this process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GBP, REC_LEN = 0.02, 100_000


def _bench(extra):
    env = dict(os.environ, PM_BENCH_REHEARSE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--gbp", str(GBP), "--rec-len", str(REC_LEN), "--no-cpu-baseline"] + extra
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]     # rank 0 alone prints
    return json.loads(lines[0])


def _local_hits(extra_k, types, config_progs):
    from patmatchdocker_amd import engine, shards
    per_rank = max(1, int(round(GBP * 1e9 / REC_LEN)))
    total = 0
    for rank in range(2):
        first, count = shards.shard_range(per_rank * 2, 2, rank)
        db = engine.SequenceDatabase.synthetic(count, REC_LEN, seed=12345 + first, device=0)
        try:
            res, _ = engine.scan(db, config_progs, k=extra_k, types=types)
            total += sum(int(r[0].size) for r in res)
        finally:
            db.close()
    return total


def _config2_progs():
    import bench
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    fwd = convert("-n", bench.MOTIF)
    return [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]


def test_two_rank_bench_substitutions():
    line = _bench([])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["ms_per_step"] > 0
    assert "x2" in line["config"]["parallelism"]
    assert line["config"]["hits"] == _local_hits(2, "s", _config2_progs())


def test_two_rank_bench_indels():
    line = _bench(["--types", "ids"])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["hits"] == _local_hits(2, "ids", _config2_progs())
