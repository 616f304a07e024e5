"""bench.py's multi-rank path, rehearsed on a one-GPU box: `--gpus 2`
spawns torch.distributed.run (spawn_ranks), the two ranks share the card
(PM_BENCH_REHEARSE=1: gloo instead of RCCL), each scans its own synthetic
records, shifts its keys to node-wide offsets (to_global) and gathers them
to rank 0 (gather_hits, fixed lengths for substitutions), and rank 0 takes
the slowest rank's time (the elapsed all_reduce).  The gathered hit keys
(pattern << 48 | node-wide offset, dumped by rank 0) and lengths must equal
the two ranks' databases scanned one by one in this process, shifted by each
rank's record offset -- configs[2] (both strands, -k 2s and -k 2ids) and
configs[4]'s 256-pattern batch (the fixed_len gather)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GBP, REC_LEN = 0.02, 100_000


def _bench(extra, tmp_path):
    env = dict(os.environ, PM_BENCH_REHEARSE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dump = str(tmp_path / "gathered")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--gbp", str(GBP), "--rec-len", str(REC_LEN), "--no-cpu-baseline", "--dump-keys", dump] + extra
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]     # rank 0 alone prints
    return json.loads(lines[0]), np.load(dump + ".keys.npy"), np.load(dump + ".lens.npy")


def _local_hits(k, types, progs):
    """(keys, lens) of both ranks' databases scanned here, in node-wide
    offsets, sorted like the gathered list (pattern, then position)."""
    from patmatchdocker_amd import engine, shards
    per_rank = max(1, int(round(GBP * 1e9 / REC_LEN)))
    rec_bytes = 10 + 1 + REC_LEN + 1
    keys, lens = [], []
    for rank in range(2):
        first, count = shards.shard_range(per_rank * 2, 2, rank)
        db = engine.SequenceDatabase.synthetic(count, REC_LEN, seed=12345 + first, device=0)
        try:
            res, _ = engine.scan(db, progs, k=k, types=types)
            for pid, (b, e) in enumerate(res):
                b = np.asarray(b, dtype=np.int64)
                keys.append((np.int64(pid) << 48) | (b + first * rec_bytes))
                lens.append(np.asarray(e, dtype=np.int64) - b)
        finally:
            db.close()
    keys, lens = np.concatenate(keys), np.concatenate(lens)
    order = np.argsort(keys, kind="stable")
    return keys[order], lens[order]


def _same(line, got_k, got_l, want):
    wk, wl = want
    assert line["config"]["hits"] == len(wk) > 0
    assert np.array_equal(got_k.astype(np.int64), wk)
    assert np.array_equal(got_l.astype(np.int64), wl)


def _config2_progs():
    import bench
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    fwd = convert("-n", bench.MOTIF)
    return [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]


def test_two_rank_bench_substitutions(tmp_path):
    line, k, ln = _bench([], tmp_path)
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["ms_per_step"] > 0
    assert "x2" in line["config"]["parallelism"]
    _same(line, k, ln, _local_hits(2, "s", _config2_progs()))


def test_two_rank_bench_indels(tmp_path):
    line, k, ln = _bench(["--types", "ids"], tmp_path)
    assert line["n_gpus"] == 2 and line["value"] > 0
    _same(line, k, ln, _local_hits(2, "ids", _config2_progs()))


def test_two_rank_bench_config4_batch(tmp_path):
    """configs[4]: the 256-pattern batch at k = 0 over two ranks -- keys only
    travel (fixed_len: rank 0 rebuilds the lengths from the pattern field)."""
    import bench
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    line, k, ln = _bench(["--config", "4", "--gbp", str(GBP)], tmp_path)
    assert line["n_gpus"] == 2 and line["config"]["patterns"] == 256
    progs = [compile_pattern(convert("-n", m)) for m in bench.batch_patterns(256)]
    _same(line, k, ln, _local_hits(0, "", progs))


def test_two_rank_bench_with_the_extras(tmp_path):
    """The default run's extras at N = 2 (the driver's multi-GPU runs print
    them too): configs4 and north_star_100gbp sub-objects from both ranks'
    timed loops, whole-job values, no CPU baseline above one rank."""
    env = dict(os.environ, PM_BENCH_REHEARSE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--gbp", str(GBP), "--rec-len", str(REC_LEN), "--no-cpu-baseline", "--extras", "on",
           "--cfg4-gbp", "0.07", "--north-gbp", "0.07"]   # >= 64 Mi positions: the specialized kernels
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    for key, kern in (("configs4", "k_batch_scan"), ("north_star_100gbp", "pm_linear_jit")):
        sub = line[key]
        assert sub["value"] > 0 and sub["ms_per_step"] > 0 and sub["hits"] > 0, (key, sub)
        assert sub["roofline"]["kernel"].startswith(kern) and sub["roofline"]["kernel_ms"] > 0
        assert sub["cpu_baseline"] is None
    assert "over 2 GPUs" in line["configs4"]["workload"]
