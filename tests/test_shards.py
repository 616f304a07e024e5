"""Sharding and the cross-rank hit gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from patmatchdocker_amd import shards


def test_shard_range_covers_records():
    for n, w in [(10, 3), (7, 8), (1000, 8), (5, 1)]:
        got = [shards.shard_range(n, w, r) for r in range(w)]
        assert sum(c for _, c in got) == n
        assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))
        assert got[0][0] == 0


def test_to_global_keeps_pattern_field():
    keys = torch.tensor([(1 << 48) | 5, (0 << 48) | 7], dtype=torch.int64)
    out = shards.to_global(keys, 1000)
    assert (out >> 48).tolist() == [1, 0]
    assert (out & shards.POS_MASK).tolist() == [1005, 1007]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r owns positions [r*1000, r*1000+1000); two patterns, uneven counts
        g = torch.Generator().manual_seed(rank)
        n = 3 + 4 * rank
        pos = torch.randint(0, 1000, (n,), generator=g) 
        pat = torch.randint(0, 3, (n,), generator=g)
        keys = (pat << 48) | pos
        order = torch.argsort(keys)
        keys, lens = keys[order], torch.full((n,), 15, dtype=torch.int32)
        out = shards.gather_hits(shards.to_global(keys, rank * 1000), lens)
        if rank == 0:
            results.put((out[0].tolist(), out[1].tolist()))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 4])
def test_gather_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    keys, lens = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # expected: union of both ranks' keys shifted by rank*1000, globally sorted
    want = []
    for rank in range(world):
        g = torch.Generator().manual_seed(rank)
        n = 3 + 4 * rank
        pos = torch.randint(0, 1000, (n,), generator=g)
        pat = torch.randint(0, 3, (n,), generator=g)
        want += (((pat << 48) | pos) + rank * 1000).tolist()
    assert keys == sorted(want)
    assert lens == [15] * len(want)


def _gather_worker(rank, world, port, dst, fixed, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 2 + 3 * rank
        keys = torch.tensor(sorted(((p % 2) << 48) | (rank * 100 + p) for p in range(n)), dtype=torch.int64)
        lens = None if fixed else torch.full((n,), 7 + rank, dtype=torch.int32)
        out = shards.gather_hits(keys, lens, dst=dst, fixed_len=[11, 13] if fixed else None)
        results.put((rank, None if out is None else (out[0].tolist(), out[1].tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,dst,fixed", [(2, 1, False), (3, 0, True), (3, None, True)])
def test_gather_to_one_rank_and_fixed_lengths(world, dst, fixed):
    """dst = r: only rank r receives the lists (dist.gather), the others get
    None; fixed_len: the length vector is never sent, it is rebuilt from the
    pattern field."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, dst, fixed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_k, want_l = [], []
    for rank in range(world):
        for p in range(2 + 3 * rank):
            key = ((p % 2) << 48) | (rank * 100 + p)
            want_k.append(key)
            want_l.append((11, 13)[p % 2] if fixed else 7 + rank)
    order = sorted(range(len(want_k)), key=lambda i: want_k[i])
    want = ([want_k[i] for i in order], [want_l[i] for i in order])
    for r in range(world):
        if dst is None or r == dst:
            assert got[r] == want, r
        else:
            assert got[r] is None


def _agree_worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        class Failing:
            def reported(self, progs, k, types):
                if rank == 1:
                    raise OSError("cannot read piece")
                return [([], [])]

        piece = shards.ShardedDatabase(b">a\nACGT\n>b\nACGT\n", world, rank, open_db=False)
        from patmatchdocker_amd.regex import compile_pattern
        try:
            shards.scan_sharded(piece, [compile_pattern("AC")], 0, "s", scanner=Failing())
            results.put((rank, "ok"))
        except Exception as exc:   # noqa: BLE001 - the test inspects it
            results.put((rank, type(exc).__name__))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_a_failing_rank_fails_every_rank():
    """A rank whose scan raises takes part in the first collective: the
    other rank raises too instead of blocking in the next one."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == {0: "RuntimeError", 1: "OSError"}


def test_split_fasta_scans_forward_from_the_targets():
    """The streaming cut finder (the pages around n*i/world only) equals the
    cut at the first header line of the whole-file index."""
    import numpy as np
    import random
    rng = random.Random(3)
    for _ in range(1500):
        parts = []
        for r in range(rng.randint(0, 12)):
            hdr = rng.choice([">r%d" % r, "> sp", ">x", ">", ">>a"])
            parts.append(hdr + "\n" + "".join(rng.choice("ACGT>\n ") for _ in range(rng.randint(0, 40))) + "\n")
        data = "".join(parts).encode()
        if rng.random() < 0.3:
            data = rng.choice([b">", b"\n>", b">a", b"", b"\n>\n"]) + data
        if rng.random() < 0.2:
            data = data + rng.choice([b">", b"\n>", b">a", b"\n>b"])
        starts, _ = shards.header_lines(data)
        n = len(data)
        for world in (1, 2, 3, 8, 40):
            cuts = [0]
            for i in range(1, world):
                j = int(np.searchsorted(starts, (n * i) // world))
                cuts.append(max(int(starts[j]) if j < starts.size else n, cuts[-1]))
            cuts.append(n)
            assert shards.split_fasta(data, world) == [(cuts[r], cuts[r + 1]) for r in range(world)]


def test_from_file_maps_the_file(tmp_path):
    data = b"".join(b">r%d\n%s\n" % (i, b"ACGT" * (i + 5)) for i in range(50))
    path = tmp_path / "db.fa"
    path.write_bytes(data)
    pieces = [shards.ShardedDatabase.from_file(str(path), 4, r, open_db=False) for r in range(4)]
    assert all(not isinstance(p.raw, bytes) for p in pieces)        # a memory map, not a copy
    assert [(p.beg, p.end) for p in pieces] == shards.split_fasta(data, 4)
    assert b"".join(bytes(p.raw[p.beg:p.end]) for p in pieces) == data
