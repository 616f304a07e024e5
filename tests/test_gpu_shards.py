"""Real-FASTA sharding on the GPU engine: two ranks (gloo, both on cuda:0)
each hold a record-aligned piece of the file in HBM; scan_sharded and
service.search_output equal the oracle's whole-file report
(patmatch.py:733-743 scans the whole file in one process)."""
import os
import random
import sys

import pytest
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_shard_fasta import CASES, SERVICE_PATTERNS, _free_port, make_fasta  # noqa: E402

pytestmark = pytest.mark.gpu


PEPTIDE_CASES = [("CXXC", 0), ("CXXCXXXC", 1), ("[LIVM]XXG", 2), ("RGD", 1), ("NX[ST]", 0), ("CX", 0),
                 ("C[DN]XXXX[FY]XCXC", 2), ("KXL", 3)]


def make_proteome(seed, n_records):
    rng = random.Random(seed)
    recs = []
    for r in range(n_records):
        seq = "".join(rng.choice("CCKLGSTRDNV" if rng.random() < 0.3 else "ACDEFGHIKLMNPQRSTVWYX")
                      for _ in range(rng.randint(1, 1500)))
        w = rng.choice([60, 80, 2000])
        recs.append(">P%05d CKLC protein %d\n%s\n" % (r, r, "\n".join(seq[i:i + w] for i in range(0, len(seq), w))))
    return "".join(recs).encode()


def _pep_worker(rank, world, port, path, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = "0"
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from patmatchdocker_amd import shards
        from patmatchdocker_amd.convert import convert
        from patmatchdocker_amd.regex import compile_pattern
        piece = shards.ShardedDatabase.from_file(path, world, rank, device=0)
        codes = piece.db.residue_codes()[0] if piece.db is not None else -1
        res = []
        for pat, k in PEPTIDE_CASES:
            (b, e), = shards.scan_sharded(piece, [compile_pattern(convert("-p", pat))], k, "s")
            res.append(list(zip(b.tolist(), e.tolist())))
        piece.close()
        q.put((rank, codes, res))
    finally:
        dist.destroy_process_group()


def _worker(rank, world, port, path, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = "0"   # both ranks on the one GPU of the box
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from patmatchdocker_amd import service, shards
        from patmatchdocker_amd.regex import compile_pattern
        piece = shards.ShardedDatabase.from_file(path, world, rank, device=0)
        res = []
        for pat, k in CASES:
            (b, e), = shards.scan_sharded(piece, [compile_pattern(pat, ignore_case=True)], k, "s")
            res.append(list(zip(b.tolist(), e.tolist())))
        piece.close()
        outs = {opt: service.search_output(SERVICE_PATTERNS, opt, path) for opt in ("0", "1s")}
        service.DATABASES.clear()
        q.put((rank, res, outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_equal_whole_file(tmp_path):
    from oracle import oracle
    from patmatchdocker_amd.regex import compile_pattern, engine_banner
    data = make_fasta(seed=21, n_records=40)
    path = str(tmp_path / "db.fasta")
    open(path, "wb").write(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        rank, res, outs = q.get(timeout=240)
        got[rank] = (res, outs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, (pat, k) in enumerate(CASES):
        want = oracle.scan_reported(data, compile_pattern(pat, ignore_case=True), k, "s", skip_headers=True)
        assert got[0][0][i] == want and got[1][0][i] == want, (pat, k)
    for opt in ("0", "1s"):
        k = int(opt[0])
        for i, pat in enumerate(SERVICE_PATTERNS):
            prog = compile_pattern(pat, ignore_case=True)
            hits = oracle.scan_reported(data, prog, k, opt[1:] or "idst", skip_headers=True)
            want = engine_banner(prog, k) + "\n" + "".join(
                "[%d, %d]: %s\n" % (b, e, data[b:e].decode("latin-1")) for b, e in hits)
            # the hits gather to the serving rank (service.SHARD_OUTPUT_RANK = 0)
            assert got[0][1][opt][i] == want and got[1][1][opt][i] == "", (pat, opt)


@pytest.mark.timeout(300)
def test_two_ranks_peptide_planes(tmp_path):
    """A proteome split over two ranks: each piece (+ halo) gets its own
    5-bit residue planes (pm_db::p5), and the sharded report equals the
    oracle's whole-file report, cross-line windows at k = 0 included."""
    from oracle import oracle
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    data = make_proteome(seed=5, n_records=60)
    path = str(tmp_path / "prot.fasta")
    open(path, "wb").write(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pep_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        rank, codes, res = q.get(timeout=240)
        got[rank] = (codes, res)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] > 0 and got[1][0] > 0, "both pieces scan on residue planes"
    for i, (pat, k) in enumerate(PEPTIDE_CASES):
        want = oracle.scan_reported(data, compile_pattern(convert("-p", pat)), k, "s", skip_headers=True)
        assert len(want) > 0
        assert got[0][1][i] == want and got[1][1][i] == want, (pat, k)
