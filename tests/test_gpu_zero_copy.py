"""Zero-copy hand-over of a hit list to torch (shards.hits_as_tensors, the
bench's collect): the tensors alias the list's device buffers and equal the
copied ones; freeing them destroys the list (the pool takes its buffers
back, so later scans run on them)."""
import gc

import pytest
import torch

from patmatchdocker_amd import engine, shards
from patmatchdocker_amd.regex import compile_pattern
from patmatchdocker_amd.convert import convert

pytestmark = pytest.mark.gpu


def _db():
    return engine.SequenceDatabase.synthetic(8, 300_000, seed=11)


@pytest.mark.parametrize("k,batch", [(0, False), (1, False), (0, True)])
def test_hits_as_tensors_equal_the_copy(k, batch):
    import bench
    dev = torch.device("cuda:0")
    motifs = bench.batch_patterns(64) if batch else ["GAATTC", "TATAWAWR", "ACGTNNAC"]
    progs = [compile_pattern(convert("-n", m)) for m in motifs]
    lb = engine.LinearBatch(progs)
    db = _db()
    try:
        for _ in range(3):   # the pool recycles the buffers of the freed lists
            h1 = lb.launch(db, k)
            try:
                want_k, want_l = shards.hits_to_tensors(h1, dev)
            finally:
                engine.destroy_hits(h1)
            h2 = lb.launch(db, k)
            keys, lens = shards.hits_as_tensors(h2, dev)
            assert keys.dtype == torch.int64 and lens.dtype == torch.int32
            assert keys.device == dev and keys.numel() == want_k.numel()
            assert torch.equal(keys, want_k) and torch.equal(lens, want_l)
            assert want_k.numel() > 0
            del keys, lens
            gc.collect()
            assert not shards._OWNERS and not shards._LIVE
    finally:
        db.close()
