"""pm_merge_parts (shards.merge_parts): the serving rank's merge of the
ranks' sorted hit lists on the device, against a sort of the same keys --
parts with padding gaps between them (the gather's receive buffer), empty
parts, patterns absent from some parts, lengths moved with their keys and
lengths rebuilt from the pattern field (fixed-length patterns); and the
gather's own device path on one rank."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from patmatchdocker_amd import _lib
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return torch.device("cuda", 0)


def _parts(rng, sizes, npat, span, absent=()):
    """Sorted (pattern << 48 | position) lists, part r's positions in
    [r * span, (r + 1) * span); patterns in `absent` never occur."""
    out = []
    allowed = np.array([p for p in range(npat) if p not in absent])
    for r, n in enumerate(sizes):
        pid = rng.choice(allowed, n).astype(np.int64)
        pos = rng.integers(r * span, (r + 1) * span, n).astype(np.int64)
        out.append(np.sort((pid << 48) | pos))
    return out


def _buffer(parts, pad, dev, dtype=torch.int64, fill=-1):
    width = max([len(p) for p in parts] + [1]) + pad
    buf = torch.full((len(parts) * width,), fill, dtype=dtype, device=dev)
    for r, p in enumerate(parts):
        if len(p):
            buf[r * width:r * width + len(p)] = torch.as_tensor(p, dtype=dtype, device=dev)
    return buf, [r * width for r in range(len(parts))]


@pytest.mark.parametrize("sizes,npat,absent", [
    ([5000, 7000, 6000], 40, ()),
    ([0, 3000, 0, 4000, 1], 7, (3,)),
    ([20000] * 8, 256, (0, 255, 17)),
    ([1], 1, ()),
    ([3000, 0, 9000, 2047, 2049], 1000, (5,)),   # more patterns than the move stages in LDS
])
def test_merge_equals_a_sort_with_fixed_lengths(dev, sizes, npat, absent):
    from patmatchdocker_amd import shards
    rng = np.random.default_rng(len(sizes) * 131 + npat)
    parts = _parts(rng, sizes, npat, 10 ** 9, absent)
    buf, begs = _buffer(parts, 13, dev)
    fixed = [10 + (p % 7) for p in range(npat)]
    k, ln = shards.merge_parts(buf, None, begs, sizes, fixed)
    torch.cuda.synchronize()
    want = np.sort(np.concatenate(parts)) if sum(sizes) else np.zeros(0, np.int64)
    assert np.array_equal(k.cpu().numpy(), want)
    assert np.array_equal(ln.cpu().numpy(), np.asarray(fixed, np.int64)[want >> 48].astype(np.int32))


def test_merge_moves_lengths_with_their_keys(dev):
    from patmatchdocker_amd import shards
    rng = np.random.default_rng(9)
    sizes = [3000, 0, 5000, 2500]
    parts = _parts(rng, sizes, 12, 10 ** 8)
    buf, begs = _buffer(parts, 5, dev)
    # a key's length is a function of the key (so a moved length is checked)
    lens = [((p & 0xFFFF) % 50 + 1).astype(np.int32) for p in parts]
    lbuf, _ = _buffer(lens, 5, dev, dtype=torch.int32, fill=0)
    k, ln = shards.merge_parts(buf, lbuf, begs, sizes)
    torch.cuda.synchronize()
    want = np.sort(np.concatenate(parts))
    assert np.array_equal(k.cpu().numpy(), want)
    assert np.array_equal(ln.cpu().numpy(), ((want & 0xFFFF) % 50 + 1).astype(np.int32))


def test_torch_and_device_merges_agree(dev):
    """The CPU / gloo path (_merge) and the device path on the same parts."""
    from patmatchdocker_amd import shards
    rng = np.random.default_rng(21)
    sizes = [4000, 4500, 100]
    parts = _parts(rng, sizes, 30, 10 ** 7)
    buf, begs = _buffer(parts, 0, dev)
    fixed = [12] * 30
    k_dev, l_dev = shards.merge_parts(buf, None, begs, sizes, fixed)
    tparts = [torch.as_tensor(p) for p in parts]
    kc = torch.cat(tparts)
    k_cpu, l_cpu = shards._merge(tparts, kc, shards._fixed_lens(kc, fixed))
    assert torch.equal(k_dev.cpu(), k_cpu) and torch.equal(l_dev.cpu(), l_cpu.to(torch.int32))
