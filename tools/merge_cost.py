"""Rank 0's side of configs[4]'s hit gather at world 8, timed on one GPU.

At 8 ranks every rank holds ~30.7 M sorted hit keys (pattern << 48 | pos,
its own increasing position range) per query; rank 0 receives the other 7
lists (1.72 GB over xGMI, not measurable on one GPU) and then runs what
shards.gather_hits runs after the receive: the concatenation of the parts,
the lengths rebuilt from the pattern field (_fixed_lens) and the O(n) merge
(_merge: searchsorted, repeat_interleave, two scatters), and since round 6
the device merge pm_merge_parts (shards.merge_parts) that replaced them.  Every rank also
shifts its keys to node-wide offsets (to_global).  This script builds 8
synthetic parts with configs[4]'s shape (256 patterns, ~120 K keys per
pattern and rank), times each stage with CUDA events over several
repetitions, and checks the merged list against a sort.

usage: python tools/merge_cost.py [keys_per_rank] [ranks] [patterns]"""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from patmatchdocker_amd import shards  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out, ms = None, []
    for _ in range(reps):
        a.record()
        out = fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return out, sorted(ms)[len(ms) // 2]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30_720_231
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    npat = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    dev = torch.device("cuda", 0)
    span = 12_500_150_000   # positions per rank (12.5 Gbp + headers)
    g = torch.Generator(device=dev).manual_seed(7)
    parts = []
    for r in range(world):
        pid = torch.randint(0, npat, (n,), device=dev, generator=g)
        pos = torch.randint(0, span, (n,), device=dev, generator=g)
        keys, _ = torch.sort((pid << 48) | pos)
        parts.append(keys)
    lens_tab = [12] * npat
    res = {"keys_per_rank": n, "ranks": world, "patterns": npat,
           "bytes_received_by_rank0": (world - 1) * n * 8}
    _, res["to_global_ms"] = timed(lambda: shards.to_global(parts[0], span))
    glob = [shards.to_global(p, r * span) for r, p in enumerate(parts)]
    k, res["cat_ms"] = timed(lambda: torch.cat(glob))
    ln, res["fixed_lens_ms"] = timed(lambda: shards._fixed_lens(k, lens_tab))
    (mk, ml), res["torch_merge_ms"] = timed(lambda: shards._merge(glob, k, ln))
    res["torch_rank0_total_ms"] = round(res["cat_ms"] + res["fixed_lens_ms"] + res["torch_merge_ms"], 3)
    # the device merge (pm_merge_parts) reads the parts where the gather put
    # them (views of one receive buffer) and writes keys and fixed lengths
    width = n
    buf = torch.cat(glob)
    begs = [r * width for r in range(world)]
    (dk, dl), res["device_merge_ms"] = timed(lambda: shards.merge_parts(buf, None, begs, [n] * world, lens_tab))
    res["device_merge_equals_torch"] = bool(torch.equal(dk, mk) and torch.equal(dl, ml.to(torch.int32)))
    # device-to-device copy of the bytes rank 0 receives: the HBM side of the receive
    recv = torch.empty((world - 1) * n, dtype=torch.int64, device=dev)
    src = torch.cat(glob[1:])
    _, res["d2d_copy_of_received_bytes_ms"] = timed(lambda: recv.copy_(src))
    t0 = time.perf_counter()
    ok = bool(torch.equal(mk, torch.sort(k)[0])) and res["device_merge_equals_torch"]
    res["merge_equals_sort"] = ok
    res["check_s"] = round(time.perf_counter() - t0, 2)
    for key in list(res):
        if key.endswith("_ms"):
            res[key] = round(res[key], 3)
    print(json.dumps(res))
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
