#!/usr/bin/env python3
"""PatMatch scan benchmark (driver contract: one JSON line on rank 0).

Workload (BASELINE.json configs[2]): a 15-nt degenerate DNA motif with k = 2
mismatches, both strands (the reference's default "Both strands" search =
pattern + reverse complement, two nrgrep_coords runs in patmatch.py:733-743)
against 10 Gbp of synthetic random DNA per GPU laid out like a FASTA file
(1 Mbp records with header lines).  A step = one query: both strands scanned
in one pass of the bit-sliced Hamming kernel over the HBM-resident database,
hits compacted + sorted on the device, copied into framework tensors and,
for N > 1, gathered to rank 0 over RCCL and merged.  Weak scaling: every GPU
owns its own 10 Gbp shard (records of one node-wide virtual FASTA).

Reported beside the throughput:
  roofline      k_linear's algorithmic bytes (2-bit planes + superblock flag
                words) / its HIP-event duration vs the 8 TB/s HBM peak;
                traffic = PMC HBM bytes per launch from profiles/ when a
                counter run of this workload is committed there, else null;
  cpu_baseline  nrgrep's own esimple engine restated from the binary
                (oracle/pm_nrgrep.c: its piece BNDM scan, two-phase verify
                and report rule), one thread per host core of the box's CPU
                share (at most 16), timed on a bounded sample of the same
                database (decoded from HBM); its matches are a bit-exact
                parity spot check of the GPU's.

`--gpus N` without torchrun: the bench starts `torch.distributed.run` with
N local ranks itself (a child process, before any GPU call) and exits with
its code; under torchrun, N must equal WORLD_SIZE.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MOTIF = "TGCTGASTCAGCANW"          # 15 nt, degenerate (S, N, W)
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md: 8.0 TB/s spec
ROUND = "r05"   # committed PMC traffic run (profiles/r05_traffic.json)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gbp", type=float, default=10.0, help="Gbp of synthetic DNA per GPU")
    ap.add_argument("--rec-len", type=int, default=1_000_000)
    ap.add_argument("--motif", default=MOTIF)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--types", default="s",
                    help="error types of '-k <k><types>': s = mismatches (default, the metric's workload); "
                         "ids = the web form's default (insertions, deletions, substitutions)")
    ap.add_argument("--sample-mbp", type=float, default=None,
                    help="CPU-baseline sample (Mbp; default 100 per CPU thread)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU-baseline threads (default: the box's CPU share, at most 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial", action="store_true",
                    help="collect each query before launching the next (default: query i+1 is launched "
                         "before query i is collected, as a server pipelines queries)")
    ap.add_argument("--config", type=int, default=2, choices=(2, 4),
                    help="BASELINE.json configs[i]: 2 = one motif both strands k=2 (default, the metric's "
                         "workload); 4 = batch of 256 degenerate patterns, 12.5 Gbp per GPU (100 Gbp on 8)")
    ap.add_argument("--batch", type=int, default=256, help="patterns in the config-5 batch")
    ap.add_argument("--dump-keys", default=None,
                    help="tests: rank 0 saves the last step's gathered hit keys and lengths (<path>.keys.npy, "
                         "<path>.lens.npy)")
    args = ap.parse_args()
    if args.config == 4 and "--gbp" not in sys.argv:
        args.gbp = 12.5
    if args.config == 4 and "--k" not in sys.argv:
        args.k = 0
    return args


def batch_patterns(n, seed=5):
    """configs[4]'s batch: n random degenerate 12-nt IUPAC motifs (70 % ACGT,
    20 % two-base codes, 10 % N), forward strand; seeded, so every rank and
    run scans the same batch."""
    import random
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        m = "".join(rng.choice("ACGT") if r < 0.7 else (rng.choice("RYSWKM") if r < 0.9 else "N")
                    for r in (rng.random() for _ in range(12)))
        out.append(m)
    return out


def load_traffic(workload):
    path = os.path.join(ROOT, "profiles", "%s_traffic.json" % ROUND)
    try:
        with open(path) as fh:
            data = json.load(fh)
        if data.get("workload") == workload:
            return data.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def load_issue(kernel_key):
    """VALU-issue occupancy of a kernel from the committed PMC run
    (profiles/<ROUND>_pmc.json): SQ_INSTS_VALU wave-instructions x 4 cycles
    over the 1024 SIMDs, divided by the dispatch's cycles at its measured
    clock (MI355X_MICROARCH.md) -- how close an integer kernel that does not
    saturate HBM sits to its own (VALU) bound."""
    path = os.path.join(ROOT, "profiles", "%s_pmc.json" % ROUND)
    try:
        with open(path) as fh:
            data = json.load(fh)
    except (OSError, ValueError):
        return None
    for name, c in data.items():
        if name.startswith(kernel_key) and isinstance(c, dict):
            try:
                busy = c["SQ_INSTS_VALU"] * 4 / 1024 / (c["effective_clock_ghz"] * 1e9) / (c["median_dispatch_ms"] * 1e-3)
            except (KeyError, TypeError, ZeroDivisionError):
                return None
            return {"valu_issue_frac": round(busy, 3), "dispatch_ms": round(c["median_dispatch_ms"], 4),
                    "source": "profiles/%s_pmc.json (rocprofv3 --pmc, median dispatch)" % ROUND}
    return None


def cpu_threads_default():
    """The box's CPU share: OMP_NUM_THREADS (16 on the GPU box), else the
    affinity mask, capped at 16."""
    n = os.environ.get("OMP_NUM_THREADS")
    n = int(n) if n and n.isdigit() else len(os.sched_getaffinity(0))
    return max(1, min(16, n))


def sample_pieces(db, sample_bp):
    """The CPU sample: the database's first `sample_bp` positions and its
    last `sample_bp` (which hold pm_linear_jit's graded-tail tiles, the
    default partition's last output segments), each decoded from HBM and
    cut to whole lines (the tail piece starts after its first '\\n', so at a
    line start, as the e* engines' records do).  Returns [(offset, text)]."""
    n = db.info()["positions"]
    head = db.decode(0, int(min(sample_bp, n)))
    head = head[:head.rfind(b"\n") + 1]
    pieces = [(0, head)]
    tb = max(len(head), n - int(sample_bp))
    if tb < n:
        tail = db.decode(tb, n - tb)
        cut = tail.find(b"\n") + 1
        if cut > 0 and cut < len(tail):
            pieces.append((tb + cut, tail[cut:]))
    return pieces


def cpu_baseline(db, progs, k, types, sample_bp, gpu_hits, threads):
    """CPU baseline + parity spot check on the first and the last
    `sample_bp` positions (decoded from HBM, so the exact bytes the GPU
    scanned; the last ones are the graded tail's tiles): what nrgrep_coords
    prints for every strand, by nrgrep's own esimple engine restated from
    the binary (oracle/pm_nrgrep.c -- its cost-model plan, piece BNDM scan,
    two-phase verify and report rule) over `threads` host threads (the text
    cut at line breaks: e* matches never span one), timed; its matches must
    equal the GPU's in both pieces.  Returns (dict, parity_ok, detail)."""
    from oracle import oracle
    from patmatchdocker_amd import engine
    pieces = sample_pieces(db, sample_bp)
    t0, c0 = time.perf_counter(), time.process_time()
    base = [[oracle.scan_threads(text, p, k, types, skip_headers=True, threads=threads, report="nrgrep")
             for p in progs] for _, text in pieces]
    dt = time.perf_counter() - t0
    cpu_s = time.process_time() - c0
    bases = sum(sum(len(line) for line in text.split(b"\n")) - text.count(b">") for _, text in pieces)
    mask = (1 << 48) - 1
    keys, lens = gpu_hits
    keys = keys.cpu().tolist()
    lens = lens.cpu().tolist()
    ok = True
    checked = 0
    for (off, text), want in zip(pieces, base):
        for pid, b in enumerate(want):
            got = [((kk & mask) - off, (kk & mask) - off + ln) for kk, ln in zip(keys, lens)
                   if (kk >> 48) == pid and (kk & mask) >= off and (kk & mask) + ln <= off + len(text)]
            ok &= got == b
            checked += len(b)
    tail_start = engine.graded_tail_start(db.info()["positions"])
    detail = {"pieces": [[off, off + len(text)] for off, text in pieces], "hits_checked": checked,
              "graded_tail_start": tail_start,
              "graded_tail_checked": tail_start is not None and len(pieces) > 1 and pieces[-1][0] <= tail_start}
    plan = oracle.nrgrep_plan(progs[0], k)
    return {"value": bases / dt / 1e9, "unit": "Gbases/s", "cores": threads, "kind": "port",
            "sample": "first and last %.0f Mbp of the synthetic database (decoded from HBM; the last ones hold "
                      "the graded tail's tiles), both strands, -k %d%s: "
                      "nrgrep's esimple engine restated from the binary (oracle/pm_nrgrep.c; plan type %d, "
                      "%s) on %d host threads, text cut at line breaks; %.1f s wall, %.1f s CPU, "
                      "%d CPUs in the affinity mask"
                      % (sample_bp / 1e6, k, types, plan["type"],
                         "%d pieces of %d found by BNDM" % (len(plan["L"]), plan["piece_len"])
                         if plan["type"] == 1 else "window %s" % (plan["window"],),
                         threads, dt, cpu_s, len(os.sched_getaffinity(0)))}, ok, detail


def spawn_ranks(args):
    """`--gpus N` outside torchrun: run this script under
    torch.distributed.run with N local ranks (a child process, started
    before this process touches a GPU) and return its exit code."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, os.environ.get("WORLD_SIZE")))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # PM_BENCH_REHEARSE=1: rehearse N ranks on fewer GPUs (ranks share cards
    # round-robin, gather over gloo) -- for checking the multi-rank path on a
    # 1-GPU box; the driver's N-GPU runs use one GPU per rank over RCCL
    rehearse = os.environ.get("PM_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)

    from patmatchdocker_amd import engine, shards
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern

    if args.config == 4:
        motifs = batch_patterns(args.batch)
        progs = [compile_pattern(convert("-n", m)) for m in motifs]
    else:
        fwd = convert("-n", args.motif)
        comp = convert("-c", fwd)
        progs = [compile_pattern(fwd), compile_pattern(comp)]
    # '-k <k>ids' (insertions / deletions): the automaton kernels, one scan
    # per strand (bit-sliced start pass pm_ids_rev + verify + report)
    indel = args.k > 0 and any(c in args.types for c in "id")
    batch = None if indel else engine.LinearBatch(progs)

    # node-wide virtual FASTA: rank r owns records [first, first+count)
    per_rank_records = max(1, int(round(args.gbp * 1e9 / args.rec_len)))
    total_records = per_rank_records * world
    first, count = shards.shard_range(total_records, world, rank)
    rec_bytes = 10 + 1 + args.rec_len + 1
    db = engine.SequenceDatabase.synthetic(count, args.rec_len, seed=12345 + first, device=local)
    info = db.info()
    jit = os.environ.get("PM_JIT", "auto") != "0" and (os.environ.get("PM_JIT") == "1"
                                                        or info["positions"] >= (64 << 20))
    offset = first * rec_bytes
    bases_local = count * args.rec_len

    def collect(h):
        try:
            ms = engine.kernel_ms(h)
        except BaseException:
            engine.destroy_hits(h)
            raise
        # the list's own device buffers become the tensors (no copy; they
        # destroy the list when freed)
        keys, lens = shards.hits_as_tensors(h, device)
        keys = shards.to_global(keys, offset)
        # substitutions only: every hit of pattern p is prog.m long, so only
        # the keys travel (to rank 0, which rebuilds the lengths)
        out = shards.gather_hits(keys, lens, fixed_len=[p.m for p in progs])
        return out, ms

    def ids_step():
        parts_k, parts_l, ms = [], [], 0.0
        for pid, prog in enumerate(progs):
            h = engine.nfa_launch(db, prog, args.k, pid, args.types)
            try:   # keys pid << 48 | beg, copied on the device
                keys, lens = shards.hits_to_tensors(h, device)
                ms += engine.kernel_ms(h)
            finally:
                engine.destroy_hits(h)
            parts_k.append(keys)
            parts_l.append(lens)
        keys = shards.to_global(torch.cat(parts_k), offset)
        out = shards.gather_hits(keys, torch.cat(parts_l))
        return out, ms / len(progs)   # per launch (one strand)

    # pipelined (default): a step launches query i+1 (pm_scan_linear_async,
    # no host sync) and then collects query i, so the host-side collection
    # and the next launch overlap the GPU scan.  The query launched before
    # the timed region finishes before t0 (synchronize below); the timed
    # region holds K launches whose GPU work all completes inside it.
    pending = [batch.launch(db, args.k, pipelined=True)] if not (args.serial or indel) else []

    def step():
        if indel:
            return ids_step()
        if args.serial:
            return collect(batch.launch(db, args.k))
        nxt = batch.launch(db, args.k, pipelined=True)
        h, pending[0] = pending[0], nxt
        return collect(h)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    result = None
    for _ in range(args.steps):
        result, ms = step()
        kernel_ms.append(ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if pending:
        engine.destroy_hits(pending[0])   # the query launched by the last step (its work is done)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0 and args.dump_keys and result is not None:
        import numpy as np
        np.save(args.dump_keys + ".keys.npy", result[0].cpu().numpy())
        np.save(args.dump_keys + ".lens.npy", result[1].cpu().numpy())
    if rank == 0:
        bases_total = bases_local * world
        ms_step = elapsed / args.steps * 1e3
        value = bases_total * args.steps / elapsed / 1e9
        mean_kms = sum(kernel_ms) / len(kernel_ms)
        # algorithmic bytes per launch: the 2-bit code of every position of
        # the file (hi + lo bit planes, 0.25 B/position); the stream tiles'
        # halo words (+3.1 %) and lane flags are layout overhead, counted in
        # `traffic` but not here
        positions = info["positions"]
        alg_bytes = -(-positions // 32) * 8
        achieved = alg_bytes / (mean_kms * 1e-3) / 1e9 if mean_kms > 0 else 0.0
        if args.config == 4:
            workload = "configs[4]: batch of %d degenerate 12-nt DNA patterns k=%d vs %.1f Gbp synthetic DNA per GPU" % (
                len(progs), args.k, args.gbp)
        elif indel:
            workload = "configs[2]: %s -k %d%s both strands vs %.0f Gbp synthetic DNA per GPU" % (
                args.motif, args.k, args.types, args.gbp)
        else:
            workload = "configs[2]: %s k=%d both strands vs %.0f Gbp synthetic DNA per GPU" % (
                args.motif, args.k, args.gbp)
        traffic = load_traffic(workload) if jit else None
        n_hits = int(result[0].numel()) if result is not None else 0
        line = {
            "metric": "Gbases/sec scanned (whole node)",
            "value": round(value, 2),
            "unit": "Gbases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (2-bit packed bases, bit-sliced)",
            "data": "synthetic random DNA generated on device (FASTA layout, 1 Mbp records)",
            "config": {"workload": workload, "motif": args.motif if args.config == 2 else "%d-pattern batch" % len(progs),
                       "k_mismatches": args.k, "patterns": len(progs),
                       "strands": 2 if args.config == 2 else 1, "gbp_per_gpu": args.gbp, "record_len": args.rec_len,
                       "hits": n_hits, "parallelism": "shard-by-record x%d + RCCL hit gather" % world,
                       "error_types": args.types if args.k else "", "pipelined": not (args.serial or indel)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": ("pm_linear_jit (hipRTC-specialized, stream tiles + LDS-DMA ring)" if jit
                                    else "k_linear_generic"),
                         "kernel_ms": round(mean_kms, 4),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "note": "VALU-issue bound (see DESIGN.md §4)"},
        }
        line["roofline"]["issue"] = load_issue("pm_linear_jit") if jit else None
        if args.config == 4:
            # per-pattern throughput beside the scanned-bases metric
            line["pattern_gbases_per_s"] = round(value * len(progs), 1)
            # the query's algorithmic traffic is ONE read of the database
            # (alg_bytes); kernel_ms sums every specialized launch of the
            # query (the batch is split into kernels of <= 8 patterns, each
            # streaming the planes), so achieved = one read / all launches --
            # the honest HBM fraction of a VALU-bound query
            batch_filter = (jit and args.k == 0 and len(progs) >= int(os.environ.get("PM_BATCH_MIN", "16"))
                            and os.environ.get("PM_BATCH", "1") != "0")
            if batch_filter:
                # one k_batch_scan launch reads the planes once (0.25 B/base)
                # and probes a 10-mer table in LDS per position (pm_batch.hip)
                line["roofline"]["kernel"] = "k_batch_scan (q-gram filter: register transpose + LDS table probe per position)"
                line["roofline"]["note"] = ("one database read per query in one launch; VALU-issue bound "
                                            "(~5 VALU + 1 ds_read per position), see DESIGN.md §3")
                line["roofline"]["issue"] = load_issue("k_batch_scan")
            else:
                line["roofline"]["note"] = ("one database read per query; kernel_ms = the sum of the query's "
                                            "specialized launches (<= 8 patterns each); VALU-bound, see DESIGN.md §4")
            line["roofline"]["traffic"] = None
        if indel:
            line["roofline"].update({
                "kernel": "pm_ids_rev (hipRTC, bit-sliced over the 32 streams of a tile) + k_es_walk",
                "note": "per strand launch: start pass + nrgrep's esimple walk over its candidates; one read of "
                        "the planes (0.25 B/base) per launch; issue / latency bound (DESIGN.md §4)",
                "issue": load_issue("pm_ids_rev")})
            line["roofline"]["traffic"] = None
        if world == 1 and not args.no_cpu_baseline and args.config == 2:
            thr = args.cpu_threads or cpu_threads_default()
            # ~10-30 s of CPU work (nrgrep's engine runs ~0.1 Gbases/s per thread)
            mbp = args.sample_mbp if args.sample_mbp is not None else 100.0 * thr
            cb, ok, detail = cpu_baseline(db, progs, args.k, args.types if args.k else "", mbp * 1e6, result, thr)
            line["cpu_baseline"] = cb
            line["parity_sample_bit_exact"] = ok
            line["parity_sample"] = detail
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    db.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
