#!/usr/bin/env python3
"""PatMatch scan benchmark (driver contract: one JSON line on rank 0).

Headline workload (BASELINE.json configs[2]): a 15-nt degenerate DNA motif
with k = 2 mismatches, both strands (the reference's default "Both strands"
search = pattern + reverse complement, two nrgrep_coords runs in
patmatch.py:733-743) against 10 Gbp of synthetic random DNA per GPU laid out
like a FASTA file (1 Mbp records with header lines).  A step = one query:
both strands scanned in one pass of the bit-sliced Hamming kernel over the
HBM-resident database, hits compacted + sorted on the device, copied into
framework tensors and, for N > 1, gathered to rank 0 over RCCL and merged.
Weak scaling: every GPU owns its own 10 Gbp shard (records of one node-wide
virtual FASTA).

The default run (no workload flags) then measures, in the same process and
after the headline (whose database is freed first), the other BASELINE
workloads that fit one GPU, each as a sub-object of the same line:
  "configs4"           configs[4]: the batch of 256 degenerate 12-nt
                       patterns at k = 0, 12.5 Gbp per GPU (100 Gbp over 8
                       GPUs), dominant kernel k_batch_scan;
  "north_star_100gbp"  the headline motif over 100 Gbp per GPU (north_star's
                       "≥ 70 % of HBM-read roofline on a 100 Gbp scan").
Each has its own roofline, and at N = 1 its own CPU baseline and parity
sample (`--extras off` skips them; `--cfg4-gbp` / `--north-gbp` resize them
for tests).

Reported beside the throughput:
  roofline      the dominant kernel's algorithmic bytes (2-bit planes,
                0.25 B per position) / its HIP-event duration vs the 8 TB/s
                HBM peak; traffic = PMC HBM bytes per launch from profiles/
                when a counter run of this workload is committed there;
  cpu_baseline  configs[2]: nrgrep's own esimple engine restated from the
                binary (oracle/pm_nrgrep.c); configs[4]: one bit-parallel
                Shift-And scan per pattern (oracle/pm_cpuscan.c), as the
                reference runs one nrgrep_coords process per pattern -- one
                thread per host core of the box's CPU share (at most 16), on
                a bounded sample of the same database decoded from HBM; the
                sample's matches are a bit-exact parity check of the GPU's.

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
ROUND = "r06"   # committed PMC traffic run (profiles/r06_traffic.json)
# flags that change the headline workload: with none of them the run also
# measures the extra workloads (configs4, north_star_100gbp)
WORKLOAD_FLAGS = ("--config", "--gbp", "--rec-len", "--motif", "--k", "--types", "--serial", "--batch")


def parse_args(argv=None):
    argv = sys.argv[1:] if argv is None else argv
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
    ap.add_argument("--extras", default="auto", choices=("auto", "on", "off"),
                    help="also measure configs4 and north_star_100gbp after the headline (auto: when no "
                         "workload flag is given)")
    ap.add_argument("--cfg4-gbp", type=float, default=12.5, help="configs4 extra: Gbp per GPU")
    ap.add_argument("--north-gbp", type=float, default=100.0, help="north_star_100gbp extra: Gbp per GPU")
    ap.add_argument("--extra-steps", type=int, default=None, help="timed steps of each extra (default --steps)")
    ap.add_argument("--dump-keys", default=None,
                    help="tests: rank 0 saves the last step's gathered hit keys and lengths (<path>.keys.npy, "
                         "<path>.lens.npy)")
    args = ap.parse_args(argv)
    given = {a.split("=")[0] for a in argv}
    if args.config == 4 and "--gbp" not in given:
        args.gbp = 12.5
    if args.config == 4 and "--k" not in given:
        args.k = 0
    args.run_extras = args.extras == "on" or (args.extras == "auto" and not given & set(WORKLOAD_FLAGS))
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
    """PMC HBM bytes per launch of `workload`'s dominant kernel from the
    committed counter run (profiles/<ROUND>_traffic.json: one object, or a
    list of them, keyed by the workload string)."""
    path = os.path.join(ROOT, "profiles", "%s_traffic.json" % ROUND)
    try:
        with open(path) as fh:
            data = json.load(fh)
    except (OSError, ValueError):
        return None
    for entry in data if isinstance(data, list) else [data]:
        if isinstance(entry, dict) and entry.get("workload") == workload:
            return entry.get("hbm_bytes_per_launch")
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


def region_pieces(db, sample_bp):
    """configs[4]'s CPU sample, cut along nrgrep's search regions (§1 of
    DESIGN.md: the k = 0 simple engine's windows may run over a '\\n', so
    only a region start is a place where the GPU's report rule and a scan of
    the piece alone restart alike): the first whole regions up to
    `sample_bp` positions and the last ones from `sample_bp` before the end.
    Returns [(offset, text, [(beg, end) regions in piece coordinates])]."""
    starts, ends = (a.tolist() for a in db.regions())
    n = db.info()["positions"]
    head_end = next((e for e in ends if e >= sample_bp), ends[-1])
    spans = [(0, head_end)]
    tail_beg = next((t for t in starts if t >= n - sample_bp), None)
    if tail_beg is not None and tail_beg >= head_end:
        spans.append((tail_beg, ends[-1]))
    out = []
    for a, b in spans:
        regs = [(t - a, e - a) for t, e in zip(starts, ends) if t >= a and e <= b]
        out.append((a, db.decode(a, b - a), regs))
    return out


def compare_sample(pieces, want, gpu_hits, n_patterns):
    """Bit-exact check of the GPU's sorted (pattern << 48 | beg) keys and
    lengths against the CPU's matches, piece by piece: want[i][p] is the
    list of (beg, end) the CPU printed for pattern p in piece i (offsets in
    the piece).  Vectorized (configs[4] lists hold ~30 M keys)."""
    import numpy as np
    keys = gpu_hits[0].cpu().numpy().astype(np.int64)
    lens = gpu_hits[1].cpu().numpy().astype(np.int64)
    pos = keys & ((1 << 48) - 1)
    ok, checked = True, 0
    for (off, text), per_pattern in zip(pieces, want):
        sel = (pos >= off) & (pos + lens <= off + len(text))
        got_k, got_l = keys[sel], lens[sel]
        wk = [np.asarray([(p << 48) | (b + off) for b, _ in hits], dtype=np.int64) for p, hits in enumerate(per_pattern)]
        wl = [np.asarray([e - b for b, e in hits], dtype=np.int64) for hits in per_pattern]
        exp_k = np.concatenate(wk) if wk else np.zeros(0, np.int64)
        exp_l = np.concatenate(wl) if wl else np.zeros(0, np.int64)
        ok &= bool(np.array_equal(got_k, exp_k) and np.array_equal(got_l, exp_l))
        checked += int(exp_k.size)
    return ok, checked


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
    ok, checked = compare_sample(pieces, base, gpu_hits, len(progs))
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


def cpu_baseline_batch(db, progs, sample_bp, gpu_hits, threads):
    """configs[4]'s CPU baseline: the reference answers a batch with one
    nrgrep_coords process per pattern (patmatch.py:733-743), each reading
    the whole file.  Here each pattern is one task on a pool of `threads`
    host threads (ctypes releases the GIL), scanning the sample with the
    bit-parallel Shift-And automaton (oracle/pm_cpuscan.c pmc_shiftadd at
    k = 0: the simple engine's windows, which may span a line break) region
    by region (nrgrep's -b 1600000 buffers, oracle.by_region), header-line
    hits dropped as process_output does.  The sample is the first and last
    `sample_bp` positions of the database, decoded from HBM; the matches of
    every pattern must equal the GPU's there.  Returns (dict, ok, detail)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle
    sample = region_pieces(db, sample_bp)
    pieces = [(off, text) for off, text, _ in sample]

    def one(task):
        text, regs, prog = task
        return oracle.by_region(text, lambda t: oracle.shiftadd_scan(t, prog, 0), skip_headers=True, regs=regs)

    t0, c0 = time.perf_counter(), time.process_time()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        base = [list(ex.map(one, [(text, regs, p) for p in progs])) for _, text, regs in sample]
    dt = time.perf_counter() - t0
    cpu_s = time.process_time() - c0
    bases = sum(sum(len(line) for line in text.split(b"\n")) - text.count(b">") for _, text in pieces)
    ok, checked = compare_sample(pieces, base, gpu_hits, len(progs))
    detail = {"pieces": [[off, off + len(text)] for off, text in pieces], "hits_checked": checked}
    return {"value": bases / dt / 1e9, "unit": "Gbases/s", "cores": threads, "kind": "port",
            "sample": "first and last %.0f Mbp of the synthetic database (decoded from HBM), all %d patterns, "
                      "k = 0: one bit-parallel Shift-And scan per pattern (oracle/pm_cpuscan.c pmc_shiftadd, "
                      "nrgrep's simple-engine windows and report rule, 1.6 MB regions) as the reference runs "
                      "one nrgrep_coords per pattern, patterns spread over %d host threads; value = sample "
                      "bases / wall time for the whole batch; %.1f s wall, %.1f s CPU, %d CPUs in the "
                      "affinity mask" % (sample_bp / 1e6, len(progs), threads, dt, cpu_s,
                                         len(os.sched_getaffinity(0)))}, ok, detail


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


class Ctx:
    """The process's place in the job: world, rank, device, collectives."""

    def __init__(self, world, rank, local, device, rehearse):
        self.world, self.rank, self.local, self.device, self.rehearse = world, rank, local, device, rehearse


def run_workload(ctx, config, motif, k, types, gbp, rec_len, n_batch, serial, steps, warmup):
    """Builds one workload's synthetic database on this rank, runs `warmup`
    untimed steps and times exactly `steps` (barrier + synchronize on both
    sides, max over ranks).  Returns a dict with the database still open
    (the caller closes it after the CPU baseline)."""
    import torch
    import torch.distributed as dist
    from patmatchdocker_amd import engine, shards
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern

    world, rank, device = ctx.world, ctx.rank, ctx.device
    if config == 4:
        progs = [compile_pattern(convert("-n", m)) for m in batch_patterns(n_batch)]
    else:
        fwd = convert("-n", motif)
        progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    # '-k <k>ids' (insertions / deletions): the automaton kernels, one scan
    # per strand (bit-sliced start pass pm_ids_rev + verify + report)
    indel = k > 0 and any(c in types for c in "id")
    batch = None if indel else engine.LinearBatch(progs)

    # node-wide virtual FASTA: rank r owns records [first, first+count)
    per_rank_records = max(1, int(round(gbp * 1e9 / rec_len)))
    first, count = shards.shard_range(per_rank_records * world, world, rank)
    rec_bytes = 10 + 1 + rec_len + 1
    db = engine.SequenceDatabase.synthetic(count, rec_len, seed=12345 + first, device=ctx.local)
    info = db.info()
    jit = os.environ.get("PM_JIT", "auto") != "0" and (os.environ.get("PM_JIT") == "1"
                                                        or info["positions"] >= (64 << 20))
    offset = first * rec_bytes

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

    def ids_launch():
        # both strands' automaton scans (PM_PIPELINED unless --serial: each
        # returns once its report pass is queued, so strand 1's scan queues
        # behind strand 0's report with no host wait between them)
        handles = []
        try:
            for pid, prog in enumerate(progs):
                handles.append(engine.nfa_launch(db, prog, k, pid, types, pipelined=not serial))
        except BaseException:
            for h in handles:
                engine.destroy_hits(h)
            raise
        return handles

    def ids_collect(handles):
        parts_k, parts_l, ms = [], [], 0.0
        try:
            for h in handles:   # keys pid << 48 | beg, copied on the device
                keys, lens = shards.hits_to_tensors(h, device)
                ms += engine.kernel_ms(h)
                parts_k.append(keys)
                parts_l.append(lens)
        finally:
            for h in handles:
                engine.destroy_hits(h)
        keys = shards.to_global(torch.cat(parts_k), offset)
        out = shards.gather_hits(keys, torch.cat(parts_l))
        return out, ms / len(progs)   # per launch (one strand)

    # pipelined (default): a step launches query i+1 (pm_scan_linear_async,
    # no host sync; '-k <k>ids': both strands' automaton scans) and then
    # collects query i, so the host-side collection and the next launch
    # overlap the GPU scan.  The query launched before the timed region
    # finishes before t0 (synchronize below); the timed region holds K
    # launches whose GPU work all completes inside it.
    pending = []
    if not serial:
        pending.append(ids_launch() if indel else batch.launch(db, k, pipelined=True))

    def step():
        if serial:
            return ids_collect(ids_launch()) if indel else collect(batch.launch(db, k))
        nxt = ids_launch() if indel else batch.launch(db, k, pipelined=True)
        h, pending[0] = pending[0], nxt
        return ids_collect(h) if indel else collect(h)

    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    result = None
    for _ in range(steps):
        result, ms = step()
        kernel_ms.append(ms)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if pending:   # the query launched by the last step (its work is done)
        for h in pending[0] if indel else pending:
            engine.destroy_hits(h)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if ctx.rehearse else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return {"db": db, "info": info, "progs": progs, "jit": jit, "indel": indel, "result": result,
            "elapsed": elapsed, "kernel_ms": kernel_ms, "bases_local": count * rec_len, "steps": steps}


def roofline(run, kernel, note):
    """The dominant kernel's HBM roofline: algorithmic bytes per launch =
    the 2-bit code of every position of the file (hi + lo bit planes,
    0.25 B/position; the stream tiles' halo words (+3.1 %) and lane flags
    are layout overhead, counted in `traffic` but not here), over the mean
    HIP-event duration of the launches in the timed steps."""
    mean_kms = sum(run["kernel_ms"]) / len(run["kernel_ms"])
    alg_bytes = -(-run["info"]["positions"] // 32) * 8
    achieved = alg_bytes / (mean_kms * 1e-3) / 1e9 if mean_kms > 0 else 0.0
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
            "kernel_ms": round(mean_kms, 4), "algorithmic_bytes_per_launch": alg_bytes, "note": note}


def throughput(run, world):
    ms_step = run["elapsed"] / run["steps"] * 1e3
    value = run["bases_local"] * world * run["steps"] / run["elapsed"] / 1e9
    return value, ms_step


def batch_filter_on(run, k):
    return (run["jit"] and k == 0 and len(run["progs"]) >= int(os.environ.get("PM_BATCH_MIN", "16"))
            and os.environ.get("PM_BATCH", "1") != "0")


def batch_roofline(run, k):
    if batch_filter_on(run, k):
        # one k_batch_scan launch reads the planes once (0.25 B/base) and
        # probes a 10-mer table in LDS per position (pm_batch.hip)
        return roofline(run, "k_batch_scan (q-gram filter: register transpose + LDS table probe per position)",
                        "one database read per query in one launch; kernel_ms = k_batch_scan alone (the "
                        "verify, exception pass, sort and report follow it in the step); see DESIGN.md §3")
    # the query's algorithmic traffic is ONE read of the database;
    # kernel_ms sums every specialized launch of the query (<= 8 patterns
    # each, each streaming the planes)
    return roofline(run, "pm_linear_jit x %d launches (<= 8 patterns each)" % -(-len(run["progs"]) // 8),
                    "one database read per query; kernel_ms = the sum of the query's specialized launches")


def extra_configs4(ctx, args, steps):
    """configs[4] (the 256-pattern batch at k = 0) as a sub-object: its
    throughput, k_batch_scan's roofline and, at N = 1, a CPU baseline +
    parity sample."""
    k = 0
    run = run_workload(ctx, 4, None, k, "", args.cfg4_gbp, args.rec_len, args.batch, False, steps,
                       max(1, args.warmup))
    try:
        if ctx.rank != 0:
            return None
        value, ms_step = throughput(run, ctx.world)
        out = {"workload": "configs[4]: batch of %d degenerate 12-nt DNA patterns k=0 vs %.1f Gbp synthetic DNA "
                           "per GPU (%.1f Gbp over %d GPU%s)" % (len(run["progs"]), args.cfg4_gbp,
                                                                 args.cfg4_gbp * ctx.world, ctx.world,
                                                                 "s" if ctx.world > 1 else ""),
               "value": round(value, 2), "unit": "Gbases/s", "ms_per_step": round(ms_step, 4), "steps": steps,
               "pattern_gbases_per_s": round(value * len(run["progs"]), 1),
               "hits": int(run["result"][0].numel()), "roofline": batch_roofline(run, k)}
        out["roofline"]["traffic"] = load_traffic(out["workload"])
        if ctx.world == 1 and not args.no_cpu_baseline:
            thr = args.cpu_threads or cpu_threads_default()
            # ~10-20 s of CPU work: Shift-And runs ~0.25 Gbases/s per thread
            # and pattern, 256 patterns per base
            mbp = 6.0 * thr
            cb, ok, detail = cpu_baseline_batch(run["db"], run["progs"], mbp * 1e6, run["result"], thr)
            out["cpu_baseline"] = cb
            out["parity_sample_bit_exact"] = ok
            out["parity_sample"] = detail
        else:
            out["cpu_baseline"] = None
        return out
    finally:
        run["db"].close()


def extra_north_star(ctx, args, steps):
    """The north-star size: the headline motif and k over `--north-gbp`
    (100) Gbp per GPU, pm_linear_jit's roofline and, at N = 1, a CPU
    baseline + parity sample over the first and last 400 Mbp."""
    run = run_workload(ctx, 2, args.motif, args.k, args.types, args.north_gbp, args.rec_len, args.batch, False,
                       steps, max(1, args.warmup))
    try:
        if ctx.rank != 0:
            return None
        value, ms_step = throughput(run, ctx.world)
        out = {"workload": "configs[2] motif at the north-star size: %s k=%d both strands vs %.0f Gbp synthetic "
                           "DNA per GPU" % (args.motif, args.k, args.north_gbp),
               "value": round(value, 2), "unit": "Gbases/s", "ms_per_step": round(ms_step, 4), "steps": steps,
               "hits": int(run["result"][0].numel()),
               "roofline": roofline(run, "pm_linear_jit (hipRTC-specialized, stream tiles + LDS-DMA ring)" if run["jit"]
                                    else "k_linear_generic", "VALU-issue bound (see DESIGN.md §4)")}
        out["roofline"]["traffic"] = load_traffic(out["workload"])
        if ctx.world == 1 and not args.no_cpu_baseline:
            thr = args.cpu_threads or cpu_threads_default()
            cb, ok, detail = cpu_baseline(run["db"], run["progs"], args.k, args.types if args.k else "",
                                          25.0 * thr * 1e6, run["result"], thr)
            out["cpu_baseline"] = cb
            out["parity_sample_bit_exact"] = ok
            out["parity_sample"] = detail
        else:
            out["cpu_baseline"] = None
        return out
    finally:
        run["db"].close()


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
    ctx = Ctx(world, rank, local, device, rehearse)

    run = run_workload(ctx, args.config, args.motif, args.k, args.types, args.gbp, args.rec_len, args.batch,
                       args.serial, args.steps, args.warmup)
    db, progs, jit, indel, result = run["db"], run["progs"], run["jit"], run["indel"], run["result"]
    line = None
    if rank == 0 and args.dump_keys and result is not None:
        import numpy as np
        np.save(args.dump_keys + ".keys.npy", result[0].cpu().numpy())
        np.save(args.dump_keys + ".lens.npy", result[1].cpu().numpy())
    if rank == 0:
        value, ms_step = throughput(run, world)
        if args.config == 4:
            workload = "configs[4]: batch of %d degenerate 12-nt DNA patterns k=%d vs %.1f Gbp synthetic DNA per GPU" % (
                len(progs), args.k, args.gbp)
        elif indel:
            workload = "configs[2]: %s -k %d%s both strands vs %.0f Gbp synthetic DNA per GPU" % (
                args.motif, args.k, args.types, args.gbp)
        else:
            workload = "configs[2]: %s k=%d both strands vs %.0f Gbp synthetic DNA per GPU" % (
                args.motif, args.k, args.gbp)
        n_hits = int(result[0].numel()) if result is not None else 0
        if args.config == 4:
            roof = batch_roofline(run, args.k)
        elif indel:
            roof = roofline(run, "pm_ids_rev (hipRTC, bit-sliced over the 32 streams of a tile) + k_es_walk",
                            "per strand launch: start pass + nrgrep's esimple walk over its candidates; one read "
                            "of the planes (0.25 B/base) per launch; issue / latency bound (DESIGN.md §4)")
            roof["issue"] = load_issue("pm_ids_rev")
        else:
            roof = roofline(run, "pm_linear_jit (hipRTC-specialized, stream tiles + LDS-DMA ring)" if jit
                            else "k_linear_generic", "VALU-issue bound (see DESIGN.md §4)")
            roof["issue"] = load_issue("pm_linear_jit") if jit else None
        roof["traffic"] = load_traffic(workload) if jit else None
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
                       "error_types": args.types if args.k else "", "pipelined": not args.serial},
            "roofline": roof,
        }
        if args.config == 4:
            # per-pattern throughput beside the scanned-bases metric
            line["pattern_gbases_per_s"] = round(value * len(progs), 1)
        line["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline:
            thr = args.cpu_threads or cpu_threads_default()
            if args.config == 2:
                # ~10-30 s of CPU work (nrgrep's engine runs ~0.1 Gbases/s per thread)
                mbp = args.sample_mbp if args.sample_mbp is not None else 100.0 * thr
                cb, ok, detail = cpu_baseline(db, progs, args.k, args.types if args.k else "", mbp * 1e6, result, thr)
            else:
                mbp = args.sample_mbp if args.sample_mbp is not None else 6.0 * thr
                cb, ok, detail = cpu_baseline_batch(db, progs, mbp * 1e6, result, thr)
            line["cpu_baseline"] = cb
            line["parity_sample_bit_exact"] = ok
            line["parity_sample"] = detail
    # the headline's database and hit list leave HBM before the extras
    result = run = None
    db.close()
    if args.run_extras:
        steps = args.extra_steps or args.steps
        sub = extra_configs4(ctx, args, steps)
        if rank == 0:
            line["configs4"] = sub
        sub = extra_north_star(ctx, args, steps)
        if rank == 0:
            line["north_star_100gbp"] = sub
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
