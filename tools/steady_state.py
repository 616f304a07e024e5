"""Steady-state dispatch means of each bench workload's dominant kernel,
from a rocprofv3 kernel trace of one default `bench.py` run (headline
configs[2] at 10 Gbp, then configs4, then north_star_100gbp), beside the
HIP-event means that bench line reports.

A workload's dispatches of its dominant kernel are told apart by grid size;
the LAST `steps` of them are the timed loop (before them: the query launched
ahead of the warm-up, and the warm-up), so their mean -- not the all-dispatch
mean of `--stats`, which includes the first, slower launches -- is the figure
comparable with the line's `kernel_ms`.

usage: python tools/steady_state.py <run_kernel_trace.csv> <bench line json> [steps]"""
import csv
import json
import statistics
import sys

HBM_PEAK = 8000.0


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    line = json.load(open(line_path))
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    work = [("configs[2] headline (10 Gbp)", line["roofline"], "pm_linear_jit")]
    if line.get("configs4"):
        work.append(("configs4 (256 patterns, 12.5 Gbp)", line["configs4"]["roofline"], "k_batch_scan"))
    if line.get("north_star_100gbp"):
        work.append(("north_star_100gbp (100 Gbp)", line["north_star_100gbp"]["roofline"], "pm_linear_jit"))
    seen_grids = set()
    out = {}
    for name, roof, kern in work:
        ds = [r for r in rows if r["Kernel_Name"].startswith(kern) or ("::" + kern + "(") in r["Kernel_Name"]]
        grids = []
        for r in ds:   # grid sizes in order of first appearance
            g = r["Grid_Size_X"]
            if g not in grids:
                grids.append(g)
        grid = next(g for g in grids if g not in seen_grids)
        seen_grids.add(grid)
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in ds if r["Grid_Size_X"] == grid]
        timed = d[-steps:]
        alg = roof["algorithmic_bytes_per_launch"]
        ss = statistics.mean(timed)
        out[name] = {
            "kernel": kern, "grid": int(grid), "dispatches": len(d),
            "all_dispatch_mean_ms": round(statistics.mean(d), 4),
            "steady_state_mean_ms": round(ss, 4), "steady_state_min_ms": round(min(timed), 4),
            "steady_state_max_ms": round(max(timed), 4),
            "frac_steady_state": round(alg / (ss * 1e-3) / 1e9 / HBM_PEAK, 4),
            "frac_all_dispatches": round(alg / (statistics.mean(d) * 1e-3) / 1e9 / HBM_PEAK, 4),
            "bench_hip_event_kernel_ms": roof["kernel_ms"], "bench_frac": roof["frac"],
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
