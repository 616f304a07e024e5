"""pm_linear_jit's effective shader clock per launch, from a bench run with
PM_JIT_CLOCK=1 (the generated kernel reads s_memtime / s_memrealtime at each
workgroup's start and end; the library prints one PM_JIT_CLOCK line per
launch on stderr, in resolution order).

    PM_JIT_CLOCK=1 python bench.py --steps 20 --warmup 5 --extras off \\
        --no-cpu-baseline 2> clk.err
    python tools/clock_trace.py clk.err [warmup] [steps] > clock_trace.json

The bench resolves 1 + warmup + steps launches of the workload: the one
launched before the warm-up, the warm-up's, the timed steps' (the last
launch of the loop is destroyed unresolved).  Reports the launches in order
and the means of the warm-up and timed groups: if a slower kernel runs at a
lower clock, the clock and the duration move together."""
import json
import re
import statistics
import sys


def main():
    path = sys.argv[1]
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    pat = re.compile(r"PM_JIT_CLOCK nwg=(\d+) kernel_ms=([\d.]+) clock_ghz=([\d.]+) min=([\d.]+) max=([\d.]+) "
                     r"span_ms=([\d.]+) t0_tick=(\d+)")
    for line in open(path):
        m = pat.search(line)
        if m:
            rows.append({"kernel_ms": float(m.group(2)), "clock_ghz": float(m.group(3)),
                         "wg_clock_min": float(m.group(4)), "wg_clock_max": float(m.group(5)),
                         "span_ms": float(m.group(6)), "t0_tick": int(m.group(7)), "nwg": int(m.group(1))})
    t0 = rows[0]["t0_tick"] if rows else 0
    for r in rows:
        r["start_ms"] = round((r.pop("t0_tick") - t0) * 1e-5, 4)
    groups = {"first": rows[:1], "warmup": rows[1:1 + warmup], "timed": rows[1 + warmup:1 + warmup + steps]}
    summary = {}
    for name, g in groups.items():
        if g:
            summary[name] = {"launches": len(g), "kernel_ms_mean": round(statistics.mean(r["kernel_ms"] for r in g), 4),
                             "clock_ghz_mean": round(statistics.mean(r["clock_ghz"] for r in g), 4)}
    if len(groups["timed"]) > 2:
        k = [r["kernel_ms"] for r in groups["timed"]]
        c = [r["clock_ghz"] for r in groups["timed"]]
        mk, mc = statistics.mean(k), statistics.mean(c)
        cov = sum((a - mk) * (b - mc) for a, b in zip(k, c))
        sk = sum((a - mk) ** 2 for a in k) ** 0.5
        sc = sum((b - mc) ** 2 for b in c) ** 0.5
        summary["timed_corr_kernel_ms_vs_clock"] = round(cov / (sk * sc), 3) if sk and sc else None
        # cycles per launch: duration x clock (constant if the clock explains the duration)
        summary["timed_mcycles_mean"] = round(statistics.mean(a * b for a, b in zip(k, c)), 4)
    json.dump({"launches": rows, "summary": summary}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
