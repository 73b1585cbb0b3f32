"""Per-launch durations of the bench's TIMED dispatches from a rocprofv3
kernel trace of `bench.py --steps K --warmup W`, beside the HIP-event times
the same process printed in its bench line.

The rocprofv3 --stats average mixes every dispatch of a kernel: the warm-up
launches, the post-timing verification reconstruct (one more full-size
decode) and the packed-layout pass (same kernel, same grid). This keeps, per
kernel, its full-size dispatches in dispatch order and takes positions
[W, W + K): the K timed launches, which bench.py issues after exactly W
warm-up launches of each kind. Everything else is counted and excluded.

usage: python tools/trace_summary.py <kernel_trace.csv> <bench stdout/stderr log> <out.json>
"""
import csv
import json
import statistics
import sys

HBM_PEAK_GBPS = 8000.0


def bench_line(path):
    for line in open(path, errors="replace"):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench line in {path}")


def trace_key(bench_kernel_name):
    """bench's kernel name -> (base, DEC) to match the trace's demangled name:
    'rs104_narrow_kernel<DEC=true, 8 B per lane> (table lookup)' ->
    ('rs104_narrow_kernel', 'true'); 'rs104_bs_encode_kernel (bit-sliced)' ->
    ('rs104_bs_encode_kernel', None)."""
    base = bench_kernel_name.split("<")[0].split(" ")[0]
    dec = None
    if "DEC=true" in bench_kernel_name:
        dec = "true"
    elif "DEC=false" in bench_kernel_name:
        dec = "false"
    return base, dec


def matches(trace_name, key):
    """A template kernel demangles as base<args>(...), a plain one as base(...)."""
    base, dec = key
    i = trace_name.find(base + "<")
    if i < 0:
        return dec is None and (base + "(") in trace_name
    return dec is None or trace_name[i + len(base) + 1:].startswith(dec)


def summarise(rows, key, warmup, steps, alg_bytes, event_ms):
    mine = [r for r in rows if matches(r["Kernel_Name"], key)]
    grid = max(int(r["Grid_Size_X"]) for r in mine)
    full = [r for r in mine if int(r["Grid_Size_X"]) == grid]
    timed = full[warmup:warmup + steps]
    if len(timed) != steps:
        raise SystemExit(f"{key}: {len(full)} full-size dispatches, need {warmup + steps}")
    ns = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    mean_ms = statistics.mean(ns) / 1e6
    frac_trace = alg_bytes / (mean_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    frac_events = alg_bytes / (event_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS
    return {
        "kernel": timed[0]["Kernel_Name"],
        "grid_size_x": grid,
        "dispatch_ids": [int(r["Dispatch_Id"]) for r in timed],
        "full_size_dispatches": len(full),
        "excluded": {"warmup": warmup, "after_timed_region": len(full) - warmup - steps,
                     "smaller_grids": len(mine) - len(full)},
        "trace_ms_mean": round(mean_ms, 4),
        "trace_ms_median": round(statistics.median(ns) / 1e6, 4),
        "trace_ms_min": round(min(ns) / 1e6, 4),
        "trace_ms_max": round(max(ns) / 1e6, 4),
        "algorithmic_bytes_per_launch": alg_bytes,
        "frac_trace": round(frac_trace, 4),
        "hip_events_ms_mean": event_ms,
        "frac_hip_events": round(frac_events, 4),
        "trace_over_events": round(mean_ms / event_ms, 4),
    }


def main():
    trace_csv, log, dst = sys.argv[1:4]
    b = bench_line(log)
    S, L = b["config"]["stripes_per_gpu"], b["config"]["shard_len"]
    rows = [r for r in csv.DictReader(open(trace_csv)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    alg = S * 14 * L  # encode: 10 reads + 4 writes; 4-erasure decode: 10 survivors + 4 rebuilt
    out = {
        "source": {"trace": trace_csv, "bench_log": log},
        "bench": {"value": b["value"], "steps": b["steps"], "warmup": b["warmup"], "workload": b["config"]["workload"],
                  "roofline_frac": b["roofline"]["frac"], "roofline_launch": b["roofline"].get("launch")},
        "selection": "per kernel: full-size dispatches in dispatch order, positions [warmup, warmup + steps)",
        "encode": summarise(rows, trace_key(b["encode"]["kernel"]), b["warmup"], b["steps"], alg,
                            b["encode"]["ms_per_launch"]),
        "decode": summarise(rows, trace_key(b["decode"]["kernel"]), b["warmup"], b["steps"], alg,
                            b["decode"]["ms_per_launch"]),
    }
    dom = "decode" if out["decode"]["trace_ms_mean"] >= out["encode"]["trace_ms_mean"] else "encode"
    out["dominant"] = {"launch": dom, "frac_trace": out[dom]["frac_trace"],
                       "frac_hip_events": out[dom]["frac_hip_events"],
                       "agree_within": round(abs(out[dom]["frac_trace"] / out[dom]["frac_hip_events"] - 1), 4)}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out["dominant"]))


if __name__ == "__main__":
    main()
