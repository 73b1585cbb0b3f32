"""Summarise a rocprofv3 SQ/GRBM counter pass over the RS kernels into
per-kernel wave-state fractions and VALU busy (profiles/r01/pmc_sq_wave_states.json).

Units (MI355X_MICROARCH.md, PMC notes): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs
(cycles = GUI_ACTIVE / 8); a wave64 VALU instruction issues in 2 cycles on a
32-wide CDNA4 SIMD, and the chip has 256 CUs x 4 SIMDs.

usage: python tools/sq_summary.py <run_counter_collection.csv> <out.json>
"""
import collections
import csv
import json
import statistics
import sys

SIMDS = 256 * 4
# input bytes one launch reads (the BASELINE batch: 4096 stripes x 10 x 1 MiB);
# set to 0 to leave valu_insts_per_KiB out for other workloads
BYTES_PER_LAUNCH = 4096 * 10 * (1 << 20)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(src)):
        key = r["Dispatch_Id"]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]),
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, int(r["VGPR_Count"]))
    big = collections.defaultdict(int)  # largest grid per kernel: the batch-size dispatches
    for name, g, _, _ in meta.values():
        big[name] = max(big[name], g)
    out = {"source": src, "units": __doc__.split("Units")[1].split("usage")[0].strip(), "kernels": {}}
    by_kernel = collections.defaultdict(list)
    for key, c in per.items():
        name, grid, ms, vgpr = meta[key]
        if grid * 2 < big[name]:  # skip the small verification dispatches
            continue
        cycles = c["GRBM_GUI_ACTIVE"] / 8
        wc = c["SQ_WAVE_CYCLES"]
        by_kernel[name].append({
            "ms": ms, "rocprof_vgpr_count_field": vgpr,
            "clock_GHz": cycles / (ms * 1e-3) / 1e9,
            "valu_busy": c["SQ_INSTS_VALU"] * 2 / (SIMDS * cycles),
            "wave_waiting_on_memory": c["SQ_WAIT_ANY"] / wc,
            "wave_issue_stalled": c["SQ_WAIT_INST_ANY"] / wc,
            "wave_issuing": c["SQ_ACTIVE_INST_ANY"] / wc,
            "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
            "valu_insts_per_KiB": c["SQ_INSTS_VALU"] * 1024 / BYTES_PER_LAUNCH if BYTES_PER_LAUNCH else None,
        })
    for name, ds in by_kernel.items():
        ds = ds[1:] if len(ds) > 1 else ds  # first dispatch is the warm-up
        out["kernels"][name] = {k: round(statistics.mean(d[k] for d in ds), 4) for k in ds[0]}
        out["kernels"][name]["dispatches"] = len(ds)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main()
