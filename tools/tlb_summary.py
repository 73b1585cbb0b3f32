"""Per process of tools/align_probe.sh: the bench line's encode / decode
fractions and batch base alignment beside the UTCL1 translation counters per
full-size dispatch (the process's arm from arm_<i>.txt).
usage: python tools/tlb_summary.py gpurun_out/align [K]"""
import csv
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len([x for x in os.listdir(d) if x.startswith("bench_")])
    for i in range(1, k + 1):
        line = [x for x in open(os.path.join(d, f"bench_{i}.log"), errors="replace") if x.startswith('{"metric"')]
        b = json.loads(line[-1]) if line else {}
        rows = list(csv.DictReader(open(os.path.join(d, f"p{i}", "run_counter_collection.csv"))))
        grid = {}
        for r in rows:
            grid[r["Kernel_Name"]] = max(grid.get(r["Kernel_Name"], 0), int(r["Grid_Size"]))
        per = {}
        for r in rows:
            if int(r["Grid_Size"]) != grid[r["Kernel_Name"]]:
                continue  # full-size dispatches only
            kind = "decode" if "narrow" in r["Kernel_Name"] else "encode"
            per.setdefault((kind, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        arm_f = os.path.join(d, f"arm_{i}.txt")
        out = {"proc": i, "arm": open(arm_f).read().strip() if os.path.exists(arm_f) else None,
               "base_alignment": b.get("config", {}).get("base_alignment"),
               "encode_frac": b.get("encode", {}).get("frac"), "decode_frac": b.get("decode", {}).get("frac")}
        for (kind, name), v in sorted(per.items()):
            out[f"{kind}.{name.replace('TCP_UTCL1_', '').replace('_sum', '')}"] = statistics.median(v)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
