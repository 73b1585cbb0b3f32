"""tools/alloc_tlb_probe.sh output: per process the HIP-event fractions and
the median UTCL1 translation misses per full-size dispatch.
usage: python tools/alloc_tlb_summary.py gpurun_out/alloc_tlb R"""
import csv
import json
import os
import statistics
import sys


def main():
    d, r = sys.argv[1], int(sys.argv[2])
    for i in range(1, r + 1):
        for kind in ("torch", "contiguous"):
            lines = [x for x in open(os.path.join(d, f"{kind}_{i}.log"), errors="replace") if x.startswith('{"kind"')]
            out = json.loads(lines[-1]) if lines else {"kind": kind, "error": "no line"}
            out["round"] = i
            p = os.path.join(d, f"{kind}_{i}", "run_counter_collection.csv")
            if os.path.exists(p):
                rows = list(csv.DictReader(open(p)))
                grid = {}
                for row in rows:
                    grid[row["Kernel_Name"]] = max(grid.get(row["Kernel_Name"], 0), int(row["Grid_Size"]))
                per = {}
                for row in rows:
                    if int(row["Grid_Size"]) != grid[row["Kernel_Name"]] or row["Counter_Name"] != "TCP_UTCL1_TRANSLATION_MISS_sum":
                        continue
                    k = "decode_miss" if "narrow" in row["Kernel_Name"] else "encode_miss"
                    per.setdefault(k, []).append(float(row["Counter_Value"]))
                out.update({k: statistics.median(v) for k, v in per.items()})
            print(json.dumps(out))


if __name__ == "__main__":
    main()
