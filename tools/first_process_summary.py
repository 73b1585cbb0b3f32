"""tools/first_process_probe.sh output: per process (in order) the arm, the
HIP-event fractions and the median UTCL1 translation misses per full-size
decode / encode dispatch.  usage: python tools/first_process_summary.py DIR"""
import csv
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    i = 1
    while os.path.exists(os.path.join(d, f"p{i}.log")):
        lines = [x for x in open(os.path.join(d, f"p{i}.log"), errors="replace") if x.startswith('{"kind"')]
        out = {"proc": i}
        out.update(json.loads(lines[-1]) if lines else {"error": "no line"})
        p = os.path.join(d, f"p{i}", "run_counter_collection.csv")
        if os.path.exists(p):
            rows = list(csv.DictReader(open(p)))
            grid = {}
            for r in rows:
                grid[r["Kernel_Name"]] = max(grid.get(r["Kernel_Name"], 0), int(r["Grid_Size"]))
            per = {}
            for r in rows:
                if int(r["Grid_Size"]) == grid[r["Kernel_Name"]] and r["Counter_Name"] == "TCP_UTCL1_TRANSLATION_MISS_sum":
                    per.setdefault("decode_miss" if "narrow" in r["Kernel_Name"] else "encode_miss", []).append(
                        float(r["Counter_Value"]))
            out.update({k: statistics.median(v) for k, v in per.items()})
        print(json.dumps(out))
        i += 1


if __name__ == "__main__":
    main()
