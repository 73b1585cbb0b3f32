"""Summarise tools/profile_mixed.sh (rocprofv3 over tools/mixed_probe.py) into
one JSON: per ragged kernel, its average dispatch duration from the kernel
trace, and HBM bytes per dispatch from the FETCH_SIZE / WRITE_SIZE passes
(same gfx950 corrections as tools/pmc_summary.py: KiB units, FETCH_SIZE x2
for 16 B/lane streams), beside the algorithmic bytes mixed_probe prints
(encode 14 L per stripe, decode (10 + e) L per stripe with e >= 1).

usage: python tools/pmc_mixed_summary.py gpurun_out/profmix out.json
"""
import csv
import json
import os
import statistics
import sys


def kernel_kind(name):
    if "rs104_bs_ragged_kernel" in name or "rs104_ragged_kernel<false" in name:
        return "encode"
    if "rs104_ragged_kernel<true" in name:
        return "decode"
    return None


def main():
    d, out = sys.argv[1], sys.argv[2]
    probe = [json.loads(line) for line in open(os.path.join(d, "mixed_trace.jsonl"))]
    algo = {"encode": probe[0]["enc_bytes"], "decode": probe[0]["dec_bytes"]}
    res = {"source": d, "workload": "tools/mixed_probe.py: 512 stripes, 64 KiB..4 MiB shards, 0..4 erasures",
           "correction": "FETCH_SIZE*1024*2, WRITE_SIZE*1024", "kernels": {}}
    durs = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
        k = kernel_kind(r["Kernel_Name"])
        if k:
            durs.setdefault((k, r["Kernel_Name"]), []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for (k, name), v in durs.items():
        timed = v[1:] if len(v) > 2 else v  # the first dispatch is the probe's warm-up
        ms = statistics.mean(timed)
        res["kernels"][k] = {"kernel": name, "dispatches": len(v), "ms_avg": round(ms, 4),
                             "algorithmic_bytes": algo[k],
                             "achieved_TBps": round(algo[k] / (ms * 1e-3) / 1e12, 3),
                             "frac_of_8TBps": round(algo[k] / (ms * 1e-3) / 8e12, 4)}
    for counter, sub, scale in (("FETCH_SIZE", "pmc_fetch", 2), ("WRITE_SIZE", "pmc_write", 1)):
        per = {}
        for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_kind(r["Kernel_Name"])
            if k:
                per.setdefault(k, []).append(float(r["Counter_Value"]) * 1024 * scale)
        for k, v in per.items():
            res["kernels"].setdefault(k, {})[counter.lower() + "_bytes_per_dispatch"] = statistics.median(v)
    for k, e in res["kernels"].items():
        if "fetch_size_bytes_per_dispatch" in e and "write_size_bytes_per_dispatch" in e:
            e["hbm_bytes_per_dispatch"] = e["fetch_size_bytes_per_dispatch"] + e["write_size_bytes_per_dispatch"]
            e["traffic_over_algorithmic"] = round(e["hbm_bytes_per_dispatch"] / algo[k], 4)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
