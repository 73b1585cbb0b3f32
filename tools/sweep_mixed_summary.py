"""Summarise tools/sweep_mixed.sh: per case and kernel, the median dispatch
duration from the rocprofv3 kernel trace (the probe's first dispatch of each
kernel is its warm-up and is dropped) and the achieved TB/s on the
algorithmic bytes the probe prints (encode 14 L per stripe, decode (10 + e) L
per stripe with e >= 1).

usage: python tools/sweep_mixed_summary.py gpurun_out/sweep [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys


def kind(name):
    if "fill_splitmix" in name:
        return None
    if "ragged" in name:
        return ("ragged", "encode" if ("bs_ragged" in name or "ragged_kernel<false" in name) else "decode")
    if "rs104" in name or "rs_apply" in name:
        return ("strided", "decode" if "<true" in name else "encode")
    return None


def main():
    d = sys.argv[1]
    rows = []
    for tr in sorted(glob.glob(os.path.join(d, "*", "run_kernel_trace.csv"))):
        case = os.path.basename(os.path.dirname(tr))
        probe = [json.loads(x) for x in open(os.path.join(d, case + ".jsonl")) if x.startswith("{")]
        if not probe:
            continue
        algo = {"encode": probe[0]["enc_bytes"], "decode": probe[0]["dec_bytes"]}
        durs = {}
        for r in csv.DictReader(open(tr)):
            k = kind(r["Kernel_Name"])
            if k:
                durs.setdefault((k, r["Kernel_Name"].split("(")[0]), []).append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        for ((path, op), name), v in sorted(durs.items()):
            ms = statistics.median(v[1:] if len(v) > 2 else v)
            rows.append({"case": case, "stripes": probe[0]["stripes"], "path": path, "op": op, "kernel": name,
                         "dispatches": len(v), "ms_median": round(ms, 4), "algorithmic_bytes": algo[op],
                         "TBps": round(algo[op] / (ms * 1e-3) / 1e12, 3),
                         "frac_of_8TBps": round(algo[op] / (ms * 1e-3) / 8e12, 4)})
    # the probe's own per-variant event timings (variants alternate inside one
    # process, so the kernel trace alone cannot tell them apart)
    for case_file in sorted(glob.glob(os.path.join(d, "*.jsonl"))):
        case = os.path.basename(case_file)[:-6]
        if case == "summary":
            continue
        groups = {}
        for x in open(case_file):
            if not x.startswith("{"):
                continue
            j = json.loads(x)
            key = ("grouped_strided",) if j.get("grouped_strided") else (
                j.get("kind", "ragged"), j.get("order", "given"), "bal%d" % j.get("balance", 0), j.get("pad", 0),
                j.get("enc_remap", 0),
                j.get("dec_vec_bytes", 8))
            groups.setdefault(key, []).append(j)
        for key, js in groups.items():
            rows.append({"case": case, "variant": "/".join(str(k) for k in key), "rounds": len(js),
                         "enc_ms_median": round(statistics.median(j["enc_ms"] for j in js), 4),
                         "dec_ms_median": round(statistics.median(j["dec_ms"] for j in js), 4),
                         "enc_TBps_median": round(statistics.median(j["enc_TBps"] for j in js), 3),
                         "dec_TBps_median": round(statistics.median(j["dec_TBps"] for j in js), 3),
                         "source": "probe HIP events"})
    for r in rows:
        print(json.dumps(r))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
