"""Stage timing of the GPU file layer (write_ec_files / rebuild_ec_files) on a
synthetic volume in /dev/shm: run with HEC_FILE_TRACE=1 to get the pipeline's
per-stage seconds on stderr. Each call also reports the process's CPU
seconds (user + system, all threads) beside its wall time, and the cgroup's
CPU quota: CPU-seconds near quota x wall means the call is CPU-bound.
Measurement only.

python tools/file_stages.py [--gib 12] [--reps 2]
(The round-5 zero-copy file path this tool also timed was removed in round 6:
profiles/r05/file_stages_b.json.)
"""
import argparse
import json
import os
import resource
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_s():
    """user + system CPU seconds of this process, all threads"""
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def cpu_quota():
    """the cgroup's CPU limit (cpu.max: quota / period), or None"""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=12.0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--fresh", action="store_true", help="delete the shard files before each timed encode")
    ap.add_argument("--dir", default="/dev/shm", help="filesystem to run on (default tmpfs: page-cache rate)")
    args = ap.parse_args()
    paths = ["staged"]
    import helyim_amd as H
    from tools.bench_files import make_volume
    d = tempfile.mkdtemp(prefix="hec_stages_", dir=args.dir)
    try:
        base = os.path.join(d, "v")
        nbytes = int(args.gib * 2**30)
        make_volume(base + ".dat", nbytes)
        out = {"dir": args.dir, "dat_bytes": nbytes, "fresh": args.fresh, "cpu_quota": cpu_quota(), "paths": {}}
        for p in paths:
            out["paths"][p] = {"encode_s": [], "rebuild_s": [], "encode_cpu_s": [], "rebuild_cpu_s": []}
        H.write_ec_files(base)  # warm-up: device tables, pinned staging
        for _ in range(args.reps):
            for p in paths:
                r = out["paths"][p]
                if args.fresh:
                    for i in range(14):
                        os.remove(base + H.to_ext(i))
                c0, t0 = cpu_s(), time.perf_counter()
                H.write_ec_files(base)
                r["encode_s"].append(round(time.perf_counter() - t0, 4))
                r["encode_cpu_s"].append(round(cpu_s() - c0, 3))
        for _ in range(args.reps):
            for p in paths:
                r = out["paths"][p]
                for i in (0, 5, 10, 13):
                    os.remove(base + H.to_ext(i))
                c0, t0 = cpu_s(), time.perf_counter()
                H.rebuild_ec_files(base)
                r["rebuild_s"].append(round(time.perf_counter() - t0, 4))
                r["rebuild_cpu_s"].append(round(cpu_s() - c0, 3))
        for p in paths:
            r = out["paths"][p]
            r["encode_GiB_s"] = round(args.gib / min(r["encode_s"]), 3)
            r["rebuild_GiB_s"] = round(args.gib / min(r["rebuild_s"]), 3)
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
