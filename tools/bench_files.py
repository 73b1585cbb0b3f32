"""File-level drop-in throughput: helyim_ec::write_ec_files / rebuild_ec_files
on the GPU (libhec) vs the C restatement of helyim-ec's CPU path
(oracle/rs_oracle.c: 256 KiB batches, AVX2 nibble-pshufb, one thread), on the
same .dat, with byte-identical outputs checked.

Config 0 of BASELINE.json (30,000,000-byte synthetic volume, drop 4 shards,
rebuild) plus a larger volume (default 8 GiB: 0 large rows + 820 small rows;
use --gib 12 to get one 1 GiB large row). Files live in --dir (default
/dev/shm when it has room, so the page cache, not a disk, is measured).
Encodes are timed on fresh shard files (the CPU run's case); the GPU encode is
also timed over existing files (gpu_encode_overwrite_s).

python tools/bench_files.py [--gib 8] [--dir /dev/shm/hec]
"""
import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        while True:
            b = f.read(1 << 24)
            if not b:
                return h.hexdigest()
            h.update(b)


def make_volume(path, nbytes, exact30=False):
    import numpy as np
    if exact30:
        from oracle import rs_oracle as O
        with open(path, "wb") as f:
            f.write(O.synthetic_volume(nbytes).tobytes())
        return
    import torch
    import helyim_amd.batch as B
    chunk = 1 << 30
    with open(path, "wb") as f:
        left, k = nbytes, 0
        while left > 0:
            n = min(chunk, left)
            t = torch.empty((1, 1, n), dtype=torch.uint8, device="cuda")
            B.fill_splitmix(t, n, 0x5EEDF11E + k)
            f.write(t.cpu().numpy().tobytes())
            left -= n
            k += 1
    del np


def run_case(workdir, nbytes, exact30, drops=(0, 5, 10, 13)):
    import helyim_amd as H
    from oracle import corc
    g, c = os.path.join(workdir, "gpu"), os.path.join(workdir, "cpu")
    make_volume(g + ".dat", nbytes, exact30)
    shutil.copyfile(g + ".dat", c + ".dat")
    res = {"dat_bytes": nbytes}
    H.write_ec_files(g)  # warm-up: device tables, pinned staging
    for i in range(14):  # timed on fresh shard files, as the CPU run below
        os.remove(g + H.to_ext(i))
    t0 = time.perf_counter()
    H.write_ec_files(g)
    res["gpu_encode_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()  # again over the existing files (create + truncate frees their pages)
    H.write_ec_files(g)
    res["gpu_encode_overwrite_s"] = round(time.perf_counter() - t0, 4)
    t0 = time.perf_counter()
    assert corc.write_ec_files(c) == 0
    res["cpu_encode_s"] = time.perf_counter() - t0
    same = all(sha(g + H.to_ext(i)) == sha(c + H.to_ext(i)) for i in range(14))
    for base in (g, c):
        for i in drops:
            os.remove(base + H.to_ext(i))
    t0 = time.perf_counter()
    ids = H.rebuild_ec_files(g)
    res["gpu_rebuild_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    rc, cids = corc.rebuild_ec_files(c)
    res["cpu_rebuild_s"] = time.perf_counter() - t0
    assert rc == 0 and ids == cids == sorted(drops)
    same &= all(sha(g + H.to_ext(i)) == sha(c + H.to_ext(i)) for i in range(14))
    res["identical_outputs"] = bool(same)
    gib = nbytes / 2**30
    for k in ("gpu_encode", "cpu_encode", "gpu_rebuild", "cpu_rebuild"):
        res[k + "_GiB_s"] = round(gib / res[k + "_s"], 3)
        res[k + "_s"] = round(res[k + "_s"], 4)
    res["shard_sha256"] = [sha(g + H.to_ext(i)) for i in range(14)] if exact30 else None
    for f in os.listdir(workdir):
        os.remove(os.path.join(workdir, f))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()
    d = args.dir
    if d is None:
        shm = "/dev/shm"
        need = args.gib * 2**30 * 2.6
        d = tempfile.mkdtemp(prefix="hec_files_", dir=shm if os.path.isdir(shm) and
                             shutil.disk_usage(shm).free > need else None)
    os.makedirs(d, exist_ok=True)
    try:
        out = {"dir": d, "cpu_model": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
               "cpu_threads_used": 1, "gpu_io_threads": 16}
        r30 = run_case(d, 30_000_000, True)
        golden = json.load(open(os.path.join(ROOT, "tests", "golden", "volume_30mb.json")))
        r30["matches_fixture"] = r30.pop("shard_sha256") == golden["shard_sha256"]
        out["config0_30MB"] = r30
        if args.gib > 0:
            rb = run_case(d, int(args.gib * 2**30), False)
            rb.pop("shard_sha256")
            out[f"volume_{args.gib:g}GiB"] = rb
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
