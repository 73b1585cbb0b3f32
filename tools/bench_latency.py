"""Per-call latency of the drop-in host API (hec_rs_encode / hec_rs_reconstruct).

helyim calls ReedSolomon::encode once per 10 x 256 KiB buffer of a row and
reconstruct once per needle interval
(helyim-ec/src/encoder.rs:208-209,288; helyim-store/src/erasure_coding/mod.rs:426),
so the per-call cost at those sizes is what a drop-in user sees. Times the
C-ABI calls with argument arrays prepared beforehand (what a Rust caller
pays), pinned staging on and off (hec_set_host_staging), beside the C oracle
on one thread. Outputs are checked against the oracle.
python tools/bench_latency.py [--reps 200]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--sizes", default="1024,4096,65536,262144,1048576,4194304")
    args = ap.parse_args()
    import helyim_amd as H
    from oracle import corc
    lib = H.lib
    rs = H.ReedSolomon(10, 4)
    crs = corc.CReedSolomon(10, 4)
    rng = np.random.default_rng(5)
    rows = []
    for L in [int(x) for x in args.sizes.split(",")]:
        reps = max(5, min(args.reps, int(args.reps * 262144 / L)))
        full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        crs.encode(full)
        sh = [f.copy() for f in full]
        for i in range(10, 14):
            sh[i][:] = 0
        ptrs = (ctypes.c_void_p * 14)(*[a.ctypes.data for a in sh])
        lens = (ctypes.c_size_t * 14)(*[L] * 14)
        erased = (0, 3, 7, 12)
        pres = (ctypes.c_uint8 * 14)(*[0 if i in erased else 1 for i in range(14)])
        rlens = (ctypes.c_size_t * 14)(*[0 if i in erased else L for i in range(14)])
        row = {"shard_len": L, "reps": reps}
        # staged_sync: completion through hipStreamSynchronize instead of the
        # kernel's own flag (hec_set_completion_signal(0))
        for mode, lim, sig in (("direct", 0, 1 << 20), ("staged_sync", 1 << 40, 0), ("staged", 1 << 40, 1 << 20)):
            lib.hec_set_host_staging(lim)
            lib.hec_set_completion_signal(sig)
            for _ in range(3):
                assert lib.hec_rs_encode(rs.handle, ptrs, lens, 14) == 0
            t0 = time.perf_counter()
            for _ in range(reps):
                lib.hec_rs_encode(rs.handle, ptrs, lens, 14)
            te = (time.perf_counter() - t0) / reps
            ok = all(np.array_equal(a, b) for a, b in zip(sh, full))
            for i in erased:
                sh[i][:] = 0
            for _ in range(3):
                assert lib.hec_rs_reconstruct(rs.handle, ptrs, rlens, pres, 14) == 0
            t0 = time.perf_counter()
            for _ in range(reps):
                lib.hec_rs_reconstruct(rs.handle, ptrs, rlens, pres, 14)
            tr = (time.perf_counter() - t0) / reps
            ok = ok and all(np.array_equal(a, b) for a, b in zip(sh, full))
            row[mode] = {"encode_us": round(te * 1e6, 1), "reconstruct_us": round(tr * 1e6, 1),
                         "encode_GiB_s": round(10 * L / te / 2**30, 2),
                         "reconstruct_GiB_s": round(10 * L / tr / 2**30, 2), "identical": bool(ok)}
        lib.hec_set_host_staging(16 << 20)
        lib.hec_set_completion_signal(1 << 20)
        cr = max(3, reps // 4)
        b = [f.copy() for f in full]
        t0 = time.perf_counter()
        for _ in range(cr):
            crs.encode(b)
        tce = (time.perf_counter() - t0) / cr
        pr = [i not in erased for i in range(14)]
        t0 = time.perf_counter()
        for _ in range(cr):
            crs.reconstruct(b, pr)
        tcr = (time.perf_counter() - t0) / cr
        row["cpu_1thread"] = {"encode_us": round(tce * 1e6, 1), "reconstruct_us": round(tcr * 1e6, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
