"""Per-call drop-in throughput under concurrency (SURVEY §8b Threading: the
volume server reconstructs needle intervals from many tokio tasks at once).
T threads each loop hec_rs_reconstruct / hec_rs_encode on their own 4 KiB (or
--len) shards with C arguments prepared beforehand (ctypes releases the GIL
around the call), for --seconds; prints calls/s per T beside the C
restatement run the same way. Outputs are checked once per thread.

python tools/concurrency_probe.py [--threads 1,2,4,8,16] [--len 4096] [--seconds 2]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--len", type=int, default=4096)
    ap.add_argument("--seconds", type=float, default=2.0)
    args = ap.parse_args()
    import helyim_amd as H
    from oracle import corc
    lib = H.lib
    rs = H.ReedSolomon(10, 4)
    L = args.len
    erased = (0, 3, 7, 12)

    def make(seed):
        rng = np.random.default_rng(seed)
        full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        corc.CReedSolomon(10, 4).encode(full)
        sh = [f.copy() for f in full]
        return {
            "full": full, "sh": sh,
            "ptrs": (ctypes.c_void_p * 14)(*[a.ctypes.data for a in sh]),
            "lens": (ctypes.c_size_t * 14)(*[L] * 14),
            "pres": (ctypes.c_uint8 * 14)(*[0 if i in erased else 1 for i in range(14)]),
            "rlens": (ctypes.c_size_t * 14)(*[0 if i in erased else L for i in range(14)]),
        }

    for T in [int(x) for x in args.threads.split(",")]:
        row = {"threads": T, "len": L}
        for op in ("reconstruct", "encode", "cpu_reconstruct"):
            ctx = [make(1000 + t) for t in range(T)]
            counts = [0] * T
            bad = []
            stop = time.perf_counter() + args.seconds
            crs = corc.CReedSolomon(10, 4)

            def work(t):
                c = ctx[t]
                n = 0
                pr = [i not in erased for i in range(14)]
                while time.perf_counter() < stop:
                    if op == "reconstruct":
                        rc = lib.hec_rs_reconstruct(rs.handle, c["ptrs"], c["rlens"], c["pres"], 14)
                    elif op == "encode":
                        rc = lib.hec_rs_encode(rs.handle, c["ptrs"], c["lens"], 14)
                    else:
                        crs.reconstruct(c["sh"], pr)
                        rc = 0
                    if rc:
                        bad.append(rc)
                        return
                    n += 1
                counts[t] = n
                if not all(np.array_equal(a, b) for a, b in zip(c["sh"], c["full"])):
                    bad.append("mismatch")

            th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            dt = time.perf_counter() - t0
            row[op + "_calls_per_s"] = round(sum(counts) / dt)
            row[op + "_ok"] = not bad
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
