"""Degraded-read reconstruct throughput.

helyim reconstructs one needle interval per ReedSolomon::reconstruct call
(helyim-store/src/erasure_coding/mod.rs:403-491). This measures N such
intervals (lengths log-uniform 1 KiB..256 KiB, 1..4 erasures, at least one
data shard erased) three ways on the same inputs, outputs compared:
  cpu_loop   -- the C restatement of the CPU path, one call per interval, 1 thread
  gpu_loop   -- libhec's drop-in hec_rs_reconstruct, one call per interval
  gpu_batch  -- hec_rs_reconstruct_batch: all intervals in one GPU round trip
                (C-ABI leg: median of --reps calls; one call is noisy: 0.05-0.09 s)
python tools/bench_intervals.py [--n 4096]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def c_abi_call(H, rs, fulls, erased, n_s, reps=1):
    """hec_rs_reconstruct_batch alone, its argument arrays prepared beforehand
    (what a Rust caller pays); returns (outputs identical, [seconds per call])."""
    import ctypes
    outs = [[np.zeros_like(f[i]) if i in e else f[i] for i in range(14)] for f, e in zip(fulls, erased)]
    ptrs = (ctypes.c_void_p * (14 * n_s))(*[b.ctypes.data for st_ in outs for b in st_])
    lens_c = (ctypes.c_size_t * (14 * n_s))(*[0 if i in e else st_[i].size for st_, e in zip(outs, erased)
                                              for i in range(14)])
    pres = (ctypes.c_uint8 * (14 * n_s))(*[0 if i in e else 1 for e in erased for i in range(14)])
    bad = ctypes.c_size_t(0)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = H.lib.hec_rs_reconstruct_batch(rs.handle, ptrs, lens_c, pres, n_s, 0, ctypes.byref(bad))
        ts.append(time.perf_counter() - t0)
        assert rc == 0
    ok_c = all(np.array_equal(o[i], f[i]) for o, f in zip(outs, fulls) for i in range(14))
    return ok_c, ts


def c_abi_leg(H, rs, fulls, erased, payload, args, out):
    ok, ts = c_abi_call(H, rs, fulls, erased, args.n, args.reps)
    med = float(np.median(ts))
    out["gpu_batch_c_abi"] = {"first_s": round(ts[0], 4), "median_s": round(med, 4), "reps": len(ts),
                              "intervals_per_s": round(args.n / med, 1), "payload_GiB_s": round(payload / med / 2**30, 3)}
    out["identical_outputs"] = bool(ok)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5, help="timed C-ABI calls (the median is reported)")
    ap.add_argument("--c-abi-only", action="store_true", help="skip the CPU, per-call and Python legs")
    args = ap.parse_args()
    import helyim_amd as H
    from oracle import corc
    rng = np.random.default_rng(42)
    crs = corc.CReedSolomon(10, 4)
    rs = H.ReedSolomon(10, 4)
    lens = np.exp(rng.uniform(np.log(1024), np.log(256 * 1024), args.n)).astype(int)
    fulls, erased = [], []
    for L in lens:
        d = [rng.integers(0, 256, int(L), dtype=np.uint8) for _ in range(10)]
        full = d + [np.zeros(int(L), np.uint8) for _ in range(4)]
        crs.encode(full)
        e = [int(rng.integers(0, 10))]
        others = [i for i in range(14) if i != e[0]]
        e += rng.choice(others, int(rng.integers(0, 4)), replace=False).tolist()
        fulls.append(full)
        erased.append(set(e))
    payload = float(sum(lens)) * 10

    def fresh():
        return [[None if i in e else f[i] for i in range(14)] for f, e in zip(fulls, erased)]

    out = {"n_intervals": args.n, "len_range": "1 KiB..256 KiB log-uniform", "erasures": "1..4 (>= 1 data)",
           "payload_GiB": round(payload / 2**30, 3)}
    if args.c_abi_only:
        return c_abi_leg(H, rs, fulls, erased, payload, args, out)
    # CPU oracle loop
    bufs = [[f[i].copy() if i not in e else np.zeros_like(f[i]) for i in range(14)] for f, e in zip(fulls, erased)]
    t0 = time.perf_counter()
    for b, e in zip(bufs, erased):
        crs.reconstruct(b, [i not in e for i in range(14)])
    t_cpu = time.perf_counter() - t0
    # GPU drop-in, one call per interval
    st = fresh()
    rs.reconstruct(st[0])  # warm-up
    st = fresh()
    t0 = time.perf_counter()
    for s in st:
        rs.reconstruct(s)
    t_loop = time.perf_counter() - t0
    # GPU batch through the Python mirror (includes building 14*N ctypes pointers)
    sb = fresh()
    rs.reconstruct_batch(sb)  # warm-up (staging, tables)
    sb = fresh()
    t0 = time.perf_counter()
    rs.reconstruct_batch(sb)
    t_batch = time.perf_counter() - t0
    ok_c, t_c = c_abi_call(H, rs, fulls, erased, args.n, args.reps)
    ok = all(np.array_equal(a[i], f[i]) and np.array_equal(b[i], f[i]) and np.array_equal(c[i], f[i])
             for a, b, c, f in zip(bufs, st, sb, fulls) for i in range(14))
    for name, t in (("cpu_loop", t_cpu), ("gpu_loop", t_loop), ("gpu_batch_python", t_batch),
                    ("gpu_batch_c_abi", float(np.median(t_c)))):
        out[name] = {"s": round(t, 4), "intervals_per_s": round(args.n / t, 1),
                     "payload_GiB_s": round(payload / t / 2**30, 3)}
    out["identical_outputs"] = bool(ok and ok_c)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
