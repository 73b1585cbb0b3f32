"""Decode rate vs erasure pattern on the BASELINE batch (4096 x 1 MiB,
device-resident): is the decode/encode gap the arithmetic or where the
erased shards sit? Same-pattern batches ({10..13} is an encode in disguise:
read data 0-9, write parity 10-13) against the bench's random 4-erasure
patterns, per launch configuration (vectors per lane: 1 = one 4 KiB chunk per
workgroup, 2 = the pair kernel), interleaved rounds in one process, with the
encode of the same batch as the reference line. HEC_LIB_PATH selects a
measurement build (Makefile VARIANTS).

python tools/decode_pattern_probe.py [--rounds 7] [--vecs 1,2]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--shard-len", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--vecs", default="1", help="16-byte vectors per lane (hec_set_launch_config)")
    ap.add_argument("--modes", default="0", help="0 = GF decode, 1 = its XOR-only twin (same traffic)")
    ap.add_argument("--decvecs", default="8", help="decode bytes per lane (hec_set_decode_vector_bytes)")
    ap.add_argument("--pad", type=int, default=64 << 10, help="gap after every shard (batch.empty_stripes)")
    ap.add_argument("--only", default="", help="comma list of patterns to run (default: all)")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    S, L = args.stripes, args.shard_len
    rs = H.ReedSolomon(10, 4)
    t = B.empty_stripes(S, 14, L, shard_pad=args.pad)
    B.fill_stripes_splitmix(t, 10, 0x5EED0000)
    B.encode_batch(rs, t)
    full = (1 << 14) - 1

    def fixed(drop):
        return np.full(S, full & ~sum(1 << i for i in drop), np.int32)

    pats = {"random4": bench.erasure_masks(S, 0), "p10-13": fixed((10, 11, 12, 13)),
            "d0-3": fixed((0, 1, 2, 3)), "d6-9": fixed((6, 7, 8, 9)), "0,5,10,13": fixed((0, 5, 10, 13)),
            "d0,d9,p10": fixed((0, 9, 10)), "one_d4": fixed((4,))}
    # the bench's patterns with stripes of one pattern adjacent (table reuse)
    pats["random4_sorted"] = np.sort(pats["random4"])
    if args.only:
        pats = {k: pats[k] for k in args.only.split(",")}
    rng = np.random.default_rng(0xE4)
    for e in (1, 2, 3):  # per-stripe random patterns with exactly e erasures
        if args.only and f"random{e}" not in args.only.split(","):
            continue
        pats[f"random{e}"] = np.array([full & ~int(sum(1 << int(i) for i in rng.choice(14, e, replace=False)))
                                       for _ in range(S)], np.int32)
    masks = {k: torch.from_numpy(v).cuda() for k, v in pats.items()}
    decs = [(int(v), int(m), int(dv)) for v in args.vecs.split(",") for m in args.modes.split(",")
            for dv in args.decvecs.split(",")]
    res = {}
    s = torch.cuda.current_stream()
    for _ in range(args.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        B.encode_batch(rs, t)
        e1.record(s)
        torch.cuda.synchronize()
        res.setdefault(("encode", (-1, 0, 0)), []).append(e0.elapsed_time(e1))
        for k, m in masks.items():
            for d in decs:
                B.set_launch_config(vec_per_thread=d[0])
                H.lib.hec_set_kernel_mode(d[1])
                H.lib.hec_set_decode_vector_bytes(d[2])
                e0.record(s)
                B.reconstruct_batch(rs, t, m)
                e1.record(s)
                torch.cuda.synchronize()
                res.setdefault((k, d), []).append(e0.elapsed_time(e1))
    B.set_launch_config()
    H.lib.hec_set_kernel_mode(0)
    H.lib.hec_set_decode_vector_bytes(8)
    for (k, d), v in res.items():
        e = {"d0,d9,p10": 3, "one_d4": 1, "random1": 1, "random2": 2, "random3": 3}.get(k, 4)
        nbytes = S * (10 + e) * L if k != "encode" else S * 14 * L
        ms = float(np.median(v))
        print(json.dumps({"pattern": k, "vec_per_thread": d[0], "mode": ["gf", "xor_only"][d[1]],
                          "dec_vec_bytes": d[2], "pad": args.pad, "lib": os.path.basename(H.LIB_PATH), "ms_med": round(ms, 3),
                          "GB_s": round(nbytes / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
