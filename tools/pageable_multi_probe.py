"""Host-batch rate on PAGEABLE memory, one call vs the same call split over a
repeated device list (the ranges of one _multi call used to share
one host worker pool, so all but one copied their staging serially; round 4
gives each device up to two pools). One GPU: the PCIe link is shared, so this
measures the host-side copy parallelism, not more bandwidth.

usage: python tools/pageable_multi_probe.py [--stripes 512] [--reps 3] [--rounds 3] [--single]
prints one JSON line per (round, device list); --single: the one-call row
only. The line names the library it loaded (HEC_LIB_PATH selects another
build, for alternating-process A/Bs on one box)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=512)
    ap.add_argument("--shard-len", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--single", action="store_true")
    ap.add_argument("--alternate", default="", help="env var libhec reads per call (e.g. HEC_STREAM_COPY): "
                    "each case runs with it =1 and =0, alternating in this process")
    args = ap.parse_args()
    import numpy as np
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    torch.cuda.set_device(0)
    S, L = args.stripes, args.shard_len
    rs = H.ReedSolomon(10, 4)
    t = torch.zeros((S, 14, L), dtype=torch.uint8)  # pageable
    t[:, :10] = torch.randint(0, 256, (S, 10, L), dtype=torch.uint8)
    masks = np.full(S, 0x3FFF & ~0b1001000010001, np.uint32)
    lists = {"single": None} if args.single else {"single": None, "[0,0]": [0, 0], "[0,0,0,0]": [0, 0, 0, 0]}
    lib_name = os.path.relpath(H._lib.LIB_PATH, ROOT)
    for name, devs in lists.items():  # warm-up: pipelines, pools, tables
        B.host_encode_batch(rs, t, devices=devs)
        B.host_reconstruct_batch(rs, t, masks, devices=devs)
    data = S * 10 * L
    settings = ["1", "0"] if args.alternate else [None]
    cases = [(name, devs, v) for name, devs in lists.items() for v in settings]
    for r in range(args.rounds):
        for name, devs, v in cases:
            if v is not None:
                os.environ[args.alternate] = v
            t0 = time.perf_counter()
            for _ in range(args.reps):
                B.host_encode_batch(rs, t, devices=devs)
            t1 = time.perf_counter()
            for _ in range(args.reps):
                B.host_reconstruct_batch(rs, t, masks, devices=devs)
            t2 = time.perf_counter()
            tag = {args.alternate: v} if v is not None else {}
            print(json.dumps({"lib": lib_name, **tag, "round": r, "devices": name, "memory": "pageable",
                              "stripes": S, "shard_len": L,
                              "encode_data_GiB_s": round(data * args.reps / (t1 - t0) / 2**30, 2),
                              "decode_data_GiB_s": round(data * args.reps / (t2 - t1) / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
