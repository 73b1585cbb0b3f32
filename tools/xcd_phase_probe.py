"""A/B of the XCD phase offset (hec_set_xcd_phase 0 / 1, alternating per
round in one process and one allocation) on the bench batch: 4096 x 1 MiB,
encode + 4-erasure decode, on the padded layout (shard stride L + 64 KiB,
the bench's) and on a packed view of the same allocation. Prints one JSON
line per (round, layout, phase) with the median of --reps launches.

python tools/xcd_phase_probe.py [--rounds 6] [--reps 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--phases", default="0,1")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    rs = H.ReedSolomon(10, 4)
    S, L, pad = args.stripes, 1 << 20, 64 << 10
    t = B.empty_stripes(S, 14, L, shard_pad=pad)
    B.fill_stripes_splitmix(t, 10, bench.rank_seed_base(0))
    packed = t.as_strided((S, 14, L), (14 * L, L, 1))  # same allocation, packed stride
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    st = torch.cuda.current_stream()
    nbytes = S * 14 * L
    for r in range(args.rounds):
        for layout, view in (("padded", t), ("packed", packed)):
            for ph in (int(x) for x in args.phases.split(",")):
                assert H.lib.hec_set_xcd_phase(ph) == 0
                B.encode_batch(rs, view)
                B.reconstruct_batch(rs, view, masks)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.reps + 1)]
                ev[0].record(st)
                for i in range(args.reps):
                    B.encode_batch(rs, view)
                    ev[2 * i + 1].record(st)
                    B.reconstruct_batch(rs, view, masks)
                    ev[2 * i + 2].record(st)
                torch.cuda.synchronize()
                enc = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.reps)]))
                dec = float(np.median([ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(args.reps)]))
                print(json.dumps({"round": r, "layout": layout, "xcd_phase": ph, "enc_ms": round(enc, 4),
                                  "dec_ms": round(dec, 4), "enc_frac": round(nbytes / enc / 1e6 / 8000, 4),
                                  "dec_frac": round(nbytes / dec / 1e6 / 8000, 4)}), flush=True)
    H.lib.hec_set_xcd_phase(0)


if __name__ == "__main__":
    main()
