"""Does the HBM layout of a uniform batch matter beyond the 64 KiB shard gap?
4096 stripes x 1 MiB, 4 erasures each (the bench batch's work), through the
ragged kernels, whose descriptors can place every stripe anywhere, over ONE
allocation, layouts alternating per round:
  packed     shard spacing 1 MiB, stripes back to back (the strided packed batch)
  pad64k     shard spacing 1 MiB + 64 KiB (the bench's layout)
  randpad    shard spacing 1 MiB + 64 KiB * k, k uniform 0..7 per stripe
  shuffled   packed spacing, stripes placed in a random order
  lenmix     (reference) the config-5 probe saw 64 KiB..4 MiB stripes decode faster
Prints one JSON line per (round, layout): encode / decode ms, TB/s.

python tools/layout_ragged_probe.py [--rounds 5] [--reps 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--layouts", default="packed,pad64k,randpad,shuffled")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    rs = H.ReedSolomon(10, 4)
    S, L, G = args.stripes, 1 << 20, 64 << 10
    masks = bench.erasure_masks(S, 0)
    rng = np.random.default_rng(77)

    def lay(name):
        if name == "packed":
            return [(s * 14 * L, L, L, int(masks[s])) for s in range(S)]
        if name == "pad64k":
            return [(s * 14 * (L + G), L + G, L, int(masks[s])) for s in range(S)]
        if name == "randpad":
            out, off = [], 0
            for s in range(S):
                st = L + G * int(rng.integers(0, 8))
                out.append((off, st, L, int(masks[s])))
                off += 14 * st
            return out
        if name == "shuffled":
            slot = rng.permutation(S)
            return [(int(slot[s]) * 14 * L, L, L, int(masks[s])) for s in range(S)]
        raise ValueError(name)

    names = args.layouts.split(",")
    lays = {n: lay(n) for n in names}
    size = max(d[0] + 14 * d[1] for n in names for d in lays[n])
    dev = torch.empty(size, dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev.view(1, -1), size, 0x5EED0000)  # any bytes: timing only
    darr = {n: np.array(lays[n], dtype=B.desc_dtype()) for n in names}
    nbytes = S * 14 * L
    st = torch.cuda.current_stream()
    for r in range(args.rounds):
        for n in names:
            B.encode_ragged(rs, dev, darr[n])
            B.reconstruct_ragged(rs, dev, darr[n])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.reps + 1)]
            ev[0].record(st)
            for i in range(args.reps):
                B.encode_ragged(rs, dev, darr[n])
                ev[2 * i + 1].record(st)
                B.reconstruct_ragged(rs, dev, darr[n])
                ev[2 * i + 2].record(st)
            torch.cuda.synchronize()
            enc = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.reps)]))
            dec = float(np.median([ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(args.reps)]))
            print(json.dumps({"round": r, "layout": n, "enc_ms": round(enc, 4), "dec_ms": round(dec, 4),
                              "enc_TBps": round(nbytes / enc / 1e9, 3), "dec_TBps": round(nbytes / dec / 1e9, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
