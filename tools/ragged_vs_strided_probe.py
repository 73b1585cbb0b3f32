"""The bench batch (4096 x 1 MiB, 4 erasures per stripe) through the strided
kernels (XCD eighths remap on / off) and through the ragged kernels (one
descriptor per stripe, the same bytes), interleaved in one process and one
allocation, at shard gaps --pads. Prints encode / decode ms per variant.

python tools/ragged_vs_strided_probe.py [--pads 0,65536] [--rounds 5]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pads", default="0,65536")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096)
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    rs = H.ReedSolomon(10, 4)
    S, L = args.stripes, 1 << 20
    pads = [int(x) for x in args.pads.split(",")]
    masks_np = bench.erasure_masks(S, 0)
    masks = torch.from_numpy(masks_np).cuda()
    buf = torch.empty(S * 14 * (L + max(pads)), dtype=torch.uint8, device="cuda")
    views, descs = {}, {}
    for p in pads:
        views[p] = buf.as_strided((S, 14, L), (14 * (L + p), L + p, 1))
        # a desc_dtype array goes to the C ABI as is (a list would be converted
        # inside the timed region, on the host, while the GPU idles)
        descs[p] = np.array([(s * 14 * (L + p), L + p, L, int(masks_np[s])) for s in range(S)],
                            dtype=B.desc_dtype())
    B.fill_stripes_splitmix(views[pads[0]], 10, 0x5EED0000)
    st = torch.cuda.current_stream()
    variants = ["strided_remap1", "strided_remap0", "ragged"]
    res = {(p, v): [[], []] for p in pads for v in variants}
    for _ in range(args.rounds):
        for p in pads:
            for v in variants:
                B.set_launch_config(xcd_remap=0 if v == "strided_remap0" else 1)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                enc = dec = 0.0
                for _ in range(args.reps):
                    e[0].record(st)
                    if v == "ragged":
                        B.encode_ragged(rs, buf, descs[p])
                    else:
                        B.encode_batch(rs, views[p])
                    e[1].record(st)
                    if v == "ragged":
                        B.reconstruct_ragged(rs, buf, descs[p])
                    else:
                        B.reconstruct_batch(rs, views[p], masks)
                    e[2].record(st)
                    torch.cuda.synchronize()
                    enc += e[0].elapsed_time(e[1]) / args.reps
                    dec += e[1].elapsed_time(e[2]) / args.reps
                res[p, v][0].append(enc)
                res[p, v][1].append(dec)
    B.set_launch_config()
    for (p, v), (enc, dec) in res.items():
        print(json.dumps({"pad": p, "variant": v, "enc_ms_med": round(float(np.median(enc)), 3),
                          "dec_ms_med": round(float(np.median(dec)), 3)}), flush=True)


if __name__ == "__main__":
    main()
