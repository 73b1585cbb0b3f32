"""Layouts compared inside ONE allocation (so HBM placement, which moves the
step time by +-2-3% between allocations, is held fixed): the bench batch
viewed with shard stride 1 MiB + pad (and stripe stride 14 x that, plus an
optional extra stripe pad: "--pads 65536:131072") over the same buffer, encode + 4-erasure decode, interleaved rounds; repeated over
--allocs fresh allocations.

python tools/layout_in_alloc_probe.py [--allocs 3] [--pads 0,4096,65536,262144] [--rounds 4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=3)
    ap.add_argument("--pads", default="0,4096,65536,262144")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import helyim_amd.batch as B
    import helyim_amd as H
    import bench
    S, L = 4096, 1 << 20
    pads = [x for x in args.pads.split(",")]

    def strides(p):
        sp, _, qp = p.partition(":")
        shard = L + int(sp)
        return shard, 14 * shard + int(qp or 0)

    rs = H.ReedSolomon(10, 4)
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    st = torch.cuda.current_stream()
    for a in range(args.allocs):
        buf = torch.empty(S * max(strides(p)[1] for p in pads), dtype=torch.uint8, device="cuda")
        views = {p: buf.as_strided((S, 14, L), (strides(p)[1], strides(p)[0], 1)) for p in pads}
        res = {p: [[], []] for p in pads}
        for r in range(args.rounds):
            for p in pads:
                t = views[p]
                B.fill_splitmix(t, 10 * L, 0x5EED0000) if r == 0 else None
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                enc = dec = 0.0
                for _ in range(args.steps):
                    e[0].record(st)
                    B.encode_batch(rs, t)
                    e[1].record(st)
                    B.reconstruct_batch(rs, t, masks)
                    e[2].record(st)
                    torch.cuda.synchronize()
                    enc += e[0].elapsed_time(e[1]) / args.steps
                    dec += e[1].elapsed_time(e[2]) / args.steps
                res[p][0].append(enc)
                res[p][1].append(dec)
        for p in pads:
            enc, dec = sorted(res[p][0]), sorted(res[p][1])
            print(json.dumps({"alloc": a, "pad": p if ":" in p else int(p), "enc_ms_med": round(enc[len(enc) // 2], 3),
                              "dec_ms_med": round(dec[len(dec) // 2], 3)}), flush=True)
        del buf, views
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
