"""First-process effect on a fresh box: the first bench process of a gpurun
call measured ~3% slower than the next ones (profiles/r02/bench_repeat_final.jsonl).
This runs the bench step (encode + 4-erasure decode of 4096 x 1 MiB) for
--steps steps on one batch and prints per-block times, then frees the batch
back to the driver (torch.cuda.empty_cache), allocates a new one and repeats:
does the slowness fade with time, or follow the allocation?

python tools/warm_probe.py [--steps 60] [--block 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--allocs", type=int, default=2)
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    S, L = 4096, 1 << 20
    rs = H.ReedSolomon(10, 4)
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    st = torch.cuda.current_stream()
    t0 = time.time()
    for a in range(args.allocs):
        t = torch.empty((S, 14, L), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(t, 10 * L, 0x5EED0000)
        torch.cuda.synchronize()
        for blk in range(args.steps // args.block):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            enc = dec = 0.0
            for _ in range(args.block):
                e[0].record(st)
                B.encode_batch(rs, t)
                e[1].record(st)
                B.reconstruct_batch(rs, t, masks)
                e[2].record(st)
                torch.cuda.synchronize()
                enc += e[0].elapsed_time(e[1]) / args.block
                dec += e[1].elapsed_time(e[2]) / args.block
            print(json.dumps({"alloc": a, "block": blk, "t_s": round(time.time() - t0, 1), "enc_ms": round(enc, 3),
                              "dec_ms": round(dec, 3)}), flush=True)
        del t
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
