"""Same-process timing of the shipped RS(10,4) device kernels on the BASELINE
config (4096 x 1 MiB stripes, 64 KiB shard gap, 4 random erasures per
stripe, device-resident), over interleaved rounds (cdna_hip_programming.md
§5.4 rule 24): one JSON line with the median / min ms per launch, TB/s of
algorithmic bytes and every round's sample; checks the batch is intact.

Kernel choice has no runtime knob since round 6: an A/B of two
kernel builds runs each build's library through HEC_LIB_PATH in alternating
processes on one lease, e.g.
    for i in 1 2 3; do HEC_LIB_PATH=a.so python tools/tune.py; HEC_LIB_PATH=b.so python tools/tune.py; done
(the round-6 32-byte-per-lane decode experiment ran in one process while it
was still a knob: profiles/r06/decode_wide_32B_vs_8B_*.jsonl).

python tools/tune.py [--stripes 4096] [--rounds 7]
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
    ap.add_argument("--pad", type=int, default=64 << 10, help="extra bytes after each shard (the bench's layout)")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    S, L = args.stripes, args.shard_len
    rs = H.ReedSolomon(10, 4)
    t = B.empty_stripes(S, 14, L, shard_pad=args.pad)
    B.fill_stripes_splitmix(t, 10, 0x5EED0000)
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    B.encode_batch(rs, t)
    torch.cuda.synchronize()
    good = t[:8].clone()
    enc, dec = [], []
    s = torch.cuda.current_stream()
    for _ in range(args.rounds):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s)
        B.encode_batch(rs, t)
        e1.record(s)
        B.reconstruct_batch(rs, t, masks)
        e2.record(s)
        torch.cuda.synchronize()
        enc.append(e0.elapsed_time(e1))
        dec.append(e1.elapsed_time(e2))
    enc, dec = np.array(enc), np.array(dec)
    nbytes = S * 14 * L  # algorithmic bytes of either launch (4 erasures: 10 reads + 4 writes)
    print(json.dumps({"lib": os.path.basename(H.LIB_PATH), "encode_kernel": H.lib.hec_encode_kernel_name(L).decode(),
                      "decode_kernel": H.lib.hec_decode_kernel_name(L).decode(), "stripes": S, "shard_len": L,
                      "pad": args.pad, "rounds": args.rounds,
                      "enc_ms_med": round(float(np.median(enc)), 4), "enc_ms_min": round(float(enc.min()), 4),
                      "dec_ms_med": round(float(np.median(dec)), 4), "dec_ms_min": round(float(dec.min()), 4),
                      "enc_TBps": round(nbytes / np.median(enc) / 1e9, 3),
                      "dec_TBps": round(nbytes / np.median(dec) / 1e9, 3),
                      "dec_over_enc_med": round(float(np.median(dec / enc)), 4),
                      "enc_ms": [round(x, 4) for x in enc.tolist()],
                      "dec_ms": [round(x, 4) for x in dec.tolist()]}), flush=True)
    assert torch.equal(t[:8], good), "batch changed across the rounds"


if __name__ == "__main__":
    main()
