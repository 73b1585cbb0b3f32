"""Same-process A/B of the RS(10,4) device kernels on the BASELINE config
(4096 x 1 MiB stripes, 64 KiB shard gap, 4 random erasures per stripe,
device-resident). Configurations alternate round by round in one process
(cdna_hip_programming.md §5.4 rule 24), so every arm sees the same
allocation; prints one JSON line per configuration (median / min ms, TB/s
of algorithmic bytes, every round's sample) and checks the batch is intact.

Today's only speed knob is the decode width (hec_set_decode_vector_bytes:
8 = shipped, 16, 32 = the round-6 experiment):

python tools/tune.py [--stripes 4096] [--rounds 7] [--decvecs 8,32]
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
    ap.add_argument("--decvecs", default="8,32", help="decode bytes per lane, alternated (8 shipped, 16, 32)")
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
    dvs = [int(x) for x in args.decvecs.split(",")]
    res = {dv: {"enc": [], "dec": []} for dv in dvs}
    names = {}
    s = torch.cuda.current_stream()
    try:
        for rnd in range(args.rounds):
            for dv in (dvs if rnd % 2 == 0 else dvs[::-1]):  # alternate the order round by round
                assert H.lib.hec_set_decode_vector_bytes(dv) == 0
                names[dv] = H.lib.hec_decode_kernel_name(L).decode()
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(s)
                B.encode_batch(rs, t)
                e1.record(s)
                B.reconstruct_batch(rs, t, masks)
                e2.record(s)
                torch.cuda.synchronize()
                res[dv]["enc"].append(e0.elapsed_time(e1))
                res[dv]["dec"].append(e1.elapsed_time(e2))
    finally:
        H.lib.hec_set_decode_vector_bytes(8)
    nbytes = S * 14 * L  # algorithmic bytes of either launch (4 erasures: 10 reads + 4 writes)
    for dv in dvs:
        enc, dec = np.array(res[dv]["enc"]), np.array(res[dv]["dec"])
        print(json.dumps({"dec_vec_bytes": dv, "decode_kernel": names[dv], "stripes": S, "shard_len": L,
                          "pad": args.pad, "rounds": args.rounds,
                          "enc_ms_med": round(float(np.median(enc)), 4), "enc_ms_min": round(float(enc.min()), 4),
                          "dec_ms_med": round(float(np.median(dec)), 4), "dec_ms_min": round(float(dec.min()), 4),
                          "enc_TBps": round(nbytes / np.median(enc) / 1e9, 3),
                          "dec_TBps": round(nbytes / np.median(dec) / 1e9, 3),
                          "dec_over_enc_med": round(float(np.median(dec / enc)), 4),
                          "enc_ms": [round(x, 4) for x in enc.tolist()],
                          "dec_ms": [round(x, 4) for x in dec.tolist()]}), flush=True)
    assert torch.equal(t[:8], good), "batch changed across the A/B"


if __name__ == "__main__":
    main()
