"""Launch-configuration sweep for the RS(10,4) kernels on the BASELINE config
(4096 x 1 MiB stripes, device-resident). Interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24); prints one JSON line per config with
the median/min encode and decode ms and HBM GB/s, plus the XOR-only ceiling.

python tools/tune.py [--stripes 4096] [--rounds 5]
"""
import argparse
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--shard-len", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--vecs", default="1,2,4")
    ap.add_argument("--blocks", default="0,2048,4096,8192")
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--remaps", default="1")
    ap.add_argument("--bpcs", default="0", help="blocks-per-CU caps (0 = none)")
    ap.add_argument("--parts", default="1", help="regions per XCD (xcd_remap 1)")
    ap.add_argument("--rots", default="0", help="hashed per-stripe chunk rotation (0/1)")
    ap.add_argument("--wgs", default="256", help="RS(10,4) workgroup sizes (256/512/1024)")
    ap.add_argument("--encs", default="0", help="encode kernel: 0 table lookup, 1 bit-sliced")
    ap.add_argument("--decvecs", default="8", help="decode bytes per lane (8 default, 16, 4)")
    ap.add_argument("--encvecs", default="16", help="table-encode bytes per lane (16 default, 8, 4)")
    ap.add_argument("--bsvecs", default="16", help="bit-sliced encode load/store bytes per lane (16 default, 8)")
    ap.add_argument("--pad", type=int, default=64 << 10,
                    help="extra bytes between shards (default: the bench's batch.SHARD_PAD)")
    ap.add_argument("--stripe-pad", type=int, default=0, help="extra bytes between stripes (shards stay 1 MiB apart)")
    ap.add_argument("--tile", type=int, default=0,
                    help="interleaved layout: every shard split in tiles of this many bytes, the 14 "
                         "tiles of one column range stored together ([S*L/tile][14][tile])")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    S, L = args.stripes, args.shard_len
    mask_np = bench.erasure_masks(S, 0)
    if args.tile:
        rep = L // args.tile
        S, L = S * rep, args.tile
        mask_np = np.repeat(mask_np, rep)
    rs = H.ReedSolomon(10, 4)
    if args.stripe_pad:
        t = torch.empty((S, 14 * L + args.stripe_pad), dtype=torch.uint8, device="cuda")[:, :14 * L].view(S, 14, L)
    else:
        t = B.empty_stripes(S, 14, L, shard_pad=args.pad)
    B.fill_stripes_splitmix(t, 10, 0x5EED0000)
    masks = torch.from_numpy(mask_np).cuda()
    B.encode_batch(rs, t)
    torch.cuda.synchronize()
    good = t[:8].clone()
    ints = lambda x: [int(y) for y in x.split(",")]
    configs = list(itertools.product(ints(args.modes), ints(args.vecs), ints(args.blocks), ints(args.remaps),
                                     ints(args.bpcs), ints(args.parts), ints(args.rots), ints(args.wgs),
                                     ints(args.encs), ints(args.decvecs), ints(args.encvecs), ints(args.bsvecs)))
    res = {c: {"enc": [], "dec": []} for c in configs}
    s = torch.cuda.current_stream()
    for _ in range(args.rounds):
        for c in configs:
            mode, v, b, rm, bpc, parts, rot, wg, enc, dv, ev, bv = c
            H.lib.hec_set_encode_kernel(enc)
            H.lib.hec_set_bitslice_vector_bytes(bv)
            H.lib.hec_set_decode_vector_bytes(dv)
            H.lib.hec_set_encode_vector_bytes(ev)
            H.lib.hec_set_kernel_mode(mode)
            H.lib.hec_set_workgroup_size(wg)
            H.lib.hec_set_xcd_parts(parts)
            H.lib.hec_set_chunk_rotation(rot)
            B.set_launch_config(v, b, rm, bpc)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(s)
            B.encode_batch(rs, t)
            e1.record(s)
            B.reconstruct_batch(rs, t, masks)
            e2.record(s)
            torch.cuda.synchronize()
            res[c]["enc"].append(e0.elapsed_time(e1))
            res[c]["dec"].append(e1.elapsed_time(e2))
    H.lib.hec_set_kernel_mode(0)
    H.lib.hec_set_encode_kernel(1)
    H.lib.hec_set_xcd_parts(1)
    H.lib.hec_set_chunk_rotation(0)
    H.lib.hec_set_workgroup_size(256)
    H.lib.hec_set_decode_vector_bytes(8)
    H.lib.hec_set_encode_vector_bytes(16)
    H.lib.hec_set_bitslice_vector_bytes(16)
    B.set_launch_config()
    nbytes = S * 14 * L
    for c in configs:
        enc, dec = np.array(res[c]["enc"]), np.array(res[c]["dec"])
        print(json.dumps({"lib": os.path.basename(H.LIB_PATH), "pad": args.pad, "stripe_pad": args.stripe_pad,
                          "tile": args.tile,
                          "mode": ["gf", "xor_ceiling"][c[0]], "vec_per_thread": c[1], "max_blocks": c[2],
                          "xcd_remap": c[3], "blocks_per_cu": c[4], "xcd_parts": c[5], "chunk_rot": c[6], "wg_threads": c[7], "encode_kernel": ["table", "bitslice"][c[8]], "dec_vec_bytes": c[9], "enc_vec_bytes": c[10], "bs_vec_bytes": c[11],
                          "enc_ms_med": round(float(np.median(enc)), 3), "enc_ms_min": round(float(enc.min()), 3),
                          "enc_GBps": round(nbytes / np.median(enc) / 1e6, 1),
                          "dec_ms_med": round(float(np.median(dec)), 3),
                          "dec_GBps": round(nbytes / np.median(dec) / 1e6, 1)}), flush=True)
    # the XOR-only rows scribbled over data shards through decode: regenerate
    B.fill_stripes_splitmix(t, 10, 0x5EED0000)
    B.encode_batch(rs, t)
    torch.cuda.synchronize()
    if not args.stripe_pad:
        assert torch.equal(t[:8], good)


if __name__ == "__main__":
    main()
