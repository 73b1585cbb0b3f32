"""Host-path (zero-copy, pinned) encode: which kernel reads host memory over
PCIe fastest? Alternating in one process over one pinned 512 x 1 MiB batch:
the bit-sliced encode (default; 8 KiB column range per workgroup), the table
encode at 16 B per lane (4 KiB) and at 8 B per lane (2 KiB, the decode's
width). The library's host-batch override (hec_set_host_encode_narrow) is
off while the probe runs, so each variant is the kernel the global knobs
pick. One JSON line per (round, kernel).

python tools/e2e_encode_kernel_probe.py [--rounds 3] [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    torch.cuda.set_device(0)
    S, L = 512, 1 << 20
    rs = H.ReedSolomon(10, 4)
    buf = H.HostBuffer(S * 14 * L)
    t = buf.tensor((S, 14, L))
    dev = torch.empty((S, 14, L), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev, 10 * L, bench.rank_seed_base(0))
    t.copy_(dev)
    del dev
    lib = H.lib
    variants = {"bitslice": (1, 16), "table16": (0, 16), "table8": (0, 8)}
    ref = None
    lib.hec_set_host_encode_narrow(0)
    try:
        for r in range(args.rounds):
            for name, (kind, vb) in variants.items():
                lib.hec_set_encode_kernel(kind)
                lib.hec_set_encode_vector_bytes(vb)
                B.host_encode_batch(rs, t)  # warm
                t0 = time.perf_counter()
                for _ in range(args.reps):
                    B.host_encode_batch(rs, t)
                dt = (time.perf_counter() - t0) / args.reps
                par = t[:4, 10:].clone()
                ref = par if ref is None else ref
                print(json.dumps({"round": r, "kernel": name, "kernel_name": lib.hec_host_encode_kernel_name(L).decode(),
                                  "encode_data_GiB_s": round(S * 10 * L / dt / 2**30, 2),
                                  "same_parity": bool(torch.equal(par, ref))}), flush=True)
    finally:
        lib.hec_set_encode_kernel(1)
        lib.hec_set_encode_vector_bytes(16)
        lib.hec_set_host_encode_narrow(1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
