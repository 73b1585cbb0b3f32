"""Device-resident mixed workload (BASELINE config 5, as bench.py's
mixed_section): 512 stripes of 64 KiB..4 MiB shards, 0..4 erasures, one
ragged encode + one ragged reconstruct per rep. Prints the data-payload
GiB/s per round and the per-launch split (HIP events) so host gaps between
launches show up: gap = wall per rep - encode - reconstruct. HEC_LIB_PATH
selects a measurement build.

python tools/mixed_probe.py [--rounds 5] [--reps 5] [--pads 0,65536]

--pads: shard gaps compared inside ONE allocation (the layouts take turns
each round), as tools/layout_in_alloc_probe.py does for the bench batch.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=512)
    ap.add_argument("--grouped", action="store_true",
                    help="also time the same stripes as one strided batch per shard length (7 encode + 7 "
                         "reconstruct launches): the ceiling a length-grouped ragged launch could reach")
    ap.add_argument("--uniform", type=int, default=0,
                    help="E > 0: every stripe 1 MiB with exactly E random erasures (the bench batch through "
                         "the ragged kernels; compare with the strided kernels' times)")
    ap.add_argument("--fixed-len", type=int, default=0,
                    help="> 0: every stripe this shard length, erasures still 0..4 mixed (separates the length mix)")
    ap.add_argument("--fixed-e", type=int, default=-1,
                    help=">= 0: every stripe exactly this many erasures, lengths still mixed (separates the e mix)")
    ap.add_argument("--pads", default="0", help="gap after every shard, one layout per value")
    ap.add_argument("--orders", default="given",
                    help="descriptor order of the ragged calls, per round: given (stripe order) or dealt "
                         "(each erasure count's stripes split into 8 parts of equal workgroup counts, part x of "
                         "every count placed in the x-th eighth of the map, so the 8 XCDs get equal decode work)")
    ap.add_argument("--strided", action="store_true",
                    help="with --uniform: also time the strided kernels on the same bytes each round")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    rs = H.ReedSolomon(10, 4)
    rng = np.random.default_rng(0x5E)
    lens = [(64 << 10) << i for i in range(7)]
    n = args.stripes
    Ls = rng.choice(lens, n)
    es = rng.integers(0, 5, n)
    if args.uniform:
        Ls = np.full(n, 1 << 20)
        es = np.full(n, args.uniform)
    if args.fixed_len > 0:
        Ls = np.full(n, args.fixed_len)
    if args.fixed_e >= 0:
        es = np.full(n, args.fixed_e)
    full = (1 << 14) - 1
    masks = [full & ~int(sum(1 << int(i) for i in rng.choice(14, int(e), replace=False))) for e in es]
    pads = [int(x) for x in args.pads.split(",")]

    def layout(pad):
        descs, off = [], 0
        for s in range(n):
            descs.append((off, int(Ls[s]) + pad, int(Ls[s]), int(masks[s])))
            off += 14 * (int(Ls[s]) + pad)
        return descs, off

    lays = {p: layout(p) for p in pads}

    def dealt_order():
        parts = [[] for _ in range(8)]
        zero = []
        for e in range(1, 15):
            idx = [s for s in range(n) if bin(masks[s]).count("1") == 14 - e]
            if not idx:
                continue
            w = np.array([(int(Ls[s]) + 4095) // 4096 for s in idx], dtype=np.int64)
            start = np.cumsum(w) - w
            for s, b in zip(idx, start):
                parts[min(7, int(8 * b // w.sum()))].append(s)
        zero = [s for s in range(n) if masks[s] == full]
        return [s for part in parts for s in part] + zero

    orders = args.orders.split(",")
    perm = {"given": list(range(n)), "dealt": dealt_order() if "dealt" in orders else None}
    # "eK": stripe order, every stripe with exactly K random erasures instead
    # (the same bytes and lengths: separates the erasure mix from the rest)
    emask = {}
    for o in orders:
        if o.startswith("e") and o[1:].isdigit():
            er = np.random.default_rng(0xE0 + int(o[1:]))
            emask[o] = [full & ~int(sum(1 << int(i) for i in er.choice(14, int(o[1:]), replace=False)))
                        for _ in range(n)]
            perm[o] = list(range(n))

    def variant(p, o):
        ds = [lays[p][0][s] for s in perm[o]]
        if o in emask:
            ds = [(d[0], d[1], d[2], emask[o][s]) for s, d in zip(perm[o], ds)]
        return ds
    # converted once, not per call
    vdescs = {(p, o): variant(p, o) for p in pads for o in orders}
    darr = {k: np.array(v, dtype=B.desc_dtype()) for k, v in vdescs.items()}
    dev = torch.empty(max(o for _, o in lays.values()), dtype=torch.uint8, device="cuda")
    for s, (o, st, L, _) in enumerate(lays[pads[0]][0]):
        if st == L:  # packed: the 10 data shards are one run
            B.fill_splitmix(dev[o:o + 10 * L].view(1, 1, -1), 10 * L, bench.rank_seed_base(0) + s)
            continue
        for i in range(10):
            B.fill_splitmix(dev[o + i * st:o + i * st + L].view(1, 1, -1), L, bench.rank_seed_base(0) + 14 * s + i)
    descs = lays[pads[0]][0]
    payload = sum(10 * d[2] for d in descs) + sum(10 * d[2] for d in descs if d[3] != full)
    for p in pads:
        B.encode_ragged(rs, dev, lays[p][0])
        B.reconstruct_ragged(rs, dev, lays[p][0])
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    kinds = ["ragged"] + (["strided"] if args.strided and (args.uniform or args.fixed_len) else [])
    mask_t = torch.tensor(masks, dtype=torch.int32, device="cuda")
    for r, p, kind, order in ((r, p, k, o) for r in range(args.rounds) for p in pads
                              for k in kinds for o in (orders if k == "ragged" else ["given"])):
        descs = lays[p][0]
        L0 = int(Ls[0])
        view = dev.as_strided((n, 14, L0), (14 * (L0 + p), L0 + p, 1))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.reps + 1)]
        ev[0].record(st)
        for i in range(args.reps):
            if kind == "ragged":
                B.encode_ragged(rs, dev, darr[p, order])
            else:
                B.encode_batch(rs, view)
            ev[2 * i + 1].record(st)
            if kind == "ragged":
                B.reconstruct_ragged(rs, dev, darr[p, order])
            else:
                B.reconstruct_batch(rs, view, mask_t)
            ev[2 * i + 2].record(st)
        torch.cuda.synchronize()
        enc = np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.reps)])
        dec = np.median([ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(args.reps)])
        wall = ev[0].elapsed_time(ev[-1]) / args.reps
        enc_b = sum(14 * d[2] for d in descs)
        if kind == "ragged":
            descs = vdescs[p, order]
        dec_b = sum((14 - bin(d[3]).count("1") + 10) * d[2] for d in descs if d[3] != full)
        print(json.dumps({"lib": os.path.basename(H.LIB_PATH), "uniform": args.uniform, "stripes": n,
                          "fixed_len": args.fixed_len, "fixed_e": args.fixed_e,
                          "kind": kind, "order": order, "pad": p,
                          "round": r,
                          "enc_TBps": round(enc_b / enc / 1e9, 3), "dec_TBps": round(dec_b / dec / 1e9, 3),
                          "GiB_s": round(payload / (wall * 1e-3) / 2**30, 1),
                          "ms_per_rep": round(wall, 3), "enc_ms": round(float(enc), 3),
                          "dec_ms": round(float(dec), 3), "payload_GiB": round(payload / 2**30, 3),
                          "enc_bytes": int(enc_b), "dec_bytes": int(dec_b)}), flush=True)
    descs = lays[pads[0]][0]
    if args.grouped:
        del dev
        grouped(rs, B, torch, Ls, masks, args.rounds, args.reps)


def grouped(rs, B, torch, Ls, masks, rounds, reps):
    """The mixed batch as one strided [n_L][14][L] tensor per length."""
    full = (1 << 14) - 1
    groups = []
    for L in sorted(set(int(x) for x in Ls)):
        idx = [s for s in range(len(Ls)) if int(Ls[s]) == L]
        t = torch.empty((len(idx), 14, L), dtype=torch.uint8, device="cuda")
        B.fill_splitmix(t, 10 * L, 0x5EED0000)
        m = torch.tensor([masks[s] for s in idx], dtype=torch.int32, device="cuda")
        groups.append((t, m))
    enc_b = sum(14 * t.shape[0] * t.shape[2] for t, _ in groups)
    dec_b = sum((24 - bin(int(x)).count("1")) * t.shape[2] for t, m in groups for x in m.tolist() if x != full)
    st = torch.cuda.current_stream()
    for r in range(rounds):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        enc = dec = 0.0
        for _ in range(reps):
            e[0].record(st)
            for t, _ in groups:
                B.encode_batch(rs, t)
            e[1].record(st)
            for t, m in groups:
                B.reconstruct_batch(rs, t, m)
            e[2].record(st)
            torch.cuda.synchronize()
            enc += e[0].elapsed_time(e[1]) / reps
            dec += e[1].elapsed_time(e[2]) / reps
        print(json.dumps({"grouped_strided": True, "round": r, "enc_TBps": round(enc_b / enc / 1e9, 3),
                          "dec_TBps": round(dec_b / dec / 1e9, 3), "enc_ms": round(enc, 3), "dec_ms": round(dec, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
