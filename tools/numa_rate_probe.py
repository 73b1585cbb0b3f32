"""Cross-socket cost of the zero-copy host path on one GPU (what
hec_host_alloc_multi's per-range placement buys on a multi-socket node).

One pinned host batch (512 x 1 MiB stripes, hec_host_alloc_multi over [0])
placed on the GPU's own NUMA node or on another node (HEC_TEST_RANGE_NODES,
the placement test hook, read per allocation), alternating near / far over
--rounds; pages sampled with move_pages (hec_host_numa_node) to confirm where
they landed; then --reps zero-copy encodes and 4-erasure reconstructs, each
arm's data GiB/s. One JSON line per arm.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def online_nodes():
    s = open("/sys/devices/system/node/online").read().strip()
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=512)
    args = ap.parse_args()
    import numpy as np
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    torch.cuda.set_device(0)
    S, L, n, k = args.stripes, 1 << 20, 14, 10
    near = H.numa_node(0)
    nodes = online_nodes()
    far = [x for x in nodes if x != near]
    if near < 0 or not far:
        print(json.dumps({"skipped": "one NUMA node or unknown GPU node", "nodes": nodes, "gpu_node": near}))
        return 0
    far = far[0]
    rs = H.ReedSolomon(k, 4)
    dev = torch.empty((S, n, L), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev, k * L, bench.rank_seed_base(0))
    masks = bench.erasure_masks(S, 0)
    for r in range(args.rounds):
        for arm in (("near", "far") if r % 2 == 0 else ("far", "near")):
            node = near if arm == "near" else far
            os.environ["HEC_TEST_RANGE_NODES"] = str(node)
            t0 = time.time()
            buf = H.HostBuffer.for_devices([0], n * L, S)
            alloc_s = time.time() - t0
            step = max(1, (S * n * L) // 64 // 4096) * 4096
            where = [buf.numa_node_at(o) for o in range(0, S * n * L, step)]
            host = buf.tensor((S, n, L))
            host.copy_(dev)
            B.host_encode_batch(rs, host)  # warm-up
            B.host_reconstruct_batch(rs, host, masks)
            e0 = time.time()
            for _ in range(args.reps):
                B.host_encode_batch(rs, host)
            e1 = time.time()
            for _ in range(args.reps):
                B.host_reconstruct_batch(rs, host, masks)
            d1 = time.time()
            data = S * k * L * args.reps
            print(json.dumps({"round": r, "arm": arm, "node": node, "gpu_node": near,
                              "pages_on_node": round(float(np.mean([w == node for w in where])), 3),
                              "alloc_place_register_s": round(alloc_s, 2),
                              "encode_data_GiB_s": round(data / (e1 - e0) / 2**30, 2),
                              "decode_data_GiB_s": round(data / (d1 - e1) / 2**30, 2)}), flush=True)
            del host
            buf.close()
    os.environ.pop("HEC_TEST_RANGE_NODES", None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
