"""Does the bench's first process on a box run slow because HBM is still busy
with work outside the process (the driver wiping VRAM that an earlier process
released) rather than because of its own allocation?

  --churn-gib N : allocate N GiB of HBM in 4 GiB tensors, write it, free it,
                  exit (what the GPU test suite does before the bench runs).
  default       : the bench's batch (4096 x 1 MiB, 64 KiB shard gap, splitmix
                  data, 4-erasure masks), then --steps encode + decode launches,
                  each timed with HIP events on the launch stream; one JSON
                  line with every launch's ms and its start time after the
                  allocation, so a rate that climbs over the first seconds
                  shows up as a trend.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def churn(gib: int) -> None:
    import torch
    t0 = time.perf_counter()
    parts = [torch.empty(4 << 30, dtype=torch.uint8, device="cuda") for _ in range(gib // 4)]
    for p in parts:
        p.fill_(0x5A)
    torch.cuda.synchronize()
    del parts
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    print(json.dumps({"churn_gib": gib, "s": round(time.perf_counter() - t0, 3)}), flush=True)


def probe(steps: int, sleep_s: float) -> None:
    import numpy as np
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    torch.cuda.set_device(0)
    S, L = 4096, 1 << 20
    rs = H.ReedSolomon(10, 4)
    t_alloc = time.perf_counter()
    t = B.empty_stripes(S, 14, L, shard_pad=64 << 10)
    B.fill_stripes_splitmix(t, 10, bench.rank_seed_base(0))
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    torch.cuda.synchronize()
    if sleep_s:
        time.sleep(sleep_s)
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    starts = []
    for i in range(steps):
        starts.append(time.perf_counter() - t_alloc)
        ev[i][0].record(stream)
        B.encode_batch(rs, t)
        ev[i][1].record(stream)
        B.reconstruct_batch(rs, t, masks)
        ev[i][2].record(stream)
    torch.cuda.synchronize()
    enc = [round(a.elapsed_time(b), 4) for a, b, _ in ev]
    dec = [round(b.elapsed_time(c), 4) for _, b, c in ev]
    byts = S * 14 * L
    print(json.dumps({"steps": steps, "sleep_s": sleep_s, "encode_ms": enc, "decode_ms": dec,
                      "issue_s_after_alloc": [round(x, 4) for x in starts],
                      "first10_frac": [round(byts / (np.mean(enc[:10]) * 1e-3) / 8e12, 4),
                                       round(byts / (np.mean(dec[:10]) * 1e-3) / 8e12, 4)],
                      "last10_frac": [round(byts / (np.mean(enc[-10:]) * 1e-3) / 8e12, 4),
                                      round(byts / (np.mean(dec[-10:]) * 1e-3) / 8e12, 4)]}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--churn-gib", type=int, default=0)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--sleep", type=float, default=0.0, help="seconds between the fill and the first launch")
    a = ap.parse_args()
    if a.churn_gib:
        churn(a.churn_gib)
    else:
        probe(a.steps, a.sleep)
