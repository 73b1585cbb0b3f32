"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into
profiles/pmc_traffic.json (HBM bytes per launch of the RS kernels).

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.

bench.py launches encode and decode alternately on the same full-size batch,
so full-grid dispatches alternate encode (even position) / decode (odd).
usage: python tools/pmc_summary.py gpurun_out/prof_r01 profiles/pmc_traffic.json
"""
import csv
import json
import os
import statistics
import sys


def load(path, counter):
    """-> ({kernel name: [bytes per full-size dispatch, ...]}, {kernel: grid})
    keeping, per kernel, only its largest-grid dispatches (the BASELINE batch;
    the bench's small verification launches are dropped)."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    grids = {}
    for r in rows:
        grids[r["Kernel_Name"]] = max(grids.get(r["Kernel_Name"], 0), int(r["Grid_Size"]))
    rows = [r for r in rows if int(r["Grid_Size"]) == grids[r["Kernel_Name"]]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = {}
    for r in rows:
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024)
    return out, grids


def split(per_kernel):
    """encode / decode series by kernel name: the encode kernel is
    rs104_bs_encode_kernel (bit-sliced) or rs104_kernel<false, ...>, decode is
    rs104_kernel<true, ...> or rs104_narrow_kernel<true, ...>; a single generic kernel alternates encode (even)
    / decode (odd)."""
    enc = [k for k in per_kernel if "rs104_bs_encode_kernel" in k or "rs104_kernel<false" in k]
    dec = [k for k in per_kernel if "rs104_kernel<true" in k or "rs104_narrow_kernel<true" in k]
    if enc and dec:
        return per_kernel[enc[0]], per_kernel[dec[0]], [enc[0], dec[0]]
    (k, v), = per_kernel.items()
    return v[0::2], v[1::2], [k]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch, grid = load(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, _ = load(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fe, fd, kname = split(fetch)
    we, wd, _ = split(write)
    enc_r = statistics.median(fe) * 2
    dec_r = statistics.median(fd) * 2
    enc_w = statistics.median(we)
    dec_w = statistics.median(wd)
    S, L = 4096, 1 << 20
    out = {
        "source": src,
        "kernel": kname,
        "grid_size_threads": {k: grid[k] for k in kname},
        "workload": f"{S} stripes x {L} B, RS(10,4)",
        "correction": "FETCH_SIZE*1024*2 (gfx950 half-count on 16B/lane streams), WRITE_SIZE*1024",
        "encode_hbm_read_bytes_per_launch": enc_r,
        "encode_hbm_write_bytes_per_launch": enc_w,
        "encode_hbm_bytes_per_launch": enc_r + enc_w,
        "encode_algorithmic_bytes_per_launch": 14 * S * L,
        "decode_hbm_read_bytes_per_launch": dec_r,
        "decode_hbm_write_bytes_per_launch": dec_w,
        "decode_hbm_bytes_per_launch": dec_r + dec_w,
        "decode_algorithmic_bytes_per_launch": 14 * S * L,
    }
    out["encode_traffic_over_algorithmic"] = out["encode_hbm_bytes_per_launch"] / out["encode_algorithmic_bytes_per_launch"]
    out["decode_traffic_over_algorithmic"] = out["decode_hbm_bytes_per_launch"] / out["decode_algorithmic_bytes_per_launch"]
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
