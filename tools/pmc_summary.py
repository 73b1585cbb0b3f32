"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into
profiles/pmc_traffic.json (HBM bytes per launch of the RS kernels).

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.

bench.py launches encode and decode alternately on the same full-size batch,
so full-grid dispatches alternate encode (even position) / decode (odd).
usage: python tools/pmc_summary.py gpurun_out/prof_r01 profiles/pmc_traffic.json [gpurun_out/calib]
  (third argument: a calibration pass, tools/pmc_calib.sh: measured factors
  replace the assumed ones)
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


def calibration(cdir):
    """Counter factors measured on KNOWN byte counts (build/membench_calib,
    tools/membench.hip calib): math-free streams in the decode's access
    pattern at 8 and 16 B per lane, in the same process and PMC pass as the
    shipped encode and decode. factor = known bytes / counter bytes.
    -> (factors, {case: ...}, shipped-kernel bytes per dispatch from the same pass)."""
    S, L = 4096, 1 << 20
    fetch = load_all(os.path.join(cdir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load_all(os.path.join(cdir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")

    def med(d, tag):
        ks = [k for k in d if tag in k]
        assert len(ks) == 1, (tag, list(d))
        return statistics.median(d[ks[0]][1:])  # the first dispatch of each case is its warm-up

    cases, f = {}, {}
    for vb in (8, 16):
        for w in (0, 4):
            tag = f"k_cal<{vb}, {w}>"
            r, wr = med(fetch, tag), med(write, tag)
            cases[f"{vb}B_10r{w}w"] = {"known_read_bytes": S * 10 * L, "fetch_size_bytes": r,
                                       "known_write_bytes": S * w * L, "write_size_bytes": wr}
        f[f"read_{vb}B"] = S * 10 * L / cases[f"{vb}B_10r0w"]["fetch_size_bytes"]
        f[f"read_{vb}B_with_writes"] = S * 10 * L / cases[f"{vb}B_10r4w"]["fetch_size_bytes"]
        f[f"write_{vb}B"] = S * 4 * L / cases[f"{vb}B_10r4w"]["write_size_bytes"]
    shipped = {"encode": (med(fetch, "rs104_bs_encode_kernel"), med(write, "rs104_bs_encode_kernel")),
               "decode": (med(fetch, "rs104_narrow_kernel<true"), med(write, "rs104_narrow_kernel<true"))}
    return f, cases, shipped


def load_all(path, counter):
    """{kernel name: [counter bytes per dispatch in dispatch order]} (every dispatch)."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = {}
    for r in rows:
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    cdir = sys.argv[3] if len(sys.argv) > 3 else None
    fetch, grid = load(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, _ = load(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fe, fd, kname = split(fetch)
    we, wd, _ = split(write)
    # default: the guide's 16 B/lane calibration (FETCH_SIZE half-count) for
    # both kernels; with a calibration pass, each kernel's own access width
    # (bit-sliced encode: 16 B/lane loads and stores; decode: 8 B/lane)
    fr_enc = fr_dec = 2.0
    fw_enc = fw_dec = 1.0
    correction = "FETCH_SIZE*1024*2 (gfx950 half-count on 16B/lane streams), WRITE_SIZE*1024"
    calib = None
    if cdir:
        fac, cases, shipped = calibration(cdir)
        fr_enc, fw_enc = fac["read_16B_with_writes"], fac["write_16B"]
        fr_dec, fw_dec = fac["read_8B_with_writes"], fac["write_8B"]
        correction = ("measured: FETCH_SIZE*1024 x known/counted bytes of a math-free stream at the kernel's own "
                      "access width with 4 write streams (encode 16 B/lane, decode 8 B/lane), WRITE_SIZE*1024 x the "
                      "same stream's write factor; calibration block below")
        calib = {"source": cdir, "factors": {k: round(v, 6) for k, v in fac.items()}, "cases": cases,
                 "method": "build/membench_calib (tools/membench.hip calib): k_cal<bytes per lane, writes> reads "
                           "shards 0..9 of [4096][14][1 MiB + 64 KiB] non-temporal (XCD eighths, one workgroup per "
                           "256 x bytes-per-lane column range) and writes 0 or 4 shards: known bytes / counter bytes. "
                           "The shipped encode and decode ran in the same process and the same PMC pass",
                 "same_pass_shipped_kernels": {
                     k: {"read_bytes": v[0] * (fr_enc if k == "encode" else fr_dec),
                         "write_bytes": v[1] * (fw_enc if k == "encode" else fw_dec),
                         "over_algorithmic": (v[0] * (fr_enc if k == "encode" else fr_dec)
                                              + v[1] * (fw_enc if k == "encode" else fw_dec)) / (14 * 4096 * (1 << 20))}
                     for k, v in shipped.items()}}
    enc_r = statistics.median(fe) * fr_enc
    dec_r = statistics.median(fd) * fr_dec
    enc_w = statistics.median(we) * fw_enc
    dec_w = statistics.median(wd) * fw_dec
    S, L = 4096, 1 << 20
    out = {
        "source": src,
        "kernel": kname,
        "grid_size_threads": {k: grid[k] for k in kname},
        "workload": f"{S} stripes x {L} B, RS(10,4)",
        "correction": correction,
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
    if calib:
        out["calibration"] = calib
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
