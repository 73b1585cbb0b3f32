"""Needle reads from a degraded EC volume.

A synthetic volume (.dat of --gib GiB with needles of 1 KiB..1 MiB,
log-uniform, back to back) is encoded with libhec, four data shards are
removed, and --n random needles are read three ways, outputs compared:
  cpu_c      -- the C restatement of helyim's read path (oracle/rs_oracle.c
                orc_read_ec_data): per interval, read every other shard and
                reconstruct on one CPU thread (erasure_coding/mod.rs:303-491)
  gpu_single -- hec_read_ec_needle, one call per needle
  gpu_batch  -- hec_read_ec_needles, all needles in one call (one GPU batch)
  vol_single -- hec_ec_volume_read_needle on a mounted EcVolume handle
  vol_batch  -- hec_ec_volume_read_needles on the handle
python tools/bench_reads.py [--gib 2] [--n 4000]
"""
import argparse
import ctypes
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--lost", default="1,4,6,8")
    args = ap.parse_args()
    import helyim_amd as H
    from oracle import corc
    rng = np.random.default_rng(21)
    tmp = tempfile.mkdtemp(prefix="hec_reads_", dir=os.environ.get("TMPDIR", "/tmp"))
    base = os.path.join(tmp, "7")
    size = int(args.gib * 2**30)
    dat = np.empty(size, np.uint8)
    corc.lib().orc_splitmix64_fill(99, dat.ctypes.data, size)
    dat.tofile(base + ".dat")
    entries, pos, nid = [], 8, 1
    while True:
        s = int(np.exp(rng.uniform(np.log(1024), np.log(1 << 20))))
        body = 16 + s + 4
        actual = body + (8 - body % 8)
        if pos + actual > size:
            break
        entries.append((nid, pos // 8, s))
        pos += actual
        nid += 1
    with open(base + ".idx", "wb") as f:
        f.write(b"".join(struct.pack(">QIi", *e) for e in entries))
    t0 = time.perf_counter()
    H.volume_ec_shards_generate(base, 3)
    t_gen = time.perf_counter() - t0
    lost = [int(x) for x in args.lost.split(",")]
    for i in lost:
        os.remove(base + H.to_ext(i))
    pick = rng.choice(len(entries), min(args.n, len(entries)), replace=False)
    sel = [entries[i] for i in pick]
    ranges = []
    for _, off, s in sel:
        body = 16 + s + 4
        ranges.append((off * 8, body + (8 - body % 8)))
    payload = sum(r[1] for r in ranges)
    want = [dat[o:o + n].tobytes() for o, n in ranges]
    out = {"volume_GiB": args.gib, "needles_in_volume": len(entries), "needles_read": len(sel),
           "needle_size": "1 KiB..1 MiB log-uniform", "lost_shards": lost, "payload_MiB": round(payload / 2**20, 1),
           "generate_s": round(t_gen, 3)}

    # CPU: the C restatement, one needle (range) per call
    t0 = time.perf_counter()
    cpu = [corc.read_ec_data(base, [r]) for r in ranges]
    t_cpu = time.perf_counter() - t0
    ok_cpu = all(rc == 0 and b == w for (rc, b), w in zip(cpu, want))

    # GPU single: hec_read_ec_needle per needle
    cap = max(r[1] for r in ranges)
    buf = ctypes.create_string_buffer(cap)
    nout = ctypes.c_size_t(0)
    name = base.encode()
    H.lib.hec_read_ec_needle(name, sel[0][0], buf, cap, ctypes.byref(nout))  # warm-up
    single = []
    t0 = time.perf_counter()
    for nid, _, _ in sel:
        rc = H.lib.hec_read_ec_needle(name, nid, buf, cap, ctypes.byref(nout))
        single.append(rc == 0 and buf.raw[:nout.value])
    t_single = time.perf_counter() - t0
    ok_single = all(b == w for b, w in zip(single, want))

    # GPU batch: hec_read_ec_needles
    n = len(sel)
    ids = (ctypes.c_uint64 * n)(*[e[0] for e in sel])
    offs = (ctypes.c_uint64 * (n + 1))()
    st = (ctypes.c_int * n)()
    big = ctypes.create_string_buffer(payload)
    H.lib.hec_read_ec_needles(name, 1 << 30, 1 << 20, ids, n, big, payload, offs, st)  # warm-up: staging sized
    t0 = time.perf_counter()
    rc = H.lib.hec_read_ec_needles(name, 1 << 30, 1 << 20, ids, n, big, payload, offs, st)
    t_batch = time.perf_counter() - t0
    raw = big.raw
    ok_batch = rc == 0 and all(st[i] == 0 and raw[offs[i]:offs[i + 1]] == want[i] for i in range(n))

    # mounted volume: files opened once
    vol = ctypes.c_void_p()
    assert H.lib.hec_ec_volume_open(name, ctypes.byref(vol)) == 0
    H.lib.hec_ec_volume_read_needle(vol, sel[0][0], buf, cap, ctypes.byref(nout))  # warm-up
    vsingle = []
    t0 = time.perf_counter()
    for nid, _, _ in sel:
        rc = H.lib.hec_ec_volume_read_needle(vol, nid, buf, cap, ctypes.byref(nout))
        vsingle.append(rc == 0 and buf.raw[:nout.value])
    t_vsingle = time.perf_counter() - t0
    ok_vsingle = all(b == w for b, w in zip(vsingle, want))
    t0 = time.perf_counter()
    rc = H.lib.hec_ec_volume_read_needles(vol, ids, n, big, payload, offs, st)
    t_vbatch = time.perf_counter() - t0
    raw = big.raw
    ok_vbatch = rc == 0 and all(st[i] == 0 and raw[offs[i]:offs[i + 1]] == want[i] for i in range(n))
    H.lib.hec_ec_volume_close(vol)

    for key, t in (("cpu_c_1thread", t_cpu), ("gpu_single", t_single), ("gpu_batch", t_batch),
                   ("vol_single", t_vsingle), ("vol_batch", t_vbatch)):
        out[key] = {"s": round(t, 4), "needles_per_s": round(n / t, 1), "GiB_s": round(payload / t / 2**30, 3)}
    out["identical_outputs"] = bool(ok_cpu and ok_single and ok_batch and ok_vsingle and ok_vbatch)
    print(json.dumps(out), flush=True)
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
