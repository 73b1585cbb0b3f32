"""Concurrency soak of the C ABI's host entry points (hec.h threading rules:
immutable contexts, per-device mutex-guarded state, reentrant calls).

Worker threads run, for --seconds, a random mix of:
  * per-call ReedSolomon encode / reconstruct (staged and direct sizes),
  * host batches (pinned zero-copy and pageable pooled staging), half of
    them split over a repeated device list (hec_host_*_batch_multi),
  * the batched ragged reconstruct (hec_rs_reconstruct_batch),
  * file-level write_ec_files / rebuild_ec_files on small volumes,
  * device batches on a private torch stream,
  * device-resident ragged encode + reconstruct on a private stream,
  * the staging census (hec_host_staging_stats) under the other threads,
every result checked bit-exact against the C oracle. Prints one JSON line.
Measurement / test tool only.

python tools/stress.py [--seconds 60] [--threads 8]
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    from oracle import corc
    from oracle import rs_oracle as O

    rs = H.ReedSolomon(10, 4)
    counts, failures = {}, []
    lock = threading.Lock()
    stop = time.monotonic() + args.seconds
    tmp = tempfile.mkdtemp(prefix="hec_stress_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)

    def note(kind):
        with lock:
            counts[kind] = counts.get(kind, 0) + 1

    def percall(rng):
        L = int(rng.choice([1, 100, 4096, 65536 + 5, 262144, 1 << 20]))
        data = rng.integers(0, 256, (10, L), dtype=np.uint8)
        ref = corc.encode_stripes(data[None].copy())[0]
        sh = [data[i].copy() for i in range(10)] + [np.zeros(L, np.uint8) for _ in range(4)]
        rs.encode(sh)
        assert all(np.array_equal(sh[10 + j], ref[j]) for j in range(4)), "encode"
        lost = set(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
        got = [None if i in lost else sh[i].copy() for i in range(14)]
        rs.reconstruct(got)
        assert all(np.array_equal(got[i], sh[i]) for i in range(14)), "reconstruct"
        note("per_call")

    def host_batch(rng):
        S, L = int(rng.integers(1, 9)), int(rng.choice([17, 4096, 65536, 1 << 20]))
        devs = [0] * int(rng.integers(1, 4)) if rng.integers(0, 2) else None
        kind = int(rng.integers(0, 3))  # pageable, torch-pinned, or a per-range placed batch
        buf = None
        if kind == 2 and devs is not None:
            buf = H.HostBuffer.for_devices(devs, 14 * L, S)  # hec_host_alloc_multi
            t = buf.tensor((S, 14, L))
        else:
            t = torch.zeros((S, 14, L), dtype=torch.uint8)
            if kind:
                t = t.pin_memory()
        a = t.numpy()
        a[:, :10] = rng.integers(0, 256, (S, 10, L), dtype=np.uint8)
        B.host_encode_batch(rs, t, devices=devs)
        assert np.array_equal(a[:, 10:], corc.encode_stripes(np.ascontiguousarray(a[:, :10]))), "host encode"
        want = a.copy()
        masks = np.full(S, 0x3FFF, np.uint32)
        for s in range(S):
            for i in rng.choice(14, int(rng.integers(0, 5)), replace=False):
                masks[s] &= ~np.uint32(1 << int(i))
                a[s, int(i)] = 0x11
        assert B.host_reconstruct_batch(rs, t, masks, devices=devs) == 0
        assert np.array_equal(a, want), "host reconstruct"
        note("host_batch" if devs is None else ("host_batch_multi_placed" if buf else "host_batch_multi"))
        if buf is not None:
            del t, a
            buf.close()

    def ragged(rng):
        n = int(rng.integers(1, 20))
        stripes, ref = [], []
        for _ in range(n):
            L = int(rng.integers(1, 20000))
            data = rng.integers(0, 256, (10, L), dtype=np.uint8)
            full = np.concatenate([data, corc.encode_stripes(data[None].copy())[0]])
            lost = set(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
            stripes.append([None if i in lost else full[i].copy() for i in range(14)])
            ref.append(full)
        rs.reconstruct_batch(stripes)
        for s, full in zip(stripes, ref):
            assert all(np.array_equal(s[i], full[i]) for i in range(14)), "ragged"
        note("ragged_batch")

    def files(rng, t_id):
        base = os.path.join(tmp, f"v{t_id}_{int(rng.integers(0, 1 << 30))}")
        size = int(rng.integers(1, 3_000_000))
        open(base + ".dat", "wb").write(O.splitmix64_bytes(int(rng.integers(0, 1 << 30)), size).tobytes())
        H.write_ec_files(base)
        want = [open(base + H.to_ext(i), "rb").read() for i in range(14)]
        drop = sorted(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
        for i in drop:
            os.remove(base + H.to_ext(i))
        assert H.rebuild_ec_files(base) == drop
        assert [open(base + H.to_ext(i), "rb").read() for i in range(14)] == want, "files"
        for i in range(14):
            os.remove(base + H.to_ext(i))
        os.remove(base + ".dat")
        note("files")

    def device(rng, stream):
        S, L = int(rng.integers(1, 64)), int(rng.choice([16, 4096, 8192, 65536]))
        with torch.cuda.stream(stream):
            t = torch.zeros((S, 14, L), dtype=torch.uint8, device="cuda")
            host = rng.integers(0, 256, (S, 10, L), dtype=np.uint8)
            t[:, :10] = torch.from_numpy(host).cuda()
            B.encode_batch(rs, t, stream=stream)
            stream.synchronize()
            par = t[:, 10:].cpu().numpy()
        assert np.array_equal(par, corc.encode_stripes(host)), "device"
        note("device_batch")

    def device_ragged(rng, stream):
        # device-resident ragged encode + reconstruct on a private stream (the
        # metadata slots are shared by every thread of the device)
        n = int(rng.integers(1, 24))
        lens = [int(rng.choice([16, 4096 + 16 * int(rng.integers(0, 64)), 8192, 3 * 8192])) for _ in range(n)]
        full = (1 << 14) - 1
        descs, off = [], 0
        for L in lens:
            drop = rng.choice(14, int(rng.integers(0, 5)), replace=False)
            descs.append((off, L, L, full & ~int(sum(1 << int(i) for i in drop))))
            off += 14 * L
        host = np.zeros(off, np.uint8)
        for (o, _, L, _) in descs:
            host[o:o + 10 * L] = rng.integers(0, 256, 10 * L, dtype=np.uint8)
        with torch.cuda.stream(stream):
            t = torch.from_numpy(host).cuda()
            B.encode_ragged(rs, t, descs, stream=stream)
            stream.synchronize()
            enc = t.cpu().numpy()
            for (o, _, L, m) in descs:
                for i in range(14):
                    if not (m >> i) & 1:
                        t[o + i * L:o + (i + 1) * L] = 0
            B.reconstruct_ragged(rs, t, descs, stream=stream)
            stream.synchronize()
            dec = t.cpu().numpy()
        for (o, _, L, _) in descs:
            want = corc.encode_stripes(np.ascontiguousarray(enc[o:o + 10 * L].reshape(1, 10, L)))[0]
            assert np.array_equal(enc[o + 10 * L:o + 14 * L].reshape(4, L), want), "device_ragged encode"
        assert np.array_equal(dec, enc), "device_ragged reconstruct"
        note("device_ragged")

    def census(rng):
        # the staging census while other threads' host batches are in flight
        # (it must not stall their leases)
        import ctypes
        n, pin, dev = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        assert H.lib.hec_host_staging_stats(ctypes.byref(n), ctypes.byref(pin), ctypes.byref(dev)) == 0
        assert 0 <= n.value <= 8, n.value
        note("census")

    def worker(t_id):
        rng = np.random.default_rng(1000 + t_id)
        torch.cuda.set_device(0)
        stream = torch.cuda.Stream()
        ops = [percall, host_batch, ragged, lambda r: files(r, t_id), lambda r: device(r, stream),
               lambda r: device_ragged(r, stream), census]
        while time.monotonic() < stop:
            op = ops[int(rng.integers(0, len(ops)))]
            try:
                op(rng)
            except Exception:
                with lock:
                    failures.append(traceback.format_exc(limit=3))
                return

    t0 = time.monotonic()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(args.threads)]
    for t in th:
        t.start()
    while any(t.is_alive() for t in th):  # progress line every 30 s (long runs must not look hung)
        next(t for t in th if t.is_alive()).join(timeout=30.0)
        with lock:
            print(json.dumps({"progress_s": round(time.monotonic() - t0, 1), "ops": dict(counts),
                              "failures": len(failures)}), file=sys.stderr, flush=True)
    for t in th:
        t.join()
    out = {"tool": "stress", "threads": args.threads, "seconds": round(time.monotonic() - t0, 1),
           "ops": counts, "failures": len(failures)}
    print(json.dumps(out), flush=True)
    for f in failures[:3]:
        print(f, file=sys.stderr)
    try:
        os.rmdir(tmp)
    except OSError:
        pass
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
