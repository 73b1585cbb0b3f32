"""Page-cache write/read ceilings of the file layer's I/O pattern.

T threads each write one file of --mib MiB in --chunk MiB pwrite calls (the
shard-file pattern of write_ec_files), optionally after fallocate, then read
them back. Files live in --dir (default /dev/shm).
python tools/iobench.py [--threads 14] [--mib 1200] [--chunk 25]
"""
import argparse
import json
import os
import tempfile
import threading
import time

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=14)
    ap.add_argument("--mib", type=int, default=1200)
    ap.add_argument("--chunk", type=int, default=25)
    ap.add_argument("--dir", default="/dev/shm")
    args = ap.parse_args()
    d = tempfile.mkdtemp(prefix="hec_io_", dir=args.dir)
    buf = np.random.default_rng(1).integers(0, 256, args.chunk << 20, dtype=np.uint8).tobytes()
    total = args.threads * (args.mib << 20)
    out = {"dir": args.dir, "threads": args.threads, "file_MiB": args.mib, "chunk_MiB": args.chunk}

    def run(fn):
        th = [threading.Thread(target=fn, args=(t,)) for t in range(args.threads)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        return time.perf_counter() - t0

    def writer(prealloc):
        def w(t):
            fd = os.open(os.path.join(d, f"f{t}"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            if prealloc:
                os.posix_fallocate(fd, 0, args.mib << 20)
            off = 0
            while off < (args.mib << 20):
                off += os.pwrite(fd, buf, off)
            os.close(fd)
        return w

    def reader(t):
        fd = os.open(os.path.join(d, f"f{t}"), os.O_RDONLY)
        off = 0
        while True:
            b = os.pread(fd, args.chunk << 20, off)
            if not b:
                break
            off += len(b)
        os.close(fd)

    for name, prealloc in (("write_fresh", False), ("write_fallocated", True), ("rewrite_existing", None)):
        if prealloc is None:
            def rw(t):
                fd = os.open(os.path.join(d, f"f{t}"), os.O_WRONLY)
                off = 0
                while off < (args.mib << 20):
                    off += os.pwrite(fd, buf, off)
                os.close(fd)
            s = run(rw)
        else:
            for t in range(args.threads):
                p = os.path.join(d, f"f{t}")
                if os.path.exists(p):
                    os.remove(p)
            s = run(writer(prealloc))
        out[name + "_GBps"] = round(total / s / 1e9, 2)
    out["read_GBps"] = round(total / run(reader) / 1e9, 2)
    for t in range(args.threads):
        os.remove(os.path.join(d, f"f{t}"))
    os.rmdir(d)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
