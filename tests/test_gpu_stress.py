"""Concurrency soak (tools/stress.py): 4 threads for 8 s mixing per-call
encode/reconstruct, host batches (pinned and pageable), ragged batched
reconstructs, file-level encode/rebuild and device batches on private
streams, every result checked against the C oracle."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_concurrent_mixed_soak(gpu):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stress.py"), "--seconds", "8", "--threads", "4"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["failures"] == 0 and sum(out["ops"].values()) > 50, out


@pytest.mark.gpu
def test_burst_slots_trim_large_staging_and_stay_exact(gpu):
    """12 threads of large per-call encodes / reconstructs (6 MiB shards: 84 MiB
    of per-call device staging) and large batched degraded reads (112 MiB of
    compact staging): slots beyond the first two of each pool free staging
    above 64 MiB when their call ends (ScratchTrim / RaggedTrim), and the next
    call on the slot reserves again. Every result is checked against the C
    oracle."""
    import threading
    import numpy as np
    import helyim_amd as H
    from oracle import corc
    rs = H.ReedSolomon(10, 4)
    ors = corc.CReedSolomon(10, 4)
    errors, start = [], threading.Barrier(12)

    def work(t):
        try:
            rng = np.random.default_rng(500 + t)
            start.wait()
            for it in range(3):
                L = (6 << 20) + 16 * int(rng.integers(0, 64))
                full = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(10)] + \
                       [np.zeros(L, np.uint8) for _ in range(4)]
                ref = [x.copy() for x in full]
                ors.encode(ref)
                rs.encode(full)
                assert all(np.array_equal(a, b) for a, b in zip(full, ref)), "encode"
                lost = set(int(i) for i in rng.choice(14, 4, replace=False))
                if it % 2 == 0:
                    got = [None if i in lost else ref[i].copy() for i in range(14)]
                    rs.reconstruct(got)
                    assert all(np.array_equal(got[i], ref[i]) for i in range(14)), "reconstruct"
                else:  # batched degraded read: 8 stripes of 1 MiB, 112 MiB of compact staging
                    stripes, refs = [], []
                    for _ in range(8):
                        d = [rng.integers(0, 256, 1 << 20, dtype=np.uint8) for _ in range(10)] + \
                            [np.zeros(1 << 20, np.uint8) for _ in range(4)]
                        ors.encode(d)
                        refs.append(d)
                        gone = set(int(i) for i in rng.choice(14, int(rng.integers(1, 5)), replace=False))
                        stripes.append([None if i in gone else d[i].copy() for i in range(14)])
                    rs.reconstruct_batch(stripes)
                    for st, d in zip(stripes, refs):
                        assert all(np.array_equal(st[i], d[i]) for i in range(14)), "reconstruct_batch"
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(repr(ex))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(12)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
