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
