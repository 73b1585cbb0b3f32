"""bench.py --gpus N as the driver runs it, without a GPU: the launcher leg
(no GPU call in the parent, N ranks through torch.distributed.run), the
refusals, and the control plane the real ranks share with the --dry-run leg
(per-rank seeds, barrier, max-over-ranks timing, one JSON line on stdout)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def test_launcher_spawns_n_ranks_and_reports_max_over_ranks():
    sys.path.insert(0, ROOT)
    import bench
    steps, step_ms = 4, 20.0
    r = _run(["--gpus", "2", "--dry-run", "--steps", str(steps), "--warmup", "1", "--dry-step-ms", str(step_ms)])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # stdout carries exactly the bench line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"] is True
    ranks = out["ranks"]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert sorted(x["local_rank"] for x in ranks) == [0, 1]
    assert all(x["world_size"] == 2 for x in ranks)
    assert len({x["pid"] for x in ranks}) == 2  # two processes
    assert out["rank_seed_bases"] == [bench.rank_seed_base(0), bench.rank_seed_base(1)]
    assert ranks[0]["masks_head"] != ranks[1]["masks_head"]  # independent stripe batches
    # rank 1's stand-in step is 2 x step_ms: the job time is the slower rank's
    slow = max(x["wall_s"] for x in ranks)
    assert out["ms_per_step"] == pytest.approx(slow / steps * 1e3, rel=0.05)
    assert out["ms_per_step"] >= 2 * step_ms * 0.95
    payload = 2 * 4096 * 10 * (1 << 20)
    assert out["value"] == pytest.approx(bench.job_throughput(payload, steps, 2, slow), rel=0.05)


def test_single_rank_default_stays_in_process():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "0", "--dry-step-ms", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_refuses_more_ranks_than_visible_gpus():
    r = _run(["--gpus", "2"], {"HIP_VISIBLE_DEVICES": "0"})
    assert r.returncode == 2 and "1 GPU(s) visible" in r.stderr


def test_visible_gpu_count_reads_env_lists(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2")
    assert bench.visible_gpu_count() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpu_count() == 0


def test_host_path_aggregation():
    sys.path.insert(0, ROOT)
    import bench
    gib = 2**30
    # rank 1 starts its encode 0.1 s late: the node's window is 0.0 .. 0.5 s
    agg = bench.aggregate_host_path([{"data_bytes": 10 * gib, "encode": [0.0, 0.2], "decode": [0.2, 0.45]},
                                     {"data_bytes": 10 * gib, "encode": [0.1, 0.5], "decode": [0.5, 0.7]}])
    assert agg["ranks"] == 2
    assert agg["encode_data_GiB_s"] == 40.0  # 20 GiB over 0.5 s
    assert agg["decode_data_GiB_s"] == 40.0  # 20 GiB over 0.2 .. 0.7 s
    assert agg["per_rank_encode_data_GiB_s"] == [50.0, 25.0]
    assert agg["per_rank_decode_data_GiB_s"] == [40.0, 50.0]
