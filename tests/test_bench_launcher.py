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


def test_eight_rank_dry_run_assembles_the_node_line():
    """VERDICT r03 "next" 5: the driver's 8-GPU scaling run rehearsed without
    hardware. 8 ranks through torch.distributed.run (gloo control plane):
    max-over-ranks job time, every rank's record gathered on rank 0, and the
    host legs' node aggregates (end_to_end.aggregate over the 8 ranks'
    windows, mixed.aggregate_end_to_end_data_GiB_s) assembled by the same
    function run_rank uses (bench.assemble_host_legs)."""
    sys.path.insert(0, ROOT)
    import bench
    steps, step_ms = 3, 10.0
    r = _run(["--gpus", "8", "--dry-run", "--steps", str(steps), "--warmup", "1", "--dry-step-ms", str(step_ms)],
             timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["verified"] is True
    ranks = out["ranks"]
    assert sorted(x["rank"] for x in ranks) == list(range(8))
    assert len({x["pid"] for x in ranks}) == 8
    assert out["rank_seed_bases"] == [bench.rank_seed_base(i) for i in range(8)]
    slow = max(x["wall_s"] for x in ranks)  # rank 7: 8 x step_ms per step
    assert out["ms_per_step"] == pytest.approx(slow / steps * 1e3, rel=0.05)
    assert out["ms_per_step"] >= 8 * step_ms * 0.95
    assert out["value"] == pytest.approx(bench.job_throughput(2 * 4096 * 10 * (1 << 20), steps, 8, slow), rel=0.05)
    e2e = out["end_to_end"]
    assert len(e2e["per_rank"]) == 8 and e2e["aggregate"]["ranks"] == 8
    # the node aggregate is every rank's bytes over ONE window: below the sum
    # of the per-rank rates (ranks overlap but are not simultaneous)
    agg = e2e["aggregate"]["encode_data_GiB_s"]
    assert 0 < agg <= sum(e2e["aggregate"]["per_rank_encode_data_GiB_s"]) * 1.001
    assert agg == bench.aggregate_host_path([p["raw"] for p in e2e["per_rank"]])["encode_data_GiB_s"]
    mixed = out["mixed"]
    assert len(mixed["per_rank"]) == 8
    window = (max(m["raw"]["e2e"][1] for m in mixed["per_rank"]) - min(m["raw"]["e2e"][0] for m in mixed["per_rank"]))
    assert mixed["aggregate_end_to_end_data_GiB_s"] == pytest.approx(sum(range(1, 9)) / window, rel=0.02)
    # VERDICT r04 "next" 2: the CPU path is in the line at every world size,
    # through the same function run_rank uses (bench.cpu_baseline_legs)
    for key, threads in (("cpu_baseline", 1), ("cpu_baseline_threads", 16)):
        assert out[key]["kind"] == "stand_in" and out[key]["cores"] == threads
    cores = out["cpu_baseline_cores"]
    assert {"physical_cores", "affinity_cpus", "cgroup_cpu_quota", "quota_bound"} <= set(cores)
    usable = min(cores["affinity_cpus"], int(cores["cgroup_cpu_quota"] or cores["affinity_cpus"]))
    assert cores["cores"] == max(1, min(cores["physical_cores"], usable))
    assert cores["quota_bound"] == (cores["physical_cores"] > usable)
    # VERDICT r05 "next" 5: the SCALE line reads directly as per-GPU
    # efficiency: value / N, the slowest / fastest rank's own step, and every
    # rank's encode / decode fraction (None in the GPU-free stand-in)
    assert out["per_gpu_GiB_s"] == pytest.approx(out["value"] / 8, rel=1e-3)
    assert out["rank_spread"] == pytest.approx(8.0, rel=1e-3)  # rank r steps (r + 1) x step_ms
    pf = out["per_rank_frac"]
    assert [x["rank"] for x in pf] == list(range(8))
    assert all({"step_ms", "encode_frac", "decode_frac"} <= set(x) for x in pf)
    assert [x["step_ms"] for x in pf] == pytest.approx([(r + 1) * step_ms for r in range(8)])


def test_scaling_fields_of_real_rank_records():
    """bench.scaling_fields on run_rank-shaped records: per-GPU rate, the
    rank spread of the ranks' own HIP-event step times, each rank's fractions."""
    sys.path.insert(0, ROOT)
    import bench
    recs = [{"rank": 0, "step_ms": 18.9, "encode_frac": 0.80, "decode_frac": 0.79},
            {"rank": 1, "step_ms": 19.8, "encode_frac": 0.77, "decode_frac": 0.75}]
    f = bench.scaling_fields(8200.0, 2, recs)
    assert f["per_gpu_GiB_s"] == 4100.0
    assert f["rank_spread"] == pytest.approx(19.8 / 18.9, abs=1e-4)
    assert f["per_rank_frac"][1] == {"rank": 1, "step_ms": 19.8, "encode_frac": 0.77, "decode_frac": 0.75}


def test_cpu_baseline_cores_sized_to_the_quota(monkeypatch):
    """cpu_baseline_cores runs one thread per CPU the process can use at once:
    under a 16-CPU cgroup quota on a 128-core host that is 16 threads, marked
    quota_bound (round 4 ran 128 threads under the quota and reported a
    throttled figure as a core-count result)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(bench, "physical_cores", lambda: {"physical_cores": 128, "logical_cpus": 256,
                                                          "affinity_cpus": 256, "cgroup_cpu_quota": 16.0})
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: None)
    runs = []
    monkeypatch.setattr(bench, "cpu_baseline", lambda s: {"value": 1.0, "cores": 1})
    monkeypatch.setattr(bench, "cpu_baseline_threads",
                        lambda s, n: runs.append(n) or {"value": float(n), "cores": n})
    out = bench.cpu_baseline_legs(1.0, set())
    assert out["cpu_baseline_cores"]["cores"] == 16 and out["cpu_baseline_cores"]["quota_bound"] is True
    assert runs == [16]  # the 16-thread leg is not run twice
    monkeypatch.setattr(bench, "physical_cores", lambda: {"physical_cores": 8, "logical_cpus": 16,
                                                          "affinity_cpus": 16, "cgroup_cpu_quota": None})
    runs.clear()
    out = bench.cpu_baseline_legs(1.0, set())
    assert runs == [16, 8] and out["cpu_baseline_cores"]["cores"] == 8
    assert out["cpu_baseline_cores"]["quota_bound"] is False


def test_dry_run_one_failing_rank_fails_the_job():
    """Verification is reduced over ranks: one rank's failed check makes the
    job's line say verified false and every rank exit 3."""
    r = _run(["--gpus", "4", "--dry-run", "--steps", "2", "--warmup", "0", "--dry-step-ms", "1",
              "--dry-fail-rank", "2"], timeout=240)
    assert r.returncode != 0
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert out["verified"] is False and out["n_gpus"] == 4


def test_multi_gpu_leg_failures_are_records_not_exceptions():
    """multi_gpu_e2e_child (the in-process multi-GPU host leg) turns every
    failure of its child into a record: a time limit, a non-zero exit, output
    that is not JSON, a child that cannot start. The headline line is
    assembled around it either way."""
    sys.path.insert(0, ROOT)
    import bench
    slow = bench.multi_gpu_e2e_child(2, timeout_s=0.5, cmd=[sys.executable, "-c", "import time; time.sleep(30)"])
    assert slow == {"error": "timed out after 0 s"} or slow["error"].startswith("timed out")
    bad = bench.multi_gpu_e2e_child(2, cmd=[sys.executable, "-c", "import sys; sys.stderr.write('boom'); sys.exit(4)"])
    assert bad["error"] == "exit 4" and "boom" in bad["stderr_tail"]
    junk = bench.multi_gpu_e2e_child(2, cmd=[sys.executable, "-c", "print('{not json')"])
    assert junk["error"].startswith("unparsable output")
    gone = bench.multi_gpu_e2e_child(2, cmd=["/nonexistent/python"])
    assert gone["error"].startswith("could not start")
    ok = bench.multi_gpu_e2e_child(2, cmd=[sys.executable, "-c", "import json; print(json.dumps({'devices': [0, 1]}))"])
    assert ok == {"devices": [0, 1]}


def test_assemble_host_legs_single_rank_passes_records_through():
    sys.path.insert(0, ROOT)
    import bench
    e, m = {"raw": {"data_bytes": 1}}, {"raw": {"payload_bytes": 1, "e2e": [0, 1]}}
    assert bench.assemble_host_legs([e], [m], 1) == {"end_to_end": e, "mixed": m}
