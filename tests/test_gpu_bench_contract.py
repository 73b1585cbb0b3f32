"""The bench line the driver parses (bench.py at N=1, a small batch): exactly
one JSON line on stdout carrying the contract's keys, a `value` that follows
from its own step time, a `roofline` whose fraction follows from its achieved
rate, a verified run and the CPU baseline beside it."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "verified")


@pytest.mark.gpu
def test_bench_line_contract():
    S, L, steps = 64, 1 << 20, 3  # 0.9 GiB: larger than the 256 MB Infinity Cache
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stripes", str(S), "--shard-len", str(L),
                        "--steps", str(steps), "--warmup", "1", "--no-extras", "--cpu-seconds", "0.4"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, p.stdout[-3000:]
    d = json.loads(lines[0])
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == steps and d["warmup"] == 1
    assert d["unit"] == "GiB/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["dtype"] == "u8" and d["vs_baseline"] is None
    assert d["verified"] is True
    v = d["verification"]  # the whole batch against the C oracle, not a sample
    assert v["stripes_checked"] == S and v["rebuilt_shards_checked"] == 4 * S and v["mismatched_stripes"] == []
    assert d["config"]["stripes_per_gpu"] == S and d["config"]["shard_len"] == L
    # value = encode + decode data payload over the timed steps
    payload = 2 * S * 10 * L
    assert d["value"] == pytest.approx(payload / (d["ms_per_step"] * 1e-3) / 2**30, rel=0.01)
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["achieved"] < r["peak"]
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)
    assert r["algorithmic_bytes_per_launch"] == S * 14 * L  # 10 reads + 4 writes per stripe either way
    assert r["traffic"] is None  # the committed PMC bytes are of the 4096 x 1 MiB batch, not this one
    pk = d["packed_layout"]  # the packed-stride rate beside the padded headline
    assert pk["shard_stride"] == L and d["config"]["shard_stride"] == L + (64 << 10)
    assert 0 < pk["encode_frac"] < 1 and 0 < pk["decode_frac"] < 1
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0 and cb["sample"]


@pytest.mark.gpu
def test_bench_multi_gpu_host_leg_child():
    """The bench's in-process multi-GPU end-to-end leg (run in a child
    process when more than one GPU is visible) rehearsed on one GPU with the
    device list 0,0: one host call split over two concurrent ranges."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--e2e-multi-child", "0,0"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert d["devices"] == [0, 0] and d["stripes"] == 512
    assert "hec_host_alloc_multi" in d["host_memory"]  # each range on its GPU's NUMA node
    assert d["encode_data_GiB_s"] > 1 and d["decode_data_GiB_s"] > 1


@pytest.mark.gpu
def test_bench_mixed_leg_verified_and_named_by_the_launcher(gpu):
    """The config-5 leg (bench.mixed_section) on 256 stripes: its kernel names
    are the ragged launch's own choice (hec_ragged_kernel_name), and its
    oracle check covers every stripe (so every length x erasure-count pair)."""
    import bench
    import helyim_amd as H
    import helyim_amd.batch as B
    rs = H.ReedSolomon(10, 4)
    m = bench.mixed_section(rs, 0, n_stripes=256, e2e_stripes=32)
    v = m["verification"]
    assert v["ok"] and v["mismatched_stripes"] == [] and v["stripes_checked"] == 256  # every stripe
    assert v["rebuilt_shards_checked"] > 0
    assert v["erasure_counts"] == [0, 1, 2, 3, 4] and len(v["shard_lens"]) == 7
    assert m["encode"]["kernel"] == "rs104_bs_ragged_kernel (bit-sliced, XCD eighths)"
    assert m["decode"]["kernel"] == "rs104_ragged_kernel<DEC=true> (table lookup, XCD eighths)"
    assert B.ragged_kernel_name([(0, 4096, 4096, 0)], False).startswith("rs104_ragged_kernel<DEC=false>")


@pytest.mark.gpu
def test_bench_base_align_and_odd_shard_length():
    """bench.py --base-align starts the batch at the
    asked alignment and still verifies; a shard length that is not a multiple
    of 8 checks parity and rebuilt shards without the seeded-data check
    (no assertion after the timed region)."""
    for extra, L, seeds in ((["--base-align", str(1 << 30)], 1 << 20, True),
                            (["--shard-pad", "0"], 4096 + 4, False)):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stripes", "32", "--shard-len", str(L),
                            "--steps", "2", "--warmup", "1", "--no-extras", "--no-packed", "--no-cpu-baseline",
                            *extra], capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert p.returncode == 0, p.stderr[-3000:]
        d = json.loads([x for x in p.stdout.splitlines() if x.strip()][-1])
        assert d["verified"] is True and d["verification"]["data_seeds_checked"] is seeds
        if extra[0] == "--base-align":
            assert d["config"]["base_alignment"] >= 1 << 30
