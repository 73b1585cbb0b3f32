"""The C ABI from a plain C process (no Python, no PyTorch in the client):
tests/c/abi_client.c compiled with gcc against include/hec.h, linked to
helyim_amd/libhec.so and the C oracle. This is the path a Rust `-sys` binding
takes; the libhec in that process brings up the system HIP
runtime itself."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    lib = os.path.join(ROOT, "helyim_amd", "libhec.so")
    orc = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        pytest.fail("libhec.so / liboracle.so not built (run make)")
    exe = str(tmp_path / "abi_client")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", os.path.join(ROOT, "tests", "c", "abi_client.c"),
                    "-I" + os.path.join(ROOT, "include"), "-L" + os.path.dirname(lib), "-lhec",
                    "-L" + os.path.dirname(orc), "-loracle",
                    "-Wl,-rpath," + os.path.dirname(lib) + ":" + os.path.dirname(orc), "-o", exe], check=True)
    return exe


def _gpu_present():
    import torch
    return torch.cuda.device_count() > 0  # counts without initialising HIP


def test_c_client_without_device(tmp_path):
    if _gpu_present():
        pytest.skip("a GPU is present; the gpu-marked C client test covers this build")
    exe = _build(tmp_path)
    r = subprocess.run([exe, "nogpu", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_c_client_parity(gpu, tmp_path):
    exe = _build(tmp_path)
    env = dict(os.environ)
    env.pop("HEC_LIB_PATH", None)
    r = subprocess.run([exe, "gpu", str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "0 failed checks" in r.stdout


@pytest.mark.gpu
def test_c_abi_bench_small(gpu):
    """tools/cabi_bench.cpp (built by `make all`): the bench workload through
    the C ABI alone, 64 stripes on each of 2 worker threads (each selecting
    its device with hec_set_device), must verify its sampled rebuilds."""
    import json
    exe = os.path.join(ROOT, "build", "cabi_bench")
    if not os.path.exists(exe):
        pytest.fail("build/cabi_bench not built (run make)")
    env = dict(os.environ)
    env.pop("HEC_LIB_PATH", None)
    r = subprocess.run([exe, "64", "2", "1", "2"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["verified"] is True and out["stripes_per_worker"] == 64 and out["workers"] == 2
