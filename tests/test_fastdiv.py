"""hec::FastDiv, the multiply-shift division of the RS(10,4) fast kernels'
workgroup -> (stripe, chunk) map (helyim_amd/csrc/fastdiv.hpp), against C's
`/` on ~90k divisors x edge and random dividends: tests/c/fastdiv_check.cpp,
compiled with g++ (the header is plain C++). A wrong quotient would code the
wrong stripe's bytes; the GPU parity suites cover the kernels themselves."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fastdiv_matches_division(tmp_path):
    exe = str(tmp_path / "fastdiv_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", os.path.join(ROOT, "tests", "c", "fastdiv_check.cpp"),
                    "-I" + os.path.join(ROOT, "helyim_amd", "csrc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
