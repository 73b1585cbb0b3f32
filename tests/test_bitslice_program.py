"""The bit-sliced RS(10,4) encode program on the CPU (no GPU needed).

helyim_amd/csrc/bitslice.hpp (8x8 bit transposes) and the generated
rs104_bitslice.inc (XOR program) are compiled for the host with g++ by
defining the header's HEC_DEVICE / HEC_BITOP3 hooks, then run on one "lane"
worth of data (32 bytes per shard, the kernel's two 16-byte vectors) and
compared with the C oracle's encode (oracle/rs_oracle.c, pinned to the
upstream KATs). A second test checks that the committed .inc is what
tools/gen_bitslice.py generates (no hand edits)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import corc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "helyim_amd", "csrc")

HARNESS = r"""
#include <cstdint>
#include <cstring>
static inline uint32_t host_bitop3(uint32_t a, uint32_t b, uint32_t c, int tt) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i)
        if ((tt >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}
#define HEC_DEVICE static inline
#define HEC_BITOP3(a, b, c, tt) host_bitop3((a), (b), (c), (tt))
#include "bitslice.hpp"

extern "C" {
// data: [n][10][32] bytes, parity: [n][4][32] bytes -- one kernel lane each
void encode_lanes(const uint8_t* data, uint8_t* parity, int n) {
    for (int s = 0; s < n; ++s) {
        uint32_t p[80], q[32];
        for (int i = 0; i < 10; ++i) {
            std::memcpy(p + 8 * i, data + (s * 10 + i) * 32, 32);
            hec::transpose8(p + 8 * i);
        }
        hec::rs104_encode_planes(p, q);
        for (int j = 0; j < 4; ++j) {
            hec::transpose8(q + 8 * j);
            std::memcpy(parity + (s * 4 + j) * 32, q + 8 * j, 32);
        }
    }
}
void transpose_rows(uint32_t* r, int n) { for (int i = 0; i < n; ++i) hec::transpose8(r + 8 * i); }
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("bs")
    src, so = d / "harness.cpp", d / "harness.so"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Werror", "-Wno-unknown-pragmas",
                    "-I" + CSRC, str(src), "-o", str(so)], check=True)
    return ctypes.CDLL(str(so))


def test_transpose_is_bit_transpose_and_involution(lib):
    rng = np.random.default_rng(3)
    r = rng.integers(0, 2**32, (64, 8), dtype=np.uint32)
    t = r.copy()
    lib.transpose_rows(t.ctypes.data_as(ctypes.c_void_p), 64)
    for g in range(64):
        for k in range(8):
            for lane in range(4):
                for i in range(8):
                    assert (int(t[g, k]) >> (8 * lane + i)) & 1 == (int(r[g, i]) >> (8 * lane + k)) & 1
    lib.transpose_rows(t.ctypes.data_as(ctypes.c_void_p), 64)
    assert np.array_equal(t, r)


def test_program_matches_oracle(lib):
    rng = np.random.default_rng(4)
    n = 512
    data = rng.integers(0, 256, (n, 10, 32), dtype=np.uint8)
    data[0] = 0
    data[1] = 255
    for s in range(2, 12):  # one shard carries every byte value position by position
        data[s] = 0
        data[s, s - 2] = np.arange(32, dtype=np.uint8) * 8 + (s - 2)
    par = np.zeros((n, 4, 32), dtype=np.uint8)
    lib.encode_lanes(data.ctypes.data_as(ctypes.c_void_p), par.ctypes.data_as(ctypes.c_void_p), n)
    assert np.array_equal(par, corc.encode_stripes(data))


def test_committed_program_is_generated(tmp_path):
    out = tmp_path / "gen.inc"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_bitslice.py"), "--out", str(out)],
                   check=True, capture_output=True)
    with open(os.path.join(CSRC, "rs104_bitslice.inc")) as f:
        assert out.read_text() == f.read()
