"""The bit-sliced RS(10,4) syndrome decode (helyim_amd/csrc/bitslice_decode.hpp)
on the CPU, no GPU needed.

The lane function the gfx950 kernel runs (rs104_bs_decode_kernel) is compiled
for the host with g++ through the header's HEC_DEVICE / HEC_BITOP3 / HEC_PERM
hooks (v_bitop3_b32 and v_perm_b32 emulated bit for bit) and run on one
"lane" worth of columns (32 bytes per shard) for EVERY present mask with
10..13 of 14 shards present (1470 patterns). The per-pattern syndrome tables
are computed here independently (oracle/rs_oracle.py's GF(2^8) matrix
restatement), and the rebuilt shards are compared with the C oracle's
reconstruct (oracle/rs_oracle.c, upstream first-10-present rule), which is
pinned to the upstream KATs. libhec's own table builder is checked by the GPU
parity tests."""
import ctypes
import itertools
import os
import subprocess

import numpy as np
import pytest

from oracle import corc
from oracle import rs_oracle as O

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
// v_perm_b32: byte i of the result = byte sel_i of the 64-bit {a:b} (b low), sel_i < 8
static inline uint32_t host_perm(uint32_t a, uint32_t b, uint32_t sel) {
    const uint64_t c = (uint64_t(a) << 32) | b;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t v = (sel >> (8 * i)) & 0xFF;
        uint32_t byte = v < 8 ? uint32_t((c >> (8 * v)) & 0xFF) : (v == 12 ? 0u : 0xFFu);
        r |= byte << (8 * i);
    }
    return r;
}
#define HEC_DEVICE static inline
#define HEC_BITOP3(a, b, c, tt) host_bitop3((a), (b), (c), (tt))
#define HEC_PERM(a, b, sel) host_perm((a), (b), (sel))
#include "bitslice_decode.hpp"

extern "C" {
// shards: [n][14][32] bytes (erased shards' contents ignored: the kernel never
// reads them); masks[n]; syn: [n][160] words. Writes the erased shards in place.
void decode_lanes(uint8_t* shards, const uint32_t* masks, const uint32_t* syn, int n) {
    for (int s = 0; s < n; ++s) {
        uint8_t* b = shards + size_t(s) * 14 * 32;
        const uint32_t mask = masks[s];
        const uint32_t erased = ~mask & 0x3FFFu;
        const uint32_t ed = __builtin_popcount(erased & 0x3FFu);
        const uint32_t sel = hec::syn_selected(mask, ed);
        uint32_t p[80], pp[32], dd[32], q[32];
        for (int i = 0; i < 10; ++i) {
            if ((mask >> i) & 1) std::memcpy(p + 8 * i, b + i * 32, 32);
            else std::memset(p + 8 * i, 0, 32);
        }
        for (int j = 0; j < 4; ++j) {
            if ((sel >> j) & 1) std::memcpy(pp + 8 * j, b + (10 + j) * 32, 32);
            else std::memset(pp + 8 * j, 0xA5, 32);  // unselected rows must not matter
        }
        hec::rs104_syndrome_decode_lane(p, pp, mask, syn + size_t(s) * 160, dd, q);
        uint32_t e = erased & 0x3FFu;
        for (uint32_t r = 0; r < ed; ++r) {
            const int id = __builtin_ctz(e);
            e &= e - 1;
            std::memcpy(b + id * 32, dd + 8 * r, 32);
        }
        for (int j = 0; j < 4; ++j)
            if ((erased >> (10 + j)) & 1) std::memcpy(b + (10 + j) * 32, q + 8 * j, 32);
    }
}
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("bsdec")
    src, so = d / "harness.cpp", d / "harness.so"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Werror", "-Wno-unknown-pragmas",
                    "-I" + CSRC, str(src), "-o", str(so)], check=True)
    return ctypes.CDLL(str(so))


def _perm_words(c: int):
    """The 5 v_perm table words of coefficient c (gf256.hpp perm_tables)."""
    t0 = bytes(O.gf_mul(c, v) for v in range(8))
    t1 = bytes(O.gf_mul(c, v << 3) for v in range(8))
    t2 = bytes(O.gf_mul(c, v << 6) for v in range(4))
    return list(np.frombuffer(t0 + t1 + t2, dtype="<u4"))


def syndrome_tables(mask: int) -> np.ndarray:
    """bitslice_decode.hpp table layout for one present mask, restated from
    the oracle's matrix: A = inverse of the parity block (selected parity rows
    x erased data), G = M[erased parity, erased data] x A."""
    M = O.build_matrix(10, 14)
    out = np.zeros(160, dtype=np.uint32)
    ed = [i for i in range(10) if not (mask >> i) & 1]
    sel = [j for j in range(4) if (mask >> (10 + j)) & 1][:len(ed)]
    if not ed:
        return out
    sub = np.array([[M[10 + j][m] for m in ed] for j in sel], dtype=np.uint8)
    A = O.mat_invert(sub)

    def put(row, j, c):
        out[(row * 4 + j) * 5:(row * 4 + j) * 5 + 5] = _perm_words(int(c))

    for r in range(len(ed)):
        for t, j in enumerate(sel):
            put(r, j, A[r][t])
    for jj in range(4):
        if (mask >> (10 + jj)) & 1:
            continue
        G = O.mat_mul(np.array([[M[10 + jj][m] for m in ed]], dtype=np.uint8), A)
        for t, j in enumerate(sel):
            put(4 + jj, j, G[0][t])
    return out


def _all_masks():
    for e in range(1, 5):
        for drop in itertools.combinations(range(14), e):
            yield 0x3FFF & ~sum(1 << i for i in drop)


def test_every_pattern_matches_oracle_reconstruct(lib):
    masks = np.array(list(_all_masks()), dtype=np.uint32)
    assert len(masks) == 14 + 91 + 364 + 1001
    n = len(masks)
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (n, 10, 32), dtype=np.uint8)
    data[0] = 0
    data[1] = 255
    full = np.concatenate([data, corc.encode_stripes(data)], axis=1)  # [n][14][32]
    syn = np.stack([syndrome_tables(int(m)) for m in masks])
    work = full.copy()
    for s, m in enumerate(masks):
        for i in range(14):
            if not (m >> i) & 1:
                work[s, i] = rng.integers(0, 256, 32, dtype=np.uint8)  # garbage in erased slots
    lib.decode_lanes(work.ctypes.data_as(ctypes.c_void_p), masks.ctypes.data_as(ctypes.c_void_p),
                     np.ascontiguousarray(syn).ctypes.data_as(ctypes.c_void_p), n)
    assert np.array_equal(work, full)


def test_inconsistent_survivors_follow_upstream_rule(lib):
    """Survivors that are NOT a codeword (a corrupted present shard): the
    bytes still equal upstream's reconstruct, which solves from the first 10
    present shards only -- so the unselected present parity row must not
    influence the result, and the selected rows must be exactly upstream's."""
    rng = np.random.default_rng(12)
    rs = corc.CReedSolomon(10, 4)
    masks = [m for m in _all_masks()]
    picks = [masks[i] for i in rng.choice(len(masks), 200, replace=False)]
    for m in picks:
        sh = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(14)]  # random, not a codeword
        present = [bool((m >> i) & 1) for i in range(14)]
        want = [x.copy() for x in sh]
        for i in range(14):
            if not present[i]:
                want[i] = np.zeros(32, np.uint8)
        rs.reconstruct(want, present)
        work = np.stack(sh)[None].copy()
        lib.decode_lanes(work.ctypes.data_as(ctypes.c_void_p),
                         np.array([m], np.uint32).ctypes.data_as(ctypes.c_void_p),
                         syndrome_tables(m).ctypes.data_as(ctypes.c_void_p), 1)
        assert np.array_equal(work[0], np.stack(want)), hex(m)
