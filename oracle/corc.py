"""ctypes front-end for oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Loads the C restatement (oracle/rs_oracle.c). Used by tests/ as a fast
bit-exact checker at MiB sizes and by bench.py's cpu_baseline leg. It is never
imported by the product package helyim_amd.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        P = ctypes.c_void_p
        L.orc_rs_new.restype = P
        L.orc_rs_new.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_rs_free.argtypes = [P]
        L.orc_rs_matrix.argtypes = [P, P]
        L.orc_encode.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int]
        L.orc_reconstruct.argtypes = [P, P, P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.orc_reconstruct.restype = ctypes.c_int
        L.orc_code_some_slices.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_size_t, ctypes.c_int]
        L.orc_splitmix64_fill.argtypes = [ctypes.c_uint64, P, ctypes.c_size_t]
        L.orc_gf_mul.restype = ctypes.c_uint8
        L.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_exp.restype = ctypes.c_uint8
        L.orc_gf_exp.argtypes = [ctypes.c_uint8, ctypes.c_uint]
        L.orc_invert.argtypes = [P, P, ctypes.c_int]
        L.orc_invert.restype = ctypes.c_int
        L.orc_have_avx2.restype = ctypes.c_int
        L.orc_write_ec_files.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_int]
        L.orc_write_ec_files.restype = ctypes.c_int
        L.orc_rebuild_ec_files.argtypes = [ctypes.c_char_p, P, P, ctypes.c_int]
        L.orc_rebuild_ec_files.restype = ctypes.c_int
        L.orc_read_ec_data.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, P, P, ctypes.c_size_t, P,
                                       ctypes.c_int]
        L.orc_read_ec_data.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptrs(bufs: Sequence[np.ndarray]):
    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        assert b.dtype == np.uint8 and b.flags.c_contiguous
        arr[i] = b.ctypes.data
    return arr


class CReedSolomon:
    def __init__(self, k: int, m: int):
        self.k, self.m, self.n = k, m, k + m
        self._h = lib().orc_rs_new(k, m)
        if not self._h:
            raise ValueError("invalid geometry")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_rs_free(self._h)
            self._h = None

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.n, self.k), dtype=np.uint8)
        lib().orc_rs_matrix(self._h, out.ctypes.data)
        return out

    def encode(self, shards: List[np.ndarray], simd: bool = True) -> None:
        lib().orc_encode(self._h, _ptrs(shards), len(shards[0]), int(simd))

    def reconstruct(self, shards: List[np.ndarray], present: Sequence[bool],
                    data_only: bool = False, simd: bool = True) -> int:
        pres = np.array([1 if p else 0 for p in present], dtype=np.uint8)
        return lib().orc_reconstruct(self._h, _ptrs(shards), pres.ctypes.data,
                                     len(shards[0]), int(data_only), int(simd))


def encode_stripes(data: np.ndarray, simd: bool = True) -> np.ndarray:
    """data [S, 10, L] -> parity [S, 4, L] with the C oracle (RS(10,4))."""
    S, k, L = data.shape
    rs = CReedSolomon(k, 4)
    par = np.zeros((S, 4, L), dtype=np.uint8)
    for s in range(S):
        shards = [data[s, i] for i in range(k)] + [par[s, j] for j in range(4)]
        rs.encode(shards, simd)
    return par


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    lib().orc_splitmix64_fill(seed, out.ctypes.data, nbytes)
    return out


def write_ec_files(base: str, buf_size: int = 256 * 1024, large: int = 1 << 30, small: int = 1 << 20,
                   simd: bool = True) -> int:
    """C restatement of helyim_ec::write_ec_files (encoder.rs:39-242)."""
    return lib().orc_write_ec_files(base.encode(), buf_size, large, small, int(simd))


def rebuild_ec_files(base: str, simd: bool = True):
    """C restatement of helyim_ec::rebuild_ec_files; -> (rc, rebuilt ids)."""
    ids = (ctypes.c_uint32 * 14)()
    n = ctypes.c_size_t(0)
    rc = lib().orc_rebuild_ec_files(base.encode(), ctypes.cast(ids, ctypes.c_void_p),
                                    ctypes.cast(ctypes.pointer(n), ctypes.c_void_p), int(simd))
    return rc, [int(ids[i]) for i in range(n.value)]


def read_ec_data(base: str, ranges, large: int = 1 << 30, small: int = 1 << 20, simd: bool = True):
    """C restatement of the needle-interval read path (erasure_coding/mod.rs:303-491):
    returns (rc, bytes); rc 0 ok, -1 io, -4 TooFewShardsPresent, -5 no shard."""
    ranges = list(ranges)
    n = len(ranges)
    offs = np.array([r[0] for r in ranges] or [0], dtype=np.uint64)
    sizes = np.array([r[1] for r in ranges] or [0], dtype=np.uint64)
    total = int(sum(r[1] for r in ranges))
    out = np.zeros(max(total, 1), dtype=np.uint8)
    rc = lib().orc_read_ec_data(base.encode(), large, small, offs.ctypes.data, sizes.ctypes.data, n,
                                out.ctypes.data, int(simd))
    return rc, out[:total].tobytes()


GAMMA = 0x9E3779B97F4A7C15


def shard_seed(seed: int, shard: int, shard_len: int) -> int:
    """splitmix64 seed of shard `shard` of a stripe seeded `seed` (its stream
    from word shard * L / 8 on; L a multiple of 8)."""
    return (seed + shard * (shard_len // 8) * GAMMA) & ((1 << 64) - 1)


def check_stripes(host: np.ndarray, masks=None, threads: int = 16, data_seeds=None) -> List[int]:
    """Bit-exact check of a chunk of RS(10,4) stripes against the C oracle, on
    a pool of threads (ctypes releases the GIL inside the C calls).

    host: [S, 14, L] uint8, each shard contiguous.
    * Always: every stripe's parity (shards 10..13) == the oracle's encode of
      its data shards 0..9.
    * data_seeds [S] (stripe s = splitmix64_bytes(data_seeds[s], 10 L)): the
      data shards also equal that stream, so the whole stripe is the oracle's
      codeword of the seeded data.
    * masks [S]: every shard erased in masks[s] (bit clear) also equals the
      oracle's reconstruct (upstream rule: first 10 present shards) from the
      present ones (stripes with all 14 or fewer than 10 present: skipped).
    Returns the indices of the stripes that differ (sorted)."""
    from concurrent.futures import ThreadPoolExecutor
    S, n, L = host.shape
    assert n == 14 and host.dtype == np.uint8
    rs = CReedSolomon(10, 4)
    full = (1 << 14) - 1
    if data_seeds is not None:
        assert L % 8 == 0, "seeded data check needs L % 8 == 0"

    def shard(s, i):
        return np.ascontiguousarray(host[s, i])

    def one(s):
        data = [shard(s, i) for i in range(10)]
        if data_seeds is not None:
            for i in range(10):
                if not np.array_equal(data[i], splitmix64_bytes(shard_seed(int(data_seeds[s]), i, L), L)):
                    return False
        par = [np.empty(L, np.uint8) for _ in range(4)]
        rs.encode(data + par)
        if not all(np.array_equal(par[j], host[s, 10 + j]) for j in range(4)):
            return False
        if masks is None:
            return True
        m = int(masks[s]) & full
        if m == full or bin(m).count("1") < 10:
            return True
        present = [bool((m >> i) & 1) for i in range(14)]
        bufs = [shard(s, i) if present[i] else np.empty(L, np.uint8) for i in range(14)]
        if rs.reconstruct(bufs, present) != 0:
            return False
        return all(np.array_equal(bufs[i], host[s, i]) for i in range(14) if not present[i])

    with ThreadPoolExecutor(max(1, threads)) as ex:
        ok = list(ex.map(one, range(S)))
    return [s for s in range(S) if not ok[s]]


def check_device_batch(t, masks=None, data_seeds=None, chunk: int = 64, threads: int = 16) -> List[int]:
    """check_stripes over a whole device batch t [S, 14, L] (torch, any shard
    and stripe strides), copied back `chunk` stripes at a time through one
    pinned host buffer. Returns the stripe indices that differ."""
    import torch
    S, n, L = t.shape
    c = min(chunk, S)
    pinned = torch.empty((c, n, L), dtype=torch.uint8, pin_memory=True)
    bad = []
    for s0 in range(0, S, c):
        s1 = min(S, s0 + c)
        h = pinned[:s1 - s0]
        h.copy_(t[s0:s1])
        m = None if masks is None else masks[s0:s1]
        seeds = None if data_seeds is None else data_seeds[s0:s1]
        bad += [s0 + s for s in check_stripes(h.numpy(), m, threads, seeds)]
    return bad
