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
