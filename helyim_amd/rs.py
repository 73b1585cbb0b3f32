"""``ReedSolomon`` -- drop-in for reed_solomon_erasure::ReedSolomon<galois_8::Field>.

Mirrors the three calls helyim makes (new / encode / reconstruct:
/root/reference/helyim-ec/src/encoder.rs:191,208-209,249-250,288 and
helyim-store/src/erasure_coding/mod.rs:411-412,426) plus the upstream
``verify`` and ``reconstruct_data`` companions, with upstream argument meaning
and error behaviour. Every computation runs in libhec's gfx950 kernels.

Shards are writable byte buffers: ``numpy.ndarray`` (uint8, C-contiguous),
``bytearray`` or anything exposing a writable buffer. ``reconstruct`` takes a
list whose missing entries are ``None`` (upstream ``Option<Vec<u8>>``) and
fills them with newly allocated zero-initialised ``numpy`` arrays, like
upstream ``get_or_initialize``.
"""
from __future__ import annotations

import ctypes
from typing import List, MutableSequence, Optional, Sequence

import numpy as np

from . import _lib
from .errors import check

lib = _lib.lib


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or not buf.flags.c_contiguous:
            raise TypeError("shards must be C-contiguous uint8 arrays")
        return buf
    return np.frombuffer(buf, dtype=np.uint8)


def _ptr_array(arrs: Sequence[Optional[np.ndarray]]):
    p = (ctypes.c_void_p * len(arrs))()
    for i, a in enumerate(arrs):
        p[i] = a.ctypes.data if (a is not None and a.size) else None
    return p


def _len_array(arrs: Sequence[Optional[np.ndarray]]):
    return (ctypes.c_size_t * len(arrs))(*[(a.size if a is not None else 0) for a in arrs])


class ReedSolomon:
    """``ReedSolomon::new(data_shards, parity_shards)``."""

    def __init__(self, data_shards: int, parity_shards: int):
        h = ctypes.c_void_p()
        check(lib.hec_rs_new(data_shards, parity_shards, ctypes.byref(h)))
        self._h = h
        self._k = data_shards
        self._m = parity_shards

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.hec_rs_free(h)
            self._h = None

    def data_shard_count(self) -> int:
        return self._k

    def parity_shard_count(self) -> int:
        return self._m

    def total_shard_count(self) -> int:
        return self._k + self._m

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.total_shard_count(), self._k), dtype=np.uint8)
        check(lib.hec_rs_matrix(self._h, out.ctypes.data, out.size))
        return out

    def encode(self, shards: Sequence) -> None:
        """Compute parity into shards[data..total] in place."""
        arrs = [_as_u8(s) for s in shards]
        check(lib.hec_rs_encode(self._h, _ptr_array(arrs), _len_array(arrs), len(arrs)))

    def verify(self, shards: Sequence) -> bool:
        arrs = [_as_u8(s) for s in shards]
        ok = ctypes.c_int(0)
        check(lib.hec_rs_verify(self._h, _ptr_array(arrs), _len_array(arrs), len(arrs), ctypes.byref(ok)))
        return bool(ok.value)

    def reconstruct(self, shards: MutableSequence[Optional[object]]) -> None:
        self._reconstruct(shards, data_only=False)

    def reconstruct_data(self, shards: MutableSequence[Optional[object]]) -> None:
        self._reconstruct(shards, data_only=True)

    def _reconstruct(self, shards, data_only: bool) -> None:
        arrs: List[Optional[np.ndarray]] = [None if s is None else _as_u8(s) for s in shards]
        present = (ctypes.c_uint8 * len(arrs))(*[0 if a is None else 1 for a in arrs])
        # Allocate missing slots of the common length (upstream get_or_initialize);
        # the library validates sizes/counts and reports upstream errors first.
        lens = [a.size for a in arrs if a is not None]
        L = lens[0] if lens else 0
        n = self.total_shard_count()
        new: List[int] = []
        if len(arrs) == n and L and all(x == L for x in lens) and len(lens) >= self._k and len(lens) < n:
            for i, a in enumerate(arrs):
                if a is None and not (data_only and i >= self._k):
                    arrs[i] = np.zeros(L, dtype=np.uint8)
                    new.append(i)
        rc = lib.hec_rs_reconstruct_data if data_only else lib.hec_rs_reconstruct
        check(rc(self._h, _ptr_array(arrs), _len_array(arrs), present, len(arrs)))
        for i in new:
            shards[i] = arrs[i]

    def reconstruct_batch(self, stripes: Sequence[MutableSequence[Optional[object]]],
                          data_only: bool = False) -> None:
        """reconstruct() over many independent stripes (any lengths) in one GPU
        round trip -- the batched form of the degraded-read reconstruct.
        Raises the first failing stripe's error (attribute .stripe) with
        nothing written."""
        n = self.total_shard_count()
        flat: List[Optional[np.ndarray]] = []
        new = []
        for si, shards in enumerate(stripes):
            arrs = [None if s is None else _as_u8(s) for s in shards]
            if len(arrs) != n:
                from .errors import TooFewShards, TooManyShards
                err = TooFewShards() if len(arrs) < n else TooManyShards()
                err.stripe = si
                raise err
            lens = [a.size for a in arrs if a is not None]
            L = lens[0] if lens else 0
            if L and all(x == L for x in lens) and self._k <= len(lens) < n:
                for i, a in enumerate(arrs):
                    if a is None and not (data_only and i >= self._k):
                        arrs[i] = np.zeros(L, dtype=np.uint8)
                        new.append((si, i, arrs[i]))
            flat.extend(arrs)
        present = (ctypes.c_uint8 * len(flat))(*[0 if a is None else 1 for a in flat])
        for si, shards in enumerate(stripes):  # presence comes from the caller's None slots
            for i, s in enumerate(shards):
                present[si * n + i] = 0 if s is None else 1
        bad = ctypes.c_size_t(0)
        rc = lib.hec_rs_reconstruct_batch(self._h, _ptr_array(flat), _len_array(
            [None if (s is None) else a for s, a in zip([x for st in stripes for x in st], flat)]),
            present, len(stripes), int(data_only), ctypes.byref(bad))
        if rc:
            try:
                check(rc)
            except Exception as e:
                e.stripe = int(bad.value)
                raise
        for si, i, a in new:
            stripes[si][i] = a
