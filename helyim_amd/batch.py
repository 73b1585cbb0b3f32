"""Device-resident stripe batches over torch tensors (ROCm).

PyTorch is plumbing here: it owns the HBM allocation and the HIP stream; the
arithmetic is libhec's gfx950 kernels (hec_gpu_encode_batch /
hec_gpu_reconstruct_batch). Layout: a uint8 tensor ``[S, total, L]`` (stripe
major, shard, byte) -- a small row of the reference's .dat layout is exactly
10 contiguous L-byte blocks, so a run of rows lands here with one copy.
"""
from __future__ import annotations

import torch

from . import _lib
from .errors import check
from .rs import ReedSolomon

lib = _lib.lib


def _stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _check_stripes(t: torch.Tensor, rs: ReedSolomon):
    if t.dtype != torch.uint8 or not t.is_cuda or t.dim() != 3:
        raise TypeError("expected a uint8 CUDA tensor [stripes, shards, L]")
    if t.stride(2) != 1:
        raise ValueError("shard bytes must be contiguous")


def encode_batch(rs: ReedSolomon, stripes: torch.Tensor, stream=None) -> None:
    """Parity of every stripe of ``stripes[S, total, L]`` into shards data..total."""
    _check_stripes(stripes, rs)
    k = rs.data_shard_count()
    S, n, L = stripes.shape
    assert n == rs.total_shard_count()
    st, sh = stripes.stride(0), stripes.stride(1)
    base = stripes.data_ptr()
    check(lib.hec_gpu_encode_batch(rs.handle, base, st, sh, base + k * sh, st, sh, L, S,
                                   _stream_ptr(stream)))


def encode_batch_sep(rs: ReedSolomon, data: torch.Tensor, parity: torch.Tensor, stream=None) -> None:
    """data[S, k, L] -> parity[S, m, L] (separate buffers)."""
    S, k, L = data.shape
    check(lib.hec_gpu_encode_batch(rs.handle, data.data_ptr(), data.stride(0), data.stride(1),
                                   parity.data_ptr(), parity.stride(0), parity.stride(1), L, S,
                                   _stream_ptr(stream)))


def reconstruct_batch(rs: ReedSolomon, stripes: torch.Tensor, present_masks: torch.Tensor,
                      bad_stripes: torch.Tensor = None, stream=None) -> None:
    """Rebuild erased shards in place; present_masks int32 [S] (bit i = shard i present)."""
    _check_stripes(stripes, rs)
    S, n, L = stripes.shape
    assert present_masks.is_cuda and present_masks.dtype == torch.int32 and present_masks.numel() == S
    bad = bad_stripes.data_ptr() if bad_stripes is not None else None
    check(lib.hec_gpu_reconstruct_batch(rs.handle, stripes.data_ptr(), stripes.stride(0),
                                        stripes.stride(1), L, S, present_masks.data_ptr(), bad,
                                        _stream_ptr(stream)))


def _check_host(t: torch.Tensor):
    if t.dtype != torch.uint8 or t.is_cuda or t.dim() != 3 or t.stride(2) != 1:
        raise TypeError("expected a host uint8 tensor [stripes, shards, L] with contiguous shards")


def host_encode_batch(rs: ReedSolomon, stripes: torch.Tensor) -> None:
    """Host-memory stripes[S, total, L] (pin_memory() for full PCIe rate):
    parity computed on the GPU, pipelined H2D -> kernel -> D2H."""
    _check_host(stripes)
    k = rs.data_shard_count()
    S, n, L = stripes.shape
    st, sh = stripes.stride(0), stripes.stride(1)
    base = stripes.data_ptr()
    check(lib.hec_host_encode_batch(rs.handle, base, st, sh, base + k * sh, st, sh, L, S))


def host_reconstruct_batch(rs: ReedSolomon, stripes: torch.Tensor, present_masks) -> int:
    """Host-memory in-place reconstruct; returns the number of skipped stripes
    (fewer than data_shards present)."""
    import ctypes
    import numpy as np
    _check_host(stripes)
    S, n, L = stripes.shape
    m = np.ascontiguousarray(np.asarray(present_masks, dtype=np.uint32))
    assert m.size == S
    bad = ctypes.c_uint32(0)
    check(lib.hec_host_reconstruct_batch(rs.handle, stripes.data_ptr(), stripes.stride(0), stripes.stride(1), L,
                                         S, m.ctypes.data, ctypes.byref(bad)))
    return int(bad.value)


def _desc_array(descs):
    """descs: iterable of (offset, shard_stride, shard_len, present_mask)."""
    import numpy as np
    dt = np.dtype([("offset", "<u8"), ("shard_stride", "<u8"), ("shard_len", "<u4"), ("present_mask", "<u4")])
    return np.array([tuple(int(x) for x in d) for d in descs], dtype=dt)


def encode_ragged(rs: ReedSolomon, base: torch.Tensor, descs, stream=None) -> None:
    """RS(10,4) encode of stripes of mixed lengths in one launch; descs rows are
    (byte offset of shard 0 in base, shard stride, shard length, unused)."""
    d = _desc_array(descs)
    check(lib.hec_gpu_encode_ragged(rs.handle, base.data_ptr(), d.ctypes.data, len(d), _stream_ptr(stream)))


def reconstruct_ragged(rs: ReedSolomon, base: torch.Tensor, descs, bad_stripes: torch.Tensor = None,
                       stream=None) -> None:
    """Reconstruct stripes of mixed lengths and patterns in place, one launch;
    descs rows are (offset, shard stride, shard length, present mask)."""
    d = _desc_array(descs)
    bad = bad_stripes.data_ptr() if bad_stripes is not None else None
    check(lib.hec_gpu_reconstruct_ragged(rs.handle, base.data_ptr(), d.ctypes.data, len(d), bad,
                                         _stream_ptr(stream)))


def fill_splitmix(t: torch.Tensor, bytes_per_stripe: int, seed_base: int, stream=None) -> None:
    """Fill the first bytes_per_stripe bytes of each t[s] with splitmix64(seed_base + s)."""
    S = t.shape[0]
    check(lib.hec_gpu_fill_splitmix(t.data_ptr(), t.stride(0), bytes_per_stripe, S, seed_base,
                                    _stream_ptr(stream)))


def set_launch_config(vec_per_thread: int = 1, max_blocks: int = 0, xcd_remap: int = 1,
                      blocks_per_cu: int = 0) -> None:
    """Process-wide kernel launch configuration (speed only; bytes identical)."""
    check(lib.hec_set_launch_config(vec_per_thread, max_blocks, xcd_remap, blocks_per_cu))
