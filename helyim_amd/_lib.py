"""Loader for the in-tree HIP library helyim_amd/libhec.so (C ABI: include/hec.h).

There is no fallback: if the library is missing or fails to load, importing
helyim_amd raises. Compute calls without a GPU return HEC_ERR_NO_DEVICE, which
surfaces as ``helyim_amd.errors.DeviceError``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# HEC_LIB_PATH: measurement builds only (tools/tune.py loads kernel variants).
LIB_PATH = os.environ.get("HEC_LIB_PATH") or os.path.join(_HERE, "libhec.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build the HIP library first (`make -C {os.path.dirname(_HERE)}` "
        "or __graft_entry__.build()). helyim_amd has no CPU fallback."
    )

# One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so
# (SONAME libamdhip64.so.7). Load it first so libhec's DT_NEEDED binds to the
# same runtime torch uses; device pointers and hipStream_t handles from torch
# are then valid in libhec. Without torch, the system ROCm runtime is used.
try:  # pragma: no cover - depends on the environment
    import torch  # noqa: F401
except ImportError:
    torch = None

lib = ctypes.CDLL(LIB_PATH)

_P = ctypes.c_void_p
_S = ctypes.c_size_t
_U64 = ctypes.c_uint64
_U32 = ctypes.c_uint32
_I = ctypes.c_int

# name -> (restype, argtypes); every function declared in include/hec.h
SIGNATURES = {
    "hec_strerror": (ctypes.c_char_p, [_I]),
    "hec_last_error_detail": (ctypes.c_char_p, []),
    "hec_last_error_values": (_I, [ctypes.POINTER(_U64), ctypes.POINTER(_U64), ctypes.POINTER(_I)]),
    "hec_rs_new": (_I, [_S, _S, ctypes.POINTER(_P)]),
    "hec_rs_free": (None, [_P]),
    "hec_rs_data_shard_count": (_S, [_P]),
    "hec_rs_parity_shard_count": (_S, [_P]),
    "hec_rs_total_shard_count": (_S, [_P]),
    "hec_rs_matrix": (_I, [_P, _P, _S]),
    "hec_rs_encode": (_I, [_P, _P, _P, _S]),
    "hec_rs_verify": (_I, [_P, _P, _P, _S, ctypes.POINTER(_I)]),
    "hec_rs_reconstruct": (_I, [_P, _P, _P, _P, _S]),
    "hec_rs_reconstruct_data": (_I, [_P, _P, _P, _P, _S]),
    "hec_rs_reconstruct_batch": (_I, [_P, _P, _P, _P, _S, _I, ctypes.POINTER(_S)]),
    "hec_gpu_encode_batch": (_I, [_P, _P, _U64, _U64, _P, _U64, _U64, _U64, _U32, _P]),
    "hec_gpu_reconstruct_batch": (_I, [_P, _P, _U64, _U64, _U64, _U32, _P, _P, _P]),
    "hec_host_encode_batch": (_I, [_P, _P, _U64, _U64, _P, _U64, _U64, _U64, _U32]),
    "hec_host_reconstruct_batch": (_I, [_P, _P, _U64, _U64, _U64, _U32, _P, _P]),
    "hec_host_encode_batch_multi": (_I, [_P, _P, _S, _P, _U64, _U64, _P, _U64, _U64, _U64, _U32]),
    "hec_host_reconstruct_batch_multi": (_I, [_P, _P, _S, _P, _U64, _U64, _U64, _U32, _P, _P]),
    "hec_gpu_encode_ragged": (_I, [_P, _P, _P, _U32, _P]),
    "hec_gpu_reconstruct_ragged": (_I, [_P, _P, _P, _U32, _P, _P]),
    "hec_gpu_fill_splitmix": (_I, [_P, _U64, _U64, _U32, _U64, _P]),
    "hec_write_ec_files": (_I, [ctypes.c_char_p]),
    "hec_write_ec_files_ex": (_I, [ctypes.c_char_p, _U64, _U64, _U64]),
    "hec_rebuild_ec_files": (_I, [ctypes.c_char_p, ctypes.POINTER(_U32), ctypes.POINTER(_S)]),
    "hec_write_sorted_file_from_index": (_I, [ctypes.c_char_p, ctypes.c_char_p]),
    "hec_rebuild_ecx_file": (_I, [ctypes.c_char_p]),
    "hec_save_volume_info": (_I, [ctypes.c_char_p, _U32]),
    "hec_find_data_filesize": (_I, [ctypes.c_char_p, ctypes.POINTER(_U64)]),
    "hec_write_data_file": (_I, [ctypes.c_char_p, ctypes.c_int64]),
    "hec_write_index_file_from_ec_index": (_I, [ctypes.c_char_p]),
    "hec_locate_data": (_I, [_U64, _U64, _U64, _U64, _U64, _P, _S, ctypes.POINTER(_S)]),
    "hec_interval_shard_id": (_U32, [_P]),
    "hec_interval_offset": (_U64, [_P, _U64, _U64]),
    "hec_find_needle_from_ecx": (_I, [ctypes.c_char_p, _U64, ctypes.POINTER(_U32), ctypes.POINTER(ctypes.c_int32)]),
    "hec_read_ec_data": (_I, [ctypes.c_char_p, _U64, _U64, _P, _P, _S, _P]),
    "hec_read_ec_needle": (_I, [ctypes.c_char_p, _U64, _P, _S, ctypes.POINTER(_S)]),
    "hec_read_ec_needle_ex": (_I, [ctypes.c_char_p, _U64, _U64, _U64, _P, _S, ctypes.POINTER(_S)]),
    "hec_read_ec_needles": (_I, [ctypes.c_char_p, _U64, _U64, _P, _S, _P, _S, _P, _P]),
    "hec_ec_volume_open": (_I, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    "hec_ec_volume_open_ex": (_I, [ctypes.c_char_p, _U64, _U64, ctypes.POINTER(_P)]),
    "hec_ec_volume_close": (None, [_P]),
    "hec_ec_volume_version": (_U32, [_P]),
    "hec_ec_volume_shard_bits": (_U32, [_P]),
    "hec_ec_volume_find_needle": (_I, [_P, _U64, ctypes.POINTER(_U32), ctypes.POINTER(ctypes.c_int32)]),
    "hec_ec_volume_delete_needle": (_I, [_P, _U64]),
    "hec_ec_volume_read_needle": (_I, [_P, _U64, _P, _S, ctypes.POINTER(_S)]),
    "hec_ec_volume_read_needles": (_I, [_P, _P, _S, _P, _S, _P, _P]),
    "hec_set_host_staging": (_I, [ctypes.c_uint64]),
    "hec_set_completion_signal": (_I, [ctypes.c_uint64]),
    "hec_set_host_zero_copy": (_I, [_I]),
    "hec_host_encode_kernel_name": (ctypes.c_char_p, [ctypes.c_uint64]),
    "hec_host_zero_copy_view": (_I, [_P, _U64, ctypes.POINTER(_I)]),
    "hec_host_staging_stats": (_I, [ctypes.POINTER(_I), ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "hec_version": (ctypes.c_char_p, []),
    "hec_device_count": (_I, [ctypes.POINTER(_I)]),
    "hec_set_device": (_I, [_I]),
    "hec_get_device": (_I, [ctypes.POINTER(_I)]),
    "hec_device_numa_node": (_I, [_I, ctypes.POINTER(_I)]),
    "hec_bind_thread_to_device": (_I, [_I, ctypes.POINTER(_I)]),
    "hec_host_alloc": (_I, [_S, ctypes.POINTER(_P)]),
    "hec_host_alloc_multi": (_I, [_P, _S, _U64, _U32, ctypes.POINTER(_P)]),
    "hec_host_free": (_I, [_P]),
    "hec_host_numa_node": (_I, [_P, ctypes.POINTER(_I)]),
    "hec_encode_kernel_name": (ctypes.c_char_p, [ctypes.c_uint64]),
    "hec_decode_kernel_name": (ctypes.c_char_p, [ctypes.c_uint64]),
    "hec_ragged_kernel_name": (ctypes.c_char_p, [_P, _U32, _I]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


def strerror(code: int) -> str:
    return lib.hec_strerror(code).decode()


def last_detail() -> str:
    return lib.hec_last_error_detail().decode()


def last_values() -> tuple:
    """(a, b, os_errno) of the last failure on this thread (hec_last_error_values)."""
    a, b, e = _U64(), _U64(), _I()
    lib.hec_last_error_values(ctypes.byref(a), ctypes.byref(b), ctypes.byref(e))
    return a.value, b.value, e.value
