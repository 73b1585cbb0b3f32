"""Device selection through the C ABI (include/hec.h ``hec_set_device``).

helyim has no GPU, so there is no reference counterpart: a multi-GPU volume
server picks the device per call (whole volumes per GPU). The
setting is the calling thread's current HIP device, the same one torch's
``torch.cuda.set_device`` changes.
"""
from __future__ import annotations

import ctypes

from . import _lib
from .errors import check

lib = _lib.lib


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib.hec_device_count(ctypes.byref(n)))
    return n.value


def set_device(device: int) -> None:
    check(lib.hec_set_device(device))


def get_device() -> int:
    d = ctypes.c_int(-1)
    check(lib.hec_get_device(ctypes.byref(d)))
    return d.value
