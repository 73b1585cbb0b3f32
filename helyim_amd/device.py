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


def numa_node(device: int) -> int:
    """NUMA node of the device's PCI function (-1 when the platform does not say)."""
    n = ctypes.c_int(-1)
    check(lib.hec_device_numa_node(device, ctypes.byref(n)))
    return n.value


def bind_host_to_device(device: int) -> dict:
    """Restrict the calling thread -- and the threads it starts later (the
    library's worker pool, torch's) -- to the device's NUMA node, so the host
    side of a per-GPU rank runs next to its pinned buffers.
    Returns what was done: the node, how many CPUs the thread now has."""
    node = numa_node(device)
    n = ctypes.c_int(0)
    check(lib.hec_bind_thread_to_device(device, ctypes.byref(n)))
    return {"device": device, "gpu_numa_node": node, "bound_cpus": n.value}


class HostBuffer:
    """Pinned host memory on the current device's NUMA node (hec_host_alloc),
    GPU-addressable, exposed as a numpy array (``.array``) or a torch CPU
    tensor view (``.tensor(shape)``). Every view holds a reference to this
    object (through the ctypes array under it), so collection -- and the
    ``hec_host_free`` in ``__del__`` -- waits for the last view; an explicit
    ``close()`` frees at once and must come after the views are gone."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib.hec_host_alloc(nbytes, ctypes.byref(p)))
        self._ptr = p.value
        self.nbytes = nbytes

    @classmethod
    def for_devices(cls, devices, stripe_stride: int, n_stripes: int) -> "HostBuffer":
        """One host batch of n_stripes stripes for ``host_*_batch(...,
        devices=devices)`` (hec_host_alloc_multi): each device's stripe range
        has its pages on that device's NUMA node."""
        self = cls.__new__(cls)
        self._ptr = None
        arr = (ctypes.c_int * len(devices))(*devices)
        p = ctypes.c_void_p()
        check(lib.hec_host_alloc_multi(arr, len(devices), stripe_stride, n_stripes, ctypes.byref(p)))
        self._ptr = p.value
        self.nbytes = stripe_stride * n_stripes
        return self

    def numa_node_at(self, offset: int) -> int:
        """Node holding the page at byte ``offset``."""
        n = ctypes.c_int(-1)
        check(lib.hec_host_numa_node(self._ptr + offset, ctypes.byref(n)))
        return n.value

    @property
    def array(self):
        """A fresh numpy view. The view holds this object (through the ctypes
        array under it) and this object holds no view, so there is no cycle:
        the buffer is freed by refcount as soon as the last view and the
        HostBuffer itself are gone."""
        import numpy as np
        if not self._ptr:
            raise ValueError("HostBuffer is closed")
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self._ptr)
        raw._owner = self
        return np.ctypeslib.as_array(raw)

    @property
    def ptr(self) -> int:
        return self._ptr

    def tensor(self, shape):
        import torch
        return torch.from_numpy(self.array).view(*shape)

    def numa_node(self) -> int:
        """Node holding the buffer's first page."""
        n = ctypes.c_int(-1)
        check(lib.hec_host_numa_node(self._ptr, ctypes.byref(n)))
        return n.value

    def close(self) -> None:
        if self._ptr:
            check(lib.hec_host_free(self._ptr))
            self._ptr = None

    def __del__(self):
        try:
            if getattr(self, "_ptr", None):
                self.close()
        except Exception:
            pass
