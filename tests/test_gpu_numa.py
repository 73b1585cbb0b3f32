"""NUMA placement of the host side of a GPU (numa.cpp): the
device's node from sysfs, pinned buffers on that node, thread binding, and a
host batch coded zero-copy from such a buffer (checked against the C oracle)."""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _online_nodes():
    try:
        s = open("/sys/devices/system/node/online").read().strip()
    except OSError:
        return 1
    n = 0
    for part in s.split(","):
        a, _, b = part.partition("-")
        n += (int(b) - int(a) + 1) if b else 1
    return n


def test_device_node_and_buffer_placement():
    import torch
    import helyim_amd as H
    torch.cuda.set_device(0)
    node = H.numa_node(0)
    assert node >= -1
    buf = H.HostBuffer(8 << 20)
    buf.array[:] = 1  # resident
    placed = buf.numa_node()
    if node >= 0 and _online_nodes() > 1:
        assert placed == node, f"pinned staging on node {placed}, GPU on node {node}"
    buf.close()


def test_bind_thread_to_device_restricts_affinity():
    import helyim_amd as H
    res = {}

    def work():  # a fresh thread, so the test process keeps its affinity
        before = os.sched_getaffinity(0)
        res["info"] = H.bind_host_to_device(0)
        res["after"] = os.sched_getaffinity(0)
        res["before"] = before

    t = threading.Thread(target=work)
    t.start()
    t.join()
    info = res["info"]
    assert res["after"] <= res["before"]
    if info["bound_cpus"]:
        assert len(res["after"]) == info["bound_cpus"]


def test_host_batch_from_numa_local_buffer():
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    from oracle import corc
    torch.cuda.set_device(0)
    S, L = 6, 65536
    buf = H.HostBuffer(S * 14 * L)
    t = buf.tensor((S, 14, L))
    rng = np.random.default_rng(7)
    t[:, :10] = torch.from_numpy(rng.integers(0, 256, (S, 10, L), dtype=np.uint8))
    rs = H.ReedSolomon(10, 4)
    B.host_encode_batch(rs, t)
    ref = corc.encode_stripes(t[:, :10].numpy().copy())
    assert np.array_equal(t[:, 10:].numpy(), ref)
    good = t.numpy().copy()
    masks = np.full(S, (1 << 14) - 1, np.uint32)
    for s, drop in enumerate([(0, 1, 2, 3), (10, 11, 12, 13), (0, 5, 10, 13), (9,), (4, 12), (1, 6, 11)]):
        for i in drop:
            t[s, i] = 0
            masks[s] &= ~np.uint32(1 << i)
    assert B.host_reconstruct_batch(rs, t, masks) == 0
    assert np.array_equal(t.numpy(), good)
    del t
    buf.close()
